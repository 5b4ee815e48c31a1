#!/bin/bash
# Round-5 profile set: kernel trace + FETCH/WRITE PMC passes of the bench (scripts/profile.sh),
# the per-kernel PMC summary, K_step SQ counters (scripts/pmc_sq.sh), and the K_step phase probe
# (scripts/dev/kstep_probe.py, library built beforehand into abpush/kprobe: ./build is not pushed),
# and the GEMM tile sweep of the learn shapes (scripts/gemm_tile_sweep.py).  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof gpurun_out/prof/pmc_summary.json gpurun_out/prof/trace/run_kernel_stats.csv > /dev/null || exit $?
python scripts/iter_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv > gpurun_out/prof/iteration_breakdown.txt 2>&1 || echo "breakdown failed (non-fatal)"
bash scripts/pmc_sq.sh || exit $?
python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq/sq_counters_k_step.json || exit $?
cd "$R"
if [ -f abpush/kprobe/libhgsim.so ]; then
  PROBE_DIR=abpush/kprobe timeout -k 10 300 python scripts/dev/kstep_probe.py run > gpurun_out/kstep_phase_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/kstep_phase_probe.txt; exit 1; }
  echo "probe ok"
fi
timeout -k 10 300 python -u scripts/gemm_tile_sweep.py > gpurun_out/gemm_tile_sweep.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/gemm_tile_sweep.log; exit 1; }
echo "sweep ok"
