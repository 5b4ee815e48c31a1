#!/bin/bash
# Round-6 profile set: kernel trace + FETCH/WRITE PMC passes of the bench (scripts/profile.sh),
# the per-kernel PMC summary, the iteration and GEMM breakdowns, K_step's SQ counters
# (scripts/pmc_sq.sh), and the GEMM occupancy-tile sweep (scripts/probes/occ_probe.py).
# Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof gpurun_out/prof/pmc_summary.json gpurun_out/prof/trace/run_kernel_stats.csv > /dev/null || exit $?
python scripts/iter_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv > gpurun_out/prof/iteration_breakdown.txt 2>&1 || echo "breakdown failed (non-fatal)"
python scripts/gemm_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv > gpurun_out/prof/gemm_breakdown.txt 2>&1 || echo "gemm breakdown failed (non-fatal)"
bash scripts/pmc_sq.sh || exit $?
python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq/sq_counters_k_step.json || exit $?
echo "profile set ok"
