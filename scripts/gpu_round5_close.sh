#!/bin/bash
# Round-5 closing GPU session after the split-K rollout layer: the -m gpu suite + smoke + the
# config-2/3/5 bench lines (scripts/gpu_round5_final.sh), then the profile set (kernel trace, HBM
# PMC passes and summary, iteration breakdown, K_step SQ counters).  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
bash scripts/gpu_round5_final.sh || exit $?
bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof gpurun_out/prof/pmc_summary.json gpurun_out/prof/trace/run_kernel_stats.csv > /dev/null || exit $?
python scripts/iter_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv > gpurun_out/prof/iteration_breakdown.txt 2>&1 || echo "breakdown failed (non-fatal)"
bash scripts/pmc_sq.sh || exit $?
python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq/sq_counters_k_step.json > /dev/null || exit $?
echo "profiles ok"
