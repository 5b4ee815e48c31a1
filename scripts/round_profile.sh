#!/bin/bash
# Everything that goes under profiles/<round>/: kernel trace stats + FETCH/WRITE PMC passes of the
# bench, SQ counter passes of K_step, the parity trajectory curves, and a bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/profile.sh || exit $?
python scripts/pmc_summary.py gpurun_out/prof gpurun_out/prof/pmc_summary.json gpurun_out/prof/trace/run_kernel_stats.csv > /dev/null || exit $?
bash scripts/pmc_sq.sh || exit $?
python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq/sq_counters_k_step.json || exit $?
cd "$R"
timeout -k 10 700 python scripts/trajectory_curve.py > gpurun_out/traj.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_round.log 2>&1 || exit $?
tail -1 gpurun_out/bench_round.log
