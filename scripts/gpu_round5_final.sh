#!/bin/bash
# Round-5 end-of-round GPU session: the -m gpu suite + smoke + the config-2 bench (scripts/gpu_round5.sh),
# then the config-3 and config-5 bench lines.  Stops at the first failure; never retries.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out
bash scripts/gpu_round5.sh || exit $?
timeout -k 10 600 python bench.py --config 3 --steps 10 --warmup 3 > gpurun_out/bench_config3.log 2>&1 || { echo "config 3 failed"; tail -5 gpurun_out/bench_config3.log; exit 1; }
tail -1 gpurun_out/bench_config3.log | cut -c1-200
timeout -k 10 600 python bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/bench_config5.log 2>&1 || { echo "config 5 failed"; tail -5 gpurun_out/bench_config5.log; exit 1; }
tail -1 gpurun_out/bench_config5.log | cut -c1-200
