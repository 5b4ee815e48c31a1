cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python bench.py --config 3 --no-cpu-baseline > gpurun_out/b3.log 2>&1 || exit 1
tail -1 gpurun_out/b3.log | cut -c1-200
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline > gpurun_out/b5.log 2>&1 || exit 1
tail -1 gpurun_out/b5.log | cut -c1-200
