# bf16 policy iteration: full GPU suite, config-5 bench, kernel trace of config 5
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
grep -E "rel errors|passed|failed" gpurun_out/t_gpu.log
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline > gpurun_out/b5.log 2>&1 || { tail -30 gpurun_out/b5.log; exit 1; }
tail -1 gpurun_out/b5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['collection_time_s'], d['learn_time_s'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p5 -o run -- python3 $R/bench.py --config 5 --steps 3 --warmup 2 --no-cpu-baseline > $R/gpurun_out/p5.log 2>&1 || { tail -20 $R/gpurun_out/p5.log; exit 1; }
echo traced
