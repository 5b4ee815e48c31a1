#!/bin/bash
# The env order built inside the post launch: the K_step / window tests, the bench, a kernel trace.
O=gpurun_out/r6_order
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "wave_balancing or window or frame_only or 4096 or runner_one or config1 or smoke" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  python -c "import json;d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/trace.log" 2>&1 || { echo trace failed; exit 1; }
echo "trace ok"
