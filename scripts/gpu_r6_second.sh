#!/bin/bash
# Round 6: the tests the first suite run did not reach, smoke, the default bench, and the 2-rank
# same-device gloo rehearsal with the all-reduce timing (profiles/r6_dist).
mkdir -p gpurun_out/r6_b
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo_full.py -x -v --timeout 300 \
  --timeout-method thread -k "fk_matches_mjcf or config1 or ppo_update_full" > gpurun_out/r6_b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/r6_b/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_b/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r6_b/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r6_b/bench.json 2> gpurun_out/r6_b/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r6_b/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/r6_b/bench.err; exit $rc; }
timeout -k 10 600 python -u bench.py --gpus 2 --same-device --dist-backend gloo --no-cpu-baseline --steps 6 --warmup 2 \
  > gpurun_out/r6_b/bench_dist2_gloo.json 2> gpurun_out/r6_b/bench_dist2_gloo.err
rc=$?; echo "dist bench rc=$rc"; tail -c 900 gpurun_out/r6_b/bench_dist2_gloo.json; [ $rc -ne 0 ] && tail -20 gpurun_out/r6_b/bench_dist2_gloo.err
exit $rc
