#!/bin/bash
# Round-6 end check on one MI355X: the full GPU suite, smoke, and the bench on configs 2 / 3 / 5.
# Logs under gpurun_out/r6_final.  Stops at the first failure.
O=gpurun_out/r6_final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
for c in 2 3 5; do
  timeout -k 10 600 python -u bench.py --config $c > $O/bench_config$c.json 2> $O/bench_config$c.err
  rc=$?; echo "bench config $c rc=$rc"; tail -c 400 $O/bench_config$c.json; echo
  [ $rc -ne 0 ] && { tail -20 $O/bench_config$c.err; exit $rc; }
done
exit 0
