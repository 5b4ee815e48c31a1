#!/bin/bash
# GPU session (round 5; HG_TOL_REPORT collects the tolerance headroom): the -m gpu suite (all tests, per-test timeout), then a short bench.  Stops at a
# crash / timeout (pytest exit codes other than 0/1), never retries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HG_TOL_REPORT=${HG_TOL_REPORT:-gpurun_out/tol_report.jsonl}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -30
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
echo "smoke rc=$src"; tail -2 gpurun_out/smoke.log
if [ $src -ne 0 ]; then exit $src; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -2 gpurun_out/bench.log
exit $brc
