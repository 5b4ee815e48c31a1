#!/bin/bash
# GPU session: parity tests then a short bench.  Stops at the first crash/timeout
# (exit codes other than 0/1 from pytest), never retries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-5}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -z "$SKIP_DP" ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 scripts/dp_check.py > gpurun_out/dp_check.log 2>&1
  drc=$?
  echo "dp_check rc=$drc"; grep "dp_check" gpurun_out/dp_check.log | tail -2
  if [ $drc -ne 0 ]; then tail -30 gpurun_out/dp_check.log; exit $drc; fi
fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
grep -v "MLP\|Linear\|ELU\|Sequential\|^)" gpurun_out/bench.log | tail -20
exit $brc
