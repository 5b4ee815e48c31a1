#!/bin/bash
# Same-box A/B of environment-selected variants: optional GPU tests (PYTEST_K), then the bench
# alternating between the default and each variant (VARIANTS="NAME=VAL ..."), ROUNDS times.
# Stops at the first failure; never retries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$PYTEST_K" \
    > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/ab/pytest.log | head -20; exit $rc; fi
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in base $VARIANTS; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
      > gpurun_out/ab/bench_${r}_${v//[=\/]/_}.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab/bench_${r}_${v//[=\/]/_}.log; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']), d['ms_per_step'], 'learn', d.get('learn_time_s'), 'coll', d.get('collection_time_s'))" gpurun_out/ab/bench_${r}_${v//[=\/]/_}.log "$v"
  done
done
