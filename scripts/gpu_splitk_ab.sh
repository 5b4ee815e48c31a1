#!/bin/bash
# Split-K rollout layer (round 5): the GEMM GPU tests, then kernel traces of the bench with the
# split-K route off and on (fused finish) for the routes in ROUTES, then the bench off / on
# alternated twice.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
OUT=gpurun_out/splitk_ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 $OUT/pytest_gemm.log; exit 1; }
tail -1 $OUT/pytest_gemm.log
bash scripts/gpu_splitk_prof.sh || exit 1
for round in 1 2; do
  for sel in 0 1; do
    HG_SPLITK_FWD=$sel timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_${sel}_$round.log 2>&1 || { echo "bench $sel failed"; tail -5 $OUT/bench_${sel}_$round.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/bench_${sel}_$round.log "splitk=$sel r$round"
  done
done
