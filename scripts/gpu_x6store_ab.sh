#!/bin/bash
# Same-box A/B of the bf16-split GEMM's staging order (round 5): the base build (BASE_LIB, default
# abpush/libhgsim_base.so) against the tree's, per shape (scripts/x6r_probe.py, with a sha256 of every
# output, so the two builds are compared bit for bit) and on the bench, alternated twice; then the
# GEMM GPU tests on the tree's library.  Every GPU step has its own time limit; the script stops at
# the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
BASE=${BASE_LIB:-abpush/libhgsim_base.so}
OUT=gpurun_out/x6store_ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -20 $OUT/pytest_gemm.log; exit 1; }
tail -1 $OUT/pytest_gemm.log
for round in 1 2; do
  HG_LIB="$BASE" ITERS=50 timeout -k 10 300 python -u scripts/x6r_probe.py base > $OUT/probe_base_$round.log 2>&1 || { echo "base probe failed"; tail -5 $OUT/probe_base_$round.log; exit 1; }
  ITERS=50 timeout -k 10 300 python -u scripts/x6r_probe.py new > $OUT/probe_new_$round.log 2>&1 || { echo "new probe failed"; tail -5 $OUT/probe_new_$round.log; exit 1; }
  python scripts/x6r_probe.py compare > $OUT/compare_$round.txt 2>&1 || exit 1
  cp gpurun_out/x6r_base.json $OUT/x6r_base_$round.json && cp gpurun_out/x6r_new.json $OUT/x6r_new_$round.json
done
cat $OUT/compare_2.txt
for round in 1 2; do
  for tag in base new; do
    if [ $tag = base ]; then LIBV="$BASE"; else LIBV=""; fi
    HG_LIB="$LIBV" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_${tag}_$round.log 2>&1 || { echo "bench $tag failed"; tail -5 $OUT/bench_${tag}_$round.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['learn_time_s'])" $OUT/bench_${tag}_$round.log "$tag r$round"
  done
done
