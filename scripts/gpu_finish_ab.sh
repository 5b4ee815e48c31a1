#!/bin/bash
# Same-box A/B of k_splitk_finish (base build BASE_LIB vs the tree's): the GEMM GPU tests on the
# tree's library, then kernel traces of the bench, alternated twice, printing the rollout split-K
# layer's two kernels.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
export TMPDIR=/tmp
BASE=${BASE_LIB:-abpush/libhgsim_base.so}
OUT=gpurun_out/finish_ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 $OUT/pytest_gemm.log; exit 1; }
tail -1 $OUT/pytest_gemm.log
for round in 1 2; do
  for tag in base new; do
    if [ $tag = base ]; then export HG_LIB="$BASE"; else unset HG_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_$round -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_${tag}_$round.log 2>&1 || { echo "profile $tag failed"; tail -5 $OUT/bench_${tag}_$round.log; exit 1; }
    python3 - $OUT/${tag}_$round/run_kernel_stats.csv "$tag r$round" <<'P'
import csv, sys
parts = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if ", 4, false, 0, false>" in n or "k_splitk_finish" in n:
        parts.append(f"{'finish' if 'finish' in n else 'gemm'} {float(r['AverageNs']) / 1e3:.2f} us")
print(sys.argv[2], "; ".join(parts))
P
  done
done
