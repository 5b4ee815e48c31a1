#!/bin/bash
# Kernel traces of the bench with the split-K rollout layer off (HG_SPLITK_FWD=0) and on for the
# routes in ROUTES (HG_SPLITK_ROUTE "tile,slices"); prints the rollout layer's kernels per route.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/splitk_prof
mkdir -p $OUT
for route in off ${ROUTES:-21,2}; do
  if [ $route = off ]; then export HG_SPLITK_FWD=0; unset HG_SPLITK_ROUTE; else export HG_SPLITK_FWD=1 HG_SPLITK_ROUTE=$route; fi
  tag=${route/,/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$tag.log 2>&1 || { echo "profile $route failed"; tail -5 $OUT/bench_$tag.log; exit 1; }
  python3 - $OUT/$tag/run_kernel_stats.csv $route <<'P'
import csv, sys
tot = 0.0
parts = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if ("k_gemm<64, 64, 2, 2, 32, 1, 0, false, 0, true>" in n) or (", 4, false, 0, false>" in n) or (", 5, true, 0, false>" in n) or "k_splitk_finish" in n:
        us = float(r["AverageNs"]) / 1e3
        tot += us
        parts.append(f"{n.split('(')[2][:60] if n.count('(') > 2 else n[:60]} {us:.2f}")
print(sys.argv[2], f"{tot:.2f} us per rollout step:", "; ".join(parts))
P
done
