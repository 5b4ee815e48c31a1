#!/bin/bash
# Same-box comparison of the round-5 final tree (commit d291d31, extracted with git archive into
# abpush/r5_tree and built there) and the current (round-6) tree: the default bench alternating between the two,
# ROUNDS times.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/r5r6"
mkdir -p "$OUT"
for i in $(seq 1 ${ROUNDS:-3}); do
  for t in r5 r6; do
    if [ $t = r5 ]; then d="$R/abpush/r5_tree"; else d="$R"; fi
    (cd "$d" && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline) > "$OUT/bench_${i}_$t.log" 2>&1 \
      || { echo "bench $t failed"; tail -20 "$OUT/bench_${i}_$t.log"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']), d['ms_per_step'], 'learn', d.get('learn_time_s'), 'coll', d.get('collection_time_s'), 'kstep', d['roofline']['avg_launch_ms'])" "$OUT/bench_${i}_$t.log" $t
  done
done
