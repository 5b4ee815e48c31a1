#!/bin/bash
# Same-box comparison of the round-4 final tree (commit bd3a0de, extracted with git archive into
# abpush/r4_tree and built there) and the current tree: the default bench alternating between the two,
# ROUNDS times.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/r4r5"
mkdir -p "$OUT"
for i in $(seq 1 ${ROUNDS:-3}); do
  for t in r4 r5; do
    if [ $t = r4 ]; then d="$R/abpush/r4_tree"; else d="$R"; fi
    (cd "$d" && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline) > "$OUT/bench_${i}_$t.log" 2>&1 \
      || { echo "bench $t failed"; tail -20 "$OUT/bench_${i}_$t.log"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']), d['ms_per_step'], 'learn', d.get('learn_time_s'), 'coll', d.get('collection_time_s'), 'kstep', d['roofline']['avg_launch_ms'])" "$OUT/bench_${i}_$t.log" $t
  done
done
