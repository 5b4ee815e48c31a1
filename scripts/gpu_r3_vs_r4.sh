#!/bin/bash
# Same-box comparison of the round-3 final tree (commit 1e8d1a9, built into build/r3_tree) and the
# current tree: the default bench alternating between the two, ROUNDS times.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/r3r4"
for i in $(seq 1 ${ROUNDS:-3}); do
  for t in r3 r4; do
    if [ $t = r3 ]; then d="$R/build/r3_tree"; else d="$R"; fi
    (cd "$d" && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline) > "$R/gpurun_out/r3r4/bench_${i}_$t.log" 2>&1 \
      || { echo "bench $t failed"; tail -20 "$R/gpurun_out/r3r4/bench_${i}_$t.log"; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']), d['ms_per_step'], 'learn', d.get('learn_time_s'), 'coll', d.get('collection_time_s'), 'kstep', d['roofline']['avg_launch_ms'])" "$R/gpurun_out/r3r4/bench_${i}_$t.log" $t
  done
done
