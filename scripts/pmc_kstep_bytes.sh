#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$R/gpurun_out/pmck_$c" -o run -- python3 "$R/scripts/kstep_sweep.py" > "$R/gpurun_out/pmck_$c.log" 2>&1 || exit 1
done
python3 - "$R/gpurun_out" <<'PY'
import csv, glob, sys, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for k in ("k_step", "k_post_step"):
        v = [float(r["Counter_Value"]) for f in glob.glob(f"{sys.argv[1]}/pmck_{c}/**/*counter_collection.csv", recursive=True)
             for r in csv.DictReader(open(f)) if k in r["Kernel_Name"][:30]]
        print(c, k, round(sum(v) / max(len(v), 1)), "KB/launch", len(v))
PY
