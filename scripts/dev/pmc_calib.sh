#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over build/dev/pmc_calib (scripts/dev/pmc_calib.hip), one counter per pass.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/calib"
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "$R/build/dev/pmc_calib" > "$OUT/fetch.log" 2>&1 || { tail -5 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "$R/build/dev/pmc_calib" > "$OUT/write.log" 2>&1 || { tail -5 "$OUT/write.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
for sub, cn in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == cn:
                acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024)
    for k, v in sorted(acc.items()):
        print(f"{cn:10s} {k:18s} counter bytes/launch {sum(v)/len(v):14.0f}  ratio to 67108864: {sum(v)/len(v)/67108864:.3f}")
PY
