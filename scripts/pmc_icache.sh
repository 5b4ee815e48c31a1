#!/bin/bash
# Instruction-cache counters of K_step (one --pmc pass, --kernel-trace only).  HG_LIB selects a library.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_ic${1:-}"
mkdir -p "$OUT"
export ITERS=5
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv -d "$OUT" -o run -- python3 "$R/scripts/kstep_sweep.py" > "$OUT/log" 2>&1 || { echo "icache pass failed"; tail -5 "$OUT/log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.Counter(); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_step" in r["Kernel_Name"][:24]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print({k: round(v / n[k]) for k, v in tot.items()})
PY
