#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) as MI355X_MICROARCH.md prescribes.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/prof"
mkdir -p "$OUT"
ARGS="--steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"
if [ -n "$NO_PMC" ]; then exit 0; fi
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
echo "pmc fetch ok"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.log"; exit 1; }
echo "pmc write ok"
