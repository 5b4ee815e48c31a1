#!/bin/bash
# K_step same-box A/B (round 5): the -m gpu suite + smoke on the tree's library, then the launch time
# at 256 and 4096 envs for the base build (HG_LIB, default abpush/libhgsim_base.so) and the tree's, the
# SQ counters of the tree's K_step, and a short bench.  Every GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out/kstep_ab
export TMPDIR=/tmp
export HG_TOL_REPORT=${HG_TOL_REPORT:-gpurun_out/tol_report.jsonl}
BASE=${BASE_LIB:-abpush/libhgsim_base.so}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -30
  tail -2 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
  echo "smoke ok"
fi
for round in 1 2; do
  ENVS=256,4096 HG_LIB="$BASE" timeout -k 10 300 python -u scripts/kstep_occupancy.py > gpurun_out/kstep_ab/base_$round.jsonl 2> gpurun_out/kstep_ab/base_$round.err || { echo "base occupancy failed"; tail -5 gpurun_out/kstep_ab/base_$round.err; exit 1; }
  ENVS=256,4096 timeout -k 10 300 python -u scripts/kstep_occupancy.py > gpurun_out/kstep_ab/new_$round.jsonl 2> gpurun_out/kstep_ab/new_$round.err || { echo "new occupancy failed"; tail -5 gpurun_out/kstep_ab/new_$round.err; exit 1; }
done
for f in gpurun_out/kstep_ab/*.jsonl; do echo "$f"; cat "$f"; done
bash scripts/pmc_sq.sh || exit 1
python scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq/sq_counters_k_step.json > /dev/null && python -c "import json; d=json.load(open('gpurun_out/pmc_sq/sq_counters_k_step.json')); print('VALU/wave', d['per_wave']['SQ_INSTS_VALU'], d['fractions_of_wave_cycles'])"
if [ -n "$SKIP_BENCH" ]; then exit 0; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
