#!/bin/bash
# Same-box A/B of the weight-gradient routes (HG_WGRAD_TR, hg_mlp.py): the bench with the default
# routes and with extra shapes on k_wgrad_tr, alternated twice.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out/wgrad_ab
for round in 1 2; do
  for sel in 1 256x512 256x512,128x705 256x512,128x705,768x219 all; do
    HG_WGRAD_TR=$sel timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/wgrad_ab/${sel}_$round.log 2>&1 || { echo "bench $sel failed"; tail -5 gpurun_out/wgrad_ab/${sel}_$round.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['learn_time_s'])" gpurun_out/wgrad_ab/${sel}_$round.log "$sel r$round"
  done
done
