#!/bin/bash
# K_step A/B timing: the product library and each variant library named in $VARIANTS
# (humanoid-gym-with-comments_amd/csrc/libhgsim_rep_<name>.so), 5 PGS sweeps, 4096 envs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export ITERS=5
for round in 1 2; do
  timeout -k 10 120 python scripts/kstep_sweep.py 2>/dev/null | grep pgs | sed "s/^/r$round main /" || exit $?
  for v in $VARIANTS; do
    HG_LIB=humanoid-gym-with-comments_amd/csrc/libhgsim_rep_$v.so timeout -k 10 120 python scripts/kstep_sweep.py 2>/dev/null | grep pgs | sed "s/^/r$round $v /" || exit $?
  done
done
