#!/bin/bash
# K_step phase costs: each variant library runs one idempotent phase twice per substep
# (-DHG_REP_<PHASE>=2); the launch-time delta vs the product library is that phase's cost.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export ITERS=5
timeout -k 10 120 python scripts/kstep_sweep.py 2>/dev/null | grep pgs | sed 's/^/base /'
for v in KIN CHOL MINV MFMA; do
  HG_LIB=humanoid-gym-with-comments_amd/csrc/libhgsim_rep_$v.so timeout -k 10 120 python scripts/kstep_sweep.py 2>/dev/null | grep pgs | sed "s/^/$v /"
done
