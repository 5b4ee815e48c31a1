#!/bin/bash
# Round-3 evidence run: the reference's trained actor closed-loop on hg_sim vs the CPU oracle
# (URDF and MJCF profiles), then a full training run + play + sim2sim of the trained policy on
# physics v4.  Outputs under gpurun_out/r3_onnx and gpurun_out/train_eval.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out/r3_onnx
export TMPDIR=/tmp
for P in urdf mjcf; do
  timeout -k 10 400 python -u scripts/onnx_closed_loop.py --profile $P --duration 5 --envs_per_command 16 \
    --ensemble 2 --out gpurun_out/r3_onnx > gpurun_out/r3_onnx/onnx_$P.log 2>&1 || { tail -20 gpurun_out/r3_onnx/onnx_$P.log; exit 1; }
  tail -9 gpurun_out/r3_onnx/onnx_$P.log
done
ITERS=${ITERS:-3000} TRAIN_TIMEOUT=600 bash scripts/train_eval.sh
