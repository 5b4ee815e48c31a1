#!/bin/bash
# Round 6 GEMM occupancy: the tile sweep, the GEMM / PPO GPU tests, then the same-box bench A/B of
# the occupancy routes (HG_OCC_TILES=0: the round-5 tiles).
mkdir -p gpurun_out/r6_gemm
timeout -k 10 400 python -u scripts/probes/occ_probe.py --out gpurun_out/r6_gemm/occ_sweep.json > gpurun_out/r6_gemm/occ_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/r6_gemm/occ_sweep.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
PYTEST_K="gemm or ppo_full or mlp or paired" VARIANTS="HG_OCC_TILES=0" ROUNDS=3 STEPS=20 bash scripts/gpu_ab.sh
