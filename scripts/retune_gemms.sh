#!/bin/bash
# Re-tune the TunableOp GEMM table for the current code path (one full PPO run with tuning on),
# then time the pipeline with the fresh table.  Output: gpurun_out/tunableop_results*.csv
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/tunableop_results*.csv
TAG=tune WARM=3 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 1000 python scripts/blas_probe.py > gpurun_out/retune.log 2>&1 || { tail -20 gpurun_out/retune.log; exit 1; }
ls -la gpurun_out/tunableop_results*.csv
grep -h "ms\|warmup" gpurun_out/retune.log
