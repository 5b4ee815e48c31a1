#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=default timeout -k 10 300 python scripts/blas_probe.py > gpurun_out/blas_default.log 2>&1 || exit $?
TAG=rocblas TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python scripts/blas_probe.py > gpurun_out/blas_rocblas.log 2>&1 || exit $?
TAG=tunable WARM=4 PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv timeout -k 10 900 python scripts/blas_probe.py > gpurun_out/blas_tunable.log 2>&1 || exit $?
grep -h "ms\|warmup" gpurun_out/blas_*.log
