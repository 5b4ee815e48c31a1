#!/bin/bash
# SQ / GRBM counters of the update's large GEMMs (scripts/gemm_micro.py), separate --pmc passes.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc_gemm"
mkdir -p "$OUT"
export ITERS=5
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS --output-format csv -d "$OUT/p1" -o run -- python3 "$R/scripts/gemm_micro.py" > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail -20 "$OUT/p1.log"; exit 1; }
echo "p1 ok"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$R/scripts/gemm_micro.py" > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail -20 "$OUT/p2.log"; exit 1; }
echo "p2 ok"
