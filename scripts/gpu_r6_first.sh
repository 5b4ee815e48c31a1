#!/bin/bash
# Round 6, first GPU call: smoke() with its K_step dump (classification of outliers offline), then
# the tests added this round.  Stops at the first step whose exit is not 0/1 (fault, abort, limit).
mkdir -p gpurun_out/r6_smoke
HG_SMOKE_DUMP=gpurun_out/r6_smoke/dump.npz timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/r6_smoke/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -4 gpurun_out/r6_smoke/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo_full.py tests/test_gpu_gemm.py -x -v \
  --timeout 300 --timeout-method thread -k "fk_matches_mjcf or config1 or stacked_image or ppo_update_full or step_physics_parity" \
  > gpurun_out/r6_smoke/pytest_new.log 2>&1
rc2=$?; echo "pytest rc=$rc2"; tail -15 gpurun_out/r6_smoke/pytest_new.log
exit $(( rc > rc2 ? rc : rc2 ))
