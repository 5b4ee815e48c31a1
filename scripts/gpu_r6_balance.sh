#!/bin/bash
# Round 6: K_step wave balancing (HG_WAVE_BALANCE).  (1) bits: 40 steps x 4096 envs with and without
# it, every physics field compared (results must not depend on which env shares a wave); (2) the
# physics parity tests; (3) same-box bench A/B.  Stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/r6_balance
STEPS=40 HG_WAVE_BALANCE=0 OUT=gpurun_out/r6_balance/a.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run > gpurun_out/r6_balance/bits.log 2>&1 || { tail gpurun_out/r6_balance/bits.log; exit 1; }
STEPS=40 HG_WAVE_BALANCE=1 OUT=gpurun_out/r6_balance/b.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run >> gpurun_out/r6_balance/bits.log 2>&1 || { tail gpurun_out/r6_balance/bits.log; exit 1; }
python scripts/dev/kstep_bits.py compare gpurun_out/r6_balance/a.npz gpurun_out/r6_balance/b.npz | tee gpurun_out/r6_balance/bits_compare.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_distributed.py -k "physics or trajectory or determinism or parity or shard or contact or balancing" > gpurun_out/r6_balance/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r6_balance/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r6_balance/pytest.log | head; exit $rc; }
VARIANTS="HG_WAVE_BALANCE=0" ROUNDS=3 STEPS=20 bash scripts/gpu_ab.sh
