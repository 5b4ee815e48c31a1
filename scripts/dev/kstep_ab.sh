R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
HG_LIB=$R/build/phase/base/libhgsim.so OUT=gpurun_out/a.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run > gpurun_out/bits.log 2>&1 || { tail gpurun_out/bits.log; exit 1; }
OUT=gpurun_out/b.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run >> gpurun_out/bits.log 2>&1 || { tail gpurun_out/bits.log; exit 1; }
python scripts/dev/kstep_bits.py compare gpurun_out/a.npz gpurun_out/b.npz
ITERS=5 timeout -k 10 200 python scripts/kstep_sweep.py 2>&1 | grep k_step
HG_LIB=$R/build/phase/base/libhgsim.so ITERS=5 timeout -k 10 200 python scripts/kstep_sweep.py 2>&1 | grep k_step
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "physics or trajectory or determinism" 2>&1 | tail -3
