#!/bin/bash
# K_step development loop on the GPU: physics parity tests, the phase probe (if built) and a short
# bench; stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/kstep_parity.log 2>&1 || { tail -30 gpurun_out/kstep_parity.log; exit 1; }
tail -3 gpurun_out/kstep_parity.log
if [ -f build/kprobe/libhgsim.so ]; then
  timeout -k 10 300 python scripts/dev/kstep_probe.py run > gpurun_out/kstep_phase_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/kstep_phase_probe.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/kstep_phase_probe.txt
fi
timeout -k 10 300 python bench.py > gpurun_out/kstep_bench.json 2> gpurun_out/kstep_bench.err || { tail -20 gpurun_out/kstep_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/kstep_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d.get('roofline'))"
