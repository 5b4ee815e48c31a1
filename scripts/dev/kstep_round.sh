#!/bin/bash
# K_step change on the GPU: bitwise A/B against build/phase/base (kstep_ab.sh: bits, timing,
# physics parity), then the phase probe of the tree's K_step (build/kprobe).  Stops at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
bash scripts/dev/kstep_ab.sh || exit $?
if [ -f build/kprobe/libhgsim.so ]; then
  timeout -k 10 300 python scripts/dev/kstep_probe.py run > gpurun_out/kstep_phase_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/kstep_phase_probe.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/kstep_phase_probe.txt
fi
