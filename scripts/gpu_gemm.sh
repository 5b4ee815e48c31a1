#!/bin/bash
# GPU session for the learn-phase GEMM work: the GEMM probe, then the -m gpu suite (optional), then
# a short bench.  Stops at the first crash / timeout; never retries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_PROBE" ]; then
timeout -k 10 300 python -u scripts/gemm_probe.py > gpurun_out/gemm_probe.jsonl 2> gpurun_out/gemm_probe.err || { echo "probe failed"; tail -20 gpurun_out/gemm_probe.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/gemm_probe.jsonl'):
    d=json.loads(l)
    if 'shape' in d and d['mode'] == 5: print(d['shape'], ' '.join('%s:%.1f'%(kk[:-3],vv) for kk,vv in d.items() if kk.endswith('_us'))); continue
    if 'shape' in d and d['mode'] == 2: print(d['shape'], 'torch', d['torch_us'], 'best', d['best_us'], d['best'], 'x', d['speedup_vs_torch'], 'rel', d['torch_relerr'], d[d['best']+'_relerr'], 'transp', d['transpose_us'], ' '.join('%s:%.1f'%(kk[:-3],vv) for kk,vv in d.items() if kk.endswith('_us') and kk.startswith('km'))); continue
    if 'shape' in d: print(d['shape'], 'torch', d['torch_us'], 'best', d['best_us'], 'tile', d['best_tile'], 'x', d['speedup_vs_torch'], 'err', '%.2e'%d['tile%d_err'%d['best_tile']], 'terr', '%.2e'%d['torch_err'], 'rel', d.get('tile%d_relerr'%d['best_tile']), d.get('torch_relerr'), ' '.join('%d:%.1f'%(t,d['tile%d_us'%t]) for t in range(1,27) if 'tile%d_us'%t in d), 'm1', ' '.join('%d:%.1f'%(t,d['tile%d_m1_us'%t]) for t in range(19,27) if 'tile%d_m1_us'%t in d))
"
fi
if [ -n "$RUN_TESTS" ]; then SKIP_BENCH=1 bash scripts/gpu_round3.sh || exit $?; fi
if [ -n "$RUN_BENCH" ]; then timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?; tail -1 gpurun_out/bench.log; fi
