"""Weight-gradient GEMMs of the small MLP layers (dW[n,k] = gh[R,n]^T x[R,k], R = 24576): torch.mm
vs a split-K batched form (S row chunks -> bmm -> sum), each with TunableOp tuning enabled in this
process so every variant gets its best kernel.  Prints us per call."""
import os
import sys

import torch

os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "gpurun_out/dw_probe_tunable.csv")
R = 24576
dev = "cuda:0"


def t_us(f, n=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


SHAPES = [tuple(int(v) for v in s.split('x')) for s in os.environ.get('DW_SHAPES', '').split(',') if s] or \
    [(128, 256), (128, 128), (256, 512), (128, 705), (512, 705), (768, 219), (256, 768)]
SPLITS = [int(v) for v in os.environ.get('DW_SPLITS', '2,4,8').split(',')]
for n, k in SHAPES:
    gh = torch.randn(R, n, device=dev)
    x = torch.randn(R, k, device=dev)
    base = t_us(lambda: torch.mm(gh.t(), x))
    ref = torch.mm(gh.t(), x)
    line = f"dW {n}x{k}: mm {base:7.1f} us ({2 * R * n * k / base / 1e6:6.1f} TF/s)"
    for S in SPLITS:
        ghs = gh.view(S, R // S, n).transpose(1, 2)
        xs = x.view(S, R // S, k)
        f = lambda: torch.bmm(ghs, xs).sum(0)  # noqa: E731
        t = t_us(lambda: torch.bmm(ghs, xs))  # the chunk sum runs in the batched end-of-backward launch
        err = (f() - ref).abs().max().item() / ref.abs().max().item()
        line += f" | S={S} {t:7.1f} us (rel err {err:.1e})"
    print(line, flush=True)
