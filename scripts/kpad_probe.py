"""Does padding the first layers' odd reduction widths (critic 219, actor 705) to a multiple of
8/16/32 let hipBLASLt pick faster kernels?  Times addmm (forward), the dX and dW products at the
minibatch (24576) and value-pass (98304) row counts for K in {219, 224, 256} and {705, 708, 712,
720, 736} under the repo's TunableOp table (new shapes tuned on the fly)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402

from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
import torch.cuda.tunable as tun  # noqa: E402
tun.tuning_enable(True)  # shapes missing from the table are tuned here (short budget per shape)
tun.set_max_tuning_iterations(10)
tun.set_max_tuning_duration(30)
dev = "cuda:0"


def t(fn, it=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


for rows, n, ks in ((24576, 768, (219, 224, 256)), (98304, 768, (219, 224, 256)), (24576, 512, (705, 708, 712, 720, 736)),
                    (24576, 128, (705, 708, 712, 720, 736))):
    for k in ks:
        x = torch.randn(rows, k, device=dev)
        W = torch.randn(n, k, device=dev)
        b = torch.randn(n, device=dev)
        g = torch.randn(rows, n, device=dev)
        fwd = t(lambda: torch.addmm(b, x, W.t()))
        dw = t(lambda: torch.mm(g.t(), x))
        print(f"rows {rows} n {n} k {k}: fwd {fwd:7.1f} us ({2 * rows * n * k / fwd * 1e-6:5.1f} TF)  "
              f"dW {dw:7.1f} us ({2 * rows * n * k / dw * 1e-6:5.1f} TF)", flush=True)
