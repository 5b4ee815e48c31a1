"""Where the bf16-split GEMM's time goes (timing only; results are wrong by design): the same
kernel with the A and / or B chunk staging (global loads, split, LDS plane writes) switched off
after the first chunk, in separately built libraries (HG_LIB).  One line per shape and tile."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402

from humanoid import _native as N  # noqa: E402

L = N.lib()
dev = "cuda:0"
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for rows, k, n in ((24576, 705, 512), (24576, 219, 768), (98304, 768, 256)):
    x = torch.randn(rows, k, device=dev)
    W = torch.randn(n, k, device=dev)
    b = torch.randn(n, device=dev)
    y = torch.empty(rows, n, device=dev)
    for tile in (20, 21, 22):
        f = lambda: L.hg_gemm_f32(0, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,  # noqa: E731
                                  y.data_ptr(), y.stride(0), None, rows, n, k, 1, tile, s)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(30):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(os.environ.get("VARIANT"), rows, k, n, tile, round(e0.elapsed_time(e1) / 30 * 1e3, 1), flush=True)
