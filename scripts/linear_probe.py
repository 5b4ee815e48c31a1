"""Fused Linear + bias + ELU forward (hg_linear_act_forward, csrc/hg_linear.hip) against torch's
addmm + ELU on the policy MLPs' hidden-layer shapes: error vs an fp64 reference and time per call
(HIP events over many back-to-back launches) for every wave tile.  Output: one JSON line per shape
plus a summary, written to stdout."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from humanoid import _native as N  # noqa: E402

dev = "cuda:0"
L = N.lib()
torch.manual_seed(0)

# (tag, rows, k, n): learn-phase minibatch (24576 rows), rollout inference (4096 rows), the
# critic's batched value pass (4096 x 24 rows)
SHAPES = [("actor0_mb", 24576, 705, 512), ("actor1_mb", 24576, 512, 256), ("actor2_mb", 24576, 256, 128),
          ("linvel0_mb", 24576, 705, 128), ("linvel1_mb", 24576, 128, 128),
          ("critic0_mb", 24576, 219, 768), ("critic1_mb", 24576, 768, 256), ("critic2_mb", 24576, 256, 128),
          ("actor0_roll", 4096, 705, 512), ("actor1_roll", 4096, 512, 256), ("actor2_roll", 4096, 256, 128),
          ("linvel0_roll", 4096, 705, 128), ("linvel1_roll", 4096, 128, 128),
          ("critic0_vals", 98304, 219, 768), ("critic1_vals", 98304, 768, 256), ("critic2_vals", 98304, 256, 128)]
ITERS = int(os.environ.get("ITERS", 50))
TILES = [int(t) for t in os.environ.get("TILES", "1,2,3,4,5").split(",")]


def ours(x, W, b, y, tile):
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.hg_linear_act_forward(x.data_ptr(), x.stride(0), W.data_ptr(), b.data_ptr(), y.data_ptr(), y.stride(0),
                                 x.shape[0], W.shape[0], W.shape[1], 1, tile, s)
    if rc != 0:
        raise RuntimeError(f"hg_linear_act_forward rc={rc}")
    return y


def timeit(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / ITERS  # us


summary = {}
for tag, rows, k, n in SHAPES:
    x = torch.randn(rows, k, device=dev)
    W = torch.randn(n, k, device=dev) * (1.0 / k ** 0.5)
    b = torch.randn(n, device=dev) * 0.1
    ref = F.elu(torch.addmm(b.double(), x.double(), W.double().t()))
    y_t = F.elu(torch.addmm(b, x, W.t()))
    scale = (x.double().abs() @ W.double().abs().t()).max().item()
    err_t = (y_t.double() - ref).abs().max().item()
    t_torch = timeit(lambda: F.elu(torch.addmm(b, x, W.t())))
    rec = {"shape": tag, "rows": rows, "k": k, "n": n, "torch_us": round(t_torch, 2), "torch_err": err_t,
           "auto_tile": int(L.hg_linear_act_tile(rows, n, k))}
    flop = 2.0 * rows * k * n
    best = None
    for tile in TILES:
        y = torch.empty(rows, n, device=dev)
        ours(x, W, b, y, tile)
        torch.cuda.synchronize()
        err = (y.double() - ref).abs().max().item()
        t = timeit(lambda: ours(x, W, b, y, tile))
        rec[f"tile{tile}_us"] = round(t, 2)
        rec[f"tile{tile}_err"] = err
        rec[f"tile{tile}_tflops"] = round(flop / t * 1e-6, 1)
        if best is None or t < best[1]:
            best = (tile, t)
    rec["err_scale"] = scale
    rec["best_tile"], rec["best_us"] = best[0], round(best[1], 2)
    rec["speedup_vs_torch"] = round(t_torch / best[1], 3)
    rec["torch_tflops_gemm_plus_elu"] = round(flop / t_torch * 1e-6, 1)
    print(json.dumps(rec), flush=True)
    summary[tag] = (rec["torch_us"], rec["best_us"], rec["best_tile"], rec[f"tile{rec['auto_tile']}_us"])
print(json.dumps({"summary_torch_best_tile_auto": summary}))
