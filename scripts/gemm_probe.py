"""LDS-staged f32 GEMM with fused epilogues (hg_gemm_f32, csrc/hg_gemm.hip) against the current
learn-phase path on the policy MLPs' shapes:
  forward:    torch addmm + ELU            vs  hg_gemm_f32 mode 0 (bias + ELU in the epilogue)
  input grad: torch mm + hg_mlp_act_backward (ELU backward + bias partials)
                                           vs  hg_gemm_f32 mode 1 (ELU backward + column partials)
Error vs an fp64 reference and time per call (HIP events over back-to-back launches) for every
block tile.  One JSON line per shape, then a summary."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from humanoid import _native as N  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

dev = "cuda:0"
L = N.lib()
print(json.dumps({"tunableop_table_loaded": use_tuned_gemms()}))
torch.manual_seed(0)
ITERS = int(os.environ.get("ITERS", 30))
TILES = [int(t) for t in os.environ.get("TILES", "5,16,17,19,20,21,22,23,24,25,26").split(",")]

FWD = [("actor0_mb", 24576, 705, 512), ("actor1_mb", 24576, 512, 256), ("actor2_mb", 24576, 256, 128),
       ("linvel0_mb", 24576, 705, 128), ("linvel1_mb", 24576, 128, 128),
       ("critic0_mb", 24576, 219, 768), ("critic1_mb", 24576, 768, 256), ("critic2_mb", 24576, 256, 128),
       ("actor0_roll", 4096, 705, 512), ("actor1_roll", 4096, 512, 256), ("linvel0_roll", 4096, 705, 128),
       ("critic0_vals", 98304, 219, 768), ("critic1_vals", 98304, 768, 256), ("critic2_vals", 98304, 256, 128)]
# input grad of layer i: g [M, n_i] x W_i [n_i, k_i] -> [M, k_i], ELU backward from y_{i-1} [M, k_i]
DX = [("actor_dx1", 24576, 256, 512), ("actor_dx2", 24576, 128, 256), ("linvel_dx1", 24576, 128, 128),
      ("critic_dx1", 24576, 256, 768), ("critic_dx2", 24576, 128, 256)]


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


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
    return e0.elapsed_time(e1) * 1e3 / ITERS


def gemm(mode, A, B, bias, Y, C, colpart, M, n, k, act, tile):
    rc = L.hg_gemm_f32(mode, A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0),
                       bias.data_ptr() if bias is not None else None, Y.data_ptr() if Y is not None else None,
                       Y.stride(0) if Y is not None else 0, C.data_ptr(), C.stride(0),
                       colpart.data_ptr() if colpart is not None else None, M, n, k, act, tile, stream())
    if rc != 0:
        raise RuntimeError(f"hg_gemm_f32 rc={rc}")


summary = {}
for tag, rows, k, n in FWD:
    x = torch.randn(rows, k, device=dev)
    W = torch.randn(n, k, device=dev) * (1.0 / k ** 0.5)
    b = torch.randn(n, device=dev) * 0.1
    ref = F.elu(torch.addmm(b.double(), x.double(), W.double().t()))
    scale = x.double().abs() @ W.double().abs().t() + b.double().abs()
    err_t = (F.elu(torch.addmm(b, x, W.t())).double() - ref).abs().max().item()
    t_torch = timeit(lambda: F.elu(torch.addmm(b, x, W.t())))
    t_gemm = timeit(lambda: torch.addmm(b, x, W.t()))
    rec_torch_relerr = ((F.elu(torch.addmm(b, x, W.t())).double() - ref).abs() / scale).max().item()
    flop = 2.0 * rows * k * n
    rec = {"shape": tag, "mode": 0, "rows": rows, "k": k, "n": n, "torch_us": round(t_torch, 2),
           "torch_gemm_only_us": round(t_gemm, 2), "torch_err": err_t, "torch_relerr": rec_torch_relerr,
           "auto_tile": int(L.hg_gemm_tile(0, rows, n, k))}
    best = None
    for tile in TILES:
        y = torch.empty(rows, n, device=dev)
        gemm(0, x, W, b, None, y, None, rows, n, k, 1, tile)
        torch.cuda.synchronize()
        rec[f"tile{tile}_err"] = (y.double() - ref).abs().max().item()
        rec[f"tile{tile}_relerr"] = ((y.double() - ref).abs() / scale).max().item()
        t = timeit(lambda: gemm(0, x, W, b, None, y, None, rows, n, k, 1, tile))
        rec[f"tile{tile}_us"] = round(t, 2)
        rec[f"tile{tile}_tflops"] = round(flop / t * 1e-6, 1)
        if best is None or t < best[1]:
            best = (tile, t)
    rec["best_tile"], rec["best_us"] = best[0], round(best[1], 2)
    rec["speedup_vs_torch"] = round(t_torch / best[1], 3)
    print(json.dumps(rec), flush=True)
    summary[tag] = (rec["torch_us"], rec["best_us"], rec["best_tile"], rec.get(f"tile{rec['auto_tile']}_us"))

for tag, rows, kr, n in DX:
    g = torch.randn(rows, kr, device=dev)
    W = torch.randn(kr, n, device=dev) * (1.0 / kr ** 0.5)
    y = F.elu(torch.randn(rows, n, device=dev))
    d = g.double() @ W.double()
    ref = torch.where(y.double() > 0, d, d * (y.double() + 1))
    ref_cs = ref.sum(0)
    scr = torch.empty(int(L.hg_mlp_act_backward_scratch(rows, n)), device=dev)
    gh = torch.empty(rows, n, device=dev)
    gb = torch.empty(n, device=dev)

    def torch_path():
        gx = torch.mm(g, W)
        rc = L.hg_mlp_act_backward(gx.data_ptr(), y.data_ptr(), gh.data_ptr(), rows, n, gb.data_ptr(),
                                   scr.data_ptr(), stream())
        assert rc == 0

    torch_path()
    torch.cuda.synchronize()
    err_t = (gh.double() - ref).abs().max().item()
    t_torch = timeit(torch_path)
    flop = 2.0 * rows * kr * n
    rec = {"shape": tag, "mode": 1, "rows": rows, "k": kr, "n": n, "torch_us": round(t_torch, 2), "torch_err": err_t,
           "torch_bias_err": (gb.double() - ref_cs).abs().max().item(), "auto_tile": int(L.hg_gemm_tile(1, rows, n, kr))}
    best = None
    Wt = W.t().contiguous()
    rec["wt_transpose_us"] = round(timeit(lambda: W.t().contiguous()), 2)
    for tile in TILES:
        parts = int(L.hg_gemm_colpart_rows(rows, tile))
        cp = torch.empty(parts, n, device=dev)
        out = torch.empty(rows, n, device=dev)
        md, BB = (3, Wt) if tile >= 19 else (1, W)
        if tile >= 19:  # the transposing staging of W as is (mode 1) beside the W^T form
            gemm(1, g, W, None, y, out, cp, rows, n, kr, 1, tile)
            torch.cuda.synchronize()
            rec[f"tile{tile}_m1_us"] = round(timeit(lambda: gemm(1, g, W, None, y, out, cp, rows, n, kr, 1, tile)), 2)
            rec[f"tile{tile}_m1_err"] = (out.double() - ref).abs().max().item()
        gemm(md, g, BB, None, y, out, cp, rows, n, kr, 1, tile)
        torch.cuda.synchronize()
        rec[f"tile{tile}_err"] = (out.double() - ref).abs().max().item()
        rec[f"tile{tile}_bias_err"] = (cp.double().sum(0) - ref_cs).abs().max().item()
        t = timeit(lambda: gemm(md, g, BB, None, y, out, cp, rows, n, kr, 1, tile))
        rec[f"tile{tile}_us"] = round(t, 2)
        rec[f"tile{tile}_tflops"] = round(flop / t * 1e-6, 1)
        if best is None or t < best[1]:
            best = (tile, t)
    rec["best_tile"], rec["best_us"] = best[0], round(best[1], 2)
    rec["speedup_vs_torch"] = round(t_torch / best[1], 3)
    print(json.dumps(rec), flush=True)
    summary[tag] = (rec["torch_us"], rec["best_us"], rec["best_tile"], rec.get(f"tile{rec['auto_tile']}_us"))
# weight gradients dW [n, k] = gh[R, n]^T x[R, k] (R = 24576 minibatch rows): torch's split-K bmm
# path of hg_mlp._weight_grad + the chunk sum, against hg_gemm_f32_wgrad slices + the slice sum
DW = [("actor_dw0", 24576, 512, 705), ("actor_dw1", 24576, 256, 512), ("actor_dw2", 24576, 128, 256),
      ("critic_dw0", 24576, 768, 219), ("critic_dw1", 24576, 256, 768), ("critic_dw2", 24576, 128, 256),
      ("linvel_dw0", 24576, 128, 705), ("linvel_dw1", 24576, 128, 128)]
from humanoid.algo.ppo import hg_mlp  # noqa: E402
DW_TILES = [int(t) for t in os.environ.get("DW_TILES", "20,22,26").split(",")]
for tag, rows, n, k in DW:
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    ref = gh.double().t() @ x.double()
    scale = gh.double().abs().t() @ x.double().abs()
    red = hg_mlp._Reductions()

    def torch_path():
        dw = hg_mlp._weight_grad(gh, x, red)
        red.launch(dev)
        return dw

    dw_t = torch_path()
    torch.cuda.synchronize()
    t_torch = timeit(torch_path)
    rec = {"shape": tag, "mode": 2, "rows": rows, "n": n, "k": k, "torch_us": round(t_torch, 2),
           "torch_err": (dw_t.double() - ref).abs().max().item(),
           "torch_relerr": ((dw_t.double() - ref).abs() / scale).max().item()}
    best = None
    for kmajor in (0, 1):
        for tile in DW_TILES:
            for S in (16, 32, 64):
                part = torch.empty(S, n, k, device=dev)
                dw = torch.empty(n, k, device=dev)

                def ours():
                    if kmajor:
                        A, B = gh.t().contiguous(), x.t().contiguous()  # the transposes, timed with the product
                    else:
                        A, B = gh, x
                    rc = L.hg_gemm_f32_wgrad(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), part.data_ptr(), k,
                                             n * k, n, k, rows, S, kmajor, tile, stream())
                    if rc != 0:
                        raise RuntimeError(f"hg_gemm_f32_wgrad rc={rc}")
                    red.add(part, dw, n * k, S)
                    red.launch(dev)
                    return dw

                out = ours()
                torch.cuda.synchronize()
                t = timeit(ours)
                key = f"km{kmajor}_tile{tile}_S{S}"
                rec[key + "_us"] = round(t, 2)
                rec[key + "_relerr"] = ((out.double() - ref).abs() / scale).max().item()
                if best is None or t < best[1]:
                    best = (key, t)
    rec["transpose_us"] = round(timeit(lambda: (gh.t().contiguous(), x.t().contiguous())), 2)
    rec["best"], rec["best_us"] = best[0], round(best[1], 2)
    rec["best_tile"] = best[0]
    rec["speedup_vs_torch"] = round(t_torch / best[1], 3)
    print(json.dumps(rec), flush=True)
print(json.dumps({"summary_torch_best_tile_auto": summary}))
