"""Pipelined bf16-split GEMM probe (k_gemm_x6p, tiles 29..39, csrc/hg_gemm.hip): both operands as
images, NS-stage LDS-DMA pipeline, against the image-fed k_gemm_x6 tiles (19..28) on the policy
MLPs' shapes — forwards (mode 0), input gradients (mode 1) and split-K weight gradients (mode 2).
Times per call (HIP events over back-to-back launches) and bitwise equality with the k_gemm_x6
tile of the same block shape.  One JSON line per (shape, tile)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from humanoid import _native as N  # noqa: E402

dev = "cuda:0"
L = N.lib()
torch.manual_seed(0)
ITERS = int(os.environ.get("ITERS", 20))
BASE = [int(t) for t in os.environ.get("BASE", "19,20,22,25").split(",")]
PIPE = [int(t) for t in os.environ.get("PIPE", "29,30,31,32,33,34,35,36,37,38,39").split(",")]
SAME = {29: 20, 30: 20, 31: 20, 32: 22, 33: 25, 34: 25, 35: 27, 38: 19, 39: 22}
FWD = [("actor0_mb", 24576, 705, 512), ("actor1_mb", 24576, 512, 256), ("linvel0_mb", 24576, 705, 128),
       ("critic0_mb", 24576, 219, 768), ("critic1_mb", 24576, 768, 256), ("actor2_mb", 24576, 256, 128),
       ("critic0_vals", 98304, 219, 768), ("critic1_vals", 98304, 768, 256)]
DX = [("actor_dx1", 24576, 256, 512), ("critic_dx1", 24576, 256, 768), ("actor_dx2", 24576, 128, 256)]
DW = [("actor_dw0", 24576, 512, 705), ("actor_dw1", 24576, 256, 512), ("critic_dw0", 24576, 768, 219),
      ("critic_dw1", 24576, 256, 768), ("linvel_dw0", 24576, 128, 705), ("actor_dw2", 24576, 128, 256)]
SHAPES = os.environ.get("SHAPES")
if SHAPES:
    keep = set(SHAPES.split(","))
    FWD, DX, DW = ([x for x in lst if x[0] in keep] for lst in (FWD, DX, DW))


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def nbytes(t):
    return t.numel() * t.element_size()


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


def ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} rc={rc}")


def image(P, trans, rows, k):
    img = torch.empty(int(L.hg_gemm_x6_image_bytes(rows, k)) // 4, device=dev)
    vp = ctypes.c_void_p
    ck(L.hg_gemm_x6_image_jobs((vp * 1)(P.data_ptr()), (ctypes.c_int64 * 1)(P.stride(0)), (ctypes.c_int * 1)(trans),
                               (ctypes.c_int64 * 1)(rows), (ctypes.c_int64 * 1)(k), (vp * 1)(img.data_ptr()), 1,
                               stream()), "image")
    return img


def run_mode01(tag, mode, rows, k, n):
    x = torch.randn(rows, k, device=dev)
    if mode == 0:
        B, trans = torch.randn(n, k, device=dev) * (1.0 / k ** 0.5), 0
    else:
        B, trans = torch.randn(k, n, device=dev) * (1.0 / k ** 0.5), 1
    b = torch.randn(n, device=dev) * 0.1
    y = F.elu(torch.randn(rows, n, device=dev))
    aimg, bimg = image(x, 0, rows, k), image(B, trans, n, k)
    outs, rec = {}, {"shape": tag, "mode": mode, "rows": rows, "k": k, "n": n}
    flop = 2.0 * rows * n * k
    for tile in BASE + PIPE:
        out = torch.empty(rows, n, device=dev)
        parts = int(L.hg_gemm_colpart_rows(rows, tile if tile <= 28 else SAME.get(tile, 20)))
        cp = torch.empty(max(parts, 1) * 2, n, device=dev) if mode == 1 else None

        def call():
            ck(L.hg_gemm_f32_img(mode, None, 0, aimg.data_ptr(), bimg.data_ptr(), b.data_ptr() if mode == 0 else None,
                                 y.data_ptr() if mode == 1 else None, y.stride(0) if mode == 1 else 0, out.data_ptr(),
                                 out.stride(0), cp.data_ptr() if cp is not None else None, rows, n, k, 1, tile,
                                 nbytes(aimg), nbytes(bimg), stream()), f"tile {tile}")
        try:
            call()
        except RuntimeError as e:
            rec[f"t{tile}"] = str(e)
            continue
        torch.cuda.synchronize()
        outs[tile] = out
        t = timeit(call)
        rec[f"t{tile}_us"] = round(t, 2)
        rec[f"t{tile}_tf"] = round(flop / t / 1e6, 1)
    for p, s in SAME.items():
        if p in outs and s in outs:
            rec[f"t{p}_eq_t{s}"] = bool(torch.equal(outs[p], outs[s]))
    print(json.dumps(rec), flush=True)


def run_dw(tag, rows, n, k):
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    ai, bi = image(gh, 1, n, rows), image(x, 1, k, rows)
    ref = gh.double().t() @ x.double()
    scale = gh.double().abs().t() @ x.double().abs()
    rec = {"shape": tag, "mode": 2, "rows": rows, "n": n, "k": k}
    flop = 2.0 * rows * n * k
    best = None
    for tile in BASE + PIPE:
        for S in (4, 8, 16, 32):
            part = torch.empty(S, n, k, device=dev)

            def call():
                ck(L.hg_gemm_wgrad_img(ai.data_ptr(), bi.data_ptr(), part.data_ptr(), k, n * k, n, k, rows, S, tile,
                                       nbytes(ai), nbytes(bi), stream()), f"wgrad {tile}")
            call()
            torch.cuda.synchronize()
            err = ((part.double().sum(0) - ref).abs() / scale).max().item()
            t = timeit(call)
            key = f"t{tile}_S{S}"
            rec[key + "_us"] = round(t, 2)
            rec[key + "_relerr"] = err
            if best is None or t < best[1]:
                best = (key, t)
    rec["best"], rec["best_us"] = best[0], round(best[1], 2)
    rec["best_tf"] = round(flop / best[1] / 1e6, 1)
    print(json.dumps(rec), flush=True)


for tag, rows, k, n in FWD:
    run_mode01(tag, 0, rows, k, n)
for tag, rows, k, n in DX:
    run_mode01(tag, 1, rows, k, n)
for tag, rows, n, k in DW:
    run_dw(tag, rows, n, k)
