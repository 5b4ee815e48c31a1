"""Operand-image probe for the bf16-split GEMM (csrc/hg_gemm.hip): per policy-MLP shape and x6
tile, hg_gemm_f32 (operands staged + split per block) against hg_gemm_f32_img with B from its
image (split once, copied to LDS by LDS-DMA) and with both A and B from images; and the weight
gradients (hg_gemm_wgrad_img from two reduction-major images, split-K) against the current torch
path.  Reports the times, the image builds, and whether the outputs (and, for the input grad, the
column partials) are bitwise equal.  One JSON line per (shape, tile)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from humanoid import _native as N  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()  # torch's weight-gradient GEMMs on the bench's tuned kernels
dev = "cuda:0"
L = N.lib()
torch.manual_seed(0)
ITERS = int(os.environ.get("ITERS", 30))
TILES = [int(t) for t in os.environ.get("TILES", "19,20,21,22,23,24,25,26").split(",")]
FWD = [("actor0_mb", 24576, 705, 512), ("actor1_mb", 24576, 512, 256), ("linvel0_mb", 24576, 705, 128),
       ("critic0_mb", 24576, 219, 768), ("critic1_mb", 24576, 768, 256), ("actor2_mb", 24576, 256, 128),
       ("actor0_roll", 4096, 705, 512), ("actor1_roll", 4096, 512, 256), ("actor2_roll", 4096, 256, 128),
       ("critic0_vals", 98304, 219, 768), ("critic1_vals", 98304, 768, 256), ("critic2_vals", 98304, 256, 128)]

DX = [("actor_dx1", 24576, 256, 512), ("actor_dx2", 24576, 128, 256), ("critic_dx1", 24576, 256, 768),
      ("critic_dx2", 24576, 128, 256), ("linvel_dx1", 24576, 128, 128)]
FWD = [f for f in FWD if not os.environ.get("SHAPES") or f[0] in os.environ["SHAPES"].split(",")]
DX = [f for f in DX if not os.environ.get("SHAPES") or f[0] in os.environ["SHAPES"].split(",")]


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


def nbytes(t):
    return t.numel() * t.element_size()


def ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} rc={rc}")


def image(P, trans, rows, k, img=None):
    if img is None:
        img = torch.empty(int(L.hg_gemm_x6_image_bytes(rows, k)) // 4, device=dev)
    vp = ctypes.c_void_p
    ck(L.hg_gemm_x6_image_jobs((vp * 1)(P.data_ptr()), (ctypes.c_int64 * 1)(P.stride(0)), (ctypes.c_int * 1)(trans),
                               (ctypes.c_int64 * 1)(rows), (ctypes.c_int64 * 1)(k), (vp * 1)(img.data_ptr()), 1,
                               stream()), "image")
    return img


for tag, rows, k, n in FWD:
    x = torch.randn(rows, k, device=dev)
    W = torch.randn(n, k, device=dev) * (1.0 / k ** 0.5)
    b = torch.randn(n, device=dev) * 0.1
    for tile in TILES:
        y0 = torch.empty(rows, n, device=dev)
        y1 = torch.empty(rows, n, device=dev)

        def plain():
            ck(L.hg_gemm_f32(0, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,
                             y0.data_ptr(), y0.stride(0), None, rows, n, k, 1, tile, stream()), "plain")

        img = image(W, 0, n, k)
        aimg = image(x, 0, rows, k)
        y2 = torch.empty(rows, n, device=dev)

        def imaged():
            ck(L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, img.data_ptr(), b.data_ptr(), None, 0,
                                 y1.data_ptr(), y1.stride(0), None, rows, n, k, 1, tile, 0, nbytes(img), stream()),
               "img")

        def imaged2():
            ck(L.hg_gemm_f32_img(0, None, 0, aimg.data_ptr(), img.data_ptr(), b.data_ptr(), None, 0,
                                 y2.data_ptr(), y2.stride(0), None, rows, n, k, 1, tile, nbytes(aimg), nbytes(img),
                                 stream()), "img2")

        plain()
        imaged()
        imaged2()
        torch.cuda.synchronize()
        rec = {"shape": tag, "mode": 0, "rows": rows, "k": k, "n": n, "tile": tile,
               "bitwise_equal": bool(torch.equal(y0, y1) and torch.equal(y0, y2)), "plain_us": round(timeit(plain), 2),
               "img_us": round(timeit(imaged), 2), "img2_us": round(timeit(imaged2), 2),
               "image_build_us": round(timeit(lambda: image(W, 0, n, k, img)), 2),
               "a_image_build_us": round(timeit(lambda: image(x, 0, rows, k, aimg)), 2)}
        if tile == TILES[0]:  # the f32-MFMA 64x64 tile (the small-row route) for reference
            rec["tile5_us"] = round(timeit(lambda: ck(L.hg_gemm_f32(
                0, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0, y0.data_ptr(),
                y0.stride(0), None, rows, n, k, 1, 5, stream()), "t5")), 2)
        print(json.dumps(rec), flush=True)

for tag, rows, kr, n in DX:
    g = torch.randn(rows, kr, device=dev)
    W = torch.randn(kr, n, device=dev) * (1.0 / kr ** 0.5)
    y = F.elu(torch.randn(rows, n, device=dev))
    for tile in TILES:
        parts = int(L.hg_gemm_colpart_rows(rows, tile))
        o0, o1 = torch.empty(rows, n, device=dev), torch.empty(rows, n, device=dev)
        c0, c1 = torch.empty(parts, n, device=dev), torch.empty(parts, n, device=dev)

        def plain():
            ck(L.hg_gemm_f32(1, g.data_ptr(), g.stride(0), W.data_ptr(), W.stride(0), None, y.data_ptr(), y.stride(0),
                             o0.data_ptr(), o0.stride(0), c0.data_ptr(), rows, n, kr, 1, tile, stream()), "plain")

        img = image(W, 1, n, kr)

        def imaged():
            ck(L.hg_gemm_f32_img(1, g.data_ptr(), g.stride(0), None, img.data_ptr(), None, y.data_ptr(), y.stride(0),
                                 o1.data_ptr(), o1.stride(0), c1.data_ptr(), rows, n, kr, 1, tile, 0, nbytes(img), stream()), "img")

        plain()
        imaged()
        torch.cuda.synchronize()
        rec = {"shape": tag, "mode": 1, "rows": rows, "k": kr, "n": n, "tile": tile,
               "bitwise_equal": bool(torch.equal(o0, o1) and torch.equal(c0, c1)),
               "plain_us": round(timeit(plain), 2), "img_us": round(timeit(imaged), 2),
               "image_build_us": round(timeit(lambda: image(W, 1, n, kr, img)), 2)}
        # the f32 tile 16 (the routed input-grad tile) for reference
        if tile == TILES[0]:
            p16 = int(L.hg_gemm_colpart_rows(rows, 16))
            c16 = torch.empty(p16, n, device=dev)
            rec["tile16_us"] = round(timeit(lambda: ck(L.hg_gemm_f32(
                1, g.data_ptr(), g.stride(0), W.data_ptr(), W.stride(0), None, y.data_ptr(), y.stride(0),
                o0.data_ptr(), o0.stride(0), c16.data_ptr(), rows, n, kr, 1, 16, stream()), "t16")), 2)
        print(json.dumps(rec), flush=True)

# weight gradients dW [n, k] = gh [R, n]^T x [R, k]: torch (hg_mlp._weight_grad: split-K bmm +
# the chunk sum) against two reduction-major images + hg_gemm_wgrad_img slices + the slice sum
from humanoid.algo.ppo import hg_mlp  # noqa: E402
DW = [("actor_dw0", 24576, 512, 705), ("actor_dw1", 24576, 256, 512), ("actor_dw2", 24576, 128, 256),
      ("critic_dw0", 24576, 768, 219), ("critic_dw1", 24576, 256, 768), ("linvel_dw0", 24576, 128, 705),
      ("linvel_dw1", 24576, 128, 128)]
DW_TILES = [int(t) for t in os.environ.get("DW_TILES", "19,20,21,22,23,25").split(",")]
for tag, rows, n, k in ([] if os.environ.get("SKIP_DW") else DW):
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    ref = gh.double().t() @ x.double()
    scale = gh.double().abs().t() @ x.double().abs()
    red = hg_mlp._Reductions()

    def torch_path():
        dw = hg_mlp._weight_grad(gh, x, red)
        red.launch(dev)
        return dw

    torch_path()
    torch.cuda.synchronize()
    rec = {"shape": tag, "mode": 2, "rows": rows, "n": n, "k": k, "torch_us": round(timeit(torch_path), 2)}
    ai, bi = image(gh, 1, n, rows), image(x, 1, k, rows)
    rec["images_us"] = round(timeit(lambda: (image(gh, 1, n, rows, ai), image(x, 1, k, rows, bi))), 2)
    best = None
    for tile in DW_TILES:
        for S in (4, 8, 16, 32):
            part = torch.empty(S, n, k, device=dev)
            dw = torch.empty(n, k, device=dev)

            def ours():
                ck(L.hg_gemm_wgrad_img(ai.data_ptr(), bi.data_ptr(), part.data_ptr(), k, n * k, n, k, rows, S, tile, nbytes(ai), nbytes(bi),
                                       stream()), "wgrad_img")
                red.add(part, dw, n * k, S)
                red.launch(dev)

            ours()
            torch.cuda.synchronize()
            key = f"tile{tile}_S{S}"
            rec[key + "_relerr"] = ((dw.double() - ref).abs() / scale).max().item()
            t = timeit(ours)
            rec[key + "_us"] = round(t, 2)
            if best is None or t < best[1]:
                best = (key, t)
    rec["best"], rec["best_us"] = best[0], round(best[1], 2)
    rec["best_plus_images_us"] = round(best[1] + rec["images_us"], 2)
    print(json.dumps(rec), flush=True)
