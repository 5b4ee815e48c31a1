"""Every bf16-split image tile (hg_gemm_f32_img tiles 20-29) on the learn phase's routed GEMM shapes
at 24576 rows, timed on the tree's library (HIP events over back-to-back launches), to re-check the
routing tables of hg_mlp.py after kernel changes.  Writes gpurun_out/gemm_tile_sweep.json."""
import json
import os
import sys
import zlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
ITERS = int(os.environ.get("ITERS", "20"))
# (name, mode, rows, k, n): mode 0 forward (+bias +ELU), mode 1 input grad (ELU backward)
SHAPES = [("actor0 705->512", 0, 24576, 705, 512), ("actor1 512->256", 0, 24576, 512, 256),
          ("linvel0 705->128", 0, 24576, 705, 128), ("critic0 219->768", 0, 24576, 219, 768),
          ("critic1 768->256", 0, 24576, 768, 256), ("fused0 705->640", 0, 24576, 705, 640),
          ("actor_dx1 256->512", 1, 24576, 256, 512), ("critic_dx1 256->768", 1, 24576, 256, 768),
          ("roll actor0 705->512", 0, 4096, 705, 512), ("roll actor1 512->256", 0, 4096, 512, 256),
          ("roll actor2 256->128", 0, 4096, 256, 128)]
SHAPES = [s for s in SHAPES if os.environ.get("ONLY", "") in s[0]]


def main():
    import torch
    from humanoid import _native as N
    from humanoid.algo.ppo import hg_mlp
    L = N.lib()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, mode, rows, k, n in SHAPES:
        g = torch.Generator(device=dev).manual_seed(zlib.crc32(name.encode()) % 100000)
        A = torch.randn(rows, k, device=dev, generator=g)
        if mode == 0:
            W = torch.randn(n, k, device=dev, generator=g) * k ** -0.5
            b = torch.randn(n, device=dev, generator=g) * 0.1
            img = hg_mlp.x6_images([(W, 0, n, k)], dev)[0]
        else:
            W = torch.randn(k, n, device=dev, generator=g) * k ** -0.5
            Y = torch.nn.functional.elu(torch.randn(rows, n, device=dev, generator=g))
            img = hg_mlp.x6_images([(W, 1, n, k)], dev)[0]
        C = torch.empty(rows, n, device=dev)
        for tile in range(1, 30):
            if tile < 19 and rows > 8192:
                continue
            if tile == 19:
                continue
            if tile < 19:
                fn = lambda: L.hg_gemm_f32(0, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,  # noqa: E731
                                           C.data_ptr(), C.stride(0), None, rows, n, k, 1, tile, s)
            elif mode == 0:
                fn = lambda: L.hg_gemm_f32_img(0, A.data_ptr(), A.stride(0), None, img.data_ptr(), b.data_ptr(), None, 0,  # noqa: E731
                                               C.data_ptr(), C.stride(0), None, rows, n, k, 1, tile, 0,
                                               img.numel() * img.element_size(), s)
            else:
                parts = int(L.hg_gemm_colpart_rows(rows, tile))
                cp = torch.empty(max(parts, 1), n, device=dev)
                fn = lambda: L.hg_gemm_f32_img(1, A.data_ptr(), A.stride(0), None, img.data_ptr(), None, Y.data_ptr(),  # noqa: E731
                                               Y.stride(0), C.data_ptr(), C.stride(0), cp.data_ptr(), rows, n, k, 1,
                                               tile, 0, img.numel() * img.element_size(), s)
            rc = fn()
            if rc != 0:
                continue
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(ITERS):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / ITERS
            res[f"{name} t{tile}"] = round(us, 2)
            print(f"{name:22s} tile {tile}: {us:8.2f} us", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "gemm_tile_sweep.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
