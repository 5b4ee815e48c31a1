"""Same-box A/B of the MLP GEMMs (round 5): the tree's library against a base build (HG_LIB) —
the batched epilogues (every epilogue load issued up front) and the ring-pipelined forward tiles
(k_gemm_x6r, tiles 30-35).  Each process times every (shape, tile) on seeded inputs (HIP events
over back-to-back launches) and records a sha256 of each output, so two runs compare bit for bit.

  HG_LIB=abpush/libhgsim_base.so python scripts/x6r_probe.py base   -> gpurun_out/x6r_base.json
  python scripts/x6r_probe.py new                               -> gpurun_out/x6r_new.json
  python scripts/x6r_probe.py compare                           -> table + bitwise check
"""
import hashlib
import zlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
OUT = os.path.join(REPO, "gpurun_out")
ITERS = int(os.environ.get("ITERS", "20"))

# (name, mode, rows, k, n, tiles); mode 0 forward (+bias +ELU) with W's image for tiles >= 19,
# mode 1 input grad (ELU backward) with W^T's image for tiles >= 19
CASES = [
    ("actor0 705->512", 0, 24576, 705, 512, [20, 30, 31, 32, 35]),
    ("actor1 512->256", 0, 24576, 512, 256, [22, 30, 31, 33, 34]),
    ("linvel0 705->128", 0, 24576, 705, 128, [29, 30, 31, 33, 34]),
    ("critic0 219->768", 0, 24576, 219, 768, [21, 30, 31, 32]),
    ("critic1 768->256", 0, 24576, 768, 256, [22, 30, 31, 33, 34]),
    ("values0 219->768", 0, 98304, 219, 768, [20, 30, 31, 32]),
    ("values1 768->256", 0, 98304, 768, 256, [20, 30, 31, 32]),
    ("values2 256->128", 0, 98304, 256, 128, [20, 30, 31]),
    ("actor2 256->128", 0, 24576, 256, 128, [5]),
    ("roll0 705->512", 0, 4096, 705, 512, [5]),
    ("roll1 512->256", 0, 4096, 512, 256, [5]),
    ("actor_dx1 256->512", 1, 24576, 256, 512, [28]),
    ("critic_dx1 256->768", 1, 24576, 256, 768, [22]),
    ("actor_dx2 128->256", 1, 24576, 128, 256, [16]),
    ("critic_dx2 128->256", 1, 24576, 128, 256, [16]),
    ("linvel_dx1 128->128", 1, 24576, 128, 128, [5]),
]


# (name, rows, n, k, [(tile, slices)]): tile 0 = torch.mm; 40-48 PF = 1, 49-54 PF = 2 (hg_gemm.hip)
WGRAD = [
    ("dW actor0 512x705", 24576, 512, 705, [(0, 1), (49, 32), (40, 32)]),
    ("dW critic0 256x768", 24576, 256, 768, [(0, 1), (49, 64), (40, 64)]),
    ("dW actor1 256x512", 24576, 256, 512, [(0, 1), (54, 64), (45, 64)]),
    ("dW critic1 768x219", 24576, 768, 219, [(0, 1), (54, 64), (45, 64)]),
    ("dW linvel0 128x705", 24576, 128, 705, [(0, 1), (48, 64)]),
    ("dW actor2 128x256", 24576, 128, 256, [(0, 1), (54, 128)]),
    ("dW critic2 128x256", 24576, 128, 256, [(0, 1), (54, 128)]),
    ("dW 128x128", 24576, 128, 128, [(0, 1), (46, 128), (52, 128)]),
]


def run(tag):
    import torch
    from humanoid import _native as N
    from humanoid.algo.ppo import hg_mlp
    L = N.lib()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, mode, rows, k, n, tiles in CASES:
        g = torch.Generator(device=dev).manual_seed(zlib.crc32(name.encode()) % 100000)
        if mode == 0:
            A = torch.randn(rows, k, device=dev, generator=g)
            W = torch.randn(n, k, device=dev, generator=g) * k ** -0.5
            b = torch.randn(n, device=dev, generator=g) * 0.1
            img = hg_mlp.x6_images([(W, 0, n, k)], dev)[0]
            C = torch.empty(rows, n, device=dev)
        else:  # gh [rows, k] x W [k, n] -> [rows, n], ELU backward from Y [rows, n]
            A = torch.randn(rows, k, device=dev, generator=g)
            W = torch.randn(k, n, device=dev, generator=g) * k ** -0.5
            Y = torch.nn.functional.elu(torch.randn(rows, n, device=dev, generator=g))
            img = hg_mlp.x6_images([(W, 1, n, k)], dev)[0]
            C = torch.empty(rows, n, device=dev)
        for tile in tiles:
            if mode == 0 and tile >= 19:
                fn = lambda: L.hg_gemm_f32_img(0, A.data_ptr(), A.stride(0), None, img.data_ptr(), b.data_ptr(), None, 0,  # noqa: E731
                                               C.data_ptr(), C.stride(0), None, rows, n, k, 1, tile, 0,
                                               img.numel() * img.element_size(), s)
            elif mode == 0:
                fn = lambda: L.hg_gemm_f32(0, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,  # noqa: E731
                                           C.data_ptr(), C.stride(0), None, rows, n, k, 1, tile, s)
            else:
                parts = int(L.hg_gemm_colpart_rows(rows, tile))
                cp = torch.empty(parts, n, device=dev)
                if tile >= 19:
                    fn = lambda: L.hg_gemm_f32_img(1, A.data_ptr(), A.stride(0), None, img.data_ptr(), None, Y.data_ptr(),  # noqa: E731
                                                   Y.stride(0), C.data_ptr(), C.stride(0), cp.data_ptr(), rows, n, k, 1,
                                                   tile, 0, img.numel() * img.element_size(), s)
                else:
                    fn = lambda: L.hg_gemm_f32(1, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), None, Y.data_ptr(),  # noqa: E731
                                               Y.stride(0), C.data_ptr(), C.stride(0), cp.data_ptr(), rows, n, k, 1, tile, s)
            C.zero_()
            rc = fn()
            if rc != 0:
                res[f"{name} t{tile}"] = {"rc": int(rc)}
                continue
            torch.cuda.synchronize()
            h = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
            if mode == 1:
                h += "/" + hashlib.sha256(cp.cpu().numpy().tobytes()).hexdigest()[:16]
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
            tf = 2.0 * rows * k * n / (us * 1e-6) / 1e12
            res[f"{name} t{tile}"] = {"us": round(us, 2), "tflops_f32": round(tf, 1), "sha": h}
            print(f"{tag:5s} {name:22s} tile {tile:2d}: {us:8.2f} us {tf:6.1f} TF/s  {h}", flush=True)
    # weight gradients dW [n, k] = gh^T x on k_wgrad_tr (split-K slices, not summed here) and on
    # torch.mm (hipBLASLt, the committed TunableOp table)
    from humanoid.utils.blas_tuning import use_tuned_gemms
    use_tuned_gemms()
    for name, rows, n, k, tiles in WGRAD:
        g = torch.Generator(device=dev).manual_seed(zlib.crc32(name.encode()) % 100000)
        gh = torch.randn(rows, n, device=dev, generator=g)
        x = torch.randn(rows, k, device=dev, generator=g)
        for tile, S in tiles:
            if tile == 0:
                fn = lambda: torch.mm(gh.t(), x)  # noqa: E731
                outp = None
            else:
                outp = torch.empty(S, n, k, device=dev)
                fn = lambda: L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), x.data_ptr(), x.stride(0), outp.data_ptr(),  # noqa: E731
                                                 k, n * k, n, k, rows, S, 0, tile, s)
            r = fn()
            if outp is not None and r != 0:
                res[f"{name} t{tile}/S{S}"] = {"rc": int(r)}
                continue
            torch.cuda.synchronize()
            h = hashlib.sha256((outp if outp is not None else r).cpu().numpy().tobytes()).hexdigest()[:16]
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
            res[f"{name} t{tile}/S{S}"] = {"us": round(us, 2), "sha": h}
            print(f"{tag:5s} {name:22s} tile {tile:2d} S{S:3d}: {us:8.2f} us  {h}", flush=True)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"x6r_{tag}.json"), "w") as f:
        json.dump(res, f, indent=1)


def compare():
    base = json.load(open(os.path.join(OUT, "x6r_base.json")))
    new = json.load(open(os.path.join(OUT, "x6r_new.json")))
    ref_sha = {}
    for key, r in base.items():
        if "sha" in r:
            if " t0/" not in key:
                ref_sha.setdefault(key.rsplit(" t", 1)[0] + ("/" + key.rsplit("/", 1)[1] if "/S" in key else ""), r["sha"])
    for key, r in new.items():
        b = base.get(key, {})
        name = key.rsplit(" t", 1)[0] + ("/" + key.rsplit("/", 1)[1] if "/S" in key else "")
        same = "sha" in r and r["sha"] == ref_sha.get(name)
        print(f"{key:30s} base {b.get('us', '-'):>8} us  new {r.get('us', '-'):>8} us  "
              f"{'bitwise = base routed tile' if same else 'DIFFERS' if 'sha' in r else r}")


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        compare()
    else:
        run(sys.argv[1])
