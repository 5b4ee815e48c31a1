"""Rollout policy layers (4096 rows) as split-K bf16-split GEMMs (round 5 probe): the shipped route
(hg_gemm_f32 with bias + ELU in the epilogue) against the forward product in S split-K slices
(hg_gemm_f32_wgrad with kmajor=1, i.e. k_gemm_x6 mode 4: C_s = A[:, slice] W[:, slice]^T) plus the
slices' sum + bias + ELU as a separate torch pass (an upper bound for a fused finishing kernel).
HIP events over back-to-back launches; max |difference| against the shipped route.

  python scripts/probes/roll_splitk_probe.py  -> gpurun_out/roll_splitk.json
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
ITERS = int(os.environ.get("ITERS", "50"))
SHAPES = [("roll0 705->512", 4096, 705, 512), ("roll1 512->256", 4096, 512, 256), ("roll2 256->128", 4096, 256, 128)]


def timeit(fn):
    import torch
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


def main():
    import torch
    from humanoid import _native as N
    L = N.lib()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, rows, k, n in SHAPES:
        g = torch.Generator(device=dev).manual_seed(rows + k + n)
        A = torch.randn(rows, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) * k ** -0.5
        b = torch.randn(n, device=dev, generator=g) * 0.1
        C = torch.empty(rows, n, device=dev)
        route = 5  # the rollout's route (hg_mlp.py)
        ship = lambda: L.hg_gemm_f32(0, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,  # noqa: E731
                                     C.data_ptr(), C.stride(0), None, rows, n, k, 1, route, s)
        assert ship() == 0
        torch.cuda.synchronize()
        ref = C.clone()
        us = timeit(ship)
        res[f"{name} shipped (tile {route})"] = {"us": round(us, 2)}
        print(f"{name:16s} shipped tile {route:2d}: {us:7.2f} us", flush=True)
        for tile in (20, 22, 23, 21, 25):
            for S in (2, 3, 4, 6, 8):
                kslice = ((k + S - 1) // S + 15) // 16 * 16
                if (S - 1) * kslice >= k:
                    continue
                out = torch.empty(S, rows, n, device=dev)
                gemm = lambda: L.hg_gemm_f32_wgrad(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0),  # noqa: E731
                                                   out.data_ptr(), n, rows * n, rows, n, k, S, 1, tile, s)
                if gemm() != 0:
                    continue
                fin = lambda: torch.nn.functional.elu(torch.add(out.sum(0), b))  # noqa: E731
                torch.cuda.synchronize()
                err = (fin() - ref).abs().max().item()
                ug, uf = timeit(gemm), timeit(fin)
                res[f"{name} t{tile} S{S}"] = {"gemm_us": round(ug, 2), "finish_us": round(uf, 2), "max_abs_diff": err}
                print(f"{name:16s} t{tile} S{S}: gemm {ug:7.2f} + finish {uf:6.2f} us  (max |d| {err:.2e})", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "roll_splitk.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
