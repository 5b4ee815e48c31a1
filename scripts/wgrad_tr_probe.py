"""Weight gradients dW[n, k] = gh[R, n]^T x[R, k] on k_wgrad_tr (hg_gemm_f32_wgrad tiles 40..45,
row-major operands read through ds_read_b64_tr_b16) against the build's current route (torch.mm /
the split-K bmm of hg_mlp._DW_SPLIT on hipBLASLt).  Per shape: error of every variant vs an f64
product (max |err| / max_j sum_r |gh_rn x_rk|, the 1e-6 bound of tests/test_gpu_gemm.py), the
GEMM time (the split-K chunk sum runs in the batched column-sum launch in both routes and is timed
separately as `sum_us`).  One JSON line per shape on stdout.
    python scripts/wgrad_tr_probe.py            (env WG_SHAPES=512x705,... WG_ROWS=24576)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "humanoid-gym-with-comments_amd"))
from humanoid import _native as N  # noqa: E402
from humanoid.algo.ppo import hg_mlp  # noqa: E402

dev = "cuda:0"
R = int(os.environ.get("WG_ROWS", "24576"))
SHAPES = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("WG_SHAPES", "").split(",") if s] or \
    [(512, 705), (256, 512), (128, 256), (768, 219), (256, 768), (128, 705), (128, 128)]
TILES = [int(v) for v in os.environ.get("WG_TILES", "40,41,42,43,44,45,46,47,48,49,50,51,52,53,54").split(",")]
SPLITS = [int(v) for v in os.environ.get("WG_SPLITS", "8,16,24,32,48,64,96,128").split(",")]


def t_us(f, n=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    L = N.lib()
    from humanoid.utils.blas_tuning import use_tuned_gemms
    tuned = use_tuned_gemms()  # the production GEMM table (lookup only), as the runner loads it
    torch.manual_seed(0)
    s = torch.cuda.current_stream().cuda_stream
    for n, k in SHAPES:
        gh = torch.randn(R, n, device=dev) * 1e-3
        x = torch.nn.functional.elu(torch.randn(R, k, device=dev))
        ref = torch.mm(gh.double().t(), x.double())
        scale = torch.mm(gh.double().abs().t(), x.double().abs()).max().item()
        out = {"shape": f"{n}x{k}", "rows": R, "tunableop_table": tuned}
        out["mm_us"] = round(t_us(lambda: torch.mm(gh.t(), x)), 2)
        # the current route (GEMM part only)
        S0 = hg_mlp._DW_SPLIT.get((n, k), 1) if R >= 8192 else 1
        if S0 > 1:
            ghs, xs = gh.view(S0, R // S0, n).transpose(1, 2), x.view(S0, R // S0, k)
            cur = lambda: torch.bmm(ghs, xs)  # noqa: E731
            val = torch.bmm(ghs, xs).sum(0)
        else:
            cur = lambda: torch.mm(gh.t(), x)  # noqa: E731
            val = torch.mm(gh.t(), x)
        out["current"] = {"S": S0, "us": round(t_us(cur), 2), "err": (val.double() - ref).abs().max().item() / scale}
        best = None
        for tile in TILES:
            for S in SPLITS:
                part = torch.empty(S, n, k, device=dev)

                def run():
                    rc = L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), x.data_ptr(), x.stride(0), part.data_ptr(),
                                             k, n * k, n, k, R, S, 0, tile, s)
                    if rc != 0:
                        raise RuntimeError(f"hg_gemm_f32_wgrad {rc}")
                run()
                torch.cuda.synchronize()
                err = (part.double().sum(0) - ref).abs().max().item() / scale
                us = t_us(run)
                sum_us = t_us(lambda: part.sum(0))
                key = f"t{tile}_S{S}"
                out[key] = {"us": round(us, 2), "sum_us": round(sum_us, 2), "err": err}
                if err < 1e-6 and (best is None or us + sum_us < best[1]):
                    best = (key, us + sum_us)
        out["best"] = best
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
