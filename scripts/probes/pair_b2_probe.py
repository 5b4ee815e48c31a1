"""A/B of the stacked 705 -> 640 forward (the actor's and lin-vel estimator's first layers, 24576
rows; hg_gemm_f32_img_split) on tile 25 (k_gemm_x6, one block per CU) against tile 30 (the same
body as k_gemm_x6_b2, held to 128 registers: two blocks per CU).  Outputs must be bit-identical;
prints us per call (HIP events, 200 calls after 20 warm-up), interleaved A/B/A/B.

  python scripts/probes/pair_b2_probe.py [--rows 24576] [--out gpurun_out/pair_b2.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--tiles", default="25,30")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from humanoid import _native as N
    from humanoid.algo.ppo import hg_mlp
    torch.manual_seed(3)
    dev = "cuda:0"
    rows, K, ma, mb = args.rows, 705, 512, 128
    x = torch.randn(rows, K, device=dev)
    Wa, Wb = torch.randn(ma, K, device=dev) * 0.04, torch.randn(mb, K, device=dev) * 0.04
    ba, bb = torch.randn(ma, device=dev) * 0.1, torch.randn(mb, device=dev) * 0.1
    img = hg_mlp.x6_images([("stack", (Wa, Wb), K)], x.device)[0]
    s = torch.cuda.current_stream().cuda_stream
    L = N.lib()
    tiles = [int(t) for t in args.tiles.split(",")]
    outs = {}

    def call(tile, ha, hb):
        rc = L.hg_gemm_f32_img_split(x.data_ptr(), x.stride(0), img.data_ptr(), ba.data_ptr(), bb.data_ptr(), ha.data_ptr(),
                                     ma, hb.data_ptr(), mb, ma, rows, ma + mb, K, 1, tile, img.numel() * img.element_size(), s)
        assert rc == 0, rc

    for t in tiles:
        ha = torch.empty(rows, ma, device=dev)
        hb = torch.empty(rows, mb, device=dev)
        call(t, ha, hb)
        torch.cuda.synchronize()
        outs[t] = (ha, hb)
    same = all(torch.equal(outs[t][0], outs[tiles[0]][0]) and torch.equal(outs[t][1], outs[tiles[0]][1]) for t in tiles)
    ref = torch.nn.functional.elu(x.double() @ torch.cat([Wa, Wb]).double().t() + torch.cat([ba, bb]).double())
    err = (torch.cat(outs[tiles[0]], 1).double() - ref).abs().max().item()
    res = {t: [] for t in tiles}
    for rep in range(3):
        for t in tiles:
            ha, hb = outs[t]
            for _ in range(20):
                call(t, ha, hb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                call(t, ha, hb)
            e1.record()
            torch.cuda.synchronize()
            res[t].append(e0.elapsed_time(e1) / 200 * 1e3)
    flop = 2.0 * rows * K * (ma + mb)
    out = {"rows": rows, "bitwise_equal": bool(same), "max_abs_err_vs_f64": err,
           "us": {str(t): [round(v, 2) for v in res[t]] for t in tiles},
           "tflops_f32": {str(t): round(flop / (min(res[t]) * 1e-6) / 1e12, 1) for t in tiles}}
    print(json.dumps(out))
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
