"""Tile sweep of the bf16-split GEMMs including the occupancy variants (k_gemm_x6_occ, tiles 30 /
31 / 32 = tiles 25 / 22 / 21 compiled for 4 / 4 / 6 waves per SIMD), on the shapes of the learn
phase.  Every tile of a case must give the same bits as the case's first tile (the bf16-split
tiles differ in blocking only, not in the per-element products or their order); us per call (HIP
events, 200 calls after 20 warm-up, three interleaved rounds).

Cases (name: kind rows k n [tiles]):
  pair    the paired 705 -> 640 forward (hg_gemm_f32_img_split, bias + ELU)
  fwd     a hidden-layer forward k -> n (hg_gemm_f32_img mode 0, bias + ELU, B image; tiles < 19:
          hg_gemm_f32's f32-MFMA tiles, compared bitwise among themselves)
  dx      an input gradient gh [rows, k] x W [k, n] with the ELU backward and bias partials
          (hg_gemm_f32_img mode 1, W^T image)

  python scripts/probes/occ_probe.py [--cases "pair:24576:705:640:25,30 dx:24576:256:768:22,31"]
                                     [--out gpurun_out/r6_gemm/occ_probe.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))

import torch  # noqa: E402

DEFAULT = ("pair:24576:705:640:25,30 dx:24576:256:768:22,31 fwd:24576:219:768:21,32 "
           "fwd:24576:768:256:22,31,21,32,20 dx:24576:256:512:28,31,22,21 fwd:98304:219:768:20,21,32 "
           "fwd:98304:768:256:20,21,32,22,31")


def timeit(fn, reps=200):
    for _ in range(20):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def build(case, L, hg_mlp, dev, s):
    kind, rows, k, n, tiles = case.split(":")
    rows, k, n = int(rows), int(k), int(n)
    tiles = [int(t) for t in tiles.split(",")]
    torch.manual_seed(rows + k + n)
    calls, outs = {}, {}
    if kind == "pair":
        ma, mb = 512, n - 512
        x = torch.randn(rows, k, device=dev)
        Wa, Wb = torch.randn(ma, k, device=dev) * 0.04, torch.randn(mb, k, device=dev) * 0.04
        ba, bb = torch.randn(ma, device=dev) * 0.1, torch.randn(mb, device=dev) * 0.1
        img = hg_mlp.x6_images([("stack", (Wa, Wb), k)], x.device)[0]
        for t in tiles:
            ha, hb = torch.empty(rows, ma, device=dev), torch.empty(rows, mb, device=dev)

            def f(t=t, ha=ha, hb=hb):
                assert L.hg_gemm_f32_img_split(x.data_ptr(), x.stride(0), img.data_ptr(), ba.data_ptr(), bb.data_ptr(),
                                               ha.data_ptr(), ma, hb.data_ptr(), mb, ma, rows, n, k, 1, t,
                                               img.numel() * img.element_size(), s) == 0
            calls[t], outs[t] = f, (ha, hb)
    elif kind == "fwd":
        x = torch.randn(rows, k, device=dev)
        W, b = torch.randn(n, k, device=dev) / k ** 0.5, torch.randn(n, device=dev) * 0.1
        img = hg_mlp.x6_images([(W, 0, n, k)], x.device)[0]
        for t in tiles:
            out = torch.empty(rows, n, device=dev)

            def f(t=t, out=out):
                if t < 19:  # the f32-MFMA tiles (no image)
                    assert L.hg_gemm_f32(0, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,
                                         out.data_ptr(), out.stride(0), None, rows, n, k, 1, t, s) == 0
                    return
                assert L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, img.data_ptr(), b.data_ptr(), None, 0,
                                         out.data_ptr(), out.stride(0), None, rows, n, k, 1, t, 0,
                                         img.numel() * img.element_size(), s) == 0
            calls[t], outs[t] = f, (out,)
    else:  # dx
        gh = torch.randn(rows, k, device=dev)
        W = torch.randn(k, n, device=dev) / k ** 0.5
        y_prev = torch.nn.functional.elu(torch.randn(rows, n, device=dev))
        img = hg_mlp.x6_images([(W, 1, n, k)], gh.device)[0]
        for t in tiles:
            out = torch.empty(rows, n, device=dev)
            cp = torch.empty(int(L.hg_gemm_colpart_rows(rows, t)), n, device=dev)

            def f(t=t, out=out, cp=cp):
                if t < 19:
                    assert L.hg_gemm_f32(1, gh.data_ptr(), gh.stride(0), W.data_ptr(), W.stride(0), None,
                                         y_prev.data_ptr(), y_prev.stride(0), out.data_ptr(), out.stride(0),
                                         cp.data_ptr(), rows, n, k, 1, t, s) == 0
                    return
                assert L.hg_gemm_f32_img(1, gh.data_ptr(), gh.stride(0), None, img.data_ptr(), None, y_prev.data_ptr(),
                                         y_prev.stride(0), out.data_ptr(), out.stride(0), cp.data_ptr(), rows, n, k, 1,
                                         t, 0, img.numel() * img.element_size(), s) == 0
            calls[t], outs[t] = f, (out,)
    for t in tiles:
        calls[t]()
    torch.cuda.synchronize()
    t0 = tiles[0]
    # f32-MFMA and bf16-split tiles differ in rounding: compare within each family only
    fam = lambda t: t >= 19  # noqa: E731
    same = all(all(torch.equal(a, b) for a, b in zip(outs[next(u for u in tiles if fam(u) == fam(t))], outs[t]))
               for t in tiles)
    return calls, same


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=os.environ.get("OCC_CASES", DEFAULT))
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from humanoid import _native as N
    from humanoid.algo.ppo import hg_mlp
    L = N.lib()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for case in args.cases.split():
        calls, same = build(case, L, hg_mlp, dev, s)
        us = {t: [] for t in calls}
        for _ in range(3):
            for t, f in calls.items():
                us[t].append(round(timeit(f), 2))
        out[case] = {"bitwise_equal": bool(same), "us": {str(t): v for t, v in us.items()},
                     "best": str(min(us, key=lambda t: min(us[t])))}
        print(case, json.dumps(out[case]), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
