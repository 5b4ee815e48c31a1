"""The image-fed bf16-split GEMMs of the update at their routed tiles against the same tiles with
A's loads two chunks ahead (hg_gemm_f32_img tiles 29..33 = 20, 21, 22, 23, 28 + APF): us per call
(torch events, REPS launches after a warm-up) and bitwise equality of the outputs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "humanoid-gym-with-comments_amd"))
from humanoid import _native as N  # noqa: E402
from humanoid.algo.ppo import hg_mlp  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
APF = {20: 29, 21: 30, 22: 31, 23: 32, 28: 33}
# (name, mode, rows, k, n, tile)
CASES = [("actor0_fwd", 0, 24576, 705, 512, 20), ("actor1_fwd", 0, 24576, 512, 256, 22),
         ("linvel0_fwd", 0, 24576, 705, 128, 23), ("critic0_fwd", 0, 24576, 219, 768, 21),
         ("critic1_fwd", 0, 24576, 768, 256, 22), ("value0_fwd", 0, 98304, 219, 768, 20),
         ("value1_fwd", 0, 98304, 768, 256, 20), ("value2_fwd", 0, 98304, 256, 128, 20),
         ("actor_dx_256_512", 1, 24576, 256, 512, 28), ("critic_dx_256_768", 1, 24576, 256, 768, 22)]


def main():
    dev = "cuda:0"
    L = N.lib()
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    for name, mode, rows, k, n, tile in CASES:
        x = torch.randn(rows, k, device=dev)
        if mode == 0:
            W = torch.randn(n, k, device=dev) * k ** -0.5
            img = hg_mlp.x6_images([(W, 0, n, k)], dev)[0]
            b = torch.randn(n, device=dev) * 0.1
            y, cp = None, None
        else:
            W = torch.randn(k, n, device=dev) * k ** -0.5  # [k, n]: dx = g W, W^T image
            img = hg_mlp.x6_images([(W, 1, n, k)], dev)[0]
            b = None
            y = torch.nn.functional.elu(torch.randn(rows, n, device=dev))
        res = {"case": name, "rows": rows, "k": k, "n": n}
        outs = {}
        for t in (tile, APF[tile]):
            out = torch.empty(rows, n, device=dev)
            cp = torch.empty(int(L.hg_gemm_colpart_rows(rows, t)), n, device=dev) if mode == 1 else None

            def call():
                N.check(L.hg_gemm_f32_img(mode, x.data_ptr(), x.stride(0), None, img.data_ptr(),
                                          b.data_ptr() if b is not None else None,
                                          y.data_ptr() if y is not None else None, y.stride(0) if y is not None else 0,
                                          out.data_ptr(), out.stride(0), cp.data_ptr() if cp is not None else None,
                                          rows, n, k, 1, t, 0, img.numel() * img.element_size(), s))
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                call()
            e1.record()
            torch.cuda.synchronize()
            res["t%d_us" % t] = round(e0.elapsed_time(e1) * 1e3 / REPS, 2)
            outs[t] = (out.clone(), cp.clone() if cp is not None else None)
        a, c = outs[tile], outs[APF[tile]]
        res["bitwise_equal"] = bool(torch.equal(a[0], c[0]) and (a[1] is None or torch.equal(a[1], c[1])))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
