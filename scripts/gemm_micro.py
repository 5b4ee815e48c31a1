"""The update's large GEMMs in isolation, for PMC passes (scripts/pmc_gemm.sh): the routed x6
forward 705->512 (tile 20, weight image), the x6 input gradient 256->768 (tile 22, W^T image,
ELU backward), the weight gradient 512x705 on k_wgrad_tr (tile 40, 32 slices; round 5: also the
routed tile 49) and on hipBLASLt (torch.mm, the committed TunableOp table), and (round 5) the
paired first layers 705->640 (tile 25, stacked image, split output), at the 24576-row minibatch;
ITERS launches each.  scripts/gemm_sq_summary.py turns the PMC passes into per-kernel figures."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "humanoid-gym-with-comments_amd"))
from humanoid import _native as N  # noqa: E402
from humanoid.algo.ppo import hg_mlp  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

R = 24576
ITERS = int(os.environ.get("ITERS", "10"))


def main():
    dev = "cuda:0"
    use_tuned_gemms()
    L = N.lib()
    s = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    x = torch.randn(R, 705, device=dev)
    W1, b1 = torch.randn(512, 705, device=dev) * 0.03, torch.zeros(512, device=dev)
    img_f = hg_mlp.x6_images([(W1, 0, 512, 705)], dev)[0]
    g = torch.randn(R, 256, device=dev)
    W2 = torch.randn(256, 768, device=dev) * 0.03
    y = torch.nn.functional.elu(torch.randn(R, 768, device=dev))
    img_d = hg_mlp.x6_images([(W2, 1, 768, 256)], dev)[0]
    gh = torch.randn(R, 512, device=dev)
    out_f = torch.empty(R, 512, device=dev)
    out_d = torch.empty(R, 768, device=dev)
    cp = torch.empty(int(L.hg_gemm_colpart_rows(R, 22)), 768, device=dev)
    part = torch.empty(32, 512, 705, device=dev)
    Wl, bl = torch.randn(128, 705, device=dev) * 0.03, torch.zeros(128, device=dev)
    img_p = hg_mlp.x6_images([("stack", (W1, Wl), 705)], dev)[0]
    out_l = torch.empty(R, 128, device=dev)
    for _ in range(ITERS):
        for img, out in ((img_f, out_f),):
            N.check(L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, img.data_ptr(), b1.data_ptr(), None, 0,
                                      out.data_ptr(), out.stride(0), None, R, 512, 705, 1, 20, 0,
                                      img.numel() * img.element_size(), s))
        N.check(L.hg_gemm_f32_img(1, g.data_ptr(), g.stride(0), None, img_d.data_ptr(), None, y.data_ptr(), y.stride(0),
                                  out_d.data_ptr(), out_d.stride(0), cp.data_ptr(), R, 768, 256, 1, 22, 0,
                                  img_d.numel() * img_d.element_size(), s))
        N.check(L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), x.data_ptr(), x.stride(0), part.data_ptr(), 705,
                                    512 * 705, 512, 705, R, 32, 0, 40, s))
        N.check(L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), x.data_ptr(), x.stride(0), part.data_ptr(), 705,
                                    512 * 705, 512, 705, R, 32, 0, 49, s))
        N.check(L.hg_gemm_f32_img_split(x.data_ptr(), x.stride(0), img_p.data_ptr(), b1.data_ptr(), bl.data_ptr(),
                                        out_f.data_ptr(), 512, out_l.data_ptr(), 128, 512, R, 640, 705, 1, 25,
                                        img_p.numel() * img_p.element_size(), s))
        torch.mm(gh.t(), x)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
