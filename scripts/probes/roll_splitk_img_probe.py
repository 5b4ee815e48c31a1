"""The rollout's split-K first policy layer (4096 x 705 -> 512) with W as a prebuilt operand image
(hg_gemm_f32_splitk_img, round 6 probe) against the shipped hg_gemm_f32_splitk (W split per
block), per tile and slice count: HIP events over back-to-back calls (GEMM slices + finishing
launch), bitwise comparison with the plain route on the same tile (the occupancy tiles 30 / 31 /
32 against 25 / 22 / 21), and the cost of one image build (paid once per weight update).

  python scripts/probes/roll_splitk_img_probe.py  -> gpurun_out/roll_splitk_img.json
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
ITERS = int(os.environ.get("ITERS", "100"))
BASE = {30: 25, 31: 22, 32: 21}


def timeit(fn):
    import torch
    for _ in range(5):
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
    rows, k, n = 4096, 705, 512
    g = torch.Generator(device=dev).manual_seed(7)
    # the rollout's A: the stacked observation rows (705 wide, a 708-float pitch as the env's window)
    Ap = torch.randn(rows, 708, device=dev, generator=g)
    A = Ap[:, :k]
    W = torch.randn(n, k, device=dev, generator=g) * k ** -0.5
    b = torch.randn(n, device=dev, generator=g) * 0.1
    nb = int(L.hg_gemm_x6_image_bytes(n, k))
    img = torch.empty(nb // 4, device=dev)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    build = lambda: L.hg_gemm_x6_image_jobs((vp * 1)(W.data_ptr()), (i64 * 1)(W.stride(0)), (ctypes.c_int * 1)(0),  # noqa: E731
                                            (i64 * 1)(n), (i64 * 1)(k), (vp * 1)(img.data_ptr()), 1, s)
    assert build() == 0
    res = {"image_build_us": round(timeit(build), 2)}
    print(f"image build: {res['image_build_us']:.2f} us", flush=True)
    plain = {}
    for tile in (20, 21, 22, 23, 25, 27, 28, 30, 31, 32):
        for S in (2, 3, 4, 6, 8):
            kslice = int(L.hg_gemm_splitk_kslice(k, S))
            if (S - 1) * kslice >= k:
                continue
            ws = torch.empty(S * rows * n, device=dev)
            C1, C2 = torch.empty(rows, n, device=dev), torch.empty(rows, n, device=dev)
            bt = BASE.get(tile, tile)
            f_plain = lambda: L.hg_gemm_f32_splitk(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(),  # noqa: E731
                                                   C1.data_ptr(), n, ws.data_ptr(), ws.numel(), rows, n, k, 1, bt, S, s)
            f_img = lambda: L.hg_gemm_f32_splitk_img(A.data_ptr(), A.stride(0), img.data_ptr(), nb, b.data_ptr(),  # noqa: E731
                                                     C2.data_ptr(), n, ws.data_ptr(), ws.numel(), rows, n, k, 1, tile, S, s)
            if f_plain() != 0 or f_img() != 0:
                print(f"t{tile} S{S}: refused", flush=True)
                continue
            torch.cuda.synchronize()
            same = bool(torch.equal(C1, C2))
            if (bt, S) not in plain:
                plain[(bt, S)] = timeit(f_plain)
            ui = timeit(f_img)
            up = plain[(bt, S)]
            res[f"t{tile} S{S}"] = {"plain_us": round(up, 2), "img_us": round(ui, 2), "bitwise": same}
            print(f"t{tile:2d} S{S}: plain (t{bt}) {up:7.2f} us  img {ui:7.2f} us  bitwise {same}", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "roll_splitk_img.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
