"""hg_gemm_f32 (csrc/hg_gemm.hip): the LDS-staged f32 GEMM of the hidden layers with the layer's
elementwise work in its epilogue (actor_critic.py:36-149, nn.Linear followed by nn.ELU), against an
fp64 reference of the same op, and the MLP backward that uses it against torch autograd.

Stated tolerance: exact f32 products with f32 accumulation in a permuted k order, so per element
|y - y_64| <= 1e-6 * (sum_k |a_k b_k| + |bias|) (the bound of tests/test_gpu_linear.py); the ELU
backward multiplies by elu'(y) <= 1, so the input-gradient bound is the product's; the bias
gradient (column sums of the input gradient, per-tile partials reduced in fixed order) within
1e-6 * sum_r |gh_r| + 1e-6 * rows of the bound.  Every block tile is exercised on the policy
shapes, ragged rows / columns / k, strided operands, and 4-byte-aligned 705-wide rows."""
import ctypes
import os
import sys

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "humanoid-gym-with-comments_amd"))

pytestmark = pytest.mark.gpu

REL = 1e-6
TILES = list(range(1, 30))  # 1..18 f32 MFMA, 19..29 bf16-split (6-term; 29 = 23 with A two chunks ahead)


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# (rows, k, n, lda pad): hidden-layer shapes (705 / 219-wide observations: 4-byte-aligned rows),
# ragged rows / columns / k, strided input
CASES = [(3001, 705, 512, 0), (4096, 512, 256, 0), (24576, 128, 128, 0), (777, 219, 768, 0), (33, 7, 5, 0),
         (1, 705, 128, 0), (130, 64, 96, 3), (200, 36, 40, 4), (65, 33, 129, 0)]


@pytest.mark.parametrize("rows,k,n,pad", CASES)
def test_gemm_forward_matches_fp64(rows, k, n, pad):
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + k + n)
    dev = "cuda:0"
    xs = torch.randn(rows, k + pad, device=dev)
    x = xs[:, :k]
    W = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev) * 0.1
    pre = torch.addmm(b.double(), x.double(), W.double().t())
    bound = REL * (x.double().abs() @ W.double().abs().t() + b.double().abs())
    for tile in TILES:
        for act in (1, 0):
            y = torch.full((rows, n + 3), 7.0, device=dev)  # strided output: columns past n untouched
            rc = L.hg_gemm_f32(0, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,
                               y.data_ptr(), y.stride(0), None, rows, n, k, act, tile, _stream())
            assert rc == 0
            ref = F.elu(pre) if act else pre
            err = (y[:, :n].double() - ref).abs()
            assert (err <= bound).all(), f"tile {tile} act {act}: worst ratio {(err / bound).max().item():.3f}"
            assert (y[:, n:] == 7.0).all()


# (rows, k_red, n): input gradient g [rows, k_red] x W [k_red, n] through the ELU backward of y [rows, n]
DX_CASES = [(24576, 256, 512), (4096, 128, 256), (3001, 256, 768), (777, 128, 128), (33, 7, 5), (65, 40, 129),
            (1, 128, 256)]


@pytest.mark.parametrize("rows,kr,n", DX_CASES)
def test_gemm_input_grad_matches_fp64(rows, kr, n):
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + kr + n)
    dev = "cuda:0"
    g = torch.randn(rows, kr, device=dev)
    W = torch.randn(kr, n, device=dev) / kr ** 0.5
    y = F.elu(torch.randn(rows, n, device=dev))
    d = g.double() @ W.double()
    ref = torch.where(y.double() > 0, d, d * (y.double() + 1))
    bound = REL * (g.double().abs() @ W.double().abs())
    cs_ref = ref.sum(0)
    cs_bound = (bound.sum(0) + REL * ref.abs().sum(0)) * 2
    Wt = W.t().contiguous()
    for tile in TILES:
        parts = int(L.hg_gemm_colpart_rows(rows, tile))
        cp = torch.full((parts, n), float("nan"), device=dev)
        out = torch.empty(rows, n, device=dev)
        md, BB = (1, W) if tile < 19 or tile % 2 else (3, Wt)  # the bf16-split tiles take both B layouts
        rc = L.hg_gemm_f32(md, g.data_ptr(), g.stride(0), BB.data_ptr(), BB.stride(0), None, y.data_ptr(),
                           y.stride(0), out.data_ptr(), out.stride(0), cp.data_ptr(), rows, n, kr, 1, tile, _stream())
        assert rc == 0
        err = (out.double() - ref).abs()
        assert (err <= bound).all(), f"tile {tile}: worst ratio {(err / bound).max().item():.3f}"
        cs_err = (cp.double().sum(0) - cs_ref).abs()
        assert (cs_err <= cs_bound).all(), f"tile {tile}: bias worst ratio {(cs_err / cs_bound).max().item():.3f}"
        # act 0: the plain product, no colpart
        out0 = torch.empty(rows, n, device=dev)
        rc = L.hg_gemm_f32(md, g.data_ptr(), g.stride(0), BB.data_ptr(), BB.stride(0), None, None, 0,
                           out0.data_ptr(), out0.stride(0), None, rows, n, kr, 0, tile, _stream())
        assert rc == 0
        assert ((out0.double() - d).abs() <= bound).all()


# (rows = reduction, n, k, slices): weight gradients dW [n, k] = gh^T x, split-K slices summed here
WG_CASES = [(24576, 512, 705, 4), (777, 128, 219, 3), (33, 5, 7, 1), (100, 130, 66, 2), (4096, 256, 512, 16),
            (24576, 768, 219, 32), (250, 64, 300, 40)]


@pytest.mark.parametrize("rows,n,k,S", WG_CASES)
def test_gemm_wgrad_matches_fp64(rows, n, k, S):
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + n + k + S)
    dev = "cuda:0"
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    ref = gh.double().t() @ x.double()
    bound = REL * (gh.double().abs().t() @ x.double().abs()) * 1.5  # + the slice sum's roundings
    ght, xt = gh.t().contiguous(), x.t().contiguous()
    for kmajor, (A, B) in ((0, (gh, x)), (1, (ght, xt))):
        for tile in range(19, 29):
            part = torch.full((S, n, k + 2), 5.0, device=dev)  # strided output: the pad columns untouched
            rc = L.hg_gemm_f32_wgrad(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), part.data_ptr(), k + 2,
                                     n * (k + 2), n, k, rows, S, kmajor, tile, _stream())
            assert rc == 0
            dw = part[:, :, :k].double().sum(0)
            err = (dw - ref).abs()
            assert (err <= bound).all(), f"kmajor {kmajor} tile {tile}: worst ratio {(err / bound).max().item():.3f}"
            assert (part[:, :, k:] == 5.0).all()
    # k_wgrad_tr (tiles 40..54: row-major operands through LDS transpose reads), with x a column
    # slice of a wider table (row stride not a multiple of 4: unaligned 16-byte row segments)
    wide = torch.randn(rows, k + 19, device=dev)
    xs = wide[:, 3:3 + k]
    xs.copy_(x)
    for tile in range(40, 55):
        part = torch.full((S, n, k + 2), 5.0, device=dev)
        rc = L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), xs.data_ptr(), xs.stride(0), part.data_ptr(), k + 2,
                                 n * (k + 2), n, k, rows, S, 0, tile, _stream())
        assert rc == 0
        dw = part[:, :, :k].double().sum(0)
        err = (dw - ref).abs()
        assert (err <= bound).all(), f"tr tile {tile}: worst ratio {(err / bound).max().item():.3f}"
        assert (part[:, :, k:] == 5.0).all()


def _image(L, P, trans, rows, k):
    img = torch.empty(int(L.hg_gemm_x6_image_bytes(rows, k)) // 4, device="cuda:0")
    vp = ctypes.c_void_p
    rc = L.hg_gemm_x6_image_jobs((vp * 1)(P.data_ptr()), (ctypes.c_int64 * 1)(P.stride(0)), (ctypes.c_int * 1)(trans),
                                 (ctypes.c_int64 * 1)(rows), (ctypes.c_int64 * 1)(k), (vp * 1)(img.data_ptr()), 1,
                                 _stream())
    assert rc == 0
    return img


def _nbytes(img):
    return img.numel() * img.element_size()


# (rows, k, n): the image forms (hg_gemm_x6_image_jobs + hg_gemm_f32_img, B from its image, A staged
# or from its image) of modes 0 and 1 against hg_gemm_f32 with the per-block staging, bit for bit
# (same split, same MFMA order), ragged shapes
IMG_CASES = [(3001, 705, 512), (777, 219, 768), (4096, 256, 128), (33, 7, 5), (65, 40, 129), (1, 705, 128)]


@pytest.mark.parametrize("rows,k,n", IMG_CASES)
def test_gemm_images_bitwise_equal(rows, k, n):
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + 3 * k + n)
    dev = "cuda:0"
    x = torch.randn(rows, k, device=dev)
    W = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev) * 0.1
    Wd = torch.randn(k, n, device=dev) / k ** 0.5  # mode 1: g [rows, k] x Wd [k, n]
    y = F.elu(torch.randn(rows, n, device=dev))
    aimg = _image(L, x, 0, rows, k)
    for mode, B, trans in ((0, W, 0), (1, Wd, 1)):
        bimg = _image(L, B, trans, n, k)
        # 30 / 31 / 32: tiles 25 / 22 / 21 at more waves per SIMD (k_gemm_x6_occ); their staged form
        # runs the base tile, so the image forms are checked bitwise against the base blocking
        for tile in range(19, 33):
            parts = int(L.hg_gemm_colpart_rows(rows, tile))
            outs = []
            for form in ("staged", "b_image", "ab_image"):
                out = torch.full((rows, n + 2), 3.0, device=dev)
                cp = torch.full((parts, n), float("nan"), device=dev) if mode == 1 else None
                bias = b.data_ptr() if mode == 0 else None
                Y, ldY = (y.data_ptr(), y.stride(0)) if mode == 1 else (None, 0)
                cpp = cp.data_ptr() if cp is not None else None
                if form == "staged":
                    rc = L.hg_gemm_f32(mode, x.data_ptr(), x.stride(0), B.data_ptr(), B.stride(0), bias, Y, ldY,
                                       out.data_ptr(), out.stride(0), cpp, rows, n, k, 1, tile, _stream())
                else:
                    ab = form == "ab_image"
                    rc = L.hg_gemm_f32_img(mode, None if ab else x.data_ptr(), 0 if ab else x.stride(0),
                                           aimg.data_ptr() if ab else None, bimg.data_ptr(), bias, Y, ldY,
                                           out.data_ptr(), out.stride(0), cpp, rows, n, k, 1, tile, _nbytes(aimg),
                                           _nbytes(bimg), _stream())
                assert rc == 0
                outs.append((form, out, cp))
            _, o0, c0 = outs[0]
            for form, o1, c1 in outs[1:]:
                assert torch.equal(o0, o1), f"tile {tile} mode {mode} {form}"
                assert (o1[:, n:] == 3.0).all()
                if mode == 1:
                    assert torch.equal(c0, c1), f"tile {tile} {form} colpart"
    # arguments: a misaligned image, a mode without an image form, no A at all, an image of another
    # shape (its byte size), tiles outside the bf16-split range
    out = torch.empty(rows, n, device=dev)
    bimg = _image(L, W, 0, n, k)
    nb = _nbytes(bimg)
    assert L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, bimg.data_ptr() + 4, None, None, 0, out.data_ptr(),
                             out.stride(0), None, rows, n, k, 0, 20, 0, nb, _stream()) != 0
    assert L.hg_gemm_f32_img(2, x.data_ptr(), x.stride(0), None, bimg.data_ptr(), None, None, 0, out.data_ptr(),
                             out.stride(0), None, rows, n, k, 0, 20, 0, nb, _stream()) != 0
    assert L.hg_gemm_f32_img(0, None, 0, None, bimg.data_ptr(), None, None, 0, out.data_ptr(),
                             out.stride(0), None, rows, n, k, 0, 20, 0, nb, _stream()) != 0
    assert L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, bimg.data_ptr(), None, None, 0, out.data_ptr(),
                             out.stride(0), None, rows, n, k + 40, 0, 20, 0, nb, _stream()) != 0
    assert L.hg_gemm_f32_img(0, x.data_ptr(), x.stride(0), None, bimg.data_ptr(), None, None, 0, out.data_ptr(),
                             out.stride(0), None, rows, n, k, 0, 33, 0, nb, _stream()) != 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("rows,n,k,S", WG_CASES)
def test_gemm_wgrad_images_match_fp64(rows, n, k, S):
    """hg_gemm_wgrad_img from the two reduction-major images of gh [rows, n] and x [rows, k]: the
    split-K slices summed here against fp64, under the bound of hg_gemm_f32_wgrad."""
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + n + k + S + 1)
    dev = "cuda:0"
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    ref = gh.double().t() @ x.double()
    bound = REL * (gh.double().abs().t() @ x.double().abs()) * 1.5
    ai, bi = _image(L, gh, 1, n, rows), _image(L, x, 1, k, rows)
    for tile in range(19, 29):
        part = torch.full((S, n, k + 2), 5.0, device=dev)
        rc = L.hg_gemm_wgrad_img(ai.data_ptr(), bi.data_ptr(), part.data_ptr(), k + 2, n * (k + 2), n, k, rows, S,
                                 tile, _nbytes(ai), _nbytes(bi), _stream())
        assert rc == 0
        dw = part[:, :, :k].double().sum(0)
        err = (dw - ref).abs()
        assert (err <= bound).all(), f"tile {tile}: worst ratio {(err / bound).max().item():.3f}"
        assert (part[:, :, k:] == 5.0).all()


def test_gemm_rejects_bad_arguments():
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    x = torch.randn(8, 16, device="cuda:0")
    W = torch.randn(4, 16, device="cuda:0")
    y = torch.empty(8, 4, device="cuda:0")
    args = [0, x.data_ptr(), 16, W.data_ptr(), 16, None, None, 0, y.data_ptr(), 4, None, 8, 4, 16, 1, 4, _stream()]
    assert L.hg_gemm_f32(*args) == 0
    for i, bad in ((0, 2), (2, 15), (4, 15), (9, 3), (11, 0), (14, 2), (15, 0), (15, 99)):
        a = list(args)
        a[i] = bad
        assert L.hg_gemm_f32(*a) != 0
    # mode 1 with the ELU backward needs Y
    a = list(args)
    a[0], a[4] = 1, 4
    a[1], a[2], a[13] = x.data_ptr(), 16, 16
    assert L.hg_gemm_f32(*a) != 0
    # weight gradients: the transposed-read tiles take row-major (kmajor 0) operands only, and tile
    # ids outside 19..28 / 40..54 are refused
    part = torch.empty(4, 16, device="cuda:0")
    wg = [x.data_ptr(), 4, y.data_ptr(), 4, part.data_ptr(), 16, 0, 4, 4, 8, 1, 0, 40, _stream()]
    assert L.hg_gemm_f32_wgrad(*wg) == 0
    for i, bad in ((11, 1), (12, 29), (12, 39), (12, 55), (10, 0)):
        a = list(wg)
        a[i] = bad
        assert L.hg_gemm_f32_wgrad(*a) != 0
    torch.cuda.synchronize()


def test_mlp_backward_with_fused_gemm_matches_autograd():
    """The actor / critic / lin-vel MLPs through hg_mlp (forward on the fused GEMM where routed,
    input gradients with the ELU backward and bias partials in the GEMM epilogue) against torch
    autograd on the same nn.Sequential, fp32: outputs and every parameter / input gradient."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, hg_mlp
    torch.manual_seed(11)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     base_lin_vel_hidden_dims=[128, 128]).cuda()
    calls = []
    orig_f, orig_g = hg_mlp.gemm_forward, hg_mlp.gemm_input_grad

    def spy_f(h, W, b, *a, **kw):
        calls.append(("f", tuple(W.shape)))
        return orig_f(h, W, b, *a, **kw)

    def spy_g(gh, W, *a, **kw):
        calls.append(("g", tuple(W.shape)))
        return orig_g(gh, W, *a, **kw)

    hg_mlp.gemm_forward, hg_mlp.gemm_input_grad = spy_f, spy_g
    try:
        for net, width in ((ac.actor, 705), (ac.critic, 219), (ac.base_lin_vel, 705)):
            x = torch.randn(24576, width, device="cuda:0", requires_grad=True)
            y = hg_mlp.mlp_forward(net, x)
            gy = torch.randn_like(y)
            grads = torch.autograd.grad(y, [x, *net.parameters()], gy)
            x2 = x.detach().clone().requires_grad_(True)
            y2 = net(x2)
            grads2 = torch.autograd.grad(y2, [x2, *net.parameters()], gy)
            torch.testing.assert_close(y, y2, rtol=1e-5, atol=1e-5)
            for a, b_ in zip(grads, grads2):
                scale = b_.abs().max().item() + 1e-12
                assert (a - b_).abs().max().item() <= 2e-5 * scale + 1e-6
    finally:
        hg_mlp.gemm_forward, hg_mlp.gemm_input_grad = orig_f, orig_g
    if hg_mlp.GEMM and hg_mlp._GEMM_DX:
        assert any(c[0] == "g" for c in calls), calls
    if hg_mlp.GEMM and hg_mlp._GEMM_FWD:
        assert any(c[0] == "f" for c in calls), calls


def test_paired_first_layers_match_separate_networks():
    """hg_mlp.mlp_pair_forward (the actor's and the lin-vel estimator's first layers as ONE stacked
    GEMM from a stacked image, the rest of each network on strided column slices of its result)
    against the two networks run apart through hg_mlp: the same products on the same operands, so
    outputs and every parameter gradient bit for bit; and against torch autograd at the MLP test's
    tolerance.  Also inside an image_scope that builds the stacked image with the other images."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, hg_mlp
    torch.manual_seed(12)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     base_lin_vel_hidden_dims=[128, 128]).cuda()
    rows = 24576
    assert hg_mlp.pair_ok(ac.actor, ac.base_lin_vel, rows)
    x = torch.randn(rows, 705, device="cuda:0")
    params = [*ac.actor.parameters(), *ac.base_lin_vel.parameters()]
    ya0 = hg_mlp.mlp_forward(ac.actor, x)
    yb0 = hg_mlp.mlp_forward(ac.base_lin_vel, x)
    ga, gb = torch.randn_like(ya0), torch.randn_like(yb0)
    ref = torch.autograd.grad((ya0, yb0), params, (ga, gb))
    for scoped in (False, True):
        ctx = (hg_mlp.image_scope([(ac.actor, rows), (ac.base_lin_vel, rows)], x.device,
                                  pairs=[(ac.actor, ac.base_lin_vel, rows)]) if scoped else hg_mlp.contextlib.nullcontext())
        with ctx:
            ya, yb = hg_mlp.mlp_pair_forward(ac.actor, ac.base_lin_vel, x)
            got = torch.autograd.grad((ya, yb), params, (ga, gb))
        assert torch.equal(ya, ya0) and torch.equal(yb, yb0)
        for a, b_ in zip(got, ref):
            assert torch.equal(a, b_), (a - b_).abs().max().item()
    x2 = x.clone()
    ya2, yb2 = ac.actor(x2), ac.base_lin_vel(x2)
    ref2 = torch.autograd.grad((ya2, yb2), params, (ga, gb))
    torch.testing.assert_close(ya, ya2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(yb, yb2, rtol=1e-5, atol=1e-5)
    for a, b_ in zip(got, ref2):
        assert (a - b_).abs().max().item() <= 2e-5 * (b_.abs().max().item() + 1e-12) + 1e-6


def test_stacked_image_bands_non_256_tail():
    """A stacked image whose last band is not a multiple of 256 rows (256 + 40 over K = 219): its
    bytes equal the image of the two weights concatenated, built as one job; a 480 + 32 split (the
    first band's zero padding would land on the second band) is refused."""
    _need_gpu()
    from humanoid.algo.ppo import hg_mlp
    torch.manual_seed(13)
    A = torch.randn(256, 219, device="cuda:0")
    B = torch.randn(40, 219, device="cuda:0")
    (stacked,) = hg_mlp.x6_images([("stack", (A, B), 219)], A.device)
    (whole,) = hg_mlp.x6_images([(torch.cat([A, B]), 0, 296, 219)], A.device)
    torch.cuda.synchronize()
    assert stacked.numel() == whole.numel() and torch.equal(stacked.view(torch.int32), whole.view(torch.int32))
    with pytest.raises(ValueError):
        hg_mlp.x6_images([("stack", (torch.randn(480, 219, device="cuda:0"), torch.randn(32, 219, device="cuda:0")),
                           219)], A.device)


@pytest.mark.parametrize("rows,n", [(24576, 12), (777, 3), (64, 1), (65, 12)])
def test_skinny_backward_act_matches_fp64(rows, n):
    """hg_linear_skinny_backward_act: the output layer's dW / db partials and its input gradient
    through the ELU backward of the layer below (h = that layer's ELU output), with that layer's
    bias-gradient partials, against fp64."""
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + n)
    dev, k = "cuda:0", 128
    g = torch.randn(rows, n, device=dev)
    h = F.elu(torch.randn(rows, k, device=dev))
    W = torch.randn(n, k, device=dev) / k ** 0.5
    gh = torch.empty(rows, k, device=dev)
    parts = int(L.hg_linear_skinny_colpart_rows(rows))
    cp = torch.empty(parts, k, device=dev)
    scratch = torch.empty(int(L.hg_linear_skinny_backward_scratch(rows, n, k)), device=dev)
    rc = L.hg_linear_skinny_backward_act(g.data_ptr(), h.data_ptr(), h.stride(0), W.data_ptr(), gh.data_ptr(),
                                         cp.data_ptr(), rows, n, k, scratch.data_ptr(), _stream())
    assert rc == 0
    torch.cuda.synchronize()
    d = g.double() @ W.double()
    ref = torch.where(h.double() > 0, d, d * (h.double() + 1))
    bound = REL * (g.double().abs() @ W.double().abs()) + 1e-12
    assert ((gh.double() - ref).abs() <= bound).all()
    cs_bound = 2 * (bound.sum(0) + REL * ref.abs().sum(0))
    assert ((cp.double().sum(0) - ref.sum(0)).abs() <= cs_bound).all()
    tiles = scratch.numel() // (n * k + n)
    wb = scratch.view(tiles, n * k + n)[:tiles].double().sum(0)
    dw_ref = (g.double().t() @ h.double()).reshape(-1)
    db_ref = g.double().sum(0)
    dw_bound = REL * (g.double().abs().t() @ h.double().abs()).reshape(-1) * 2 + 1e-9
    assert ((wb[: n * k] - dw_ref).abs() <= dw_bound).all()
    assert ((wb[n * k:] - db_ref).abs() <= REL * g.double().abs().sum(0) * 2 + 1e-9).all()


@pytest.mark.parametrize("parts,width", [(8, 90240), (32, 360960), (64, 196608), (5, 4100), (40, 768)])
def test_colsum_jobs_wide_and_narrow_orders(parts, width):
    """hg_colsum_jobs in one launch over several jobs: wide split-K jobs (width >= 4096, a multiple
    of 4) sum part p into accumulator p % 8 and combine the eight as a fixed tree above 16 parts,
    in part order up to 16 — both reproduced bitwise here in float32 numpy; narrow jobs (bias-tile
    partials) keep the 16-column blocks' order, checked against float64 within rounding."""
    _need_gpu()
    import numpy as np
    from humanoid import _native as N
    g = torch.Generator(device="cuda:0").manual_seed(parts * 7 + 1)
    src = torch.randn(parts, width, device="cuda:0", generator=g) * 3.0
    nar = torch.randn(37, 768, device="cuda:0", generator=g)
    dst, dst_n = torch.empty(width, device="cuda:0"), torch.empty(768, device="cuda:0")
    vp = ctypes.c_void_p
    rc = N.lib().hg_colsum_jobs((vp * 2)(src.data_ptr(), nar.data_ptr()), (vp * 2)(dst.data_ptr(), dst_n.data_ptr()),
                                (ctypes.c_int64 * 2)(width, 768), (ctypes.c_int * 2)(parts, 37), 2,
                                vp(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    a = src.cpu().numpy()
    if width >= 4096 and width % 4 == 0 and parts > 16:
        acc = [np.zeros(width, np.float32) for _ in range(8)]
        for p in range(parts):
            acc[p % 8] = (acc[p % 8] + a[p]).astype(np.float32)
        want = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))
    elif parts <= 16:
        want = a[0].copy()
        for p in range(1, parts):
            want = (want + a[p]).astype(np.float32)
    else:  # narrow job with many parts: the bias-partial blocks' order
        want = None
        assert torch.allclose(dst.double(), src.double().sum(0), rtol=1e-5, atol=1e-4)
    if want is not None:
        assert np.array_equal(dst.cpu().numpy(), want)
    ref = nar.double().sum(0)
    assert torch.allclose(dst_n.double(), ref, rtol=1e-5, atol=1e-4)


# (rows, k, n, lda pad, output pad): the rollout's first policy layer, 16-byte rows (the staged
# float4 loads), ragged rows / k / columns (n % 4 != 0: the finishing pass's scalar path), a strided
# input and a strided output
SPLITK_CASES = [(4096, 705, 512, 0, 0), (4096, 512, 256, 0, 0), (777, 219, 768, 0, 0), (65, 33, 129, 0, 0), (130, 64, 96, 3, 3)]


@pytest.mark.parametrize("rows,k,n,pad,opad", SPLITK_CASES)
def test_gemm_splitk_forward_matches_fp64(rows, k, n, pad, opad):
    """hg_gemm_f32_splitk (slices of k_gemm_x6 mode 4 + the fixed-order finishing launch) within the
    stated per-element bound of the fp64 product, for every bf16-split tile and 2-4 slices; a repeat
    is bit-identical (the workspace is refilled with NaN before every call: every slice element is
    written before the finish reads it)."""
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + k + n + 1)
    dev = "cuda:0"
    xs = torch.randn(rows, k + pad, device=dev)
    x = xs[:, :k]
    W = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev) * 0.1
    pre = torch.addmm(b.double(), x.double(), W.double().t())
    bound = REL * (x.double().abs() @ W.double().abs().t() + b.double().abs())
    ran = 0
    for tile in range(20, 29):
        for S in (2, 3, 4):
            if (S - 1) * L.hg_gemm_splitk_kslice(k, S) >= k:
                continue
            for act in (1, 0):
                outs = []
                for _ in range(2):
                    ws = torch.full((S * rows * n,), float("nan"), device=dev)
                    y = torch.full((rows, n + opad), 7.0, device=dev)
                    rc = L.hg_gemm_f32_splitk(x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(),
                                              y.data_ptr(), y.stride(0), ws.data_ptr(), ws.numel(), rows, n, k, act,
                                              tile, S, _stream())
                    assert rc == 0
                    outs.append(y)
                y = outs[0]
                ref = F.elu(pre) if act else pre
                err = (y[:, :n].double() - ref).abs()
                assert (err <= bound).all(), f"tile {tile} S {S} act {act}: worst ratio {(err / bound).max().item():.3f}"
                assert (y[:, n:] == 7.0).all()
                assert torch.equal(outs[0], outs[1]), f"tile {tile} S {S} act {act}"
                ran += 1
    assert ran > 0


@pytest.mark.parametrize("rows,k,n,pad,opad", SPLITK_CASES)
def test_gemm_splitk_img_is_bitwise_the_plain_splitk(rows, k, n, pad, opad):
    """hg_gemm_f32_splitk_img (the split-K forward with W as its prebuilt operand image) writes the
    same bits as hg_gemm_f32_splitk on the same tile and slice count (the occupancy tiles 30 / 31 /
    32 as tiles 25 / 22 / 21), columns past n untouched; the tiles with two chunks per stage are
    refused (profiles/r6_gemm/roll_splitk_img.json: measured, not routed)."""
    _need_gpu()
    from humanoid import _native as N
    L = N.lib()
    torch.manual_seed(rows + k + n + 2)
    dev = "cuda:0"
    x = torch.randn(rows, k + pad, device=dev)[:, :k]
    W = torch.randn(n, k, device=dev) / k ** 0.5
    b = torch.randn(n, device=dev) * 0.1
    nb = int(L.hg_gemm_x6_image_bytes(n, k))
    img = torch.full((nb // 4,), float("nan"), device=dev)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    assert L.hg_gemm_x6_image_jobs((vp * 1)(W.data_ptr()), (i64 * 1)(W.stride(0)), (ctypes.c_int * 1)(0),
                                   (i64 * 1)(n), (i64 * 1)(k), (vp * 1)(img.data_ptr()), 1, _stream()) == 0
    base = {30: 25, 31: 22, 32: 21}
    ran = 0
    for tile in (20, 21, 22, 23, 25, 27, 28, 30, 31, 32):
        for S in (2, 4):
            if (S - 1) * L.hg_gemm_splitk_kslice(k, S) >= k:
                continue
            for act in (1, 0):
                ys = []
                for fn in ("plain", "img"):
                    ws = torch.full((S * rows * n,), float("nan"), device=dev)
                    y = torch.full((rows, n + opad), 7.0, device=dev)
                    if fn == "plain":
                        rc = L.hg_gemm_f32_splitk(x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(),
                                                  y.data_ptr(), y.stride(0), ws.data_ptr(), ws.numel(), rows, n, k,
                                                  act, base.get(tile, tile), S, _stream())
                    else:
                        rc = L.hg_gemm_f32_splitk_img(x.data_ptr(), x.stride(0), img.data_ptr(), nb, b.data_ptr(),
                                                      y.data_ptr(), y.stride(0), ws.data_ptr(), ws.numel(), rows, n,
                                                      k, act, tile, S, _stream())
                    assert rc == 0
                    ys.append(y)
                assert torch.equal(ys[0], ys[1]), f"tile {tile} S {S} act {act}"
                ran += 1
    assert ran > 0
    ws = torch.empty(2 * rows * n, device=dev)
    y = torch.empty(rows, n, device=dev)
    for tile in (24, 26, 29):
        assert L.hg_gemm_f32_splitk_img(x.data_ptr(), x.stride(0), img.data_ptr(), nb, b.data_ptr(), y.data_ptr(), n,
                                        ws.data_ptr(), ws.numel(), rows, n, k, 1, tile, 2, _stream()) != 0
    torch.cuda.synchronize()


def test_rollout_first_layer_routes_to_splitk():
    """The rollout's 4096-row 705 -> 512 hidden layer goes through hg_gemm_f32_splitk
    (_GEMM_FWD_SPLITK) and matches the one-pass route within the stated bound; 24576 rows keep
    the one-pass tiles."""
    _need_gpu()
    from humanoid.algo.ppo import hg_mlp
    dev = "cuda:0"
    torch.manual_seed(7)
    W = torch.randn(512, 705, device=dev) / 705 ** 0.5
    b = torch.randn(512, device=dev) * 0.1
    calls = []
    orig = hg_mlp.gemm_forward_splitk

    def spy(*a, **kw):
        calls.append(a[0].shape[0])
        return orig(*a, **kw)
    hg_mlp.gemm_forward_splitk = spy
    try:
        for rows in (4096, 24576):
            x = torch.randn(rows, 705, device=dev)
            y = hg_mlp._hidden_forward(x, W, b)
            pre = torch.addmm(b.double(), x.double(), W.double().t())
            bound = REL * (x.double().abs() @ W.double().abs().t() + b.double().abs())
            assert ((y.double() - F.elu(pre)).abs() <= bound).all()
    finally:
        hg_mlp.gemm_forward_splitk = orig
    assert calls == ([4096] if hg_mlp.SPLITK_FWD else [])
