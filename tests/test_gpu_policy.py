"""The rollout's fused policy forward (hg_policy_forward, csrc/hg_policy.hip) against the actor MLP
of the reference (actor_critic.py:36-149: Linear + ELU x 3, Linear) in fp64, at the bench's 4096
rows and ragged row counts, on a strided input view like the env's observation window.

Stated tolerance: per output element, |fused - fp64| <= 2 x the largest |torch f32 - fp64| of the
same batch + 1e-6 (the hidden products are exact three-term bf16 splits with f32 accumulation,
the bf16-split GEMM's arithmetic, whose error per element is below torch's f32 GEMM's)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _actor(k0=705, nout=12, seed=0):
    from humanoid.algo.ppo.actor_critic import _mlp
    torch.manual_seed(seed)
    return _mlp(k0, [512, 256, 128], nout, nn.ELU()).cuda()


def _window_view(rows, k0, ld, off, seed=1):
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    buf = torch.randn(rows * ld + off + k0, device="cuda:0", generator=g) * 2.0
    return buf[off:off + rows * ld].view(rows, ld)[:, :k0]


@pytest.mark.parametrize("rows", [4096, 1, 33, 4097, 8192])
def test_policy_forward_matches_fp64(rows):
    _need_gpu()
    from humanoid.algo.ppo import hg_mlp
    net = _actor()
    x = _window_view(rows, 705, 1880, 47 * 3)   # window row 1880 floats, a 188-byte column offset
    params = [p.detach() for p in hg_mlp._params(net)]
    assert hg_mlp._policy_ok(params, x)
    with torch.no_grad():
        y = hg_mlp.policy_forward(params, x)
        y32 = net(x.contiguous())
        y64 = net.double()(x.double()).float().double()
        net.float()
    torch.cuda.synchronize()
    e_fused = (y.double() - y64).abs()
    e_torch = (y32.double() - y64).abs().max().item()
    bound = 2 * e_torch + 1e-6
    assert e_fused.max().item() <= bound, f"fused {e_fused.max().item():.3e} torch f32 {e_torch:.3e}"
    # deterministic: the same launch twice, bit for bit
    y2 = hg_mlp.policy_forward(params, x)
    assert torch.equal(y, y2)


def test_rollout_act_uses_fused_policy():
    """ActorCritic._mlp(actor, obs) without autograd (PPO.act's path) runs hg_policy_forward."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, hg_mlp
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128]).cuda()
    obs = _window_view(4096, 705, 1880, 0)
    calls = []
    real = hg_mlp.policy_forward

    def spy(params, x, out=None):
        calls.append(x.shape)
        return real(params, x, out)
    hg_mlp.policy_forward = spy
    try:
        with torch.inference_mode():
            mean = ac._mlp(ac.actor, obs)
    finally:
        hg_mlp.policy_forward = real
    assert calls == [(4096, 705)]
    ref = real([p.detach() for p in hg_mlp._params(ac.actor)], obs)
    assert torch.equal(mean, ref)


def test_policy_forward_rejects_bad_arguments():
    _need_gpu()
    from humanoid import _native as N
    from humanoid.algo.ppo import hg_mlp
    net = _actor()
    params = [p.detach() for p in hg_mlp._params(net)]
    x = torch.randn(64, 705, device="cuda:0")
    imgs = hg_mlp.x6_images([(params[0], 0, 512, 705), (params[2], 0, 256, 512), (params[4], 0, 128, 256)], x.device)
    y = torch.empty(64, 12, device="cuda:0")
    vp = ctypes.c_void_p
    L = N.lib()
    s = vp(torch.cuda.current_stream().cuda_stream)

    def call(k0=705, dims=(512, 256, 128), nbytes=None, nout=12):
        nb = nbytes or [im.numel() * 4 for im in imgs]
        return L.hg_policy_forward(x.data_ptr(), x.stride(0), 64, k0, *dims, (vp * 3)(*[im.data_ptr() for im in imgs]),
                                   (ctypes.c_int64 * 3)(*nb), (vp * 3)(params[1].data_ptr(), params[3].data_ptr(),
                                                                       params[5].data_ptr()),
                                   params[6].data_ptr(), params[7].data_ptr(), nout, y.data_ptr(), 12, s)
    assert call() == 0
    assert call(k0=700) != 0                       # images built for another K0
    assert call(dims=(256, 256, 128)) != 0         # an un-instantiated chain
    assert call(nbytes=[1, 2, 3]) != 0
    assert call(nout=17) != 0
    torch.cuda.synchronize()
