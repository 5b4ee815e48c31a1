"""The PPO minibatch loss on the fused HIP kernels ``hg_ppo_loss`` / ``hg_ppo_loss_backward``
(csrc/hg_optim.hip).

Between the three network outputs (actor mean, critic value, lin-vel estimate) and
``loss.backward()`` the reference runs ~40 elementwise/reduction ops forward and as many backward
(ppo.py:155-210: log-prob, ratio, clipped surrogate, clipped value loss, entropy, lin-vel MSE,
plus the adaptive schedule's KL mean).  ``ppo_loss`` replaces them with an autograd Function of
three launches: the forward kernel writes the loss, its parts and the KL mean together with the
gradients of the loss with respect to (mean, std, value, lin-vel); the backward scales those by
the incoming gradient.  Values and gradients are the reference expressions (torch's tie rules
for ``max`` and ``clamp``); reductions run in float64 in a fixed order, so the result is
deterministic.  Device tensors only.
"""
import ctypes
import os

import torch

from humanoid import _native as N


class _Batch(ctypes.Structure):
    _fields_ = [(name, t) for pair in (
        ("mu", "mu_ld"), ("std", None), ("value", "value_ld"), ("lin_vel", "lin_vel_ld"),
        ("lin_vel_target", "lin_vel_target_ld"), ("actions", "actions_ld"), ("old_logp", "old_logp_ld"),
        ("advantages", "advantages_ld"), ("target_values", "target_values_ld"), ("returns", "returns_ld"),
        ("old_mu", "old_mu_ld"), ("old_sigma", "old_sigma_ld"))
        for name, t in ((pair[0], ctypes.c_void_p), (pair[1], ctypes.c_int64)) if name is not None]


def _lib():
    return N.lib()


def _row(t, width):
    """(pointer, row stride) of a [rows, width] (or [rows]) float32 view with unit column stride."""
    if t.dtype != torch.float32 or not t.is_cuda:
        raise RuntimeError("ppo_loss needs float32 device tensors")
    if t.dim() == 1:
        t = t.unsqueeze(1)
    if t.shape[1] != width or (width > 1 and t.stride(1) != 1):
        raise RuntimeError(f"ppo_loss: expected a [rows, {width}] view with unit column stride, got "
                           f"{tuple(t.shape)} / {t.stride()}")
    return t.data_ptr(), t.stride(0)


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, std, value, lin_vel, data, params):
        rows, A = mu.shape
        dev = mu.device
        b = _Batch()
        b.mu, b.mu_ld = _row(mu, A)
        b.std = std.data_ptr()
        b.value, b.value_ld = _row(value.reshape(rows, 1) if value.dim() == 2 else value, 1)
        b.lin_vel, b.lin_vel_ld = _row(lin_vel, 3)
        for name, width in (("lin_vel_target", 3), ("actions", A), ("old_logp", 1), ("advantages", 1),
                            ("target_values", 1), ("returns", 1), ("old_mu", A), ("old_sigma", A)):
            ptr, ld = _row(data[name], width)
            setattr(b, name, ptr)
            setattr(b, name + "_ld", ld)
        if not std.is_contiguous() or std.numel() != A:
            raise RuntimeError("ppo_loss: std must be a contiguous [num_actions] tensor")
        L = _lib()
        loss = torch.empty((), dtype=torch.float32, device=dev)
        stats_buf, accumulate = params[5], params[6]
        stats = torch.empty(4, dtype=torch.float32, device=dev) if stats_buf is None else stats_buf
        g_mu = torch.empty(rows, A, dtype=torch.float32, device=dev)
        g_std = torch.empty(A, dtype=torch.float32, device=dev)
        g_v = torch.empty(value.shape, dtype=torch.float32, device=dev)
        g_p = torch.empty(rows, 3, dtype=torch.float32, device=dev)
        scratch = torch.empty(int(L.hg_ppo_loss_scratch(rows, A)), dtype=torch.float64, device=dev)
        clip, vcoef, ecoef, lcoef, clipped = params[:5]
        lr_rule = params[7]
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        head = (ctypes.byref(b), rows, A, float(1.0 - clip), float(1.0 + clip), float(clip), int(bool(clipped)),
                float(vcoef), float(ecoef), float(lcoef), loss.data_ptr(), stats.data_ptr(), int(bool(accumulate)),
                g_mu.data_ptr(), g_std.data_ptr(), g_v.data_ptr(), g_p.data_ptr(), scratch.data_ptr())
        if lr_rule is None:
            rc = L.hg_ppo_loss(*head, s)
        else:
            # the adaptive-KL rule on this minibatch's KL mean in the same launch (hg_ppo_loss_lr)
            lr64, lr32, desired, lr_min, lr_max = lr_rule
            rc = L.hg_ppo_loss_lr(*head, lr64.data_ptr(), lr32.data_ptr(), float(desired), float(lr_min),
                                  float(lr_max), s)
        if rc != 0:
            raise RuntimeError(f"hg_ppo_loss failed ({rc})")
        ctx.save_for_backward(g_mu, g_std, g_v, g_p)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        if stats_buf is not None:
            return loss  # the statistics went to the caller's buffer
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, g_loss, g_stats=None):
        g_mu, g_std, g_v, g_p = ctx.saved_tensors
        rows, A = g_mu.shape
        if g_loss.data_ptr() in UNIT_SEEDS:
            # seeded by a registered constant 1.0 (PPO's graphed update): scaling by exactly 1.0 is
            # the identity on every float, so the scaling launch is left out
            return g_mu, g_std, g_v, g_p, None, None
        g_loss = g_loss.contiguous()
        s = ctypes.c_void_p(torch.cuda.current_stream(g_mu.device).cuda_stream)
        rc = _lib().hg_ppo_loss_backward(g_loss.data_ptr(), rows, A, g_mu.data_ptr(), g_std.data_ptr(),
                                         g_v.data_ptr(), g_p.data_ptr(), s)
        if rc != 0:
            raise RuntimeError(f"hg_ppo_loss_backward failed ({rc})")
        return g_mu, g_std, g_v, g_p, None, None


# persistent device scalars holding exactly 1.0 that seed loss.backward(), by data pointer.  The
# contract (register_unit_seed): the owner never writes the tensor after registering it, and
# releases it (release_unit_seed) before dropping it; the registry keeps it referenced meanwhile,
# so its address cannot be reused by another tensor while registered.
UNIT_SEEDS = {}


def register_unit_seed(t):
    """Register a [] float32 device tensor holding 1.0 as a backward seed whose scaling launch may
    be skipped; returns it.  HG_DEBUG_UNIT_SEEDS=1 checks the value (a host read: not under capture)."""
    if t.numel() != 1 or t.dtype != torch.float32:
        raise ValueError("a unit seed is a float32 scalar")
    if os.environ.get("HG_DEBUG_UNIT_SEEDS") == "1" and float(t) != 1.0:
        raise ValueError("a unit seed must hold exactly 1.0")
    UNIT_SEEDS[t.data_ptr()] = t
    return t


def release_unit_seed(t):
    UNIT_SEEDS.pop(t.data_ptr(), None)


def ppo_loss(mu, std, value, lin_vel, data, clip_param, value_loss_coef, entropy_coef, lin_vel_coef,
             use_clipped_value_loss=True, stats_out=None, accumulate=False, lr_rule=None):
    """(loss, stats) with stats = [value_loss, surrogate_loss, lin_vel_loss, kl_mean] (detached).
    With ``stats_out`` (a float32 [4] device buffer) the statistics are written there instead —
    ``accumulate`` adds the three losses to its first entries — and only the loss is returned.

    ``mu`` [B, A] actor mean, ``std`` [A] the policy's std parameter, ``value`` [B, 1] critic
    output, ``lin_vel`` [B, 3] lin-vel estimate; ``data``: dict of the minibatch's stored
    tensors ``actions``, ``old_logp``, ``advantages``, ``target_values``, ``returns``,
    ``old_mu``, ``old_sigma`` and ``lin_vel_target`` (row views with unit column stride).
    ``lr_rule`` = (lr64 [1] float64, lr32 [1] float32, desired_kl, lr_min, lr_max) device scalars and
    bounds: the adaptive schedule's rule applied to this minibatch's KL mean in the same launch."""
    return _PPOLoss.apply(mu, std, value, lin_vel, data,
                          (clip_param, value_loss_coef, entropy_coef, lin_vel_coef, use_clipped_value_loss,
                           stats_out, accumulate, lr_rule))
