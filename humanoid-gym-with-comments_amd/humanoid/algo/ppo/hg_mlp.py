"""Forward/backward of a Linear/ELU chain (the actor, lin-vel and critic MLPs of
actor_critic.py:36-149) with the activation backward and bias gradient fused into one HIP pass
per layer (``hg_mlp_act_backward``, csrc/hg_mlp.hip).

The GEMMs are torch's (``addmm`` forward, ``mm`` for the weight and input gradients — the same
hipBLASLt/rocBLAS calls nn.Linear makes, so the TunableOp table applies unchanged).  What changes
is the per-layer elementwise/reduction tail of the backward: torch runs ELU-backward and a
separate ``grad.sum(0)`` reduction over the [rows, width] gradient; here it is one pass that
reads the incoming gradient and the layer's ELU output once.  The layer output y (not the
pre-activation) is kept for the backward: elu'(h) = y + 1 for h <= 0.  Parameters stay in the
nn.Sequential (state_dict keys unchanged).  Device float32 only.
"""
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from humanoid import _native as N


def fusable(net):
    """True when ``net`` is Linear (ELU(alpha=1) Linear)* — the shape the fused backward handles."""
    mods = list(net)
    if not mods or not isinstance(mods[-1], nn.Linear):
        return False
    for i, m in enumerate(mods):
        want = nn.Linear if i % 2 == 0 else nn.ELU
        if not isinstance(m, want):
            return False
        if isinstance(m, nn.ELU) and (m.alpha != 1.0 or m.inplace):
            return False
        if isinstance(m, nn.Linear) and m.bias is None:
            return False
    return True


def _act_backward(gy, y, rows, width, gb):
    """gh = gy * elu'(from y) (y None: gh = gy) and gb = gh.sum(0), in one fused pass."""
    L = N.lib()
    scratch = torch.empty(int(L.hg_mlp_act_backward_scratch(rows, width)), dtype=torch.float32, device=gy.device)
    gh = torch.empty_like(gy) if y is not None else gy
    s = ctypes.c_void_p(torch.cuda.current_stream(gy.device).cuda_stream)
    rc = L.hg_mlp_act_backward(gy.data_ptr(), y.data_ptr() if y is not None else None,
                               gh.data_ptr() if y is not None else None, rows, width, gb.data_ptr(),
                               scratch.data_ptr(), s)
    if rc != 0:
        raise RuntimeError(f"hg_mlp_act_backward failed ({rc})")
    return gh


class _MLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        n = len(params) // 2
        acts = [x]
        h = x
        for i in range(n):
            W, b = params[2 * i], params[2 * i + 1]
            h = torch.addmm(b, h, W.t())
            if i < n - 1:
                h = F.elu(h)
            acts.append(h)
        # inputs of every layer (x, y_0 .. y_{n-2}) and the weights
        ctx.save_for_backward(*acts[:-1], *params[0::2])
        ctx.n = n
        return h

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        ins, Ws = saved[:n], saved[n:]
        grads = [None] * (2 * n)
        g = g.contiguous()
        gx = None
        for i in range(n - 1, -1, -1):
            rows, width = g.shape
            gb = torch.empty(width, dtype=torch.float32, device=g.device)
            # layer i's output is ins[i + 1] (the ELU output) for hidden layers; identity for the last
            gh = _act_backward(g, ins[i + 1] if i < n - 1 else None, rows, width, gb)
            grads[2 * i + 1] = gb
            grads[2 * i] = torch.mm(gh.t(), ins[i])
            if i > 0:
                g = torch.mm(gh, Ws[i])
            elif ctx.needs_input_grad[0]:
                gx = torch.mm(gh, Ws[0])
        return (gx, *grads)


def mlp_forward(net, x):
    """net(x) for a fusable Linear/ELU nn.Sequential, with the fused backward."""
    params = []
    for m in net:
        if isinstance(m, nn.Linear):
            params += [m.weight, m.bias]
    return _MLP.apply(x, *params)
