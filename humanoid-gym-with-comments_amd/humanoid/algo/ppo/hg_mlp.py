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
import os

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


class _Reductions:
    """The column sums of one MLP backward (bias-gradient tile partials, split-K weight-gradient
    chunks), deferred and launched together as ONE hg_colsum_jobs kernel at the end of the
    backward instead of one reduction launch per layer."""

    def __init__(self):
        self.jobs = []  # (src [parts, width], dst [width], width, parts)

    def add(self, src, dst, width, parts):
        self.jobs.append((src, dst, int(width), int(parts)))

    def launch(self, dev):
        n = len(self.jobs)
        if n == 0:
            return
        vp = ctypes.c_void_p
        src = (vp * n)(*[j[0].data_ptr() for j in self.jobs])
        dst = (vp * n)(*[j[1].data_ptr() for j in self.jobs])
        width = (ctypes.c_int64 * n)(*[j[2] for j in self.jobs])
        parts = (ctypes.c_int * n)(*[j[3] for j in self.jobs])
        rc = N.lib().hg_colsum_jobs(src, dst, width, parts, n, _stream(dev))
        if rc != 0:
            raise RuntimeError(f"hg_colsum_jobs failed ({rc})")
        self.jobs = []


def _act_backward(gy, y, rows, width, gb, red=None):
    """gh = gy * elu'(from y) (y None: gh = gy) and gb = gh.sum(0), in one fused pass (the final
    column sum of gb deferred to ``red`` when given)."""
    L = N.lib()
    scratch = torch.empty(int(L.hg_mlp_act_backward_scratch(rows, width)), dtype=torch.float32, device=gy.device)
    gh = torch.empty_like(gy) if y is not None else gy
    s = ctypes.c_void_p(torch.cuda.current_stream(gy.device).cuda_stream)
    rc = L.hg_mlp_act_backward(gy.data_ptr(), y.data_ptr() if y is not None else None,
                               gh.data_ptr() if y is not None else None, rows, width,
                               gb.data_ptr() if red is None else None, scratch.data_ptr(), s)
    if rc != 0:
        raise RuntimeError(f"hg_mlp_act_backward failed ({rc})")
    if red is not None:
        red.add(scratch, gb, width, scratch.numel() // width)
    return gh


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _skinny_ok(h, W):
    n, k = W.shape
    return (bool(N.lib().hg_linear_skinny_supported(n, k)) and h.dim() == 2 and h.stride(1) == 1
            and h.stride(0) % 4 == 0 and h.data_ptr() % 16 == 0 and W.is_contiguous())


def _skinny_forward(h, W, b, out=None):
    rows, n = h.shape[0], W.shape[0]
    y = torch.empty(rows, n, dtype=torch.float32, device=h.device) if out is None else out
    if y.numel() != rows * n or not y.is_contiguous() or y.dtype != torch.float32:
        raise RuntimeError("skinny forward: out must be a contiguous float32 tensor of rows x n elements")
    rc = N.lib().hg_linear_skinny_forward(h.data_ptr(), h.stride(0), W.data_ptr(), b.data_ptr(), y.data_ptr(), rows,
                                          n, W.shape[1], _stream(h.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_skinny_forward failed ({rc})")
    return y


def _skinny_backward(g, h, W, need_dx, red=None):
    rows, (n, k) = g.shape[0], W.shape
    L = N.lib()
    wb = torch.empty(n * k + n, dtype=torch.float32, device=g.device)
    dx = torch.empty(rows, k, dtype=torch.float32, device=g.device) if need_dx else None
    scratch = torch.empty(int(L.hg_linear_skinny_backward_scratch(rows, n, k)), dtype=torch.float32, device=g.device)
    rc = L.hg_linear_skinny_backward(g.data_ptr(), h.data_ptr(), h.stride(0), W.data_ptr(),
                                     dx.data_ptr() if need_dx else None, wb.data_ptr() if red is None else None,
                                     rows, n, k, scratch.data_ptr(), _stream(g.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_skinny_backward failed ({rc})")
    if red is not None:
        red.add(scratch, wb, n * k + n, scratch.numel() // (n * k + n))
    return wb[: n * k].view(n, k), wb[n * k:], dx


# Split-K factors for the weight gradients dW[n, k] = gh[R, n]^T x[R, k] at the 24576-row
# minibatch: the reduction over R is cut into S row chunks computed as one batched GEMM; the chunk
# sum runs in the batched end-of-backward column-sum launch.  Small outputs (128 x 256, 256 x 512,
# ...) expose too few output tiles to fill 256 CUs, so BLAS runs them at 25-80 TFLOP/s; measured on
# MI355X, bmm only, TunableOp-tuned kernels for every variant (scripts/dw_probe.py): 128x128
# 31 -> 17 us (S=16), 128x256 52 -> 20 us (S=32), 256x512 79 -> 55 us (S=4), 768x219 105 -> 78 us
# (S=32), 256x768 106 -> 86 us (S=4).
_DW_SPLIT = {(128, 256): 32, (128, 128): 16, (256, 512): 4, (128, 705): 8, (512, 705): 2, (768, 219): 32,
             (256, 768): 4}


def _weight_grad(gh, x, red=None):
    rows, n = gh.shape
    k = x.shape[1]
    S = _DW_SPLIT.get((n, k), 1) if rows >= 8192 else 1
    if S == 1 or rows % S or not (gh.is_contiguous() and x.is_contiguous()):
        return torch.mm(gh.t(), x)
    chunks = torch.bmm(gh.view(S, rows // S, n).transpose(1, 2), x.view(S, rows // S, k))
    if red is None:
        return chunks.sum(0)
    dw = torch.empty(n, k, dtype=torch.float32, device=gh.device)
    red.add(chunks, dw, n * k, S)  # chunk sum p = 0 .. S-1, in the batched end-of-backward launch
    return dw


# the per-layer column sums of the backward run as one batched launch at its end (hg_colsum_jobs)
DEFER_REDUCTIONS = os.environ.get("HG_DEFER_REDUCTIONS", "1") != "0"


class _MLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        n = len(params) // 2
        acts = [x]
        h = x
        for i in range(n):
            W, b = params[2 * i], params[2 * i + 1]
            if i == n - 1 and _skinny_ok(h, W):
                h = _skinny_forward(h, W, b)
            else:
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
        red = _Reductions() if DEFER_REDUCTIONS else None
        for i in range(n - 1, -1, -1):
            need_dx = i > 0 or ctx.needs_input_grad[0]
            if i == n - 1 and _skinny_ok(ins[i], Ws[i]):
                # output layer: dW, db and dx as streaming passes (hg_linear_skinny_backward)
                grads[2 * i], grads[2 * i + 1], gnext = _skinny_backward(g, ins[i], Ws[i], need_dx, red)
            else:
                rows, width = g.shape
                gb = torch.empty(width, dtype=torch.float32, device=g.device)
                # layer i's output is ins[i + 1] (the ELU output) for hidden layers; identity for the last
                gh = _act_backward(g, ins[i + 1] if i < n - 1 else None, rows, width, gb, red)
                grads[2 * i + 1] = gb
                grads[2 * i] = _weight_grad(gh, ins[i], red)
                gnext = torch.mm(gh, Ws[i]) if need_dx else None
            if i > 0:
                # the next (lower) layer's incoming gradient goes through its ELU backward
                g = gnext
            else:
                gx = gnext
        if red is not None:
            red.launch(g.device)
        return (gx, *grads)


def _params(net):
    params = []
    for m in net:
        if isinstance(m, nn.Linear):
            params += [m.weight, m.bias]
    return params


def mlp_forward(net, x):
    """net(x) for a fusable Linear/ELU nn.Sequential, with the fused backward."""
    return _MLP.apply(x, *_params(net))


def mlp_infer(net, x, out=None):
    """net(x) without autograd (rollout inference): torch's Linear/ELU for the hidden layers, the
    skinny HIP kernel for the output layer (written into ``out`` when given)."""
    mods = list(net)
    h = x
    for m in mods[:-1]:
        h = m(h)
    last = mods[-1]
    if _skinny_ok(h, last.weight):
        return _skinny_forward(h, last.weight, last.bias, out)
    y = last(h)
    if out is not None:
        out.view_as(y).copy_(y)
        return out
    return y
