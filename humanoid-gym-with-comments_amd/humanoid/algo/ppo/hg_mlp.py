"""Forward/backward of a Linear/ELU chain (the actor, lin-vel and critic MLPs of
actor_critic.py:36-149) with the activation backward and bias gradient fused into one HIP pass
per layer (``hg_mlp_act_backward``, csrc/hg_mlp.hip).

The weight-gradient GEMMs are torch's (hipBLASLt/rocBLAS through the TunableOp table, split-K
where it pays).  The hidden layers' forward and input-gradient products run on the build's own
LDS-staged f32 MFMA GEMM where it was measured faster (``_GEMM_FWD`` / ``_GEMM_DX``), with the bias
+ ELU, respectively the lower layer's ELU backward + bias-gradient partials, in its epilogue; the
other shapes keep torch's addmm / mm, and the ELU backward and the ``grad.sum(0)`` reduction then
run as one pass that reads the incoming gradient and the layer's ELU output once.  The layer output y (not the
pre-activation) is kept for the backward: elu'(h) = y + 1 for h <= 0.  Parameters stay in the
nn.Sequential (state_dict keys unchanged).  Device float32 only.
"""
import contextlib
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


def _skinny_backward_act(g, h, W, red):
    """The output layer's dW, db (partials into ``red``) and its input gradient through the ELU
    backward of the layer below (h = that layer's ELU output): (gh_prev, gb_prev), gb_prev's
    column sums deferred to ``red`` (hg_linear_skinny_backward_act)."""
    rows, (n, k) = g.shape[0], W.shape
    L = N.lib()
    wb = torch.empty(n * k + n, dtype=torch.float32, device=g.device)
    gh_prev = torch.empty(rows, k, dtype=torch.float32, device=g.device)
    parts = int(L.hg_linear_skinny_colpart_rows(rows))
    cp = torch.empty(parts, k, dtype=torch.float32, device=g.device)
    gb_prev = torch.empty(k, dtype=torch.float32, device=g.device)
    scratch = torch.empty(int(L.hg_linear_skinny_backward_scratch(rows, n, k)), dtype=torch.float32, device=g.device)
    rc = L.hg_linear_skinny_backward_act(g.data_ptr(), h.data_ptr(), h.stride(0), W.data_ptr(), gh_prev.data_ptr(),
                                         cp.data_ptr(), rows, n, k, scratch.data_ptr(), _stream(g.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_skinny_backward_act failed ({rc})")
    r = red if red is not None else _Reductions()
    r.add(scratch, wb, n * k + n, scratch.numel() // (n * k + n))
    r.add(cp, gb_prev, k, parts)
    if red is None:
        r.launch(g.device)
    return wb[: n * k].view(n, k), wb[n * k:], gh_prev, gb_prev


_BIG_ROWS = 1 << 40
# Split-K factors for the weight gradients dW[n, k] = gh[R, n]^T x[R, k] at the 24576-row
# minibatch: the reduction over R is cut into S row chunks computed as one batched GEMM; the chunk
# sum runs in the batched end-of-backward column-sum launch.  Small outputs (128 x 256, 256 x 512,
# ...) expose too few output tiles to fill 256 CUs, so BLAS runs them at 25-80 TFLOP/s; measured on
# MI355X, bmm only, TunableOp-tuned kernels for every variant (scripts/dw_probe.py): 128x128
# 31 -> 17 us (S=16), 128x256 52 -> 20 us (S=32), 256x512 79 -> 55 us (S=4), 768x219 105 -> 78 us
# (S=32), 256x768 106 -> 86 us (S=4).
# Re-measured with the chunk sum included (scripts/probes/dw_split_probe.py,
# profiles/r3_gemm/dw_split_with_chunk_sum.jsonl): 512x705 S=2 176 us -> S=16 161 us on hipBLASLt's
# default kernel for that bmm (a TunableOp entry tuned for it measured 185 us in place,
# dw_split_tuned_s16.jsonl, so the table keeps no entry for it); the others keep their factors
# (within 1-2 us of the best).
_DW_SPLIT = {(128, 256): 32, (128, 128): 16, (256, 512): 4, (128, 705): 8, (512, 705): 16, (768, 219): 32,
             (256, 768): 4}


# Weight gradients on the bf16-split GEMM with LDS transpose reads (hg_gemm_f32_wgrad tiles 40..54,
# k_wgrad_tr: the row-major gh and x staged as they lie, read back with ds_read_b64_tr_b16):
# (n, k) -> [(max rows, (tile, split-K slices))], first entry whose row bound covers the call
# ((tile, S) = 0: the hipBLASLt route below); the slices are summed in the batched end-of-backward
# column-sum launch.  Measured on MI355X per shape at 24576 rows (scripts/wgrad_tr_probe.py,
# profiles/r4_gemm/wgrad_tr_probe.jsonl; kernel us + the slices' share of the column sums) against
# the hipBLASLt kernels the runner's TunableOp table runs in the update (the traced minibatch,
# profiles/r4_v1): actor 512x705 147.8 -> 106 + ~8 (tile 49: 256 x 192, loads two chunks ahead,
# 32 slices), critic 256x768 76.6 -> 60 + ~8 (tile 49, 64 slices); the other products measured
# within a few us of hipBLASLt or slower (768x219 70.5 vs 64 + 10, 256x512 50.9 vs 43 + 6,
# 128x705 42.5 vs 39 + 6, 128x256 / 128x128 16.5 / 13.8 vs 17 + 7 / 12 + 6) and stay there.
WGRAD_TR = os.environ.get("HG_WGRAD_TR", "1") != "0"
_GEMM_DW = {(512, 705): [(8191, 0), (_BIG_ROWS, (49, 32))],
            (256, 768): [(8191, 0), (_BIG_ROWS, (49, 64))]} if WGRAD_TR else {}
# the other products' best tr tiles (probe); HG_WGRAD_TR=all routes all of them, a list such as
# "256x512,128x705" only those: measured 0.25 ms per iteration slower for "all" on one box
# (profiles/r4_ab), so none is routed by default
_GEMM_DW_EXTRA = {(256, 512): (54, 64), (768, 219): (54, 64), (128, 705): (48, 64), (128, 256): (54, 128),
                  (128, 128): (46, 128)}
_sel = os.environ.get("HG_WGRAD_TR", "1")
if _sel not in ("0", "1"):
    for _shape, _route_tr in _GEMM_DW_EXTRA.items():
        if _sel == "all" or "%dx%d" % _shape in _sel.split(","):
            _GEMM_DW[_shape] = [(8191, 0), (_BIG_ROWS, _route_tr)]


def _weight_grad(gh, x, red=None):
    rows, n = gh.shape
    k = x.shape[1]
    ok = red is not None and gh.is_contiguous() and x.dim() == 2 and x.stride(1) == 1
    route = _route(_GEMM_DW, rows, n, k) if ok else 0
    if route:
        tile, S = route
        L = N.lib()
        part = torch.empty(S, n, k, dtype=torch.float32, device=gh.device)
        rc = L.hg_gemm_f32_wgrad(gh.data_ptr(), gh.stride(0), x.data_ptr(), x.stride(0), part.data_ptr(), k, n * k,
                                 n, k, rows, S, 0, tile, _stream(gh.device))
        if rc != 0:
            raise RuntimeError(f"hg_gemm_f32_wgrad failed ({rc})")
        dw = torch.empty(n, k, dtype=torch.float32, device=gh.device)
        red.add(part, dw, n * k, S)
        return dw
    S = _DW_SPLIT.get((n, k), 1) if rows >= 8192 else 1
    if S == 1 or rows % S or not (gh.is_contiguous() and x.is_contiguous()):
        return torch.mm(gh.t(), x)
    chunks = torch.bmm(gh.view(S, rows // S, n).transpose(1, 2), x.view(S, rows // S, k))
    if red is None:
        return chunks.sum(0)
    dw = torch.empty(n, k, dtype=torch.float32, device=gh.device)
    red.add(chunks, dw, n * k, S)  # chunk sum p = 0 .. S-1, in the batched end-of-backward launch
    return dw


# Hidden layers y = elu(x W^T + b) on the fused f32-MFMA kernel (hg_linear_act_forward,
# csrc/hg_linear.hip: bias + ELU applied to the accumulators, one store) where it beats torch's
# addmm + ELU, i.e. the small, latency-bound products; hipBLASLt's tuned kernels stay on the large
# ones.  (k, n) -> largest row count routed to the fused kernel.  Measured on MI355X
# (scripts/linear_probe.py, profiles/r2_v3/linear_probe*.jsonl; torch addmm + ELU -> fused, us):
# 4096 rows: 512x256 24.5 -> 21.0, 256x128 24.4 -> 10.6, 128x128 24.2 -> 7.6 (16x16 wave tiles);
# 24576 rows: 128x128 24.7 -> 20.2; 705x512, 705x128, 219x768, 768x256 and every larger row count
# stay on torch.
_FUSED_FWD_ROWS = {(512, 256): 8192, (256, 128): 8192, (128, 128): 32768}
FUSED_FORWARD = os.environ.get("HG_FUSED_FORWARD", "1") != "0"


def _fused_ok(h, W, b):
    rows = h.shape[0]
    k = W.shape[1]
    return (FUSED_FORWARD and rows <= _FUSED_FWD_ROWS.get((k, W.shape[0]), 0) and h.dim() == 2 and h.stride(1) == 1
            and h.dtype == torch.float32 and W.is_contiguous() and b is not None and b.is_contiguous())


def linear_act(h, W, b, elu=True, out=None, tile=0):
    """y = elu(h W^T + b) (``elu`` False: h W^T + b) in one HIP launch on the f32 matrix cores."""
    rows, n = h.shape[0], W.shape[0]
    y = torch.empty(rows, n, dtype=torch.float32, device=h.device) if out is None else out
    if y.shape != (rows, n) or y.stride(1) != 1 or y.dtype != torch.float32:
        raise RuntimeError("linear_act: out must be a float32 [rows, n] tensor with unit column stride")
    rc = N.lib().hg_linear_act_forward(h.data_ptr(), h.stride(0), W.data_ptr(), b.data_ptr(), y.data_ptr(),
                                       y.stride(0), rows, n, W.shape[1], 1 if elu else 0, tile, _stream(h.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_act_forward failed ({rc})")
    return y


# LDS-staged f32 GEMM with the layer's elementwise work in its epilogue (hg_gemm_f32,
# csrc/hg_gemm.hip): the hidden-layer forward with bias + ELU (no separate ELU pass), and the
# input-gradient product of layer i fused with layer i-1's ELU backward and bias-gradient column
# partials (no separate hg_mlp_act_backward pass).  Routing: (k, n) of the product -> [(max rows,
# block tile)], first entry whose row bound covers the call; shapes absent from the table keep the
# previous path.  Tiles measured on MI355X per shape against torch (addmm + ELU, mm + the fused
# ELU-backward pass) and the register-operand kernel above (scripts/gemm_probe.py,
# profiles/r3_gemm/gemm_probe.jsonl).
# profiles/r3_gemm/gemm_probe_x6.jsonl (us per call, torch addmm + ELU -> this kernel): the
# bf16-split tiles (>= 19) on the large products — 24576 rows 705x512 174 -> 126 (tile 20),
# 219x768 102 -> 79 (21), 768x256 82 -> 81 (19), 512x256 60.2 -> 60.3 (22), 705x128 46.5 -> 47.6
# (23); the critic's 98304-row value pass 219x768 424 -> 305, 768x256 311 -> 264, 256x128 72 ->
# 56 (20); the f32-MFMA 64x64 tile on the small / rollout products — 24576 rows 256x128 30 -> 22.4,
# 128x128 (fused register kernel 20.2) -> 15.2; 4096 rows 705x512 35.5 -> 34.3, 512x256 21 ->
# 17.5, 705x128 26 -> 22.5.  Equal-time routes still pay: the separate ELU pass is gone.
_BIG = 1 << 40
X6_TILE0 = 19  # tiles >= 19: the bf16-split (6-term) kernels of hg_gemm_f32
_GEMM_FWD = {(705, 512): [(8192, 5), (_BIG, 20)], (512, 256): [(8192, 5), (_BIG, 22)],
             (256, 128): [(8192, 0), (32768, 5), (_BIG, 20)], (705, 128): [(8192, 5), (_BIG, 29)],
             (128, 128): [(8192, 0), (_BIG, 5)], (219, 768): [(8192, 21), (_BIG, 32)],
             (768, 256): [(32768, 22), (_BIG, 20)]}
# input gradients (24576 rows, torch mm + ELU-backward pass -> fused; gemm_probe_x6.jsonl): 256->512
# 84.7 -> 72.9 (bf16-split tile 22), 256->768 118 -> 103 (f32 tile 16), 128->256 33 -> 24.8 (16),
# 128->128 22 -> 17.9 (f32 tile 5); with the B image (below) 256->512 72.4 -> 68.6 (22), 256->768
# 103 -> 93.2 (22), 768x256 forward 84.9 (19) -> 71.2 (22) (profiles/r3_gemm/x6_image_probe.jsonl).
# Weight gradients stay on hipBLASLt: the bf16-split kernel with
# split-K slices (LDS-transposed staging of the row-major gh and x, or explicit transposes) was
# 0.57-0.94x of its tuned TN kernels on every shape.
# The 64x256 tile on 8 waves (28) with the W^T image: 256->512 72.9 -> 67.5 us (x6_image_probe_wide.jsonl).
# lin-vel's first layer 705 -> 128 on tile 29 (tile 23 with A's loads two chunks ahead): 54.3 ->
# 50.9 us at 24576 rows; the same variant of the other tiles was slower on every routed shape
# (scripts/x6_apf_probe.py, profiles/r4_gemm/x6_apf_probe.jsonl)
if os.environ.get("HG_X6_APF", "1") == "0":
    _GEMM_FWD[(705, 128)] = [(8192, 5), (_BIG, 23)]
# Round 6: tiles 30 / 31 / 32 are tiles 25 / 22 / 21 compiled for more waves per SIMD
# (k_gemm_x6_occ: registers held to 128 / 128 / 85, so 2 / 4 / 3 blocks share a CU; the same
# products in the same order, bit-identical; scripts/probes/occ_probe.py,
# profiles/r6_gemm/occ_sweep.json): at 24576 rows the paired 705 -> 640 forward 139 -> 126 us (the
# 480-block grid in one dispatch round instead of 1.875), the critic's 219 -> 768 forward 70.5 ->
# 64, its 256 -> 768 input gradient 82 -> 80; the critic's 98304-row value pass 219 -> 768 259 ->
# 243.  The same sweep moved the actor's 256 -> 512 input gradient from tile 28 (55.1 us) to 22
# (53.9).  Same-box bench A/B (HG_OCC_TILES=0, three alternations): 5.469-5.485 -> 5.495-5.503 M
# env-steps/s.  The 128 -> 256 input gradients (actor and critic, 24576 rows) moved from the f32 tile
# 16 (24.0 us) to tile 31 (20.2 us, profiles/r6_gemm/occ_sweep2.json).
_GEMM_DX = {(256, 512): [(_BIG, 22)], (128, 256): [(_BIG, 31)], (256, 768): [(_BIG, 31)], (128, 128): [(_BIG, 5)]}
GEMM = os.environ.get("HG_GEMM", "1") != "0"
# The bf16-split tiles read B (the weight) from an image split once per MLP call
# (hg_gemm_x6_image_jobs: every routed layer's forward and input-grad image in ONE launch) and
# copied to LDS by LDS-DMA, instead of loading + splitting + writing it per row tile: same result
# bit for bit, 5-15 % less time per GEMM (profiles/r3_gemm/x6_image_probe.jsonl).  Activation
# images (A) and the weight gradients from two images were measured there too and are not routed:
# a separate split pass over an activation (24576 x 705: 41 us) costs more than the GEMM saves
# (actor 705->512 117 -> 103 us), and the image-fed split-K weight gradient (123 us + 58 us of
# images for 512x705) loses to hipBLASLt's 181 us once the images are counted.
X6_IMAGE = os.environ.get("HG_X6_IMAGE", "1") != "0"
# the output layer's input gradient with the ELU backward of the layer below fused in
SKINNY_ACT = os.environ.get("HG_SKINNY_ACT", "1") != "0"


def _route(table, rows, k, n):
    if not GEMM:
        return 0
    for max_rows, tile in table.get((k, n), ()):
        if rows <= max_rows:
            return tile
    return 0


def _gemm_fwd_tile(h, W, b):
    if not (h.dim() == 2 and h.stride(1) == 1 and h.dtype == torch.float32 and W.is_contiguous() and b is not None
            and b.is_contiguous()):
        return 0
    return _route(_GEMM_FWD, h.shape[0], W.shape[1], W.shape[0])


# Split-K forwards (hg_gemm_f32_splitk): (k, n) -> [(max rows, (tile, slices))].  At the rollout's
# 4096 rows the first policy layer's one-pass tiles leave most CUs idle behind the K loop's
# per-chunk latency: 705 -> 512 on tile 5 40.4 us, as two split-K slices on tile 21 26.7 us + the
# fused sum / bias / ELU pass (profiles/r5_gemm/roll_splitk/, scripts/probes/roll_splitk_probe.py;
# the 512 -> 256 and 256 -> 128 layers gain nothing).  In the bench's kernel trace (same box):
# 37.3 us on tile 5 -> 25.6 + 8.9 us as four slices on tile 25 (21 x 2: 28.2 + 7.0 us; r5_v4: 26.0 + 9.0); a finish
# inside the GEMM launch (per-tile tickets, the last slice block summing) measured 97-174 us: its
# device-scope fences write back and invalidate the XCD's L2 under every other block
# (profiles/r5_gemm/roll_splitk/).  Rows above the bound keep _GEMM_FWD.
_GEMM_FWD_SPLITK = {(705, 512): [(4096, (25, 4))]}
SPLITK_FWD = os.environ.get("HG_SPLITK_FWD", "1") != "0"
if os.environ.get("HG_SPLITK_ROUTE"):  # "tile,slices": a diagnostic override of the 705 -> 512 route
    _GEMM_FWD_SPLITK[(705, 512)] = [(4096, tuple(int(v) for v in os.environ["HG_SPLITK_ROUTE"].split(",")))]


def _gemm_fwd_splitk(h, W, b):
    if not SPLITK_FWD or not _gemm_fwd_tile(h, W, b):
        return None
    for max_rows, route in _GEMM_FWD_SPLITK.get((W.shape[1], W.shape[0]), ()):
        if h.shape[0] <= max_rows:
            return route
    return None


def gemm_forward_splitk(h, W, b, tile, slices, elu=True):
    """y = elu(h W^T + b) as ``slices`` split-K partial products on bf16-split ``tile`` plus one
    fixed-order finishing launch (hg_gemm_f32_splitk); the slices' workspace is a per-call tensor."""
    rows, n, k = h.shape[0], W.shape[0], W.shape[1]
    y = torch.empty(rows, n, dtype=torch.float32, device=h.device)
    ws = torch.empty(slices * rows * n, dtype=torch.float32, device=h.device)
    rc = N.lib().hg_gemm_f32_splitk(h.data_ptr(), h.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), y.data_ptr(),
                                    y.stride(0), ws.data_ptr(), ws.numel(), rows, n, k, 1 if elu else 0, tile, slices,
                                    _stream(h.device))
    if rc != 0:
        raise RuntimeError(f"hg_gemm_f32_splitk failed ({rc})")
    return y


def _img_rows(r):
    return (r + 255) // 256 * 256


def x6_images(jobs, dev):
    """Operand images of the bf16-split tiles in one launch (hg_gemm_x6_image_jobs_pitched): jobs
    [(P, trans, rows, K)] (trans 0: element (r, k) = P[r][k]; trans 1: P[k][r]) or
    [("stack", (P_1, .., P_m), K)] (the trans-0 image of the P_i's rows stacked, each band written
    by its own job into the shared image; every band but the last a multiple of 256 rows, since
    each job zero-pads its band to a multiple of 256 — hgsim.h) -> one image tensor each, slices of
    a single allocation."""
    if not jobs:
        return []
    L = N.lib()

    def rows_of(j):
        return sum(P.shape[0] for P in j[1]) if j[0] == "stack" else j[2]

    sizes = [int(L.hg_gemm_x6_image_bytes(rows_of(j), j[-1])) for j in jobs]
    buf = torch.empty(sum(sizes) // 4, dtype=torch.float32, device=dev)
    imgs, off = [], 0
    for sz in sizes:
        imgs.append(buf[off // 4:(off + sz) // 4])
        off += sz
    cj = []  # (P, trans, rows, K, image address, pitch rows)
    for j, im in zip(jobs, imgs):
        if j[0] == "stack":
            total, r0 = rows_of(j), 0
            for P in j[1]:
                if r0 % 256:
                    raise ValueError("x6_images: stacked bands must start on a multiple of 256 rows "
                                     "(every band but the last a multiple of 256 rows)")
                cj.append((P, 0, P.shape[0], j[2], im.data_ptr() + 32 * r0, total))
                r0 += P.shape[0]
        else:
            cj.append((j[0], j[1], j[2], j[3], im.data_ptr(), 0))
    m = len(cj)
    vp = ctypes.c_void_p
    i64 = ctypes.c_int64
    rc = L.hg_gemm_x6_image_jobs_pitched((vp * m)(*[c[0].data_ptr() for c in cj]), (i64 * m)(*[c[0].stride(0) for c in cj]),
                                         (ctypes.c_int * m)(*[c[1] for c in cj]), (i64 * m)(*[c[2] for c in cj]),
                                         (i64 * m)(*[c[3] for c in cj]), (vp * m)(*[c[4] for c in cj]),
                                         (i64 * m)(*[c[5] for c in cj]), m, _stream(dev))
    if rc != 0:
        raise RuntimeError(f"hg_gemm_x6_image_jobs_pitched failed ({rc})")
    return imgs


def _image_specs(params, n, rows, dx, first=0):
    """The operand images an n-layer MLP call on ``rows`` rows uses: (kind, layer, W, trans, R, K)
    for its routed bf16-split forward GEMMs of layers >= ``first`` (kind "f": W itself) and, when
    ``dx``, input-grad GEMMs (kind "d": W^T)."""
    out = []
    if not (X6_IMAGE and GEMM):
        return out
    for i in range(n):
        W = params[2 * i]
        if not W.is_contiguous():
            continue
        nn_, kk = W.shape
        if first <= i < n - 1 and _route(_GEMM_FWD, rows, kk, nn_) >= X6_TILE0:
            out.append(("f", i, W, 0, nn_, kk))
        if dx and i > 0 and _route(_GEMM_DX, rows, nn_, kk) >= X6_TILE0:
            out.append(("d", i, W, 1, kk, nn_))
    return out


_SCOPE = None  # {(weight address, trans): image} while an image_scope is active


@contextlib.contextmanager
def image_scope(specs, dev, pairs=()):
    """The weight images of several fusable MLPs (``specs``: [(net, rows)]) built in ONE launch
    for the MLP calls inside the block — one image launch per PPO minibatch instead of one per
    network; ``pairs`` [(net_a, net_b, rows)]: the stacked first-layer image of mlp_pair_forward
    (those nets' own first-layer images are then not built).  The weights must not change inside
    the block."""
    global _SCOPE
    jobs, keys = [], []
    paired = set()
    for net_a, net_b, rows in pairs:
        if pair_ok(net_a, net_b, rows):
            Wa, Wb = net_a[0].weight, net_b[0].weight
            keys.append(("stack", Wa.data_ptr(), Wb.data_ptr()))
            jobs.append(("stack", (Wa, Wb), Wa.shape[1]))
            paired.update((id(net_a), id(net_b)))
    for net, rows in specs:
        if not fusable(net):
            continue
        params = _params(net)
        first = 1 if id(net) in paired else 0
        for _, _, W, trans, R, K in _image_specs(params, len(params) // 2, rows, True, first):
            key = (W.data_ptr(), trans)
            if key not in keys:
                keys.append(key)
                jobs.append((W, trans, R, K))
    prev = _SCOPE
    _SCOPE = dict(zip(keys, x6_images(jobs, dev)))
    try:
        yield
    finally:
        _SCOPE = prev


def _forward_images(params, n, rows, dev, dx, first=0):
    """{layer: image} of W for the routed bf16-split forward GEMMs (layers >= ``first``) of an
    n-layer MLP call on ``rows`` rows and, when ``dx``, of W^T for its routed bf16-split input-grad
    GEMMs — taken from the active image_scope or built in one launch."""
    fwd, dxi = {}, {}
    specs = _image_specs(params, n, rows, dx, first)
    if not specs:
        return fwd, dxi
    if _SCOPE is not None and all((W.data_ptr(), trans) in _SCOPE for _, _, W, trans, _, _ in specs):
        imgs = [_SCOPE[(W.data_ptr(), trans)] for _, _, W, trans, _, _ in specs]
    else:
        imgs = x6_images([(W, trans, R, K) for _, _, W, trans, R, K in specs], dev)
    for (kind, i, _, _, _, _), im in zip(specs, imgs):
        (fwd if kind == "f" else dxi)[i] = im
    return fwd, dxi


def _img_for(images, i, tile):
    return images.get(i) if images and tile >= X6_TILE0 else None


def gemm_forward(h, W, b, elu=True, tile=0, out=None, img=None):
    """y = elu(h W^T + b) (``elu`` False: h W^T + b) on hg_gemm_f32 (mode 0); ``img`` = W's B image
    for ``tile`` (x6_images) when given."""
    rows, n, k = h.shape[0], W.shape[0], W.shape[1]
    L = N.lib()
    if tile == 0:
        tile = int(L.hg_gemm_tile(0, rows, n, k))
    y = torch.empty(rows, n, dtype=torch.float32, device=h.device) if out is None else out
    if y.shape != (rows, n) or y.stride(1) != 1 or y.dtype != torch.float32:
        raise RuntimeError("gemm_forward: out must be a float32 [rows, n] tensor with unit column stride")
    if img is not None:
        rc = L.hg_gemm_f32_img(0, h.data_ptr(), h.stride(0), None, img.data_ptr(), b.data_ptr(), None, 0,
                               y.data_ptr(), y.stride(0), None, rows, n, k, 1 if elu else 0, tile, 0,
                               img.numel() * img.element_size(), _stream(h.device))
    else:
        rc = L.hg_gemm_f32(0, h.data_ptr(), h.stride(0), W.data_ptr(), W.stride(0), b.data_ptr(), None, 0,
                           y.data_ptr(), y.stride(0), None, rows, n, k, 1 if elu else 0, tile, _stream(h.device))
    if rc != 0:
        raise RuntimeError(f"hg_gemm_f32 (forward) failed ({rc})")
    return y


def gemm_input_grad(gh, W, y_prev, gb, red=None, tile=0, img=None):
    """(gh W) * elu'(y_prev) — layer i's input gradient through layer i-1's ELU backward (its
    pre-activation gradient) — with layer i-1's bias gradient gb = column sums, on hg_gemm_f32
    (mode 1).  gh [rows, n_i] contiguous, W [n_i, k_i] (nn.Linear.weight), y_prev [rows, k_i]."""
    rows, kr = gh.shape
    n = W.shape[1]
    L = N.lib()
    if tile == 0:
        tile = int(L.hg_gemm_tile(1, rows, n, kr))
    out = torch.empty(rows, n, dtype=torch.float32, device=gh.device)
    parts = int(L.hg_gemm_colpart_rows(rows, tile))
    cp = torch.empty(parts, n, dtype=torch.float32, device=gh.device)
    # W read as is ([n_i, k_i], n-contiguous in the reduction index): the f32 tiles stage it with
    # coalesced scalar loads, the bf16-split tiles through an LDS transpose (mode 3 with a W^T copy
    # measured no faster, profiles/r3_gemm/gemm_probe_x6.jsonl)
    # (``img``: W^T's B image for ``tile``, x6_images trans 1)
    if img is not None:
        rc = L.hg_gemm_f32_img(1, gh.data_ptr(), gh.stride(0), None, img.data_ptr(), None, y_prev.data_ptr(),
                               y_prev.stride(0), out.data_ptr(), out.stride(0), cp.data_ptr(), rows, n, kr, 1, tile,
                               0, img.numel() * img.element_size(), _stream(gh.device))
    else:
        rc = L.hg_gemm_f32(1, gh.data_ptr(), gh.stride(0), W.data_ptr(), W.stride(0), None, y_prev.data_ptr(),
                           y_prev.stride(0), out.data_ptr(), out.stride(0), cp.data_ptr(), rows, n, kr, 1, tile,
                           _stream(gh.device))
    if rc != 0:
        raise RuntimeError(f"hg_gemm_f32 (input grad) failed ({rc})")
    if red is None:
        r = _Reductions()
        r.add(cp, gb, n, parts)
        r.launch(gh.device)
    else:
        red.add(cp, gb, n, parts)
    return out


def _gemm_dx_tile(gh, W, y_prev):
    if not (gh.is_contiguous() and W.is_contiguous() and y_prev.dim() == 2 and y_prev.stride(1) == 1
            and y_prev.dtype == torch.float32):
        return 0
    return _route(_GEMM_DX, gh.shape[0], W.shape[0], W.shape[1])


# the per-layer column sums of the backward run as one batched launch at its end (hg_colsum_jobs)
DEFER_REDUCTIONS = os.environ.get("HG_DEFER_REDUCTIONS", "1") != "0"


def _hidden_forward(h, W, b, images=None, i=0):
    """One hidden layer: the LDS-staged GEMM (with layer i's B image from ``images`` when built for
    the routed tile), the register-operand fused kernel, or addmm + ELU."""
    split = _gemm_fwd_splitk(h, W, b)
    if split is not None:
        return gemm_forward_splitk(h, W, b, *split)
    tile = _gemm_fwd_tile(h, W, b)
    if tile:
        return gemm_forward(h, W, b, True, tile, img=_img_for(images, i, tile))
    if _fused_ok(h, W, b):
        return linear_act(h, W, b)
    return F.elu(torch.addmm(b, h, W.t()))


def _mlp_forward_layers(h, params, n, fimg, first, acts):
    """Layers ``first`` .. n-1 of an n-layer MLP from h (layer ``first``'s input, appended to
    ``acts`` with every later layer's input); returns the output."""
    acts.append(h)
    for i in range(first, n):
        W, b = params[2 * i], params[2 * i + 1]
        if i == n - 1 and _skinny_ok(h, W):
            h = _skinny_forward(h, W, b)
        elif i < n - 1:
            h = _hidden_forward(h, W, b, fimg, i)
        else:
            h = torch.addmm(b, h, W.t())
        if i < n - 1:
            acts.append(h)
    return h


def _mlp_backward_layers(g, ins, Ws, n, dximg, need_x, red):
    """The backward of an n-layer MLP from the output gradient g: ins = the inputs of every layer
    (x, y_0 .. y_{n-2}), Ws its weights; returns ([dW_0, db_0, ..], dx or None).  The column sums
    go to ``red`` (launched by the caller)."""
    grads = [None] * (2 * n)
    g = g.contiguous()
    gx = None
    pre = None  # (gh, gb) of layer i when the layer above produced them in its input-grad GEMM
    for i in range(n - 1, -1, -1):
        need_dx = i > 0 or need_x
        gnext = None
        if i == n - 1 and _skinny_ok(ins[i], Ws[i]):
            if i > 0 and SKINNY_ACT:
                # output layer: dW, db and the layer below's pre-activation gradient + bias
                # gradient partials (its ELU backward fused into the skinny dX pass)
                grads[2 * i], grads[2 * i + 1], gh_prev, gb_prev = _skinny_backward_act(g, ins[i], Ws[i], red)
                pre = (gh_prev, gb_prev)
            else:
                # output layer: dW, db and dx as streaming passes (hg_linear_skinny_backward)
                grads[2 * i], grads[2 * i + 1], gnext = _skinny_backward(g, ins[i], Ws[i], need_dx, red)
        else:
            if pre is not None:
                gh, gb = pre
                pre = None
            else:
                rows, width = g.shape
                gb = torch.empty(width, dtype=torch.float32, device=g.device)
                # layer i's output is ins[i + 1] (the ELU output) for hidden layers; identity for the last
                gh = _act_backward(g, ins[i + 1] if i < n - 1 else None, rows, width, gb, red)
            grads[2 * i + 1] = gb
            grads[2 * i] = _weight_grad(gh, ins[i], red)
            if need_dx:
                tile = _gemm_dx_tile(gh, Ws[i], ins[i]) if i > 0 else 0
                if tile:
                    # layer i-1's pre-activation gradient and bias gradient straight from this GEMM
                    gb_prev = torch.empty(Ws[i].shape[1], dtype=torch.float32, device=gh.device)
                    pre = (gemm_input_grad(gh, Ws[i], ins[i], gb_prev, red, tile, _img_for(dximg, i, tile)),
                           gb_prev)
                else:
                    gnext = torch.mm(gh, Ws[i])
        if i > 0:
            # the next (lower) layer's incoming gradient goes through its ELU backward
            g = gnext
        else:
            gx = gnext
    return grads, gx


class _MLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        n = len(params) // 2
        fimg, ctx.dximg = _forward_images(params, n, x.shape[0], x.device, any(ctx.needs_input_grad))
        acts = []
        h = _mlp_forward_layers(x, params, n, fimg, 0, acts)
        # inputs of every layer (x, y_0 .. y_{n-2}) and the weights
        ctx.save_for_backward(*acts, *params[0::2])
        ctx.n = n
        return h

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        ins, Ws = saved[:n], saved[n:]
        red = _Reductions() if DEFER_REDUCTIONS else None
        grads, gx = _mlp_backward_layers(g, ins, Ws, n, ctx.dximg, ctx.needs_input_grad[0], red)
        if red is not None:
            red.launch(ins[0].device)
        ctx.dximg = None
        return (gx, *grads)


# Two MLPs reading the same input (the actor and the lin-vel estimator, both on the actor
# observations: actor_critic.py act / base_get_lin_vel) with their first layers as ONE GEMM: the
# stacked weight [n_a + n_b, K] from a stacked image (x6_images "stack", no weight copy), bias +
# ELU in the epilogue (each network's own bias), each network's columns stored to its own contiguous [rows, n] output
# (hg_gemm_f32_img_split), so the rest of each network and its backward run exactly as apart.
# (K, n_a + n_b) -> [(max rows, tile)]: 705 -> 640 at 24576 rows on tile 25, 143 us against 128 + 40
# for the two products apart (scripts/gemm_tile_sweep.py, profiles/r5_gemm/gemm_tile_sweep.json).
_PAIR_FWD = {(705, 640): [(8192, 0), (_BIG, 30)]}
if os.environ.get("HG_OCC_TILES", "1") == "0":  # A/B: the round-5 tiles
    _PAIR_FWD[(705, 640)] = [(8192, 0), (_BIG, 25)]
    _GEMM_DX[(256, 768)] = [(_BIG, 22)]
    _GEMM_DX[(256, 512)] = [(_BIG, 28)]
    _GEMM_DX[(128, 256)] = [(_BIG, 16)]
    _GEMM_FWD[(219, 768)] = [(32768, 21), (_BIG, 20)]
PAIR_FIRST = os.environ.get("HG_PAIR_FIRST", "1") != "0"


def pair_ok(net_a, net_b, rows):
    """net_a and net_b (fusable, fp32) can run their first layers as one stacked GEMM on ``rows``."""
    if not (PAIR_FIRST and GEMM and X6_IMAGE and fusable(net_a) and fusable(net_b)):
        return False
    la, lb = net_a[0], net_b[0]
    if len(net_a) < 3 or len(net_b) < 3 or la.in_features != lb.in_features or la.out_features % 256:
        return False
    ps = (la.weight, lb.weight, la.bias, lb.bias)
    if not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in ps):
        return False
    return _route(_PAIR_FWD, rows, la.in_features, la.out_features + lb.out_features) >= X6_TILE0


class _MLPPair(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, na, *params):
        pa, pb = params[:2 * na], params[2 * na:]
        nb = len(pb) // 2
        rows, K = x.shape
        Wa, Wb = pa[0], pb[0]
        ma, mb = Wa.shape[0], Wb.shape[0]
        key = ("stack", Wa.data_ptr(), Wb.data_ptr())
        img = _SCOPE.get(key) if _SCOPE is not None else None
        if img is None:
            img = x6_images([("stack", (Wa, Wb), K)], x.device)[0]
        tile = _route(_PAIR_FWD, rows, K, ma + mb)
        ha = torch.empty(rows, ma, dtype=torch.float32, device=x.device)
        hb = torch.empty(rows, mb, dtype=torch.float32, device=x.device)
        # one GEMM, each network's columns into its own contiguous output (the later layers and the
        # backward then see exactly the operands of the separate calls)
        rc = N.lib().hg_gemm_f32_img_split(x.data_ptr(), x.stride(0), img.data_ptr(), pa[1].data_ptr(), pb[1].data_ptr(),
                                           ha.data_ptr(), ma,
                                           hb.data_ptr(), mb, ma, rows, ma + mb, K, 1, tile,
                                           img.numel() * img.element_size(), _stream(x.device))
        if rc != 0:
            raise RuntimeError(f"hg_gemm_f32_img_split (paired first layers) failed ({rc})")
        need = any(ctx.needs_input_grad)
        fa, ctx.dxa = _forward_images(pa, na, rows, x.device, need, first=1)
        fb, ctx.dxb = _forward_images(pb, nb, rows, x.device, need, first=1)
        acts_a, acts_b = [x], [x]
        ya = _mlp_forward_layers(ha, pa, na, fa, 1, acts_a)
        yb = _mlp_forward_layers(hb, pb, nb, fb, 1, acts_b)
        ctx.save_for_backward(*acts_a, *acts_b, *pa[0::2], *pb[0::2])
        ctx.na, ctx.nb = na, nb
        return ya, yb

    @staticmethod
    def backward(ctx, ga, gb):
        na, nb = ctx.na, ctx.nb
        saved = ctx.saved_tensors
        ins_a, ins_b = saved[:na], saved[na:na + nb]
        Wsa, Wsb = saved[na + nb:2 * na + nb], saved[2 * na + nb:]
        red = _Reductions() if DEFER_REDUCTIONS else None
        need_x = ctx.needs_input_grad[0]
        dev = ins_a[0].device
        if ga is None:
            ga = torch.zeros(ins_a[0].shape[0], Wsa[-1].shape[0], dtype=torch.float32, device=dev)
        if gb is None:
            gb = torch.zeros(ins_b[0].shape[0], Wsb[-1].shape[0], dtype=torch.float32, device=dev)
        grads_a, gxa = _mlp_backward_layers(ga, ins_a, Wsa, na, ctx.dxa, need_x, red)
        grads_b, gxb = _mlp_backward_layers(gb, ins_b, Wsb, nb, ctx.dxb, need_x, red)
        if red is not None:
            red.launch(dev)
        ctx.dxa = ctx.dxb = None
        gx = None if not need_x else gxa + gxb
        return (gx, None, *grads_a, *grads_b)


def mlp_pair_forward(net_a, net_b, x):
    """(net_a(x), net_b(x)) with the two first layers as one stacked GEMM (pair_ok) and the fused
    backward of each network; the separate mlp_forward calls otherwise."""
    if x.dim() == 2 and x.is_cuda and x.dtype == torch.float32 and x.stride(1) == 1 and pair_ok(net_a, net_b, x.shape[0]):
        pa, pb = _params(net_a), _params(net_b)
        return _MLPPair.apply(x, len(pa) // 2, *pa, *pb)
    return mlp_forward(net_a, x), mlp_forward(net_b, x)


def _params(net):
    params = []
    for m in net:
        if isinstance(m, nn.Linear):
            params += [m.weight, m.bias]
    return params


def mlp_forward(net, x):
    """net(x) for a fusable Linear/ELU nn.Sequential, with the fused backward."""
    return _MLP.apply(x, *_params(net))


def mlp_infer_hidden(net, x):
    """mlp_infer's hidden layers only: the last hidden activation, for callers that fuse the output
    layer into their own launch (hg_rollout_act_head); None when ``net`` is not fusable."""
    if not fusable(net):
        return None
    mods = list(net)
    params = _params(net)
    fimg = _forward_images(params, len(params) // 2, x.shape[0], x.device, False)[0]
    h = x
    for j in range(0, len(mods) - 1, 2):
        lin = mods[j]
        if isinstance(mods[j + 1], nn.ELU) and mods[j + 1].alpha == 1.0 and not mods[j + 1].inplace:
            h = _hidden_forward(h, lin.weight, lin.bias, fimg, j // 2)
        else:
            h = mods[j + 1](lin(h))
    return h


# the actor's last hidden layer folded into the sampling launch as well (hg_rollout_act_tail)
TAIL_FUSED = os.environ.get("HG_ACT_TAIL", "1") != "0"


def mlp_infer_tail(net, x):
    """For hg_rollout_act_tail: the hidden layers of ``net`` but its last one, as mlp_infer_hidden
    runs them, and that last hidden layer's (W, b) -> (h, W, b); None (nothing computed) unless
    that layer is 128 wide and its separate route would be linear_act's 16 x 16 tile on aligned
    rows — so the fused launch gives the separate launches' bits."""
    if not (TAIL_FUSED and fusable(net)):
        return None
    mods = list(net)
    if len(mods) < 5:
        return None
    lin = mods[-3]
    W, b = lin.weight, lin.bias
    rows, K = x.shape[0], W.shape[1]
    if (W.device != x.device or not x.is_cuda or x.dim() != 2 or x.dtype != torch.float32
            or W.shape[0] != 128 or K % 4 or not W.is_contiguous() or W.data_ptr() % 16 or not b.is_contiguous()
            or _route(_GEMM_FWD, rows, K, 128) or (K, 128) in _GEMM_FWD_SPLITK or not FUSED_FORWARD
            or rows > _FUSED_FWD_ROWS.get((K, 128), 0) or int(N.lib().hg_linear_act_tile(rows, 128, K)) != 5):
        return None
    params = _params(net)
    fimg = _forward_images(params, len(params) // 2, rows, x.device, False)[0]
    h = x
    for j in range(0, len(mods) - 3, 2):
        h = _hidden_forward(h, mods[j].weight, mods[j].bias, fimg, j // 2)
    if not (h.dim() == 2 and h.dtype == torch.float32 and h.stride(1) == 1 and h.stride(0) % 4 == 0
            and h.data_ptr() % 16 == 0 and h.shape[1] == K):
        h = h.contiguous()
    return h, W, b


def head_fusable(h, W):
    """The output layer W applied to h can run inside hg_rollout_act_head (12 x 128, aligned rows)."""
    return (h is not None and tuple(W.shape) == (12, 128) and W.is_contiguous() and h.dim() == 2
            and h.dtype == torch.float32 and h.stride(1) == 1 and h.stride(0) % 4 == 0 and h.data_ptr() % 16 == 0
            and W.data_ptr() % 16 == 0)


def mlp_infer(net, x, out=None):
    """net(x) without autograd (rollout inference): hidden layers on the LDS-staged GEMM or the
    register-operand fused kernel where ``_GEMM_FWD`` / ``_FUSED_FWD_ROWS`` route them, torch's
    Linear/ELU otherwise; the skinny HIP kernel for the output layer (written into ``out`` when
    given)."""
    mods = list(net)
    h = x
    fimg = None
    if fusable(net):
        params = _params(net)
        fimg = _forward_images(params, len(params) // 2, x.shape[0], x.device, False)[0]
    for j in range(0, len(mods) - 1, 2):
        lin = mods[j]
        if isinstance(mods[j + 1], nn.ELU) and mods[j + 1].alpha == 1.0 and not mods[j + 1].inplace:
            h = _hidden_forward(h, lin.weight, lin.bias, fimg, j // 2)
        else:
            h = mods[j + 1](lin(h))
    last = mods[-1]
    if _skinny_ok(h, last.weight):
        return _skinny_forward(h, last.weight, last.bias, out)
    y = last(h)
    if out is not None:
        out.view_as(y).copy_(y)
        return out
    return y


# ---------------------------------------------------------------------------------------------
# bf16 policy (config 5, ``policy_dtype="bf16"``).  Master weights, gradients and Adam stay fp32
# (HgAdam unchanged); a forward casts the hidden layers' weights and biases to bf16 in one launch
# (hg_cast_bf16_jobs) and runs the hidden GEMMs as bf16 x bf16 -> bf16 with fp32 accumulation
# (hipBLASLt on the bf16 matrix cores), ELU in bf16.  The skinny output layer reads its bf16 input
# with the fp32 W and writes fp32 (the loss, the sample and the value see fp32 outputs).  Backward:
# the activation gradients flow in bf16 through the fused ELU-backward/bias pass
# (hg_mlp_act_backward_bf16, fp32 bias partials), the weight gradients are bf16 GEMMs with fp32
# output (``out_dtype=torch.float32``: no bf16 rounding of the accumulated gradient), and the
# skinny layer's dW/db are fp32 partials of the same deterministic column sums.
# ---------------------------------------------------------------------------------------------
_BF16 = torch.bfloat16


def fusable_bf16(net):
    """fusable(net) with an output layer the skinny bf16-input kernels handle."""
    if not fusable(net):
        return False
    last = list(net)[-1]
    return bool(N.lib().hg_linear_skinny_supported(last.out_features, last.in_features))


def cast_hidden_bf16(params):
    """bf16 copies of the hidden layers' (W, b) — all but the last pair of ``params`` — in ONE
    hg_cast_bf16_jobs launch.  Returns [W0, b0, W1, b1, ...] as bf16 tensors."""
    src = [p.detach() for p in params[:-2]]
    if not src:
        return []
    src = [p if p.is_contiguous() else p.contiguous() for p in src]
    dst = [torch.empty(p.shape, dtype=_BF16, device=p.device) for p in src]
    n = len(src)
    vp = ctypes.c_void_p
    rc = N.lib().hg_cast_bf16_jobs((vp * n)(*[p.data_ptr() for p in src]), (vp * n)(*[d.data_ptr() for d in dst]),
                                   (ctypes.c_int64 * n)(*[p.numel() for p in src]), n, _stream(src[0].device))
    if rc != 0:
        raise RuntimeError(f"hg_cast_bf16_jobs failed ({rc})")
    return dst


def _skinny_ok_bf16(h, W):
    n, k = W.shape
    return (bool(N.lib().hg_linear_skinny_supported(n, k)) and h.dim() == 2 and h.dtype == _BF16
            and h.stride(1) == 1 and h.stride(0) % 8 == 0 and h.data_ptr() % 16 == 0 and W.is_contiguous())


def _skinny_forward_bf16(h, W, b, out=None):
    rows, n = h.shape[0], W.shape[0]
    y = torch.empty(rows, n, dtype=torch.float32, device=h.device) if out is None else out
    if y.numel() != rows * n or not y.is_contiguous() or y.dtype != torch.float32:
        raise RuntimeError("skinny forward: out must be a contiguous float32 tensor of rows x n elements")
    rc = N.lib().hg_linear_skinny_forward_bf16(h.data_ptr(), h.stride(0), W.data_ptr(), b.data_ptr(), y.data_ptr(),
                                               rows, n, W.shape[1], _stream(h.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_skinny_forward_bf16 failed ({rc})")
    return y


def _skinny_backward_bf16(g, h, W, need_dx, red):
    rows, (n, k) = g.shape[0], W.shape
    L = N.lib()
    wb = torch.empty(n * k + n, dtype=torch.float32, device=g.device)
    dx = torch.empty(rows, k, dtype=_BF16, device=g.device) if need_dx else None
    scratch = torch.empty(int(L.hg_linear_skinny_backward_scratch(rows, n, k)), dtype=torch.float32, device=g.device)
    rc = L.hg_linear_skinny_backward_bf16(g.data_ptr(), h.data_ptr(), h.stride(0), W.data_ptr(),
                                          dx.data_ptr() if need_dx else None, None, rows, n, k, scratch.data_ptr(),
                                          _stream(g.device))
    if rc != 0:
        raise RuntimeError(f"hg_linear_skinny_backward_bf16 failed ({rc})")
    red.add(scratch, wb, n * k + n, scratch.numel() // (n * k + n))
    return wb[: n * k].view(n, k), wb[n * k:], dx


def _act_backward_bf16(gy, y, gb, red):
    rows, width = gy.shape
    L = N.lib()
    scratch = torch.empty(int(L.hg_mlp_act_backward_scratch(rows, width)), dtype=torch.float32, device=gy.device)
    gh = torch.empty_like(gy)
    rc = L.hg_mlp_act_backward_bf16(gy.data_ptr(), y.data_ptr(), gh.data_ptr(), rows, width, None,
                                    scratch.data_ptr(), _stream(gy.device))
    if rc != 0:
        raise RuntimeError(f"hg_mlp_act_backward_bf16 failed ({rc})")
    red.add(scratch, gb, width, scratch.numel() // width)
    return gh


# Split-K of the bf16 weight gradients as rows per chunk (S = rows / chunk, a power of two that
# divides rows): hipBLASLt's bf16 -> fp32 GEMM over the whole minibatch runs the [n, k] output on a
# handful of tiles (160-260 us at 49152 rows).  Measured on MI355X (scripts/bf16_gemm_probe.py,
# 49152 / 24576 rows, bmm with fp32 chunk outputs + the chunk-sum read): 512x705 260 -> 64 us
# (S=32), 256x512 219 -> 30, 128x256 171 -> 21, 128x705 202 -> 42, 768x219 216 -> 44, 256x768
# 226 -> 44; best at 1536-3072 rows per chunk (128x128: 6144).
_DW_CHUNK_BF16 = {(128, 128): 6144, (128, 256): 3072}
_DW_CHUNK_BF16_DEFAULT = 1536


def _bf16_split(rows, n, k):
    S = 1
    chunk = _DW_CHUNK_BF16.get((n, k), _DW_CHUNK_BF16_DEFAULT)
    while S < 64 and rows % (2 * S) == 0 and rows // (2 * S) >= chunk:
        S *= 2
    return S


def _weight_grad_bf16(gh, x, red):
    """dW[n, k] = gh^T x from bf16 operands, accumulated and returned in fp32."""
    rows, n = gh.shape
    k = x.shape[1]
    S = _bf16_split(rows, n, k)
    if S == 1:
        return torch.mm(gh.t(), x, out_dtype=torch.float32)
    chunks = torch.bmm(gh.view(S, rows // S, n).transpose(1, 2), x.view(S, rows // S, k), out_dtype=torch.float32)
    dw = torch.empty(n, k, dtype=torch.float32, device=gh.device)
    red.add(chunks, dw, n * k, S)
    return dw


def _hidden_forward_bf16(x, wb):
    """bf16 input of every layer: [x, y_0, ..., y_{n-2}] (y_i = elu(h W_i^T + b_i) in bf16)."""
    h = x if x.dtype == _BF16 else x.to(_BF16)
    if not h.is_contiguous():
        h = h.contiguous()
    ins = [h]
    for i in range(len(wb) // 2):
        h = F.elu(torch.addmm(wb[2 * i + 1], h, wb[2 * i].t()))
        ins.append(h)
    return ins


class _MLPbf16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        n = len(params) // 2
        wb = cast_hidden_bf16(params)
        ins = _hidden_forward_bf16(x, wb)
        Wl, bl = params[-2], params[-1]
        y = _skinny_forward_bf16(ins[-1], Wl, bl)
        ctx.save_for_backward(*ins, *wb[0::2], Wl)
        ctx.n = n
        ctx.x_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        ins, Wbs, Wl = saved[:n], saved[n:2 * n - 1], saved[2 * n - 1]
        grads = [None] * (2 * n)
        g = g.contiguous().float()
        red = _Reductions()
        need_x = ctx.needs_input_grad[0]
        grads[-2], grads[-1], g = _skinny_backward_bf16(g, ins[n - 1], Wl, n > 1 or need_x, red)
        for i in range(n - 2, -1, -1):
            rows, width = g.shape
            gb = torch.empty(width, dtype=torch.float32, device=g.device)
            gh = _act_backward_bf16(g, ins[i + 1], gb, red)
            grads[2 * i + 1] = gb
            grads[2 * i] = _weight_grad_bf16(gh, ins[i], red)
            g = torch.mm(gh, Wbs[i]) if (i > 0 or need_x) else None
        red.launch(ins[0].device)
        gx = g.to(ctx.x_dtype) if (need_x and g is not None) else None
        return (gx, *grads)


def mlp_forward_bf16(net, x):
    """net(x) for a ``fusable_bf16`` nn.Sequential on the bf16 path, fp32 output, fused backward."""
    return _MLPbf16.apply(x, *_params(net))


def mlp_infer_bf16(net, x, out=None):
    """net(x) on the bf16 path without autograd (rollout inference); fp32 output (into ``out``)."""
    params = [p.detach() for p in _params(net)]
    ins = _hidden_forward_bf16(x, cast_hidden_bf16(params))
    return _skinny_forward_bf16(ins[-1], params[-2], params[-1], out)
