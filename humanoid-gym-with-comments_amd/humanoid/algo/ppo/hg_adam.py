"""Adam with fused global-norm clipping on the HIP kernel ``hg_adam_step`` (csrc/hg_optim.hip).

A ``torch.optim.Optimizer`` with torch.optim.Adam's state layout (per-parameter ``step``,
``exp_avg``, ``exp_avg_sq``; one param group with ``lr``, ``betas``, ``eps``), so checkpoints
written by the reference's runner (``optimizer_state_dict``, on_policy_runner.py:294-301) load
into it and vice versa.  ``step(max_norm=...)`` performs the reference's
``clip_grad_norm_(params, max_norm); optimizer.step()`` (ppo.py:212-214) in two launches and
without host synchronisation; ``lr`` may be a device tensor (the adaptive-KL schedule keeps it on
the GPU).  Device (ROCm) tensors only — there is no CPU path.
"""
import ctypes

import torch

from humanoid import _native as N


class _TensorList(ctypes.Structure):
    M = 32
    _fields_ = [("count", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("param", ctypes.c_void_p * M), ("grad", ctypes.c_void_p * M), ("exp_avg", ctypes.c_void_p * M),
                ("exp_avg_sq", ctypes.c_void_p * M), ("step", ctypes.c_void_p * M),
                ("numel", ctypes.c_int64 * M), ("chunk_start", ctypes.c_int32 * (M + 1))]


class HgAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False,
                                      maximize=False, foreach=None, capturable=True, differentiable=False,
                                      fused=None))
        if len(self.param_groups) != 1:
            raise ValueError("HgAdam supports one parameter group")
        self._lib = N.lib()
        self._lib.hg_adam_step.restype = ctypes.c_int
        self._lib.hg_adam_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        self._chunk = int(self._lib.hg_adam_chunk())
        self.version = 0  # bumped when state tensors are replaced (captured graphs must be rebuilt)
        self._partial = None
        self._lr_host = None

    def _init_state(self):
        for p in self.param_groups[0]["params"]:
            if p.device.type != "cuda" or p.dtype != torch.float32:
                raise RuntimeError("HgAdam needs float32 parameters on a ROCm device (no CPU path)")
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            elif st["step"].device != p.device or st["step"].dtype != torch.float32:
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32)

    def load_state_dict(self, state_dict):
        # the group's lr is the live device scalar the PPO adaptive-KL rule writes (PPO._lr_f32);
        # torch's loader would replace it by the checkpoint's value and cut that link, so the
        # update graph would keep a stale constant.  The reference re-assigns param_group['lr']
        # from PPO.learning_rate before every step (ppo.py:173-174), so the loaded lr is never
        # used there either: keep the live tensor.
        lr = self.param_groups[0]["lr"]
        super().load_state_dict(state_dict)
        if torch.is_tensor(lr):
            self.param_groups[0]["lr"] = lr
        self.version += 1

    def state_dict(self):
        # lr as a Python float, as torch.optim.Adam writes it (reference checkpoints stay loadable both ways)
        sd = super().state_dict()
        for g in sd["param_groups"]:
            if torch.is_tensor(g.get("lr")):
                g["lr"] = float(g["lr"].item())
        return sd

    def _lr_tensor(self, device):
        lr = self.param_groups[0]["lr"]
        if torch.is_tensor(lr):
            return lr
        if self._lr_host is None or self._lr_host.device != device:
            self._lr_host = torch.empty((), dtype=torch.float32, device=device)
        self._lr_host.fill_(float(lr))
        return self._lr_host

    @torch.no_grad()
    def step(self, closure=None, max_norm=0.0):
        if closure is not None:
            raise ValueError("HgAdam.step does not take a closure")
        self._init_state()
        g = self.param_groups[0]
        params = [p for p in g["params"] if p.grad is not None]
        if not params:
            return None
        if len(params) > _TensorList.M:
            raise ValueError(f"HgAdam handles at most {_TensorList.M} tensors")
        T = _TensorList()
        T.count = len(params)
        c = 0
        for i, p in enumerate(params):
            if not (p.is_contiguous() and p.grad.is_contiguous()):
                raise RuntimeError("HgAdam needs contiguous parameters and gradients")
            st = self.state[p]
            T.param[i] = p.data_ptr()
            T.grad[i] = p.grad.data_ptr()
            T.exp_avg[i] = st["exp_avg"].data_ptr()
            T.exp_avg_sq[i] = st["exp_avg_sq"].data_ptr()
            T.step[i] = st["step"].data_ptr()
            T.numel[i] = p.numel()
            T.chunk_start[i] = c
            c += (p.numel() + self._chunk - 1) // self._chunk
        T.chunk_start[len(params)] = c
        dev = params[0].device
        if self._partial is None or self._partial.numel() < c or self._partial.device != dev:
            self._partial = torch.empty(max(c, 1), dtype=torch.float32, device=dev)
        lr = self._lr_tensor(dev)
        b1, b2 = g["betas"]
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        rc = self._lib.hg_adam_step(ctypes.byref(T), ctypes.c_void_p(lr.data_ptr()), float(b1), float(b2),
                                    float(g["eps"]), float(max_norm), ctypes.c_void_p(self._partial.data_ptr()), s)
        if rc != 0:
            raise RuntimeError(f"hg_adam_step failed ({rc})")
        return None
