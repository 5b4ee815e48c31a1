"""RolloutStorage (API of humanoid/algo/ppo/rollout_storage.py:35-191).

Buffers are [T, N, ...] device tensors as in the reference.  compute_returns runs the fused HIP
GAE kernel (csrc/hg_gae.hip) — reverse-time scan + fp64 statistics + normalisation in two
launches instead of T eager steps — and, when a torch.distributed group of size > 1 is active,
all-reduces the (sum A, sum A^2) statistics between the two passes so advantages are normalised
with global statistics (collective (3)).

There is no CPU path: GAE needs the HIP kernel (tensors on a ROCm device).  Test code may set
``storage.gae_fn`` to an oracle explicitly.

Frame-only observations (``obs_frames=(F, W)``, device rollouts of a frame-stacking env): the
actor observation of slot t is the env's F-frame stack (humanoid_env.py:880-887), so the storage
keeps only its newest W-element frame per slot plus slot 0's whole stack, and a minibatch's rows
are rebuilt from them by ``hg_gather_stacked`` (the dones mark where a reset zeroed the history):
W instead of F*W observation elements written per env-step.  ``observations`` materialises the
[T, N, F*W] view on demand.
"""
import ctypes
import os

import torch
import torch.distributed as dist


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.critic_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None
            self.fused_slot = None  # storage slot already written by hg_rollout_act (device path)

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, actions_shape,
                 device="cpu", obs_dtype=torch.float32, obs_frames=None):
        """obs_dtype float16 (config 5) halves the observation buffers, the largest part of the
        storage (705 + 219 floats per env-step); minibatches are handed out in that dtype and the
        policy consumes them under autocast.  obs_frames = (F, W) with F * W = obs_shape[0]: the
        frame-only actor observation storage (module docstring)."""
        self.device = device
        self.obs_shape = obs_shape
        self.privileged_obs_shape = privileged_obs_shape
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs

        def z(*shape, dtype=torch.float32):
            return torch.zeros(T, N, *shape, device=device, dtype=dtype)

        self.obs_dtype = obs_dtype
        self.obs_frames = self.obs_init = None
        if obs_frames is not None:
            F, W = int(obs_frames[0]), int(obs_frames[1])
            if F * W != int(obs_shape[0]) or len(obs_shape) != 1:
                raise ValueError(f"obs_frames {obs_frames} do not tile the observation shape {obs_shape}")
            self.frame_stack, self.frame_width = F, W
            # [N, T, W] env-major: the newest frame of each slot's stack, a minibatch row's frames
            # one contiguous run; slot t of all envs is the strided view obs_frames[:, t]
            self.obs_frames = torch.zeros(N, T, W, device=device, dtype=obs_dtype)
            self._dones_t = None  # [N, T] u8 copy of the dones for the minibatch gathers (prepare_gather)
            self.obs_init = torch.zeros(N, F * W, device=device, dtype=obs_dtype)  # slot 0's stack
            self._observations = None
        else:
            self._observations = z(*obs_shape, dtype=obs_dtype)
        self.privileged_observations = (z(*privileged_obs_shape, dtype=obs_dtype)
                                        if privileged_obs_shape[0] is not None else None)
        self.rewards = z(1)
        self.actions = z(*actions_shape)
        self.dones = z(1, dtype=torch.uint8)
        self.actions_log_prob = z(1)
        self.values = z(1)
        self.returns = z(1)
        self.advantages = z(1)
        self.mu = z(*actions_shape)
        self.sigma = z(*actions_shape)
        self.num_transitions_per_env = T
        self.num_envs = N
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0
        self.writes = 0          # bumped by every write of a slot (add_transitions, PPO's fused act)
        self.gae_fn = None  # optional override (tests); default: HIP kernel
        self.time_outs = None  # [T, N, 1] u8, only when PPO defers the value pass (device path)
        self.values_deferred = False
        self._stats_buf = None  # [hg_gae_stats_len(N)] f64: (sum A, sum A^2) + the kernel's block partials
        self._stats = torch.zeros(2, dtype=torch.float64, device=device)

    @property
    def observations(self):
        """[T, N, obs] actor observations.  Frame-only storage: a READ-ONLY reconstruction (writing
        into it does not reach the storage — write through add_transitions), rebuilt from the
        frames + dones on every access and not kept: a cached copy would hold T x N x 705 floats
        through the next rollout and go stale under any direct write of the frames or dones.  The
        update itself never reads it (its minibatch rows come from gather_stacked)."""
        if self.obs_frames is None:
            return self._observations
        T, N = self.num_transitions_per_env, self.num_envs
        idx = torch.arange(T * N, device=self.device, dtype=torch.int64)
        out = torch.empty(T * N, self.obs_shape[0], dtype=self.obs_dtype, device=self.device)
        self.gather_stacked(idx, out)
        return out.view(T, N, -1)

    def prepare_gather(self):
        """Env-major copy of the dones ([N, T]: a row's reset scan reads one run) for the
        minibatch gathers of this update; the buffer is persistent (captured graphs read it)."""
        if self.obs_frames is None:
            return
        if self._dones_t is None:
            self._dones_t = torch.empty(self.num_envs, self.num_transitions_per_env, dtype=torch.uint8,
                                        device=self.dones.device)
        self._dones_t.copy_(self.dones.view(self.num_transitions_per_env, self.num_envs).t())

    def obs_key(self):
        """Address identifying the actor observation buffers (captured-graph keys)."""
        return (self.obs_frames if self.obs_frames is not None else self._observations).data_ptr()

    def gather_stacked(self, idx, dst, tables=(), use_prepared=False):
        """dst[i] = the stacked actor observation of storage row idx[i] (frame-only storage), one
        hg_gather_stacked launch on the current stream; dst [rows, F*W] of the storage dtype, or
        bfloat16.  ``tables``: up to two more (src [T*N, w], dst [rows, w]) pairs gathered for the
        same rows in the same launch (as gather_rows).  ``use_prepared``: read the env-major dones
        copy of prepare_gather (the caller refreshed it after the rollout)."""
        from humanoid import _native as N
        T, Nn, F, W = self.num_transitions_per_env, self.num_envs, self.frame_stack, self.frame_width
        if (idx.dtype != torch.int64 or not idx.is_contiguous() or not dst.is_contiguous()
                or dst.shape != (idx.numel(), F * W)):
            raise RuntimeError("gather_stacked: idx contiguous int64, dst contiguous [rows, F*W]")
        codes = N.DTYPE_CODES
        if len(tables) > 2:
            raise ValueError("gather_stacked takes at most two plain tables")
        tabs = (N.GatherTable * 2)()
        for k, (src, d) in enumerate(tables):
            _check_table(src, d, idx.numel(), T * Nn)
            tabs[k] = N.GatherTable(src.data_ptr(), d.data_ptr(), src.shape[1], codes[str(src.dtype)[6:]],
                                    codes[str(d.dtype)[6:]])
        s = ctypes.c_void_p(torch.cuda.current_stream(idx.device).cuda_stream)
        p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        if self._dones_t is not None and use_prepared:  # env-major copy (prepare_gather)
            dones, dts, des = self._dones_t, 1, T
        else:
            dones, dts, des = self.dones, Nn, 1
        rc = N.lib().hg_gather_stacked(p(idx), idx.numel(), p(self.obs_frames), p(self.obs_init), p(dones), dts, des,
                                       T, Nn, F, W, codes[str(self.obs_dtype)[6:]], p(dst), codes[str(dst.dtype)[6:]],
                                       tabs, len(tables), s)
        if rc != 0:
            raise RuntimeError(f"hg_gather_stacked failed ({rc})")

    def add_transitions(self, transition: Transition):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        t = self.step
        self.writes += 1
        if self.obs_frames is not None:
            if t == 0:
                self.obs_init.copy_(transition.observations)
            self.obs_frames[:, t].copy_(transition.observations[:, -self.frame_width:])
        else:
            self._observations[t].copy_(transition.observations)
        if self.privileged_observations is not None:
            self.privileged_observations[t].copy_(transition.critic_observations)
        self.actions[t].copy_(transition.actions)
        self.rewards[t].copy_(transition.rewards.view(-1, 1))
        self.dones[t].copy_(transition.dones.view(-1, 1))
        self.values[t].copy_(transition.values)
        self.actions_log_prob[t].copy_(transition.actions_log_prob.view(-1, 1))
        self.mu[t].copy_(transition.action_mean)
        self.sigma[t].copy_(transition.action_sigma)
        self.step += 1

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam):
        """GAE(gamma, lam) + advantage normalisation (rollout_storage.py:122-143)."""
        T, Nn = self.num_transitions_per_env, self.num_envs
        if self.gae_fn is not None:
            # test hook: gae_fn returns (returns, raw advantages); statistics and normalisation
            # follow the same (distributed) path as the kernel
            self.returns, raw = self.gae_fn(self.rewards, self.dones, self.values, last_values, gamma, lam)
            a = raw.double()
            self._stats = torch.stack([a.sum(), (a * a).sum()])
            count = self._reduce_stats(T * Nn)
            mean = self._stats[0] / count
            std = ((self._stats[1] - self._stats[0] * mean) / (count - 1)).clamp_min(0).sqrt()
            self.advantages = ((raw - mean.float()) / (std.float() + 1e-8)).float()
            return
        if self.rewards.device.type != "cuda":
            raise RuntimeError("RolloutStorage.compute_returns needs the HIP GAE kernel: storage must live on a "
                               "ROCm device (no CPU fallback)")
        from humanoid import _native as N
        L = N.lib()
        lv = last_values.detach().reshape(-1).contiguous().float()
        if self._stats_buf is None:
            L.hg_gae_stats_len.restype = ctypes.c_int64
            L.hg_gae_stats_len.argtypes = [ctypes.c_int]
            self._stats_buf = torch.zeros(int(L.hg_gae_stats_len(Nn)), dtype=torch.float64, device=self.rewards.device)
        # the kernel writes its block partials past stats[0..1]: always hand it the whole buffer
        # (the gae_fn hook rebinds self._stats to a fresh 2-element tensor)
        self._stats = self._stats_buf[:2]
        s = ctypes.c_void_p(torch.cuda.current_stream(self.rewards.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        N.check(L.hg_gae_scan(p(self.rewards), p(self.dones), p(self.values), p(lv), p(self.returns),
                              p(self.advantages), p(self._stats_buf), ctypes.c_int64(self._stats_buf.numel()), T, Nn,
                              ctypes.c_float(gamma), ctypes.c_float(lam), 1, s))
        count = self._reduce_stats(T * Nn)
        N.check(L.hg_gae_normalize(p(self.advantages), p(self._stats), ctypes.c_int64(count),
                                   ctypes.c_int64(T * Nn), s))

    def _reduce_stats(self, count):
        """All-reduce (sum A, sum A^2) over the data-parallel group; returns the global count."""
        if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1
                                                              or os.environ.get("HG_DP_FORCE") == "1"):
            tm = getattr(self, "comm_timer", None)
            if tm is not None:
                tm.start("allreduce_adv_stats")
            dist.all_reduce(self._stats)
            if tm is not None:
                tm.stop("allreduce_adv_stats")
            count *= dist.get_world_size()
        return count

    def get_statistics(self):
        done = self.dones
        done[-1] = 1
        flat_dones = done.permute(1, 0, 2).reshape(-1, 1)
        done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64),
                                  flat_dones.nonzero(as_tuple=False)[:, 0]))
        trajectory_lengths = done_indices[1:] - done_indices[:-1]
        return trajectory_lengths.float().mean(), self.rewards.mean()

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        """One randperm for all epochs; 12-tuple per minibatch (rollout_storage.py:153-191).
        The lin-vel target is critic_obs[:, 53:56] (base_lin_vel * 2 of the oldest critic frame)."""
        batch_size = self.num_envs * self.num_transitions_per_env
        mb = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mb, requires_grad=False, device=self.device)
        obs = self.observations.flatten(0, 1)
        critic = self.privileged_observations.flatten(0, 1) if self.privileged_observations is not None else obs
        lin_vel = critic[:, 53:56]
        actions = self.actions.flatten(0, 1)
        values = self.values.flatten(0, 1)
        returns = self.returns.flatten(0, 1)
        old_logp = self.actions_log_prob.flatten(0, 1)
        adv = self.advantages.flatten(0, 1)
        old_mu = self.mu.flatten(0, 1)
        old_sigma = self.sigma.flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mb:(i + 1) * mb]
                yield (obs[idx], critic[idx], lin_vel[idx], actions[idx], values[idx], adv[idx], returns[idx],
                       old_logp[idx], old_mu[idx], old_sigma[idx], (None, None), None)


def _check_table(src, dst, rows, src_rows):
    from humanoid import _native as N
    conv = src.dtype == dst.dtype or (dst.dtype == torch.bfloat16 and src.dtype in (torch.float16, torch.float32))
    if (src.dim() != 2 or not src.is_contiguous() or not dst.is_contiguous() or not conv
            or dst.shape != (rows, src.shape[1]) or src.shape[0] != src_rows
            or str(src.dtype)[6:] not in N.DTYPE_CODES or str(dst.dtype)[6:] not in N.DTYPE_CODES):
        raise RuntimeError("gather_rows: src [R, W] and dst [rows, W] must be contiguous float32 / float16 / "
                           "bfloat16, same dtype or a bfloat16 dst")


def gather_rows(idx, tables):
    """dst[i] = src[idx[i]] for up to three (src, dst) pairs of row-major [rows, width] device
    tensors (float32 / float16 / bfloat16), in one launch of the HIP gather kernel
    (``hg_gather_rows_ex``, csrc/hg_rollout.hip) on the current stream — graph-capturable.  Replaces
    the `table[batch_idx]` gathers of the minibatch generator (rollout_storage.py:153-191).  A
    bfloat16 dst of a float16 / float32 src is converted on the way (the bf16 policy's inputs)."""
    from humanoid import _native as N
    if not 1 <= len(tables) <= 3:
        raise ValueError("gather_rows takes one to three (src, dst) pairs")
    if idx.dtype != torch.int64 or not idx.is_cuda or not idx.is_contiguous():
        raise RuntimeError("gather_rows: idx must be a contiguous int64 device tensor")
    rows, src_rows = idx.numel(), tables[0][0].shape[0]
    tabs = (N.GatherTable * 3)()
    for t, (src, dst) in enumerate(tables):
        _check_table(src, dst, rows, src_rows)
        tabs[t] = N.GatherTable(src.data_ptr(), dst.data_ptr(), src.shape[1], N.DTYPE_CODES[str(src.dtype)[6:]],
                                N.DTYPE_CODES[str(dst.dtype)[6:]])
    s = ctypes.c_void_p(torch.cuda.current_stream(idx.device).cuda_stream)
    rc = N.lib().hg_gather_rows_ex(ctypes.c_void_p(idx.data_ptr()), rows, src_rows, tabs, len(tables), s)
    if rc != 0:
        raise RuntimeError(f"hg_gather_rows_ex failed ({rc})")
