"""PPO (constructor kwargs, act/process_env_step/compute_returns/update and the 4-tuple return of
humanoid/algo/ppo/ppo.py:44-226).

Update math (per minibatch, in the reference's order): adaptive-KL learning rate, clipped
surrogate, clipped value loss, lin-vel MSE, entropy bonus, Adam step after global-norm clipping.

Data parallel (new): when torch.distributed is initialised with world_size > 1
(backend "nccl" = RCCL on ROCm), parameters are broadcast from rank 0 once, each rank's gradients
live in ONE flat buffer that is all-reduced (SUM / world) before clip_grad_norm_, and kl_mean is
all-reduced so the adaptive learning rate stays identical on every rank.  With world_size 1 the
path is the reference's.

Sync-free update on a ROCm device: the adaptive learning rate is a float64 device scalar updated
with the reference's rule (torch.where instead of Python branches on kl_mean.item()) and fed to
the fused Adam kernel as a tensor; the three loss means are accumulated on the device and read
once per update.  The host therefore never waits for the GPU inside the minibatch loop.  On the
CPU the reference's host-side arithmetic is kept verbatim (this is what the golden tests pin).
"""
import contextlib
import ctypes
import os
import warnings

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim

from .actor_critic import ActorCritic, _DiagGaussian
from .hg_adam import HgAdam
from . import hg_mlp
from . import hg_loss
from .hg_loss import ppo_loss
from .rollout_storage import RolloutStorage, gather_rows

# the actor's 12 x 128 output layer fused into the rollout's sampling launch (hg_rollout_act_head)
HEAD_FUSED = os.environ.get("HG_HEAD_FUSED", "1") != "0"
# the env's post launch writes the rollout slot's rewards / dones / time-outs (set_rollout_sink)
ROLLOUT_SINK = os.environ.get("HG_ROLLOUT_SINK", "1") != "0"
# the adaptive-KL learning-rate rule inside the loss's final launch (hg_ppo_loss_lr), one process
FUSED_LR_RULE = os.environ.get("HG_FUSED_LR_RULE", "1") != "0"


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def _data_parallel():
    """True when the update all-reduces its gradients: world size > 1, or (HG_DP_FORCE=1) an
    initialised world-size-1 group, which runs the multi-rank code path — flat gradient buffer, the
    per-minibatch collective between the two captured graphs — on one device (test of the RCCL path
    on a one-GPU box)."""
    if _world() > 1:
        return True
    return (os.environ.get("HG_DP_FORCE") == "1" and dist.is_available() and dist.is_initialized())



@contextlib.contextmanager
def _capturing(g, mode, pool=None):
    """torch.cuda.graph without its one failure mode that matters here: when the body raises and
    capture_end raises too, torch.cuda.graph leaves the side stream current.  The stream context is
    the outer one, so it is restored whatever happens inside."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    with torch.cuda.stream(torch.cuda.Stream()):
        g.capture_begin(*(() if pool is None else (pool,)), capture_error_mode=mode)
        try:
            yield
        finally:
            g.capture_end()


def _slot_views(st, t):
    """Per-slot views and device pointers of the rollout storage, built once per (storage, slot):
    indexing eleven storage tensors per policy step cost tens of microseconds of host time, on a
    step whose GPU time is ≈340 us.  The storage tensors are allocated once and written in place."""
    cache = st.__dict__.setdefault("_slot_cache", {})
    sl = cache.get(t)
    if sl is None:
        vp = ctypes.c_void_p
        priv = st.privileged_observations
        sl = {"actions": st.actions[t], "values": st.values[t], "logp": st.actions_log_prob[t].view(-1),
              "mu": st.mu[t], "sigma": st.sigma[t], "rewards": st.rewards[t], "dones": st.dones[t]}
        sl.update(p_actions=vp(sl["actions"].data_ptr()), p_logp=vp(st.actions_log_prob[t].data_ptr()),
                  p_mu=vp(sl["mu"].data_ptr()), p_sigma=vp(sl["sigma"].data_ptr()), p_values=vp(sl["values"].data_ptr()),
                  p_obs=vp(st.obs_frames[:, t].data_ptr() if st.obs_frames is not None else st.observations[t].data_ptr()),
                  p_priv=vp(priv[t].data_ptr()) if priv is not None else None,
                  p_rewards=vp(sl["rewards"].data_ptr()), p_dones=vp(sl["dones"].data_ptr()))
        cache[t] = sl
    return sl


def _as_u8(x):
    """0/1 byte mask for the HIP kernels: bool/uint8 reinterpreted in place, any other dtype (the
    reference's int64 reset_buf) converted."""
    x = x.contiguous()
    if x.dtype in (torch.bool, torch.uint8):
        return x.view(torch.uint8)
    return (x != 0).to(torch.uint8)

class PPO:
    actor_critic: ActorCritic

    def __init__(self, actor_critic, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998,
                 lam=0.95, value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu", sym_loss=False,
                 obs_permutation=None, act_permutation=None, frame_stack=0, sym_coef=1.0, base_lin_vel_coef=1.0):
        self.device = device
        self._lr = float(learning_rate)
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.actor_critic = actor_critic
        self.actor_critic.to(self.device)
        self.storage = None
        self.world_size = _world()
        self._dp = _data_parallel()
        self._params = list(self.actor_critic.parameters())
        self._on_device = torch.device(device).type == "cuda"
        self.use_graphs = self._on_device
        self._graphs = None
        self._graph_warm = False
        self.update_graph = "eager"   # the update form last run: "eager" | "one" | "two" graphs
        self.capture_error = None     # why the in-graph collective fell back, if it did
        # optional timer with start(name) / stop(name) (bench.py KernelTimer: HIP events on the
        # current stream, sampled): brackets every eager data-parallel all-reduce as "allreduce"
        self.comm_timer = None
        self._flat_grad = None
        if self._dp:
            with torch.no_grad():
                for p in self._params:
                    dist.broadcast(p.data, src=0)
        if self._dp:
            # persistent flat gradient buffer: one all-reduce per minibatch, no pack/unpack copies
            numel = sum(p.numel() for p in self._params)
            # + one trailing slot: the minibatch KL mean rides along with the gradient all-reduce
            self._flat_grad = torch.zeros(numel + 1, device=self._params[0].device, dtype=torch.float32)
            self._kl_slot = self._flat_grad[numel:]
            off = 0
            for p in self._params:
                p.grad = self._flat_grad[off:off + p.numel()].view_as(p)
                off += p.numel()
        if self._on_device:
            # float64 master (the reference's Python-float arithmetic) + the float32 copy the fused
            # Adam kernel reads
            self._lr_t = torch.tensor(float(learning_rate), dtype=torch.float64, device=device)
            self._lr_f32 = self._lr_t.float()
            # fused clip + Adam HIP kernel (csrc/hg_optim.hip); torch.optim.Adam state layout
            self.optimizer = HgAdam(self._params, lr=self._lr_f32)
        else:
            self._lr_t = None
            self.optimizer = optim.Adam(self._params, lr=learning_rate)
        self.transition = RolloutStorage.Transition()
        # fused rollout-storage writes on the device (hg_rollout_act / hg_rollout_env); the
        # action noise is Philox keyed by this seed (drawn from torch's generator) and a counter
        self.use_fused_rollout = True
        # global id of storage row 0 (data parallel: the runner sets the env shard's offset), so the
        # action noise of a sharded run is the single run's
        self.row_offset = 0
        # the minibatch loss and its gradient on the fused HIP kernels (hg_loss.py); the symmetry
        # loss configuration keeps the op-by-op expression
        self.use_fused_loss = True
        self.defer_values = True
        self._rollout_seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self._on_device else 0
        self._rollout_counter = 0
        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.base_lin_vel_coef = base_lin_vel_coef
        self.sym_loss = sym_loss
        self.sym_coef = sym_coef
        if self.sym_loss:
            # mirror matrices built on the policy's device (the reference hard-codes .cuda(), ppo.py:96,103)
            n_act = len(act_permutation)
            self.act_perm_mat = torch.zeros(n_act, n_act, device=device)
            for i, perm in enumerate(act_permutation):
                self.act_perm_mat[int(abs(perm))][i] = float(torch.sign(torch.tensor(perm)))
            stack = []
            for i in range(frame_stack):
                for p in obs_permutation:
                    s = 1.0 if p >= 0 else -1.0
                    stack.append(s * (abs(p) + i * len(obs_permutation)))
            self.obs_perm_mat = torch.zeros(len(stack), len(stack), device=device)
            for i, perm in enumerate(stack):
                self.obs_perm_mat[int(abs(perm))][i] = 1.0 if perm >= 0 else -1.0

    @property
    def learning_rate(self):
        """Current learning rate as a Python float (reads the device scalar: logging only)."""
        if self._lr_t is not None:
            return float(self._lr_t.item())
        return self._lr

    @learning_rate.setter
    def learning_rate(self, value):
        self._lr = float(value)
        if getattr(self, "_lr_t", None) is not None:
            self._lr_t.fill_(self._lr)
            self._lr_f32.fill_(self._lr)
        elif hasattr(self, "optimizer"):
            for g in self.optimizer.param_groups:
                g["lr"] = self._lr

    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape, action_shape,
                     obs_dtype=torch.float32, obs_frames=None):
        """obs_frames = (frame_stack, frame width) of a frame-stacking env: frame-only actor
        observation storage (rollout_storage.py module docstring) on the device path."""
        if not self._on_device or critic_obs_shape[0] is None:
            obs_frames = None
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                                      action_shape, self.device, obs_dtype=obs_dtype, obs_frames=obs_frames)

    def test_mode(self):
        self.actor_critic.eval()

    def train_mode(self):
        self.actor_critic.train()

    def _fused_rollout_ok(self, obs, critic_obs):
        st = self.storage
        return (self._on_device and self.use_fused_rollout and st is not None and hasattr(self.actor_critic, "_mlp")
                and obs.is_cuda and obs.dtype == torch.float32 and obs.dim() == 2 and obs.stride(1) == 1
                and critic_obs.dtype == torch.float32 and critic_obs.dim() == 2 and critic_obs.stride(1) == 1
                and st.step < st.num_transitions_per_env)

    def _act_fused(self, obs, critic_obs):
        """PPO.act + the pre-step half of add_transitions in one HIP launch (hg_rollout_act):
        the policy MLPs run in torch, the sample / log-prob / storage writes in the kernel."""
        from humanoid import _native as N
        st, ac, tr = self.storage, self.actor_critic, self.transition
        t = st.step
        # the actor's output layer runs inside the sampling launch when it is the 12 x 128 head
        # (hg_rollout_act_head: bitwise the separate output-layer launch); the mean lands in mu
        mean = head = tail = None
        last = ac.actor[-1]
        if (HEAD_FUSED and ac.policy_dtype == "fp32" and ac.fused_mlp and not torch.is_grad_enabled()
                and isinstance(last, torch.nn.Linear) and tuple(last.weight.shape) == (12, 128)
                and last.bias is not None and last.bias.is_contiguous() and hg_mlp.fusable(ac.actor)):
            # the last hidden layer too when its route allows (hg_rollout_act_tail), else the head only
            if last.weight.is_contiguous() and last.weight.data_ptr() % 16 == 0:
                tail = hg_mlp.mlp_infer_tail(ac.actor, obs)
            if tail is not None:
                head = tail
            else:
                h = hg_mlp.mlp_infer_hidden(ac.actor, obs)
                if hg_mlp.head_fusable(h, last.weight):
                    head = (h, last.weight, last.bias)
                else:
                    mean = last(h).contiguous()
        else:
            mean = ac._mlp(ac.actor, obs).contiguous()
        defer = self._defer_values()
        value = None if defer else ac._mlp(ac.critic, critic_obs).contiguous()
        std = ac.std.detach().contiguous()
        p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        priv = st.privileged_observations
        sl = _slot_views(st, t)
        if head is not None:
            mean = sl["mu"]  # written by the launch below
        ac.distribution = _DiagGaussian(mean, std.expand_as(mean))
        s = ctypes.c_void_p(torch.cuda.current_stream(obs.device).cuda_stream)
        if st.obs_frames is not None:
            # frame-only storage: the newest frame of the stack per slot, slot 0's whole stack
            if t == 0:
                st.obs_init.copy_(obs)
            w, c0 = st.frame_width, obs.shape[1] - st.frame_width
        else:
            w, c0 = obs.shape[1], 0
        if tail is not None:
            x3, W3, b3 = tail
            W, b = last.weight, last.bias
            fn = N.lib().hg_rollout_act_tail
            lead = (p(x3), ctypes.c_int64(x3.stride(0)), p(W3), p(b3), W3.shape[1], p(W), p(b), p(std))
        elif head is not None:
            h, W, b = head
            fn = N.lib().hg_rollout_act_head
            lead = (p(h), ctypes.c_int64(h.stride(0)), p(W), p(b), W.shape[1], p(std))
        else:
            fn = N.lib().hg_rollout_act
            lead = (p(mean), p(std))
        N.check(fn(
            *lead, p(value) if value is not None else None, p(obs),
            p(critic_obs) if priv is not None else None, obs.shape[0],
            mean.shape[1], ctypes.c_int64(w), ctypes.c_int64(critic_obs.shape[1] if priv is not None else 0),
            ctypes.c_int64(obs.stride(0)), ctypes.c_int64(c0), ctypes.c_int64(critic_obs.stride(0)),
            sl["p_actions"], sl["p_logp"], sl["p_mu"], sl["p_sigma"], sl["p_values"] if value is not None else None,
            sl["p_obs"], ctypes.c_int64(st.obs_frames.stride(0) if st.obs_frames is not None else 0), sl["p_priv"], int(st.obs_dtype == torch.float16), int(self.row_offset),
            ctypes.c_uint64(self._rollout_seed), ctypes.c_uint64(self._rollout_counter), s))
        self._rollout_counter += 1
        st.writes += 1
        tr.actions = sl["actions"]
        tr.values = sl["values"]
        tr.actions_log_prob = sl["logp"]
        tr.action_mean = sl["mu"]
        tr.action_sigma = sl["sigma"]
        tr.observations = obs
        tr.critic_observations = critic_obs
        tr.fused_slot = t
        return tr.actions

    def act(self, obs, critic_obs):
        if self._fused_rollout_ok(obs, critic_obs):
            return self._act_fused(obs, critic_obs)
        t = self.transition
        # actor_critic.act() would also run the lin-vel MLP, whose output the rollout discards
        self.actor_critic.update_distribution(obs)
        t.actions = self.actor_critic.distribution.sample().detach()
        t.values = self.actor_critic.evaluate(critic_obs).detach()
        t.actions_log_prob = self.actor_critic.get_actions_log_prob(t.actions).detach()
        t.action_mean = self.actor_critic.action_mean.detach()
        t.action_sigma = self.actor_critic.action_std.detach()
        # the reference keeps the obs tensors and copies them into the storage after env.step
        # (ppo.py:123-125, rollout_storage.py:90-91), relying on the env allocating new ones per
        # step — as hg_sim does by default (stable_observations); its live window views (the
        # runner's mode, tagged hg_live_view) are rewritten in place by the next step (a reset
        # zeroes the older frames), so those are copied here, before the step
        t.observations = obs.clone() if getattr(obs, "hg_live_view", False) else obs
        t.critic_observations = (critic_obs.clone() if getattr(critic_obs, "hg_live_view", False)
                                 else critic_obs)
        return t.actions

    def rollout_sink(self):
        """(rewards, dones, time_outs) views of the rollout storage slot the current transition
        fills, for an env that writes them inside its step (set_rollout_sink: the post launch fills
        the slot, process_env_step then launches nothing); None unless the fused device rollout
        with the deferred value pass is active."""
        t = self.transition
        st = self.storage
        if not (ROLLOUT_SINK and getattr(t, "fused_slot", None) is not None and self._defer_values()):
            return None
        if st.time_outs is None:
            st.time_outs = torch.zeros_like(st.dones)
        k = t.fused_slot
        return st.rewards[k].view(-1), st.dones[k].view(-1), st.time_outs[k].view(-1)

    def process_env_step(self, rewards, dones, infos):
        t = self.transition
        if getattr(t, "fused_slot", None) is not None:
            # post-step half of add_transitions (hg_rollout_env): time-out bootstrap, dones
            from humanoid import _native as N
            st, k = self.storage, t.fused_slot
            if st.step != k:
                raise AssertionError("rollout storage slot mismatch")
            p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
            to = infos.get("time_outs")
            r = rewards.contiguous().float()
            d, to = _as_u8(dones), (_as_u8(to) if to is not None else None)
            s = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
            sl = _slot_views(st, k)
            if self._defer_values():
                # time-out bootstrap deferred to the batched value pass in compute_returns
                if st.time_outs is None:
                    st.time_outs = torch.zeros_like(st.dones)
                sink = infos.get("rollout_sink")
                written = (sink is not None and sink[0].data_ptr() == sl["rewards"].data_ptr()
                           and sink[2] is not None and sink[2].data_ptr() == st.time_outs[k].data_ptr())
                if not written:  # else the env's post launch already filled this slot
                    if "p_time_outs" not in sl:
                        sl["p_time_outs"] = ctypes.c_void_p(st.time_outs[k].data_ptr())
                    N.check(N.lib().hg_rollout_env(p(r), p(d), p(to) if to is not None else None, None, r.shape[0],
                                                   ctypes.c_float(self.gamma), sl["p_rewards"], sl["p_dones"],
                                                   sl["p_time_outs"], s))
                st.values_deferred = True
            else:
                N.check(N.lib().hg_rollout_env(p(r), p(d), p(to) if to is not None else None, sl["p_values"],
                                               r.shape[0], ctypes.c_float(self.gamma), sl["p_rewards"],
                                               sl["p_dones"], None, s))
            st.step += 1
            self.transition.clear()
            self.actor_critic.reset(dones)
            return
        t.rewards = rewards.clone()
        t.dones = dones
        if "time_outs" in infos:  # bootstrap on time-outs (ppo.py:132-133)
            t.rewards += self.gamma * torch.squeeze(t.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(t)
        self.transition.clear()
        self.actor_critic.reset(dones)

    def _defer_values(self):
        """Values V(s_t) of the whole rollout in one batched critic pass at compute_returns
        instead of T per-step passes (the critic does not change during collection); only with
        fp32 observation storage, so the critic sees exactly the observations the step saw."""
        st = self.storage
        return (self.defer_values and self._on_device and st is not None and st.privileged_observations is not None
                and st.privileged_observations.dtype == torch.float32)

    def _finish_deferred_values(self):
        st, ac = self.storage, self.actor_critic
        T, n = st.num_transitions_per_env, st.num_envs
        x = st.privileged_observations.flatten(0, 1)
        if ac.policy_dtype == "fp32" and ac.fused_mlp and hg_mlp.fusable(ac.critic):
            hg_mlp.mlp_infer(ac.critic, x if x.dtype == torch.float32 else x.float(), out=st.values)
            # time-out bootstrap, as process_env_step (ppo.py:132-133): r += gamma * V * time_out,
            # in place over the whole [T, N] rollout in one launch (hg_rollout_env)
            from humanoid import _native as N
            p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
            N.check(N.lib().hg_rollout_env(p(st.rewards), p(st.dones), p(st.time_outs), p(st.values), T * n,
                                           ctypes.c_float(self.gamma), p(st.rewards), p(st.dones), None, s))
        else:
            v = ac._mlp(ac.critic, x).view(T, n, 1)
            st.values.copy_(v)
            st.rewards.add_(self.gamma * (st.values * st.time_outs))
        st.values_deferred = False

    def compute_returns(self, last_critic_obs):
        if getattr(self.storage, "values_deferred", False):
            self._finish_deferred_values()
        last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam)

    def _kl_mean(self, mu, sigma, old_mu, old_sigma, out=None):
        if self._on_device:
            # one HIP launch (csrc/hg_optim.hip k_kl_mean) instead of ~13 elementwise kernels
            from humanoid import _native as N
            out = torch.empty((), dtype=torch.float32, device=mu.device) if out is None else out
            t = [x.detach().contiguous() for x in (mu, sigma, old_mu, old_sigma)]
            rows, A = t[0].shape[0], t[0].shape[-1]
            nb = (rows + 255) // 256
            if getattr(self, "_kl_scratch", None) is None or self._kl_scratch.numel() < nb:
                self._kl_scratch = torch.empty(nb, dtype=torch.float64, device=mu.device)
            s = ctypes.c_void_p(torch.cuda.current_stream(mu.device).cuda_stream)
            N.check(N.lib().hg_kl_mean(*[ctypes.c_void_p(x.data_ptr()) for x in t], ctypes.c_int64(rows), A,
                                       ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(self._kl_scratch.data_ptr()), s))
            return out
        with torch.inference_mode():
            kl = torch.sum(torch.log(sigma / old_sigma + 1.0e-5)
                           + (torch.square(old_sigma) + torch.square(old_mu - mu)) / (2.0 * torch.square(sigma))
                           - 0.5, axis=-1)
            return torch.mean(kl)

    def _lr_rule_device(self, kl_mean):
        """The reference's adaptive rule (ppo.py:168-176) in float64 on the device (kl promoted
        exactly as Python promotes kl_mean.item())."""
        from humanoid import _native as N
        s = ctypes.c_void_p(torch.cuda.current_stream(self._lr_t.device).cuda_stream)
        N.check(N.lib().hg_kl_lr_rule(ctypes.c_void_p(kl_mean.data_ptr()), ctypes.c_void_p(self._lr_t.data_ptr()),
                                      ctypes.c_void_p(self._lr_f32.data_ptr()), float(self.desired_kl), 1e-5, 1e-2, s))

    def _adapt_lr(self, mu, sigma, old_mu, old_sigma):
        self._adapt_lr_from_kl(self._kl_mean(mu, sigma, old_mu, old_sigma))

    def _adapt_lr_from_kl(self, kl_mean):
        if self._dp:
            with torch.inference_mode():
                dist.all_reduce(kl_mean)
                kl_mean /= self.world_size
        if self._lr_t is not None:
            self._lr_rule_device(kl_mean)
            return
        kl_mean = kl_mean.item()
        if kl_mean > self.desired_kl * 2.0:
            self._lr = max(1e-5, self._lr / 1.5)
        elif kl_mean < self.desired_kl / 2.0 and kl_mean > 0.0:
            self._lr = min(1e-2, self._lr * 1.5)
        for g in self.optimizer.param_groups:
            g["lr"] = self._lr

    @property
    def _adaptive(self):
        return self.desired_kl is not None and self.schedule == "adaptive"

    @property
    def _fused_loss(self):
        return self._on_device and self.use_fused_loss and not self.sym_loss

    def _losses_fused(self, obs_b, critic_b, lin_vel_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b,
                      old_mu_b, old_sigma_b, stats_out=None, lr_rule=None):
        """The loss of _losses (and the adaptive schedule's KL mean) from the three network
        outputs in one fused HIP forward launch pair and one backward launch (hg_loss.py).
        Returns (loss, stats) with stats = [value_loss, surrogate_loss, lin_vel_loss, kl_mean]."""
        ac = self.actor_critic
        own = ac.policy_dtype == "fp32" and ac.fused_mlp and obs_b.is_cuda
        # the actor and the lin-vel estimator read the same observations: their first layers as one
        # stacked GEMM (hg_mlp.mlp_pair_forward) where it is routed
        pair = (own and obs_b.dtype == torch.float32 and obs_b.dim() == 2 and obs_b.stride(1) == 1
                and hg_mlp.pair_ok(ac.actor, ac.base_lin_vel, obs_b.shape[0]))
        scope = (hg_mlp.image_scope([(ac.actor, obs_b.shape[0]), (ac.base_lin_vel, obs_b.shape[0]),
                                     (ac.critic, critic_b.shape[0])], obs_b.device,
                                    pairs=[(ac.actor, ac.base_lin_vel, obs_b.shape[0])] if pair else ())
                 if own else contextlib.nullcontext())
        with scope:  # the three networks' weight images in one launch
            if pair:
                mu, est_lin_vel = hg_mlp.mlp_pair_forward(ac.actor, ac.base_lin_vel, obs_b)
            else:
                mu = ac._mlp(ac.actor, obs_b)
                est_lin_vel = ac.base_get_lin_vel(obs_b)
            ac.distribution = _DiagGaussian(mu, ac.std.expand_as(mu))
            value_b = ac.evaluate(critic_b)
        data = {"actions": actions_b, "old_logp": old_logp_b, "advantages": adv_b, "target_values": target_values_b,
                "returns": returns_b, "old_mu": old_mu_b, "old_sigma": old_sigma_b,
                "lin_vel_target": lin_vel_b if lin_vel_b.dtype == torch.float32 else lin_vel_b.float()}
        return ppo_loss(mu, ac.std, value_b, est_lin_vel, data, self.clip_param, self.value_loss_coef,
                        self.entropy_coef, self.base_lin_vel_coef, self.use_clipped_value_loss,
                        stats_out=stats_out, accumulate=stats_out is not None, lr_rule=lr_rule)

    def _losses(self, obs_b, critic_b, lin_vel_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b):
        """Minibatch loss (ppo.py:155-214).  The reference calls actor_critic.act() here and
        discards the sampled action; only the distribution and the lin-vel estimate are used, so
        the sample is not drawn."""
        ac = self.actor_critic
        ac.update_distribution(obs_b)
        est_lin_vel = ac.base_get_lin_vel(obs_b)
        logp_b = ac.get_actions_log_prob(actions_b)
        value_b = ac.evaluate(critic_b)
        mu_b = ac.action_mean
        entropy_b = ac.entropy
        # clipped surrogate
        ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
        adv = torch.squeeze(adv_b)
        surrogate = -adv * ratio
        surrogate_clipped = -adv * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        # value loss
        if self.use_clipped_value_loss:
            value_clipped = target_values_b + (value_b - target_values_b).clamp(-self.clip_param, self.clip_param)
            value_losses = (value_b - returns_b).pow(2)
            value_losses_clipped = (value_clipped - returns_b).pow(2)
            value_loss = torch.max(value_losses, value_losses_clipped).mean()
        else:
            value_loss = (returns_b - value_b).pow(2).mean()
        sym_loss = 0
        if self.sym_loss:
            mirror_act = ac.actor(torch.matmul(obs_b, self.obs_perm_mat))
            sym_loss = (mu_b - torch.matmul(mirror_act, self.act_perm_mat)).pow(2).mean()
        base_lin_vel_loss = F.mse_loss(est_lin_vel, lin_vel_b.float())
        loss = (surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_b.mean()
                + self.sym_coef * sym_loss + self.base_lin_vel_coef * base_lin_vel_loss)
        return loss, value_loss, surrogate_loss, base_lin_vel_loss, sym_loss

    def _clip_and_step(self):
        """clip_grad_norm_(params, max_grad_norm); optimizer.step() (ppo.py:212-214) — one fused
        HIP launch pair on the device."""
        if isinstance(self.optimizer, HgAdam):
            self.optimizer.step(max_norm=self.max_grad_norm)
        else:
            nn.utils.clip_grad_norm_(self._params, self.max_grad_norm)
            self.optimizer.step()

    def update(self, sync=True):
        """ppo.py:140-226.  Returns the mean value / surrogate / sym / lin-vel losses as floats; with
        sync=False (device path) the means stay on the device (0-d tensors; no host wait)."""
        if self._on_device and self.use_graphs:
            return self._update_graphed(sync)
        out = self._update_eager()
        return out

    def _update_eager(self):
        mean_value_loss = 0.0
        mean_surrogate_loss = 0.0
        mean_base_lin_vel_loss = 0.0
        sym_loss = 0
        sums = None
        ac = self.actor_critic
        gen = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        for (obs_b, critic_b, lin_vel_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
             old_sigma_b, hid_b, masks_b) in gen:
            if self._fused_loss:
                loss, stats = self._losses_fused(obs_b, critic_b, lin_vel_b, actions_b, target_values_b, adv_b,
                                                 returns_b, old_logp_b, old_mu_b, old_sigma_b)
                value_loss, surrogate_loss, base_lin_vel_loss = stats[0], stats[1], stats[2]
                if self._adaptive:
                    self._adapt_lr_from_kl(stats[3].clone())
            else:
                loss, value_loss, surrogate_loss, base_lin_vel_loss, sym_loss = self._losses(
                    obs_b, critic_b, lin_vel_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b)
                if self._adaptive:
                    self._adapt_lr(ac.action_mean, ac.action_std, old_mu_b, old_sigma_b)
            if self._flat_grad is not None:
                self._flat_grad.zero_()
                loss.backward()
                if self._dp:
                    self._timed_all_reduce(self._flat_grad)
                    self._flat_grad /= self.world_size
            else:
                self.optimizer.zero_grad()
                loss.backward()
            self._clip_and_step()
            if self._on_device:
                acc = torch.stack([value_loss.detach(), surrogate_loss.detach(), base_lin_vel_loss.detach()])
                sums = acc if sums is None else sums + acc
            else:
                mean_value_loss += value_loss.item()
                mean_surrogate_loss += surrogate_loss.item()
                mean_base_lin_vel_loss += base_lin_vel_loss.item()
        num_updates = self.num_learning_epochs * self.num_mini_batches
        if sums is not None:
            mean_value_loss, mean_surrogate_loss, mean_base_lin_vel_loss = sums.tolist()  # one host read
        mean_value_loss /= num_updates
        mean_surrogate_loss /= num_updates
        mean_base_lin_vel_loss /= num_updates
        self.storage.clear()
        # release the last minibatch's autograd graph (ac.distribution holds its mean): a graph kept
        # alive pins each parameter's AccumulateGrad node to the stream it was created on, and the
        # captured update (another stream) would then accumulate across streams
        self.actor_critic.distribution = None
        return mean_value_loss, mean_surrogate_loss, sym_loss, mean_base_lin_vel_loss

    # ------------------------------------------------------------------------------------------
    # HIP-graph update: the minibatch step is captured once as two graphs and replayed
    #   A: gather the minibatch rows (static index buffer) -> losses -> backward into the flat
    #      gradient buffer; KL mean; loss sums
    #   (data parallel: all-reduce of the flat gradients and of the KL mean — eager between the two
    #   graphs' replays by default; captured in the one update graph with HG_DP_GRAPH_COLLECTIVE=1)
    #   B: adaptive learning rate, global-norm clip, fused Adam
    # The first update() runs eagerly on a side stream (the warm-up graph capture needs); the
    # graphs are captured at the start of the second one.  Minibatch order: one randperm per
    # update, as the reference's generator (rollout_storage.py:153-191).
    # ------------------------------------------------------------------------------------------
    def _storage_key(self):
        st = self.storage
        return (st.obs_key(), st.num_envs, st.num_transitions_per_env,
                getattr(self.optimizer, "version", 0))

    def _capture(self, mb):
        st = self.storage
        dev = st.rewards.device
        frames = st.obs_frames is not None  # frame-only storage: the obs rows come from hg_gather_stacked
        obs = None if frames else st.observations.flatten(0, 1)
        critic = (st.privileged_observations.flatten(0, 1) if st.privileged_observations is not None else obs)
        # the per-sample scalars/12-vectors are packed once per update into one [T*N, 40] table so a
        # minibatch needs three gathers (obs, critic obs, table) instead of ten
        A = st.actions.shape[-1]
        self._pack_src = [st.actions, st.values, st.returns, st.actions_log_prob, st.advantages, st.mu, st.sigma]
        # bf16 policy on the fused path: the obs / critic minibatch rows are converted to bf16 by the
        # gather (the networks' input dtype), and the lin-vel target — privileged obs [53:56],
        # rollout_storage.py / ppo.py:160 — travels in the fp32 table so it keeps the storage's bits
        ac = self.actor_critic
        mb_dtype = (torch.bfloat16 if getattr(ac, "policy_dtype", "fp32") == "bf16" and ac.fused_mlp
                    and self._fused_loss else None)
        self._lin_vel_packed = mb_dtype is not None
        if self._lin_vel_packed:
            self._pack_src.append(critic.view(st.num_transitions_per_env, st.num_envs, -1)[..., 53:56])
        widths = [t.shape[-1] for t in self._pack_src]
        self._packed = torch.empty(st.num_transitions_per_env * st.num_envs, sum(widths), dtype=torch.float32,
                                   device=dev)
        self._idx = torch.zeros(mb, dtype=torch.int64, device=dev)
        if getattr(self, "_one_grad", None) is not None:
            hg_loss.release_unit_seed(self._one_grad)  # the graphs that read it are replaced below
        self._one_grad = hg_loss.register_unit_seed(torch.ones((), dtype=torch.float32, device=dev))
        # [value, surrogate, lin-vel loss sums, KL mean of the current minibatch]: the fused loss
        # accumulates into it directly
        self._stats4 = torch.zeros(4, dtype=torch.float32, device=dev)
        self._sums = self._stats4[:3]
        self._kl = self._stats4[3:]
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        if self._flat_grad is None:
            self.optimizer.zero_grad(set_to_none=True)  # backward allocates the grads in the graph pool
        self._whole = (not self._dp and self._flat_grad is None) or self._collective_in_graph()
        # minibatch rows land in static buffers: the three row gathers are one HIP launch.  The
        # reference draws ONE permutation per update and walks the same minibatches in every epoch
        # (rollout_storage.py:153-177), so the one-graph form keeps one buffer set per minibatch and
        # gathers only in the first epoch (380 MB at the bench's size); the two-graph form re-gathers
        reuse = self._whole and self.num_learning_epochs > 1 and os.environ.get("HG_MB_REUSE", "1") != "0"
        nsets = self.num_mini_batches if reuse else 1
        self._mb_sets = []
        for _ in range(nsets):
            m_obs = torch.empty(mb, st.obs_shape[0], dtype=mb_dtype or st.obs_dtype, device=dev)
            m_critic = (torch.empty(mb, critic.shape[1], dtype=mb_dtype or critic.dtype, device=dev)
                        if critic is not obs else m_obs)
            m_packed = torch.empty(mb, self._packed.shape[1], dtype=torch.float32, device=dev)
            tables = [(self._packed, m_packed)]
            if not frames:
                tables.insert(0, (obs, m_obs))
            if critic is not obs:
                tables.insert(1 if not frames else 0, (critic, m_critic))
            self._mb_sets.append((m_obs, m_critic, m_packed, tables))
        self._mb_widths = widths
        # the whole update (epochs x minibatches, each with its LR rule and Adam step) is ONE graph
        # reading its row indices from a static permutation buffer at world size 1.  Data parallel,
        # the default is two graphs per minibatch with the eager gradient all-reduce between their
        # replays (RCCL or gloo; timed by comm_timer).  On request (HG_DP_GRAPH_COLLECTIVE=1, RCCL
        # only) the all-reduce is captured inside the one graph between each backward and its step;
        # a rank whose capture fails pulls every rank back to the two-graph form in this process.
        if self._whole:
            nmb = self.num_mini_batches
            self._perm = torch.zeros(nmb * mb, dtype=torch.int64, device=dev)
            g = torch.cuda.CUDAGraph()
            ok = True
            try:
                # thread_local: the process group's watchdog thread may query its events meanwhile
                with _capturing(g, "thread_local" if self._dp else "global"):
                    for ep in range(self.num_learning_epochs):
                        for i in range(nmb):
                            if self._flat_grad is None:
                                self.optimizer.zero_grad(set_to_none=True)  # fresh gradients from each backward
                            k = i if len(self._mb_sets) > 1 else 0
                            # zeroes the flat buffer (dp); gathers minibatch i's rows in the first epoch only
                            self._mb_backward(self._perm[i * mb:(i + 1) * mb], k, ep == 0 or len(self._mb_sets) == 1)
                            if self._dp:
                                dist.all_reduce(self._flat_grad)  # gradients + the KL slot, in the graph
                            self._mb_step()
            except Exception as e:  # noqa: BLE001 — the collective's capture is the known risk
                if not self._dp:
                    raise
                ok = False
                self.capture_error = f"{type(e).__name__}: {e}"
            if self._dp:
                # every rank takes the same form: a rank whose capture failed pulls all to two graphs
                flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                ok = bool(flag.item())
            if ok:
                self._graphs = (g, None, mb, self._storage_key())
                self.update_graph = "one"
                return
            # fall back in this process (never a re-exec): the two-graph form, all-reduce between
            del g
            torch.cuda.synchronize(dev)
            self._whole = False
            if self.capture_error is None:
                self.capture_error = "another rank's capture failed"
            warnings.warn(f"PPO: the in-graph all-reduce could not be captured ({self.capture_error}); "
                          "using two graphs per minibatch with the all-reduce between them")
        with _capturing(ga, "global"):
            self._mb_backward(self._idx)
        with _capturing(gb, "global", pool=ga.pool()):
            self._mb_step()
        self._graphs = (ga, gb, mb, self._storage_key())
        self.update_graph = "two"

    def _timed_all_reduce(self, t):
        """The eager per-minibatch all-reduce, bracketed by comm_timer when one is attached (the
        in-graph form of the one-graph update cannot be bracketed: its time is inside the replay)."""
        tm = self.comm_timer
        if tm is not None:
            tm.start("allreduce")
        dist.all_reduce(t)
        if tm is not None:
            tm.stop("allreduce")

    def _collective_in_graph(self):
        """Whether the per-minibatch gradient all-reduce is captured inside the one update graph.
        Only on RCCL ("nccl" backend; gloo collectives cannot be captured) and only on request
        (HG_DP_GRAPH_COLLECTIVE=1): the in-graph collective is verified at world size 1 only, so
        the default data-parallel form is the two-graph one with the eager all-reduce between the
        replays.  A failed capture falls back to that form on every rank (`update_graph`)."""
        return (self._dp and dist.is_initialized() and dist.get_backend() == "nccl"
                and os.environ.get("HG_DP_GRAPH_COLLECTIVE", "0") == "1")

    def collectives_per_update(self):
        """Collectives one update() issues: per minibatch the flat-gradient (+ KL slot) all-reduce,
        plus the advantage-statistics all-reduce of compute_returns; 0 on one process."""
        if not self._dp:
            return 0
        return self.num_learning_epochs * self.num_mini_batches + 1

    def _mb_backward(self, idx, k=0, gather=True):
        """Captured minibatch body: gather rows (into buffer set k; ``gather`` False: the set
        already holds these rows) -> losses -> backward (+ KL mean, loss sums)."""
        if self._flat_grad is not None:
            self._flat_grad.zero_()
        m_obs, m_critic, m_packed, tables = self._mb_sets[k]
        if gather:
            if self.storage.obs_frames is not None:
                # frame-only storage: the stacked obs rows and the plain tables in one launch
                self.storage.gather_stacked(idx, m_obs, tables, use_prepared=True)
            else:
                gather_rows(idx, tables)
        crit_b = m_critic
        b = {"obs": m_obs, "critic": crit_b, "lin_vel": crit_b[:, 53:56]}
        pk = m_packed
        for name, part in zip(("actions", "values", "returns", "logp", "adv", "mu", "sigma", "lin_vel"),
                              pk.split(self._mb_widths, dim=1)):
            b[name] = part
        if self._fused_loss:
            loss = self._losses_fused(b["obs"], b["critic"], b["lin_vel"], b["actions"], b["values"],
                                      b["adv"], b["returns"], b["logp"], b["mu"], b["sigma"],
                                      stats_out=self._stats4, lr_rule=self._fused_lr_rule())
        else:
            loss, value_loss, surrogate_loss, lin_vel_loss, _ = self._losses(
                b["obs"], b["critic"], b["lin_vel"], b["actions"], b["values"], b["adv"], b["returns"],
                b["logp"])
            if self._adaptive:
                ac = self.actor_critic
                self._kl_mean(ac.action_mean, ac.action_std, b["mu"], b["sigma"], out=self._kl)
            self._sums.add_(torch.stack([value_loss.detach(), surrogate_loss.detach(), lin_vel_loss.detach()]))
        if self._dp and self._adaptive:
            self._kl_slot.copy_(self._kl)
        # d loss / d loss = 1 from a persistent tensor: no fill launch per minibatch in the graph
        loss.backward(gradient=self._one_grad)

    def _fused_lr_rule(self):
        """The adaptive rule's device state for hg_ppo_loss_lr (the rule inside the loss launch):
        one process with the device learning rate; None otherwise (data parallel: the rule needs
        the all-reduced KL mean, _mb_step applies it)."""
        if FUSED_LR_RULE and self._adaptive and not self._dp and self._lr_t is not None and self._fused_loss:
            return (self._lr_t, self._lr_f32, self.desired_kl, 1e-5, 1e-2)
        return None

    def _mb_step(self):
        """Captured minibatch step: adaptive learning rate, global-norm clip, fused Adam."""
        kl = self._kl
        if self._dp:
            # gradients and the KL mean were summed over ranks in ONE all-reduce
            self._flat_grad.div_(self.world_size)
            kl = self._kl_slot
        if self._adaptive and self._fused_lr_rule() is None:  # else applied by the loss launch
            self._lr_rule_device(kl)
        self._clip_and_step()

    def _update_graphed(self, sync=True):
        st = self.storage
        nmb = self.num_mini_batches
        batch = st.num_envs * st.num_transitions_per_env
        mb = batch // nmb
        if self.sym_loss or (self._graphs is None and not self._graph_warm):
            # warm-up (and the symmetry-loss configuration, which stays eager)
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                out = self._update_eager()
            cur.wait_stream(side)
            self._graph_warm = True
            return out
        st.prepare_gather()  # before a capture: the captured gathers read its persistent buffer
        if self._graphs is None or self._graphs[2] != mb or self._graphs[3] != self._storage_key():
            self._capture(mb)
        ga, gb = self._graphs[0], self._graphs[1]
        dev = st.rewards.device
        torch.cat([t.flatten(0, 1) for t in self._pack_src], dim=1, out=self._packed)
        self._sums.zero_()
        if gb is None:  # the whole update as one graph
            torch.randperm(nmb * mb, out=self._perm, device=dev)
            ga.replay()
        else:
            indices = torch.randperm(nmb * mb, requires_grad=False, device=dev)
            for _ in range(self.num_learning_epochs):
                for i in range(nmb):
                    self._idx.copy_(indices[i * mb:(i + 1) * mb])
                    ga.replay()
                    if self._dp:
                        self._timed_all_reduce(self._flat_grad)  # gradients + the KL slot
                    gb.replay()
        num_updates = self.num_learning_epochs * nmb
        means = self._sums / num_updates
        st.clear()
        if not sync:
            return means[0], means[1], 0, means[2]
        v, s, lv = means.tolist()  # the one host read of the update
        return v, s, 0, lv
