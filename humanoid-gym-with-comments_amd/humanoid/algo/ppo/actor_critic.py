"""ActorCritic with the reference's constructor, module names and distribution semantics
(humanoid/algo/ppo/actor_critic.py:36-149): ``actor``, ``base_lin_vel`` and ``critic`` are
nn.Sequential MLPs (state_dict keys ``actor.0.weight`` ... ``std``), the policy is a diagonal
Gaussian N(actor(obs), std) with an unclamped learnable std.

The Gaussian is a tiny local class that evaluates exactly the formulas of
torch.distributions.Normal (same sampling call, log_prob and entropy expressions), without
the distribution object's per-call overhead on the rollout hot loop.
"""
import math

import torch
import torch.nn as nn

from . import hg_mlp

_LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
_ENTROPY_CONST = 0.5 + 0.5 * math.log(2 * math.pi)


class _DiagGaussian:
    __slots__ = ("loc", "scale")

    def __init__(self, loc, scale):
        self.loc, self.scale = loc, scale

    @property
    def mean(self):
        return self.loc

    @property
    def stddev(self):
        return self.scale

    def sample(self):
        # torch.normal(loc, scale) computes normal_(0, 1) * scale + loc after checking
        # scale >= 0 with a host round trip (two device syncs per call); this is the same
        # arithmetic on the same generator stream without the check
        with torch.no_grad():
            return torch.randn_like(self.loc).mul_(self.scale).add_(self.loc)

    def log_prob(self, value):
        var = self.scale ** 2
        return -((value - self.loc) ** 2) / (2 * var) - self.scale.log() - _LOG_SQRT_2PI

    def entropy(self):
        return _ENTROPY_CONST + torch.log(self.scale)


def _mlp(in_dim, hidden, out_dim, activation):
    layers, d = [], in_dim
    for h in hidden:
        layers += [nn.Linear(d, h), activation]
        d = h
    layers.append(nn.Linear(d, out_dim))
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=[256, 256, 256],
                 critic_hidden_dims=[256, 256, 256], base_lin_vel_hidden_dims=[128, 128], init_noise_std=1.0,
                 activation=nn.ELU(), policy_dtype="fp32", **kwargs):
        """policy_dtype "bf16" (config 5): the three MLPs run with bf16 activations and bf16
        matrix-core GEMMs on the GPU (fp32 accumulation, fp32 master weights, gradients and
        outputs; hg_mlp.mlp_forward_bf16); "fp32" is the reference."""
        if policy_dtype not in ("fp32", "bf16"):
            raise ValueError(f"policy_dtype must be 'fp32' or 'bf16', got {policy_dtype!r}")
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs)))
        super().__init__()
        self.actor = _mlp(num_actor_obs, actor_hidden_dims, num_actions, activation)
        self.base_lin_vel = _mlp(num_actor_obs, base_lin_vel_hidden_dims, 3, activation)
        self.critic = _mlp(num_critic_obs, critic_hidden_dims, 1, activation)
        print(f"Actor MLP: {self.actor}")
        print(f"Lin vel MLP: {self.base_lin_vel}")
        print(f"Critic MLP: {self.critic}")
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        self.policy_dtype = policy_dtype
        self.fused_mlp = True
        self._fusable = {}

    def _mlp(self, net, x):
        if self.policy_dtype == "bf16" and x.is_cuda:
            if self.fused_mlp:
                ok = self._fusable.get(("bf16", id(net)))
                if ok is None:
                    ok = self._fusable[("bf16", id(net))] = hg_mlp.fusable_bf16(net)
                if ok:
                    # bf16 activations / GEMMs with fp32 accumulation, fp32 master weights and
                    # outputs, fused bf16 backward (hg_mlp.py, csrc/hg_mlp.hip)
                    return (hg_mlp.mlp_forward_bf16(net, x) if torch.is_grad_enabled()
                            else hg_mlp.mlp_infer_bf16(net, x))
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return net(x).float()
        x = x if x.dtype == torch.float32 else x.float()
        if self.fused_mlp and x.is_cuda:
            ok = self._fusable.get(id(net))
            if ok is None:
                ok = self._fusable[id(net)] = hg_mlp.fusable(net)
            if ok:
                # training pass: activation backward + bias gradient fused per layer, skinny output
                # layer on its own kernels (hg_mlp.py); inference: the output layer's kernel only
                return hg_mlp.mlp_forward(net, x) if torch.is_grad_enabled() else hg_mlp.mlp_infer(net, x)
        return net(x)

    @staticmethod
    def init_weights(sequential, scales):
        [torch.nn.init.orthogonal_(m.weight, gain=scales[i])
         for i, m in enumerate(mod for mod in sequential if isinstance(mod, nn.Linear))]

    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def update_distribution(self, observations):
        mean = self._mlp(self.actor, observations)
        # the reference's `mean * 0.0 + self.std` materialises the same [B, A] values; the
        # broadcast view avoids two kernels per call (and their backward) with identical
        # values and gradients (d std = sum over the batch either way)
        self.distribution = _DiagGaussian(mean, self.std.expand_as(mean))

    def act(self, observations, **kwargs):
        self.update_distribution(observations)
        return self.distribution.sample(), self.base_get_lin_vel(observations)

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_inference(self, observations):
        return self._mlp(self.actor, observations)

    def evaluate(self, critic_observations, **kwargs):
        return self._mlp(self.critic, critic_observations)

    def base_get_lin_vel(self, observations):
        return self._mlp(self.base_lin_vel, observations)
