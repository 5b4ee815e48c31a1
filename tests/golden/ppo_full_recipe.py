"""Seeded input recipe of the production-size PPO.update golden (ppo_update_full.npz).

Shared by the generator (gen_goldens.py gen_ppo_update_full, which runs the REFERENCE's
PPO.update, /root/reference/humanoid/algo/ppo/ppo.py:144-226, on these inputs) and the GPU test
(tests/test_gpu_ppo_full.py, which runs the build's update on the same inputs), so only the
outputs — the four losses, the learning rate and the final parameters — are committed.

Sizes: the production networks (XBotLCfgPPO: ActorCritic 705 / 219 / 12, actor [512, 256, 128],
critic [768, 256, 128], lin-vel [128, 128]) and a 2048-env x 24-step rollout, so each of the 4
minibatches holds 12288 rows — above the 8192-row bounds of hg_mlp's routes: every bf16-split
forward / input-gradient tile, the weight images and the split-K weight gradients of the
production update run.  CONFIG1_ENVS: BASELINE config 1's rollout (4 envs x 24 steps, 24-row
minibatches; ppo_update_config1.npz), the smallest shapes every route handles.  numpy's Generator draws are platform independent and the recipe uses
no BLAS, so the generator and the GPU box build bit-identical inputs.
"""
import math

import numpy as np

N_ENVS, T = 2048, 24
CONFIG1_ENVS = 4
DIMS = dict(num_actor_obs=705, num_critic_obs=219, num_actions=12, actor_hidden_dims=[512, 256, 128],
            critic_hidden_dims=[768, 256, 128], base_lin_vel_hidden_dims=[128, 128], init_noise_std=1.0)
PPO_KW = dict(num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9, value_loss_coef=1.0,
              entropy_coef=0.001, learning_rate=1e-5, max_grad_norm=1.0, use_clipped_value_loss=True,
              schedule="adaptive", desired_kl=0.01)
PERM_SEED = 1234  # torch.manual_seed before update(): the minibatch permutation (rollout_storage.py:156)
STORAGE_KEYS = ("observations", "privileged_observations", "actions", "values", "actions_log_prob", "mu", "sigma",
                "returns", "advantages")


def parameters(shapes):
    """Initial parameters for an ordered [(state_dict key, shape)] list: nn.Linear's default range
    U(+-1/sqrt(fan_in)) for weights and biases, the actor's output layer scaled by 0.1 (its mean
    stays small, so the minibatch KL sits near 0.0025, well inside the adaptive rule's raise branch
    kl < desired_kl / 2 for every minibatch), std = linspace(0.8, 1.2)."""
    rng = np.random.default_rng(20241017)
    out = {}
    last_actor = max(k for k, _ in shapes if k.startswith("actor.") and k.endswith(".weight"))
    fan_in = {}
    for k, shp in shapes:
        if k == "std":
            out[k] = np.linspace(0.8, 1.2, shp[0]).astype(np.float32)
            continue
        layer = k.rsplit(".", 1)[0]
        if k.endswith(".weight"):
            fan_in[layer] = shp[1]
        bound = 1.0 / math.sqrt(fan_in[layer])
        x = rng.uniform(-bound, bound, size=shp).astype(np.float32)
        if layer == last_actor.rsplit(".", 1)[0]:
            x *= np.float32(0.1)
        out[k] = x
    return out


def storage(std, n_envs=None):
    """Rollout-storage contents [T, N, .] (float32) the update reads: observations, privileged
    observations (whose [53:56] columns are the lin-vel target), actions drawn around small old
    means with the policy's std, their Normal log-probabilities (+ - * / and the 12 logs of std
    only), values, returns and advantages."""
    N_ENVS = n_envs or globals()["N_ENVS"]  # noqa: N806  (config 1's golden: 4 envs)
    rng = np.random.default_rng(20241018)
    f32 = np.float32
    obs = rng.standard_normal((T, N_ENVS, DIMS["num_actor_obs"]), dtype=f32)
    priv = rng.standard_normal((T, N_ENVS, DIMS["num_critic_obs"]), dtype=f32)
    A = DIMS["num_actions"]
    sigma = np.broadcast_to(np.asarray(std, f32), (T, N_ENVS, A)).copy()
    mu = (0.02 * rng.standard_normal((T, N_ENVS, A))).astype(f32)
    z = rng.standard_normal((T, N_ENVS, A))
    actions = (mu.astype(np.float64) + sigma.astype(np.float64) * z).astype(f32)
    s64 = sigma.astype(np.float64)
    logs = np.array([math.log(float(s)) for s in np.asarray(std, np.float64)])
    d = (actions.astype(np.float64) - mu.astype(np.float64)) / s64
    logp = (-0.5 * (d * d) - logs - 0.5 * math.log(2.0 * math.pi)).sum(-1, keepdims=True).astype(f32)
    values = (0.5 * rng.standard_normal((T, N_ENVS, 1))).astype(f32)
    returns = (values.astype(np.float64) + 0.5 * rng.standard_normal((T, N_ENVS, 1))).astype(f32)
    adv = rng.standard_normal((T, N_ENVS, 1), dtype=f32)
    return dict(observations=obs, privileged_observations=priv, actions=actions, values=values,
                actions_log_prob=logp, mu=mu, sigma=sigma, returns=returns, advantages=adv)
