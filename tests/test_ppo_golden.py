"""ActorCritic and PPO.update against golden vectors from the reference algo/ppo (CPU)."""
import numpy as np
import torch

from humanoid.algo.ppo import ActorCritic, PPO

SMALL = dict(num_actor_obs=141, num_critic_obs=73, num_actions=12, actor_hidden_dims=[64, 32, 16],
             critic_hidden_dims=[48, 32, 16], base_lin_vel_hidden_dims=[24, 24], init_noise_std=1.0)


def sd(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


def test_actor_critic(golden):
    g = golden("actor_critic.npz")
    ac = ActorCritic(**SMALL)
    ac.load_state_dict(sd(g, "sd/"))
    obs, cobs, acts = (torch.from_numpy(g[k]) for k in ("obs", "critic_obs", "actions"))
    with torch.no_grad():
        np.testing.assert_allclose(ac.act_inference(obs).numpy(), g["mean"], rtol=1e-6, atol=1e-6)
        ac.update_distribution(obs)
        np.testing.assert_allclose(ac.get_actions_log_prob(acts).numpy(), g["log_prob"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(ac.entropy.numpy(), g["entropy"], rtol=1e-6)
        np.testing.assert_allclose(ac.action_std.numpy(), g["action_std"], rtol=1e-7)
        np.testing.assert_allclose(ac.evaluate(cobs).numpy(), g["value"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(ac.base_get_lin_vel(obs).numpy(), g["lin_vel"], rtol=1e-6, atol=1e-6)
    assert list(ac.state_dict().keys()) == [k[3:] for k in g.files if k.startswith("sd/")]


def test_ppo_update(golden):
    g = golden("ppo_update.npz")
    torch.manual_seed(0)
    ac = ActorCritic(**SMALL)
    ac.load_state_dict(sd(g, "init/"))
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9,
              value_loss_coef=1.0, entropy_coef=0.001, learning_rate=1e-5, max_grad_norm=1.0,
              use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01, device="cpu")
    ppo.init_storage(8, 24, [141], [73], [12])
    st = ppo.storage
    for k in ("observations", "privileged_observations", "actions", "rewards", "dones", "values", "actions_log_prob",
              "mu", "sigma", "returns", "advantages"):
        getattr(st, k).copy_(torch.from_numpy(g["st/" + k]))
    st.step = 24
    torch.manual_seed(1234)
    vloss, sloss, sym, lvloss = ppo.update()
    np.testing.assert_allclose(vloss, g["value_loss"], rtol=1e-5)
    np.testing.assert_allclose(sloss, g["surrogate_loss"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(lvloss, g["lin_vel_loss"], rtol=1e-5)
    np.testing.assert_allclose(ppo.learning_rate, g["learning_rate"], rtol=1e-12)
    assert sym == 0
    final = sd(g, "final/")
    for k, v in ac.state_dict().items():
        np.testing.assert_allclose(v.numpy(), final[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)


def test_storage_overflow():
    from humanoid.algo.ppo import RolloutStorage
    st = RolloutStorage(2, 1, [3], [4], [1])
    t = RolloutStorage.Transition()
    t.observations, t.critic_observations = torch.zeros(2, 3), torch.zeros(2, 4)
    t.actions, t.rewards, t.dones, t.values = torch.zeros(2, 1), torch.zeros(2), torch.zeros(2), torch.zeros(2, 1)
    t.actions_log_prob, t.action_mean, t.action_sigma = torch.zeros(2), torch.zeros(2, 1), torch.zeros(2, 1)
    st.add_transitions(t)
    import pytest
    with pytest.raises(AssertionError):
        st.add_transitions(t)


def test_gae_requires_hip_on_cpu():
    import pytest
    from humanoid.algo.ppo import RolloutStorage
    st = RolloutStorage(2, 3, [3], [4], [1])
    with pytest.raises(RuntimeError):
        st.compute_returns(torch.zeros(2, 1), 0.99, 0.95)


def test_ppo_update_full_dims_cpu(golden):
    """The production-size golden (ppo_update_full.npz) on the CPU path (the reference's
    arithmetic verbatim): the same comparison the GPU test applies (tests/test_gpu_ppo_full.py)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import ppo_full_recipe as R
    from test_gpu_ppo_full import _compare, _load_storage
    g = golden("ppo_update_full.npz")
    torch.manual_seed(0)
    ac = ActorCritic(**R.DIMS)
    init = R.parameters([(k, tuple(v.shape)) for k, v in ac.state_dict().items()])
    ac.load_state_dict({k: torch.from_numpy(v) for k, v in init.items()})
    ppo = PPO(ac, device="cpu", **R.PPO_KW)
    ppo.init_storage(R.N_ENVS, R.T, [705], [219], [12])
    _load_storage(ppo, R.storage(init["std"]))
    torch.manual_seed(R.PERM_SEED)
    losses = ppo.update()
    fails, _ = _compare(ac, losses, ppo.learning_rate, g, init)
    assert not fails, "; ".join(fails)
