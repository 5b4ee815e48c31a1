"""Observation lifetime across env.step for the reference's PPO call pattern.

The reference stores the obs TENSORS in PPO.act and copies them into the rollout storage only
after env.step, in add_transitions (/root/reference/humanoid/algo/ppo/ppo.py:123-136,
rollout_storage.py:90-91): it relies on the env allocating a new obs_buf per step
(humanoid_env.py:880-887).  hg_sim's stacks are sliding-window views whose older frames a reset
zeroes in place, so (a) the non-fused PPO.act copies device observations before the step and (b)
the env hands out stable copies unless a runner whose PPO copies them turns that off.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

T = 8
RESET_AT = {2: slice(0, 8), 5: slice(8, 16), 6: slice(0, 4)}  # step -> envs forced to time out


def _env(n=64):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    torch.manual_seed(5)
    np.random.seed(5)
    cfg = XBotLCfg()
    cfg.env.num_envs = n
    cfg.seed = 5
    return XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)


@pytest.mark.parametrize("frames", [False, True])
def test_nonfused_ppo_stores_the_returned_stacks_across_resets(frames):
    """act -> step -> process_env_step (add_transitions) with PPO(use_fused_rollout=False) on the
    env's live window views (the runner's setting), resets forced at three steps: every stored
    [T, N, 705] / [T, N, 219] row equals, bit for bit, the stack the env returned for it."""
    from humanoid.algo.ppo import ActorCritic, PPO
    from humanoid.envs import XBotLCfgPPO
    from humanoid.utils.helpers import class_to_dict
    env = _env()
    env.stable_observations = False
    pol = class_to_dict(XBotLCfgPPO())["policy"]
    ac = ActorCritic(705, 219, 12, **pol)
    ppo = PPO(ac, device="cuda:0", gamma=0.994)
    ppo.use_fused_rollout = False
    ppo.init_storage(env.num_envs, T, [705], [219], [12], obs_frames=(15, 47) if frames else None)
    obs, cobs = env.get_observations(), env.get_privileged_observations()
    seen, resets = [], []
    with torch.inference_mode():
        for t in range(T):
            seen.append((obs.clone(), cobs.clone()))
            a = ppo.act(obs, cobs)
            if t in RESET_AT:
                env.episode_length_buf[RESET_AT[t]] = int(env.max_episode_length)
            obs, cobs, rew, dones, infos = env.step(a)
            resets.append(dones.clone())
            ppo.process_env_step(rew, dones, infos)
    torch.cuda.synchronize()
    for t in RESET_AT:
        assert resets[t][RESET_AT[t]].all(), f"forced resets at step {t} did not happen"
    st = ppo.storage
    stored_obs = st.observations  # frame-only storage: rebuilt from the frames + dones
    for t, (o, c) in enumerate(seen):
        assert torch.equal(stored_obs[t], o), f"actor observation row of slot {t} differs"
        assert torch.equal(st.privileged_observations[t], c), f"critic observation row of slot {t} differs"
    # the envs that reset at step t start slot t + 1 from a zeroed history (the hazard this guards)
    for t, ids in RESET_AT.items():
        if t + 1 < T:
            assert (seen[t + 1][0][ids, :14 * 47] == 0).all()


def test_default_env_returns_stable_copies():
    """Without a runner the env's step() / get_observations() return tensors a later step (with
    resets) leaves untouched, as the reference's per-step allocations."""
    env = _env()
    assert env.stable_observations
    obs0, cobs0 = env.get_observations(), env.get_privileged_observations()
    keep = (obs0.clone(), cobs0.clone())
    with torch.inference_mode():
        o1, c1, _, _, _ = env.step(torch.zeros(env.num_envs, 12, device="cuda:0"))
        k1 = (o1.clone(), c1.clone())
        env.episode_length_buf[:16] = int(env.max_episode_length)
        _, _, _, dones, _ = env.step(torch.zeros(env.num_envs, 12, device="cuda:0"))
    torch.cuda.synchronize()
    assert dones[:16].all()
    assert torch.equal(obs0, keep[0]) and torch.equal(cobs0, keep[1])
    assert torch.equal(o1, k1[0]) and torch.equal(c1, k1[1])
    assert o1.data_ptr() != env.obs_buf.data_ptr()


def test_runner_hands_out_views():
    """OnPolicyRunner turns the copies off (its PPO copies before stepping)."""
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.envs import XBotLCfgPPO
    from humanoid.utils.helpers import class_to_dict
    env = _env()
    tcfg = XBotLCfgPPO()
    tcfg.runner.num_steps_per_env = 4
    OnPolicyRunner(env, class_to_dict(tcfg), log_dir=None, device="cuda:0")
    assert not env.stable_observations
    assert env.get_observations().data_ptr() == env.obs_buf.data_ptr()
