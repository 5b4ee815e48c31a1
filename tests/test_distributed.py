"""Data-parallel PPO over torch.distributed (gloo, 2 processes on CPU): the same code path that
runs over RCCL on the GPU node (parameter broadcast, flat-gradient all-reduce, global advantage
statistics, all-reduced KL for the adaptive learning rate)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = dict(num_actor_obs=141, num_critic_obs=73, num_actions=12, actor_hidden_dims=[64, 32, 16],
             critic_hidden_dims=[48, 32, 16], base_lin_vel_hidden_dims=[24, 24], init_noise_std=1.0)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    import sys
    for p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _make_ppo(seed):
    from humanoid.algo.ppo import ActorCritic, PPO
    torch.manual_seed(seed)
    ac = ActorCritic(**SMALL)
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9,
              value_loss_coef=1.0, entropy_coef=0.001, learning_rate=1e-5, max_grad_norm=1.0,
              use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01, device="cpu")
    ppo.init_storage(8, 24, [141], [73], [12])
    return ac, ppo


def _worker_same_data(rank, world, port, golden_path, out_q):
    """Both ranks hold the reference's golden storage: the all-reduced mean gradient equals the
    single-process gradient, so the update must reproduce the reference's golden parameters."""
    _setup(rank, world, port)
    g = np.load(golden_path)
    ac, ppo = _make_ppo(seed=100 + rank)            # different init per rank ...
    if rank == 0:                                   # ... rank 0 holds the golden init, broadcast at PPO()
        pass
    sd0 = {k[len("init/"):]: torch.from_numpy(g[k]) for k in g.files if k.startswith("init/")}
    ac.load_state_dict(sd0)
    st = ppo.storage
    for k in ("observations", "privileged_observations", "actions", "rewards", "dones", "values", "actions_log_prob",
              "mu", "sigma", "returns", "advantages"):
        getattr(st, k).copy_(torch.from_numpy(g["st/" + k]))
    st.step = 24
    torch.manual_seed(1234)
    v, s, _, lv = ppo.update()
    final = {k[len("final/"):]: g[k] for k in g.files if k.startswith("final/")}
    err = max(float(np.abs(p.detach().numpy() - final[k]).max()) for k, p in ac.state_dict().items())
    out_q.put((rank, v, s, lv, ppo.learning_rate, err))
    dist.destroy_process_group()


def _worker_diff_data(rank, world, port, out_q):
    """Different rollouts per rank: parameters start identical (broadcast) and stay identical."""
    _setup(rank, world, port)
    import envlogic_ref as E
    ac, ppo = _make_ppo(seed=7 + rank)
    first = torch.cat([p.detach().flatten() for p in ac.parameters()])
    st = ppo.storage
    gen = torch.Generator().manual_seed(50 + rank)
    st.observations.normal_(generator=gen)
    st.privileged_observations.normal_(generator=gen)
    st.actions.normal_(generator=gen)
    st.rewards.uniform_(generator=gen)
    st.values.normal_(generator=gen)
    st.actions_log_prob.normal_(generator=gen)
    st.mu.normal_(generator=gen)
    st.sigma.uniform_(0.5, 1.5, generator=gen)
    st.dones.copy_((torch.rand(24, 8, 1, generator=gen) < 0.1).to(torch.uint8))
    st.gae_fn = lambda r, d, v, lv, g_, l_: tuple(
        torch.from_numpy(x)[..., None] for x in E.gae(r[..., 0].numpy(), d[..., 0].numpy(), v[..., 0].numpy(),
                                                      lv[:, 0].numpy(), g_, l_, normalize=False))
    st.compute_returns(torch.randn(8, 1, generator=gen), 0.994, 0.9)
    adv_local = st.advantages.clone()
    raw = (st.returns - st.values).double()
    st.step = 24
    torch.manual_seed(99)
    ppo.update()
    final = torch.cat([p.detach().flatten() for p in ac.parameters()])
    out_q.put((rank, first.numpy(), final.numpy(), adv_local.numpy(), raw.numpy(), ppo.learning_rate))
    dist.destroy_process_group()


def _run(target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, 2, port) + args + (q,)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_dp_update_matches_reference_golden():
    res = _run(_worker_same_data, os.path.join(REPO, "tests", "golden", "ppo_update.npz"))
    g = np.load(os.path.join(REPO, "tests", "golden", "ppo_update.npz"))
    for rank, v, s, lv, lr, err in res:
        np.testing.assert_allclose(v, g["value_loss"], rtol=1e-5)
        np.testing.assert_allclose(lv, g["lin_vel_loss"], rtol=1e-5)
        np.testing.assert_allclose(lr, g["learning_rate"], rtol=1e-12)
        assert err < 1e-5, err


def test_dp_ranks_stay_in_sync_and_normalise_globally():
    (r0, f0, p0, a0, raw0, lr0), (r1, f1, p1, a1, raw1, lr1) = _run(_worker_diff_data)
    np.testing.assert_array_equal(f0, f1)          # broadcast at construction
    np.testing.assert_allclose(p0, p1, atol=0)     # identical after the all-reduced update
    assert not np.allclose(p0, f0)
    assert lr0 == lr1
    allraw = np.concatenate([raw0.ravel(), raw1.ravel()])
    m, sd = allraw.mean(), allraw.std(ddof=1)
    np.testing.assert_allclose(a0.ravel(), (raw0.ravel() - m) / (sd + 1e-8), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(a1.ravel(), (raw1.ravel() - m) / (sd + 1e-8), rtol=1e-4, atol=1e-5)
