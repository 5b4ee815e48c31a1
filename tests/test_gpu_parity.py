"""GPU parity tests: the HIP path (through the C ABI) against the oracle on the same inputs.

  * K_gae vs the reference golden (rollout_storage.py:122-143)           -> bitwise returns
  * K_post vs oracle/pipeline_ref.post on a snapshot of the GPU state      -> rewards/obs/resets
  * K_step vs oracle/physics_ref.c (f64 and f32) from the same state       -> fp32 tolerance
  * 1000-step seeded trajectories, fixed base (tight) and floating base (divergence curve)
  * determinism: the same state and actions twice -> bitwise identical
"""
import math
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_ENVS = 64


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _make_env(n, **over):
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    torch.manual_seed(5)
    np.random.seed(5)
    cfg = XBotLCfg()
    cfg.env.num_envs = n
    cfg.seed = 5
    for k, v in over.items():
        sec, name = k.split("__")
        setattr(getattr(cfg, sec), name, v)
    return XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)


@pytest.fixture(scope="module")
def physics_env():
    _need_gpu()
    return _make_env(N_ENVS)


@pytest.fixture(scope="module")
def env():
    _need_gpu()
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    torch.manual_seed(5)
    np.random.seed(5)
    cfg = XBotLCfg()
    cfg.env.num_envs = N_ENVS
    cfg.seed = 5
    e = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    return e


def snapshot(env):
    torch.cuda.synchronize()
    g = lambda t: t.detach().cpu().numpy().copy()  # noqa: E731
    S = dict(root_states=g(env.root_states), dof_pos=g(env.dof_pos), dof_vel=g(env.dof_vel),
             contact_forces=g(env.contact_forces), rigid_state=g(env.rigid_state), torques=g(env.torques),
             actions=g(env.actions), last_actions=g(env.last_actions), last_last_actions=g(env.last_last_actions),
             last_dof_vel=g(env.last_dof_vel), last_root_vel=g(env.last_root_vel), commands=g(env.commands),
             episode_length_buf=g(env.episode_length_buf), feet_air_time=g(env.feet_air_time),
             last_contacts=g(env.last_contacts), feet_height=g(env.feet_height), last_feet_z=g(env.last_feet_z),
             env_frictions=g(env.env_frictions), body_mass=g(env.body_mass), rand_push_force=g(env.rand_push_force),
             rand_push_torque=g(env.rand_push_torque), ref_dof_pos=g(env.ref_dof_pos), env_origins=g(env.env_origins),
             lambda_=g(env._view(__import__("humanoid._native", fromlist=["T"]).T["CONTACT_LAMBDA"])),
             base_lin_vel=g(env.base_lin_vel), base_ang_vel=g(env.base_ang_vel))
    S["lambda"] = S.pop("lambda_")
    if getattr(env, "custom_origins", False):
        S["terrain_levels"] = g(env.terrain_levels).astype(np.int64)
        S["terrain_types"] = g(env.terrain_types).astype(np.int64)
        S["terrain_origins"] = g(env.terrain_origins)
    from humanoid.envs.custom.humanoid_env import REWARD_NAMES
    S["episode_sums"] = {n: g(env._sums[k]) for k, n in enumerate(REWARD_NAMES)}
    return S, g(env.obs_buf), g(env.privileged_obs_buf)


def _hg():
    from humanoid import _native as N
    return N


def test_library_version():
    _need_gpu()
    assert b"gfx950" in _hg().lib().hg_version()


@pytest.mark.parametrize("N", [4, 64])
def test_gae_kernel_matches_reference_golden(golden, N):
    _need_gpu()
    from humanoid.algo.ppo import RolloutStorage
    g = golden("gae.npz")
    T = 24
    st = RolloutStorage(N, T, [5], [7], [3], device="cuda:0")
    st.rewards.copy_(torch.from_numpy(g[f"N{N}_rewards"])[..., None])
    st.values.copy_(torch.from_numpy(g[f"N{N}_values"])[..., None])
    st.dones.copy_(torch.from_numpy(g[f"N{N}_dones"])[..., None])
    st.compute_returns(torch.from_numpy(g[f"N{N}_last_values"])[:, None].cuda(), 0.994, 0.9)
    np.testing.assert_array_equal(st.returns[..., 0].cpu().numpy(), g[f"N{N}_returns"])
    np.testing.assert_allclose(st.advantages[..., 0].cpu().numpy(), g[f"N{N}_advantages"], rtol=1e-5, atol=2e-6)


def test_gae_kernel_large_properties():
    """Full config-2 size (T=24, N=4096): normalised advantages have mean 0 / std 1 and the
    returns satisfy the GAE recursion checked against the oracle on a column sample."""
    _need_gpu()
    import envlogic_ref as E
    from humanoid.algo.ppo import RolloutStorage
    T, N = 24, 4096
    st = RolloutStorage(N, T, [1], [1], [1], device="cuda:0")
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    st.rewards.copy_(torch.randn(T, N, 1, device="cuda:0", generator=gen))
    st.values.copy_(torch.randn(T, N, 1, device="cuda:0", generator=gen))
    st.dones.copy_((torch.rand(T, N, 1, device="cuda:0", generator=gen) < 0.05).to(torch.uint8))
    last = torch.randn(N, 1, device="cuda:0", generator=gen)
    st.compute_returns(last, 0.994, 0.9)
    adv = st.advantages.double()
    assert abs(adv.mean().item()) < 1e-5 and abs(adv.std().item() - 1) < 1e-4
    ret, _ = E.gae(st.rewards[..., 0].cpu().numpy(), st.dones[..., 0].cpu().numpy(), st.values[..., 0].cpu().numpy(),
                   last[:, 0].cpu().numpy(), 0.994, 0.9)
    np.testing.assert_array_equal(st.returns[..., 0].cpu().numpy(), ret)


def test_gae_deterministic():
    """Two identical compute_returns calls give bitwise-identical normalised advantages: the
    (sum A, sum A^2) statistics are block partials summed in a fixed order (no float atomics)."""
    _need_gpu()
    from humanoid.algo.ppo import RolloutStorage
    T, N = 24, 4096
    gen = torch.Generator(device="cuda:0").manual_seed(11)
    r = torch.randn(T, N, 1, device="cuda:0", generator=gen)
    v = torch.randn(T, N, 1, device="cuda:0", generator=gen)
    d = (torch.rand(T, N, 1, device="cuda:0", generator=gen) < 0.05).to(torch.uint8)
    last = torch.randn(N, 1, device="cuda:0", generator=gen)
    outs = []
    for _ in range(2):
        st = RolloutStorage(N, T, [1], [1], [1], device="cuda:0")
        st.rewards.copy_(r)
        st.values.copy_(v)
        st.dones.copy_(d)
        st.compute_returns(last, 0.994, 0.9)
        outs.append((st.advantages.clone(), st._stats.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def _oracle_cfg(env):
    import pipeline_ref as PR
    return PR.Cfg(env._hgcfg)


def _post_once(env, counter):
    N = _hg()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().hg_post(env.sim, ctypes.c_uint64(counter), s), env.sim)
    torch.cuda.synchronize()


def test_post_parity(env):
    """K_post (rewards, commands, push, termination, masked reset, obs + noise, stacking) vs
    the numpy pipeline on the identical GPU state, with forced resets/timeouts/resample/push."""
    _post_parity(env)


def test_post_parity_heightfield(terrain_env):
    """Same on the heightfield terrain: resets land at the sub-terrain origins +- 1 m."""
    _post_parity(terrain_env)


def _post_parity(env, steps=3):
    import pipeline_ref as PR
    for _ in range(steps):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
    torch.cuda.synchronize()
    # force the branches: base contact on some envs, timeouts, command resample
    env.contact_forces[0:4, 0, 2] = 50.0
    env.episode_length_buf[4:8] = 2400
    env.episode_length_buf[8:12] = 799
    counter = 400 * 3  # push step
    S, hist_o, hist_p = snapshot(env)
    cfg = _oracle_cfg(env)
    obs, priv, rew, reset, timeout, terms = PR.post(cfg, S, counter, hist_o, hist_p)
    _post_once(env, counter)
    gpu = lambda t: t.detach().cpu().numpy()  # noqa: E731
    np.testing.assert_array_equal(gpu(env.reset_buf), reset)
    np.testing.assert_array_equal(gpu(env.time_out_buf), timeout)
    assert reset[:8].all() and not reset[8:12].any()
    np.testing.assert_allclose(gpu(env.rew_buf), rew, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(gpu(env.commands), S["commands"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(gpu(env.root_states), S["root_states"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gpu(env.dof_pos), S["dof_pos"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gpu(env.obs_buf), obs, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gpu(env.privileged_obs_buf), priv, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gpu(env.feet_air_time), S["feet_air_time"], atol=1e-6)
    np.testing.assert_allclose(gpu(env.feet_height), S["feet_height"], atol=1e-6)
    np.testing.assert_array_equal(gpu(env.last_contacts), S["last_contacts"])
    for k, n in enumerate(__import__("envlogic_ref").REWARD_NAMES):
        np.testing.assert_allclose(gpu(env._sums[k]), S["episode_sums"][n], rtol=2e-4, atol=1e-6, err_msg=n)


def _hf(env):
    return env.height_samples.cpu().numpy() if getattr(env, "height_samples", None) is not None else None


def _ref_sim(env, S, precision):
    import step_tolerance as ST
    return ST.ref_sim(env._hgcfg, env._model, S, precision, _hf(env))


# members of the CPU f32 ensemble behind the yardstick (oracle/step_tolerance.py: the state as
# given + members - 1 copies perturbed by a few ulp); at 4096 envs a single CPU draw under-estimates
# the tail (13 of 49152 torque elements in the first 4096-env run)
F32_STEP_ENSEMBLE = 3
# independent f32 builds judged against that yardstick (excluded from it): their count of envs
# outside the element tolerance is the fp32 discrete-event rate the GPU's count is held to
F32_NULL_CANDIDATES = 4


def _step_only(env, actions, counter):
    N = _hg()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = actions.contiguous()
    N.check(N.lib().hg_step(env.sim, ctypes.c_void_p(a.data_ptr()), ctypes.c_uint64(counter), s), env.sim)
    torch.cuda.synchronize()


# multiple of the fp32 yardstick max(gap32, spread) the GPU step may deviate by: the achieved
# maximum over every _step_parity call is 6.11 (qd of the hand-thigh test; 4.4 on the 4096-env
# rigid states, 2.6 at 8192 envs: profiles/r4_tol/tol_report_k20.jsonl, measured with K = 20), so
# K = 12 keeps a 2x margin (round 3 used 20); the value lives in oracle/step_tolerance.py, shared
# with smoke()
STEP_TOL_K = __import__("step_tolerance").STEP_TOL_K


def _report_headroom(env, headroom, key="ratio"):
    """Append the achieved max |gpu - f64| / max(gap32, spread) per field (beyond the rounding
    term) of one _step_parity call to $HG_TOL_REPORT (JSON lines), when set."""
    path = os.environ.get("HG_TOL_REPORT")
    if not path:
        return
    import json
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, "envs": env.num_envs, "k": STEP_TOL_K, key: headroom}) + "\n")


def _step_parity(env, counter, fields=("q", "qd", "root", "torques", "rigid"), scale=0.5, actions=None):
    """One K_step (prologue + 10 substeps + rigid states) from the env's current state vs the C
    reference simulator (f64, f32) on the identical state and preprocessed actions.  Stated fp32
    tolerance (oracle/step_tolerance.py): per element, STEP_TOL_K (12) x the
    larger of the CPU f32-vs-f64 gap and the local conditioning spread of the f64 step, plus fp32
    rounding (2^-20 relative, ~8 ulp), no absolute floor.  On contact steps at thousands of envs,
    rare discrete events (a joint-friction row between stick and slip, a contact crossing the
    offset) put any fp32 build outside that bound in a few envs; the count of envs with an element
    outside is therefore held to the fp32 rate measured on the same state — at most twice the mean
    count of F32_NULL_CANDIDATES independent CPU f32 builds judged against the same yardstick — and
    their deviations to 4 x the largest such a build shows there (zero envs whenever those builds
    have none).  Rows dropped over the budget: equal env for env.  The achieved multiples and the
    counts go to $HG_TOL_REPORT.  Returns the reference f64 sim."""
    import pipeline_ref as PR
    import step_tolerance as ST
    S, _, _ = snapshot(env)
    cfg = _oracle_cfg(env)
    if actions is None:
        actions = torch.randn(env.num_envs, 12, device="cuda:0") * scale
    a_ref = PR.preprocess_actions(cfg, actions.cpu().numpy(), S["actions"], counter)
    dropped0 = env.rows_dropped.clone()
    _step_only(env, actions, counter)
    g = lambda t: t.detach().cpu().numpy()  # noqa: E731
    np.testing.assert_allclose(g(env.actions), a_ref, rtol=1e-5, atol=1e-6)
    hc, model, hf = env._hgcfg, env._model, _hf(env)
    gpu = {"q": g(env.dof_pos), "qd": g(env.dof_vel), "root": g(env.root_states), "torques": g(env.torques),
           "rigid": g(env.rigid_state)}
    r64, report, fails, _ = ST.check_step(hc, model, S, a_ref, gpu, fields, hf, K=STEP_TOL_K,
                                          members=F32_STEP_ENSEMBLE, candidates=F32_NULL_CANDIDATES)
    _report_headroom(env, report, key="step")
    assert not fails, " | ".join(fails)
    assert not r64.nonfinite.any() and not g(env.nonfinite_count).any()
    # rows / contact points over the budget: the same count per env
    np.testing.assert_array_equal(g(env.rows_dropped - dropped0), r64.dropped)
    return r64


# policy steps before a compared contact step: from the 0.95 m spawn the first foot lands at step 9
# and every env is on the ground by step 12 (oracle, 0.3 randn actions)
TOUCHDOWN_STEPS = 24


def _assert_contact_step(env, r64, sloped_min=None):
    """The compared K_step is a contact step: >= 95 % of envs hold a ground
    contact with a positive normal impulse after the step, on the GPU and in the oracle (warm-start
    slots 3c of the ground candidates, the last substep's impulses); with `sloped_min`, at least
    that fraction of envs has such a contact on a heightfield triangle whose normal has z < 0.995
    (the terrain, not a flat patch, is in the compared step).  Returns the per-env statistics."""
    N = _hg()
    import physics_ref as P
    nc = N.HG_MAX_CONTACTS
    lam_gpu = env._view(N.T["CONTACT_LAMBDA"]).cpu().numpy()[:, 0:3 * nc:3]
    lam_ref = r64.lam[:, 0:3 * nc:3]
    on_gpu, on_ref = (lam_gpu > 0).any(axis=1), (lam_ref > 0).any(axis=1)
    stats = {"envs": env.num_envs, "ground_contact_gpu": float(on_gpu.mean()),
             "ground_contact_oracle": float(on_ref.mean()),
             "contacts_per_env_gpu": float((lam_gpu > 0).sum(axis=1).mean())}
    if sloped_min is not None:
        hf = env.height_samples.cpu().numpy()
        x = P.ground_candidates(env._model, env.rigid_state.cpu().numpy())
        _, nrm = P.ground(env._hgcfg, hf, x[..., 0], x[..., 1])
        steep = nrm[..., 2] < 0.995
        stats["sloped_contact_gpu"] = float(((lam_gpu > 0) & steep).any(axis=1).mean())
        stats["sloped_contact_oracle"] = float(((lam_ref > 0) & steep).any(axis=1).mean())
    print("contact step:", stats)
    _report_headroom(env, stats, key="contact")
    assert stats["ground_contact_gpu"] >= 0.95 and stats["ground_contact_oracle"] >= 0.95, stats
    if sloped_min is not None:
        assert stats["sloped_contact_gpu"] >= sloped_min and stats["sloped_contact_oracle"] >= sloped_min, stats
    return stats


def test_step_physics_parity(physics_env):
    """One K_step (prologue + 10 substeps + rigid states) vs the C reference simulator."""
    env = physics_env
    for _ in range(5):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    _step_parity(env, 77)


def test_step_physics_parity_after_update_cfg():
    """K_step takes its physics scalars by value from the handle's host copy of hg_cfg at each
    launch: after hg_update_cfg changes the PGS sweeps, the contact offset and the Baumgarte
    factor mid-run, the next step (on a contact state) matches the oracle run with the new values."""
    _need_gpu()
    import ctypes
    from humanoid import _native as N
    env = _make_env(N_ENVS)
    for _ in range(TOUCHDOWN_STEPS):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    hc = env._hgcfg
    hc.pgs_iterations, hc.contact_offset, hc.baumgarte = 2, 0.02, 0.1
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(env.hg.hg_update_cfg(env.sim, ctypes.byref(hc), stream), env.sim)
    _step_parity(env, 91)


@pytest.fixture(scope="module")
def bench_env():
    """The bench's size (4096 envs: 2048 blocks, 256 per XCD, the full XCD-aware block -> env-pair
    map of K_step and K_post's full grid)."""
    _need_gpu()
    return _make_env(4096)


@pytest.fixture(scope="module")
def bench_terrain_env():
    _need_gpu()
    return _make_env(4096, terrain__mesh_type="heightfield")


@pytest.mark.parametrize("which", ["plane", "heightfield"])
def test_step_and_post_parity_4096_envs(which, request):
    """K_step and K_post against the oracle at the bench's 4096 envs (config 2 plane, config 3
    heightfield): the same stated tolerances as the 64-env tests, every env checked, on a contact
    step (>= 95 % of envs on the ground, >= 10 % on a sloped heightfield triangle; rows dropped
    equal env for env)."""
    env = request.getfixturevalue("bench_env" if which == "plane" else "bench_terrain_env")
    for _ in range(TOUCHDOWN_STEPS):  # past touchdown: the compared step resolves ground contact
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    r64 = _step_parity(env, 131)
    _assert_contact_step(env, r64, sloped_min=0.10 if which == "heightfield" else None)
    _post_parity(env, steps=0)


def test_hand_thigh_self_collision_parity():
    """Base-link shapes vs the legs (humanoid_config.py:103, XBot-L.urdf:37-42 +
    the merged arm / hand shapes): fixed base, each hip rolled 0.34 rad outward so the thigh sits
    in its hand capsule (contact at ~0.31 rad).  K_step vs the oracle at the stated tolerance, the
    hand-thigh pair impulse positive in both, forces on base and thigh equal and opposite."""
    _need_gpu()
    from humanoid import _native as N
    env = _make_env(N_ENVS, asset__fix_base_link=True)
    js = env._model_js if hasattr(env, "_model_js") else N.load_model()[1]
    caps, pairs = js["capsules"], js["pairs"]
    hp = {caps[a]["side"]: p for p, (a, b) in enumerate(pairs) if caps[a]["part"] == "hand" and caps[b]["part"] == "leg_pitch"}
    half = N_ENVS // 2
    env.dof_pos[:half, 0] = 0.34
    env.dof_pos[half:, 6] = -0.34
    act = env.dof_pos / env.cfg.control.action_scale
    r64 = _step_parity(env, 55, actions=act.contiguous())
    lam = env._view(N.T["CONTACT_LAMBDA"]).cpu().numpy()
    lp = N.HG_MAX_CONTACTS * 3
    cf = env.contact_forces.cpu().numpy()
    for rows, side, thigh in ((slice(0, half), "left", 3), (slice(half, N_ENVS), "right", 9)):
        k = lp + 3 * hp[side]
        # the thigh is pushed out of the hand within the step in some envs (impulse back to 0 at
        # the last substep); the pair carries an impulse in most, on the GPU and in the oracle
        on_gpu, on_ref = lam[rows, k] > 0, r64.lam[rows, k] > 0
        print(side, "pair impulse > 0 in", int(on_gpu.sum()), "(GPU) /", int(on_ref.sum()), "(oracle) of", half)
        assert on_gpu.mean() >= 0.5 and on_ref.mean() >= 0.5, side
        assert (on_gpu == on_ref).mean() >= 0.9, side
        np.testing.assert_allclose(cf[rows, 0], -cf[rows, thigh], rtol=1e-4, atol=1e-3)
        assert (np.linalg.norm(cf[rows, thigh], axis=1)[on_gpu] > 1.0).all()


def test_row_budget_parity_standing_mjcf_friction():
    """Row budget order on the GPU: the MJCF friction profile (12 friction rows) on
    robots standing on both soles (24 rows) with both hip yaws 0.01 rad past their lower limit:
    38 rows wanted, 6 dropped per substep, and they are the 0.01 N m hip-yaw / hip-pitch / knee
    friction rows of both legs — the same counts and the same kept / cleared warm-start slots as
    the oracle, env for env."""
    _need_gpu()
    from humanoid import _native as N
    from humanoid.scripts import sim2sim as S2
    env = S2.make_env("mjcf", N_ENVS, 5.0)
    for _ in range(80):
        S2.step_direct(env, torch.zeros(N_ENVS, 12, device="cuda:0"))
    torch.cuda.synchronize()
    lo = torch.tensor([env._model.lower[b] for b in range(1, 13)], device="cuda:0")
    env.dof_pos[:, [1, 7]] = lo[[1, 7]] - 0.01
    act = torch.zeros(N_ENVS, 12, device="cuda:0")
    act[:, [1, 7]] = (lo[[1, 7]] - 0.01) / env.cfg.control.action_scale
    env.actions[:] = act
    r64 = _step_parity(env, 300, fields=("q", "qd", "root", "torques"), actions=act)  # dropped counts equal
    # envs in double support through the whole step (8 sole points every substep: 6 x 10 dropped)
    ds = r64.dropped == 60
    print("double-support envs", int(ds.sum()), "of", N_ENVS, "dropped counts", np.bincount(r64.dropped)[np.bincount(r64.dropped) > 0])
    assert ds.mean() >= 0.5
    lam = env._view(N.T["CONTACT_LAMBDA"]).cpu().numpy()
    lf = (N.HG_MAX_CONTACTS + N.HG_MAX_PAIRS) * 3 + N.HG_MAX_DOF
    for L in (lam[ds], r64.lam[ds]):
        assert (L[:, [lf + j for j in (4, 10, 5, 11, 0, 6)]] != 0).all()
        assert (L[:, [lf + j for j in (1, 7, 2, 8, 3, 9)]] == 0).all()


def test_nonfinite_guard_resets_and_counts():
    """Fault injection into the non-finite guard (csrc/hg_physics.hip epilogue): NaN joint
    velocities in two envs make their substeps non-finite; K_step keeps their pre-step pose, counts
    the event in HG_T_NONFINITE and pushes the base below ground with a base contact, so K_post's
    termination resets them.  Every other env must be bit-identical to an untouched twin."""
    _need_gpu()
    env, twin = _make_env(N_ENVS), _make_env(N_ENVS)
    for e in (env, twin):  # the same run twice (same seeds, same actions): bitwise-equal states
        gen = torch.Generator(device="cpu").manual_seed(21)
        for _ in range(3):
            e.step((torch.randn(N_ENVS, 12, generator=gen) * 0.3).to("cuda:0"))
    torch.cuda.synchronize()
    assert torch.equal(env.dof_vel, twin.dof_vel) and torch.equal(env.root_states, twin.root_states)
    bad = [5, 40]
    before = env.nonfinite_count.clone()
    env.dof_vel[bad, 3] = float("nan")
    a = torch.randn(N_ENVS, 12, device="cuda:0") * 0.3
    counter = 1000 + env.common_step_counter
    _step_only(env, a, counter)
    _step_only(twin, a, counter)
    g = lambda t: t.detach().cpu().numpy()  # noqa: E731
    cnt = g(env.nonfinite_count - before)
    assert cnt[bad].tolist() == [1, 1] and cnt.sum() == 2
    assert (g(env.root_states)[bad, 2] < -5).all() and (g(env.contact_forces)[bad, 0, 2] > 1.0).all()
    assert np.isfinite(g(env.dof_vel)[bad]).all()
    others = np.setdiff1d(np.arange(N_ENVS), bad)
    for k in ("root_states", "dof_pos", "dof_vel", "torques", "contact_forces", "rigid_state"):
        np.testing.assert_array_equal(g(getattr(env, k))[others], g(getattr(twin, k))[others], err_msg=k)
    # K_post terminates and resets exactly the faulted envs; their state is finite again
    _post_once(env, counter + 1)
    reset = g(env.reset_buf).astype(bool)
    assert reset[bad].all()
    assert np.isfinite(g(env.root_states)).all() and np.isfinite(g(env.dof_vel)).all()
    assert (g(env.root_states)[bad, 2] > 0.5).all()


# Stated fp32 tolerances of the SURVEY §8d parity trajectory (1000 policy steps = 10,000
# substeps, seed 5, open-loop a_t[j] = 0.5 sin(2 pi t 0.01 / 0.64 + j pi / 6), DR and noise off),
# HIP K_step vs the f64 reference simulator (oracle/physics_ref.c), DESIGN.md §4:
#   variant A (fixed base): |dq| <= TRAJ_FIXED_DQ rad, |dtau| <= TRAJ_FIXED_DTAU N m over all steps;
#   variant B (floating base, chaotic contact dynamics): the running max of |dq| stays within
#   TRAJ_FLOAT_K x the running max of the CPU fp32-vs-f64 divergence (+ TRAJ_FLOAT_FLOOR rad) at
#   every step — the HIP fp32 path diverges from f64 no faster than fp32 arithmetic itself does.
#   The fp32 yardstick is an ensemble: the CPU f32 run plus F32_ENSEMBLE - 1 runs from the same
#   state perturbed by 2^-23 relative.  One fp32 run alone is a single draw of when a bifurcation
#   (a foot catching, the fall) separates from f64; the GPU, summing in other orders, is another
#   draw, and against one CPU run it led by up to 3.7x for ~20 steps at the fall (seed 5, step 150).
F32_ENSEMBLE = 4
TRAJ_FIXED_DQ = 1e-5
TRAJ_FIXED_DTAU = 1e-2
TRAJ_FLOAT_K = 2.0
TRAJ_FLOAT_FLOOR = 1e-5


def test_trajectory_1000_steps_fixed_base():
    """SURVEY §8d parity trajectory, variant A (fix_base_link): joint angles / torques of the HIP
    path vs the f64 reference simulator over 1000 policy steps (10,000 substeps)."""
    _need_gpu()
    c = _run_trajectory(fixed=True, steps=1000)
    print("fixed base: gpu-vs-f64 |dq| %.3g |dtau| %.3g; cpu f32-vs-f64 |dq| %.3g |dtau| %.3g" % (
        c["gpu_q"].max(), c["gpu_tau"].max(), c["f32_q"].max(), c["f32_tau"].max()))
    assert c["gpu_q"].max() <= TRAJ_FIXED_DQ, c["gpu_q"].max()
    assert c["gpu_tau"].max() <= TRAJ_FIXED_DTAU, c["gpu_tau"].max()


def test_trajectory_floating_base():
    """Variant B (floating base on the plane, the robot falls under open-loop actions): the
    fp32 HIP path tracks f64 within TRAJ_FLOAT_K x the CPU fp32 divergence envelope at every one
    of the 1000 steps."""
    _need_gpu()
    c = _run_trajectory(fixed=False, steps=1000)
    env_gpu, env_f32 = np.maximum.accumulate(c["gpu_q"]), np.maximum.accumulate(c["f32_q"])
    print("floating base |dq| gpu/f32 at steps 100/300/1000:", [(env_gpu[i], env_f32[i]) for i in (99, 299, 999)])
    bad = env_gpu > TRAJ_FLOAT_K * env_f32 + TRAJ_FLOAT_FLOOR
    assert not bad.any(), f"first step over the envelope: {int(np.argmax(bad))}"


def _run_trajectory(fixed, steps, n=16):
    """Per-step max |dq|, |dtau| of the HIP path and of the CPU fp32 oracle, both vs the f64 oracle
    (curves also written to $HG_TRAJ_OUT/trajectory_<variant>.json when set)."""
    import json
    import pipeline_ref as PR
    env = _make_env(n, asset__fix_base_link=fixed, domain_rand__dynamic_randomization=0.0,
                    domain_rand__push_robots=False, noise__add_noise=False)
    S, _, _ = snapshot(env)
    oc = _oracle_cfg(env)
    r64 = _ref_sim(env, S, "f64")
    r32s = [_ref_sim(env, S, "f32") for _ in range(F32_ENSEMBLE)]
    rng = np.random.default_rng(77)
    for m in r32s[1:]:  # fp32-rounding-sized perturbations of the initial state (2^-23 relative)
        for a in (m.root, m.q, m.qd):
            a *= (1 + 2.0 ** -23 * rng.standard_normal(a.shape)).astype(a.dtype)
    prev_gpu = np.zeros((n, 12), np.float32)
    c = {k: [] for k in ("gpu_q", "gpu_tau", "f32_q", "f32_tau")}
    j = np.arange(12)
    for t in range(steps):
        a = np.tile(0.5 * np.sin(2 * np.pi * t * 0.01 / 0.64 + j * np.pi / 6), (n, 1)).astype(np.float32)
        a_ref = PR.preprocess_actions(oc, a, prev_gpu, t)
        _step_only(env, torch.from_numpy(a).cuda(), t)
        prev_gpu = env.actions.cpu().numpy()
        r64.step(a_ref.astype(np.float64))
        for m in r32s:
            m.step(a_ref)
        q, tau = env.dof_pos.cpu().numpy(), env.torques.cpu().numpy()
        c["gpu_q"].append(np.abs(q - r64.q).max())
        c["gpu_tau"].append(np.abs(tau - r64.torques).max())
        c["f32_q"].append(max(np.abs(m.q - r64.q).max() for m in r32s))
        c["f32_tau"].append(max(np.abs(m.torques - r64.torques).max() for m in r32s))
    assert np.isfinite(env.dof_pos.cpu().numpy()).all()
    c = {k: np.array(v) for k, v in c.items()}
    out = os.environ.get("HG_TRAJ_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"trajectory_{'fixed' if fixed else 'floating'}.json"), "w") as f:
            json.dump({k: [float(x) for x in v] for k, v in c.items()}, f)
    return c


def test_determinism(env):
    """Same state + same actions -> bitwise-identical steps (no inter-env atomics on the path, no
    unsynchronised cross-lane LDS traffic): 10 consecutive steps from one snapshot, twice, with
    some envs' legs rolled into each other so the self-collision rows are exercised too."""
    from humanoid import _native as N
    for _ in range(3):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    torch.cuda.synchronize()
    env.dof_pos[0:8, 0] = -0.12
    env.dof_pos[0:8, 6] = 0.12
    S, _, _ = snapshot(env)
    acts = [torch.randn(env.num_envs, 12, device="cuda:0") for _ in range(10)]
    lam = env._view(N.T["CONTACT_LAMBDA"])
    outs = []
    pair_slots = slice(24 * 3, 32 * 3)
    pair_active = False
    for _ in range(2):
        for k in ("root_states", "dof_pos", "dof_vel", "actions"):
            getattr(env, k).copy_(torch.from_numpy(S[k]).cuda())
        lam.copy_(torch.from_numpy(S["lambda"]).cuda())
        for t, a in enumerate(acts):
            _step_only(env, a, 999 + t)
            pair_active |= bool((lam[:, pair_slots] != 0).any())
        outs.append((env.dof_pos.cpu().clone(), env.root_states.cpu().clone(), env.contact_forces.cpu().clone(),
                     lam.cpu().clone(), env.rigid_state.cpu().clone()))
    assert pair_active, "no self-collision row was active"
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_runner_one_iteration():
    """Config-2 shape end to end at small N: OnPolicyRunner.learn on the GPU env (1 iteration)."""
    _need_gpu()
    from humanoid.envs import XBotLCfg, XBotLCfgPPO
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.utils.helpers import SimParams, class_to_dict
    cfg = XBotLCfg()
    cfg.env.num_envs = 128
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    tcfg = XBotLCfgPPO()
    tcfg.runner.num_steps_per_env = 8
    runner = OnPolicyRunner(env, class_to_dict(tcfg), log_dir=None, device="cuda:0")
    runner.learn(2, init_at_random_ep_len=True)
    st = runner.last_iteration_stats
    assert np.isfinite(st["value_loss"]) and np.isfinite(st["surrogate_loss"])
    assert torch.isfinite(env.obs_buf).all()


def test_ppo_update_sync_free_matches_golden(golden, monkeypatch):
    """The device-resident update (fused Adam with a float64 device learning rate, adaptive-KL
    rule evaluated with torch.where, losses read once) against the reference golden update.
    Minibatch order is drawn on the CPU generator exactly as in the golden run."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from test_ppo_golden import SMALL, sd
    g = golden("ppo_update.npz")
    torch.manual_seed(0)
    ac = ActorCritic(**SMALL)
    ac.load_state_dict(sd(g, "init/"))
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, clip_param=0.2, gamma=0.994, lam=0.9,
              value_loss_coef=1.0, entropy_coef=0.001, learning_rate=1e-5, max_grad_norm=1.0,
              use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01, device="cuda:0")
    assert ppo._lr_t is not None and ppo._lr_t.is_cuda
    ppo.init_storage(8, 24, [141], [73], [12])
    st = ppo.storage
    for k in ("observations", "privileged_observations", "actions", "rewards", "dones", "values", "actions_log_prob",
              "mu", "sigma", "returns", "advantages"):
        getattr(st, k).copy_(torch.from_numpy(g["st/" + k]))
    st.step = 24
    real = torch.randperm
    monkeypatch.setattr(torch, "randperm", lambda n, **kw: real(n).to(kw.get("device", "cpu")))
    torch.manual_seed(1234)
    vloss, sloss, sym, lvloss = ppo.update()
    np.testing.assert_allclose(vloss, g["value_loss"], rtol=1e-4)
    np.testing.assert_allclose(sloss, g["surrogate_loss"], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(lvloss, g["lin_vel_loss"], rtol=1e-4)
    np.testing.assert_allclose(ppo.learning_rate, g["learning_rate"], rtol=1e-12)
    final = sd(g, "final/")
    for k, v in ac.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), final[k].numpy(), rtol=1e-4, atol=2e-6, err_msg=k)


def test_ppo_graphed_update_matches_eager():
    """Three updates replayed from the captured HIP graphs == three eager updates (same data,
    same minibatch permutations)."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from test_ppo_golden import SMALL
    torch.manual_seed(3)
    init = ActorCritic(**SMALL).state_dict()
    data = {}
    g = torch.Generator().manual_seed(11)
    shapes = {"observations": (24, 64, 141), "privileged_observations": (24, 64, 73), "actions": (24, 64, 12),
              "rewards": (24, 64, 1), "values": (24, 64, 1), "actions_log_prob": (24, 64, 1), "mu": (24, 64, 12),
              "sigma": (24, 64, 12), "returns": (24, 64, 1), "advantages": (24, 64, 1)}
    for k, sh in shapes.items():
        data[k] = torch.randn(*sh, generator=g)
    data["sigma"] = data["sigma"].abs() + 0.5
    runs = []
    for graphs in (False, True):
        ac = ActorCritic(**SMALL)
        ac.load_state_dict(init)
        ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=4, learning_rate=1e-3, entropy_coef=0.001,
                  schedule="adaptive", desired_kl=0.01, device="cuda:0")
        ppo.use_graphs = graphs
        ppo.init_storage(64, 24, [141], [73], [12])
        losses = []
        import warnings
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            for it in range(3):
                for k, v in data.items():
                    getattr(ppo.storage, k).copy_(v)
                torch.cuda.manual_seed(100 + it)
                losses.append(ppo.update())
        # no autograd graph from the eager warm-up survives into the captured update
        assert not [w for w in caught if "AccumulateGrad" in str(w.message)]
        runs.append(({k: v.detach().cpu() for k, v in ac.state_dict().items()}, losses, ppo.learning_rate))
    (sd0, l0, lr0), (sd1, l1, lr1) = runs
    assert lr0 == lr1
    np.testing.assert_allclose(np.array(l1)[:, [0, 1, 3]].astype(float), np.array(l0)[:, [0, 1, 3]].astype(float),
                               rtol=1e-5, atol=1e-7)
    for k in sd0:
        np.testing.assert_allclose(sd1[k].numpy(), sd0[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.fixture(scope="module")
def terrain_env():
    _need_gpu()
    return _make_env(N_ENVS, terrain__mesh_type="heightfield", terrain__measure_heights=True)


def test_step_physics_parity_heightfield(terrain_env):
    """K_step on the generated heightfield (config 3 terrain) vs the C reference simulator
    colliding against the same int16 samples, at the plane test's stated tolerance (no absolute
    floor)."""
    env = terrain_env
    assert env._hgcfg.terrain_type == 1 and tuple(env.height_samples.shape) == (2100, 2100)
    for _ in range(30):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    _step_parity(env, 91, fields=("q", "qd", "root", "torques"))
    # the robots stand on terrain: base heights follow the sub-terrain origins, not z = 0
    assert np.isfinite(env.root_states.cpu().numpy()).all()


def test_measured_heights(terrain_env):
    env = terrain_env
    for _ in range(5):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    import pipeline_ref as PR
    h = env._get_heights().cpu()
    # oracle: pipeline_ref.heights, pinned against the reference's _get_heights (tests/golden/heights.npz)
    ref = torch.from_numpy(PR.heights(_oracle_cfg(env), env.root_states.cpu().numpy(), env._height_xy.cpu().numpy(),
                                      env.height_samples.cpu().numpy()))
    assert h.shape == (env.num_envs, 187)
    exact = (h == ref).float().mean().item()
    assert exact > 0.999, exact  # cell-boundary float ties aside, bit-exact
    assert (h - ref).abs().max().item() <= 0.1
    sub = env._get_heights(env_ids=[3, 5]).cpu()
    torch.testing.assert_close(sub, h[[3, 5]])


def test_terrain_curriculum_parity():
    """Curriculum on: resets move robots that walked > 4 m one level up, robots that walked less
    than |cmd| * T_ep / 2 one level down, past-the-top levels re-drawn (Philox), origins follow
    (humanoid_env.py:1075-1095); against the numpy pipeline on the same state."""
    _need_gpu()
    import pipeline_ref as PR
    env = _make_env(N_ENVS, terrain__mesh_type="heightfield", terrain__curriculum=True)
    assert env._hgcfg.curriculum == 1
    for _ in range(3):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    torch.cuda.synchronize()
    n = 16
    env.contact_forces[0:n, 0, 2] = 50.0                          # terminate envs 0..15
    env.root_states[0:4, 0] = env.env_origins[0:4, 0] + 5.0        # walked far: level up
    env.terrain_levels[2:4] = env.cfg.terrain.num_rows - 1         # ... past the top: re-draw
    env.root_states[4:8, :2] = env.env_origins[4:8, :2]            # stood still ...
    env.commands[4:8, 0] = 0.5                                     # ... under a command: level down
    env.terrain_levels[6:8] = 0                                    # ... already at 0: clip
    counter = 777
    S, hist_o, hist_p = snapshot(env)
    cfg = _oracle_cfg(env)
    lv0 = S["terrain_levels"].copy()
    obs, priv, rew, reset, timeout, terms = PR.post(cfg, S, counter, hist_o, hist_p)
    _post_once(env, counter)
    gpu = lambda t: t.detach().cpu().numpy()  # noqa: E731
    assert reset[:n].all()
    np.testing.assert_array_equal(gpu(env.terrain_levels), S["terrain_levels"])
    np.testing.assert_allclose(gpu(env.env_origins), S["env_origins"], rtol=0, atol=0)
    np.testing.assert_allclose(gpu(env.root_states), S["root_states"], rtol=1e-6, atol=1e-6)
    lv = S["terrain_levels"]
    assert (lv[0:2] == lv0[0:2] + 1).all() and (lv[4:6] == lv0[4:6] - 1).all() and (lv[6:8] == 0).all()
    assert ((lv[2:4] >= 0) & (lv[2:4] < env.cfg.terrain.num_rows)).all()


def test_train_checkpoint_resume_export(tmp_path):
    """Caller path of train.py / play.py: task_registry.make_env + make_alg_runner, learn with
    logging and checkpoints, resume through get_load_path, export TorchScript + ONNX."""
    _need_gpu()
    import os
    from humanoid.envs import XBotLCfgPPO  # noqa: F401  (registers humanoid_ppo)
    from humanoid.utils import get_args, task_registry
    from humanoid.utils.helpers import export_policy_as_jit, get_load_path
    from humanoid.utils.onnx_io import export_policy_as_onnx, load_onnx_mlp
    args = get_args(["--num_envs", "64", "--max_iterations", "2", "--headless", "--run_name", "t"])
    env, _ = task_registry.make_env("humanoid_ppo", args=args)
    _, tcfg = task_registry.get_cfgs("humanoid_ppo")
    tcfg.runner.num_steps_per_env = 8
    runner, tcfg = task_registry.make_alg_runner(env, args=args, train_cfg=tcfg, log_root=str(tmp_path))
    runner.learn(2, init_at_random_ep_len=True)
    ckpt = get_load_path(str(tmp_path))
    assert ckpt.endswith("model_2.pt") and os.path.exists(ckpt)
    logs = os.listdir(os.path.dirname(ckpt))
    assert any(f.startswith("events") or f.endswith(".jsonl") for f in logs), logs
    sd = {k: v.clone() for k, v in runner.alg.actor_critic.state_dict().items()}
    args2 = get_args(["--num_envs", "64", "--headless", "--resume"])
    runner2, _ = task_registry.make_alg_runner(env, args=args2, train_cfg=tcfg, log_root=str(tmp_path))
    for k, v in runner2.alg.actor_critic.state_dict().items():
        torch.testing.assert_close(v, sd[k])
    assert runner2.current_learning_iteration == 2
    out = tmp_path / "exported"
    export_policy_as_jit(runner2.alg.actor_critic, str(out))
    export_policy_as_onnx(runner2.alg.actor_critic, str(out))
    policy = runner2.get_inference_policy(device="cuda:0")
    obs = env.get_observations()
    m = load_onnx_mlp(str(out / "policy.onnx")).to("cuda:0")
    with torch.no_grad():
        torch.testing.assert_close(m(obs), policy(obs), rtol=1e-5, atol=1e-5)


def test_hg_adam_matches_torch_clip_adam():
    """hg_adam_step (fused global-norm clip + Adam, csrc/hg_optim.hip) == clip_grad_norm_ +
    torch.optim.Adam over several steps, including steps where clipping is active; state dicts
    interchange with torch.optim.Adam."""
    _need_gpu()
    from humanoid.algo.ppo.hg_adam import HgAdam
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(512, 705), (512,), (256, 512), (256,), (12, 128), (12,), (12,)]
    init = [torch.randn(*s, generator=g) * 0.1 for s in shapes]
    grads = [[torch.randn(*s, generator=g) * sc for s in shapes] for sc in (0.001, 0.5, 0.01, 2.0)]
    lr = torch.tensor(3e-4, device="cuda:0")
    pa = [torch.nn.Parameter(x.clone().cuda()) for x in init]
    pb = [torch.nn.Parameter(x.clone().cuda()) for x in init]
    oa = HgAdam(pa, lr=lr)
    ob = torch.optim.Adam(pb, lr=3e-4, foreach=False)
    for gs in grads:
        for p, x in zip(pa, gs):
            p.grad = x.cuda()
        for p, x in zip(pb, gs):
            p.grad = x.cuda()
        oa.step(max_norm=1.0)
        torch.nn.utils.clip_grad_norm_(pb, 1.0)
        ob.step()
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-7)
    sa = oa.state_dict()
    assert set(sa["state"][0]) == {"step", "exp_avg", "exp_avg_sq"} and float(sa["state"][0]["step"]) == 4
    oc = HgAdam([torch.nn.Parameter(x.clone().cuda()) for x in init], lr=lr)
    oc.load_state_dict(ob.state_dict())
    assert oc.version == 1
    torch.testing.assert_close(oc.state_dict()["state"][0]["exp_avg"], ob.state_dict()["state"][0]["exp_avg"])


def test_config5_bf16_policy_fp16_storage_push_curriculum():
    """Config 5 pieces: push-recovery curriculum through hg_update_cfg (pushes reach the ramped
    1.0 m/s bound, post still matches the oracle with the updated cfg), bf16-autocast policy and
    fp16 observation storage through two captured PPO iterations."""
    _need_gpu()
    import pipeline_ref as PR
    from humanoid.algo.ppo import OnPolicyRunner
    import bench
    env = _make_env(N_ENVS, domain_rand__push_curriculum=True)
    env.update_push_curriculum(0)
    assert abs(env._hgcfg.max_push_vel_xy - 0.2) < 1e-6
    env.update_push_curriculum(10 ** 6)
    assert abs(env._hgcfg.max_push_vel_xy - 1.0) < 1e-6 and abs(env._hgcfg.max_push_ang_vel - 1.0) < 1e-6
    for _ in range(2):
        env.step(torch.zeros(env.num_envs, 12, device="cuda:0"))
    counter = int(env._hgcfg.push_interval) * 7
    S, hist_o, hist_p = snapshot(env)
    obs, priv, rew, reset, timeout, _ = PR.post(_oracle_cfg(env), S, counter, hist_o, hist_p)
    _post_once(env, counter)
    v = env.root_states[:, 7:9].cpu().numpy()
    np.testing.assert_allclose(v, S["root_states"][:, 7:9], rtol=1e-6, atol=1e-6)
    assert np.abs(v).max() > 0.2 and np.abs(v).max() <= 1.0 + 1e-6
    runner = OnPolicyRunner(env, bench.train_cfg(8, "bf16", "fp16"), log_dir=None, device="cuda:0")
    assert runner.alg.storage.observations.dtype == torch.float16
    assert runner.alg.actor_critic.policy_dtype == "bf16"
    runner.learn(3, init_at_random_ep_len=True)
    st = runner.last_iteration_stats
    assert np.isfinite(st["value_loss"]) and np.isfinite(st["surrogate_loss"])
    assert all(torch.isfinite(p).all() for p in runner.alg.actor_critic.parameters())


def test_config5_8192_envs_per_rank():
    """Config 5 at its per-rank size (65536 envs on 8 GPUs = 8192 per rank):
    one K_step (a contact step, after touchdown) + K_post against the oracle at the stated
    tolerances with the push curriculum
    ramped to its final bounds, then two runner iterations of the bf16 policy with fp16
    observation storage: finite losses, finite parameters that moved."""
    _need_gpu()
    from humanoid.algo.ppo import OnPolicyRunner
    import bench
    env = _make_env(8192, domain_rand__push_curriculum=True)
    env.update_push_curriculum(10 ** 6)
    for _ in range(TOUCHDOWN_STEPS):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    r64 = _step_parity(env, 211)
    _assert_contact_step(env, r64)
    _post_parity(env, steps=0)
    runner = OnPolicyRunner(env, bench.train_cfg(24, "bf16", "fp16"), log_dir=None, device="cuda:0")
    assert runner.alg.storage.privileged_observations.dtype == torch.float16
    assert runner.alg.actor_critic.policy_dtype == "bf16"
    p0 = {k: v.detach().clone() for k, v in runner.alg.actor_critic.state_dict().items()}
    runner.learn(2, init_at_random_ep_len=True)
    st = runner.last_iteration_stats
    assert all(np.isfinite(st[k]) for k in ("value_loss", "surrogate_loss", "lin_vel_loss"))
    moved = 0
    for k, v in runner.alg.actor_critic.state_dict().items():
        assert torch.isfinite(v).all(), k
        moved += int(not torch.equal(v, p0[k]))
    assert moved >= len(p0) - 1
    assert torch.isfinite(env.obs_buf).all() and not env.nonfinite_count.any()


def test_kl_mean_and_lr_rule_kernels():
    """hg_kl_mean == the reference KL expression (ppo.py:162-166) in fp64; hg_kl_lr_rule == the
    Python schedule (ppo.py:168-176) bit for bit in float64 for kl above, inside and below the band."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from test_ppo_golden import SMALL
    ppo = PPO(ActorCritic(**SMALL), learning_rate=1e-3, schedule="adaptive", desired_kl=0.01, device="cuda:0")
    g = torch.Generator().manual_seed(7)
    mu, omu = torch.randn(3000, 12, generator=g), torch.randn(3000, 12, generator=g) * 0.1
    sg, osg = torch.rand(3000, 12, generator=g) + 0.3, torch.rand(3000, 12, generator=g) + 0.3
    ref = (torch.log(sg.double() / osg.double() + 1e-5) + (osg.double() ** 2 + (omu.double() - mu.double()) ** 2)
           / (2 * sg.double() ** 2) - 0.5).sum(-1).mean().item()
    kl = ppo._kl_mean(mu.cuda(), sg.cuda(), omu.cuda(), osg.cuda())
    assert abs(kl.item() - ref) <= 1e-5 * abs(ref)
    lr = 1e-3
    for k in (0.5, 0.03, 0.015, 0.004, 0.0, -1.0, 0.001, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3,
              1e3, 1e3, 1e3, 1e3, 1e3, 1e-4, 1e-4):
        kt = torch.tensor(k, dtype=torch.float32, device="cuda:0")
        ppo._lr_rule_device(kt)
        kf = float(np.float32(k))
        if kf > 0.02:
            lr = max(1e-5, lr / 1.5)
        elif kf < 0.005 and kf > 0.0:
            lr = min(1e-2, lr * 1.5)
        assert ppo.learning_rate == lr, (k, ppo.learning_rate, lr)
        assert ppo._lr_f32.item() == np.float32(lr)


@pytest.mark.parametrize("obs_dtype", [torch.float32, torch.float16])
def test_fused_rollout_writes(obs_dtype):
    """hg_rollout_act / hg_rollout_env == the reference PPO.act + process_env_step +
    add_transitions arithmetic (ppo.py:116-138, rollout_storage.py:83-100): same mu / sigma /
    value / obs rows, log-prob of the drawn action by the Normal formula, N(0,1) noise
    statistics, time-out bootstrap and dones."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    torch.manual_seed(2)
    n = 4096
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     init_noise_std=0.7)
    ppo = PPO(ac, device="cuda:0", gamma=0.994)
    ppo.defer_values = False
    ppo.init_storage(n, 4, [705], [219], [12], obs_dtype=obs_dtype)
    obs, cobs = torch.randn(n, 705, device="cuda:0"), torch.randn(n, 219, device="cuda:0")
    with torch.inference_mode():
        a = ppo.act(obs, cobs)
        mean, val = ac._mlp(ac.actor, obs), ac._mlp(ac.critic, cobs)  # the policy forward the rollout runs
    st = ppo.storage
    assert ppo.transition.fused_slot == 0
    torch.testing.assert_close(st.mu[0], mean, rtol=0, atol=0)
    torch.testing.assert_close(st.values[0], val, rtol=0, atol=0)
    torch.testing.assert_close(st.sigma[0], ac.std.detach().expand_as(mean), rtol=0, atol=0)
    torch.testing.assert_close(st.observations[0], obs.to(obs_dtype), rtol=0, atol=0)
    torch.testing.assert_close(st.privileged_observations[0], cobs.to(obs_dtype), rtol=0, atol=0)
    scale = ac.std.detach().expand_as(mean)
    ref_lp = (-((a - mean) ** 2) / (2 * scale ** 2) - scale.log() - np.log(np.sqrt(2 * np.pi))).sum(-1)
    torch.testing.assert_close(st.actions_log_prob[0, :, 0], ref_lp, rtol=1e-5, atol=1e-4)
    z = ((a - mean) / scale).double()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    rew = torch.randn(n, device="cuda:0")
    dones = (torch.rand(n, device="cuda:0") < 0.1).to(torch.uint8)
    to = (torch.rand(n, device="cuda:0") < 0.5).to(torch.uint8)
    ppo.process_env_step(rew, dones, {"time_outs": to})
    assert st.step == 1
    ref_r = rew + 0.994 * torch.squeeze(val * to.unsqueeze(1), 1)
    torch.testing.assert_close(st.rewards[0, :, 0], ref_r, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(st.dones[0, :, 0], dones, rtol=0, atol=0)


def test_fused_head_matches_two_launches():
    """hg_rollout_act_head (the actor's 12 x 128 output layer inside the sampling launch) writes
    bitwise the actions, log-probs, mu, sigma and observation rows of the two-launch form
    (hg_linear_skinny_forward, then hg_rollout_act) on the same seed and counter, on a strided
    observation view like the env's history windows."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from humanoid.algo.ppo import ppo as ppo_mod
    torch.manual_seed(3)
    n = 4096
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     init_noise_std=0.8)
    big = torch.randn(n, 705 + 47, device="cuda:0")
    obs, cobs = big[:, 47:], torch.randn(n, 219, device="cuda:0")  # row stride 752
    out = {}
    try:
        for fused in (False, True):
            ppo_mod.HEAD_FUSED = fused
            ppo = PPO(ac, device="cuda:0")
            ppo._rollout_seed = 12345  # the same action noise in both runs
            ppo.init_storage(n, 2, [705], [219], [12])
            with torch.inference_mode():
                ppo.act(obs, cobs)
            st = ppo.storage
            out[fused] = {k: getattr(st, k)[0].clone() for k in
                          ("actions", "actions_log_prob", "mu", "sigma", "observations", "privileged_observations")}
    finally:
        ppo_mod.HEAD_FUSED = True
    for k in out[True]:
        assert torch.equal(out[True][k], out[False][k]), k
    with torch.inference_mode():
        torch.testing.assert_close(out[True]["mu"], ac.actor(obs), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n", [4096, 1000])
def test_fused_tail_matches_head_and_two_launches(n):
    """hg_rollout_act_tail (the actor's last hidden layer 256 -> 128 + ELU and its 12 x 128 output
    layer inside the sampling launch) writes bitwise what the head-only fused launch
    (linear_act, then hg_rollout_act_head) and the two-launch form write, at the bench's row count
    and at a ragged one (a partial 16-row block)."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO, hg_mlp
    from humanoid.algo.ppo import ppo as ppo_mod
    torch.manual_seed(7)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     init_noise_std=0.8).to("cuda:0")
    big = torch.randn(n, 705 + 47, device="cuda:0")
    obs, cobs = big[:, 47:], torch.randn(n, 219, device="cuda:0")
    with torch.inference_mode():
        assert hg_mlp.mlp_infer_tail(ac.actor, obs) is not None  # the tail route is the one taken
        assert hg_mlp.mlp_infer_tail(ac.actor, obs.cpu()) is None  # never a host tensor's address
    out = {}
    try:
        for mode in ("two", "head", "tail"):
            ppo_mod.HEAD_FUSED = mode != "two"
            hg_mlp.TAIL_FUSED = mode == "tail"
            ppo = PPO(ac, device="cuda:0")
            ppo._rollout_seed = 777
            ppo.init_storage(n, 2, [705], [219], [12])
            with torch.inference_mode():
                ppo.act(obs, cobs)
            st = ppo.storage
            out[mode] = {k: getattr(st, k)[0].clone() for k in
                         ("actions", "actions_log_prob", "mu", "sigma", "observations", "privileged_observations")}
    finally:
        ppo_mod.HEAD_FUSED = True
        hg_mlp.TAIL_FUSED = True
    for mode in ("head", "tail"):
        for k in out[mode]:
            assert torch.equal(out[mode][k], out["two"][k]), (mode, k)
    with torch.inference_mode():
        torch.testing.assert_close(out["tail"]["mu"], ac.actor(obs), rtol=1e-5, atol=1e-5)


def test_rollout_sink_matches_the_env_launch():
    """With the rollout sink (the env's post launch writes the storage slot's rewards, dones and
    time-outs: hg_set_rollout_sink) a collection leaves bit-for-bit the storage the separate
    hg_rollout_env launch leaves, on short episodes (resets and time-outs within the rollout); and
    the slot equals the env's own step outputs."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from humanoid.algo.ppo import ppo as ppo_mod
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    T, n = 12, 128
    out = {}
    try:
        for mode in (False, True):
            ppo_mod.ROLLOUT_SINK = mode
            cfg = XBotLCfg()
            cfg.env.num_envs = n
            cfg.env.episode_length_s = 0.05  # 5 policy steps: time-outs inside the rollout
            cfg.seed = 3
            env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
            torch.manual_seed(4)
            ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                             init_noise_std=1.0)
            ppo = PPO(ac, device="cuda:0")
            ppo._rollout_seed = 99
            ppo.init_storage(n, T, [705], [219], [12])
            obs, cobs = env.get_observations(), env.get_privileged_observations()
            used = 0
            with torch.inference_mode():
                for _ in range(T):
                    a = ppo.act(obs, cobs)
                    sink = ppo.rollout_sink()
                    assert (sink is not None) == mode
                    if sink is not None:
                        env.set_rollout_sink(*sink)
                    obs, cobs, rew, dones, infos = env.step(a)
                    used += "rollout_sink" in infos
                    ppo.process_env_step(rew, dones, infos)
                    k = ppo.storage.step - 1
                    st = ppo.storage
                    assert torch.equal(st.rewards[k, :, 0], rew) and torch.equal(st.dones[k, :, 0], dones.to(torch.uint8))
                    assert torch.equal(st.time_outs[k, :, 0], infos["time_outs"].to(torch.uint8))
            assert used == (T if mode else 0)
            st = ppo.storage
            out[mode] = (st.rewards.clone(), st.dones.clone(), st.time_outs.clone())
            assert st.time_outs.any() and st.dones.any()
    finally:
        ppo_mod.ROLLOUT_SINK = True
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)


def test_set_root_state_and_env_props(env):
    """hg_set_root_state (all envs, clears contact warm-starts) and hg_set_env_props (DR
    friction / base mass) through the C ABI."""
    import ctypes as C
    from humanoid import _native as N
    L, s = N.lib(), C.c_void_p(torch.cuda.current_stream().cuda_stream)
    root = torch.randn(env.num_envs, 13, device="cuda:0")
    N.check(L.hg_set_root_state(env.sim, C.c_void_p(root.data_ptr()), s), env.sim)
    fr = torch.rand(env.num_envs, device="cuda:0") + 0.1
    ms = torch.rand(env.num_envs, device="cuda:0") + 30.0
    N.check(L.hg_set_env_props(env.sim, C.c_void_p(fr.data_ptr()), C.c_void_p(ms.data_ptr()), s), env.sim)
    torch.cuda.synchronize()
    torch.testing.assert_close(env.root_states, root, rtol=0, atol=0)
    torch.testing.assert_close(env.env_frictions.reshape(-1), fr, rtol=0, atol=0)
    torch.testing.assert_close(env.body_mass.reshape(-1), ms, rtol=0, atol=0)
    lam = env._view(N.T["CONTACT_LAMBDA"])
    assert (lam[:, :48] == 0).all()


def test_deferred_value_pass_matches_per_step():
    """Values of the rollout computed in one batched critic pass at compute_returns (with the
    time-out bootstrap applied there) == per-step values and bootstrap in process_env_step."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    torch.manual_seed(4)
    n, T = 1024, 6
    init = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128]).state_dict()
    g = torch.Generator(device="cpu").manual_seed(9)
    steps = [(torch.randn(n, 705, generator=g), torch.randn(n, 219, generator=g), torch.randn(n, generator=g),
              (torch.rand(n, generator=g) < 0.1).to(torch.uint8), (torch.rand(n, generator=g) < 0.3).to(torch.uint8))
             for _ in range(T + 1)]
    res = []
    for defer in (False, True):
        ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128])
        ac.load_state_dict(init)
        ppo = PPO(ac, device="cuda:0", gamma=0.994, lam=0.9)
        ppo.defer_values = defer
        ppo.init_storage(n, T, [705], [219], [12])
        with torch.inference_mode():
            for t in range(T):
                o, c, r, d, to = (x.cuda() for x in steps[t])
                ppo.act(o, c)
                ppo.process_env_step(r, d, {"time_outs": to})
            assert ppo.storage.values_deferred == defer
            ppo.compute_returns(steps[T][1].cuda())
        st = ppo.storage
        res.append({k: getattr(st, k).detach().cpu().clone() for k in ("values", "rewards", "returns", "advantages")})
    for k in res[0]:
        torch.testing.assert_close(res[1][k], res[0][k], rtol=1e-5, atol=1e-5, msg=k)


def test_initial_state_parity():
    """hg_create + the construction-time masked reset of every env (k_init + hg_reset_masked at
    step 0) vs pipeline_ref.initial_state: root/dof state, commands, first observation stacks."""
    _need_gpu()
    import pipeline_ref as PR
    env = _make_env(N_ENVS)
    g = lambda t: t.detach().cpu().numpy()  # noqa: E731
    S, obs, priv = PR.initial_state(_oracle_cfg(env), g(env.env_origins), g(env.body_mass)[:, 0],
                                    g(env.env_frictions)[:, 0])
    np.testing.assert_allclose(g(env.root_states), S["root_states"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(g(env.dof_pos), S["dof_pos"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(g(env.commands), S["commands"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(g(env.obs_buf), obs, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(g(env.privileged_obs_buf), priv, rtol=1e-4, atol=1e-4)


def test_reset_idx_and_indexed_writes():
    """reset_idx(env_ids) (hg_reset_masked) resets exactly those envs as the oracle's reset_envs
    (humanoid_env.py:1109-1163) and leaves the others untouched; hg_set_dof_state_indexed /
    hg_set_root_state_indexed write only the listed envs and clear their warm-starts."""
    _need_gpu()
    import copy
    import ctypes as C
    import pipeline_ref as PR
    from humanoid import _native as N
    env = _make_env(N_ENVS)
    for _ in range(4):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    torch.cuda.synchronize()
    S, _, _ = snapshot(env)
    g = lambda t: t.detach().cpu().numpy()  # noqa: E731
    S["projected_gravity"] = g(env.projected_gravity)
    ids = np.array([1, 5, 9, 33])
    R = copy.deepcopy(S)
    PR.reset_envs(_oracle_cfg(env), R, ids, env.common_step_counter)
    env.reset_idx(torch.tensor(ids, device="cuda:0"))
    torch.cuda.synchronize()
    keep = np.setdiff1d(np.arange(env.num_envs), ids)
    for k in ("root_states", "dof_pos", "dof_vel", "commands", "last_actions", "episode_length_buf"):
        np.testing.assert_allclose(g(getattr(env, k))[ids], R[k][ids], rtol=1e-6, atol=1e-6, err_msg=k)
        np.testing.assert_array_equal(g(getattr(env, k))[keep], S[k][keep], err_msg=k)
    assert (g(env.reset_buf)[ids] == 1).all()
    # indexed state writes
    L, s = N.lib(), C.c_void_p(torch.cuda.current_stream().cuda_stream)
    wid = torch.tensor([2, 7], dtype=torch.int32, device="cuda:0")
    q, qd = torch.randn(2, 12, device="cuda:0"), torch.randn(2, 12, device="cuda:0")
    root = torch.randn(2, 13, device="cuda:0")
    before = g(env.dof_pos).copy()
    N.check(L.hg_set_dof_state_indexed(env.sim, C.c_void_p(wid.data_ptr()), 2, C.c_void_p(q.data_ptr()),
                                       C.c_void_p(qd.data_ptr()), s), env.sim)
    N.check(L.hg_set_root_state_indexed(env.sim, C.c_void_p(wid.data_ptr()), 2, C.c_void_p(root.data_ptr()), s),
            env.sim)
    torch.cuda.synchronize()
    torch.testing.assert_close(env.dof_pos[[2, 7]], q, rtol=0, atol=0)
    torch.testing.assert_close(env.dof_vel[[2, 7]], qd, rtol=0, atol=0)
    torch.testing.assert_close(env.root_states[[2, 7]], root, rtol=0, atol=0)
    others = [i for i in range(env.num_envs) if i not in (2, 7)]
    np.testing.assert_array_equal(g(env.dof_pos)[others], before[others])
    lam = g(env._view(N.T["CONTACT_LAMBDA"]))
    assert (lam[[2, 7]] == 0).all()


@pytest.mark.parametrize("clipped_value", [True, False])
def test_fused_ppo_loss_matches_torch(clipped_value):
    """hg_ppo_loss / hg_ppo_loss_backward (hg_loss.py) == the op-by-op minibatch loss of
    ppo.py:155-210 (PPO._losses + KL expression): loss, its parts, KL mean and every parameter
    gradient, with ratios inside and on both sides of the clip band, value deltas on both sides
    of the value clip, and exact ties (torch's max/clamp backward rules)."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    from test_ppo_golden import SMALL
    torch.manual_seed(11)
    ac = ActorCritic(**SMALL).cuda()
    with torch.no_grad():
        ac.std.copy_(torch.rand(12) * 0.8 + 0.4)
    ppo = PPO(ac, clip_param=0.2, value_loss_coef=1.0, entropy_coef=0.001, use_clipped_value_loss=clipped_value,
              learning_rate=1e-3, schedule="adaptive", desired_kl=0.01, device="cuda:0")
    B = 5000
    g = torch.Generator().manual_seed(5)
    obs = torch.randn(B, 141, generator=g).cuda()
    critic = torch.randn(B, 73, generator=g).cuda()
    with torch.no_grad():
        mu0 = ac.act_inference(obs)
        v0 = ac.evaluate(critic)
    actions = (mu0 + torch.randn(B, 12, generator=g).cuda() * ac.std.detach()).contiguous()
    with torch.no_grad():
        logp_cur = _DiagGaussianLogp(mu0, ac.std, actions)
    # old log-probs: ratio exactly 1 (ties) for a third, spread inside / outside the band for the rest
    shift = torch.randn(B, generator=g).cuda() * 0.4
    shift[: B // 3] = 0.0
    old_logp = (logp_cur - shift).unsqueeze(1)
    adv = torch.randn(B, 1, generator=g).cuda()
    target_values = v0 + torch.randn(B, 1, generator=g).cuda() * 0.3
    target_values[:100] = v0[:100]  # value delta exactly 0
    returns = target_values + torch.randn(B, 1, generator=g).cuda()
    old_mu = mu0 + torch.randn(B, 12, generator=g).cuda() * 0.05
    old_sigma = ac.std.detach().expand(B, 12) * (1 + torch.rand(B, 12, generator=g).cuda() * 0.1)
    lin_vel = critic[:, 53:56]

    def run(fused):
        ppo.use_fused_loss = fused
        for p in ac.parameters():
            p.grad = None
        if fused:
            loss, stats = ppo._losses_fused(obs, critic, lin_vel, actions, target_values, adv, returns, old_logp,
                                            old_mu, old_sigma)
            parts = stats.clone()
        else:
            loss, vl, sl, lvl, _ = ppo._losses(obs, critic, lin_vel, actions, target_values, adv, returns, old_logp)
            kl = ppo._kl_mean(ac.action_mean, ac.action_std, old_mu, old_sigma)
            parts = torch.stack([vl.detach(), sl.detach(), lvl.detach(), kl])
        (loss * 0.7).backward()  # a non-unit incoming gradient exercises the backward scaling
        return loss.detach().clone(), parts, [p.grad.clone() for p in ac.parameters()]

    l_ref, p_ref, g_ref = run(False)
    l_f, p_f, g_f = run(True)
    torch.testing.assert_close(l_f, l_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p_f, p_ref, rtol=1e-5, atol=1e-6)
    bad = []
    for (name, _), a, b in zip(ac.named_parameters(), g_f, g_ref):
        if not torch.allclose(a, b, rtol=1e-4, atol=1e-6):
            bad.append(f"{name}: max|d| {(a - b).abs().max().item():.3e} max|ref| {b.abs().max().item():.3e}"
                       f" fused[:4] {a.flatten()[:4].tolist()} ref[:4] {b.flatten()[:4].tolist()}")
    assert not bad, "\n".join(bad)


def _DiagGaussianLogp(mu, std, a):
    var = std ** 2
    return (-((a - mu) ** 2) / (2 * var) - std.log() - math.log(math.sqrt(2 * math.pi))).sum(-1)


def test_fused_mlp_backward_matches_torch():
    """hg_mlp_act_backward (ELU backward + bias gradient in one pass, hg_mlp.py) == torch's
    nn.Sequential backward for the full-size actor / lin-vel / critic MLPs (actor_critic.py:36-149),
    at a row count that is not a multiple of the 128-row tile."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic
    torch.manual_seed(3)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     base_lin_vel_hidden_dims=[128, 128]).cuda()
    B = 3001
    obs = torch.randn(B, 705, device="cuda:0")
    critic = torch.randn(B, 219, device="cuda:0")
    w_mu, w_v, w_lv = (torch.randn(B, 12, device="cuda:0"), torch.randn(B, 1, device="cuda:0"),
                       torch.randn(B, 3, device="cuda:0"))

    def run(fused):
        ac.fused_mlp = fused
        for p in ac.parameters():
            p.grad = None
        x = obs.clone().requires_grad_()
        mu = ac._mlp(ac.actor, x)
        v = ac._mlp(ac.critic, critic)
        lv = ac._mlp(ac.base_lin_vel, x)
        ((mu * w_mu).sum() + (v * w_v).sum() + (lv * w_lv).sum()).backward()
        return [t.detach().clone() for t in (mu, v, lv)], [p.grad.clone() for p in ac.parameters() if p.grad is not None], x.grad.clone()

    out_t, g_t, gx_t = run(False)
    out_f, g_f, gx_f = run(True)
    for a, b in zip(out_f, out_t):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    assert len(g_f) == len(g_t)
    with torch.no_grad():  # inference path (rollout): skinny output-layer kernel
        ac.fused_mlp = True
        for net, inp in ((ac.actor, obs), (ac.critic, critic), (ac.base_lin_vel, obs)):
            torch.testing.assert_close(ac._mlp(net, inp), net(inp), rtol=1e-5, atol=1e-5)
    for (name, _), a, b in zip([(n, p) for n, p in ac.named_parameters() if n != "std"], g_f, g_t):
        torch.testing.assert_close(a, b, rtol=2e-4, atol=2e-5, msg=lambda m: f"{name}: {m}")
    torch.testing.assert_close(gx_f, gx_t, rtol=2e-4, atol=2e-5)


# bf16 policy tolerance (config 5), relative L2 error ||a - b|| / ||b|| against the fp32 torch
# reference on the same fp32 master weights: outputs and every parameter / input gradient.  bf16
# keeps 8 significant bits (unit roundoff 2^-9 = 2e-3); over the 3-4 layers the measured errors are
# (1-7)e-3 (autocast: (1-8)e-3), so the bound is BF16_REL_TOL = 1.5e-2.  And the fused path must be as accurate as torch
# autocast on the same network: error <= 1.25 x autocast's + 1e-3.
BF16_REL_TOL = 1.5e-2


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("B", [3001, 8192])
def test_bf16_mlp_matches_fp32_reference(B):
    """policy_dtype "bf16": hg_mlp.mlp_forward_bf16 (bf16 activations and matrix-core GEMMs, fused
    bf16 ELU-backward / bias pass, fp32-output weight gradients, skinny bf16-input output layer)
    against torch fp32 autograd of the same nn.Sequential (actor_critic.py:36-149), at the stated
    bf16 tolerance; 8192 rows take the split-K weight-gradient path.  Also the rollout inference
    path (no autograd)."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic
    torch.manual_seed(11)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     base_lin_vel_hidden_dims=[128, 128], policy_dtype="bf16").cuda()
    obs = torch.randn(B, 705, device="cuda:0")
    critic = torch.randn(B, 219, device="cuda:0")
    w_mu, w_v, w_lv = (torch.randn(B, 12, device="cuda:0"), torch.randn(B, 1, device="cuda:0"),
                       torch.randn(B, 3, device="cuda:0"))

    def run(mode):
        for p in ac.parameters():
            p.grad = None
        x = obs.clone().requires_grad_()
        if mode == "fp32":
            mu, v, lv = ac.actor(x), ac.critic(critic), ac.base_lin_vel(x)
        else:
            ac.fused_mlp = mode == "fused"
            mu, v, lv = ac._mlp(ac.actor, x), ac._mlp(ac.critic, critic), ac._mlp(ac.base_lin_vel, x)
            assert mu.dtype == torch.float32 and v.dtype == torch.float32
        ((mu * w_mu).sum() + (v * w_v).sum() + (lv * w_lv).sum()).backward()
        names = [n for n, p in ac.named_parameters() if p.grad is not None]
        return ([t.detach().clone() for t in (mu, v, lv)], dict(zip(names, [p.grad.clone() for n, p in
                ac.named_parameters() if p.grad is not None])), x.grad.clone())

    out_r, g_r, gx_r = run("fp32")
    out_a, g_a, gx_a = run("autocast")
    out_f, g_f, gx_f = run("fused")
    assert set(g_f) == set(g_r)
    errs = {}
    for name, a, ac_, r in [(f"out{i}", out_f[i], out_a[i], out_r[i]) for i in range(3)] + \
            [(n, g_f[n], g_a[n], g_r[n]) for n in g_r if n != "std"] + [("dx", gx_f, gx_a, gx_r)]:
        e, ea = _rel(a, r), _rel(ac_, r)
        errs[name] = (e, ea)
        assert e <= BF16_REL_TOL, f"{name}: bf16 rel err {e:.3e} > {BF16_REL_TOL}"
        assert e <= 1.25 * ea + 1e-3, f"{name}: fused bf16 rel err {e:.3e} vs autocast {ea:.3e}"
    print("bf16 rel errors (fused, autocast):", {k: (round(v[0], 5), round(v[1], 5)) for k, v in errs.items()})
    with torch.no_grad():
        ac.fused_mlp = True
        for net, inp in ((ac.actor, obs), (ac.critic, critic), (ac.base_lin_vel, obs)):
            y = ac._mlp(net, inp)
            assert _rel(y, net(inp)) <= BF16_REL_TOL
            # inference and training forward compute the same bf16 arithmetic
            with torch.enable_grad():
                torch.testing.assert_close(y, ac._mlp(net, inp).detach(), rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_gather_rows_matches_torch_indexing(dtype):
    """hg_gather_rows vs table[idx] (the reference generator's gathers, rollout_storage.py:153-191):
    bitwise, for the 705-wide observation rows (not 16-byte aligned), the 219-wide critic rows,
    a narrow per-sample table, and a ragged row count."""
    _need_gpu()
    from humanoid.algo.ppo.rollout_storage import gather_rows
    g = torch.Generator(device="cuda:0").manual_seed(3)
    R = 24 * 96
    obs = torch.randn(R, 705, device="cuda:0", generator=g).to(dtype)
    crit = torch.randn(R, 219, device="cuda:0", generator=g).to(dtype)
    pk = torch.randn(R, 40, device="cuda:0", generator=g)
    for rows in (R // 4, 1, 333):
        idx = torch.randperm(R, device="cuda:0", generator=g)[:rows]
        d0, d1, d2 = (torch.empty(rows, t.shape[1], dtype=t.dtype, device="cuda:0") for t in (obs, crit, pk))
        gather_rows(idx, [(obs, d0), (crit, d1), (pk, d2)])
        torch.cuda.synchronize()
        assert torch.equal(d0, obs[idx]) and torch.equal(d1, crit[idx]) and torch.equal(d2, pk[idx])
    with pytest.raises(RuntimeError):
        gather_rows(idx, [(obs, torch.empty(rows, 705, dtype=torch.float64, device="cuda:0"))])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_gather_rows_to_bf16(dtype):
    """hg_gather_rows_ex with a bfloat16 destination (the bf16 policy's minibatch inputs): the
    gathered rows equal torch's table[idx].to(bfloat16) bitwise (round-to-nearest-even), an fp32
    table in the same launch is copied unchanged."""
    _need_gpu()
    from humanoid.algo.ppo.rollout_storage import gather_rows
    g = torch.Generator(device="cuda:0").manual_seed(4)
    R = 24 * 96
    obs = (torch.randn(R, 705, device="cuda:0", generator=g) * 7).to(dtype)
    crit = (torch.randn(R, 219, device="cuda:0", generator=g) * 1e-3).to(dtype)
    pk = torch.randn(R, 43, device="cuda:0", generator=g)
    for rows in (R // 4, 1, 333):
        idx = torch.randperm(R, device="cuda:0", generator=g)[:rows]
        d0 = torch.empty(rows, 705, dtype=torch.bfloat16, device="cuda:0")
        d1 = torch.empty(rows, 219, dtype=torch.bfloat16, device="cuda:0")
        d2 = torch.empty(rows, 43, device="cuda:0")
        gather_rows(idx, [(obs, d0), (crit, d1), (pk, d2)])
        torch.cuda.synchronize()
        assert torch.equal(d0, obs[idx].to(torch.bfloat16)) and torch.equal(d1, crit[idx].to(torch.bfloat16))
        assert torch.equal(d2, pk[idx])
    with pytest.raises(RuntimeError):  # bf16 -> fp16 is not a supported conversion
        gather_rows(idx, [(d0, torch.empty(rows, 705, dtype=torch.float16, device="cuda:0"))])


def test_deferred_mlp_reductions_match():
    """The batched end-of-backward column sums (hg_colsum_jobs) at the 24576-row minibatch, where
    the weight gradients run split-K: bias gradients bitwise those of the per-layer reductions,
    weight gradients equal to the per-layer chunk sums up to summation order, and both within
    tolerance of torch's nn.Sequential backward."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic
    from humanoid.algo.ppo import hg_mlp
    torch.manual_seed(4)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                     base_lin_vel_hidden_dims=[128, 128]).cuda()
    B = 24576
    obs = torch.randn(B, 705, device="cuda:0")
    critic = torch.randn(B, 219, device="cuda:0")
    w_mu, w_v, w_lv = (torch.randn(B, 12, device="cuda:0"), torch.randn(B, 1, device="cuda:0"),
                       torch.randn(B, 3, device="cuda:0"))

    def run(fused, defer):
        ac.fused_mlp = fused
        hg_mlp.DEFER_REDUCTIONS = defer
        for p in ac.parameters():
            p.grad = None
        mu = ac._mlp(ac.actor, obs)
        v = ac._mlp(ac.critic, critic)
        lv = ac._mlp(ac.base_lin_vel, obs)
        ((mu * w_mu).sum() + (v * w_v).sum() + (lv * w_lv).sum()).backward()
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in ac.named_parameters() if p.grad is not None}

    try:
        g_t = run(False, False)
        g_i = run(True, False)
        g_d = run(True, True)
    finally:
        hg_mlp.DEFER_REDUCTIONS = True
    assert g_d.keys() == g_i.keys() == g_t.keys()
    # the deferred path routes the weight gradients in hg_mlp._GEMM_DW to the bf16-split k_wgrad_tr
    # (its split-K slices need the batched column sums), the immediate path keeps hipBLASLt: those
    # two differ by the split's error (<= 4e-8 of sum |gh||x| per element, tests/test_gpu_gemm.py)
    # on top of the summation order, so they are held to a relative Frobenius bound instead
    tr_routed = {n for n, p in ac.named_parameters() if tuple(p.shape) in hg_mlp._GEMM_DW}
    for n in g_d:
        if n.endswith("bias"):
            assert torch.equal(g_d[n], g_i[n]), n
        elif n in tr_routed:
            rel = float((g_d[n] - g_i[n]).norm() / g_i[n].norm())
            assert rel <= 2e-6, (n, rel)
            torch.testing.assert_close(g_d[n], g_i[n], rtol=1e-4, atol=1e-4, msg=lambda m: f"{n}: {m}")
        else:
            torch.testing.assert_close(g_d[n], g_i[n], rtol=1e-5, atol=1e-5, msg=lambda m: f"{n}: {m}")
        torch.testing.assert_close(g_d[n], g_t[n], rtol=2e-4, atol=2e-4, msg=lambda m: f"{n}: {m}")


def test_episode_extras_ring_snapshots():
    """extras["episode"] (reset_idx's episode reward means, humanoid_env.py:1109-1163) is a view of
    the EP_STATS snapshot ring: each step's dict holds the EP_STATS values as they were after that
    step, and stays intact while later steps run (up to the ring length)."""
    _need_gpu()
    env = _make_env(N_ENVS)
    snaps, dicts = [], []
    for t in range(40):
        if t % 7 == 3:  # force resets so the statistics change
            env.reset_buf[: N_ENVS // 4] = True
            env.reset_idx(torch.arange(N_ENVS // 4, device="cuda:0"))
        env.step(torch.randn(N_ENVS, 12, device="cuda:0") * 0.3)
        torch.cuda.synchronize()
        snaps.append(env._ep_stats.clone())
        dicts.append(env.extras["episode"])
    from humanoid.envs.custom.humanoid_env import REWARD_NAMES
    for t, (snap, d) in enumerate(zip(snaps, dicts)):
        for name, v in d.items():
            assert torch.equal(v, snap[REWARD_NAMES.index(name[4:])]), (t, name)
    assert any(not torch.equal(snaps[0], s) for s in snaps[1:])


def test_runner_lazy_stats_are_last_iteration():
    """OnPolicyRunner.learn without a log writer reads each iteration's phase events and loss means
    one iteration late (no host wait at the iteration boundary); after learn() the stats are
    those of the last iteration: its loss means exactly as the update accumulated them."""
    _need_gpu()
    from humanoid.envs import XBotLCfgPPO  # noqa: F401  (registers humanoid_ppo)
    from humanoid.utils import get_args, task_registry
    args = get_args(["--num_envs", "64", "--headless", "--run_name", "t"])
    env, _ = task_registry.make_env("humanoid_ppo", args=args)
    _, tcfg = task_registry.get_cfgs("humanoid_ppo")
    tcfg.runner.num_steps_per_env = 8
    runner, _ = task_registry.make_alg_runner(env, args=args, train_cfg=tcfg, log_root=None)
    assert runner.log_dir is None
    runner.learn(4, init_at_random_ep_len=True)
    st = runner.last_iteration_stats
    assert st["collection_time"] > 0 and st["learn_time"] > 0
    alg = runner.alg
    v, s_, lv = (alg._sums / (alg.num_learning_epochs * alg.num_mini_batches)).tolist()
    assert (st["value_loss"], st["surrogate_loss"], st["lin_vel_loss"]) == (v, s_, lv)
    assert all(math.isfinite(x) for x in (v, s_, lv))


def test_play_script(tmp_path, monkeypatch):
    """humanoid/scripts/play.py (reference play.py:49-176) end to end: a checkpoint written by
    train's caller path under the default log root, then play() resumes it, exports the actor
    (TorchScript + ONNX), runs the policy on one env with the reference's play settings and writes
    the action / state traces (the action trace on disk is the one play() returns)."""
    _need_gpu()
    import sys
    import humanoid.scripts.play as play_mod
    from humanoid.envs import XBotLCfgPPO  # noqa: F401  (registers humanoid_ppo)
    from humanoid.utils import get_args, task_registry
    tr_mod = sys.modules["humanoid.utils.task_registry"]  # the module (humanoid.utils re-exports the registry object)
    monkeypatch.setattr(tr_mod, "LEGGED_GYM_ROOT_DIR", str(tmp_path))
    monkeypatch.setattr(play_mod, "LEGGED_GYM_ROOT_DIR", str(tmp_path))
    args = get_args(["--num_envs", "64", "--headless", "--run_name", "p"])
    env, _ = task_registry.make_env("humanoid_ppo", args=args)
    _, tcfg = task_registry.get_cfgs("humanoid_ppo")
    tcfg.runner.num_steps_per_env = 8
    runner, tcfg = task_registry.make_alg_runner(env, args=args, train_cfg=tcfg)
    runner.learn(1, init_at_random_ep_len=True)
    exp = tcfg.runner.experiment_name
    assert os.path.isdir(tmp_path / "logs" / exp)
    trained = {k: v.detach().cpu().clone() for k, v in runner.alg.actor_critic.actor.state_dict().items()}
    del runner, env
    torch.cuda.synchronize()
    actions = play_mod.play(get_args(["--task", "humanoid_ppo", "--headless"]), steps=40)
    assert actions.shape == (40, 12) and np.isfinite(actions).all()
    root = tmp_path / "logs" / exp
    for f in ("exported/policies/policy_1.pt", "exported/policies/policy.onnx", "openloop_action/openloop_action.npz",
              "openloop_action/states.npz"):
        assert (root / f).exists(), f
    st = np.load(root / "openloop_action" / "states.npz")
    assert st["dof_pos"].shape == (40, 12) and np.isfinite(st["dof_pos"]).all()
    np.testing.assert_array_equal(np.load(root / "openloop_action" / "openloop_action.npz")["action"], actions)
    # the exported actor is the trained one (play resumes the checkpoint without --resume, see play.py)
    jit = torch.jit.load(str(root / "exported" / "policies" / "policy_1.pt"))
    for k, v in trained.items():
        assert torch.equal(jit.state_dict()[k], v), k


def test_sim2sim_obs_matches_env_obs():
    """humanoid/scripts/sim2sim.py builds the policy input from the raw simulator state as the
    reference's sim2sim.py does (get_obs + the frame of sim2sim.py:186-202); on the training
    (URDF) profile with noise off, every column of that frame except the gait phase equals the
    newest frame of the env's own observation (K_post), step after step."""
    _need_gpu()
    import humanoid.scripts.sim2sim as S2S
    env = S2S.make_env("urdf", 64, duration=5.0)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    cmd = torch.tensor([[0.4, 0.1, -0.2]], device="cuda:0").repeat(64, 1)
    act = torch.zeros(64, 12, device="cuda:0")
    nso = env.cfg.env.num_single_obs
    worst = 0.0
    for k in range(30):
        env.commands[:, :3] = cmd
        act = torch.randn(64, 12, device="cuda:0", generator=g) * 0.5
        _, _, _, reset, _ = S2S.step_direct(env, act)
        env.commands[:, :3] = cmd
        frame = S2S.obs_frame(env, cmd, act, (k + 1) * env.dt)
        ours = env.obs_buf[:, -nso:]
        # envs reset by this step start over with zeroed actions in their frame (reset_idx); the
        # rest must agree.  Euler yaw: the two wraps agree except at +-pi exactly (never reached)
        keep = ~reset.bool()
        assert int(keep.sum()) >= 48
        d = (frame[keep, 2:] - ours[keep, 2:]).abs()
        worst = max(worst, float(d.max()))
        assert float(d.max()) < 2e-5, (k, int(d.max(0).values.argmax()) + 2, float(d.max()))
    assert worst < 2e-5


def test_sim2sim_mjcf_profile(tmp_path):
    """sim2sim.py end to end on the MJCF parameter profile: an exported TorchScript actor driven by
    the sim2sim loop for 1 s at three commands; the profile reached the simulator (friction 0.9,
    200 N m torque clip, 50 solver sweeps, lighter trunk, leg-joint frictionloss) and the summary /
    traces are written and finite."""
    _need_gpu()
    import json
    import humanoid.scripts.sim2sim as S2S
    from humanoid.algo.ppo import ActorCritic
    from humanoid.utils.helpers import export_policy_as_jit
    torch.manual_seed(0)
    ac = ActorCritic(705, 219, 12, [512, 256, 128], [768, 256, 128]).to("cuda:0")
    export_policy_as_jit(ac, str(tmp_path))
    env = S2S.make_env("mjcf", 8, duration=1.0)
    assert torch.allclose(env.env_frictions, torch.full_like(env.env_frictions, 0.9))
    assert float(env.body_mass[0]) == pytest.approx(env._model.mass[0] - 0.951, abs=1e-4)
    assert [env._hgcfg.torque_limit[j] for j in range(12)] == [200.0] * 12
    assert env._hgcfg.pgs_iterations == 50
    fr = [env._model.joint_friction[b] for b in range(1, 13)]
    assert fr == pytest.approx([0.01, 0.01, 0.01, 0.01, 0.05, 0.05] * 2)
    del env
    out = tmp_path / "s2s"
    summary = S2S.main(["--load_model", str(tmp_path / "policy_1.pt"), "--duration", "1", "--vx", "-0.25", "0.0",
                        "0.4", "--envs_per_command", "2", "--out", str(out)])
    js = json.load(open(out / "sim2sim.json"))
    assert js["profile"] == "mjcf" and js["pgs_iterations"] == 50 and len(js["commands"]) == 3
    # rows over the solver budget are counted (double support on the MJCF profile wants 24 contact
    # + 12 friction rows: the 0.01 N m pitch / knee friction rows of both legs are the ones dropped)
    assert isinstance(js["rows_dropped"], int) and js["rows_dropped"] >= 0
    assert js == json.loads(json.dumps(summary))
    for c in js["commands"]:
        assert np.isfinite(c["lin_vel_error"]) and np.isfinite(c["yaw_rate_error"])
    tr = np.load(out / "sim2sim_traces.npz")
    assert tr["q"].shape == (100, 12) and np.isfinite(tr["q"]).all() and np.isfinite(tr["target_q"]).all()


def test_obs_window_stacking_over_wraps():
    """The observation history windows (HG_T_OBS_BUF / HG_T_PRIV_BUF, hg_obs_head): over 60 steps
    (two wraps of the window) every new stack is the previous one shifted by a frame, zeroed for
    the envs the step reset — obs_{t+1}[:, :(F-1)W] == reset ? 0 : obs_t[:, W:] — bit for bit, for
    both tables (the deque stacking of humanoid_env.py:880-887), with resets forced."""
    _need_gpu()
    env = _make_env(N_ENVS)
    W, Wp = 47, 73
    prev_o, prev_p = env.obs_buf.clone(), env.privileged_obs_buf.clone()
    heads = set()
    for k in range(60):
        if k % 6 == 2:
            env.episode_length_buf[k % N_ENVS:k % N_ENVS + 3] = 2400  # time-out resets next step
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
        heads.add(int(env.hg.hg_obs_head(env.sim)))
        o, p = env.obs_buf, env.privileged_obs_buf
        rs = env.reset_buf.view(-1, 1)
        assert torch.equal(o[:, :-W], torch.where(rs, torch.zeros_like(prev_o[:, W:]), prev_o[:, W:])), k
        assert torch.equal(p[:, :-Wp], torch.where(rs, torch.zeros_like(prev_p[:, Wp:]), prev_p[:, Wp:])), k
        assert o.shape == (N_ENVS, 705) and p.shape == (N_ENVS, 219)
        prev_o, prev_p = o.clone(), p.clone()
    assert 0 in heads and len(heads) == int(env.hg.hg_obs_window_advance(env.sim))  # wrapped


@pytest.mark.parametrize("obs_dtype", [torch.float32, torch.float16])
def test_frame_only_storage_rebuilds_stacks(obs_dtype):
    """Frame-only rollout storage (RolloutStorage obs_frames, hg_rollout_act writing the newest
    frame, hg_gather_stacked): over a 30-step rollout of the env through PPO's fused path, with
    resets forced and a window wrap inside, the rebuilt [T, N, 705] observations equal the stacks
    the policy was given, bit for bit (in the storage dtype), and so do minibatch rows gathered
    in the storage dtype and as bfloat16."""
    _need_gpu()
    from humanoid.algo.ppo import ActorCritic, PPO
    torch.manual_seed(3)
    n, T = 256, 30
    env = _make_env(n)
    ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128]).cuda()
    ppo = PPO(ac, device="cuda:0")
    ppo.init_storage(n, T, [705], [219], [12], obs_dtype=obs_dtype, obs_frames=(15, 47))
    st = ppo.storage
    assert st.obs_frames is not None and st.obs_frames.shape == (n, T, 47)  # env-major
    obs, cobs = env.obs_buf, env.privileged_obs_buf
    rec, rec_c = [], []
    with torch.inference_mode():
        for t in range(T):
            if t % 5 == 2:
                env.episode_length_buf[7 * t % n:7 * t % n + 4] = 2400
            rec.append(obs.clone())
            rec_c.append(cobs.clone())
            a = ppo.act(obs, cobs)
            assert ppo.transition.fused_slot == t
            obs, cobs, r, d, info = env.step(a)
            ppo.process_env_step(r, d, info)
    torch.cuda.synchronize()
    want = torch.stack(rec).to(obs_dtype)
    assert bool(st.dones.any())
    assert torch.equal(st.observations, want)
    assert torch.equal(st.privileged_observations, torch.stack(rec_c).to(obs_dtype))
    idx = torch.randperm(T * n, device="cuda:0")[:1000].contiguous()
    flat = want.flatten(0, 1)
    crit = st.privileged_observations.flatten(0, 1)
    extra = torch.randn(T * n, 43, device="cuda:0")
    for dt in (obs_dtype, torch.bfloat16):
        dst = torch.empty(1000, 705, dtype=dt, device="cuda:0")
        st.gather_stacked(idx, dst)
        assert torch.equal(dst, flat[idx].to(dt)), dt
        # with the plain tables of the minibatch gathered by the same launch
        dst.zero_()
        dc, de = torch.empty(1000, 219, dtype=dt, device="cuda:0"), torch.empty(1000, 43, device="cuda:0")
        st.gather_stacked(idx, dst, [(crit, dc), (extra, de)])
        assert torch.equal(dst, flat[idx].to(dt)) and torch.equal(dc, crit[idx].to(dt)) and torch.equal(de, extra[idx])
        # with the env-major dones copy the graphed update reads
        st.prepare_gather()
        dst.zero_()
        st.gather_stacked(idx, dst, [(crit, dc)], use_prepared=True)
        assert torch.equal(dst, flat[idx].to(dt)) and torch.equal(dc, crit[idx].to(dt))


def test_kstep_fk_matches_mjcf_at_random_poses():
    """K_step's body states pinned by the reference's robot description (VERDICT r5 missing #1):
    256 fixed-base envs set to random in-limit poses through hg_set_dof_state_indexed, one K_step
    holding them (actions = q / action_scale; about 0.01 rad median drift), then every env's rigid_state against the
    independent MJCF walk (oracle/mjcf_fk.py, XBot-L.xml:394-481) at the GPU's own post-step root,
    q and qd: positions and orientations to 2e-5 (the MJCF's 6-digit quaternions + fp32), linear
    and angular velocities to 2e-5 x (1 + the env's largest |qd|) (the held poses that collide
    leave the step with tens of rad/s on some joint)."""
    _need_gpu()
    import ctypes as C
    import mjcf_fk as MF
    from humanoid import _native as N
    n = 256
    env = _make_env(n, asset__fix_base_link=True)
    js = N.load_model()[1]
    lower = np.array([js["bodies"][j + 1]["joint"]["lower"] for j in range(12)])
    upper = np.array([js["bodies"][j + 1]["joint"]["upper"] for j in range(12)])
    rng = np.random.default_rng(17)
    q = torch.tensor(lower + (upper - lower) * rng.random((n, 12)), dtype=torch.float32, device="cuda:0")
    qd = torch.zeros(n, 12, device="cuda:0")
    ids = torch.arange(n, dtype=torch.int32, device="cuda:0")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().hg_set_dof_state_indexed(env.sim, C.c_void_p(ids.data_ptr()), n, C.c_void_p(q.data_ptr()),
                                             C.c_void_p(qd.data_ptr()), s), env.sim)
    _step_only(env, (q / env.cfg.control.action_scale).contiguous(), 5)
    g = lambda t: t.detach().cpu().numpy().astype(np.float64)  # noqa: E731
    rs, root, qq, qqd = g(env.rigid_state), g(env.root_states), g(env.dof_pos), g(env.dof_vel)
    # the held poses drift where random legs interpenetrate or sit on a limit (self-collision and
    # limit rows act within the step): the FK is compared at the GPU's own post-step state anyway
    assert np.median(np.abs(qq - g(q))) < 0.05
    bodies = MF.load()
    worst = dict(pos=0.0, rot=0.0, vel=0.0, ang=0.0, max_qd=0.0)
    for e in range(n):
        o, R, v, w = MF.fk_array(bodies, root[e], qq[e], qqd[e])
        sc = 1.0 + np.abs(qqd[e]).max()  # velocities: relative to the env's fastest joint
        worst["pos"] = max(worst["pos"], np.abs(rs[e, :, 0:3] - o).max())
        worst["rot"] = max(worst["rot"], np.abs(MF.quat_xyzw_to_mat(rs[e, :, 3:7]) - R).max())
        worst["vel"] = max(worst["vel"], np.abs(rs[e, :, 7:10] - v).max() / sc)
        worst["ang"] = max(worst["ang"], np.abs(rs[e, :, 10:13] - w).max() / sc)
        worst["max_qd"] = max(worst["max_qd"], sc - 1.0)
    print("K_step rigid_state vs MJCF FK, worst over 256 envs x 13 bodies:", worst)
    assert worst["pos"] < 2e-5 and worst["rot"] < 2e-5, worst
    assert worst["vel"] < 2e-5 and worst["ang"] < 2e-5, worst


def test_config1_workload_through_the_product():
    """BASELINE config 1's workload (XBot-L plane, 4 envs, T = 24; base_task.py:54-57,
    on_policy_runner.py:93-182) through the HIP product, not the oracle port: a 2-wave K_step grid
    and a K_post block with 4 of its lanes valid, compared with the oracle on a contact step (K_step
    by the shared rule, K_post on the same state), then OnPolicyRunner.learn at 4 envs x 24 steps
    (96 samples: 24-row minibatches through every GEMM route; the first update eager, the second
    replayed from its captured graph).  The 24-row update itself is pinned against the reference's
    PPO.update in tests/test_gpu_ppo_full.py (case config1)."""
    _need_gpu()
    from humanoid.envs import XBotLCfgPPO
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.utils.helpers import class_to_dict
    env = _make_env(4)
    for _ in range(TOUCHDOWN_STEPS):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    r64 = _step_parity(env, 141)
    _assert_contact_step(env, r64)
    _post_parity(env, steps=0)
    tcfg = XBotLCfgPPO()
    tcfg.runner.num_steps_per_env = 24
    tcfg.seed = 5
    runner = OnPolicyRunner(env, class_to_dict(tcfg), log_dir=None, device="cuda:0")
    runner.learn(2, init_at_random_ep_len=True)
    st = runner.last_iteration_stats
    assert runner.alg.storage.num_transitions_per_env * env.num_envs // runner.alg.num_mini_batches == 24
    assert runner.alg._graphs is not None, "the second update should replay a captured graph"
    for k in ("value_loss", "surrogate_loss"):
        assert np.isfinite(st[k]), (k, st[k])
    assert torch.isfinite(env.obs_buf).all() and torch.isfinite(env.privileged_obs_buf).all()
    for p in runner.alg.actor_critic.parameters():
        assert torch.isfinite(p).all()


def test_wave_balancing_does_not_change_results(monkeypatch):
    """K_step's wave balancing (HG_WAVE_BALANCE, on by default: each XCD's envs re-paired by the
    previous step's constraint rows, heaviest wave and lightest on one SIMD) only changes which
    env shares a wave: 30 policy steps of 512 envs (spawn, touchdown, contact) with and without it
    give every physics field and the rewards bit for bit."""
    _need_gpu()
    from humanoid import _native as N
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("HG_WAVE_BALANCE", flag)
        env = _make_env(512)
        gen = torch.Generator(device="cuda:0").manual_seed(21)
        for _ in range(30):
            env.step(torch.randn(env.num_envs, 12, device="cuda:0", generator=gen) * 0.4)
        torch.cuda.synchronize()
        outs.append({k: getattr(env, k).detach().cpu().numpy().copy() for k in
                     ("root_states", "dof_pos", "dof_vel", "torques", "contact_forces", "rigid_state", "rew_buf")})
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_learn_is_bitwise_reproducible():
    """The whole loop (collection: K_step, K_post, K_window, the fused rollout launches; update:
    the eager first update, the captured graphs of the second, the replay of the third) is a
    deterministic function of the seeds: two OnPolicyRunner.learn(3) runs from one seed give the
    same parameters, optimizer state, env state, rollout slots and loss statistics bit for bit (no
    atomics with run-dependent order on the path; the property DESIGN §7's identical training
    curves rest on)."""
    _need_gpu()
    from humanoid.envs import XBotLCfg, XBotLCfgPPO
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.utils.helpers import SimParams, class_to_dict, set_seed
    runs = []
    for _ in range(2):
        set_seed(11)
        cfg = XBotLCfg()
        cfg.env.num_envs = 256
        cfg.seed = 11
        env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
        tcfg = XBotLCfgPPO()
        tcfg.runner.num_steps_per_env = 24
        tcfg.seed = 11
        runner = OnPolicyRunner(env, class_to_dict(tcfg), log_dir=None, device="cuda:0")
        runner.learn(3, init_at_random_ep_len=True)
        torch.cuda.synchronize()
        alg, st = runner.alg, runner.alg.storage
        assert alg._graphs is not None, "the third update should replay a captured graph"
        out = {"p%d" % i: p.detach().cpu().clone() for i, p in enumerate(alg.actor_critic.parameters())}
        for i, group in enumerate(alg.optimizer.state.values()):
            for k, v in group.items():
                if torch.is_tensor(v):
                    out["opt%d_%s" % (i, k)] = v.detach().cpu().clone()
        for k in ("root_states", "dof_pos", "dof_vel", "obs_buf", "privileged_obs_buf", "rew_buf", "episode_length_buf"):
            out[k] = getattr(env, k).detach().cpu().clone()
        for k in ("rewards", "actions", "actions_log_prob", "values", "returns", "advantages"):
            out["st_" + k] = getattr(st, k).detach().cpu().clone()
        out["stats"] = torch.tensor([float(runner.last_iteration_stats[k]) for k in ("value_loss", "surrogate_loss")],
                                    dtype=torch.float64)
        runs.append(out)
        del runner, env
        torch.cuda.synchronize()
    assert runs[0].keys() == runs[1].keys()
    for k in runs[0]:
        assert torch.isfinite(runs[0][k].double()).all(), k
        assert torch.equal(runs[0][k], runs[1][k]), k
