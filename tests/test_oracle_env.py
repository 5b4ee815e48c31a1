"""The env-logic oracle (oracle/envlogic_ref.py) against golden vectors produced by the
reference's own humanoid_env.py (tests/golden/gen_goldens.py) at its native 18-DOF layout."""
import numpy as np
import pytest

import envlogic_ref as E

RTOL, ATOL = 1e-5, 1e-5


@pytest.fixture(scope="module")
def g(golden):
    return golden("env18.npz")


def state(g):
    S = {k[3:]: g[k].copy() for k in g.files if k.startswith("in/")}
    S["default_dof_pos"] = S["default_dof_pos"].astype(np.float32)
    return S


def test_torques(g):
    t = E.compute_torques(g["pd/actions"], g["pd/p_gains"], g["pd/d_gains"], g["in/default_dof_pos"],
                          g["in/dof_pos"], g["in/dof_vel"], g["pd/torque_limits"], 0.25)
    np.testing.assert_allclose(t, g["pd/torques"], rtol=1e-6, atol=1e-4)


def test_phase_gait_ref(g):
    P = E.Params()
    ep = g["in/episode_length_buf"]
    np.testing.assert_allclose(E.phase(ep, P), g["phase"], rtol=1e-6)
    _, _, st = E.gait(ep, P)
    np.testing.assert_array_equal(st, g["stance_mask"])
    ref = E.ref_state(ep, E.LAYOUT18, P)
    np.testing.assert_allclose(ref, g["ref_dof_pos"], atol=2e-6)


def test_noise_vec(g):
    np.testing.assert_allclose(E.noise_vec(E.LAYOUT18, E.Params()), g["noise_vec"], rtol=1e-7)


def test_termination(g):
    reset, to = E.termination(g["in/contact_forces"], g["in/episode_length_buf"], E.LAYOUT18, E.Params())
    np.testing.assert_array_equal(reset, g["reset_buf"])
    np.testing.assert_array_equal(to, g["time_out_buf"])


def test_rewards_term_by_term(g):
    P = E.Params()
    S = state(g)
    S["ref_dof_pos"] = g["ref_dof_pos"]
    terms = E.rewards(S, E.LAYOUT18, P)
    for name in g["reward_names"]:
        np.testing.assert_allclose(terms[str(name)], g["term/" + str(name)], rtol=RTOL, atol=ATOL, err_msg=str(name))
    # mutated state
    np.testing.assert_allclose(S["feet_air_time"], g["post/feet_air_time"], atol=1e-6)
    np.testing.assert_array_equal(S["last_contacts"], g["post/last_contacts"])
    np.testing.assert_allclose(S["feet_height"], g["post/feet_height"], atol=1e-6)
    np.testing.assert_allclose(S["last_feet_z"], g["post/last_feet_z"], atol=1e-6)
    scales = dict(zip([str(n) for n in g["reward_names"]], g["reward_scales"]))
    sums = {n: np.zeros(len(S["dof_pos"]), np.float32) for n in scales}
    rew = E.total_reward(terms, scales, sums, P)
    np.testing.assert_allclose(rew, g["rew_buf"], rtol=1e-4, atol=1e-6)
    for n in scales:
        np.testing.assert_allclose(sums[n], g["sum/" + n], rtol=1e-4, atol=1e-7)


def test_observation_stacking(g):
    P = E.Params()
    S = state(g)
    N = len(S["dof_pos"])
    hist_o = np.zeros((N, 15 * 65), np.float32)
    hist_p = np.zeros((N, 3 * 97), np.float32)
    for it in range(3):
        S["dof_pos"] = g[f"obs{it}/dof_pos"]
        S["actions"] = g[f"obs{it}/actions"]
        S["episode_length_buf"] = g[f"obs{it}/episode_length_buf"]
        o, p, _ = E.obs_frames(S, E.LAYOUT18, P, noise=None)
        hist_o = E.stack(hist_o, o)
        hist_p = E.stack(hist_p, p)
        np.testing.assert_allclose(hist_o, g[f"obs{it}/obs_buf"], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(hist_p, g[f"obs{it}/privileged_obs_buf"], rtol=1e-5, atol=2e-6)


def test_layout12_widths():
    P = E.Params()
    assert len(E.noise_vec(E.LAYOUT12, P)) == 47
