"""The oracle's pipeline (oracle/pipeline_ref.py) against the REFERENCE itself, on the draws the
reference consumed (CPU).

tests/golden/gen_goldens.py ran the reference's own step() (humanoid_env.py:616-660) with
gym.simulate a no-op, at the fork's 18-DOF layout, with torch's RNG calls intercepted: the raw
uniforms / normals / integers it drew are in pipeline18.npz next to its inputs and outputs.
Running pipeline_ref.step_without_physics with ``InjectedDraws`` over the same inputs must
reproduce the reference: this pins the step prologue (:616-635), _post_physics_step_callback /
_resample_commands (:1000-1032), _push_robots (:665-681), check_termination, compute_reward,
reset_idx / _reset_dofs / _reset_root_states (:1034-1072, 1109-1163), _update_terrain_curriculum
(:1075-1095), the derived state (:784-788), the observation noise and stacking (:818-887) and the
obs clip (:654-657).  heights.npz pins _get_heights (:949-985); terrain.npz pins HumanoidTerrain's
control flow (utils/terrain.py:38-231) with the build's terrain_utils primitives.
Floats: 1e-6 (float32 reassociation of the same formulas); ints, masks and levels: exact.
"""
import types

import numpy as np
import pytest

import envlogic_ref as E
import pipeline_ref as PR

f32 = np.float32


def _cfg_ns(z, tag):
    pre = f"{tag}/cfg/"
    d = {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}
    ns = types.SimpleNamespace()
    for k, v in d.items():
        v = v.tolist() if v.ndim else v.item()
        setattr(ns, k, v)
    ns.default_dof_pos = z[f"{tag}/in/default_dof_pos"][0].tolist()
    return ns


def _state(z, tag):
    pre = f"{tag}/in/"
    S = {}
    for k in z.files:
        if k.startswith(pre) and "/sum/" not in k:
            S[k[len(pre):]] = np.array(z[k])
    S["last_contacts"] = S["last_contacts"].astype(bool)
    S["episode_sums"] = {k[len(pre) + 4:]: np.array(z[k]) for k in z.files if k.startswith(pre + "sum/")}
    return S


def _draws(z, tag, n):
    pre = f"{tag}/draw/"
    rec = {}
    for k in sorted(z.files):
        if k.startswith(pre):
            purpose, idx = k[len(pre):].rsplit("/", 1)
            rec.setdefault(purpose, []).append((int(idx), np.array(z[k])))
    rec = {p: [a for _, a in sorted(v)] for p, v in rec.items()}
    return PR.InjectedDraws(rec).bind(n)


@pytest.mark.parametrize("tag", ["plane", "curriculum"])
def test_step_pipeline_matches_reference(golden, tag):
    z = golden("pipeline18.npz")
    ns = _cfg_ns(z, tag)
    cfg = PR.Cfg(ns, L=E.LAYOUT18, default=ns.default_dof_pos)
    S = _state(z, tag)
    n = S["dof_pos"].shape[0]
    draws = _draws(z, tag, n)
    counter = int(S.pop("common_step_counter")) + 1  # post_physics_step's increment (:781)
    gains = (S.pop("p_gains"), S.pop("d_gains"), S.pop("torque_limits"), float(S.pop("action_scale")))
    hist_o, hist_p = S.pop("obs_history"), S.pop("critic_history")
    actions = S.pop("policy_actions")
    extras = {}
    obs, priv, rew, reset, timeout, _ = PR.step_without_physics(cfg, S, actions, counter, hist_o, hist_p, gains,
                                                                draws=draws, extras=extras)
    out = lambda k: z[f"{tag}/out/{k}"]  # noqa: E731
    clip = f32(ns.clip_observations)
    np.testing.assert_array_equal(reset, out("reset_buf"))
    np.testing.assert_array_equal(timeout, out("time_out_buf"))
    np.testing.assert_array_equal(S["episode_length_buf"], out("episode_length_buf"))
    assert reset.any() and timeout.any()
    close = dict(rtol=1e-6, atol=1e-6)
    for k in ("actions", "torques", "commands", "root_states", "dof_pos", "dof_vel", "rand_push_force",
              "rand_push_torque", "last_actions", "last_last_actions", "last_dof_vel", "last_root_vel",
              "feet_air_time", "feet_height", "last_feet_z", "env_origins", "base_lin_vel", "base_ang_vel",
              "projected_gravity"):
        np.testing.assert_allclose(S[k], out(k), err_msg=k, **close)
    np.testing.assert_array_equal(S["last_contacts"], out("last_contacts"))
    np.testing.assert_allclose(S["base_euler_xyz"], out("base_euler_xyz"), rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(rew, out("rew_buf"), rtol=1e-5, atol=1e-6)
    for name, v in S["episode_sums"].items():
        np.testing.assert_allclose(v, out(f"sum/{name}"), rtol=1e-5, atol=1e-6, err_msg=name)
    for name, v in extras["episode"].items():
        np.testing.assert_allclose(v, out(f"episode/rew_{name}"), rtol=1e-5, atol=1e-7, err_msg=name)
    np.testing.assert_allclose(np.clip(obs, -clip, clip), out("obs_buf"), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.clip(priv, -clip, clip), out("privileged_obs_buf"), rtol=1e-5, atol=1e-5)
    if tag == "curriculum":
        np.testing.assert_array_equal(S["terrain_levels"], out("terrain_levels"))
    for k, q in draws.q.items():
        assert not q, f"unconsumed reference draws for {k}"


def test_heights_match_reference(golden):
    z = golden("heights.npz")
    ns = types.SimpleNamespace(hf_border=float(z["border_size"]), hf_horizontal_scale=float(z["horizontal_scale"]),
                               hf_vertical_scale=float(z["vertical_scale"]))
    cfg = types.SimpleNamespace(c=ns)
    h = PR.heights(cfg, z["root_states"], z["points_xy"], z["heightfield"])
    np.testing.assert_allclose(h, z["heights"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_terrain_generator_matches_reference(golden, tag):
    """The build's HumanoidTerrain (humanoid/utils/terrain.py) on the same seed and reduced map as
    the reference's own class: identical heightfield and env origins, bit for bit."""
    import numpy as _np
    from humanoid.envs import XBotLCfg
    from humanoid.utils.terrain import HumanoidTerrain
    z = golden("terrain.npz")
    tc = XBotLCfg.terrain()
    tc.mesh_type = "heightfield"
    tc.num_rows, tc.num_cols = int(z[f"{tag}/rows"]), int(z[f"{tag}/cols"])
    tc.border_size = 2.0
    tc.curriculum = False
    np.testing.assert_array_equal(np.asarray(tc.terrain_proportions, np.float64), z["proportions"])
    saved = _np.random.get_state()
    try:
        _np.random.seed(int(z[f"{tag}/seed"]))
        t = HumanoidTerrain(tc, 64)
    finally:
        _np.random.set_state(saved)
    np.testing.assert_array_equal(t.heightsamples, z[f"{tag}/heightsamples"])
    np.testing.assert_array_equal(t.env_origins, z[f"{tag}/env_origins"])
