"""CPU checks of the sim2sim MJCF profile (humanoid/scripts/sim2sim.py): the configuration it
builds and the per-joint frictionloss override of the model loader.  The run itself is a GPU test
(tests/test_gpu_parity.py::test_sim2sim_mjcf_profile)."""
import numpy as np
import pytest
import torch


def test_mjcf_profile_cfg():
    import humanoid.scripts.sim2sim as S2S
    from humanoid.envs import XBotLCfg
    base = XBotLCfg()
    c = S2S.make_cfg("mjcf", 6, duration=3.0)
    assert c.sim.hg.armature == 0.01 and c.sim.hg.pgs_iterations == 50
    assert c.sim.hg.joint_friction == {"joint": 0.01, "ankle": 0.05}
    assert c.terrain.static_friction == 0.9
    assert {k: v - base.control.damping[k] for k, v in c.control.damping.items()} == pytest.approx(
        {k: 0.01 for k in base.control.damping})
    assert not c.noise.add_noise and not c.domain_rand.push_robots and c.domain_rand.dynamic_randomization == 0
    assert not c.commands.heading_command and c.commands.resampling_time > 3.0
    u = S2S.make_cfg("urdf", 6, duration=3.0)
    assert u.sim.hg.armature == base.sim.hg.armature and u.control.damping == base.control.damping
    with pytest.raises(ValueError):
        S2S.make_cfg("mujoco", 6, 1.0)


def test_joint_friction_override():
    from humanoid import _native as N
    m, js = N.load_model(joint_friction={"joint": 0.01, "ankle": 0.05})
    names = [b["joint"]["name"] for b in js["bodies"][1:]]
    got = [m.joint_friction[b] for b in range(1, 13)]
    want = [0.05 if "ankle" in n else 0.01 for n in names]
    assert got == pytest.approx(want)
    m0, _ = N.load_model()
    assert [m0.joint_friction[b] for b in range(1, 13)] == pytest.approx([0.1 if "ankle" in n else 0.0 for n in names])


def test_quat_to_euler_matches_reference_formula():
    """sim2sim.quat_to_euler restates sim2sim.py:53-76 (roll/pitch/yaw of an (x, y, z, w) quaternion)."""
    import humanoid.scripts.sim2sim as S2S
    from scipy.spatial.transform import Rotation as R
    rng = np.random.default_rng(0)
    q = rng.normal(size=(64, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    e = S2S.quat_to_euler(torch.tensor(q, dtype=torch.float64)).numpy()
    ref = R.from_quat(q).as_euler("xyz")  # extrinsic x-y-z == the script's roll, pitch, yaw
    d = np.abs(np.angle(np.exp(1j * (e - ref))))
    assert d.max() < 1e-9
    v = rng.normal(size=(64, 3))
    w = S2S.quat_rotate_inverse(torch.tensor(q), torch.tensor(v)).numpy()
    np.testing.assert_allclose(w, R.from_quat(q).inv().apply(v), atol=1e-12)
