"""Kinematic conventions of the simulator pinned by the reference's own robot description.

tests/test_model_mjcf.py checks the compiled model TABLE (frames, axes, inertias) against the MJCF
(resources/robots/XBot/mjcf/XBot-L.xml).  This file checks what the simulator DOES with it: the
oracle's forward kinematics (physics_ref.c rigid_states, the same body states K_step writes)
against an independent numpy walk of the MJCF tree by MuJoCo's conventions (oracle/mjcf_fk.py), at
256 random poses within the joint limits and random root poses / velocities.  A joint rotated by
-q, about the wrong axis or in the wrong frame moves some body by centimetres; the MJCF's 6-digit
quaternions bound the honest disagreement at ~1e-5.

Then the reference's gait definition (humanoid_env.py:716-744, compute_ref_state: left pitch /
knee / ankle pitch -0.17 / -0.34 / -0.17 at the gait's left-swing extreme, right +0.17 / +0.34 /
+0.17 at the other) must be a swing on THIS robot: the swing foot rises by 6.21 cm and its knee
moves forward (+x of the base) by 4.46 cm, in the oracle and in the MJCF alike.
"""
import numpy as np
import pytest

import mjcf_fk as MF
import physics_ref as P
from humanoid import _native as N


@pytest.fixture(scope="module")
def setup():
    m, js = N.load_model()
    lower = np.array([js["bodies"][j + 1]["joint"]["lower"] for j in range(12)])
    upper = np.array([js["bodies"][j + 1]["joint"]["upper"] for j in range(12)])
    return m, js, MF.load(), lower, upper


def _random_states(n, lower, upper, seed):
    rng = np.random.default_rng(seed)
    q = lower + (upper - lower) * rng.random((n, 12))
    qd = rng.standard_normal((n, 12)) * 2.0
    root = np.zeros((n, 13))
    root[:, 0:3] = rng.standard_normal((n, 3))
    quat = rng.standard_normal((n, 4))
    root[:, 3:7] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
    root[:, 7:13] = rng.standard_normal((n, 6))
    return root, q, qd


def test_body_names_match_the_compiled_model(setup):
    _, js, _, _, _ = setup
    assert [b["name"] for b in js["bodies"]] == MF.BODIES


@pytest.mark.parametrize("fixed_base", [True, False])
def test_oracle_fk_matches_mjcf_at_random_poses(setup, fixed_base):
    """Every body's position, orientation, linear and angular velocity from the oracle's FK equal
    the MJCF walk at 256 random in-limit poses (fixed base: identity root at rest; floating: random
    root pose and twist) to the MJCF's printed precision."""
    m, _, bodies, lower, upper = setup
    n = 256
    root, q, qd = _random_states(n, lower, upper, seed=7 if fixed_base else 8)
    if fixed_base:
        root[:] = 0
        root[:, 2] = 0.95
        root[:, 6] = 1.0
    rs = P.rigid_states(m, root, q, qd)
    worst = dict(pos=0.0, rot=0.0, vel=0.0, ang=0.0)
    for e in range(n):
        o, R, v, w = MF.fk_array(bodies, root[e], q[e], qd[e])
        Ro = MF.quat_xyzw_to_mat(rs[e, :, 3:7])
        worst["pos"] = max(worst["pos"], np.abs(rs[e, :, 0:3] - o).max())
        worst["rot"] = max(worst["rot"], np.abs(Ro - R).max())
        worst["vel"] = max(worst["vel"], np.abs(rs[e, :, 7:10] - v).max())
        worst["ang"] = max(worst["ang"], np.abs(rs[e, :, 10:13] - w).max())
    print("oracle FK vs MJCF, worst over 256 poses x 13 bodies:", worst)
    assert worst["pos"] < 1e-5 and worst["rot"] < 1e-5, worst   # achieved 1.2e-6 / 2.3e-6
    assert worst["vel"] < 1e-4 and worst["ang"] < 1e-4, worst   # achieved 6.4e-6 / 1.7e-5


def test_a_flipped_joint_would_be_caught(setup):
    """The check has teeth: negating any one joint angle at a typical in-limit pose moves some
    body by > 1 cm or turns some body frame by > 0.1 (rotation-matrix entries; the ankle joints sit
    at their body's origin, so they show in orientation)."""
    m, _, bodies, lower, upper = setup
    root = np.zeros((1, 13))
    root[0, 6] = 1.0
    q = 0.5 * np.minimum(np.abs(lower), upper)
    o_ref, R_ref = MF.fk_array(bodies, root[0], q)[0:2]
    for j in range(12):
        qf = q.copy()
        qf[j] = -qf[j]
        rs = P.rigid_states(m, root, qf[None], np.zeros((1, 12)))[0]
        moved = np.abs(rs[:, 0:3] - o_ref).max()
        turned = np.abs(MF.quat_xyzw_to_mat(rs[:, 3:7]) - R_ref).max()
        assert moved > 0.01 or turned > 0.1, (j, moved, turned)


def _gait_pose(side):
    """compute_ref_state's extreme (humanoid_env.py:728-739 with the 12-DOF index map, SURVEY.md
    App. A): sin_pos = -1 lifts the LEFT leg (pitch, knee, ankle pitch at 2, 3, 4 get
    min(sin, 0) x (0.17, 0.34, 0.17)); sin_pos = +1 the RIGHT (8, 9, 10 get max(sin, 0) x the same)."""
    q = np.zeros(12)
    if side == "left":
        q[2], q[3], q[4] = -0.17, -0.34, -0.17
    else:
        q[8], q[9], q[10] = 0.17, 0.34, 0.17
    return q


@pytest.mark.parametrize("side", ["left", "right"])
def test_reference_gait_pose_lifts_the_swing_foot(setup, side):
    m, _, bodies, _, _ = setup
    root = np.zeros(13)
    root[2], root[6] = 0.95, 1.0
    foot, knee = (6, 4) if side == "left" else (12, 10)
    other = 12 if side == "left" else 6
    z0 = P.rigid_states(m, root, np.zeros(12), np.zeros(12))[0]
    z1 = P.rigid_states(m, root, _gait_pose(side), np.zeros(12))[0]
    o0, o1 = MF.fk_array(bodies, root, np.zeros(12))[0], MF.fk_array(bodies, root, _gait_pose(side))[0]
    lift, fwd = z1[foot, 2] - z0[foot, 2], z1[knee, 0] - z0[knee, 0]
    print(f"{side} swing: foot +{100 * lift:.2f} cm, knee +{100 * fwd:.2f} cm forward")
    assert lift == pytest.approx(0.0621, abs=5e-4) and fwd == pytest.approx(0.0446, abs=5e-4)
    assert o1[foot, 2] - o0[foot, 2] == pytest.approx(lift, abs=5e-5)
    assert o1[knee, 0] - o0[knee, 0] == pytest.approx(fwd, abs=5e-5)
    assert abs(z1[other, 2] - z0[other, 2]) < 1e-12   # the stance leg does not move
