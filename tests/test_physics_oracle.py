"""Analytic known-answer tests for the CPU reference simulator (oracle/physics_ref.c).

PhysX is unavailable, so physics parity against the reference is unpinned; these checks pin the
oracle's mechanics to first principles instead: mass matrix symmetric positive
definite and consistent with the bodies' kinetic energy, free fall, momentum conservation in
flight, energy conservation without actuation, and static support ≈ m·g (mechanics tests run
without self-collision and joint friction: random poses interpenetrate the legs).  The collision
and friction features have their own checks: self-collision impulses are equal and opposite and
separate the legs, the ankle joint friction holds a sub-threshold load and releases a larger one,
and armature 0 with the implicit PD damping stands stably."""
import ctypes

import numpy as np
import pytest

import physics_ref as P
from humanoid import _native as N

G = 9.81


def quat_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


@pytest.fixture(scope="module")
def model():
    m, js = N.load_model(armature=0.0, joint_friction=False, self_collisions=False)
    return m, js


def make_cfg(n, gz=-9.81, kp=0.0, kd=0.0, fixed=False, pgs=6):
    c = N.HgCfg()
    c.num_envs, c.decimation, c.pgs_iterations, c.fix_base_link = n, 1, pgs, int(fixed)
    c.sim_dt, c.gravity_z, c.contact_offset, c.max_depenetration_vel = 0.001, gz, 0.01, 1.0
    c.baumgarte, c.ground_friction, c.action_scale = 0.2, 0.6, 0.25
    for j in range(12):
        c.kp[j], c.kd[j], c.torque_limit[j] = kp, kd, 1e6
    return c


def body_energy(m, js, rigid, mass0=None, gz=-9.81):
    """Kinetic and potential energy from per-body states (independent of M)."""
    ke = pe = 0.0
    for b, bd in enumerate(js["bodies"]):
        s = rigid[b]
        R = quat_R(s[3:7])
        mb = bd["mass"] if (b > 0 or mass0 is None) else mass0
        r = R @ np.array(bd["com"])
        c = s[0:3] + r
        w = s[10:13]
        vc = s[7:10] + np.cross(w, r)
        I = np.array(bd["inertia"])
        Ib = np.array([[I[0], I[3], I[4]], [I[3], I[1], I[5]], [I[4], I[5], I[2]]])
        Iw = R @ Ib @ R.T
        ke += 0.5 * mb * vc @ vc + 0.5 * w @ Iw @ w
        pe += -mb * gz * c[2]
    return ke, pe


def momentum(js, rigid):
    p = np.zeros(3)
    L = np.zeros(3)
    mtot = 0.0
    cs = []
    for b, bd in enumerate(js["bodies"]):
        s = rigid[b]
        R = quat_R(s[3:7])
        r = R @ np.array(bd["com"])
        c = s[0:3] + r
        vc = s[7:10] + np.cross(s[10:13], r)
        cs.append((bd["mass"], c, vc, R, s[10:13], bd["inertia"]))
        p += bd["mass"] * vc
        mtot += bd["mass"]
    com = sum(m * c for m, c, *_ in cs) / mtot
    for mb, c, vc, R, w, I in cs:
        Ib = np.array([[I[0], I[3], I[4]], [I[3], I[1], I[5]], [I[4], I[5], I[2]]])
        L += mb * np.cross(c - com, vc) + R @ Ib @ R.T @ w
    return p, L


def random_state(rng, n, z=2.0):
    root = np.zeros((n, 13))
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    root[:, 2] = z
    root[:, 3:7] = q
    root[:, 7:13] = rng.normal(size=(n, 6)) * 0.5
    return root, rng.uniform(-0.4, 0.4, (n, 12)), rng.normal(size=(n, 12))


def test_mass_matrix_spd(model):
    m, js = model
    rng = np.random.default_rng(0)
    root, q, qd = random_state(rng, 5)
    for e in range(5):
        M, h = P.dynamics(m, root[e], q[e], qd[e])
        assert np.abs(M - M.T).max() < 1e-12
        assert np.linalg.eigvalsh(M).min() > 0
        np.testing.assert_allclose(M[0, 0], js["total_mass"], rtol=1e-6)   # base linear block = m I


def test_kinetic_energy_matches_bodies(model):
    """0.5 nu^T M nu equals the sum of body kinetic energies computed from the rigid states."""
    m, js = model
    rng = np.random.default_rng(1)
    n = 4
    cfg = make_cfg(n, gz=0.0)
    cfg.sim_dt = 1e-9   # effectively freeze the state; rigid states reflect the initial state
    sim = P.RefSim(cfg, m, n)
    root, q, qd = random_state(rng, n, z=5.0)
    sim.root[:], sim.q[:], sim.qd[:] = root, q, qd
    sim.step(np.zeros((n, 12)))
    for e in range(n):
        M, _ = P.dynamics(m, sim.root[e], sim.q[e], sim.qd[e], gz=0.0)
        nu = np.concatenate([sim.root[e, 7:13], sim.qd[e]])
        ke, _ = body_energy(m, js, sim.rigid[e])
        np.testing.assert_allclose(0.5 * nu @ M @ nu, ke, rtol=1e-7)


def test_free_fall(model):
    m, js = model
    n = 2
    cfg = make_cfg(n)
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 10.0
    for k in range(100):
        sim.step(np.zeros((n, 12)))
    t = 100 * 0.001
    np.testing.assert_allclose(sim.root[:, 9], -G * t, rtol=1e-6)  # g is a float32 config value
    np.testing.assert_allclose(sim.root[:, 2], 10.0 - G * 0.001 ** 2 * 100 * 101 / 2, rtol=1e-7)
    assert np.abs(sim.q).max() < 1e-9 and np.abs(sim.root[:, 10:13]).max() < 1e-9


def test_momentum_conservation_in_flight(model):
    m, js = model
    rng = np.random.default_rng(2)
    n = 4
    cfg = make_cfg(n, gz=0.0)
    sim = P.RefSim(cfg, m, n)
    root, q, qd = random_state(rng, n, z=10.0)
    sim.root[:], sim.q[:], sim.qd[:] = root, q, qd * 0.5
    sim.step(np.zeros((n, 12)))
    p0 = [momentum(js, sim.rigid[e]) for e in range(n)]
    for _ in range(200):
        sim.step(np.zeros((n, 12)))
    for e in range(n):
        p1, L1 = momentum(js, sim.rigid[e])
        np.testing.assert_allclose(p1, p0[e][0], rtol=1e-3, atol=1e-3)   # no external force; O(dt) integrator drift
        np.testing.assert_allclose(L1, p0[e][1], rtol=5e-3, atol=5e-3)   # semi-implicit Euler drift


def test_energy_conservation_fixed_base(model):
    """Unactuated fixed-base swing under gravity with joint limits removed (no constraint
    impulses): total energy is conserved up to the integrator's O(dt) error."""
    m, js = model
    free = N.HgModel.from_buffer_copy(m)
    for b in range(1, 13):
        free.lower[b], free.upper[b] = -100.0, 100.0
    rng = np.random.default_rng(3)
    n = 3
    cfg = make_cfg(n, fixed=True)
    sim = P.RefSim(cfg, free, n)
    sim.root[:, 2] = 3.0
    sim.q[:] = rng.uniform(-0.5, 0.5, (n, 12))
    sim.step(np.zeros((n, 12)))
    e0 = np.array([sum(body_energy(m, js, sim.rigid[e])) for e in range(n)])
    swing = np.zeros(n)
    for _ in range(500):
        sim.step(np.zeros((n, 12)))
        for e in range(n):
            swing[e] = max(swing[e], body_energy(m, js, sim.rigid[e])[0])
    e1 = np.array([sum(body_energy(m, js, sim.rigid[e])) for e in range(n)])
    assert (swing > 0.5).all()                      # it really swings
    assert (np.abs(e1 - e0) < 0.03 * swing).all(), (e1 - e0, swing)   # semi-implicit Euler: bounded O(dt) error


def test_static_support_equals_weight():
    m, js = N.load_model()   # the product model: armature 0 (implicit PD damping), friction, self-collision
    n = 2
    cfg = make_cfg(n, kp=0.0)
    for j in range(12):
        cfg.kp[j] = [200, 200, 350, 350, 15, 15][j % 6]
        cfg.kd[j] = 10.0
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 0.90
    sim.fric[:] = 1.0
    for _ in range(300):
        sim.step(np.zeros((n, 12)))
    fz = sim.contact[:, 6, 2] + sim.contact[:, 12, 2] + sim.contact[:, 0, 2]
    np.testing.assert_allclose(fz, js["total_mass"] * G, rtol=0.05)
    sole_z = sim.rigid[:, 6, 2]
    assert (sole_z > 0.03).all()          # no deep penetration (sole is 0.056 below the foot frame)


def _capsule_world(js, rigid, c):
    s = rigid[c["body"]]
    R = quat_R(s[3:7])
    return s[:3] + R @ np.array(c["p0"]), s[:3] + R @ np.array(c["p1"])


def test_self_collision_separates_legs():
    """Legs rolled into each other (fixed base in the air): the pair rows produce equal and
    opposite net forces on the touching left/right bodies and push them apart over a few steps."""
    m, js = N.load_model()
    n = 1
    cfg = make_cfg(n, fixed=True)
    for j in range(12):
        cfg.kp[j], cfg.kd[j] = [200, 200, 350, 350, 15, 15][j % 6], 10.0
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 3.0
    sim.q[0, 0], sim.q[0, 6] = -0.12, 0.12      # shins (bodies 4, 10) overlap by ~2 cm
    act = np.zeros((n, 12))
    act[0, 0], act[0, 6] = -0.12 / 0.25, 0.12 / 0.25   # PD target holds the pose: only the contact separates
    cfg.decimation = 1
    sim.step(act)
    f = sim.contact[0]
    left = f[1:7].sum(0)
    right = f[7:13].sum(0)
    assert np.abs(left).max() > 10.0                      # a real contact force
    np.testing.assert_allclose(left, -right, atol=1e-6 * np.abs(left).max())
    caps = js["capsules"]
    a0, a1 = _capsule_world(js, sim.rigid[0], caps[1])    # left shin
    b0, b1 = _capsule_world(js, sim.rigid[0], caps[4])    # right shin
    gap0 = np.linalg.norm(0.5 * (a0 + a1) - 0.5 * (b0 + b1))
    for _ in range(50):
        sim.step(act)
    a0, a1 = _capsule_world(js, sim.rigid[0], caps[1])
    b0, b1 = _capsule_world(js, sim.rigid[0], caps[4])
    assert np.linalg.norm(0.5 * (a0 + a1) - 0.5 * (b0 + b1)) > gap0 + 5e-3
    assert sim.nonfinite[0] == 0


def test_ankle_joint_friction_holds_and_slips():
    """The 0.1 N m ankle friction (XBot-L.urdf:1675-1677): a 0.05 N m torque on a fixed-base,
    unactuated ankle is held (joint velocity stays 0), a 0.5 N m torque turns it."""
    m, js = N.load_model()
    n = 2
    cfg = make_cfg(n, fixed=True, gz=0.0)
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 3.0
    # kp-only PD as a constant torque source: tau = kp * (a * 0.25 - q) with q ~ 0
    for j in range(12):
        cfg.kp[j], cfg.kd[j] = 0.0, 0.0
    cfg.kp[5] = 1.0
    act = np.zeros((n, 12))
    act[0, 5] = 0.05 / 0.25
    act[1, 5] = 0.5 / 0.25
    cfg.decimation = 1
    for _ in range(20):
        sim.step(act)
    assert abs(sim.qd[0, 5]) < 1e-9 and abs(sim.q[0, 5]) < 1e-9
    assert sim.qd[1, 5] > 0.1


def test_armature_zero_stands_stably():
    """Armature 0 (the asset's value) with kd = 10 on the foot at dt = 1 ms: the explicit damping
    term alone would be unstable on the 1e-3 kg m^2 foot; integrated implicitly it settles."""
    m, js = N.load_model()
    assert m.armature[6] == 0.0
    n = 1
    cfg = make_cfg(n, kp=0.0)
    cfg.decimation = 10
    for j in range(12):
        cfg.kp[j] = [200, 200, 350, 350, 15, 15][j % 6]
        cfg.kd[j] = 10.0
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 0.90
    sim.qd[0, 5] = 5.0   # kick the left ankle roll
    for _ in range(100):
        sim.step(np.zeros((n, 12)))
    assert sim.nonfinite[0] == 0
    assert np.abs(sim.qd).max() < 0.2


LAM_PAIR = N.HG_MAX_CONTACTS * 3
LAM_LIM = LAM_PAIR + N.HG_MAX_PAIRS * 3
LAM_FRIC = LAM_LIM + N.HG_MAX_DOF


def test_hand_thigh_contact_stops_hip_roll():
    """Base-link shapes vs the legs (self-collision, humanoid_config.py:103): with the base fixed in
    the air and the hip-roll PD target at 0.6 rad outward, each thigh swings into its hand capsule
    (merged into base_link, XBot-L.urdf:728-742, :2979-2993) and stops there (0.2-0.36 rad); the pair
    impulse is positive and its forces on the base and the thigh are equal and opposite."""
    m, js = N.load_model()
    caps, pairs = js["capsules"], js["pairs"]
    hand_thigh = {caps[a]["side"]: p for p, (a, b) in enumerate(pairs)
                  if caps[a]["part"] == "hand" and caps[b]["part"] == "leg_pitch"}
    n = 2
    cfg = make_cfg(n, fixed=True)
    for j in range(12):
        cfg.kp[j], cfg.kd[j] = [200, 200, 350, 350, 15, 15][j % 6], 10.0
    cfg.decimation = 10
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 3.0
    act = np.zeros((n, 12))
    act[0, 0] = 0.6 / 0.25     # left hip roll outward (+)
    act[1, 6] = -0.6 / 0.25    # right hip roll outward (-)
    for _ in range(30):
        sim.step(act)
    assert abs(sim.q[0, 0]) < 0.36 and abs(sim.q[1, 6]) < 0.36
    assert abs(sim.q[0, 0]) > 0.2 and abs(sim.q[1, 6]) > 0.2
    for e, side, thigh in ((0, "left", 3), (1, "right", 9)):
        p = hand_thigh[side]
        assert sim.lam[e, LAM_PAIR + 3 * p] > 0.0, side
        f = sim.contact[e]
        assert np.linalg.norm(f[thigh]) > 50.0
        np.testing.assert_allclose(f[0], -f[thigh], atol=1e-6 * np.abs(f[thigh]).max())
    assert (sim.dropped == 0).all() and (sim.nonfinite == 0).all()


def test_row_budget_keeps_joint_limits_before_friction():
    """Row budget (32 rows: <= 9 contact points = 27 rows, then joint limits, then the joint
    friction rows).  The robot stands on both soles (8 points = 24 rows) with friction
    on all 12 joints (the MJCF profile's frictionloss) and both hip-yaw joints 0.01 rad past their
    lower limit: 24 + 2 limit rows + 12 friction rows = 38 wanted, so 6 rows are dropped per
    substep, never a joint limit, and they are the friction rows of smallest bound taken from both
    legs alike: the 0.05 N m ankle rows and the hip-roll rows are kept, the 0.01 N m hip-yaw /
    hip-pitch / knee rows of BOTH legs are dropped (warm-start slots cleared).  (Limits after
    friction in joint order, round 2, dropped both limits and the whole right leg's friction.)"""
    m, js = N.load_model(joint_friction={"joint": 0.01, "ankle": 0.05})
    n = 1
    cfg = make_cfg(n)
    for j in range(12):
        cfg.kp[j], cfg.kd[j] = [200, 200, 350, 350, 15, 15][j % 6], 10.0
    cfg.decimation = 10
    sim = P.RefSim(cfg, m, n)
    sim.root[:, 2] = 0.87
    for _ in range(80):                      # settle on both feet
        sim.step(np.zeros((n, 12)))
    assert sim.dropped[0] > 0                # 24 + 12 friction rows: the budget already overflows
    lo = np.array([m.lower[b] for b in range(1, 13)])
    sim.q[0, [1, 7]] = lo[[1, 7]] - 0.01     # hip yaw past its limit: the foot turns about z, the
    act = np.zeros((n, 12))                  # soles stay on the ground
    act[0, [1, 7]] = (lo[[1, 7]] - 0.01) / 0.25
    cfg.decimation = 1
    before = int(sim.dropped[0])
    sim.step(act)
    assert int(sim.dropped[0]) - before == 6
    fr = sim.lam[0, LAM_FRIC:LAM_FRIC + 12]
    assert (fr[[4, 10, 5, 11, 0, 6]] != 0).all() and (fr[[1, 7, 2, 8, 3, 9]] == 0).all()
    assert sim.nonfinite[0] == 0
