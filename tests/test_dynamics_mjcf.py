"""The simulator's equations of motion pinned by the reference's robot description.

physics_ref.c — the oracle K_step is held to by every GPU parity test — builds the joint-space
inertia M by the composite-rigid-body algorithm and the bias force h (Coriolis, centrifugal,
gravity) by recursive Newton-Euler, over the compiled URDF model.  oracle/mjcf_dyn.py gets the
same M and h by Kane's method over the reference's separately written MuJoCo description
(resources/robots/XBot/mjcf/XBot-L.xml via tests/golden/mjcf_xbotl.json; the trunk's mass
properties from the URDF, the documented MJCF difference of tests/test_model_mjcf.py): body
Jacobians read off an independent forward kinematics, bias accelerations by differentiating the
body velocities along the nu-dot = 0 motion.  No code and no model data of the simulator enter
it.  Agreement at random floating-base states (measured: M within 9.4e-8 and h within 2.6e-7 of their largest
entries — the MJCF's printed precision and the difference step) pins the
dynamics the build integrates; PhysX itself stays absent.
"""
import numpy as np
import pytest

import mjcf_dyn as MD
import mjcf_fk as MF
import physics_ref as P
from humanoid import _native as N

REL = 2e-6  # of the largest |entry|; measured <= 2.6e-7


@pytest.fixture(scope="module")
def setup():
    m, js = N.load_model(armature=0.0)
    b0 = js["bodies"][0]
    I = b0["inertia"]
    trunk = (b0["mass"], np.array(b0["com"]), np.array([[I[0], I[3], I[4]], [I[3], I[1], I[5]], [I[4], I[5], I[2]]]))
    bodies = MF.load()
    lower = np.array([js["bodies"][j + 1]["joint"]["lower"] for j in range(12)])
    upper = np.array([js["bodies"][j + 1]["joint"]["upper"] for j in range(12)])
    return m, bodies, MD.mass_props(bodies, trunk), lower, upper


def _state(rng, lower, upper, moving=True):
    root = np.zeros(13)
    root[0:3] = rng.standard_normal(3)
    qq = rng.standard_normal(4)
    root[3:7] = qq / np.linalg.norm(qq)
    if moving:
        root[7:13] = rng.standard_normal(6)
    q = lower + (upper - lower) * rng.random(12)
    qd = 2.0 * rng.standard_normal(12) if moving else np.zeros(12)
    return root, q, qd


@pytest.mark.parametrize("moving", [False, True])
def test_oracle_dynamics_match_mjcf_kane(setup, moving):
    """M and h of physics_ref (CRBA + RNEA, armature 0) equal Kane's method over the MJCF at 24
    random in-limit floating-base states (at rest: h is the gravity load alone)."""
    m, bodies, props, lower, upper = setup
    rng = np.random.default_rng(11 if moving else 12)
    worst = {"M": 0.0, "h": 0.0}
    for _ in range(24):
        root, q, qd = _state(rng, lower, upper, moving)
        Mk, hk = MD.dynamics(bodies, props, root, q, qd)
        Mo, ho = P.dynamics(m, root, q, qd)
        assert np.abs(Mo - Mo.T).max() < 1e-12
        worst["M"] = max(worst["M"], np.abs(Mk - Mo).max() / np.abs(Mo).max())
        worst["h"] = max(worst["h"], np.abs(hk - ho).max() / np.abs(ho).max())
    print("physics_ref vs Kane over the MJCF, worst relative to the largest entry:", worst)
    assert worst["M"] < REL and worst["h"] < REL, worst


def test_static_gravity_load(setup):
    """At rest the base force is the robot's weight (53.04 kg x 9.81 up), in both."""
    m, bodies, props, lower, upper = setup
    root, q, qd = _state(np.random.default_rng(3), lower, upper, moving=False)
    _, hk = MD.dynamics(bodies, props, root, q, qd)
    total = sum(p[0] for p in props)
    assert total == pytest.approx(53.036, abs=1e-2)
    assert hk[0:2] == pytest.approx([0.0, 0.0], abs=1e-9) and hk[2] == pytest.approx(total * 9.81, rel=1e-9)


def test_the_pin_has_teeth(setup):
    """A dynamics without the gyroscopic term w x I w, or with one leg link's mass 1 % off, is far
    outside the bound: the agreement is not an artefact of the tolerance."""
    m, bodies, props, lower, upper = setup
    root, q, qd = _state(np.random.default_rng(5), lower, upper, moving=True)
    Mo, ho = P.dynamics(m, root, q, qd)
    heavy = list(props)
    heavy[4] = (props[4][0] * 1.01, props[4][1], props[4][2])
    Mh, hh = MD.dynamics(bodies, heavy, root, q, qd)
    assert np.abs(Mh - Mo).max() / np.abs(Mo).max() > 50 * REL
    # the gyroscopic term alone: recompute h with it removed
    nu = np.concatenate([root[7:13], qd])
    Jc, Jw, _, Iw = MD._jacobians(bodies, props, root, q)
    wb = Jw @ nu
    gyro = sum(Jw[b].T @ np.cross(wb[b], Iw[b] @ wb[b]) for b in range(13))
    assert np.abs(gyro).max() / np.abs(ho).max() > 50 * REL
