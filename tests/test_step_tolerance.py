"""CPU tests of the K_step tolerance machinery (oracle/step_tolerance.py) on an oracle contact
state (scripts/contact_flip_rate.py: 24 policy steps from the spawn, then one compared step).

  * the f64 step itself is inside its own tolerance everywhere; an offset on one joint
    velocity of one env (twice its tolerance) is caught, in that env only;
  * on a contact step, independent fp32 builds (perturbed CPU f32 members judged against the
    yardstick that excludes them) land outside the element tolerance in a small fraction of envs:
    the discrete stick / slip and contact-offset events the GPU tests' outlier allowance is
    calibrated on — nonzero, and a small fraction;
  * dropped-row counts of those builds equal the f64 step's env for env.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))

import step_tolerance as ST  # noqa: E402


@pytest.fixture(scope="module")
def contact_step():
    import contact_flip_rate as C
    import pipeline_ref as PR
    n = 1024
    hc, model, oc, S, rng, counter = C.contact_state(n)
    a_ref = PR.preprocess_actions(oc, (0.5 * rng.standard_normal((n, 12))).astype(np.float32), S["actions"], counter)
    S["body_mass"] = S["body_mass"].reshape(-1, 1)
    S["env_frictions"] = S["env_frictions"].reshape(-1, 1)
    r64 = ST.ref_sim(hc, model, S, "f64")
    r64.step(a_ref)
    fields = ST.FIELDS
    spread = ST.f64_spread(hc, model, S, a_ref, r64, fields)
    g32 = ST.gap(ST.f32_members(hc, model, S, a_ref, fields, members=3), r64, fields)
    kp = np.array([hc.kp[j] for j in range(12)])
    kd = np.array([hc.kd[j] for j in range(12)])
    return dict(hc=hc, model=model, S=S, a_ref=a_ref, r64=r64, spread=spread, g32=g32, kp=kp, kd=kd, n=n)


def test_contact_state_is_on_the_ground(contact_step):
    r64 = contact_step["r64"]
    nc = len(contact_step["model"].contact_body)
    assert (r64.lam[:, 0:3 * nc:3] > 0).any(axis=1).mean() >= 0.95


def test_tolerance_accepts_f64_and_catches_an_offset(contact_step):
    c = contact_step
    fields = ST.FIELDS
    exact = {f: ST.outputs(c["r64"])[f].copy() for f in fields}
    bad, head, tol = ST.compare(exact, c["r64"], c["g32"], c["spread"], fields, c["kp"], c["kd"], 12.0)
    assert not ST.bad_envs(bad).any() and all(v == 0 for v in head.values())
    off = {f: v.copy() for f, v in exact.items()}
    off["qd"][17, 3] += 2 * tol["qd"][17, 3]
    bad, _, _ = ST.compare(off, c["r64"], c["g32"], c["spread"], fields, c["kp"], c["kd"], 12.0)
    assert np.flatnonzero(ST.bad_envs(bad)).tolist() == [17]


def test_fp32_builds_have_rare_contact_outliers(contact_step):
    c = contact_step
    null = ST.flip_null_rate(c["hc"], c["model"], c["S"], c["a_ref"], c["r64"], c["spread"], ST.FIELDS, c["kp"],
                             c["kd"], 12.0, candidates=3)
    frac = np.array(null["bad_envs"]) / c["n"]
    print("independent f32 builds outside the K = 12 element tolerance:", null["bad_envs"], "of", c["n"])
    assert frac.max() < 0.05          # a small fraction ...
    assert sum(null["bad_envs"]) > 0  # ... but not zero: the allowance is needed on contact steps
    assert null["dropped_mismatch_envs"] == [0, 0, 0]


def test_allowance_is_twice_the_rate_with_a_floor():
    # large checks: twice the null builds' mean; small checks: twice the 1 % floor rate
    assert ST.allowed_outliers([39, 36, 43, 36], 4096) == 82
    assert ST.allowed_outliers([0, 0, 0, 0], 64) == 2
    assert ST.allowed_outliers([0, 0, 0, 0], 4096) == 82
    assert ST.allowed_outliers([3, 0, 1, 0], 64) == 2


def test_nan_in_a_candidate_is_caught(contact_step):
    """A non-finite candidate element is outside every tolerance (|NaN - x| <= tol is False) and
    check_step names it (the old `> tol` test let a NaN through)."""
    c = contact_step
    fields = ST.FIELDS
    cand = {f: ST.outputs(c["r64"])[f].copy() for f in fields}
    cand["q"][5, 2] = np.nan
    cand["rigid"][9, 3, 4] = np.inf
    bad, head, _ = ST.compare(cand, c["r64"], c["g32"], c["spread"], fields, c["kp"], c["kd"], 12.0)
    assert np.flatnonzero(ST.bad_envs(bad)).tolist() == [5, 9]
    assert head["q"] == float("inf") and head["rigid"] == float("inf")


def test_check_step_bounds_outlier_size(contact_step):
    """check_step (the rule smoke() and the GPU parity tests share): the f64 step itself passes; an
    env pushed far outside (1 rad on one joint) fails by count or by the 4 x deviation bound even
    when the count alone would be allowed; a NaN fails as non-finite."""
    c = contact_step
    n = 64
    S = {k: np.asarray(v)[:n] for k, v in c["S"].items() if hasattr(v, "shape") and np.asarray(v).shape[:1] == (c["n"],)}
    a = c["a_ref"][:n]
    r64 = ST.ref_sim(c["hc"], c["model"], S, "f64")
    r64.step(a)
    exact = {f: ST.outputs(r64)[f].copy() for f in ST.FIELDS}
    _, rep, fails, _ = ST.check_step(c["hc"], c["model"], S, a, exact)
    assert not fails and rep["outlier_envs"] == 0
    off = {f: v.copy() for f, v in exact.items()}
    off["q"][3, 7] += 1.0
    _, rep, fails, _ = ST.check_step(c["hc"], c["model"], S, a, off)
    assert rep["outlier_envs"] >= 1 and 3 in rep["outlier_ids"] and fails
    assert any("outlier deviation" in f or "envs outside" in f for f in fails)
    nan = {f: v.copy() for f, v in exact.items()}
    nan["torques"][0, 0] = np.nan
    _, _, fails, _ = ST.check_step(c["hc"], c["model"], S, a, nan)
    assert any("non-finite" in f for f in fails)


def test_round6_smoke_outlier_is_a_cone_event():
    """The K_step outlier of round 6's smoke() dump (tests/golden/kstep_outlier_r6.npz: the GPU's
    pre-step state, actions and outputs; profiles/r6_smoke/classification.md): the shared rule
    passes it with env 54 the only outlier, and in the f64 step that env's sole contact ground6
    comes within 0.5 % of its friction cone at substep 6 (the stick / slip boundary fp32 rounding
    decides; plain and kernel-quotient f32 builds flip it alike)."""
    import classify_kstep_outlier as C
    D = np.load(os.path.join(REPO, "tests", "golden", "kstep_outlier_r6.npz"), allow_pickle=False)
    S = {k[2:]: D[k] for k in D.files if k.startswith("S_")}
    gpu = {k[4:]: D[k] for k in D.files if k.startswith("gpu_")}
    hc, model, _ = C.smoke_cfg(D["a_ref"].shape[0])
    _, rep, fails, _ = ST.check_step(hc, model, S, D["a_ref"], gpu)
    assert not fails and rep["outlier_ids"] == [54]
    e = 54
    S1 = {k: np.asarray(v)[e:e + 1] for k, v in S.items()}
    _, lams, _ = C.replay(hc, model, S1, D["a_ref"][e:e + 1], "f64")
    mu = 0.5 * (float(S["env_frictions"].reshape(-1)[e]) + float(hc.ground_friction))
    lv = lams[6]
    ratio = np.hypot(lv[3 * 6 + 1], lv[3 * 6 + 2]) / (mu * lv[3 * 6])
    assert 0.995 < ratio < 1.0
