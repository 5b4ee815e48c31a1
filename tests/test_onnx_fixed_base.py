"""CPU pins of the suspended-robot probe of the reference's trained actor (scripts/onnx_fixed_base.py,
profiles/r5_onnx_fixed_base/): conventions vs physics.

  * suspended (base fixed, no contact), the actor's joints move against compute_ref_state
    (humanoid_env.py:714-744) on the left knee, right hip pitch and right ankle pitch at every
    command, while the actor trained on this physics (tests/golden/hg_trained_actor.npz) moves
    both legs' hip pitch and knee in phase with it;
  * with those joints — and both hip yaws, which the air gait cannot judge — driven with the
    opposite sign, the PhysX-trained actor stands and walks on the ground in this physics where the
    trained conventions make it fall within half a second;
  * the committed profile carries the same derived signs.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))

DERIVED_FLIPS = ("l_yaw", "l_knee", "r_yaw", "r_pitch", "r_ankle")


@pytest.fixture(scope="module")
def fb():
    import onnx_fixed_base as FB
    import physics_ref as P
    P.set_threads(min(8, os.cpu_count() or 1))
    return FB


def _derived_sign(FB):
    s = np.ones(12)
    for n in DERIVED_FLIPS:
        s[FB.DOF_NAMES.index(n)] = -1.0
    return s


def test_air_gait_inverts_three_joints(fb):
    W = fb.load(fb.FIXTURE)
    r = fb.run_fixed("baseline", {}, W, 2.6)
    inv = [fb.DOF_NAMES[j] for j in fb.inverted_joints(r)]
    assert inv == ["l_knee", "r_pitch", "r_ankle"], inv
    assert not r["reproduces"]
    signed = fb.run_fixed("signed", {"sign": _derived_sign(fb)}, W, 2.6)
    assert signed["reproduces"] and not fb.inverted_joints(signed)


def test_control_actor_matches_reference_gait(fb):
    r = fb.run_fixed("baseline", {}, fb.load(fb.OWN), 2.6)
    assert r["reproduces"], fb.summary_row(r)


def test_derived_signs_walk_where_trained_conventions_fall(fb):
    import onnx_sweep as SW
    W = fb.load(fb.FIXTURE)
    base = SW.run_variant("baseline", {}, W, 1, 3.0)
    signed = SW.run_variant("signed", {"sign": _derived_sign(fb)}, W, 1, 3.0)
    print("baseline", base["falls"], base["mean_survival_s"], "signed", signed["falls"], signed["mean_survival_s"])
    assert base["falls"] == base["envs"] and base["mean_survival_s"] < 1.0
    assert signed["falls"] == 0


def test_committed_profile_has_the_derived_signs(fb):
    with open(os.path.join(REPO, "profiles", "r5_onnx_fixed_base", "onnx_fixed_base.json")) as f:
        d = json.load(f)
    assert d["derived_signs"] == _derived_sign(fb).tolist()
    rows = d["closed_loop_under_derived_signs"]
    assert rows[0]["falls"] <= rows[0]["envs"] // 4       # the derived conventions alone: most envs walk 20 s
