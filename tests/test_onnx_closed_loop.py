"""The reference's trained XBot-L actor (humanoid/OnnxTest.onnx -> tests/golden/onnx_actor.npz,
weights only) driven closed-loop on the CPU reference physics in the reference's sim2sim loop
(oracle/sim2sim_ref.py; humanoid/scripts/sim2sim.py:185-280).  CPU tests: the fixture, the
policy restatement, and the recorded outcome that DESIGN.md section 4 reports as the PhysX-side
evidence (the GPU leg and the GPU-vs-oracle agreement are tests/test_gpu_onnx_closed_loop.py):

  * with the self-collision model (hands vs thighs / shins), every episode is terminated by a
    hand-leg contact (net force on the base link > 1 N, humanoid_env.py:811-816), half of them
    within 0.5 s, all within 1 s;
  * without self-collision, every episode ends by the base box hitting the ground, 0.8-1.4 s in.
"""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))


def test_fixture_is_the_705_512_256_128_12_elu_actor(golden):
    w = golden("onnx_actor.npz")
    assert [w[f"W{k}"].shape for k in range(4)] == [(512, 705), (256, 512), (128, 256), (12, 128)]
    assert [w[f"b{k}"].shape for k in range(4)] == [(512,), (256,), (128,), (12,)]
    assert list(w["activations"]) == ["elu"] * 3 and "OnnxTest.onnx" in str(w["source"])


def test_numpy_policy_matches_the_torch_policy(golden):
    """The oracle's float64 numpy MLP and the module sim2sim.py drives on the GPU (built from the
    same weights) agree to fp32 rounding."""
    import sim2sim_ref as SR
    from humanoid.scripts.sim2sim import mlp_from_weights
    w = golden("onnx_actor.npz")
    x = np.random.default_rng(0).standard_normal((64, 705))
    y64 = SR.mlp(w)(x)
    with torch.no_grad():
        y32 = mlp_from_weights(w)(torch.from_numpy(x).float()).double().numpy()
    np.testing.assert_allclose(y32, y64, rtol=1e-4, atol=1e-4)


def _run(self_collisions, steps=150, epc=2):
    import physics_ref as P
    import pipeline_ref as PR
    import sim2sim_ref as SR
    import onnx_closed_loop as OC
    from humanoid import _native as N
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    from humanoid.scripts import sim2sim as S2
    cmds = np.repeat(np.array(OC.COMMANDS, np.float32), epc, axis=0)
    n = len(cmds)
    cfg = S2.make_cfg("urdf", n, steps * 0.01, self_collisions)
    model, js = N.load_model(armature=cfg.sim.hg.armature, self_collisions=self_collisions)
    hc, _ = build_hg_cfg(cfg, n, cfg.sim.dt, 5, js)
    mass, fric = np.full(n, model.mass[0]), np.ones(n)
    S, _, _ = PR.initial_state(PR.Cfg(hc), np.zeros((n, 3), np.float32), mass, fric)
    P.set_threads(min(8, os.cpu_count() or 1))
    W = np.load(OC.FIXTURE, allow_pickle=False)
    sim = SR.Sim2SimRef(hc, model, SR.mlp(W), S["root_states"], S["dof_pos"], S["dof_vel"], mass, fric, cmds,
                        cycle_time=cfg.rewards.cycle_time, cause_slots=OC.cause_slots(js, model))
    return sim.run(steps)


def test_closed_loop_terminates_on_hand_leg_contact():
    out = _run(True, steps=100)
    assert out["fell"].all()
    assert set(out["fall_cause"]) == {"hand_leg"}
    assert np.median(out["fall_step"]) <= 50 and (out["fall_step"] <= 100).all()


def test_closed_loop_without_self_collision_falls_on_the_base():
    out = _run(False, steps=150)
    assert out["fell"].all()
    assert set(out["fall_cause"]) == {"base_ground"}
    assert (out["fall_step"] >= 80).all() and (out["fall_step"] <= 140).all()
