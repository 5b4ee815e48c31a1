"""scripts/onnx_sweep.py (the committed OnnxTest.onnx convention sweep, profiles/r4_onnx_sweep/)
runs and writes its table; the switches it applies act on the policy's view of the robot."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sweep_script_writes_table(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "onnx_sweep.py"), "--duration", "0.3",
                        "--envs_per_command", "1", "--threads", "2", "--only", "baseline", "hip_roll_yaw_sign_both",
                        "--out", str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.load(open(tmp_path / "onnx_sweep.json"))
    assert [v["name"] for v in d["variants"]] == ["baseline", "hip_roll_yaw_sign_both"]
    assert "| hip_roll_yaw_sign_both |" in open(tmp_path / "onnx_sweep.md").read()


def test_joint_sign_switch_flips_observation_and_action():
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import onnx_sweep as S
    import sim2sim_ref as SR
    v = S.variants()["hip_roll_sign_left"]
    hc, model, default, cfg = S.build(v, 1)
    root = np.zeros((1, 13))
    root[0, 2], root[0, 6] = 2.0, 1.0   # in the air: no contact
    q = default + 0.1
    seen = {}

    def policy(x):
        seen["obs"] = x[:, -47:].copy()
        a = np.zeros((1, 12))
        a[0, 0] = 1.0
        return a
    sim = SR.Sim2SimRef(hc, model, policy, root, q[None], np.zeros((1, 12)), np.full(1, model.mass[0]), np.ones(1),
                        np.zeros((1, 3)), joint_sign=v["sign"])
    sim.step()
    assert np.isclose(seen["obs"][0, 5], -0.1) and np.isclose(seen["obs"][0, 6], 0.1)
    # the policy's +1 on joint 0 reaches the simulator as -1: the left hip rolls the other way
    assert sim.sim.q[0, 0] < q[0]
