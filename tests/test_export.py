"""Policy export (next-row 2): TorchScript policy_1.pt / base_lin_vel.pt (helpers.py:242-254)
and the ONNX actor wire format (humanoid/OnnxTest.onnx: Gemm/Elu, input -> output)."""
import os

import numpy as np
import pytest
import torch

from humanoid.algo.ppo import ActorCritic
from humanoid.utils.helpers import export_policy_as_jit
from humanoid.utils.onnx_io import export_policy_as_onnx, load_onnx_mlp, read_onnx_graph

DIMS = dict(num_actor_obs=705, num_critic_obs=219, num_actions=12, actor_hidden_dims=[512, 256, 128],
            critic_hidden_dims=[768, 256, 128], init_noise_std=1.0)


def test_jit_export_roundtrip(tmp_path):
    torch.manual_seed(0)
    ac = ActorCritic(**DIMS)
    export_policy_as_jit(ac, str(tmp_path))
    pol = torch.jit.load(os.path.join(tmp_path, "policy_1.pt"))
    lv = torch.jit.load(os.path.join(tmp_path, "base_lin_vel.pt"))
    x = torch.randn(7, 705)
    torch.testing.assert_close(pol(x), ac.actor(x))
    torch.testing.assert_close(lv(x), ac.base_lin_vel(x))


def test_onnx_roundtrip(tmp_path):
    torch.manual_seed(1)
    ac = ActorCritic(**DIMS)
    p = export_policy_as_onnx(ac, str(tmp_path))
    g = read_onnx_graph(p)
    assert [n["op_type"] for n in g["nodes"]] == ["Gemm", "Elu", "Gemm", "Elu", "Gemm", "Elu", "Gemm"]
    assert g["inputs"] == ["input"] and g["outputs"] == ["output"] and g["opset"] == 11
    m = load_onnx_mlp(p)
    x = torch.randn(5, 705)
    with torch.no_grad():
        torch.testing.assert_close(m(x), ac.actor(x), rtol=0, atol=0)
    # the reader output loads straight into the actor's state dict
    ac2 = ActorCritic(**DIMS)
    ac2.actor.load_state_dict(m.state_dict())
    with torch.no_grad():
        torch.testing.assert_close(ac2.act_inference(x), ac.act_inference(x), rtol=0, atol=0)


REF_ONNX = "/root/reference/humanoid/OnnxTest.onnx"


@pytest.mark.skipif(not os.path.exists(REF_ONNX), reason="reference tree not present (GPU box)")
def test_reads_reference_onnx():
    """The reference's shipped ONNX actor parses into a Gemm/Elu chain (data only; nothing in the
    file is executed)."""
    g = read_onnx_graph(REF_ONNX)
    ops = [n["op_type"] for n in g["nodes"]]
    assert set(ops) <= {"Gemm", "Elu"} and ops[0] == "Gemm" and ops[-1] == "Gemm"
    m = load_onnx_mlp(REF_ONNX)
    lin = [l for l in m if isinstance(l, torch.nn.Linear)]
    x = torch.randn(3, lin[0].in_features)
    with torch.no_grad():
        y = m(x)
    assert y.shape == (3, lin[-1].out_features) and torch.isfinite(y).all()
    # numpy evaluation of the same graph straight from the initializers agrees
    h = x.numpy().astype(np.float64)
    for nd in g["nodes"]:
        if nd["op_type"] == "Gemm":
            W = g["init"][nd["input"][1]].astype(np.float64)
            W = W.T if nd["attrs"].get("transB", 0) else W
            h = nd["attrs"].get("alpha", 1.0) * h @ W + nd["attrs"].get("beta", 1.0) * g["init"][nd["input"][2]]
        else:
            a = nd["attrs"].get("alpha", 1.0)
            h = np.where(h > 0, h, a * (np.exp(h) - 1))
    np.testing.assert_allclose(y.numpy(), h, rtol=1e-4, atol=1e-4)
