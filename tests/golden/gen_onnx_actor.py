"""Weights-only fixture of the reference's trained XBot-L actor (humanoid/OnnxTest.onnx).

OnnxTest.onnx is the one artefact in the reference that carries PhysX behaviour: a 12-DOF XBot-L
policy (705 -> 512 -> 256 -> 128 -> 12, Gemm/Elu; input = 15 stacked 47-wide frames) trained in
Isaac Gym.  Its float32 initializers are copied here, read with the build's protobuf reader
(humanoid/utils/onnx_io.read_onnx_graph: numbers and strings only, nothing in the file runs),
into tests/golden/onnx_actor.npz as W0, b0, ..., W3, b3 (nn.Linear layout [out, in]) plus the
activation between layers.  The GPU box never reads the reference; the tests load the npz.

Usage (build container only):  python tests/golden/gen_onnx_actor.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
SRC = "/root/reference/humanoid/OnnxTest.onnx"


def main():
    from humanoid.utils.onnx_io import read_onnx_graph
    g = read_onnx_graph(SRC)
    out, cur, k, acts = {}, g["inputs"][0], 0, []
    for nd in g["nodes"]:
        assert nd["input"][0] == cur, "single chain"
        if nd["op_type"] == "Gemm":
            a = nd["attrs"]
            assert a.get("transB", 0) == 1 and not a.get("transA", 0) and a.get("alpha", 1.0) == 1.0 \
                and a.get("beta", 1.0) == 1.0
            out[f"W{k}"] = np.ascontiguousarray(g["init"][nd["input"][1]], np.float32)
            out[f"b{k}"] = np.ascontiguousarray(g["init"][nd["input"][2]], np.float32).reshape(-1)
            k += 1
        elif nd["op_type"] == "Elu":
            assert nd["attrs"].get("alpha", 1.0) == 1.0
            acts.append("elu")
        else:
            raise ValueError(nd["op_type"])
        cur = nd["output"][0]
    assert cur == g["outputs"][0] and k == 4 and acts == ["elu"] * 3
    out["activations"] = np.array(acts)
    out["source"] = np.array("humanoid/OnnxTest.onnx (reference), opset %d" % g["opset"])
    np.savez_compressed(os.path.join(HERE, "onnx_actor.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
