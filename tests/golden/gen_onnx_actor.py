"""Weights-only fixture of the reference's trained XBot-L actor (humanoid/OnnxTest.onnx).

OnnxTest.onnx is the one artefact in the reference that carries PhysX behaviour: a 12-DOF XBot-L
policy (705 -> 512 -> 256 -> 128 -> 12, Gemm/Elu; input = 15 stacked 47-wide frames) trained in
Isaac Gym.  Its float32 initializers are copied here, read with the build's protobuf reader
(humanoid/utils/onnx_io.read_onnx_graph: numbers and strings only, nothing in the file runs),
into tests/golden/onnx_actor.npz as W0, b0, ..., W3, b3 (nn.Linear layout [out, in]) plus the
activation between layers.  The GPU box never reads the reference; the tests load the npz.

Usage (build container only):  python tests/golden/gen_onnx_actor.py
       python tests/golden/gen_onnx_actor.py <policy.onnx> <out.npz> "<source note>"
The second form makes the same fixture from a policy exported by THIS build (humanoid.utils.onnx_io,
scripts/train_eval.sh -> gpurun_out/train_eval/policy.onnx): tests/golden/hg_trained_actor.npz, the
positive control of scripts/onnx_fixed_base.py.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
SRC = "/root/reference/humanoid/OnnxTest.onnx"


def main(src=SRC, dst=os.path.join(HERE, "onnx_actor.npz"), note=None):
    from humanoid.utils.onnx_io import read_onnx_graph
    g = read_onnx_graph(src)
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
    out["source"] = np.array(note or "humanoid/OnnxTest.onnx (reference), opset %d" % g["opset"])
    np.savez_compressed(dst, **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        main()
