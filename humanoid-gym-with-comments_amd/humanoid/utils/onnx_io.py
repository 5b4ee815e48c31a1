"""ONNX wire format for the exported actor MLP, without the ``onnx`` package (not installed).

The deployment artefact the reference ships (humanoid/OnnxTest.onnx) is a plain MLP graph:
``Gemm`` (transB = 1) / ``Elu`` nodes from ``input`` to ``output`` with float32 initializers.
This module reads and writes exactly that subset of ModelProto with a hand-rolled protobuf
encoder/decoder (field numbers from onnx.proto3):

  ModelProto   1 ir_version, 2 producer_name, 7 graph, 8 opset_import{1 domain, 2 version}
  GraphProto   1 node, 2 name, 5 initializer, 11 input, 12 output
  NodeProto    1 input, 2 output, 3 name, 4 op_type, 5 attribute
  AttributeProto 1 name, 2 f, 3 i, 20 type
  TensorProto  1 dims, 2 data_type, 4 float_data, 8 name, 9 raw_data
  ValueInfoProto 1 name, 2 type{1 tensor_type{1 elem_type, 2 shape{1 dim{1 dim_value, 2 dim_param}}}}

``load_onnx_mlp(path)`` -> torch nn.Sequential (Linear/ELU) equivalent to the graph;
``export_policy_as_onnx(actor_critic, path)`` writes ``policy.onnx`` for the actor (the ONNX
counterpart of helpers.export_policy_as_jit, humanoid/utils/helpers.py:242-254).
Nothing in a loaded file is executed: the parser only reads numbers and strings.
"""
import os
import struct

import numpy as np


# ------------------------------------------------------------------------------------------------
# protobuf wire format
# ------------------------------------------------------------------------------------------------
def _varint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        if c < 0x80:
            return x, i
        s += 7


def _fields(b):
    """Yield (field_number, wire_type, value) over one message; value is int for varints,
    bytes for length-delimited, raw 4/8 bytes for fixed32/fixed64."""
    i, n = 0, len(b)
    while i < n:
        key, i = _varint(b, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(b, i)
            v, i = b[i:i + ln], i + ln
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _enc_varint(x):
    out = bytearray()
    x &= (1 << 64) - 1
    while True:
        c = x & 0x7F
        x >>= 7
        if x:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _key(fn, wt):
    return _enc_varint((fn << 3) | wt)


def _ld(fn, payload):
    if isinstance(payload, str):
        payload = payload.encode()
    return _key(fn, 2) + _enc_varint(len(payload)) + payload


def _vi(fn, x):
    return _key(fn, 0) + _enc_varint(x)


def _f32(fn, x):
    return _key(fn, 5) + struct.pack("<f", x)


# ------------------------------------------------------------------------------------------------
# reader
# ------------------------------------------------------------------------------------------------
def _tensor(b):
    dims, dtype, name, raw, fl = [], 1, "", None, []
    for fn, wt, v in _fields(b):
        if fn == 1:
            if wt == 2:  # packed
                j = 0
                while j < len(v):
                    d, j = _varint(v, j)
                    dims.append(d)
            else:
                dims.append(v)
        elif fn == 2:
            dtype = v
        elif fn == 4:
            if wt == 2:
                fl.extend(struct.unpack(f"<{len(v) // 4}f", v))
            else:
                fl.append(struct.unpack("<f", v)[0])
        elif fn == 8:
            name = v.decode()
        elif fn == 9:
            raw = v
    if dtype != 1:
        raise ValueError(f"initializer {name}: only float32 tensors are supported (data_type {dtype})")
    arr = np.frombuffer(raw, dtype="<f4").copy() if raw is not None else np.array(fl, np.float32)
    return name, arr.reshape(dims) if dims else arr


def _attr(b):
    name, val = "", None
    for fn, wt, v in _fields(b):
        if fn == 1:
            name = v.decode()
        elif fn == 2:
            val = struct.unpack("<f", v)[0]
        elif fn == 3:
            val = v - (1 << 64) if v >= 1 << 63 else v
    return name, val


def _node(b):
    node = {"input": [], "output": [], "op_type": "", "attrs": {}}
    for fn, _, v in _fields(b):
        if fn == 1:
            node["input"].append(v.decode())
        elif fn == 2:
            node["output"].append(v.decode())
        elif fn == 4:
            node["op_type"] = v.decode()
        elif fn == 5:
            k, val = _attr(v)
            node["attrs"][k] = val
    return node


def _value_info_name(b):
    for fn, _, v in _fields(b):
        if fn == 1:
            return v.decode()
    return ""


def read_onnx_graph(path):
    """Parse an ONNX file into {"nodes": [...], "init": {name: ndarray}, "inputs", "outputs",
    "opset"}."""
    with open(path, "rb") as f:
        data = f.read()
    graph, opset = None, None
    for fn, _, v in _fields(data):
        if fn == 7:
            graph = v
        elif fn == 8:
            for f2, _, v2 in _fields(v):
                if f2 == 2:
                    opset = v2
    if graph is None:
        raise ValueError(f"{path}: no graph")
    nodes, init, ins, outs = [], {}, [], []
    for fn, _, v in _fields(graph):
        if fn == 1:
            nodes.append(_node(v))
        elif fn == 5:
            k, a = _tensor(v)
            init[k] = a
        elif fn == 11:
            ins.append(_value_info_name(v))
        elif fn == 12:
            outs.append(_value_info_name(v))
    return {"nodes": nodes, "init": init, "inputs": [i for i in ins if i not in init], "outputs": outs,
            "opset": opset}


def load_onnx_mlp(path):
    """The Gemm/Elu (also Relu/Tanh/Identity) chain of an actor ONNX file as an nn.Sequential."""
    import torch
    import torch.nn as nn
    g = read_onnx_graph(path)
    layers, cur = [], g["inputs"][0]
    for nd in g["nodes"]:
        if nd["input"][0] != cur:
            raise ValueError(f"{path}: not a single chain at node {nd['op_type']} ({nd['input'][0]} != {cur})")
        op, a = nd["op_type"], nd["attrs"]
        if op == "Gemm":
            W = g["init"][nd["input"][1]].astype(np.float32)
            if not a.get("transB", 0):
                W = W.T
            if a.get("transA", 0):
                raise ValueError("Gemm with transA is not an MLP layer")
            B = g["init"][nd["input"][2]].astype(np.float32) if len(nd["input"]) > 2 else np.zeros(W.shape[0], np.float32)
            alpha, beta = a.get("alpha", 1.0), a.get("beta", 1.0)
            lin = nn.Linear(W.shape[1], W.shape[0])
            with torch.no_grad():
                lin.weight.copy_(torch.from_numpy(np.ascontiguousarray(W * alpha)))
                lin.bias.copy_(torch.from_numpy(np.ascontiguousarray(B.reshape(-1) * beta)))
            layers.append(lin)
        elif op == "Elu":
            layers.append(nn.ELU(alpha=a.get("alpha", 1.0)))
        elif op == "Relu":
            layers.append(nn.ReLU())
        elif op == "Tanh":
            layers.append(nn.Tanh())
        elif op == "Identity":
            pass
        else:
            raise ValueError(f"{path}: unsupported op {op}")
        cur = nd["output"][0]
    if cur != g["outputs"][0]:
        raise ValueError(f"{path}: chain ends at {cur}, graph output is {g['outputs'][0]}")
    return nn.Sequential(*layers)


# ------------------------------------------------------------------------------------------------
# writer
# ------------------------------------------------------------------------------------------------
def _value_info(name, dims):
    shape = b"".join(_ld(1, _vi(1, d) if isinstance(d, int) else _ld(2, d)) for d in dims)
    tensor_type = _vi(1, 1) + _ld(2, shape)
    return _ld(1, name) + _ld(2, _ld(1, tensor_type))


def write_onnx_mlp(seq, path, input_name="input", output_name="output", opset=11):
    """Serialise an nn.Sequential of Linear/ELU/ReLU/Tanh as Gemm(transB=1)/Elu/... nodes."""
    import torch.nn as nn
    nodes, inits = [], []
    cur, k = input_name, 0
    mods = [m for m in seq if not isinstance(m, nn.Identity)]
    in_dim = next(m.in_features for m in mods if isinstance(m, nn.Linear))
    out_dim = [m.out_features for m in mods if isinstance(m, nn.Linear)][-1]
    for idx, m in enumerate(mods):
        out = output_name if idx == len(mods) - 1 else f"/{k}/out"
        if isinstance(m, nn.Linear):
            w = m.weight.detach().cpu().float().numpy()
            b = m.bias.detach().cpu().float().numpy() if m.bias is not None else np.zeros(w.shape[0], np.float32)
            wn, bn = f"{k}.weight", f"{k}.bias"
            inits.append(_ld(5, b"".join(_vi(1, d) for d in w.shape) + _vi(2, 1) + _ld(8, wn) + _ld(9, w.astype("<f4").tobytes())))
            inits.append(_ld(5, _vi(1, b.shape[0]) + _vi(2, 1) + _ld(8, bn) + _ld(9, b.astype("<f4").tobytes())))
            attrs = [_ld(5, _ld(1, "alpha") + _f32(2, 1.0) + _vi(20, 1)),
                     _ld(5, _ld(1, "beta") + _f32(2, 1.0) + _vi(20, 1)),
                     _ld(5, _ld(1, "transB") + _vi(3, 1) + _vi(20, 2))]
            nodes.append(_ld(1, _ld(1, cur) + _ld(1, wn) + _ld(1, bn) + _ld(2, out) + _ld(3, f"/{k}/Gemm")
                             + _ld(4, "Gemm") + b"".join(attrs)))
        elif isinstance(m, nn.ELU):
            nodes.append(_ld(1, _ld(1, cur) + _ld(2, out) + _ld(3, f"/{k}/Elu") + _ld(4, "Elu")
                             + _ld(5, _ld(1, "alpha") + _f32(2, float(m.alpha)) + _vi(20, 1))))
        elif isinstance(m, nn.ReLU):
            nodes.append(_ld(1, _ld(1, cur) + _ld(2, out) + _ld(3, f"/{k}/Relu") + _ld(4, "Relu")))
        elif isinstance(m, nn.Tanh):
            nodes.append(_ld(1, _ld(1, cur) + _ld(2, out) + _ld(3, f"/{k}/Tanh") + _ld(4, "Tanh")))
        else:
            raise ValueError(f"cannot export {type(m).__name__}")
        cur, k = out, k + 1
    graph = (b"".join(nodes) + _ld(2, "main_graph") + b"".join(inits)
             + _ld(11, _value_info(input_name, [1, in_dim])) + _ld(12, _value_info(output_name, [1, out_dim])))
    model = _vi(1, 6) + _ld(2, "humanoid-gym-amd") + _ld(3, "0.2") + _ld(7, graph) + _ld(8, _ld(1, "") + _vi(2, opset))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(model)
    return path


def export_policy_as_onnx(actor_critic, path, filename="policy.onnx"):
    """ONNX counterpart of export_policy_as_jit: the actor MLP, input ``input`` [1, num_obs],
    output ``output`` [1, num_actions] (the layout of the reference's OnnxTest.onnx)."""
    return write_onnx_mlp(actor_critic.actor, os.path.join(path, filename))
