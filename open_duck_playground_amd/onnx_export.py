"""ONNX export of the trained policy (common/export_onnx.py:7-175), without onnx/tf2onnx.

The reference rebuilds the brax policy MLP in Keras (normalise with the running mean/std of
``state``, swish hidden layers, split the logits, ``tanh(loc)``) and converts it with
tf2onnx at opset 11: input ``obs`` float32 [1, obs_size], output ``continuous_actions``
float32 [1, action_size]. Neither tensorflow nor onnx is installed here, so this module
writes the same graph straight into the ONNX protobuf wire format:

    obs -> Sub(mean) -> Div(std) -> [Gemm -> Sigmoid, Mul (swish)] x hidden -> Gemm(loc half) -> Tanh

The last Gemm keeps only the ``loc`` half of the output layer (the reference splits the logits
and drops the scale half), so the graph computes exactly the deterministic policy
``tanh(loc)`` the reference exports.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

IR_VERSION = 6  # ONNX IR version that goes with opset 11
OPSET = 11
FLOAT = 1  # TensorProto.DataType.FLOAT


# --- protobuf wire format -------------------------------------------------------------
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _int(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def _bytes(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def _str(field: int, s: str) -> bytes:
    return _bytes(field, s.encode())


# --- ONNX messages (field numbers of onnx.proto) --------------------------------------
def tensor(name: str, arr: np.ndarray) -> bytes:
    a = np.ascontiguousarray(arr, dtype="<f4")
    return b"".join(_int(1, d) for d in a.shape) + _int(2, FLOAT) + _str(8, name) + _bytes(9, a.tobytes())


def value_info(name: str, shape: Sequence[int]) -> bytes:
    dims = b"".join(_bytes(1, _int(1, d)) for d in shape)  # TensorShapeProto.dim{dim_value}
    tensor_type = _int(1, FLOAT) + _bytes(2, dims)  # TypeProto.Tensor{elem_type, shape}
    return _str(1, name) + _bytes(2, _bytes(1, tensor_type))  # ValueInfoProto{name, type{tensor_type}}


def node(op: str, inputs: List[str], outputs: List[str], name: str) -> bytes:
    return (b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outputs) + _str(3, name)
            + _str(4, op))


def policy_graph(layers: List[tuple], mean: np.ndarray, std: np.ndarray, obs_size: int, action_size: int) -> bytes:
    """ModelProto bytes. ``layers`` = [(W [in, out], b [out]), ...] with the loc-only last layer."""
    nodes, inits = [], [tensor("mean", mean), tensor("std", std)]
    nodes.append(node("Sub", ["obs", "mean"], ["x_centered"], "normalize_sub"))
    nodes.append(node("Div", ["x_centered", "std"], ["h_in"], "normalize_div"))
    x = "h_in"
    for i, (w, b) in enumerate(layers):
        inits += [tensor(f"hidden_{i}/kernel", w), tensor(f"hidden_{i}/bias", b)]
        y = f"hidden_{i}/out"
        nodes.append(node("Gemm", [x, f"hidden_{i}/kernel", f"hidden_{i}/bias"], [y], f"hidden_{i}"))
        if i < len(layers) - 1:
            nodes.append(node("Sigmoid", [y], [f"hidden_{i}/sig"], f"hidden_{i}/sigmoid"))
            nodes.append(node("Mul", [y, f"hidden_{i}/sig"], [f"hidden_{i}/swish"], f"hidden_{i}/swish"))
            x = f"hidden_{i}/swish"
        else:
            x = y
    nodes.append(node("Tanh", [x], ["continuous_actions"], "tanh"))
    graph = (b"".join(_bytes(1, n) for n in nodes) + _str(2, "policy")
             + b"".join(_bytes(5, t) for t in inits)
             + _bytes(11, value_info("obs", [1, obs_size]))
             + _bytes(12, value_info("continuous_actions", [1, action_size])))
    opset = _str(1, "") + _int(2, OPSET)
    return (_int(1, IR_VERSION) + _str(2, "open_duck_playground_amd") + _str(3, "1")
            + _bytes(7, graph) + _bytes(8, opset))


def export_onnx(net, action_size: int, obs_size: int, output_path: str = "ONNX.onnx") -> bytes:
    """Write the policy of an ``ppo.ActorCritic`` as ONNX (export_onnx.py:7-175's contract)."""
    lin = [m for m in net.policy if isinstance(m, torch.nn.Linear)]
    layers = []
    for i, m in enumerate(lin):
        w = m.weight.detach().double().cpu().numpy().T  # [in, out]
        b = m.bias.detach().double().cpu().numpy()
        if i == len(lin) - 1:
            w, b = w[:, :action_size], b[:action_size]  # loc half of the logits
        layers.append((w, b))
    if getattr(net, "normalize", True):
        mean = net.obs_norm.mean.detach().cpu().numpy()
        std = net.obs_norm.std.detach().cpu().numpy()
    else:
        mean, std = np.zeros(obs_size), np.ones(obs_size)
    blob = policy_graph(layers, mean, std, obs_size, action_size)
    with open(output_path, "wb") as f:
        f.write(blob)
    return blob

