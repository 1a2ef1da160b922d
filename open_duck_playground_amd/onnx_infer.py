"""ONNX policy inference on the host (mirror of playground/common/onnx_infer.py:4-24).

The reference runs the exported policy with onnxruntime's CPU provider; onnxruntime is not
installed here, so this module decodes the ONNX protobuf itself (a wire-format reader, no
generated classes) and evaluates the graph with numpy. It supports the operator set the policy
export emits (common/export_onnx.py via onnx_export.py: Sub, Div, Gemm, Sigmoid, Mul, Tanh, Relu,
Add, MatMul, Identity) and raises on anything else, so a graph it cannot run fails loudly.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np


def _varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, i
        shift += 7


def _fields(b: bytes):
    """(field number, wire type, value) of one protobuf message; length-delimited values as bytes."""
    i, n = 0, len(b)
    while i < n:
        key, i = _varint(b, i)
        f, w = key >> 3, key & 7
        if w == 0:
            v, i = _varint(b, i)
        elif w == 2:
            ln, i = _varint(b, i)
            v, i = b[i:i + ln], i + ln
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        else:
            raise ValueError(f"unsupported protobuf wire type {w}")
        yield f, w, v


def _tensor(b: bytes) -> Tuple[str, np.ndarray]:
    dims, dtype, name, raw, floats = [], 1, "", None, []
    for f, w, v in _fields(b):
        if f == 1:
            if w == 2:  # packed dims
                j = 0
                while j < len(v):
                    d, j = _varint(v, j)
                    dims.append(d)
            else:
                dims.append(v)
        elif f == 2:
            dtype = v
        elif f == 8:
            name = v.decode()
        elif f == 9:
            raw = v
        elif f == 4:  # float_data
            floats.append(np.frombuffer(v, "<f4") if w == 2 else np.frombuffer(v, "<f4"))
    if dtype != 1:
        raise ValueError(f"initializer {name}: only float32 tensors are supported")
    a = np.frombuffer(raw, "<f4") if raw is not None else np.concatenate(floats)
    return name, a.reshape(dims).astype(np.float32)


def _node(b: bytes):
    ins, outs, op, attrs = [], [], "", {}
    for f, _, v in _fields(b):
        if f == 1:
            ins.append(v.decode())
        elif f == 2:
            outs.append(v.decode())
        elif f == 4:
            op = v.decode()
        elif f == 5:  # AttributeProto: name 1, f 2, i 3
            an, av = "", None
            for g, w, x in _fields(v):
                if g == 1:
                    an = x.decode()
                elif g == 2:
                    av = float(np.frombuffer(x, "<f4")[0])
                elif g == 3:
                    av = x
            attrs[an] = av
    return op, ins, outs, attrs


class OnnxGraph:
    def __init__(self, blob: bytes):
        graph = next(v for f, _, v in _fields(blob) if f == 7)
        self.nodes: List[tuple] = []
        self.init: Dict[str, np.ndarray] = {}
        self.inputs: List[str] = []
        self.outputs: List[str] = []
        for f, _, v in _fields(graph):
            if f == 1:
                self.nodes.append(_node(v))
            elif f == 5:
                k, a = _tensor(v)
                self.init[k] = a
            elif f == 11:
                self.inputs.append(next(x.decode() for g, _, x in _fields(v) if g == 1))
            elif f == 12:
                self.outputs.append(next(x.decode() for g, _, x in _fields(v) if g == 1))

    def run(self, feeds: Dict[str, np.ndarray]) -> List[np.ndarray]:
        env = dict(self.init)
        env.update({k: np.asarray(v, dtype=np.float32) for k, v in feeds.items()})
        for op, ins, outs, attrs in self.nodes:
            x = [env[i] for i in ins]
            if op == "Sub":
                y = x[0] - x[1]
            elif op == "Div":
                y = x[0] / x[1]
            elif op == "Add":
                y = x[0] + x[1]
            elif op == "Mul":
                y = x[0] * x[1]
            elif op == "Gemm":
                a = x[0].T if attrs.get("transA") else x[0]
                b = x[1].T if attrs.get("transB") else x[1]
                y = attrs.get("alpha", 1.0) * (a @ b)
                if len(x) > 2:
                    y = y + attrs.get("beta", 1.0) * x[2]
            elif op == "MatMul":
                y = x[0] @ x[1]
            elif op == "Sigmoid":
                y = 1.0 / (1.0 + np.exp(-x[0]))
            elif op == "Tanh":
                y = np.tanh(x[0])
            elif op == "Relu":
                y = np.maximum(x[0], 0)
            elif op == "Identity":
                y = x[0]
            else:
                raise NotImplementedError(f"ONNX op {op} is not supported by onnx_infer")
            env[outs[0]] = y.astype(np.float32)
        return [env[o] for o in self.outputs]


class OnnxInfer:
    """``OnnxInfer(onnx_model_path, input_name="obs", awd=False).infer(inputs)`` as in
    common/onnx_infer.py: with ``awd`` the input is one observation, fed as a batch of one."""

    def __init__(self, onnx_model_path: str, input_name: str = "obs", awd: bool = False):
        self.onnx_model_path = onnx_model_path
        with open(onnx_model_path, "rb") as f:
            self.graph = OnnxGraph(f.read())
        self.input_name = input_name
        self.awd = awd

    def infer(self, inputs):
        if self.awd:
            return self.graph.run({self.input_name: np.asarray([inputs], dtype=np.float32)})[0][0]
        return self.graph.run({self.input_name: np.asarray(inputs, dtype=np.float32)})[0]
