"""ONNX export (common/export_onnx.py:7-175).

The file is decoded with google.protobuf (an independent parser) through message classes built
from the onnx.proto field numbers, then the graph is evaluated op by op with numpy and compared
with the torch policy's deterministic action tanh(loc). onnx / onnxruntime are not installed, so
a check by those runtimes is not available here ("parity unpinned" against tf2onnx's output).
"""

import numpy as np
import pytest
import torch
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from open_duck_playground_amd import onnx_export, ppo

F = descriptor_pb2.FieldDescriptorProto


def _onnx_classes():
    fd = descriptor_pb2.FileDescriptorProto(name="onnx_subset.proto", package="onnxsub", syntax="proto2")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = ".onnxsub." + tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("OperatorSetIdProto", [("domain", 1, F.TYPE_STRING, O, None), ("version", 2, F.TYPE_INT64, O, None)])
    msg("TensorProto", [("dims", 1, F.TYPE_INT64, R, None), ("data_type", 2, F.TYPE_INT32, O, None),
                        ("name", 8, F.TYPE_STRING, O, None), ("raw_data", 9, F.TYPE_BYTES, O, None)])
    msg("Dimension", [("dim_value", 1, F.TYPE_INT64, O, None), ("dim_param", 2, F.TYPE_STRING, O, None)])
    msg("TensorShapeProto", [("dim", 1, F.TYPE_MESSAGE, R, "Dimension")])
    msg("TensorTypeProto", [("elem_type", 1, F.TYPE_INT32, O, None), ("shape", 2, F.TYPE_MESSAGE, O, "TensorShapeProto")])
    msg("TypeProto", [("tensor_type", 1, F.TYPE_MESSAGE, O, "TensorTypeProto")])
    msg("ValueInfoProto", [("name", 1, F.TYPE_STRING, O, None), ("type", 2, F.TYPE_MESSAGE, O, "TypeProto")])
    msg("NodeProto", [("input", 1, F.TYPE_STRING, R, None), ("output", 2, F.TYPE_STRING, R, None),
                      ("name", 3, F.TYPE_STRING, O, None), ("op_type", 4, F.TYPE_STRING, O, None)])
    msg("GraphProto", [("node", 1, F.TYPE_MESSAGE, R, "NodeProto"), ("name", 2, F.TYPE_STRING, O, None),
                       ("initializer", 5, F.TYPE_MESSAGE, R, "TensorProto"),
                       ("input", 11, F.TYPE_MESSAGE, R, "ValueInfoProto"),
                       ("output", 12, F.TYPE_MESSAGE, R, "ValueInfoProto")])
    msg("ModelProto", [("ir_version", 1, F.TYPE_INT64, O, None), ("producer_name", 2, F.TYPE_STRING, O, None),
                       ("producer_version", 3, F.TYPE_STRING, O, None), ("graph", 7, F.TYPE_MESSAGE, O, "GraphProto"),
                       ("opset_import", 8, F.TYPE_MESSAGE, R, "OperatorSetIdProto")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("onnxsub.ModelProto"))


def run_graph(model, obs):
    """Evaluate the exported graph with numpy (fp32, op by op)."""
    env = {t.name: np.frombuffer(t.raw_data, dtype="<f4").reshape(tuple(t.dims)) for t in model.graph.initializer}
    env["obs"] = obs.astype(np.float32)
    ops = {"Sub": lambda a, b: a - b, "Div": lambda a, b: a / b, "Mul": lambda a, b: a * b,
           "Sigmoid": lambda a: 1 / (1 + np.exp(-a)), "Tanh": np.tanh, "Gemm": lambda a, b, c: a @ b + c}
    for nd in model.graph.node:
        env[nd.output[0]] = ops[nd.op_type](*(env[i] for i in nd.input)).astype(np.float32)
    return env[model.graph.output[0].name]


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    torch.manual_seed(0)
    net = ppo.ActorCritic(101, 212, 14, ppo.PPOConfig())
    rng = np.random.default_rng(0)
    net.obs_norm.update(torch.tensor(rng.normal(2.0, 3.0, size=(500, 101)), dtype=torch.float32))
    path = str(tmp_path_factory.mktemp("onnx") / "policy.onnx")
    onnx_export.export_onnx(net, 14, 101, output_path=path)
    return net, path


def test_onnx_structure(trained):
    _, path = trained
    m = _onnx_classes()()
    m.ParseFromString(open(path, "rb").read())
    assert m.ir_version == 6 and m.opset_import[0].version == 11 and m.opset_import[0].domain == ""
    g = m.graph
    assert [i.name for i in g.input] == ["obs"] and [o.name for o in g.output] == ["continuous_actions"]
    assert [d.dim_value for d in g.input[0].type.tensor_type.shape.dim] == [1, 101]
    assert [d.dim_value for d in g.output[0].type.tensor_type.shape.dim] == [1, 14]
    assert g.input[0].type.tensor_type.elem_type == 1
    ops = [n.op_type for n in g.node]
    assert ops == ["Sub", "Div"] + ["Gemm", "Sigmoid", "Mul"] * 3 + ["Gemm", "Tanh"]
    shapes = {t.name: tuple(t.dims) for t in g.initializer}
    assert shapes["hidden_0/kernel"] == (101, 512) and shapes["hidden_3/kernel"] == (128, 14)
    assert shapes["mean"] == (101,) and shapes["std"] == (101,)


def test_onnx_matches_policy(trained):
    net, path = trained
    m = _onnx_classes()()
    m.ParseFromString(open(path, "rb").read())
    rng = np.random.default_rng(1)
    for _ in range(5):
        obs = rng.normal(2.0, 3.0, size=(1, 101))
        got = run_graph(m, obs)
        with torch.no_grad():
            exp = ppo.NormalTanh(net.policy_logits(torch.tensor(obs, dtype=torch.float32))).mode().numpy()
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-5)


def test_varint_encoding():
    assert onnx_export._varint(0) == b"\x00" and onnx_export._varint(300) == b"\xac\x02"
    assert onnx_export._varint(2 ** 63) == b"\x80" * 9 + b"\x01"


def test_product_onnx_infer_matches_policy(trained):
    """onnx_infer.OnnxInfer (the sim2sim loop's runtime: its own protobuf reader + numpy) runs the
    exported file to the torch policy's deterministic action, awd=True feeding one observation."""
    from open_duck_playground_amd.onnx_infer import OnnxInfer
    net, path = trained
    oi = OnnxInfer(path, awd=True)
    rng = np.random.default_rng(2)
    for _ in range(5):
        obs = rng.normal(2.0, 3.0, size=101)
        with torch.no_grad():
            exp = ppo.NormalTanh(net.policy_logits(torch.tensor(obs[None], dtype=torch.float32))).mode().numpy()[0]
        np.testing.assert_allclose(oi.infer(obs), exp, rtol=1e-5, atol=1e-5)
    assert oi.graph.inputs == ["obs"] and oi.graph.outputs == ["continuous_actions"]


def test_product_onnx_infer_rejects_unknown_ops(trained, tmp_path):
    from open_duck_playground_amd import onnx_export as ox
    from open_duck_playground_amd.onnx_infer import OnnxGraph
    nodes = ox._bytes(1, ox.node("Softmax", ["obs"], ["y"], "sm"))
    graph = nodes + ox._str(2, "g") + ox._bytes(11, ox.value_info("obs", [1, 3])) + ox._bytes(12, ox.value_info("y", [1, 3]))
    g = OnnxGraph(ox._int(1, 6) + ox._bytes(7, graph))
    with pytest.raises(NotImplementedError):
        g.run({"obs": np.zeros((1, 3))})
