"""Single-robot 50 Hz control loop with the ONNX policy in the loop (sim2sim.MjInfer, mirror of
mujoco_infer.py:16-241) on the HIP kernels, against the same loop with the oracle as physics.

Teacher forced per control period: before each period the GPU loop takes the oracle loop's
physics state, so every period compares 10 substeps + the 101-d observation + the policy's
action from identical inputs.
"""

import numpy as np
import pytest
import torch

from open_duck_playground_amd import onnx_export, ppo
from open_duck_playground_amd.sim2sim import MjInfer
from tests.oracle_ffi import OracleModel

pytestmark = pytest.mark.gpu


class OracleMjInfer(MjInfer):
    """The same host loop with the fp64 oracle stepping the physics (mj_step x decimation)."""

    def __init__(self, *a, **kw):
        self._om = None
        super().__init__(*a, **kw)

    def _oracle(self):
        if self._om is None:
            self._om = OracleModel(self.model)
        return self._om

    def _run_oracle(self, nsub):
        m, om = self.model, self._oracle()
        g = lambda t: t[:, 0].cpu().numpy().astype(np.float64)  # noqa: E731
        d = om.new_data(qpos=g(self.qpos), qvel=g(self.qvel), ctrl=g(self.ctrl), warm=g(self.warm))
        om.step(d, nsub)
        for t, name, k in ((self.qpos, "qpos", m.nq), (self.qvel, "qvel", m.nv), (self.warm, "qacc_warmstart", m.nv)):
            t.copy_(torch.tensor(d.arr(name, k)[:, None], dtype=torch.float32, device=t.device))
        aux = np.concatenate([d.arr("qacc", m.nv), d.arr("qacc_smooth", m.nv), d.arr("qvel", m.nv),
                              d.arr("qfrc_smooth", m.nv), d.arr("actuator_force", m.nu),
                              d.arr("sensordata", m.nsensordata), d.arr("con_dist", 4 * m.npair)])
        self._aux_np = aux
        # keep the fp64 state for the next period (the tensors above are its fp32 view)
        self._d = d

    def _physics(self):
        self._run_oracle(self.decimation)


@pytest.fixture(scope="module")
def policy_file(tmp_path_factory):
    torch.manual_seed(3)
    net = ppo.ActorCritic(101, 212, 14, ppo.PPOConfig())
    rng = np.random.default_rng(0)
    net.obs_norm.update(torch.tensor(rng.normal(0.0, 1.0, size=(500, 101)), dtype=torch.float32))
    path = str(tmp_path_factory.mktemp("onnx") / "policy.onnx")
    onnx_export.export_onnx(net, 14, 101, output_path=path)
    return net, path


def test_control_loop_matches_oracle_loop(policy_file, gpu):
    net, path = policy_file
    cmd = [0.1, 0.0, 0.3, 0.0, 0.0, 0.0, 0.0]
    hip = MjInfer("flat_terrain", onnx_model_path=path, device=gpu)
    ref = OracleMjInfer("flat_terrain", onnx_model_path=path, device=gpu)
    hip.commands = ref.commands = cmd
    errs = []
    for k in range(25):                     # 0.5 s of control at 50 Hz
        for a in ("qpos", "qvel", "warm", "ctrl"):
            getattr(hip, a).copy_(getattr(ref, a))
        for a in ("last_action", "last_last_action", "last_last_last_action", "motor_targets", "prev_motor_targets",
                  "imitation_i"):
            setattr(hip, a, np.copy(getattr(ref, a)))
        o_ref, a_ref = ref.control_step()
        o_hip, a_hip = hip.control_step()
        errs.append(np.abs(o_hip - o_ref).max() / (1 + np.abs(o_ref).max()))
        assert o_hip.shape == (101,)
        np.testing.assert_allclose(a_hip, a_ref, atol=2e-3)
    errs = np.array(errs)
    print("per-period obs rel err: median %.2e max %.2e" % (np.median(errs), errs.max()))
    assert np.median(errs) < 1e-4 and (errs < 2e-3).mean() >= 0.96, errs


def test_observation_contract_and_policy_in_loop(policy_file, gpu):
    """101 values in mujoco_infer.py's order, the accelerometer's +1.3 on x, the command, unit-circle
    phase; the action is the exported policy's deterministic tanh(loc) on that observation."""
    net, path = policy_file
    hip = MjInfer("flat_terrain", onnx_model_path=path, device=gpu)
    cmd = [0.05, -0.1, 0.2, 0.1, 0.0, 0.3, 0.0]
    for _ in range(5):
        obs, action = hip.run(1, command=cmd)[-1], hip.last_action
        acc = hip.get_accelerometer()
        np.testing.assert_allclose(obs[3:6], acc + np.array([1.3, 0, 0]))
        np.testing.assert_allclose(obs[6:13], cmd)
        assert set(np.unique(obs[97:99])) <= {0.0, 1.0}
        np.testing.assert_allclose(np.hypot(obs[99], obs[100]), 1.0, atol=1e-12)
        with torch.no_grad():
            exp = ppo.NormalTanh(net.policy_logits(torch.tensor(obs[None], dtype=torch.float32))).mode().numpy()[0]
        np.testing.assert_allclose(action, exp, atol=1e-5)
    np.testing.assert_array_equal(hip.saved_obs[-1], obs)


def test_control_loop_rate(policy_file, gpu):
    """The loop runs far faster than real time (the reference paces it at 50 Hz)."""
    import time
    _, path = policy_file
    hip = MjInfer("flat_terrain", onnx_model_path=path, device=gpu)
    hip.run(10)
    t0 = time.perf_counter()
    hip.run(200)
    hz = 200 / (time.perf_counter() - t0)
    print(f"control loop: {hz:.0f} periods/s ({hz / 50:.0f}x real time)")
    assert hz > 50
