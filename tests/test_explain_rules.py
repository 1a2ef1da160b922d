"""The teacher-forcing explanation rules on the CPU (tests/teacher_forcing.py), oracle against
oracle: a rule that accepts a GPU substep as "sensitive" must accept a result the oracle itself
produces from an fp32-sized perturbation of the input, and must reject the result of a
deliberately wrong model (the CPU half of test_gpu_teacher_forced.py::test_explain_has_teeth)."""

import os

import numpy as np
import pytest

from open_duck_playground_amd import joystick
from open_duck_playground_amd.config import default_config, env_config_struct
from open_duck_playground_amd.mjcf import Model
from tests.oracle_ffi import OracleBatch, OracleModel
from tests.teacher_forcing import (DEFECTS, _state_rel, backward_error_landing, copy_model, flip_level,
                                   oracle_substep)

ASSETS = os.path.join(os.path.dirname(joystick.__file__), "assets")


def _states(task: str, n: int = 24, steps: int = 12, seed: int = 3):
    """substep inputs (qpos, qvel, qacc_warmstart, ctrl) of an oracle rollout with U(-1,1) actions"""
    m = Model.load(os.path.join(ASSETS, task + ".npz"))
    ob = OracleBatch(OracleModel(m), env_config_struct(m, default_config(), False), n)
    ob.reset(seed=seed)
    rng = np.random.default_rng(seed)
    for _ in range(steps):
        ob.step(rng.uniform(-1, 1, (n, 14)))
    L = ob.L
    F = ob.fs.reshape(L.nfloat, n)
    o = L.off
    xs = [np.concatenate([F[o["qpos"]:o["qpos"] + m.nq, e], F[o["qvel"]:o["qvel"] + m.nv, e],
                          F[o["qacc_warmstart"]:o["qacc_warmstart"] + m.nv, e], F[o["ctrl"]:o["ctrl"] + m.nu, e]])
          for e in range(n)]
    return m, xs


@pytest.mark.parametrize("defect", [d for d in DEFECTS if DEFECTS[d][0] == "flat"])
def test_backward_error_rule_rejects_model_defects(defect):
    m, xs = _states("flat_terrain")
    om = OracleModel(m)
    bad = OracleModel(DEFECTS[defect][1](copy_model(m)))
    rng = np.random.default_rng(0)
    checked = accepted = 0
    for x in xs:
        g = oracle_substep(bad, x)                      # the "GPU" runs the wrong model
        if _state_rel(m, g, oracle_substep(om, x)) <= 1e-4:
            continue                                    # not an outlier substep
        checked += 1
        accepted += backward_error_landing(om, x, g) is not None or flip_level(om, x, g, rng) is not None
    assert checked >= 8, checked
    assert accepted <= 0.1 * checked, (accepted, checked)


def test_backward_error_rule_accepts_perturbed_inputs():
    """the oracle's own substep from a 3e-7-perturbed input (below the rule's 1e-6 box) lands"""
    m, xs = _states("flat_terrain")
    om = OracleModel(m)
    rng = np.random.default_rng(1)
    k = m.nq + 2 * m.nv
    checked = landed = 0
    for x in xs:
        y = x.copy()
        y[:k] *= 1 + 3e-7 * rng.uniform(-1, 1, k)
        g = oracle_substep(om, y)
        if _state_rel(m, g, oracle_substep(om, x)) <= 1e-7:
            continue
        checked += 1
        landed += backward_error_landing(om, x, g) is not None
    assert checked >= 8 and landed >= 0.9 * checked, (landed, checked)
