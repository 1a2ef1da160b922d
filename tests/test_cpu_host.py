"""Host-side checks that need no GPU: compiled model facts, the safe pkl decoder,
the C-ABI library (loads, exports every declared symbol, layout agrees with Python).

Model facts follow SURVEY.md appendix A (derived from the reference XMLs:
playground/open_duck_mini_v2/xmls/open_duck_mini_v2.xml, scene_flat_terrain.xml, ...).
"""

import ctypes as C
import os
import pickle
import re

import numpy as np
import pytest

from open_duck_playground_amd import constants, native
from open_duck_playground_amd.cabi import dr_layout, layout
from open_duck_playground_amd.mjcf import Model, mass_matrix_np
from open_duck_playground_amd.refmotion import read_poly_pkl

ROOT = os.path.join(os.path.dirname(__file__), "..")


@pytest.fixture(scope="module", params=["flat_terrain", "flat_terrain_backlash", "rough_terrain"])
def model(request):
    return request.param, Model.load(constants.task_to_xml(request.param))


def test_model_dimensions(model):
    task, m = model
    backlash = "backlash" in task
    assert (m.nq, m.nv, m.nu) == ((31, 30, 14) if backlash else (21, 20, 14))
    assert m.nbody == 18  # backlash hinges sit on the actuated bodies
    assert m.njnt == (25 if backlash else 15)
    assert m.nsensordata == 46
    assert m.npair == 3
    # pair 0 = foot-foot, pairs 1-2 = floor vs each foot, floor friction 0.6 (flat) via priority
    names = m.names["geom"]
    assert names[m.pair_geom1[1]] == "floor" and names[m.pair_geom1[2]] == "floor"
    assert {names[m.pair_geom2[1]], names[m.pair_geom2[2]]} == {"left_foot_bottom_tpu", "right_foot_bottom_tpu"} or \
        m.pair_geom2[1] != m.pair_geom2[2]
    if task.startswith("flat"):
        assert np.isclose(m.pair_friction[1][0], 0.6)
    np.testing.assert_allclose(m.opt_timestep, 0.002)
    assert m.opt_iterations == 1 and m.opt_ls_iterations == 5


def test_actuators_and_keyframe(model):
    task, m = model
    kp = 17.11 if "backlash" in task else 13.37
    np.testing.assert_allclose(m.actuator_kp, kp)
    np.testing.assert_allclose(m.actuator_forcerange, np.tile([-3.23, 3.23], (14, 1)))
    key = m.names["key"].index("home")
    assert np.isclose(m.key_qpos[key][2], 0.15, atol=0.05)  # standing height
    q = m.key_qpos[key][3:7]
    assert np.isclose(np.linalg.norm(q), 1.0, atol=1e-6)


def test_foot_hull():
    m = Model.load(constants.task_to_xml("flat_terrain"))
    h = m.hulls[0]
    assert (len(h.vert), len(h.face_normal), len(h.edge)) == (17, 30, 45)  # V - E + F = 2
    assert len(h.vert) - len(h.edge) + len(h.face_normal) == 2
    # every vertex lies on or inside every face plane
    d = h.vert @ np.asarray(h.face_normal).T - np.asarray(h.face_offset)[None, :]
    assert d.max() < 1e-6


def test_mass_matrix_spd_and_energy():
    """M(q) is SPD, and 1/2 qd' M qd equals the sum of body kinetic energies (independent path)."""
    m = Model.load(constants.task_to_xml("flat_terrain"))
    rng = np.random.default_rng(0)
    for _ in range(3):
        q = m.qpos0.copy()
        q[7:] += rng.uniform(-0.3, 0.3, m.nq - 7)
        quat = rng.normal(size=4)
        q[3:7] = quat / np.linalg.norm(quat)
        M, kin = mass_matrix_np(m, q)
        assert np.allclose(M, M.T)
        assert np.linalg.eigvalsh(M).min() > 0
        # finite-difference body velocities from kinematics at q and q + eps * qd
        qd = rng.normal(size=m.nv)
        eps = 1e-6
        from open_duck_playground_amd.mjcf import _kinematics_np, quat_mul
        q2 = q.copy()
        q2[:3] += eps * qd[:3]
        w = qd[3:6] * eps  # local angular velocity
        dq = np.concatenate([[1.0], 0.5 * w])
        q2[3:7] = quat_mul(q[3:7], dq)
        q2[3:7] /= np.linalg.norm(q2[3:7])
        q2[7:] += eps * qd[6:]
        k1 = _kinematics_np(m, q)
        k2 = _kinematics_np(m, q2)
        ke = 0.0
        for b in range(1, m.nbody):
            v = (k2[2][b] - k1[2][b]) / eps
            dR = (k2[3][b] - k1[3][b]) / eps
            W = dR @ k1[3][b].T
            om = np.array([W[2, 1], W[0, 2], W[1, 0]])
            Ib = k1[3][b] @ np.diag(m.body_inertia[b]) @ k1[3][b].T
            ke += 0.5 * m.body_mass[b] * v @ v + 0.5 * om @ Ib @ om
        arm = 0.5 * np.sum(m.dof_armature * qd * qd)
        np.testing.assert_allclose(0.5 * qd @ M @ qd - arm, ke, rtol=1e-4)


def test_pkl_decoder_refuses_code(tmp_path):
    import collections
    p = tmp_path / "bad.pkl"
    p.write_bytes(pickle.dumps(collections.OrderedDict(a=1)))
    with pytest.raises(ValueError):
        read_poly_pkl(str(p))
    p.write_bytes(pickle.dumps({"x": [1.0, 2.0], "n": 3}))
    assert read_poly_pkl(str(p)) == {"x": [1.0, 2.0], "n": 3}


def _declared_symbols():
    syms = set()
    for f in os.listdir(os.path.join(ROOT, "include")):
        txt = open(os.path.join(ROOT, "include", f)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for mm in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(duck_[a-z_0-9]+)\s*\(", txt, flags=re.M):
            if "static inline" not in txt[max(0, mm.start() - 40):mm.start() + 1]:
                syms.add(mm.group(1))
    return syms


def test_cabi_exports_every_declared_symbol():
    if not os.path.exists(native.LIB_PATH):
        native.build()
    syms = _declared_symbols()
    assert {"duck_create", "duck_step", "duck_reset", "duck_destroy", "duck_last_error"} <= syms
    L = C.CDLL(native.LIB_PATH)
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing
    assert set(native.EXPORTS) >= syms


def test_ppo_loss_sizes_and_argument_checks():
    """Host-side contract of duck_ppo_loss (no GPU call): the out array's length and the refusals."""
    lib = native.lib()
    assert [lib.duck_ppo_loss_out_size(n) for n in (0, 1, 128, 129, 5120)] == [6, 9, 30, 33, 966]
    assert lib.duck_ppo_loss(0, 14, *([None] * 7), 0.2, 0.005, 1, None, None, None, None) < 0
    assert b"empty batch" in lib.duck_last_error()
    assert lib.duck_ppo_loss(8, 14, *([None] * 7), 0.2, 0.005, 1, None, None, None, None) < 0
    assert b"null pointer" in lib.duck_last_error()


@pytest.mark.parametrize("nq,nv,nu,imit,task", [(21, 20, 14, 0, 0), (21, 20, 14, 1, 0), (31, 30, 14, 1, 0),
                                                (21, 20, 14, 0, 1), (31, 30, 14, 1, 1)])
def test_layout_matches_c(nq, nv, nu, imit, task):
    lib = native.lib()
    cl = native.DuckLayout()
    assert lib.duck_layout_get(nq, nv, nu, imit, task, C.byref(cl)) == 0
    pl = layout(nq, nv, nu, bool(imit), task)
    for name, _ in native.DuckLayout._fields_:
        v = getattr(cl, name)
        if name in pl.off:
            assert v == pl.off[name], name
        elif name in pl.ioff:
            assert v == pl.ioff[name], name
    assert (cl.nfloat, cl.nint, cl.obs_size, cl.priv_size) == (pl.nfloat, pl.nint, pl.obs_size, pl.priv_size)
    if task == 0:
        assert pl.obs_size == 101 and pl.priv_size == (212 if imit else 172)
    else:  # standing.py: state 85 (3+3+7+14*5+2), privileged 153; no imitation
        assert pl.obs_size == 85 and pl.priv_size == 153 and cl.imitation == 0


def test_dr_layout():
    d = dr_layout(18, 14)
    assert d["nfloat"] == 1 + 3 + 18 + 4 * 14


def test_product_fails_loudly_without_library(monkeypatch, tmp_path):
    monkeypatch.setattr(native, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(native, "_libs", {})
    with pytest.raises(native.DuckError):
        native.lib()


# --- register-allocation fault gate (tools/isa_exec_check.py) ---
_BAD_JOIN = """
_Z6kernelv:
	s_and_saveexec_b64 s[0:1], s[50:51]
	s_cbranch_execz .LBB0_2
	v_add_f32_e32 v1, v2, v3
.LBB0_2:
	v_accvgpr_write_b32 a81, v107
	s_or_b64 exec, exec, s[0:1]
	s_endpgm
"""
_GOOD_JOIN = """
_Z6kernelv:
	s_and_saveexec_b64 s[0:1], s[50:51]
	s_cbranch_execz .LBB0_2
	v_mov_b32_e32 v9, v19
.LBB0_2:
	v_mov_b32_e32 v9, v4
	s_or_b64 exec, exec, s[0:1]
	v_accvgpr_write_b32 a81, v107
	s_endpgm
"""


def _isa_check_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_exec_check", os.path.join(ROOT, "tools", "isa_exec_check.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_isa_check_flags_lane_masked_split_copies():
    """The checker flags an AGPR move ahead of a join's exec restore (the pattern that cost lanes
    14-15 their LDS row address in the max-ILP physics_kernel) and accepts a region phi copy."""
    mod = _isa_check_module()
    assert len(mod.scan(_BAD_JOIN, "bad")) == 1
    assert mod.scan(_GOOD_JOIN, "good") == []


@pytest.mark.skipif(not os.path.exists(native.LIB_PATH), reason="libduck.so not built")
def test_built_library_has_no_lane_masked_split_copies():
    """Every kernel of the shipped libduck.so (all four scenes, max-ILP schedule) is free of
    register moves placed ahead of an exec restore -- and the gate really disassembled them: the
    objdump path build() uses finds the step / physics / reset kernels of every scene."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_exec_check", os.path.join(ROOT, "tools", "isa_exec_check.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    kern = native.isa_kernels(mod.code_objects(native.LIB_PATH))
    for scene in ("flat", "backlash", "rough", "rough_backlash"):
        for k in ("step_kernel", "physics_kernel", "reset_kernel"):
            sym = f"DuckModel_{scene}"
            assert any(k in x and f"{len(sym)}{sym}" in x for x in kern), (k, scene, kern)
    assert native.isa_exec_faults(native.LIB_PATH, min_step_kernels=4) == []


def test_isa_gate_fails_closed(tmp_path):
    """A library without gfx950 code objects (here: a host-only shared object) is an error for the
    gate, not a clean bill of health."""
    import subprocess
    src = tmp_path / "x.c"
    src.write_text("int f(void) { return 1; }\n")
    so = tmp_path / "libx.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)])
    with pytest.raises(native.DuckError):
        native.isa_exec_faults(str(so))


def test_round4_entry_points_refuse_bad_arguments():
    """Host-side checks of the round-4 C-ABI entries (no GPU call is reached): the grouped MLP launch,
    the minibatch gather and the step-mode switch refuse malformed arguments with a message."""
    import ctypes as C
    from open_duck_playground_amd.native import DuckGatherField, DuckMlpProblem
    lib = native.lib()
    assert lib.duck_mlp_group(5, (DuckMlpProblem * 5)(), None) < 0
    assert b"problems" in lib.duck_last_error()
    bad = (DuckMlpProblem * 1)(DuckMlpProblem(7, 8, 8, 8))
    assert lib.duck_mlp_group(1, bad, None) < 0 and b"kind" in lib.duck_last_error()
    nul = (DuckMlpProblem * 1)(DuckMlpProblem(1, 8, 8, 8))  # operands missing
    assert lib.duck_mlp_group(1, nul, None) < 0 and b"operands" in lib.duck_last_error()
    off = (DuckMlpProblem * 1)(DuckMlpProblem(3, 64, 8, 8, 1, 1, None, None, None, None, None, None, 2, 10, 0, 0, 1))
    assert lib.duck_mlp_group(1, off, None) < 0 and b"offsets" in lib.duck_last_error()
    assert lib.duck_mlp_group(0, None, None) == 0
    assert lib.duck_gather_columns(9, (DuckGatherField * 9)(), C.c_void_p(1), 4, None) < 0
    f = (DuckGatherField * 1)(DuckGatherField(None, None, 2, 4, 3))
    assert lib.duck_gather_columns(1, f, C.c_void_p(1), 4, None) < 0 and b"bad field" in lib.duck_last_error()
    assert lib.duck_set_step_mode(None, 0) < 0
    assert lib.duck_step_kernel_for(None, 4) < 0


def test_bench_self_launch_command(monkeypatch, capsys):
    """bench.py --gpus N (N > 1, no WORLD_SIZE) starts torch.distributed.run as a child with the same
    arguments and returns its exit code; --gpus 1 runs in-process. No GPU call here."""
    import subprocess
    import sys
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    seen = {}

    class FakePopen:
        def __init__(self, cmd, env=None, **kw):
            seen["cmd"], seen["env"] = cmd, env
            # what the ranks write: gloo's peer notice glued to the front of rank 0's line
            self.stdout = iter(["[Gloo] Rank 0 is connected to 1 peer ranks.[Gloo] Rank\n",
                                '1 is connected{"metric": "m", "value": 1}\n'])

        def wait(self):
            return 7

    monkeypatch.setattr(subprocess, "Popen", FakePopen)
    assert bench._self_launch(["--gpus", "1", "--steps", "3"]) == -1 and not seen
    assert bench._self_launch(["--gpus", "4", "--steps", "3", "--strong"]) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3", "--strong"][-4:] and cmd[-5] == "--gpus"
    assert os.path.basename(cmd[-6]) == "bench.py"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench._self_launch(["--gpus=2"]) == 7 and "--nproc-per-node=2" in seen["cmd"]
    out = capsys.readouterr()
    assert out.out.splitlines() == ['{"metric": "m", "value": 1}'] * 2     # stdout: only the bench lines
    assert "[Gloo]" in out.err and "1 is connected" in out.err
