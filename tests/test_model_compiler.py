"""The kernels are specialised per model like MJX specialises per MJCF (codegen.py,
native.model_library): the C-ABI fingerprint binds a model to its compiled kernels, the shipped
library holds the four Open Duck scenes, and an edited scene gets a library of its own.
CPU-only checks (the libraries load without a GPU); tests/test_gpu_models.py runs them."""

import ctypes as C
import glob
import os

import numpy as np
import pytest

from open_duck_playground_amd import codegen, constants, native
from open_duck_playground_amd.cabi import ModelDescHolder, model_fingerprint
from open_duck_playground_amd.mjcf import Model
from tests.kat_checks import MODELS

SHIPPED = ["flat_terrain", "flat_terrain_backlash", "rough_terrain", "rough_terrain_backlash"]
EDITED = sorted(glob.glob(os.path.join(MODELS, "*.npz")))


def _fp_c(lib, m):
    h = ModelDescHolder(m)
    return int(lib.duck_model_fingerprint(C.byref(h.desc))), int(lib.duck_model_supported(C.byref(h.desc)))


@pytest.mark.parametrize("path", [constants.task_to_xml(t) for t in SHIPPED] + EDITED)
def test_fingerprint_c_equals_python(path):
    m = Model.load(path)
    fp, _ = _fp_c(native.lib(), m)
    assert fp == model_fingerprint(m)


def test_shipped_library_holds_exactly_the_four_scenes():
    L = native.lib()
    for t in SHIPPED:
        assert _fp_c(L, Model.load(constants.task_to_xml(t)))[1] == 1
        assert native.model_library(Model.load(constants.task_to_xml(t))) == native.LIB_PATH
    for p in EDITED:
        assert _fp_c(L, Model.load(p))[1] == 0


@pytest.mark.parametrize("path", EDITED)
def test_edited_scene_gets_its_own_library(path):
    m = Model.load(path)
    lib_path = native.model_library(m)   # built by __graft_entry__.build(); up to date here
    assert lib_path != native.LIB_PATH and os.path.exists(lib_path)
    L = native.lib(lib_path)
    assert _fp_c(L, m) == (model_fingerprint(m), 1)
    for sym in native.EXPORTS:
        if not sym.startswith(("duck_gae", "duck_ppo", "duck_mlp", "duck_policy", "duck_clip", "duck_gather",
                               "duck_column_stats")):  # the PPO kernels ship with libduck.so only
            assert hasattr(L, sym), sym


def test_generated_headers_match_the_assets():
    for var, task in codegen.DEFAULT_VARIANTS:
        m = Model.load(constants.task_to_xml(task))
        hdr = os.path.join(native.CSRC, "generated", f"duck_model_{var}.h")
        assert open(hdr).read() == codegen.model_header(m, var), var


def test_fingerprint_sees_every_baked_edit():
    base = Model.load(constants.task_to_xml("flat_terrain"))
    fp0 = model_fingerprint(base)
    for key, k in (("dof_damping", 8), ("actuator_kp", 3), ("body_mass", 5), ("jnt_range", 4)):
        m = Model.load(constants.task_to_xml("flat_terrain"))
        a = m.arrays[key].copy()
        a.flat[k] *= 1.01
        m.arrays[key] = a
        assert model_fingerprint(m) != fp0, key
    m = Model.load(constants.task_to_xml("rough_terrain"))
    m2 = Model.load(constants.task_to_xml("rough_terrain"))
    m2.arrays["hfield_data"] = np.zeros_like(m2.arrays["hfield_data"])  # uploaded at create, not baked
    assert model_fingerprint(m) == model_fingerprint(m2)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference XMLs (build container)")
def test_edited_scenes_are_reproducible_from_the_xml():
    """The committed test scenes are exactly what the model compiler makes of the edited reference
    XML (tools/build_assets.py EDITED), and the shipped flat scene of the unedited XML."""
    import sys
    import tempfile
    sys.path.insert(0, os.path.join(os.path.dirname(MODELS), "..", "..", "tools"))
    import build_assets as B
    from open_duck_playground_amd.mjcf import compile_mjcf
    for name, (re_, se) in B.EDITED.items():
        with tempfile.TemporaryDirectory() as td:
            m = compile_mjcf(B.edited_scene(td, re_, se), timestep=0.002)
        assert model_fingerprint(m) == model_fingerprint(Model.load(os.path.join(MODELS, f"{name}.npz"))), name
    with tempfile.TemporaryDirectory() as td:
        m = compile_mjcf(B.edited_scene(td, [], []), timestep=0.002)
    assert model_fingerprint(m) == model_fingerprint(Model.load(constants.task_to_xml("flat_terrain")))


def _header_tables(variant):
    """The blob and the scalar constants of a generated model header (codegen.model_header)."""
    import re
    txt = open(os.path.join(native.CSRC, "generated", f"duck_model_{variant}.h")).read()
    blob = np.array([int(x) for x in re.search(r"_blob\[\d+\] = \{([^}]*)\}", txt).group(1).split(",")])
    const = {k: int(v) for k, v in re.findall(r"\b([A-Z][A-Z0-9_]*) = (-?\d+)", txt)}
    brb = re.search(r"T_BRB\[(\d+)\]\[(\d+)\] = \{(.*?)\};", txt)
    nbr, brlen = int(brb.group(1)), int(brb.group(2))
    t_brb = np.array([int(x) for x in re.findall(r"-?\d+", brb.group(3))]).reshape(nbr, brlen)
    return blob, const, t_brb


@pytest.mark.parametrize("variant", ["flat", "backlash", "rough", "rough_backlash"])
def test_register_column_table_points_outside_entries_at_the_zero_word(variant):
    """load_cols' per-lane table (codegen mcolz): entry (s, r, lane) is M's address of (row r,
    column 16 s + lane) where the tree pattern has one, else NM, the zero word after M."""
    blob, c, _ = _header_tables(variant)
    nv, nm = c["NV"], c["NM"]
    nc = (nv + 15) // 16
    madr = blob[c["B_MADR"]:c["B_MADR"] + nv * nv].reshape(nv, nv)
    mcolz = blob[c["B_MCOLZ"]:c["B_MCOLZ"] + nc * nv * 16].reshape(nc, nv, 16)
    for s in range(nc):
        for r in range(nv):
            for ln in range(16):
                col = 16 * s + ln
                want = madr[r, col] if col < nv and madr[r, col] >= 0 else nm
                assert mcolz[s, r, ln] == want, (s, r, ln)
    assert sorted(set(madr[madr >= 0].tolist())) == list(range(nm))  # every M entry addressed once per pair


@pytest.mark.parametrize("variant", ["flat", "backlash", "rough", "rough_backlash"])
def test_compile_time_limb_bodies_match_the_blob(variant):
    """rne's component-per-lane subtree sums walk Md::T_BRB; the other passes read the blob's copy."""
    blob, c, t_brb = _header_tables(variant)
    nbr, brlen = t_brb.shape
    assert nbr == c["T_NBR"] and brlen == c["T_BRLEN"]
    assert (blob[c["B_BR"]:c["B_BR"] + nbr * brlen].reshape(nbr, brlen) == t_brb).all()
