"""The teacher-forcing outliers dumped on MI355X by tools/diag_tf_substep.py (profiles/r03_tf_long/:
every substep, at rough + DR and rough + DR + backlash over 1024 envs x 10 env-steps, where the kernel
and the oracle differ beyond 1e-3 from the same input), checked against the oracle on the CPU.

1. Every one is a contact-generation difference: the oracle continued from the kernel's own contact
   set (oracle_set_con_override) lands on the kernel's substep to fp32 (<= 1e-5). Kinematics, mass
   matrix, constraint rows, the Newton solve and the integration agree at all of them.

2. The height-field SAT near-tie rule of teacher forcing's `declared_difference` ("sat_tie"), on the
substep dumped by tools/diag_tf_substep.py at rough + DR + backlash, env-step 7, env 377
(profiles/r03_tf_long/): a foot/prism pair whose prism side face and a vertical-edge pair overlap
within 1e-7 m. The HIP kernel's fp32 overlaps took the edge pair, the oracle (first axis of the
declared priority order) the side face: same depth and point, normals 2.9 degrees apart, and a Newton
step 1.5e-2 apart. The oracle resolving the tie to the other axis lands on the kernel's result."""
import ctypes as C
import os

import numpy as np

import pytest

from tests.teacher_forcing import CASES, _split, _state_rel, oracle_substep, oracle_substep_with_contacts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "profiles", "r03_tf_long", "diag_tf_rough_backlash_dr.npz")


@pytest.mark.parametrize("case", ["rough_dr", "rough_backlash_dr"])
def test_dumped_outliers_are_contact_generation_differences(case):
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.mjcf import Model
    from tests.helpers import parse_aux
    from tests.oracle_ffi import OracleModel
    spec = CASES[case]
    m = Model.load(constants.task_to_xml(spec["task"]))
    base = OracleModel(m)
    z = np.load(os.path.join(ROOT, "profiles", "r03_tf_long", f"diag_tf_{case}.npz"))
    assert len(z["env"]) >= 8
    for i in range(len(z["env"])):
        e = int(z["env"][i])
        om = OracleModel(m, dr=base.dr_sample(7 + 1, e)) if spec.get("dr") else base
        x, g = z["x"][i], z["gnext"][i]
        ga = parse_aux(m, z["aux"][i][:, None])
        assert _state_rel(m, g, oracle_substep(om, x)) > 1e-4, e          # a real outlier
        assert _state_rel(m, g, oracle_substep_with_contacts(om, x, ga)) <= 1e-5, e


def test_onset_prism_cascade_explains_env_335():
    """Env-step 9, env 335: the right foot over four penetrating prisms (17.3, 15.1, 2.0 mm and 1e-7 m).
    The onset prism's point has ~1e-7 weights, so the two sides place it 1.6 cm apart and the manifold
    keeps different slots; the "onset_cascade" rule: the differing pair holds an onset-depth contact, and
    the oracle from the kernel's contacts lands on the kernel."""
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.mjcf import Model
    from tests.helpers import parse_aux
    from tests.oracle_ffi import OracleModel
    spec = CASES["rough_backlash_dr"]
    m = Model.load(constants.task_to_xml(spec["task"]))
    z = np.load(DUMP)
    i = [k for k in range(len(z["env"])) if int(z["env"][k]) == 335][0]
    om = OracleModel(m, dr=OracleModel(m).dr_sample(7 + 1, 335))
    x, g = z["x"][i], z["gnext"][i]
    ga = parse_aux(m, z["aux"][i][:, None])
    q, v, w, c = _split(m, x)
    d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
    om.forward(d)
    ncon = 4 * m.npair
    gd, od = ga["con_dist"][0][:ncon], d.arr("con_dist", ncon)
    gp, op = ga["con_pos"][0].reshape(-1, 3)[:ncon], np.ctypeslib.as_array(d.con_pos)[:ncon]
    differ = ((gd < 0) != (od < 0)) | ((gd < 0) & (od < 0) & (np.abs(gp - op).max(axis=1) > 1e-4))
    onset = (((gd < 0) & (gd >= -1e-6)) | ((od < 0) & (od >= -1e-6))).reshape(m.npair, 4).any(axis=1)
    pd = differ.reshape(m.npair, 4).any(axis=1)
    assert pd.any() and onset[pd].all()
    assert _state_rel(m, g, oracle_substep(om, x)) > 0.5
    assert _state_rel(m, g, oracle_substep_with_contacts(om, x, ga)) <= 1e-5


def test_hfield_sat_near_tie_explains_env_377():
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.mjcf import Model
    from tests.oracle_ffi import OracleModel, lib
    spec = CASES["rough_backlash_dr"]
    m = Model.load(constants.task_to_xml(spec["task"]))
    z = np.load(DUMP)
    i = [k for k in range(len(z["env"])) if int(z["env"][k]) == 377][0]
    om = OracleModel(m, dr=OracleModel(m).dr_sample(7 + 1, 377))
    x, g = z["x"][i], z["gnext"][i]
    r0 = oracle_substep(om, x)
    assert _state_rel(m, g, r0) > 1e-2                     # the declared rule: 1.5e-2 from the kernel
    lib().oracle_set_hf_tie_last(1e-6)
    try:
        r1 = oracle_substep(om, x)
    finally:
        lib().oracle_set_hf_tie_last(0.0)
    assert _state_rel(m, g, r1) <= 1e-4                    # the other tied axis: the kernel's result
    assert _state_rel(m, oracle_substep(om, x), r0) == 0   # the aid is off again
    # the Newton Hessian is well conditioned and no row is near its active-set boundary: the
    # difference is the contact normal, not the solve
    NV = 32
    buf = np.zeros(1 + NV * NV + 3 * 256)
    lib().oracle_set_hdump(buf.ctypes.data_as(C.POINTER(C.c_double)))
    try:
        q, v, w, c = _split(m, x)
        d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
        om.forward(d)
    finally:
        lib().oracle_set_hdump(None)
    nefc = int(buf[0])
    H = buf[1:1 + NV * NV].reshape(NV, NV)[:m.nv, :m.nv]
    ev = np.linalg.eigvalsh(H)
    assert ev[0] > 0 and ev[-1] / ev[0] < 1e4
    rows = buf[1 + NV * NV:1 + NV * NV + 3 * nefc].reshape(nefc, 3)
    marg = np.where(rows[:, 2] == 0, np.abs(rows[:, 0]), np.abs(np.abs(rows[:, 0]) - rows[:, 2])) / rows[:, 1]
    assert marg.min() > 1e-2
