"""The teacher-forcing outliers dumped on MI355X by tools/diag_tf_substep.py in round 3
(profiles/r03_tf_long/: every substep, at rough + DR and rough + DR + backlash over 1024 envs x 10
env-steps, where the kernel and the oracle differed beyond 1e-3 from the same input), checked against
the oracle on the CPU: every one is a contact-generation difference -- the oracle continued from the
kernel's own contact set (oracle_set_con_override) lands on the kernel's substep to fp32 (<= 1e-5);
kinematics, mass matrix, constraint rows, the Newton solve and the integration agree at all of them.

Those contact differences were SAT near-ties (env 377: a prism side face and a vertical-edge pair within
1e-7 m) and onset prisms whose penetration-weighted point had ~1e-7 m weights (env 335). Round 4 made
the contact model continuous there (the tie-band blend of the two smallest
overlaps' axes, the point band), and the teacher-forcing rules that accepted them ("sat_tie",
"onset_cascade") are gone; the dumps stay as the record of what the kernel computed then."""
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
        assert _state_rel(m, g, oracle_substep_with_contacts(om, x, ga)) <= 1e-5, e
