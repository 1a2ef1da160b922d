"""The teacher-forcing outliers dumped on MI355X by tools/diag_tf_substep.py in round 3
(profiles/r03_tf_long/: every substep, at rough + DR and rough + DR + backlash over 1024 envs x 10
env-steps, where the kernel and the oracle differed beyond 1e-3 from the same input), checked against
the oracle on the CPU: every one is a contact-generation difference -- the oracle continued from the
kernel's own contact set (oracle_set_con_override) lands on the kernel's substep to fp32 (<= 1e-5);
kinematics, mass matrix, constraint rows, the Newton solve and the integration agree at all of them.

Those contact differences were SAT near-ties (env 377: a prism side face and a vertical-edge pair within
1e-7 m) and onset prisms whose penetration-weighted point had ~1e-7 m weights (env 335). Round 4 made
the point continuous at the onset (the point band); a two-axis blend at SAT ties
was tried and made fp32 and fp64 differ more often (10 -> 43 long-case outliers), so near-ties stay a
declared fp32 behaviour ("sat_tie": the oracle resolving a tie within 1e-6 m to the other axis lands on
the kernel). The round-4 dump (profiles/r04_tf/, rough + DR, 256 envs x 6 env-steps on MI355X) holds
the mirror case of env 377: the fp64 minimum is a vertical-edge pair below a prism side face by less
than 1e-6 m, the kernel's fp32 overlaps pick the side face (the first axis in the band)."""
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


def test_round4_tie_first_outlier():
    """profiles/r04_tf/diag_tf_rough_dr.npz, env 242 (step 4, substep 2): same contacts except one
    prism's normal, (0, 1, 0) on the kernel -- a side face -- and (0.0072, 0.99997, 0) in the oracle --
    a vertical-edge pair overlapping less by under 1e-6 m. The oracle taking the first axis within
    1e-6 m of the minimum (oracle_set_hf_tie_first) lands on the kernel; the default rule does not."""
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.mjcf import Model
    from tests.oracle_ffi import OracleModel, lib
    m = Model.load(constants.task_to_xml(CASES["rough_dr"]["task"]))
    base = OracleModel(m)
    z = np.load(os.path.join(ROOT, "profiles", "r04_tf", "diag_tf_rough_dr.npz"))
    i = list(z["env"]).index(242)
    om = OracleModel(m, dr=base.dr_sample(7 + 1, 242))
    x, g = z["x"][i], z["gnext"][i]
    assert _state_rel(m, g, oracle_substep(om, x)) > 1e-3
    lib().oracle_set_hf_tie_first(1e-6)
    try:
        assert _state_rel(m, g, oracle_substep(om, x)) <= 1e-5
    finally:
        lib().oracle_set_hf_tie_first(0.0)
