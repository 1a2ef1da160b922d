"""One substep of the physics kernel from states dumped by tools/diag_tf_substep.py, with the library
named by DUCK_LIB (e.g. an older build from tools/ab_build.sh): does the result depend on the build?
usage: DUCK_LIB=... python tools/diag_substep_lib.py <case> <env> [envs]  -> prints the distance to the
dumped GPU result and to the dumped oracle result."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests.teacher_forcing import _state_rel, gpu_substep, run_case
    case, e = sys.argv[1], int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    z = np.load(os.path.join(ROOT, "profiles", "r03_tf_long", f"diag_tf_{case}.npz"))
    i = [k for k in range(len(z["env"])) if int(z["env"][k]) == e][0]
    rep = run_case(case, "cuda:0", n=n, steps=1)
    m = rep.env.mj_model
    g = gpu_substep(rep.env, e, z["x"][i])
    print(f"{case} env {e}: this build vs dumped GPU {_state_rel(m, g, z['gnext'][i]):.3e}, "
          f"vs oracle {_state_rel(m, g, z['rnext'][i]):.3e} (dumped GPU vs oracle "
          f"{_state_rel(m, z['gnext'][i], z['rnext'][i]):.3e})")


if __name__ == "__main__":
    main()
