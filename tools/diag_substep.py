#!/usr/bin/env python3
"""Field-by-field HIP vs oracle errors after one substep (debug aid for test_substep_parity)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.test_gpu_physics import _run  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "rough_terrain_backlash"
for nsub in (0, 1):
    m, g, r = _run(task, 64, nsub, seed=2, gpu="cuda:0")
    print("nsub", nsub)
    for k in ("qacc_smooth", "qacc", "sensordata", "con_dist", "actuator_force"):
        a = g[k]
        b = r[{"actuator_force": "af"}.get(k, k)]
        err = np.abs(a - b).max(axis=1)
        print(f"  {k:14s} median {np.median(err):.3e} max {err.max():.3e} finite {np.isfinite(a).all()}")
    Md = g["Mdense"]
    print("  M max err %.3e" % np.abs(Md - r["M"]).max())
    print("  qpos_out finite", np.isfinite(g["qpos_out"]).all(), "qvel_out max", np.abs(g["qvel_out"]).max())
