#!/usr/bin/env python3
"""How often the feet touch each other (the foot/foot hull pair has an active contact) in the
benchmark workloads: oracle rollouts of C2..C5 scenes with U(-1,1) actions, every substep of every
env-step sampled. Bounds the practical weight of DESIGN.md §5 item 1 (the hull/hull manifold is a
face manifold or one edge point instead of MJX's polygon clipping). CPU only.

usage: python tools/foot_foot_frequency.py [n_envs] [n_steps]   (one JSON line per scene)
"""

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from open_duck_playground_amd import constants  # noqa: E402
from open_duck_playground_amd.config import default_config, env_config_struct  # noqa: E402
from open_duck_playground_amd.mjcf import Model  # noqa: E402
from tests.oracle_ffi import OracleEnv, OracleModel, lib  # noqa: E402


def measure(task, dr, n_envs, n_steps, seed=0):
    m = Model.load(constants.task_to_xml(task))
    base = OracleModel(m)
    cfg = env_config_struct(m, default_config(), False, domain_randomize=dr)
    lf, rf = m.id("geom", "left_foot_bottom_tpu"), m.id("geom", "right_foot_bottom_tpu")
    p = [k for k in range(m.npair) if {int(m.pair_geom1[k]), int(m.pair_geom2[k])} == {lf, rf}][0]
    rng = np.random.default_rng(seed)
    K = m.nq + 2 * m.nv + m.nu
    touch = total = 0
    for e in range(n_envs):
        om = OracleModel(m, dr=base.dr_sample(seed + 1, e)) if dr else base
        env = OracleEnv(om, cfg)
        env.reset(seed=seed, env_id=e)
        tr = np.zeros((cfg.n_substeps, K))
        for t in range(n_steps):
            lib().oracle_set_trace(tr.ctypes.data_as(C.POINTER(C.c_double)))
            env.step(rng.uniform(-1, 1, m.nu))
            lib().oracle_set_trace(None)
            for s in range(cfg.n_substeps):   # forward at each substep's input: its contacts
                x = tr[s]
                d = om.new_data(qpos=x[:m.nq], qvel=x[m.nq:m.nq + m.nv], warm=x[m.nq + m.nv:m.nq + 2 * m.nv],
                                ctrl=x[m.nq + 2 * m.nv:])
                om.forward(d)
                touch += int((d.arr("con_dist", 4 * m.npair)[4 * p:4 * p + 4] < 0).any())
                total += 1
    return {"scene": task, "dr": dr, "env_substeps": total, "foot_foot_contact_substeps": touch,
            "fraction": touch / total}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    for task, dr in (("flat_terrain", False), ("flat_terrain_backlash", False), ("rough_terrain", True),
                     ("rough_terrain_backlash", True)):
        print(json.dumps(measure(task, dr, n, steps)), flush=True)


if __name__ == "__main__":
    main()
