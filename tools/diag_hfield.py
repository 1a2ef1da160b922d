#!/usr/bin/env python3
"""Dump the HIP forward's floor contacts for random rough-terrain states (GPU side of the
height-field parity check; compare on the CPU with the oracle: tools/diag_hfield.py compare)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def states(task, n, seed, height):
    from open_duck_playground_amd.joystick import Joystick
    from tests.helpers import random_states
    from open_duck_playground_amd.mjcf import Model
    from open_duck_playground_amd import constants
    m = Model.load(constants.task_to_xml(task))
    return m, random_states(m, n, seed, height=height)


def run(task="rough_terrain", n=1024, seed=11, height=(0.14, 0.20)):
    import torch
    from open_duck_playground_amd.joystick import Joystick
    from tests.helpers import parse_aux
    env = Joystick(task, num_envs=1, device="cuda:0", use_imitation=False)
    m, (qpos, qvel, ctrl) = states(task, n, seed, height)
    T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device="cuda:0")  # noqa: E731
    aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device="cuda:0").view(-1, n)
    env.physics_step(T(qpos), T(qvel), T(np.zeros((n, m.nv))), T(ctrl), 0, aux)
    torch.cuda.synchronize()
    g = parse_aux(m, aux.cpu().numpy().astype(np.float64))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"diag_hfield_{task}.npz"), con_dist=g["con_dist"], con_pos=g["con_pos"])


def compare(task="rough_terrain", n=1024, seed=11, height=(0.14, 0.20), show=5):
    from tests.oracle_ffi import OracleModel
    m, (qpos, qvel, ctrl) = states(task, n, seed, height)
    z = np.load(os.path.join(ROOT, "gpurun_out", f"diag_hfield_{task}.npz"))
    om = OracleModel(m)
    bad = 0
    for e in range(n):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        rd = d.arr("con_dist", 4 * m.npair)
        rp = np.ctypeslib.as_array(d.con_pos)[:4 * m.npair]
        gd, gp = z["con_dist"][e], z["con_pos"][e].reshape(-1, 3)
        act = (gd < 0) | (rd < 0)
        if np.any((np.abs(gd - rd) > 2e-5) & act):
            bad += 1
            if bad <= show:
                print("env", e)
                for s in range(4, 4 * m.npair):
                    print(f"  slot {s}: gpu {gd[s]: .6f} {gp[s]}  oracle {rd[s]: .6f} {rp[s]}")
    print("bad", bad, "of", n)




def stats(task="rough_terrain", n=1024, seed=11, height=(0.14, 0.20)):
    from tests.oracle_ffi import OracleModel
    m, (qpos, qvel, ctrl) = states(task, n, seed, height)
    z = np.load(os.path.join(ROOT, "gpurun_out", f"diag_hfield_{task}.npz"))
    om = OracleModel(m)
    dd, dp = [], []
    for e in range(n):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        om.forward(d)
        rd = d.arr("con_dist", 4 * m.npair)
        rp = np.ctypeslib.as_array(d.con_pos)[:4 * m.npair]
        gd, gp = z["con_dist"][e], z["con_pos"][e].reshape(-1, 3)
        for s in range(4, 4 * m.npair):
            if rd[s] < 0 and gd[s] < 0 and abs(rd[s] - gd[s]) < 1e-4:
                dd.append(abs(rd[s] - gd[s]))
                dp.append(np.abs(rp[s] - gp[s]).max())
    dd, dp = np.array(dd), np.array(dp)
    q = lambda a: " ".join(f"{x:.2e}" for x in np.quantile(a, [0.5, 0.9, 0.99, 1.0]))  # noqa: E731
    print("depth |diff| p50 p90 p99 max:", q(dd))
    print("pos   |diff| p50 p90 p99 max:", q(dp))


if __name__ == "__main__":
    {"compare": compare, "stats": stats}.get(sys.argv[1] if len(sys.argv) > 1 else "", run)()
