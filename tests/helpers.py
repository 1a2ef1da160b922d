"""Shared test helpers: random physics states, aux-record parsing."""

import numpy as np

from open_duck_playground_amd.codegen import sparse_pattern
from open_duck_playground_amd.mjcf import Model, quat_mul, axis_angle_quat


def random_states(m: Model, n: int, seed: int, height=(0.14, 0.20), tilt=0.15, vel=0.3):
    """Near-keyframe states (feet near/through the floor), SoA-friendly [n, k] arrays."""
    rng = np.random.default_rng(seed)
    key = m.key_qpos[0]
    qpos = np.tile(key, (n, 1))
    qpos[:, 0:2] += rng.uniform(-0.05, 0.05, (n, 2))
    qpos[:, 2] = rng.uniform(*height, n)
    for e in range(n):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        q = quat_mul(axis_angle_quat([0, 0, 1], rng.uniform(-3.14, 3.14)), axis_angle_quat(ax, rng.uniform(-tilt, tilt)))
        qpos[e, 3:7] = q
    act_q = np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])
    qpos[:, act_q] *= rng.uniform(0.7, 1.3, (n, len(act_q)))
    qvel = rng.uniform(-vel, vel, (n, m.nv))
    ctrl = m.key_ctrl[0] + rng.uniform(-0.2, 0.2, (n, m.nu))
    return qpos, qvel, ctrl


def parse_aux(m: Model, aux: np.ndarray):
    """aux [K, n] -> dict of [n, k] arrays (layout of Phys::write_aux)."""
    nv, nu, nsd = m.nv, m.nu, m.nsensordata
    ncon = 4 * m.npair
    _, adr, nm = sparse_pattern(m)
    out, o = {}, 0
    for name, k in (("qacc", nv), ("qacc_smooth", nv), ("qvel", nv), ("qfrc_smooth", nv), ("actuator_force", nu),
                    ("sensordata", nsd), ("con_dist", ncon), ("con_pos", 3 * ncon), ("con_normal", 3 * ncon),
                    ("M", nm)):
        out[name] = aux[o:o + k].T
        o += k
    n = aux.shape[1]
    Md = np.zeros((n, nv, nv))
    for i in range(nv):
        for j in range(nv):
            if adr[i, j] >= 0:
                Md[:, i, j] = out["M"][:, adr[i, j]]
                Md[:, j, i] = out["M"][:, adr[i, j]]
    out["Mdense"] = Md
    return out
