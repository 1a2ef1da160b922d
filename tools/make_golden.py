#!/usr/bin/env python3
"""Generate golden vectors from the reference's own NumPy twins (build container only).

Uses, by file path under /root/reference (imported, never copied):
  playground/common/rewards_numpy.py            (twin of common/rewards.py)
  playground/open_duck_mini_v2/custom_rewards_numpy.py   (twin of custom_rewards.py)
  playground/common/poly_reference_motion_numpy.py       (twin of poly_reference_motion.py)
The reference-motion class is instantiated without its constructor (which unpickles the
table); its own ``process`` is fed the table decoded by refmotion.read_poly_pkl, which
interprets pickle opcodes as data without executing anything.

Writes tests/golden/rewards.npz and tests/golden/refmotion.npz (inputs + expected outputs).
"""

import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(__file__), "..")
sys.path.insert(0, ROOT)
from open_duck_playground_amd.refmotion import read_poly_pkl  # noqa: E402

REF = "/root/reference/playground"
OUT = os.path.join(ROOT, "tests", "golden")


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    os.makedirs(OUT, exist_ok=True)
    rw = load("ref_rewards_numpy", f"{REF}/common/rewards_numpy.py")
    cr = load("ref_custom_rewards_numpy", f"{REF}/open_duck_mini_v2/custom_rewards_numpy.py")
    pm = load("ref_poly_numpy", f"{REF}/common/poly_reference_motion_numpy.py")
    rng = np.random.default_rng(20250410)
    n, nu = 256, 14
    cmd = rng.uniform(-1, 1, (n, 7)) * np.array([0.15, 0.2, 1.0, 1.0, 0.8, 1.5, 0.5])
    cmd[::10] = 0.0                      # zero commands (stand-still / imitation gates)
    cmd[5::17, :3] = 0.004               # |cmd| just under the 0.01 gate
    local_linvel = rng.normal(0, 0.2, (n, 3))
    gyro = rng.normal(0, 0.5, (n, 3))
    af = rng.uniform(-3.23, 3.23, (n, nu))
    act = rng.uniform(-1, 1, (n, nu))
    last_act = rng.uniform(-1, 1, (n, nu))
    default = np.array([0.002, 0.053, -0.63, 1.368, -0.784, 0, 0, 0, 0, -0.003, -0.065, 0.635, 1.379, -0.796])
    jq = default + rng.normal(0, 0.1, (n, nu))
    jqd = rng.normal(0, 1.0, (n, nu))
    base_qpos = np.concatenate([rng.normal(0, 0.1, (n, 3)), rng.normal(0, 1, (n, 4))], axis=1)
    base_qvel = rng.normal(0, 0.3, (n, 6))
    contacts = rng.integers(0, 2, (n, 2)).astype(np.float64)
    ref = rng.normal(0, 0.5, (n, 40))
    ref[:, 32:34] = rng.uniform(0, 1, (n, 2))
    sigma = 0.01
    out = np.zeros((n, 7))
    for i in range(n):
        out[i, 0] = rw.reward_tracking_lin_vel(cmd[i], local_linvel[i], sigma)
        out[i, 1] = rw.reward_tracking_ang_vel(cmd[i], gyro[i], sigma)
        out[i, 2] = rw.cost_torques(af[i])
        out[i, 3] = rw.cost_action_rate(act[i], last_act[i])
        out[i, 4] = rw.cost_stand_still(cmd[i], jq[i], jqd[i], default, ignore_head=False)
        out[i, 5] = rw.reward_alive()
        out[i, 6] = cr.reward_imitation(base_qpos[i], base_qvel[i], jq[i], jqd[i], contacts[i], ref[i], cmd[i], True)
    np.savez_compressed(os.path.join(OUT, "rewards.npz"), cmd=cmd, local_linvel=local_linvel, gyro=gyro,
                        actuator_force=af, action=act, last_act=last_act, joints_qpos=jq, joints_qvel=jqd,
                        default_actuator=default, base_qpos=base_qpos, base_qvel=base_qvel, contacts=contacts,
                        reference_frame=ref, tracking_sigma=np.array(sigma),
                        expected=out,
                        columns=np.array(["tracking_lin_vel", "tracking_ang_vel", "torques", "action_rate",
                                          "stand_still", "alive", "imitation"]))
    # Standing reward terms (standing.py:584-606): orientation on the upvector, stand_still over
    # the legs (ignore_head=True), head_pos; the same random inputs plus an upvector
    up = np.random.default_rng(7).normal(0, 0.3, (n, 3))  # own stream: the cases below stay put
    up[:, 2] += 1.0
    st = np.zeros((n, 6))
    for i in range(n):
        st[i, 0] = rw.cost_orientation(up[i])
        st[i, 1] = rw.cost_torques(af[i])
        st[i, 2] = rw.cost_action_rate(act[i], last_act[i])
        st[i, 3] = rw.reward_alive()
        st[i, 4] = rw.cost_stand_still(cmd[i], jq[i], jqd[i], default, True)
        st[i, 5] = rw.cost_head_pos(jq[i], jqd[i], cmd[i])
    np.savez_compressed(os.path.join(OUT, "standing_rewards.npz"), cmd=cmd, upvector=up, actuator_force=af,
                        action=act, last_act=last_act, joints_qpos=jq, joints_qvel=jqd, default_actuator=default,
                        expected=st, columns=np.array(["orientation", "torques", "action_rate", "alive",
                                                       "stand_still", "head_pos"]))
    # reference motion
    data = read_poly_pkl(f"{REF}/open_duck_mini_v2/data/polynomial_coefficients.pkl")
    prm = pm.PolyReferenceMotion.__new__(pm.PolyReferenceMotion)
    for k, v in dict(dx_range=[0, 0], dy_range=[0, 0], dtheta_range=[0, 0], dxs=[], dys=[], dthetas=[],
                     data_array=[], period=None, fps=None, frame_offsets=None,
                     startend_double_support_ratio=None, start_offset=None, nb_steps_in_period=None).items():
        setattr(prm, k, v)
    prm.process(data)
    cases = []
    for ix, dx in enumerate(prm.dxs):           # every grid cell at two phases
        for dy in prm.dys:
            for dth in prm.dthetas:
                cases.append((dx, dy, dth, (ix * 7) % 27))
    for _ in range(200):                          # off-grid, out-of-range and all phases
        cases.append((rng.uniform(-0.3, 0.35), rng.uniform(-0.2, 0.2), rng.uniform(-1.5, 1.5),
                      int(rng.integers(0, 60))))
    for i in range(27):
        cases.append((0.0, -0.05, -0.1, i))     # the reference module's own demo command
    cases = np.array(cases, dtype=np.float64)
    exp = np.array([prm.get_reference_motion(c[0], c[1], c[2], int(c[3])) for c in cases])
    np.savez_compressed(os.path.join(OUT, "refmotion.npz"), cases=cases, expected=exp,
                        nb_steps_in_period=np.array(prm.nb_steps_in_period))
    print("golden:", out.shape, exp.shape)


if __name__ == "__main__":
    main()
