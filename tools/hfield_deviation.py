#!/usr/bin/env python3
"""The oracle's height-field contacts (collide_hfield_convex: MuJoCo's prism decomposition with the
Minkowski-face axis set, the tie rule and MJX's 4 slots) against the brute-force prism reference
(oracle_hfield_prisms: the same prisms, every separating axis, no filter, no tie rule).

Both are evaluated by the oracle on the same states: the final substep of env-steps of the rough
scenes with domain randomisation (C4: rough_terrain, C5's shard: rough_terrain_backlash), random
U(-1,1) actions. Per foot and env-step: contact flag (any penetration) of each, the deepest
penetration of each, the angle between their deepest contacts' normals, and which class of axis
gave the prism contacts (the kernel skips the bottom-edge pairs: never the minimum). CPU only.

usage: python tools/hfield_deviation.py [n_envs] [n_steps] [--gpu]   (one JSON line per scene)
  --gpu: the HIP kernel's contacts at the oracle's rollout states against the brute-force prisms
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
from tests.oracle_ffi import OracleData, OracleEnv, OracleModel, lib  # noqa: E402


def prisms(om, d, g_hf, g_foot, max_n=64):
    dep, nrm, pt = np.zeros(max_n), np.zeros(3 * max_n), np.zeros(3 * max_n)
    idx = np.zeros(max_n, dtype=np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    n = lib().oracle_hfield_prisms(om.ptr, C.byref(d), g_hf, g_foot, max_n, dp(dep), dp(nrm), dp(pt),
                                   idx.ctypes.data_as(C.POINTER(C.c_int32)))
    return dep[:n], nrm[:3 * n].reshape(n, 3)


def measure(task: str, n_envs: int, n_steps: int, seed: int = 0, blend: bool = False):
    m = Model.load(constants.task_to_xml(task))
    base = OracleModel(m)
    cfg = env_config_struct(m, default_config(), False, domain_randomize=True)
    floor = m.id("geom", "floor")
    pairs = {}
    for foot in constants.FEET_GEOMS:
        g = m.id("geom", foot)
        p = [k for k in range(m.npair) if {int(m.pair_geom1[k]), int(m.pair_geom2[k])} == {floor, g}][0]
        pairs[g] = p
    rng = np.random.default_rng(seed)
    rows = []
    wins = (C.c_longlong * 14)()
    lib().oracle_hfield_axis_wins(wins, 1)
    # blend=True: round 4's point band (oracle_set_hf_band_scale(1)) in place of the declared plain
    # penetration-weighted centroid
    lib().oracle_set_hf_band_scale(1.0 if blend else 0.0)
    try:
        rows = _rollout(m, base, cfg, pairs, floor, n_envs, n_steps, seed, rng)
    finally:
        lib().oracle_set_hf_band_scale(0.0)
    lib().oracle_hfield_axis_wins(wins, 1)
    return _summary(task, rows, wins, blend)


def _rollout(m, base, cfg, pairs, floor, n_envs, n_steps, seed, rng):
    rows = []
    for e in range(n_envs):
        om = OracleModel(m, dr=base.dr_sample(seed + 1, e))
        env = OracleEnv(om, cfg)
        env.reset(seed=seed, env_id=e)
        d = OracleData()
        for t in range(n_steps):
            env.step(rng.uniform(-1, 1, m.nu), d)
            for g, p in pairs.items():
                dist = d.arr("con_dist", 4 * m.npair)[4 * p:4 * p + 4]
                frames = np.ctypeslib.as_array(d.con_frame)[4 * p:4 * p + 4]
                dep, nrm = prisms(om, d, floor, g)
                ours = -dist.min()
                ref = dep.max() if len(dep) else -1.0
                ang = np.nan
                if ours > 0 and ref > 0:
                    n1 = frames[int(np.argmin(dist))][:3]
                    n2 = nrm[int(np.argmax(dep))]
                    ang = float(np.degrees(np.arccos(np.clip(n1 @ n2, -1, 1))))
                rows.append((ours > 0, ref > 0, max(ours, 0.0), max(ref, 0.0), ang, len(dep)))
    return rows


def _summary(task, rows, wins, blend):
    a = np.array(rows, dtype=float)
    flag_o, flag_r, dep_o, dep_r, ang, nprism = a.T
    both = (flag_o > 0) & (flag_r > 0)
    dd = np.abs(dep_o - dep_r)[both]
    return {"scene": task, "blend": blend, "foot_samples": len(a), "contact_ours": int(flag_o.sum()), "contact_prism": int(flag_r.sum()),
            "flag_agreement": float((flag_o == flag_r).mean()),
            "flag_disagree_max_depth_m": float(np.max(np.maximum(dep_o, dep_r)[flag_o != flag_r], initial=0.0)),
            "depth_abs_diff_m": {"median": float(np.median(dd)), "p99": float(np.quantile(dd, 0.99)), "max": float(dd.max())},
            "depth_prism_median_m": float(np.median(dep_r[both])),
            "normal_angle_deg": {"median": float(np.nanmedian(ang)), "p99": float(np.nanquantile(ang, 0.99)),
                                 "max": float(np.nanmax(ang))},
            "axis_wins": dict(zip(("top", "side", "bottom", "hull_face", "top_edge", "vertical_edge", "bottom_edge"),
                                  [int(x) for x in wins[:7]])),
            "separated_past_prism_faces_by": dict(zip(("hull_face", "top_edge", "vertical_edge", "bottom_edge"),
                                                      [int(x) for x in wins[10:14]])),
            "penetrating_prisms_per_foot": {"mean": float(nprism[flag_r > 0].mean()), "max": int(nprism.max())}}


def measure_gpu(task: str, n_envs: int, n_steps: int, seed: int = 0, device="cuda:0"):
    """The HIP kernel's contacts (TPhys::collide_hfield, through duck_physics_step's forward) against
    the brute-force prisms and the oracle at the same states: oracle rollouts (rough + DR, U(-1,1)
    actions) give the states; per foot the contact flag and the deepest depth are compared with the
    brute force, the deepest slot's normal with the oracle's (normal_angle_vs_brute_deg: against the
    brute force's single minimum axis), and the contact points with the oracle's declared rule (the
    penetration-weighted centroid): the deepest slot's point against the oracle
    slot of the same depth (within HF_DEPTH_TIE) nearest to it, and every active kernel slot against
    the nearest active oracle slot. band_point_shift_m: how far round 4's point band (the oracle with
    oracle_set_hf_band_scale(1)) moves the oracle's own deepest point at the same states."""
    import torch
    from open_duck_playground_amd.joystick import Joystick, domain_randomize
    from tests.helpers import parse_aux
    m = Model.load(constants.task_to_xml(task))
    base = OracleModel(m)
    cfg = env_config_struct(m, default_config(), False, domain_randomize=True)
    floor = m.id("geom", "floor")
    pairs = {}
    for foot in constants.FEET_GEOMS:
        g = m.id("geom", foot)
        pairs[g] = [k for k in range(m.npair) if {int(m.pair_geom1[k]), int(m.pair_geom2[k])} == {floor, g}][0]
    env = Joystick(task, num_envs=n_envs, device=device, use_imitation=False)
    domain_randomize(env, rng=seed + 1)  # column e carries dr_sample(seed + 1, e), as the oracle models
    models = [OracleModel(m, dr=base.dr_sample(seed + 1, e)) for e in range(n_envs)]
    envs = [OracleEnv(models[e], cfg) for e in range(n_envs)]
    for e in range(n_envs):
        envs[e].reset(seed=seed, env_id=e)
    rng = np.random.default_rng(seed)
    L = envs[0].L
    o = L.off
    rows, pts, slot_pts, band = [], [], [], []
    for t in range(n_steps):
        X = np.zeros((n_envs, m.nq + 2 * m.nv + m.nu))
        for e in range(n_envs):
            envs[e].step(rng.uniform(-1, 1, m.nu))
            f = envs[e].fs
            X[e] = np.concatenate([f[o["qpos"]:o["qpos"] + m.nq], f[o["qvel"]:o["qvel"] + m.nv],
                                   f[o["qacc_warmstart"]:o["qacc_warmstart"] + m.nv], f[o["ctrl"]:o["ctrl"] + m.nu]])
        X = X.astype(np.float32).astype(np.float64)  # the state the kernel sees
        T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device=device)  # noqa: E731
        sl = np.cumsum([0, m.nq, m.nv, m.nv, m.nu])
        tq, tv, tw, tc = (T(X[:, sl[i]:sl[i + 1]]) for i in range(4))
        aux = torch.zeros(env.aux_size() * n_envs, dtype=torch.float32, device=device).view(-1, n_envs)
        env.physics_step(tq, tv, tw, tc, 0, aux)
        torch.cuda.synchronize()
        g = parse_aux(m, aux.cpu().numpy().astype(np.float64))
        for e in range(n_envs):
            def fwd(scale):
                lib().oracle_set_hf_band_scale(scale)
                try:
                    d = models[e].new_data(qpos=X[e, :m.nq], qvel=X[e, m.nq:m.nq + m.nv], ctrl=X[e, sl[3]:],
                                           warm=X[e, sl[2]:sl[3]])
                    models[e].forward(d)
                finally:
                    lib().oracle_set_hf_band_scale(0.0)
                return d
            d, db = fwd(0.0), fwd(1.0)
            for gid, p in pairs.items():
                gd = g["con_dist"][e, 4 * p:4 * p + 4]
                gn = g["con_normal"][e].reshape(-1, 3)[4 * p:4 * p + 4]
                gp = g["con_pos"][e].reshape(-1, 3)[4 * p:4 * p + 4]
                dep, nrm = prisms(models[e], d, floor, gid)
                od = d.arr("con_dist", 4 * m.npair)[4 * p:4 * p + 4]
                on = np.ctypeslib.as_array(d.con_frame)[4 * p:4 * p + 4, :3]
                op = np.ctypeslib.as_array(d.con_pos)[4 * p:4 * p + 4]
                ours = -gd.min()
                ref = dep.max() if len(dep) else -1.0
                ang = angb = np.nan
                if ours > 0 and ref > 0:
                    k = int(np.argmin(gd))
                    n1 = gn[k] / np.linalg.norm(gn[k])
                    angb = float(np.degrees(np.arccos(np.clip(n1 @ nrm[int(np.argmax(dep))], -1, 1))))
                    if od.min() < 0:
                        ang = float(np.degrees(np.arccos(np.clip(n1 @ on[int(np.argmin(od))], -1, 1))))
                        tie = (od < 0) & (np.abs(od - gd[k]) <= 1e-6)
                        cand = op[tie] if tie.any() else op[[int(np.argmin(od))]]
                        pts.append(float(np.min(np.linalg.norm(cand - gp[k], axis=1))))
                        act = op[od < 0]
                        slot_pts += [float(np.min(np.linalg.norm(act - gp[j], axis=1))) for j in range(4) if gd[j] < 0]
                        odb = db.arr("con_dist", 4 * m.npair)[4 * p:4 * p + 4]
                        if odb.min() < 0:
                            opb = np.ctypeslib.as_array(db.con_pos)[4 * p:4 * p + 4]
                            band.append(float(np.linalg.norm(opb[int(np.argmin(odb))] - op[int(np.argmin(od))])))
                rows.append((ours > 0, ref > 0, max(ours, 0.0), max(ref, 0.0), ang, angb))
    a = np.array(rows, dtype=float)
    flag_o, flag_r, dep_o, dep_r, ang, angb = a.T
    both = (flag_o > 0) & (flag_r > 0)
    dd = np.abs(dep_o - dep_r)[both]
    q = lambda x: {"median": float(np.median(x)), "p99": float(np.quantile(x, 0.99)), "max": float(np.max(x)),  # noqa: E731
                   "frac_over_1mm": float(np.mean(np.asarray(x) > 1e-3))}
    return {"scene": task, "side": "HIP kernel (fp32) vs brute-force prisms / the oracle (fp64)", "foot_samples": len(a),
            "contact_kernel": int(flag_o.sum()), "contact_prism": int(flag_r.sum()),
            "flag_agreement": float((flag_o == flag_r).mean()),
            "flag_disagree_max_depth_m": float(np.max(np.maximum(dep_o, dep_r)[flag_o != flag_r], initial=0.0)),
            "depth_abs_diff_m": q(dd), "normal_angle_deg": q(ang[both & np.isfinite(ang)]),
            "normal_angle_vs_brute_deg": q(angb[both & np.isfinite(angb)]),
            "deepest_point_m": q(pts), "slot_point_m": q(slot_pts), "band_point_shift_m": q(band)}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if len(args) > 0 else 64
    steps = int(args[1]) if len(args) > 1 else 50
    for task in ("rough_terrain", "rough_terrain_backlash"):
        r = measure_gpu(task, n, steps) if "--gpu" in sys.argv else measure(task, n, steps)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
