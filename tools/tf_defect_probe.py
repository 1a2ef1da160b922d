#!/usr/bin/env python3
"""Contact sets at a teacher-forcing defect (GPU box): replays env-step t of env e of a rough case
as single substeps (the explain() chain), and at the first substep the oracle does not reproduce
prints the GPU's and the oracle's contact slots (depth, point, normal) and the oracle's prism
candidates of the differing pairs. usage: python tools/tf_defect_probe.py <case> <seed> t:e [t:e ...]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    import torch
    from tests.helpers import parse_aux
    from tests.oracle_ffi import lib
    from tests.teacher_forcing import _split, _state_rel, gpu_substep, oracle_substep, run_case, substep_trace
    case, seed = sys.argv[1], int(sys.argv[2])
    rep = run_case(case, "cuda:0", n=1024, steps=10, keep_states=True, seed=seed)
    env = rep.env
    m = env.mj_model
    np.set_printoptions(precision=7, suppress=True, linewidth=160)
    for te in sys.argv[3:]:
        t, e = (int(v) for v in te.split(":"))
        om, tr = substep_trace(rep, e, t)
        x = tr[0].astype(np.float32).astype(np.float64)
        for s in range(env.n_substeps):
            g = gpu_substep(env, e, x)
            r = oracle_substep(om, x)
            err = _state_rel(m, g, r)
            if err > 1e-4:
                print(f"== {case} seed {seed} step {t} env {e}: substep {s} err {err:.3g}")
                n = env.num_envs
                T = lambda y: torch.tensor(np.tile(y.astype(np.float32)[:, None], (1, n)), device=env.device).contiguous()  # noqa: E731
                tq, tv, tw, tc = (T(y) for y in _split(m, x))
                aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device=env.device).view(-1, n)
                env.physics_step(tq, tv, tw, tc, 0, aux)
                torch.cuda.synchronize()
                ga = parse_aux(m, aux[:, e].cpu().numpy().astype(np.float64)[:, None])
                q, v, w, c = _split(m, x)
                d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
                om.forward(d)
                od = d.arr("con_dist", 4 * m.npair)
                op = np.ctypeslib.as_array(d.con_pos)[:3 * 4 * m.npair].reshape(-1, 3)
                gd = np.asarray(ga["con_dist"][0])[:4 * m.npair]
                gp = np.asarray(ga["con_pos"][0]).reshape(-1, 3)[:4 * m.npair]
                gn = np.asarray(ga["con_normal"][0]).reshape(-1, 3)[:4 * m.npair]
                for sl in range(4 * m.npair):
                    print(f"  slot {sl:2d} gpu {gd[sl]: .7f} {gp[sl]} n {gn[sl]}   oracle {od[sl]: .7f} {op[sl]}")
                floor = m.id("geom", "floor")
                for p in range(m.npair):
                    g1, g2 = int(m.pair_geom1[p]), int(m.pair_geom2[p])
                    if floor not in (g1, g2):
                        continue
                    foot = g2 if g1 == floor else g1
                    dep, nrm, pt = np.zeros(128), np.zeros(3 * 128), np.zeros(3 * 128)
                    k = lib().oracle_hfield_contacts(om.ptr, C.byref(d), floor, foot, 128, dep.ctypes.data_as(C.POINTER(C.c_double)),
                                                     nrm.ctypes.data_as(C.POINTER(C.c_double)), pt.ctypes.data_as(C.POINTER(C.c_double)))
                    print(f"  pair {p}: oracle prism contacts {k}")
                    for i in range(k):
                        print(f"    depth {dep[i]: .7f} pt {pt[3 * i:3 * i + 3]} n {nrm[3 * i:3 * i + 3]}")
                break
            x = g


if __name__ == "__main__":
    main()
