#!/usr/bin/env python3
"""The substep an unexplained teacher-forced outlier ("defect") fails at, in detail (GPU box): the per-substep
errors of the GPU's physics-kernel chain against the oracle from the same inputs, and at the first substep
above 1e-4 that no declared fp32 behaviour explains: both contact sets slot by slot (depth, point, normal),
whether the oracle continued from the GPU's contact set lands on the GPU's result (a contact-generation
difference) or not (a dynamics difference), and the oracle's own spread under 1e-6 / 1e-5 input
perturbations. usage: python tools/tf_defect_detail.py <case> <seed> <t> <env> [<t> <env> ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.teacher_forcing import (_state_rel, declared_difference, flip_level, gpu_contact_aux,  # noqa: E402
                                   gpu_substep, oracle_contact_aux, oracle_substep, oracle_substep_with_contacts,
                                   run_case, substep_trace)


def main():
    case, seed = sys.argv[1], int(sys.argv[2])
    pairs = [(int(a), int(b)) for a, b in zip(sys.argv[3::2], sys.argv[4::2])]
    rep = run_case(case, "cuda:0", n=1024, steps=10, keep_states=True, seed=seed)
    env, m = rep.env, rep.env.mj_model
    np.set_printoptions(precision=6, suppress=False, linewidth=160)
    for t, e in pairs:
        om, tr = substep_trace(rep, e, t)
        x = tr[0].astype(np.float32).astype(np.float64)
        rng = np.random.default_rng(0)
        per = []
        print(f"== {case} seed {seed} env-step {t} env {e}", flush=True)
        for s in range(env.n_substeps):
            g = gpu_substep(env, e, x)
            r = oracle_substep(om, x)
            err = _state_rel(m, g, r)
            per.append(err)
            if err > 1e-4:
                lev = flip_level(om, x, g, rng)
                info = {}
                why = None if lev is not None else declared_difference(env, e, om, x, g, 1e-4, info=info)
                print(f"substep {s}: err {err:.3e} flip {lev} declared {why} info {info}", flush=True)
                if lev is None and why is None:
                    ga, oa = gpu_contact_aux(env, e, x), oracle_contact_aux(om, x)
                    gd, od = ga["con_dist"][0], oa["con_dist"][0]
                    gp, op = ga["con_pos"][0].reshape(-1, 3), oa["con_pos"][0].reshape(-1, 3)
                    gn, on = ga["con_normal"][0].reshape(-1, 3), oa["con_normal"][0].reshape(-1, 3)
                    for k in range(4 * m.npair):
                        if gd[k] < 0 or od[k] < 0:
                            print(f"  slot {k:2d} (pair {k // 4}): gpu d {gd[k]: .6e} p {gp[k]} n {gn[k]} | "
                                  f"oracle d {od[k]: .6e} p {op[k]} n {on[k]}")
                    wc = oracle_substep_with_contacts(om, x, ga)
                    print(f"  oracle continued from the GPU's contact set vs the GPU: {_state_rel(m, g, wc):.3e}; "
                          f"vs the oracle's own substep: {_state_rel(m, r, wc):.3e}", flush=True)
                    sp = []
                    for lvl in (1e-6, 1e-5):
                        for _ in range(8):
                            xp = x.copy()
                            kq = m.nq + 2 * m.nv
                            xp[:kq] *= 1 + lvl * rng.choice([-1.0, 1.0], kq)
                            sp.append((lvl, _state_rel(m, oracle_substep(om, xp), r)))
                    print("  oracle spread under input perturbations (level, err vs its own substep):",
                          [(lv, f"{v:.2e}") for lv, v in sp], flush=True)
                    break
            x = g
        print("substep errors", [f"{v:.1e}" for v in per], flush=True)


if __name__ == "__main__":
    main()
