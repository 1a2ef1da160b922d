#!/usr/bin/env python3
"""Per-outlier report of a teacher-forced case (GPU box): for every env-step whose GPU
result is outside the group tolerances, which groups cross and by how much (err / tol), the explain()
classification, and for the "agree" kind (every substep within 1e-4 of the oracle's, relative to the
state's largest |qvel|, |qacc|) what that normalisation admits: the trace's largest |qacc|, the per-substep
absolute qvel differences, the dof that carries the largest final qvel difference (joint name) and
whether the backlash hinges sit on their stops (limit rows active). For "gpu_flip" outliers the chain /
step / oracle distances. usage: python tools/tf_outlier_report.py <case> <seed> [<seed> ...]"""
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.teacher_forcing import (GROUPS, explain, gpu_substep, oracle_substep, rule_of, run_case,  # noqa: E402
                                   substep_trace)


def backlash_state(m, q):
    """(hinges at their stops, hinges) of the backlash joints in qpos q (range +-0.00873 rad)"""
    names = m.names["jnt"] if "jnt" in m.names else m.names.get("joint", [])
    at, tot = 0, 0
    for j, nm in enumerate(names):
        if nm and nm.endswith("_backlash"):
            tot += 1
            lo, hi = m.jnt_range[j]
            qa = q[m.jnt_qposadr[j]]
            at += int(qa <= lo + 1e-4 or qa >= hi - 1e-4)
    return at, tot


def main():
    case, seeds = sys.argv[1], [int(s) for s in sys.argv[2:]]
    for seed in seeds:
        rep = run_case(case, "cuda:0", n=1024, steps=10, keep_states=True, seed=seed)
        env = rep.env
        m = env.mj_model
        names = m.names["jnt"] if "jnt" in m.names else m.names.get("joint", [])
        dof_name = {}
        for j, nm in enumerate(names):
            dof_name[m.jnt_dofadr[j]] = nm or f"jnt{j}"
        rules = Counter()
        print(f"== {case} seed {seed}: {rep.summary()['outliers']} outliers of {rep.summary()['env_steps']} env-steps",
              flush=True)
        for t, st in enumerate(rep.steps):
            bad = rep.outliers(st) | st.done_mismatch | st.int_mismatch
            for e in bad.nonzero()[0]:
                e = int(e)
                cross = {g: round(float(st.err[g][e] / rep.tol[g]), 2) for g in GROUPS if st.err[g][e] > rep.tol[g]}
                x = explain(rep, t, e)
                r = rule_of(x)
                rules.update(r)
                line = f"t {t} env {e:4d} {'+'.join(r):24s} crosses {cross}"
                if st.done_mismatch[e]:
                    line += " done-mismatch"
                if r == ["agree"] or "gpu_flip" in x:
                    _, tr = substep_trace(rep, e, t)
                    qa = np.abs(tr[:, m.nq + m.nv:m.nq + 2 * m.nv]).max()
                    # per-substep |qvel| difference of the GPU substep against the oracle's from the same input
                    xi = tr[0].astype(np.float32).astype(np.float64)
                    dq = []
                    for _ in range(env.n_substeps):
                        g = gpu_substep(env, e, xi)
                        o = oracle_substep(rep.models[e] if isinstance(rep.models, list) else rep.models, xi)
                        dq.append(float(np.abs(g[m.nq:m.nq + m.nv] - o[m.nq:m.nq + m.nv]).max()))
                        xi = g
                    # the oracle's own sensitivity: its 10-substep chain from the same input perturbed by a
                    # relative 1e-7 (fp32 rounding size), 8 random sign patterns, against the unperturbed chain
                    om = rep.models[e] if isinstance(rep.models, list) else rep.models
                    x0 = tr[0].astype(np.float32).astype(np.float64)

                    def ochain(y):
                        for _ in range(env.n_substeps):
                            y = oracle_substep(om, y)
                        return y
                    base = ochain(x0)
                    rng = np.random.default_rng(0)
                    kq = m.nq + 2 * m.nv
                    divs = []
                    for _ in range(8):
                        xp = x0.copy()
                        xp[:kq] *= 1 + 1e-7 * rng.choice([-1.0, 1.0], kq)
                        divs.append(float(np.abs(ochain(xp)[m.nq:m.nq + m.nv] - base[m.nq:m.nq + m.nv]).max()))
                    L, n = env._layout, env.num_envs
                    G = rep.post[t].reshape(L.nfloat, n)[:, e]
                    dv = np.abs(G[L.off["qvel"]:L.off["qvel"] + m.nv] - tr[-1, m.nq:m.nq + m.nv])
                    k = int(dv.argmax())
                    dof = max((d for d in dof_name if d <= k), default=0)
                    at, tot = backlash_state(m, G[L.off["qpos"]:L.off["qpos"] + m.nq])
                    line += (f" | max|qacc| {qa:.3g} substep |dqvel| max {max(dq):.2e} sum {sum(dq):.2e};"
                             f" final |dqvel| {dv[k]:.2e} at dof {k} ({dof_name.get(dof, '?')}); backlash at stops {at}/{tot}")
                    line += (f"; oracle self-divergence at 1e-7: median {np.median(divs):.2e} max {max(divs):.2e}"
                             f" (amplification {np.median(divs) / max(sum(dq), 1e-30):.0f}x of the GPU's summed substep |dqvel|)")
                    line += (f"; chain_vs_step {x['chain_vs_step']:.2e} step_vs_oracle {x['step_vs_oracle']:.2e}"
                             f" chain_vs_oracle {x['chain_vs_oracle']:.2e}")
                    if "gpu_flip" in x:
                        line += f" gpu_flip {x['gpu_flip']}"
                print(line, flush=True)
        print(f"rules {dict(sorted(rules.items()))}", flush=True)


if __name__ == "__main__":
    main()
