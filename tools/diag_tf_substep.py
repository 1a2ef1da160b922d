#!/usr/bin/env python3
"""Locate teacher-forcing defects at substep resolution and dump what the GPU computed there.

GPU: python tools/diag_tf_substep.py run <case> [max] [envs] [steps] [thr]  -> gpurun_out/diag_tf_<case>.npz
CPU: python tools/diag_tf_substep.py show <case>        (oracle forward at the same inputs)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(case, mx=6, n=256, steps=6, thr=1e-3):
    import torch
    from tests.helpers import parse_aux
    from tests.teacher_forcing import _split, _state_rel, gpu_substep, oracle_substep, run_case, substep_trace
    rep = run_case(case, "cuda:0", n=n, steps=steps, keep_states=True)
    env, m = rep.env, rep.env.mj_model
    out = {"x": [], "aux": [], "env": [], "gnext": [], "rnext": [], "dr": []}
    for t, st in enumerate(rep.steps):
        for e in (rep.outliers(st) | st.done_mismatch | st.int_mismatch).nonzero()[0]:
            if len(out["x"]) >= mx:
                break
            om, tr = substep_trace(rep, int(e), t)
            x = tr[0].astype(np.float32).astype(np.float64)
            for s in range(env.n_substeps):
                g = gpu_substep(env, int(e), x)
                r = oracle_substep(om, x)
                if _state_rel(m, g, r) > thr:
                    n = env.num_envs
                    T = lambda y: torch.tensor(np.tile(y.astype(np.float32)[:, None], (1, n)), device=env.device).contiguous()  # noqa: E731
                    tq, tv, tw, tc = (T(y) for y in _split(m, x))
                    aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device=env.device).view(-1, n)
                    env.physics_step(tq, tv, tw, tc, 0, aux)
                    torch.cuda.synchronize()
                    out["x"].append(x)
                    out["aux"].append(aux[:, int(e)].cpu().numpy().astype(np.float64))
                    out["env"].append(int(e))
                    out["gnext"].append(g)
                    out["rnext"].append(r)
                    out["dr"].append(np.array([t, s]))
                    print(f"step {t} env {e} substep {s} err {_state_rel(m, g, r):.3e}", flush=True)
                    break
                x = g
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"diag_tf_{case}.npz"), **{k: np.array(v) for k, v in out.items()})


def show(case):
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.mjcf import Model
    from tests.helpers import parse_aux
    from tests.oracle_ffi import OracleModel
    from tests.teacher_forcing import CASES, _split
    spec = CASES[case]
    m = Model.load(constants.task_to_xml(spec["task"]))
    base = OracleModel(m)
    z = np.load(os.path.join(ROOT, "gpurun_out", f"diag_tf_{case}.npz"))
    np.set_printoptions(precision=5, suppress=True, linewidth=150)
    for i in range(len(z["x"])):
        e = int(z["env"][i])
        om = OracleModel(m, dr=base.dr_sample(7 + 1, e)) if spec.get("dr") else base
        q, v, w, c = _split(m, z["x"][i])
        d = om.new_data(qpos=q, qvel=v, ctrl=c, warm=w)
        om.forward(d)
        g = parse_aux(m, z["aux"][i][:, None])
        rd = d.arr("con_dist", 4 * m.npair)
        rp = np.ctypeslib.as_array(d.con_pos)[:4 * m.npair]
        print(f"== {case} step/substep {z['dr'][i]} env {e}")
        print("  qacc gpu   ", g["qacc"][0][:8])
        print("  qacc oracle", d.arr("qacc", m.nv)[:8])
        print("  qsm  gpu   ", g["qacc_smooth"][0][:8])
        print("  qsm  oracle", d.arr("qacc_smooth", m.nv)[:8])
        gp = g["con_pos"][0].reshape(-1, 3)
        for s in range(4 * m.npair):
            if rd[s] < 0 or g["con_dist"][0][s] < 0:
                print(f"  slot {s}: gpu {g['con_dist'][0][s]: .6f} {gp[s]}  oracle {rd[s]: .6f} {rp[s]}")


if __name__ == "__main__":
    {"run": lambda: run(sys.argv[2], *[f(a) for f, a in zip((int, int, int, float), sys.argv[3:])]),
     "show": lambda: show(sys.argv[2])}[sys.argv[1]]()
