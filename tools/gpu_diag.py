#!/usr/bin/env python3
"""GPU diagnostics: per-quantity HIP-vs-oracle errors + a quick env-step timing.

Prints numbers instead of asserting, to debug parity on the box in one call.
"""

import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from open_duck_playground_amd.joystick import Joystick  # noqa: E402
from tests.helpers import parse_aux, random_states  # noqa: E402
from tests.oracle_ffi import OracleModel  # noqa: E402


def forward_errors(task, n=256, nsub=0, seed=1):
    env = Joystick(task, num_envs=1, device="cuda:0", use_imitation=False)
    m = env.mj_model
    qpos, qvel, ctrl = random_states(m, n, seed)
    T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device="cuda:0")
    tq, tv, tw, tc = T(qpos), T(qvel), T(np.zeros((n, m.nv))), T(ctrl)
    aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device="cuda:0").view(-1, n)
    t = time.time()
    env.physics_step(tq, tv, tw, tc, nsub, aux)
    torch.cuda.synchronize()
    print(f"[{task}] physics_step n={n} nsub={nsub}: {time.time() - t:.3f}s (first call)")
    g = parse_aux(m, aux.cpu().numpy().astype(np.float64))
    om = OracleModel(m)
    keys = ("qacc", "qacc_smooth", "sensordata", "con_dist", "actuator_force", "qfrc_smooth")
    r = {k: [] for k in keys + ("M",)}
    for e in range(n):
        d = om.new_data(qpos=qpos[e], qvel=qvel[e], ctrl=ctrl[e])
        if nsub > 0:
            om.step(d, nsub - 1)
        om.forward(d)
        r["qacc"].append(d.arr("qacc", m.nv).copy())
        r["qacc_smooth"].append(d.arr("qacc_smooth", m.nv).copy())
        r["sensordata"].append(d.arr("sensordata", m.nsensordata).copy())
        r["con_dist"].append(d.arr("con_dist", 4 * m.npair).copy())
        r["actuator_force"].append(d.arr("actuator_force", m.nu).copy())
        r["qfrc_smooth"].append(d.arr("qfrc_smooth", m.nv).copy())
        r["M"].append(np.ctypeslib.as_array(d.qM)[:m.nv, :m.nv].copy())
    r = {k: np.array(v) for k, v in r.items()}
    g["M"] = g["Mdense"]
    for k in keys + ("M",):
        a, b = g[k].reshape(n, -1), r[k].reshape(n, -1)
        err = np.abs(a - b).max(axis=1)
        rel = err / (1 + np.abs(b).max(axis=1))
        print(f"  {k:15s} max_abs {err.max():.3e}  p50_rel {np.median(rel):.3e}  p99_rel {np.quantile(rel, 0.99):.3e}"
              f"  frac_rel<1e-3 {np.mean(rel < 1e-3):.3f}  finite {np.isfinite(a).all()}")
    a, b = g["qacc"].reshape(n, -1), r["qacc"].reshape(n, -1)
    rel = np.abs(a - b).max(axis=1) / (1 + np.abs(b).max(axis=1))
    ok = np.quantile(rel, 0.99) < 1e-3 and np.isfinite(a).all()
    worst = int(np.argmax(np.abs(g["qacc"] - r["qacc"]).max(axis=1)))
    print("  worst env", worst, "con_dist gpu", np.round(g["con_dist"][worst], 5), "ref", np.round(r["con_dist"][worst], 5))
    print("  qacc gpu", np.round(g["qacc"][worst][:8], 4), "ref", np.round(r["qacc"][worst][:8], 4))
    return ok


def timing(task="flat_terrain", n=4096, steps=20, imit=False):
    env = Joystick(task, num_envs=n, device="cuda:0", use_imitation=imit)
    st = env.reset(rng=0)
    a = torch.zeros(n, env.action_size, device="cuda:0")
    for _ in range(3):
        env.step(st, a, inplace=True)
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(steps):
        env.step(st, a, inplace=True)
    torch.cuda.synchronize()
    dt = (time.time() - t) / steps
    print(f"[timing {task} imit={imit}] n={n}: {dt * 1e3:.2f} ms/env-step -> {n / dt:,.0f} env-steps/s;"
          f" done frac {st.done.float().mean().item():.3f} reward mean {st.reward.mean().item():.3f}")


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "fwd", "fwdcheck"):
        ok = forward_errors("flat_terrain")
        ok = forward_errors("flat_terrain", nsub=1, seed=2) and ok
        ok = forward_errors("flat_terrain_backlash") and ok
        if which == "fwdcheck" and not ok:
            print("FORWARD PARITY FAILED")
            sys.exit(1)
    if which in ("all", "time"):
        timing()
        timing(imit=True)
        timing(n=8192)
