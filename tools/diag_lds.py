#!/usr/bin/env python3
"""Diff the env's LDS slice after one forward between two inlined copies of the substep.

physics_kernel inlines the substep twice: nsub=0 (mjx.forward) and the nsub>=1 loop. From the
same state (zero warm start) both compute the same forward, so the nsub=0 copy is an exact
reference for the loop copy. Needs a library built with -DDUCK_AUX_LDS (write_aux appends the
whole slice). Prints, per Lay field in pipeline order, the envs that differ and by how much."""
import os
import re
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from open_duck_playground_amd.joystick import Joystick  # noqa: E402
from tests.helpers import random_states  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "rough_terrain_backlash"
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = 512
gen = os.path.join(os.path.dirname(__file__), "..", "open_duck_playground_amd", "csrc", "generated",
                   {"flat_terrain": "duck_model_flat.h", "flat_terrain_backlash": "duck_model_backlash.h",
                    "rough_terrain": "duck_model_rough.h",
                    "rough_terrain_backlash": "duck_model_rough_backlash.h"}[task])
txt = open(gen).read()
C = {k: int(v) for k, v in re.findall(r"\b(NB|NQ|NV|NU|NM|MAXCHAIN|NSENSORDATA|NPAIR|NFRIC|NLIM|NHE|NHF|FLOOR_TYPE) = (\d+)", txt)}
NB, NQ, NV, NU, NM = C["NB"], C["NQ"], C["NV"], C["NU"], C["NM"]
NCON = 4 * C["NPAIR"]
NROW = C["NFRIC"] + C["NLIM"] + 4 * NCON
# Lay::HSZ: the scratch in front of the rows, sized for its largest user
need = max(12 * NB + 6 * NV, 6 * (C["NHE"] + C["NHF"]), 3 + 28 * 16 if C["FLOOR_TYPE"] == 1 else 0, 86 + 9 * NU)
HSZ = (max(need - 4 * NROW - C["NLIM"], 0) + 3) // 4 * 4
# Lay<Md> (csrc/duck_physics.h) in order
fields = [("QPOS", NQ), ("QVEL", NV), ("WARM", NV), ("CTRL", NU), ("QACC", NV), ("QSM", NV), ("FSM", NV),
          ("SRCH", NV), ("GRAD", NV), ("MA", NV), ("DMASS", NB), ("DIPOS", 3), ("DARM", NV), ("DFRIC", NV),
          ("DQ0", NQ), ("DKP", NU), ("XPOS", 3 * NB), ("XQ", 4 * NB), ("XMAT", 9 * NB), ("CIN", 10 * NB),
          ("CVEL", 6 * NB), ("COM", 3), ("CDOF", 6 * NV), ("CDD1", 18), ("M", NM), ("MZERO", 1), ("H", HSZ), ("JA", NROW),
          ("JV", NROW), ("RD", NROW), ("AREF", NROW), ("LSGN", C["NLIM"]), ("CR", 3 * NCON), ("CFR", 9 * NCON),
          ("CDIST", NCON), ("AF", NU), ("SENS", C["NSENSORDATA"]), ("OCON", 2), ("IMUR", 3), ("FOOTZ", 2),
          ("FLAGS", 2), ("SINK", 32)]
total = sum(k for _, k in fields)

env = Joystick(task, num_envs=1, device="cuda:0", use_imitation=False)
m = env.mj_model
qpos, qvel, ctrl = random_states(m, n, seed)
T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device="cuda:0")
outs = []
for nsub in (0, 1):
    tq, tv, tw, tc = T(qpos), T(qvel), T(np.zeros((n, m.nv))), T(ctrl)
    aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device="cuda:0").view(-1, n)
    env.physics_step(tq, tv, tw, tc, nsub, aux)
    torch.cuda.synchronize()
    outs.append(aux.cpu().numpy()[-total:].T.astype(np.float64))
a, b = outs
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/diag_lds_{task}_{seed}_{os.path.basename(os.environ.get('DUCK_LIB', 'libduck.so'))}.npz",
                    a=a, b=b, qpos=qpos, qvel=qvel, ctrl=ctrl)
o = 0
for name, k in fields:
    x, y = a[:, o:o + k], b[:, o:o + k]
    o += k
    if name in ("QPOS", "QVEL"):
        continue  # the loop copy integrates after write_aux? (aux is written before euler)
    d = np.abs(x - y) / (1 + np.abs(x))
    d[~(np.isfinite(x) & np.isfinite(y) & (np.abs(x) < 1e20))] = 0.0  # never-written slots (world/floor bodies)
    bad = np.where(d.max(axis=1) > 1e-5)[0]
    if len(bad):
        cols = np.argsort(-d[bad].max(axis=0))[:6]
        print(f"{name:6s} {len(bad):4d} envs differ; worst {d.max():.3e}; envs {bad[:12].tolist()} cols {cols.tolist()}",
              flush=True)
    else:
        print(f"{name:6s} identical (<=1e-5)", flush=True)
