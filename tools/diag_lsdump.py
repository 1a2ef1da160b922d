#!/usr/bin/env python3
"""Compare the line search's inputs (DUCK_LS_DUMP builds: G0, G1, G2, gtol, |s|^2 and each lane's
partial row coefficients at alpha = 0, stored into the KC scratch) between the two inlined
substep copies of physics_kernel. Reads the .npz that tools/diag_lds.py saved."""
import re
import sys

import numpy as np

path = sys.argv[1]
d = np.load(path)
a, b = d["a"], d["b"]
txt = open("open_duck_playground_amd/csrc/generated/duck_model_rough_backlash.h").read()
C = {k: int(v) for k, v in re.findall(r"\b(NB|NQ|NV|NU|NM|MAXCHAIN|NSENSORDATA|NPAIR|NFRIC|NLIM) = (\d+)", txt)}
NB, NQ, NV, NU, NM = C["NB"], C["NQ"], C["NV"], C["NU"], C["NM"]
NCON = 4 * C["NPAIR"]
NROW = C["NFRIC"] + C["NLIM"] + 4 * NCON
sizes = [NQ, NV, NV, NU, NV, NV, NV, NV, NV, NV, NB, 3, NV, NV, NQ, NU, 3 * NB, 4 * NB, 9 * NB, 10 * NB, 6 * NB, 3,
         6 * NV, 18, NM, NM, NROW, NROW, NROW, NROW, C["NLIM"], 3 * NCON, 9 * NCON, NCON, NU, C["NSENSORDATA"], 2, 3,
         2, 2]
KC = sum(sizes)
ka, kb = a[:, KC:KC + 136], b[:, KC:KC + 136]
for i, nm in enumerate(["G0", "G1", "G2", "gtol", "sn"]):
    dd = np.abs(ka[:, i] - kb[:, i]) / (1 + np.abs(ka[:, i]))
    print(f"{nm:5s} envs differing {(dd > 1e-6).sum()} worst {dd.max():.3e}")
q, qb = ka[:, 8:56].reshape(-1, 16, 3), kb[:, 8:56].reshape(-1, 16, 3)
dd = np.abs(q - qb) / (1 + np.abs(q))
bad = np.where(dd.max(axis=(1, 2)) > 1e-6)[0]
print("lane partials differ in", len(bad), "envs")
if len(bad):
    print("lanes differing (count over envs):", (dd[bad].max(axis=2) > 1e-6).sum(axis=0).tolist())
    print("which of q0,q1,q2:", (dd[bad].max(axis=1) > 1e-6).sum(axis=0).tolist())
    e = bad[0]
    print("env", e)
    print(np.c_[q[e], qb[e]])

la, lb = ka[:, 56:72], kb[:, 56:72]
print("lane ids differ in", int((la != lb).any(axis=1).sum()), "envs; ilp copy lane row of env 0:", lb[0].tolist())
pa, pb = ka[:, 72:88], kb[:, 72:88]
dd = np.abs(pa - pb) / (1 + np.abs(pa))
bad = np.where(dd.max(axis=1) > 1e-6)[0]
print("partial |s|^2 per lane differ in", len(bad), "envs; lanes:", (dd[bad] > 1e-6).sum(axis=0).tolist())
if len(bad):
    print(np.c_[pa[bad[0]], pb[bad[0]]])

ea = ka[:, 88:120].astype(np.float32).view(np.uint32).astype(np.uint64)
eb = kb[:, 88:120].astype(np.float32).view(np.uint32).astype(np.uint64)
exa = ea[:, :16] | (ea[:, 16:] << 32)
exb = eb[:, :16] | (eb[:, 16:] << 32)
print("exec before the sum loop, env 0 lanes 0..15: ref", [hex(int(x)) for x in exa[0, :2]], "ilp", [hex(int(x)) for x in exb[0, :2]])
print("lanes with exec differing:", int((exa != exb).sum()))
sa, sb = ka[:, 120:136], kb[:, 120:136]
print("SRCH[lane] as read before the loop differ in", int((np.abs(sa - sb) > 1e-6 * (1 + np.abs(sa))).any(axis=1).sum()), "envs")
