#!/usr/bin/env python3
"""Per-env HIP vs oracle qacc errors of one forward pass, with the failing envs classified.

Debug aid for the Newton-step miscompute: DUCK_LIB selects the library under
test (e.g. a max-ILP build of every variant). Prints, for the worst envs, the qacc error, the
dofs it sits on, whether the foot/foot pair has active contacts (the dense Newton path), the
number of active floor contacts, and the qacc_smooth error (the solve's input)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.test_gpu_physics import _run  # noqa: E402

tasks = sys.argv[1:] or ["rough_terrain_backlash"]
for task in tasks:
    for nsub, seed in ((0, 1), (0, 2), (1, 1), (1, 2)):
        m, g, r = _run(task, 512, nsub, seed=seed, gpu="cuda:0")
        rel = np.abs(g["qacc"] - r["qacc"]).max(axis=1) / (1 + np.abs(r["qacc"]).max(axis=1))
        rs = np.abs(g["qacc_smooth"] - r["qacc_smooth"]).max(axis=1) / (1 + np.abs(r["qacc_smooth"]).max(axis=1))
        cd = r["con_dist"]
        npair = cd.shape[1] // 4
        bad = np.where(~(rel < 2e-2))[0]
        print(f"{task} nsub={nsub} seed={seed} lib={os.path.basename(os.environ.get('DUCK_LIB', 'libduck.so'))}: {len(bad)}/{len(rel)} envs with qacc rel err >= 2e-2; "
              f"median {np.median(rel):.2e}; qacc_smooth max rel {rs.max():.2e}; "
              f"non-finite {int((~np.isfinite(g['qacc'])).any(axis=1).sum())}", flush=True)
        for e in bad[np.argsort(-rel[bad])][:4]:
            dofs = np.argsort(-np.abs(g["qacc"][e] - r["qacc"][e]))[:4]
            ff = [(cd[e, 4 * p:4 * p + 4] < 0).sum() for p in range(npair)]
            ffg = [(g["con_dist"][e, 4 * p:4 * p + 4] < 0).sum() for p in range(npair)]
            print(f"  env {e:4d} rel {rel[e]:.3e} dofs {dofs.tolist()} gpu {g['qacc'][e, dofs[0]]:.4e} "
                  f"ref {r['qacc'][e, dofs[0]]:.4e} active/pair oracle {ff} gpu {ffg} smooth rel {rs[e]:.1e}",
                  flush=True)
