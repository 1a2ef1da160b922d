#!/usr/bin/env python3
"""Teacher-forced parity report (tests/teacher_forcing.py) for every case: per-group error
quantiles (median, p99, max of |gpu - oracle| / (1 + |oracle|)) and the outlier count, one JSON line
per case; every outlier explained at substep resolution (`explain`). Needs a GPU.

usage: python tools/teacher_forced_report.py [n_envs] [steps] [case ...]
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.teacher_forcing import CASES, explain, run_case  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    names = sys.argv[3:] or list(CASES)
    for name in names:
        rep = run_case(name, "cuda:0", n=n, steps=steps, keep_states=True)
        s = rep.summary()
        s["case"] = name
        s["outlier_kinds"] = []
        for t, st in enumerate(rep.steps):
            for e in (rep.outliers(st) | st.done_mismatch | st.int_mismatch).nonzero()[0]:
                x = explain(rep, t, int(e))
                s["outlier_kinds"].append({"step": t, "env": int(e), "kind": x["kind"],
                                           "max_substep_err": max(x["substep_err"]), "flips": x.get("flips"),
                                           "substep_err": [float(f"{v:.2e}") for v in x["substep_err"]]})
        print(json.dumps(s), flush=True)


if __name__ == "__main__":
    main()
