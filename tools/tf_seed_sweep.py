#!/usr/bin/env python3
"""Teacher-forced rough cases over several seeds (GPU box): per seed, the outliers and how explain()
classifies them -- to tell a kernel change's new unexplained outliers from the classifier's base rate.
usage: DUCK_LIB=... python tools/tf_seed_sweep.py <case> <seed> [<seed> ...]"""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.teacher_forcing import explain, rule_of, run_case  # noqa: E402


def main():
    case, seeds = sys.argv[1], [int(s) for s in sys.argv[2:]]
    for seed in seeds:
        rep = run_case(case, "cuda:0", n=1024, steps=10, keep_states=True, seed=seed)
        rules, bad = Counter(), []
        for t, st in enumerate(rep.steps):
            for e in (rep.outliers(st) | st.done_mismatch | st.int_mismatch).nonzero()[0]:
                x = explain(rep, t, int(e))
                rules.update(rule_of(x))
                if x["kind"] != "sensitive":
                    bad.append((t, int(e), round(max(x["substep_err"]), 4)))
        sm = rep.summary()
        p99 = {k: f"{sm['err_median_p99_max'][k][1]:.2e}" for k in ("qpos", "qvel", "qacc_warmstart")}
        print(f"{case} seed {seed}: good_frac {sm['good_frac']:.5f} outliers {sm['outliers']} p99 {p99} "
              f"rules {dict(sorted(rules.items()))} unexplained {bad}", flush=True)


if __name__ == "__main__":
    main()
