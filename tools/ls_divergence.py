#!/usr/bin/env python3
"""Can grouping envs by their line-search work pay? (CPU only, the fp64 oracle with the
kernel's fp32 line-search stop, oracle_set_ls_floor(1e-6)).

A wave of the throughput kernel runs 4 envs (16-lane teams) in lockstep, so each substep's line search
costs the wave the MAX of its 4 envs' iteration counts. This runs the C2 workload (flat, auto-reset, U(-1,1)
actions) for n envs x T env-steps, records every env's iteration count at every substep (oracle_ls_trace),
and compares the per-wave cost of
  fixed       the kernel's grouping (envs 4w .. 4w+3)
  predicted   envs regrouped every env-step by the previous env-step's iteration total (the permutation a
              kernel could apply from information it already has)
  oracle      envs regrouped by the CURRENT env-step's totals (the unreachable bound)
and prints the correlation of an env's totals at consecutive env-steps.
usage: python tools/ls_divergence.py [--envs 1024] [--steps 40]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def wave_cost(its, order):
    """mean over env-steps and substeps of the max over each wave's 4 envs; its [n, S], order [n]"""
    g = its[order].reshape(-1, 4, its.shape[1])
    return float(g.max(axis=1).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    from open_duck_playground_amd import constants
    from open_duck_playground_amd.config import default_config, env_config_struct
    from open_duck_playground_amd.joystick import OpenDuckMiniV2Env
    from tests.oracle_ffi import OracleEnv, OracleModel, lib
    base = OpenDuckMiniV2Env(xml_path=constants.task_to_xml("flat_terrain"), config=default_config())
    m = base.mj_model
    cfg = env_config_struct(m, base._config, False, True, False)
    om = OracleModel(m)
    L = lib()
    L.oracle_set_ls_floor(1e-6)
    n, T, S = a.envs, a.steps, 10
    envs = [OracleEnv(om, cfg) for _ in range(n)]
    for e, env in enumerate(envs):
        env.reset(seed=0, env_id=e)
    rng = np.random.default_rng(1234)
    its = np.zeros((T, n, S), dtype=np.int32)
    buf = (C.c_int * 64)()
    for t in range(T):
        acts = rng.uniform(-1, 1, (n, m.nu))
        for e, env in enumerate(envs):
            L.oracle_ls_trace(None, 0, 1)
            env.step(acts[e])
            k = L.oracle_ls_trace(buf, 64, 1)
            its[t, e, :min(k, S)] = np.frombuffer(buf, dtype=np.int32, count=min(k, S))
    tot = its.sum(axis=2)
    ident = np.arange(n)
    fixed = [wave_cost(its[t], ident) for t in range(1, T)]
    pred = [wave_cost(its[t], np.argsort(-tot[t - 1], kind="stable")) for t in range(1, T)]
    best = [wave_cost(its[t], np.argsort(-tot[t], kind="stable")) for t in range(1, T)]
    team = float(its[1:].mean())
    r = [np.corrcoef(tot[t - 1], tot[t])[0, 1] for t in range(1, T)]
    print(f"C2 flat, {n} envs x {T} env-steps (first dropped), fp64 oracle with the kernel's 1e-6 line-search stop")
    print(f"line-search iterations per substep: per env {team:.3f}; per 4-env wave (max): fixed grouping "
          f"{np.mean(fixed):.3f}, regrouped by the previous env-step's totals {np.mean(pred):.3f}, by the current "
          f"env-step's (bound) {np.mean(best):.3f}")
    print(f"correlation of an env's per-env-step totals between consecutive env-steps: mean {np.mean(r):.3f} "
          f"(min {np.min(r):.3f}); totals: mean {tot[1:].mean():.2f}, std {tot[1:].std():.2f} per env-step")
    hist = np.bincount(its[1:].ravel(), minlength=6)
    print("per-substep iteration histogram (0..5):", (hist / hist.sum()).round(4).tolist())


if __name__ == "__main__":
    main()
