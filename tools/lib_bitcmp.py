#!/usr/bin/env python3
"""Bit-identity of two libduck builds on a bench workload (GPU box, one library per process).

Runs a bench.py configuration (C2-C5: task, imitation, domain randomization) with the library in
DUCK_LIB for --steps env-steps of bench.py's action pool, then writes the SoA state (fstate,
istate), obs and reward to --out. With --cmp A.npz B.npz (no GPU) it reports the first step and
field where the two runs differ, or that they are identical bit for bit. A kernel change meant to
reorder work without changing any arithmetic (tools/gpu_ab_bitcmp.sh) is checked this way.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def run(args):
    import torch
    from bench import CONFIGS
    from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training
    cfg = CONFIGS[args.config]
    n = args.envs or cfg["envs"]
    env = Joystick(cfg["task"], num_envs=n, device="cuda:0", use_imitation=cfg["imitation"])
    env = wrap_for_brax_training(env, episode_length=1000, randomization_fn=domain_randomize if cfg["dr"] else None)
    st = env.reset(rng=0)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1234)
    pool = [torch.rand(n, env.action_size, device="cuda:0", generator=g) * 2 - 1 for _ in range(8)]
    snaps = {}
    for i in range(args.steps):
        st = env.step(st, pool[i % len(pool)], inplace=True)
        if (i + 1) % args.every == 0 or i + 1 == args.steps:
            torch.cuda.synchronize()
            snaps[f"f{i + 1}"] = st.fstate.detach().cpu().numpy().copy()
            snaps[f"i{i + 1}"] = st.istate.detach().cpu().numpy().copy()
    np.savez_compressed(args.out, **snaps)
    print(f"{args.config} {n} envs, {args.steps} steps -> {args.out}")


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    keys = sorted(A.files, key=lambda k: (int(k[1:]), k[0]))
    for k in keys:
        x, y = A[k], B[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        if not same:
            bad = np.argwhere(x.view(np.uint32) != y.view(np.uint32))
            fx, fy = x.reshape(-1), y.reshape(-1)
            i0 = int(np.argmax(fx.view(np.uint32) != fy.view(np.uint32)))
            msg = f"DIFFER at {k}: {len(bad)} of {x.size} words, first flat index {i0}: {fx[i0]!r} vs {fy[i0]!r}"
            if x.dtype.kind == "f":
                d = np.abs(fx.astype(np.float64) - fy.astype(np.float64))
                msg += f", max |diff| {np.nanmax(d):.3g}"
            print(msg)
            return 1
    print(f"bit-identical over {len(keys)} snapshots")
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/bitcmp.npz")
    ap.add_argument("--cmp", nargs=2)
    ap.add_argument("--envs-of", type=int, default=0, help="with --cmp: per-env summary (fstate as [nfloat, n])")
    args = ap.parse_args()
    if args.cmp:
        if args.envs_of:
            A, B = np.load(args.cmp[0]), np.load(args.cmp[1])
            for k in sorted((k for k in A.files if k[0] == "f"), key=lambda k: int(k[1:])):
                x = A[k].reshape(-1, args.envs_of).astype(np.float64)
                y = B[k].reshape(-1, args.envs_of).astype(np.float64)
                d = np.abs(x - y)
                rel = d / np.maximum(np.abs(x), 1e-3)
                print(f"{k}: envs differing {int((d > 0).any(0).sum())}, rel > 1e-5 {int((rel > 1e-5).any(0).sum())}, "
                      f"rel > 1e-3 {int((rel > 1e-3).any(0).sum())}, max rel {np.nanmax(rel):.3g}")
            sys.exit(0)
        sys.exit(cmp(*args.cmp))
    run(args)


if __name__ == "__main__":
    main()
