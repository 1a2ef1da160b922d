#!/usr/bin/env python3
"""Per-stage cycle breakdown of step_kernel (needs a -DDUCK_STAGE_PROF build in DUCK_LIB).

Counters are wave-0 clock64 deltas summed over workgroups; printed per substep per wave.
Top-level stages (they partition a substep): 0-8, 20 and 28. Sub-stage counters measure from
the start of their parent stage: 9-13 solve, 16-18 newton direction, 19 crb limb/root
sums, 21/22 rne passes A/B, 24 kinematics local transforms, 26 floor collision.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from open_duck_playground_amd import native  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, wrap_for_brax_training  # noqa: E402

TOP = {0: "kinematics", 1: "com_pos", 2: "rne", 3: "crb", 28: "smooth (actuation, damping)",
       5: "collision", 6: "make_rows", 20: "M columns -> registers", 4: "qacc_smooth solve", 7: "solve",
       8: "sensors+euler"}
SUB = {24: "kinematics:local", 21: "rne:A vel/acc", 22: "rne:A+B forces", 35: "rne:C limb sums", 36: "rne:C root sums", 19: "crb:inertia sums",
       26: "collision:floor", 25: "solve:warm J,M products", 9: "solve:warm costs+select", 10: "solve:newton_dir", 16: "  newton:grad+diag",
       17: "  newton:+J'DJ", 18: "  newton:+factor_solve", 11: "solve:(dense fallback)", 12: "solve:jmul+mulM",
       13: "solve:linesearch", 37: "hfield: setup+screen+silhouettes", 38: "hfield: survivor queue", 39: "hfield: slots",
       41: "  queue: descriptors", 42: "  queue: per-lane SAT", 43: "  queue: gather",
       44: "    sat: vertical pairs", 45: "    sat: pass 1 (arc tests)", 47: "    sat: pass 2 (crossing pairs)"}
NSTAGE = 60  # DUCK_NSTAGE
ENV = {32: "env: hot state load", 33: "env: rng draws", 29: "env: pre-physics (per env-step)", 30: "env: contacts+obs",
       31: "env: termination+rewards+state", 34: "env: obs/priv stores", 15: "env: hot state store"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    rand = "--random" in sys.argv  # bench.py's U(-1,1) actions (more contacts than zero actions)
    task = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--task=")), "flat_terrain")
    env = wrap_for_brax_training(Joystick(task, num_envs=n, device="cuda:0", use_imitation=False),
                                 episode_length=1000)
    st = env.reset(rng=0)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1234)
    pool = [torch.rand(n, env.action_size, device="cuda:0", generator=g) * 2 - 1 for _ in range(8)] if rand else \
        [torch.zeros(n, env.action_size, device="cuda:0")]
    warm = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--warm=")), 20)
    for i in range(warm):
        st = env.step(st, pool[i % len(pool)], inplace=True)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (NSTAGE + 3 * 1024))()
    lib = native.lib()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    steps = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--steps=")), 5)
    for i in range(steps):
        st = env.step(st, pool[(warm + i) % len(pool)], inplace=True)
    torch.cuda.synchronize()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    nwg = (n + 15) // 16
    per_sub = lambda k: buf[k] / (nwg * steps * 10)
    tot = sum(buf[k] for k in TOP) or 1  # (0 in a -DDUCK_WAVE_PROF build: wave times only)
    for k, name in TOP.items():
        print(f"{name:28s} {per_sub(k):10.0f} cycles/substep/wave  {100 * buf[k] / tot:5.1f}%")
    for k, name in SUB.items():
        print(f"{name:28s} {per_sub(k):10.0f}")
    per = lambda k: buf[k] / (nwg * steps)
    for k, name in ENV.items():
        print(f"{name:28s} {per(k):10.0f} cycles/env-step/wave")
    import numpy as np
    w = np.array([buf[NSTAGE + i] for i in range(min(1024, 4 * nwg))], dtype=np.float64)
    w = w[w > 0]
    if len(w):
        print(f"{'wave cycles (last launch)':28s} mean {w.mean():.0f}  p50 {np.median(w):.0f}  p99 {np.quantile(w, 0.99):.0f}  "
              f"max {w.max():.0f}  max/mean {w.max() / w.mean():.3f}")
        if len(w) == 4 * nwg and "--waves" in sys.argv:
            wg = w.reshape(-1, 4)
            print("  per-workgroup max/min spread: mean %.3f" % (wg.max(1) / wg.min(1)).mean())
            print("  per-XCD (blockIdx % 8) mean wave cycles:", [int(wg[x::8].mean()) for x in range(8)])
            print("  per wave-in-workgroup mean:", [int(wg[:, k].mean()) for k in range(4)])
            print("  slowest workgroups:", [int(x) for x in np.argsort(wg.max(1))[-8:]])
            t0 = np.array([buf[NSTAGE + 1024 + i] for i in range(4 * nwg)], dtype=np.float64).reshape(-1, 4)
            t1 = np.array([buf[NSTAGE + 2048 + i] for i in range(4 * nwg)], dtype=np.float64).reshape(-1, 4)
            base = t0.min()
            us = lambda a: (a - base) / 100.0  # s_memrealtime: 100 MHz
            print("  wall clock per XCD (us from the first wave's start): start mean/max, end mean/max")
            for x in range(8):
                print(f"    XCD {x}: start {us(t0[x::8]).mean():7.1f} {us(t0[x::8]).max():7.1f}  "
                      f"end {us(t1[x::8]).mean():7.1f} {us(t1[x::8]).max():7.1f}  "
                      f"duration mean {((t1[x::8] - t0[x::8]) / 100).mean():7.1f}")
            print(f"  launch span (first start to last end): {us(t1).max():.1f} us")
    print(f"{'dense Newton fallbacks':28s} {buf[23] / steps:10.1f} per env-step (all {n} envs)")
    print(f"{'foot/foot SAT runs':28s} {buf[27] / steps:10.1f} per env-step (all {n} envs)")
    if buf[40]:
        print(f"{'hfield survivors':28s} {buf[40] / (nwg * steps * 10):10.2f} per substep (wave 0 of each workgroup: 8 feet)")
        print(f"{'hfield queue rounds':28s} {buf[46] / (nwg * steps * 10):10.2f} per substep (wave 0)")
        print(f"{'hfield pass-2 iterations':28s} {buf[48] / (nwg * steps * 10):10.2f} per substep (wave 0: the most crossing pairs of a lane)")
        print(f"{'hfield crossing pairs':28s} {buf[49] / (nwg * steps * 10):10.2f} per substep (wave 0: all survivors)")
        print(f"{'hfield crossing edges':28s} {buf[50] / (nwg * steps * 10):10.2f} per substep (wave 0: hull edges crossing in any survivor)")
        hist = [buf[k] for k in range(51, 56)]
        if sum(hist):
            print(f"{'hfield survivors per wave':28s} " + ", ".join(
                f"{lab}: {100 * v / sum(hist):.1f} %" for lab, v in zip(("<=21", "22-32", "33-42", "43-64", ">64"), hist)))
    outside = per(14) + sum(per(k) for k in ENV)
    kern = outside + tot / (nwg * steps)
    if per(14) == 0:
        return
    if buf[58] > 0:
        # line search (wave 0 of each workgroup): iterations the wave ran vs its teams needed
        print(f"{'line search iterations':28s} per team {buf[57] / buf[58]:.2f}, per wave {4 * buf[56] / buf[58]:.2f} "
              f"({buf[58] / (nwg * steps * 10) / 4:.2f} searches per team and substep)")
    print(f"{'kernel (per env-step)':28s} {kern:10.0f} cycles/env-step/wave (sum of the marked sections)")
    print(f"{'  model-table copy':28s} {per(14):10.0f}  {100 * per(14) / kern:5.1f}%")
    print(f"{'  10 substeps':28s} {tot / (nwg * steps):10.0f}  {100 * tot / (nwg * steps) / kern:5.1f}%")
    print(f"{'  env code outside':28s} {outside - per(14):10.0f}  {100 * (outside - per(14)) / kern:5.1f}%")


if __name__ == "__main__":
    main()
