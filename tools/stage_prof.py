#!/usr/bin/env python3
"""Per-stage cycle breakdown of step_kernel (needs a -DDUCK_STAGE_PROF build in DUCK_LIB)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from open_duck_playground_amd import native  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, wrap_for_brax_training  # noqa: E402

NAMES = ["kinematics", "com_pos", "rne", "crb", "smooth+factor+solve_H", "collision", "make_rows", "solve",
         "sensors+euler", "solve:warmstart", "solve:newton_dir", "solve:factor+solve", "solve:jmul+mulM",
         "solve:linesearch"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    rand = "--random" in sys.argv  # bench.py's U(-1,1) actions (more contacts than zero actions)
    env = wrap_for_brax_training(Joystick("flat_terrain", num_envs=n, device="cuda:0", use_imitation=False),
                                 episode_length=1000)
    st = env.reset(rng=0)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1234)
    pool = [torch.rand(n, env.action_size, device="cuda:0", generator=g) * 2 - 1 for _ in range(8)] if rand else \
        [torch.zeros(n, env.action_size, device="cuda:0")]
    a = pool[0]
    for i in range(20):
        env.step(st, pool[i % len(pool)])
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    lib = native.lib()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    steps = 5
    for i in range(steps):
        env.step(st, pool[i % len(pool)])
    torch.cuda.synchronize()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    tot = sum(buf[k] for k in range(9))
    nwg = (n + 15) // 16
    for k, name in enumerate(NAMES):
        print(f"{name:24s} {buf[k] / (nwg * steps * 10):12.0f} cycles/substep/wave  {100 * buf[k] / tot:5.1f}%")
    per = lambda k: buf[k] / (nwg * steps)
    kern = per(14) + per(15)
    print(f"{'kernel (per env-step)':24s} {kern:12.0f} cycles/env-step/wave")
    print(f"{'  model-table copy':24s} {per(14):12.0f}  {100 * per(14) / kern:5.1f}%")
    print(f"{'  10 substeps':24s} {tot / (nwg * steps):12.0f}  {100 * tot / (nwg * steps) / kern:5.1f}%")
    print(f"{'  env code outside':24s} {per(15) - tot / (nwg * steps):12.0f}  "
          f"{100 * (per(15) - tot / (nwg * steps)) / kern:5.1f}%")


if __name__ == "__main__":
    main()
