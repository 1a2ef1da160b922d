#!/usr/bin/env python3
"""Per-stage cycle breakdown of step_kernel (needs a -DDUCK_STAGE_PROF build in DUCK_LIB)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from open_duck_playground_amd import native  # noqa: E402
from open_duck_playground_amd.joystick import Joystick  # noqa: E402

NAMES = ["kinematics", "com_pos", "rne", "crb", "smooth+factor+solve_H", "collision", "make_rows", "solve",
         "sensors+euler", "solve:warmstart", "solve:newton_dir", "solve:factor+solve", "solve:jmul+mulM",
         "solve:linesearch"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    env = Joystick("flat_terrain", num_envs=n, device="cuda:0", use_imitation=False)
    st = env.reset(rng=0)
    a = torch.zeros(n, env.action_size, device="cuda:0")
    for _ in range(3):
        env.step(st, a)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    lib = native.lib()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    steps = 5
    for _ in range(steps):
        env.step(st, a)
    torch.cuda.synchronize()
    lib.duck_debug_stage_cycles(env._sim, buf, 1)
    tot = sum(buf[k] for k in range(9))
    nwg = (n + 15) // 16
    for k, name in enumerate(NAMES):
        print(f"{name:24s} {buf[k] / (nwg * steps * 10):12.0f} cycles/substep/wave  {100 * buf[k] / tot:5.1f}%")


if __name__ == "__main__":
    main()
