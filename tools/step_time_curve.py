#!/usr/bin/env python3
"""Kernel time of each env-step after reset (C2 shape by default): does the driver's short bench
(--steps 20 --warmup 5) time a slower phase of the episode than a long run does?
usage: python tools/step_time_curve.py [--config C2] [--steps 120]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", type=int, default=120)
    a = ap.parse_args()
    c = CONFIGS[a.config]
    dev = torch.device("cuda:0")
    env = wrap_for_brax_training(Joystick(c["task"], num_envs=c["envs"], device=dev, use_imitation=c["imitation"]),
                                 episode_length=1000, randomization_fn=domain_randomize if c["dr"] else None)
    st = env.reset(rng=0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    pool = [torch.rand(c["envs"], env.action_size, device=dev, generator=g) * 2 - 1 for _ in range(8)]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    for i in range(a.steps):
        ev[i][0].record()
        st = env.step(st, pool[i % 8], inplace=True)
        ev[i][1].record()
    torch.cuda.synchronize()
    ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
    for lo in range(0, a.steps, 10):
        print(f"steps {lo:3d}-{lo + 9:3d}: " + " ".join(f"{x:.4f}" for x in ms[lo:lo + 10]))
    print(f"mean 5-25 {ms[5:25].mean():.4f}  mean 25-{a.steps} {ms[25:].mean():.4f}  "
          f"contacts at step 20: {int((st.obs['state'][:, 97:99] > 0).sum())}")


if __name__ == "__main__":
    main()
