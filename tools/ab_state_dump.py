#!/usr/bin/env python3
"""Dump the state after K env-steps of a fixed seeded rollout (for bit-identity A/B checks between two
builds: run once per library with DUCK_LIB set, then compare the .npz files).
usage: DUCK_LIB=... python tools/ab_state_dump.py out.npz [--task flat_terrain] [--envs 1024] [--steps 50]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--task", default="flat_terrain")
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    env = wrap_for_brax_training(Joystick(a.task, num_envs=a.envs, device="cuda:0"), episode_length=1000,
                                 randomization_fn=domain_randomize, rng=7)
    state = env.reset(rng=3)
    g = torch.Generator(device="cuda:0").manual_seed(11)
    for _ in range(a.steps):
        act = torch.rand(a.envs, env.action_size, device="cuda:0", generator=g) * 2 - 1
        env.step(state, act, inplace=True)
    torch.cuda.synchronize()
    np.savez(a.out, obs=state.obs["state"].cpu().numpy(), priv=state.obs["privileged_state"].cpu().numpy(),
             fstate=state.fstate.cpu().numpy(), reward=state.reward.cpu().numpy())


if __name__ == "__main__":
    main()
