"""Training throughput of the PPO outer loop at the reference's config (8192 envs, unroll 20).

python tools/ppo_throughput.py [--updates 5] [--task flat_terrain]
Prints one JSON line: env-steps/s of whole PPO updates (rollout + learning), and the split.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from open_duck_playground_amd import ppo  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=5)
    ap.add_argument("--task", default="flat_terrain")
    ap.add_argument("--envs", type=int, default=8192)
    a = ap.parse_args()
    cfg = ppo.PPOConfig(num_envs=a.envs, num_evals=0)
    env = wrap_for_brax_training(Joystick(a.task, num_envs=a.envs, device="cuda:0"), episode_length=1000,
                                 randomization_fn=domain_randomize, rng=0)
    ppo.train(env, cfg, max_updates=1)  # warm-up (allocations, kernels)
    torch.cuda.synchronize()
    t0 = time.time()
    res = ppo.train(env, cfg, max_updates=a.updates)
    torch.cuda.synchronize()
    dt = time.time() - t0
    out = {"what": "PPO training env-steps/s (rollout + learning)", "task": a.task, "envs": a.envs,
           "updates": a.updates, "env_steps": res.env_steps, "seconds": dt, "value": res.env_steps / dt,
           "timing": res.timing, "last": res.metrics[-1]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
