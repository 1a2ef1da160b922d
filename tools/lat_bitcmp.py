#!/usr/bin/env python3
"""Latency vs throughput kernel, bit for bit (GPU box): each env-step taken by both kernels from the same
state (the throughput kernel's), 8 env-steps over auto-resets; prints, per config, how many fstate/obs
words differ, and (at the first env-step) which fstate fields. A config name may end in +dr / -dr to switch
domain randomisation on / off, and in @paired for the paired latency kernel.
usage: [DUCK_LIB=...] python tools/lat_bitcmp.py [C2 C3 C4 C5 C2+dr C4-dr C2@paired ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import CONFIGS  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402


def main():
    n = 512
    for name in sys.argv[1:] or ["C2", "C3"]:
        name, _, lmode = name.partition("@")
        lmode = lmode or "latency"
        cfg = name.rstrip("+-dr")
        c = dict(CONFIGS[cfg])
        if name.endswith("+dr") or name.endswith("-dr"):
            c["dr"] = name.endswith("+dr")
        g = torch.Generator(device="cuda:0")
        g.manual_seed(11)
        envs = {}
        for mode in ("throughput", lmode):
            env = wrap_for_brax_training(Joystick(c["task"], num_envs=n, device="cuda:0", use_imitation=c["imitation"]),
                                         episode_length=5, randomization_fn=domain_randomize if c["dr"] else None)
            env.set_step_mode(mode)
            envs[mode] = env
        st = envs["throughput"].reset(rng=4)
        diff = []
        for t in range(8):
            a = torch.rand(n, 14, device="cuda:0", generator=g) * 2 - 1
            s_t = envs["throughput"].step(st, a)
            s_l = envs[lmode].step(st, a)
            torch.cuda.synchronize()
            diff.append(int((s_t.fstate != s_l.fstate).sum()) + int((s_t.obs["state"] != s_l.obs["state"]).sum()))
            if t == 0:
                L = envs["throughput"]._layout
                d = (s_t.fstate != s_l.fstate).view(L.nfloat, n).sum(dim=1).cpu().numpy()
                bounds = sorted(L.off.items(), key=lambda kv: kv[1]) + [("end", L.nfloat)]
                first = {k: int(d[a:b].sum()) for (k, a), (_, b) in zip(bounds[:-1], bounds[1:]) if d[a:b].sum()}
            st = s_t
        print(f"{name}@{lmode}: differing fstate+obs words per env-step {diff}; first env-step by field {first}", flush=True)


if __name__ == "__main__":
    main()
