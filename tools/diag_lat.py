#!/usr/bin/env python3
"""Latency vs throughput step kernel from identical states: per env-step, the largest relative
difference of qpos / qvel / obs / privileged obs / reward and how many envs differ at all or by more
than 1e-5 (rounding-level differences of differently inlined fp32 code vs a schedule defect).
usage: python tools/diag_lat.py [--config C2] [--envs 512] [--steps 8]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402


def rel(x, y):
    return ((x - y).abs() / (1 + y.abs())).max(dim=-1).values if x.dim() > 1 else (x - y).abs() / (1 + y.abs())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    c = CONFIGS[a.config]
    dev = torch.device("cuda:0")
    envs = {}
    for mode in ("throughput", "latency"):
        e = wrap_for_brax_training(Joystick(c["task"], num_envs=a.envs, device=dev, use_imitation=c["imitation"]),
                                   episode_length=1000, randomization_fn=domain_randomize if c["dr"] else None)
        e.set_step_mode(mode)
        e.lat_timeouts(reset=True)
        envs[mode] = e
    st = envs["throughput"].reset(rng=4)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    L = envs["throughput"]._layout
    o = L.off
    nq, nv = envs["throughput"].mj_model.nq, envs["throughput"].mj_model.nv
    for t in range(a.steps):
        act = torch.rand(a.envs, 14, device=dev, generator=g) * 2 - 1
        s_t = envs["throughput"].step(st, act)
        s_l = envs["latency"].step(st, act)
        torch.cuda.synchronize()
        ft, fl = s_t.fstate.view(L.nfloat, a.envs).T, s_l.fstate.view(L.nfloat, a.envs).T
        d = {"qpos": rel(fl[:, o["qpos"]:o["qpos"] + nq], ft[:, o["qpos"]:o["qpos"] + nq]),
             "qvel": rel(fl[:, o["qvel"]:o["qvel"] + nv], ft[:, o["qvel"]:o["qvel"] + nv]),
             "warm": rel(fl[:, o["qacc_warmstart"]:o["qacc_warmstart"] + nv], ft[:, o["qacc_warmstart"]:o["qacc_warmstart"] + nv]),
             "obs": rel(s_l.obs["state"], s_t.obs["state"]),
             "priv": rel(s_l.obs["privileged_state"], s_t.obs["privileged_state"]),
             "reward": rel(s_l.reward, s_t.reward)}
        line = " ".join(f"{k} {v.max().item():.1e}/{int((v > 0).sum())}/{int((v > 1e-5).sum())}" for k, v in d.items())
        print(f"step {t}: {line}  done mismatch {int((s_l.done != s_t.done).sum())}  "
              f"istate mismatch {int((s_l.istate != s_t.istate).sum())}", flush=True)
        st = s_t  # both continue from the throughput kernel's state
    print("timeouts", envs["latency"].lat_timeouts())


if __name__ == "__main__":
    main()
