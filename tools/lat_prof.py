#!/usr/bin/env python3
"""Timeline of one substep of the latency kernel (step_kernel_lat): clock64 at every cross-wave event of
substep 5 in workgroup 0, from a -DDUCK_LAT_PROF build (DUCK_LIB=...libduck_latprof.so), in cycles after
wave 0 starts the substep, averaged over the last launches.
usage: DUCK_LIB=open_duck_playground_amd/libduck_latprof.so python tools/lat_prof.py [--config C2] [--envs 512]"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402

NAMES = {0: "w0 start (Euler of s-1 seen)", 1: "w0 kinematics+com_pos done", 2: "w0 rne velocities done",
         3: "w0 rne + actuation done (qfrc_smooth)",
         10: "w1 com_pos seen", 11: "w1 composite inertias + crb done", 12: "w1 M columns loaded",
         13: "w1 rows seen", 14: "w1 warm start (qacc_warmstart) done", 15: "w1 qacc_smooth seen",
         16: "w1 warm start done", 17: "w1 Newton + line search done", 18: "w1 Euler done",
         20: "w2 com_pos seen", 21: "w2 collision done", 22: "w2 rne velocities seen", 23: "w2 rows done",
         30: "w3 crb seen", 31: "w3 M factored", 32: "w3 qfrc_smooth seen", 33: "w3 qacc_smooth done",
         34: "w3 warm start's rows seen", 35: "w3 speculative Newton direction done", 19: "w1 direction seen"}
# the paired kernel (step_kernel_lat<Md, 2>: waves A and B of env set 0 in workgroup 0)
NAMES2 = {0: "A start (Euler of s-1 seen)", 1: "A kinematics+com_pos done", 2: "A rne velocities done",
          3: "A rne + actuation done (qfrc_smooth)", 4: "A collision done", 5: "A rows done", 6: "A crb seen",
          7: "A warm start's rows seen", 8: "A speculative Newton direction done",
          10: "B com_pos seen", 11: "B composite inertias + crb done", 12: "B M columns loaded",
          13: "B warm start (qacc_warmstart products) done", 14: "B M factored", 15: "B qfrc_smooth seen",
          16: "B qacc_smooth done", 17: "B rows seen", 18: "B warm start's rows done", 19: "B warm start done",
          20: "B direction seen / own", 21: "B Newton + line search done", 22: "B Euler done"}
LAUNCH = {40: "kernel start", 41: "model blob in LDS", 42: "hot state staged", 43: "w0 env code before the substeps done",
          44: "w0 last Euler seen", 45: "w0 env code after the substeps done", 46: "final barrier"}
NSTAGE = 56


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--mode", default="latency", choices=["latency", "paired"])
    a = ap.parse_args()
    c = CONFIGS[a.config]
    dev = torch.device("cuda:0")
    env = wrap_for_brax_training(Joystick(c["task"], num_envs=a.envs, device=dev, use_imitation=c["imitation"]),
                                 episode_length=1000, randomization_fn=domain_randomize if c["dr"] else None)
    env.set_step_mode(a.mode)
    st = env.reset(rng=0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    buf = (C.c_ulonglong * (NSTAGE + 3 * 1024))()
    rows = []
    stage = np.zeros(64)
    nl = 0
    for t in range(a.steps):
        st = env.step(st, torch.rand(a.envs, 14, device=dev, generator=g) * 2 - 1, inplace=True)
        torch.cuda.synchronize()
        if env._lib.duck_debug_stage_cycles(env._sim, buf, 1) != 0:
            raise SystemExit("not a DUCK_LAT_PROF build")
        if t >= 10:
            stage += np.array([buf[NSTAGE + 64 + k] for k in range(64)], dtype=np.float64)
            nl += 1
            v = np.array([buf[NSTAGE + k] for k in range(48)], dtype=np.float64)
            v[:40] -= v[0]
            v[40:] -= v[40]
            rows.append(v)
    r = np.mean(rows, axis=0)
    print("launch (wave 0 of workgroup 0, cycles after its start):")
    for k in sorted(LAUNCH):
        print(f"{r[k]:9.0f}  {LAUNCH[k]}")
    print("substep 5:")
    names, last = (NAMES, 18) if a.mode == "latency" else (NAMES2, 22)
    for k in sorted(names, key=lambda k: r[k]):
        print(f"{r[k]:9.0f}  {names[k]}")
    print(f"substep (start -> Euler): {r[last]:.0f} cycles")
    # per-stage cycles (STAGE_MARK sums, workgroup 0), per substep
    from stage_prof import ENV, SUB, TOP  # noqa: E402
    names = {**TOP, **SUB, **ENV}
    per = stage / max(nl, 1) / env.n_substeps
    print("stage cycles per substep (marks from each stage function's start):")
    for k in np.argsort(-per):
        if per[k] > 0 and k in names:
            print(f"{per[k]:9.0f}  {names[k]}")


if __name__ == "__main__":
    main()
