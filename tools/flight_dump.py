#!/usr/bin/env python3
"""Dump the HIP forward qacc (and aux record) of the Newton-Euler flight states for offline analysis."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from open_duck_playground_amd.joystick import Joystick  # noqa: E402
from tests.physics_laws import flight_states  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "flat_terrain"
n = 4096
env = Joystick(task, num_envs=1, device="cuda:0", use_imitation=False)
m = env.mj_model
qpos, qvel, ctrl = flight_states(m, n, seed=7)
T = lambda a: torch.tensor(np.ascontiguousarray(a.T), dtype=torch.float32, device="cuda:0")
tq, tv, tw, tc = T(qpos), T(qvel), T(np.zeros((n, m.nv))), T(ctrl)
aux = torch.zeros(env.aux_size() * n, dtype=torch.float32, device="cuda:0").view(-1, n)
env.physics_step(tq, tv, tw, tc, 0, aux)
torch.cuda.synchronize()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/flight_{task}.npz", aux=aux.cpu().numpy())
print("saved", aux.shape)
