#!/usr/bin/env python3
"""Env-step throughput of the batched Open Duck Mini v2 Joystick env on MI355X.

Metric (BASELINE.json): env steps/sec (all envs), open_duck_mini_v2 flat, 4096 envs per GPU.
One env-step = one ``Joystick.step`` (joystick.py:323-481): 10 physics substeps + obs +
termination + reward, under the training wrappers (episode_length 1000, auto-reset), i.e.
what brax PPO drives through ``wrap_for_brax_training`` (common/runner.py:117).

Workload C2 (BASELINE.json configs[1]): flat terrain, no imitation reward, 4096 envs per
GPU, inputs (state, actions) resident in HBM. Actions are i.i.d. U(-1,1)^14 (seed 1234).
Multi-GPU: one process per GPU, envs sharded by global env id (env_offset = rank * envs),
no collective in the step -> weak scaling; the timed region is bracketed by barrier +
synchronize and the max over ranks is reported.

Extra JSON objects:
  roofline        the step kernel against HBM: algorithmic bytes per env-step
                  x envs per launch / average launch time from HIP events on the launch stream.
  issue_roofline  the same kernel against the chip's FP32 VALU issue rate (78.6 T lane-instr/s, a
                  wave64 v_fma_f32 every 2 cycles per SIMD), from the SQ counters of the committed
                  rocprofv3 run of this library (profiles/, checked against the library's build id),
                  with the rates measured on MI355X beside it (profiles/r06_valu_occupancy_probe.txt):
                  55.7 T at 8 waves per SIMD (measured_peak) and 29.1 T for one wave per SIMD, this
                  kernel's occupancy (one_wave_ceiling).
  cpu_baseline    the fp64 C oracle (oracle/, a restatement of the same step) over OpenMP on the
                  host cores this job may use (affinity, capped by the cgroup CPU quota), on a
                  bounded sample (rank 0, N=1 only), plus BASELINE configs[0] (C1): 1 env, 1 core.

--strong keeps 4096 envs in total over the N ranks (strong scaling) instead of 4096 per rank.

Launch: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>` as a child process
(before anything touches the GPU) and exits with its code; rank 0's JSON line reaches stdout
unchanged. Under an external torch.distributed.run (WORLD_SIZE set) it runs as that rank.
"""

from __future__ import annotations

import os
import sys


def _self_launch(argv) -> int:
    """Start one rank per GPU through torch.distributed.run as a child process (common/runner.py:104-118
    runs one pmap replica per local device; here one process per GPU). Nothing here initialises HIP:
    the parent only parses --gpus and waits, so there is no exec after a GPU context exists."""
    import socket
    import subprocess
    n = None
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            n = int(argv[i + 1])
        elif a.startswith("--gpus="):
            n = int(a.split("=", 1)[1])
    if n is None or n <= 1:
        return -1
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    # the ranks' stdout is relayed line by line: the bench line to stdout, anything else the launcher or a
    # communication library writes there (gloo announces its peers) to stderr, so stdout holds one line
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    import signal

    def _forward(sig, _frame):  # a time limit that stops this process stops the ranks too
        p.send_signal(sig)
    signal.signal(signal.SIGTERM, _forward)
    signal.signal(signal.SIGINT, _forward)
    for line in p.stdout:
        k = line.find('{"metric"')
        if k > 0:
            sys.stderr.write(line[:k] + "\n")
        if k >= 0:
            sys.stdout.write(line[k:])
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ:
    _rc = _self_launch(sys.argv[1:])
    if _rc >= 0:
        sys.exit(_rc)

import argparse  # noqa: E402
import glob  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from open_duck_playground_amd.joystick import Joystick, domain_randomize, wrap_for_brax_training  # noqa: E402
from open_duck_playground_amd.sharding import shard_from_env  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# FP32 VALU issue peak of the chip: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz = 78.6 T lane-instructions/s
# (a wave64 v_fma_f32 every 2 cycles on the 32-lane SIMD = the 157.3 TFLOPS vector spec / 2 for the FMA).
# Measured (profiles/r06_valu_occupancy_probe.txt, tools/valu_occupancy_probe.hip: independent v_fma_f32
# streams, wall clock of the whole launch): one wave per SIMD issues every 4.9 cycles (29.1 T for the
# chip), two waves 47.6 T, eight 55.7 T -- so the SIMD does issue faster than one wave alone can, and a
# kernel that registers hold at one wave per SIMD (this one) is capped near the one-wave rate
VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12
VALU_MEASURED_PEAK_TLANE = 55.74     # 8 waves per SIMD
VALU_ONE_WAVE_TLANE = 29.12          # 1 wave per SIMD
# newest tools/gpu_pmc.sh <rNN> C2 summary; only used when its build id matches the loaded library
def pmc_profile(config: str) -> str:
    """the newest committed rocprofv3 summary of a configuration (tools/gpu_pmc.sh), or a path that
    does not exist"""
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_{config.lower()}.json")))
    return found[-1] if found else os.path.join(ROOT, "profiles", f"r00_pmc_{config.lower()}.json")


# BASELINE.json configs[1..4] (configs[0] is the reference's 1-env CPU plumbing case)
CONFIGS = {
    "C2": dict(task="flat_terrain", imitation=False, dr=False, envs=4096),
    "C3": dict(task="flat_terrain", imitation=True, dr=False, envs=4096),
    "C4": dict(task="rough_terrain", imitation=False, dr=True, envs=8192),
    "C5": dict(task="rough_terrain_backlash", imitation=False, dr=True, envs=4096),  # 32768 over 8 GPUs
}


def algorithmic_bytes(env: Joystick) -> int:
    """Compulsory HBM bytes of one env-step of one env.

    read + write of the persistent per-env state the step carries (qpos .. imitation_phase,
    int counters and RNG words), read of the action, write of obs, privileged obs, reward,
    done, truncation and the 8 metrics. The auto-reset snapshot (first_*) is read only by
    envs that terminate and is not counted; the reference-motion row is counted only with
    imitation (it is untouched otherwise).
    """
    L = env._layout
    o = L.off
    state_f = o["metrics"] - o["qpos"]
    if not env.use_imitation:
        state_f -= 40
    state_i = L.nint
    rd = 4 * (state_f + state_i + L.nu)
    wr = 4 * (state_f + state_i + L.obs_size + L.priv_size + 1 + 1 + 1 + 8)
    if env.dr is not None:
        rd += 4 * env.dr.numel() // env.num_envs
    return rd + wr


def host_cores() -> int:
    """Host cores this process may use: its CPU affinity, capped by the cgroup CPU quota (the GPU box
    gives a job a share of a larger machine; nproc/affinity show the whole machine there)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def build_id() -> str:
    """sha1 of the sources + flags libduck.so was built from (duck_build_id, native.build)."""
    from open_duck_playground_amd.native import lib
    return lib().duck_build_id().decode()


def cpu_baseline_c1(task: str, use_imitation: bool, budget_s: float):
    """BASELINE configs[0]: one env on one core (the reference's CPU plumbing case)."""
    from open_duck_playground_amd.config import default_config, env_config_struct
    from open_duck_playground_amd.joystick import OpenDuckMiniV2Env
    from open_duck_playground_amd import constants
    from tests.oracle_ffi import OracleBatch, OracleModel

    base = OpenDuckMiniV2Env(xml_path=constants.task_to_xml(task), config=default_config())
    m = base.mj_model
    batch = OracleBatch(OracleModel(m), env_config_struct(m, base._config, use_imitation, True, False), 1)
    batch.reset(seed=0, threads=1)
    acts = np.random.default_rng(1234).uniform(-1, 1, (4, 1, m.nu))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        batch.step(acts[steps % 4], threads=1)
        steps += 1
    el = time.perf_counter() - t0
    return {"value": steps / el, "unit": "env-steps/s", "cores": 1, "envs": 1,
            "sample": f"C1: {task}, 1 env x {steps} env-steps ({el:.1f} s), fp64 oracle, 1 thread"}


def cpu_baseline(task: str, use_imitation: bool, budget_s: float, threads: int):
    """Time the fp64 C oracle (same step semantics) on host cores: OpenMP, one env per thread-iteration."""
    from open_duck_playground_amd.config import default_config, env_config_struct
    from open_duck_playground_amd.joystick import OpenDuckMiniV2Env
    from open_duck_playground_amd import constants
    from tests.oracle_ffi import OracleBatch, OracleModel

    base = OpenDuckMiniV2Env(xml_path=constants.task_to_xml(task), config=default_config())
    m = base.mj_model
    cfg = env_config_struct(m, base._config, use_imitation, True, False)
    n = 32 * threads
    batch = OracleBatch(OracleModel(m), cfg, n)
    batch.reset(seed=0, threads=threads)
    rng = np.random.default_rng(1234)
    acts = rng.uniform(-1, 1, (4, n, m.nu))
    batch.step(acts[0], threads=threads)  # warm-up
    steps, t0 = 0, time.perf_counter()
    while True:
        batch.step(acts[steps % 4], threads=threads)
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": n * steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{task} (nominal model), {n} envs x {steps} env-steps ({el:.1f} s), fp64 oracle, "
                      f"OpenMP {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS),
                    help="BASELINE.json workload: C2 flat (the metric), C3 +imitation, C4 rough+DR, C5 rough+DR+backlash")
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (0 = the config's)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline sampling (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every host core this job may use")
    ap.add_argument("--strong", action="store_true", help="4096 envs in total over the ranks (strong scaling)")
    ap.add_argument("--step-mode", default="auto", choices=["auto", "throughput", "latency", "paired", "latency_x2"],
                    help="duck_set_step_mode: auto = the latency kernel at <= 4 envs per CU, at <= 8 the latency "
                         "kernel at two workgroups per CU (flat scenes) or the paired latency kernel (strong scaling)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: one rank per GPU "
                         "(run `bench.py --gpus N` directly, or under torch.distributed.run --nproc-per-node N)")
    ndev = torch.cuda.device_count()
    backend = os.environ.get("DUCK_DIST_BACKEND", "nccl")  # nccl = RCCL; gloo only to rehearse on one GPU
    if world > 1 and backend == "nccl" and world > ndev:
        raise SystemExit(f"--gpus {world} but only {ndev} visible GPU(s): RCCL runs one rank per device "
                         "(DUCK_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    cfg = CONFIGS[args.config]
    n = args.envs or cfg["envs"]
    if args.strong:
        n = max(1, n // world)
    shard = shard_from_env(n)
    env = Joystick(cfg["task"], num_envs=n, device=dev, use_imitation=cfg["imitation"], env_offset=shard.env_offset)
    env = wrap_for_brax_training(env, episode_length=1000, randomization_fn=domain_randomize if cfg["dr"] else None)
    env.set_step_mode(args.step_mode)
    state = env.reset(rng=0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    pool = [torch.rand(n, env.action_size, device=dev, generator=g) * 2 - 1 for _ in range(8)]

    for i in range(args.warmup):
        env.step(state, pool[i % len(pool)], inplace=True)
    K = args.steps
    # launch durations from HIP events on every 8th timed launch: bracketing every launch puts two
    # event records between back-to-back kernels and cost 2.3 % of the wall time (same box, 400
    # steps: 0.2815 vs 0.2753 ms per step) without changing the measured launch duration
    EV_EVERY = int(os.environ.get("DUCK_EV_EVERY", "8"))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if i % EV_EVERY == 0 else None
          for i in range(K)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_all = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev_all[0].record()
    for i in range(K):
        if ev[i] is not None:
            ev[i][0].record()
            env.step(state, pool[i % len(pool)], inplace=True)
            ev[i][1].record()
        else:
            env.step(state, pool[i % len(pool)], inplace=True)
    ev_all[1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # average launch duration: events around every 8th launch, never above the events around all
    # K back-to-back launches on the same stream (a true upper bound: the launches serialise)
    kern_ms = min(float(np.mean([p[0].elapsed_time(p[1]) for p in ev if p is not None])),
                  ev_all[0].elapsed_time(ev_all[1]) / K)
    ok = bool(torch.isfinite(state.obs["state"]).all().item())

    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        thr = args.cpu_threads or host_cores()
        cpu = cpu_baseline(cfg["task"], cfg["imitation"], args.cpu_budget, thr)
        cpu["host_cores"] = host_cores()
        cpu["affinity_cpus"] = len(os.sched_getaffinity(0))
        cpu["c1"] = cpu_baseline_c1(cfg["task"], cfg["imitation"], min(5.0, args.cpu_budget))

    # PMC numbers of the committed rocprofv3 run of this configuration (tools/gpu_pmc.sh); valid
    # only for the library they were measured on
    traffic, issue_rf = None, None
    pmc = pmc_profile(args.config)
    if os.path.exists(pmc) and n == CONFIGS[args.config]["envs"]:
        prof = json.load(open(pmc))
        current = prof.get("build_id") == build_id()
        src = {"source": os.path.relpath(pmc, ROOT), "build_id_matches": current}
        if current:
            traffic = prof["hbm_bytes_per_launch"]
            valu = prof["SQ_INSTS_VALU"] * 64 / (kern_ms * 1e-3) / 1e12     # lane-instructions / s
            issue_rf = {"bound": "valu", "achieved": valu, "peak": VALU_PEAK_TLANE, "unit": "T lane-instr/s",
                        "frac": valu / VALU_PEAK_TLANE, "measured_peak": VALU_MEASURED_PEAK_TLANE,
                        "frac_of_measured_peak": valu / VALU_MEASURED_PEAK_TLANE,
                        "one_wave_ceiling": VALU_ONE_WAVE_TLANE,
                        "frac_of_one_wave_ceiling": valu / VALU_ONE_WAVE_TLANE,
                        "valu_insts_per_launch": prof["SQ_INSTS_VALU"],
                        "valu_busy_frac": prof["valu_busy_frac"], "waitcnt_frac": prof["waitcnt_frac"], **src}
        else:  # another build's counters: no rate is derived from them
            issue_rf = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_TLANE, "unit": "T lane-instr/s",
                        "frac": None, **src}
    if rank == 0:
        B = algorithmic_bytes(env)
        achieved = B * n / (kern_ms * 1e-3) / 1e9
        total = world * n * K
        metric = "env steps/sec (all envs) open_duck_mini_v2 flat, 4096 envs, 1/2/4/8 GPUs"  # BASELINE.json
        if args.config != "C2" or args.strong or n != cfg["envs"]:
            metric = (f"env steps/sec (all envs) open_duck_mini_v2 {cfg['task']}"
                      f"{' + imitation' if cfg['imitation'] else ''}{' + DR' if cfg['dr'] else ''}, "
                      f"{world * n} envs over {world} GPU(s)")
        line = {
            "metric": metric,
            "value": total / el, "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
            "ms_per_step": el / K * 1e3, "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (keyframe home + reset randomisation, actions U(-1,1)^14)",
            "config": {"workload": f"{args.config}: {cfg['task']}, {'imitation' if cfg['imitation'] else 'no imitation'}"
                                   f"{', domain randomization' if cfg['dr'] else ''}, {n} envs per GPU, "
                                   "episode_length 1000 + auto-reset",
                       "envs_per_gpu": n, "total_envs": world * n, "substeps": env.n_substeps,
                       "parallelism": f"env-shard x{world}", "step_kernel": env.step_kernel},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": {"throughput": "step_kernel", "latency": "step_kernel_lat<1>",
                                    "paired": "step_kernel_lat<2>", "latency_x2": "step_kernel_lat_x2"}[env.step_kernel],
                         "kernel_ms": kern_ms, "bytes_per_env_step": B},
            "issue_roofline": issue_rf,
            "cpu_baseline": cpu,
            "finite": ok,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
