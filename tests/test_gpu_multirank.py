"""Two ranks through bench.py on the one GPU of a test box (gloo stands in for RCCL, which refuses
two ranks on one device): the rank launch, env sharding by global env id, the barrier-bracketed
timed region with the max over ranks, weak and strong scaling lines. The 1/2/4/8-GPU RCCL runs are
the driver's (SCALE_rNN.json)."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(extra):
    env = dict(os.environ, DUCK_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "20", "--warmup", "5", "--cpu-budget", "0"] + extra
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout   # rank 0 prints one line
    return json.loads(lines[0])


def _bench_direct(extra):
    """`python bench.py --gpus 2` with no launcher: bench.py starts torch.distributed.run itself."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DUCK_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--cpu-budget", "0"] + extra
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout   # exactly rank 0's line
    return json.loads(lines[0])


def test_direct_launch_two_ranks(gpu):
    """the driver's `python3 bench.py --gpus N ...` form (no WORLD_SIZE) runs N ranks."""
    d = _bench_direct([])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["finite"]
    assert d["config"]["total_envs"] == 8192 and d["config"]["step_kernel"] == "throughput"


def test_direct_launch_strong_takes_the_x2_latency_kernel(gpu):
    d = _bench_direct(["--strong"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["envs_per_gpu"] == 2048
    assert d["config"]["step_kernel"] == "latency_x2"


def test_two_rank_weak_scaling_line(gpu):
    d = _bench([])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["finite"]
    assert d["config"]["total_envs"] == 8192 and d["config"]["envs_per_gpu"] == 4096
    assert d["value"] == pytest.approx(8192 * 20 / (d["ms_per_step"] * 20 / 1e3), rel=1e-6)


def test_two_rank_strong_scaling_line(gpu):
    d = _bench(["--strong"])
    assert d["scaling"] == "strong" and d["config"]["total_envs"] == 4096 and d["config"]["envs_per_gpu"] == 2048
