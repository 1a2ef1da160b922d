"""N>1 path on CPU: two gloo ranks each step their shard of envs (oracle), the gathered
result equals one rank stepping all envs (global-env-id keyed RNG, no data-path collective)."""

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from open_duck_playground_amd import constants
from open_duck_playground_amd.config import default_config, env_config_struct
from open_duck_playground_amd.mjcf import Model
from open_duck_playground_amd.sharding import Shard

PER_RANK, WORLD, STEPS = 5, 2, 3


def _run(shard: Shard, seed=4):
    from tests.oracle_ffi import OracleBatch, OracleModel
    m = Model.load(constants.task_to_xml("flat_terrain"))
    cfg = env_config_struct(m, default_config(), False, True)
    n = shard.per_rank
    b = OracleBatch(OracleModel(m), cfg, n)
    b.reset(seed=seed, env_offset=shard.env_offset, threads=1)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (STEPS, shard.total_envs, m.nu))
    for a in acts:
        b.step(a[shard.env_offset:shard.env_offset + n], threads=1)
    return np.concatenate([b.obs, b.priv, b.rew[:, None], b.done[:, None]], axis=1)


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    out = torch.from_numpy(_run(Shard(rank, WORLD, PER_RANK)))
    parts = [torch.zeros_like(out) for _ in range(WORLD)]
    dist.all_gather(parts, out)
    if rank == 0:
        q.put(torch.cat(parts).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_rank():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    got = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _run(Shard(0, 1, PER_RANK * WORLD))
    np.testing.assert_array_equal(got, ref)
