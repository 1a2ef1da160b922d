"""Env-batch sharding across ranks (one process per GPU).

Envs are independent, so rank r of W owns the contiguous global env ids
[r * per_rank, (r + 1) * per_rank). Every per-env random stream (reset noise, commands,
pushes, domain randomisation) is keyed by the GLOBAL env id, so a sharded run produces
exactly the envs a single-rank run of W * per_rank envs would. No collective runs in the
step; callers that need batch statistics (the PPO outer loop) reduce them themselves.
"""

from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    per_rank: int

    @property
    def env_offset(self) -> int:
        return self.rank * self.per_rank

    @property
    def total_envs(self) -> int:
        return self.world * self.per_rank


def shard_from_env(per_rank: int) -> Shard:
    """Read RANK / WORLD_SIZE as set by torch.distributed.run."""
    return Shard(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(per_rank))
