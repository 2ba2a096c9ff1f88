"""Multi-GPU sharding of the env batch (one process per GPU, RCCL over xGMI).

Envs are independent (no cross-env term anywhere in BallEnv.step /
prep_state4), so the batch is split into contiguous global-env-id ranges with
no data-path collective.  Every Philox stream is keyed by the global env id,
so a given env's trajectory is the same at 1, 2, 4 or 8 GPUs.  The only
collective is a periodic all_gather of each rank's fixed-size episode-return
record (8 f64) -- latency-bound, KB-sized.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard(total_envs: int, rank: int, world_size: int) -> Tuple[int, int]:
    """(env_offset, num_local) of ``rank``: contiguous, sizes differ by at most one."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("bad rank / world_size")
    base, rem = divmod(int(total_envs), int(world_size))
    n = base + (1 if rank < rem else 0)
    off = rank * base + min(rank, rem)
    return off, n


def gather_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """all_gather the (8,) f64 stats record of every rank -> (world, 8)."""
    if not (dist.is_available() and dist.is_initialized()):
        return stats.reshape(1, -1).clone()
    world = dist.get_world_size(group)
    src = stats.contiguous()
    if src.is_cuda and dist.get_backend(group) == "gloo":   # gloo rehearsal: gather through the host
        src = src.cpu()
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src, group=group)
    return torch.stack(out).to(stats.device)


def combine_stats(per_rank: torch.Tensor) -> dict:
    """Merge gathered records: counts/sums add, min/max reduce."""
    s = per_rank.double().cpu()
    n = float(s[:, 0].sum())
    tot = float(s[:, 1].sum())
    return {"episodes": int(n), "mean_return": tot / n if n else float("nan"),
            "sum_return": tot, "sum_return_sq": float(s[:, 2].sum()),
            "mean_length": float(s[:, 3].sum()) / n if n else float("nan"),
            "min_return": float(s[:, 4].min()), "max_return": float(s[:, 5].max())}
