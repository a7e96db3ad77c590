"""World sharding across ranks: one process per GPU, rank r
owning the contiguous global worlds [r * W, (r + 1) * W) -- the simulator's
`world_offset` keys their RNG streams and synthetic actions, so the shards
concatenate bit-exactly to the unsharded run.  There is no collective on the
step path; `gather_observations` is the optional observation all-gather for a
learner that wants every world's rows in one tensor (RCCL over xGMI on the
GPU, gloo on the host), off unless called.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(total_worlds: int, rank: int, world_size: int) -> tuple[int, int]:
    """(world_offset, num_worlds) of `rank`'s contiguous shard; every rank gets
    the same count (total_worlds must divide evenly, as bench.py's weak
    scaling does)."""
    if total_worlds % world_size:
        raise ValueError(f"{total_worlds} worlds do not split evenly over {world_size} ranks")
    w = total_worlds // world_size
    return rank * w, w


def gather_observations(sim, agent: int | None = None, out: torch.Tensor | None = None, group=None) -> torch.Tensor:
    """All-gather of every rank's observation rows into one tensor, world-major
    in rank order: [world_size * W, N, OBSW] (or [world_size * W, OBSW] for one
    `agent`).  `out` may be passed to reuse a buffer.  Must be called by every
    rank of `group` (torch.distributed semantics)."""
    obs = sim.observations_tensor().to_torch()
    src = obs if agent is None else obs[:, agent]
    src = src.contiguous()
    ws = dist.get_world_size(group)
    shape = (ws * src.shape[0],) + tuple(src.shape[1:])
    if out is None:
        out = torch.empty(shape, dtype=src.dtype, device=src.device)
    elif tuple(out.shape) != shape or out.dtype != src.dtype or out.device != src.device or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous {src.dtype} tensor of shape {shape} on {src.device}")
    if src.device.type == "cuda":
        dist.all_gather_into_tensor(out, src, group=group)
    else:  # gloo: the list form
        dist.all_gather(list(out.chunk(ws)), src, group=group)
    return out
