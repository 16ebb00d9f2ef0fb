"""Frame sharding across the GPUs of one node (one process per GPU).

The hot path is independent per frame: each rank owns a
contiguous slice of the batch, voxelises it with no communication, and the
compact per-frame results (top-K proposal values and flat indices) are
collected with ONE all-gather -- RCCL over xGMI with the "nccl" backend, gloo
on CPU for tests.  Cubes and planes never leave their GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_frames(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, end) slice of ``n_frames`` for ``rank`` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack_proposals(vals: torch.Tensor, flat: torch.Tensor) -> torch.Tensor:
    """[B,K] fp32 values + [B,K] int64 indices -> [B, 2K] int64 (values bit-cast, lossless)."""
    return torch.cat([flat.to(torch.int64), vals.contiguous().view(torch.int32).to(torch.int64)], dim=1)


def unpack_proposals(packed: torch.Tensor, K: int) -> tuple[torch.Tensor, torch.Tensor]:
    flat = packed[:, :K].contiguous()
    vals = packed[:, K:].to(torch.int32).contiguous().view(torch.float32)
    return vals, flat


def gather_proposals(vals: torch.Tensor, flat: torch.Tensor, group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """All ranks' proposals in rank order (every rank must hold the same number of frames)."""
    K = vals.shape[1]
    local = pack_proposals(vals, flat)
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
    try:
        dist.all_gather_into_tensor(out, local, group=group)
    except (RuntimeError, NotImplementedError):  # backends without the fused form (older gloo)
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local, group=group)
        out = torch.cat(parts)
    return unpack_proposals(out, K)
