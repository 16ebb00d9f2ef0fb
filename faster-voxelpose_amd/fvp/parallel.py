"""Frame sharding across the GPUs of one node (one process per GPU).

The hot path is independent per frame: each rank owns a
contiguous slice of the batch, voxelises it with no communication, and the
compact per-frame results (top-K proposal values and flat indices) are
collected with ONE all-gather -- RCCL over xGMI with the "nccl" backend, gloo
on CPU for tests.  Cubes and planes never leave their GPU.

Large-frame mode (for C5-sized grids at small batch): every
rank holds the same frames and voxelises one x-slab of each
(ProjectLayer.forward_slab); ONE all-gather assembles the xy planes for the
replicated CenterNet / NMS, and ONE all-reduce of the K proposal columns
(each owned by exactly one rank, zeros elsewhere) replaces the local column
gather.  Cube slabs never leave their GPU.
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


def _joint_buffer(vals: torch.Tensor, flat: torch.Tensor):
    """The uint8 buffer holding flat [B,K] int64 then vals [B,K] fp32 back to back
    (fvp.ops.proposal_buffers, as the NMS writes them), or None."""
    n = flat.numel()
    if (flat.dtype != torch.int64 or vals.dtype != torch.float32 or vals.shape != flat.shape or n == 0
            or not flat.is_contiguous() or not vals.is_contiguous()):
        return None
    st = flat.untyped_storage()
    if (vals.untyped_storage().data_ptr() != st.data_ptr() or st.nbytes() != 12 * n or flat.storage_offset() != 0
            or vals.data_ptr() != flat.data_ptr() + 8 * n):
        return None
    return torch.empty(0, dtype=torch.uint8, device=flat.device).set_(st, 0, (12 * n,))


def gather_proposals(vals: torch.Tensor, flat: torch.Tensor, group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """All ranks' proposals in rank order (every rank must hold the same number of frames)."""
    B, K = vals.shape
    world = dist.get_world_size(group)
    if world == 1:  # nothing to exchange: the rank's own proposals (no collective launch)
        return vals, flat
    buf = _joint_buffer(vals, flat)
    # (nccl = RCCL and gloo both implement the fused form; any failure, a
    # timeout included, propagates -- no second collective is attempted)
    if buf is None:  # separate tensors: pack them into one (two small kernels)
        local = pack_proposals(vals, flat)
        out = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local, group=group)
        return unpack_proposals(out, K)
    # the NMS wrote both into one buffer: it leaves as it is, and every rank's
    # part is read back through views (copies only to merge ranks, N > 1)
    n = B * K
    out = torch.empty((world * 12 * n,), dtype=torch.uint8, device=buf.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    rows = out.view(world, 12 * n)
    flat_all = rows[:, : 8 * n].contiguous().view(torch.int64) if world > 1 else rows[0, : 8 * n].view(torch.int64)
    vals_all = rows[:, 8 * n:].contiguous().view(torch.float32) if world > 1 else rows[0, 8 * n:].view(torch.float32)
    return vals_all.reshape(world * B, K), flat_all.reshape(world * B, K)


def shard_slab(X: int, world: int, rank: int) -> tuple[int, int]:
    """x-slab [x0, x1) of an X-row voxel grid for ``rank`` (sizes differ by at most one)."""
    if X < world:
        raise ValueError(f"cannot split {X} x-rows over {world} ranks")
    return shard_frames(X, world, rank)


def gather_xy_slabs(xy_slab: torch.Tensor, X: int, group=None) -> torch.Tensor:
    """Every rank's [B,J,x1-x0,Y] xy slab -> the full [B,J,X,Y] planes on every rank."""
    world = dist.get_world_size(group)
    B, J, _, Y = xy_slab.shape
    spans = [shard_slab(X, world, r) for r in range(world)]
    xm = max(e - s for s, e in spans)
    local = xy_slab.new_zeros((xm, B, J, Y))
    local[: xy_slab.shape[2]] = xy_slab.permute(2, 0, 1, 3)  # x-major so the gather concatenates slabs
    out = xy_slab.new_empty((world * xm, B, J, Y))
    dist.all_gather_into_tensor(out, local, group=group)
    rows = torch.cat([out[r * xm: r * xm + (e - s)] for r, (s, e) in enumerate(spans)])
    return rows.permute(1, 2, 0, 3).contiguous()


def owned_columns(cube_slab: torch.Tensor, flat: torch.Tensor, x0: int, gather=None) -> torch.Tensor:
    """This rank's share of feature_1d [B,K,J,Z] (human_detection_net.py:199-200)
    for proposals at global flat index x*Y + y, from x-slabs [B,J,Xs,Y,Z]
    starting at row x0: the columns whose x-row lies in the slab, zeros
    elsewhere (every column is owned by exactly one slab)."""
    if gather is None:
        from .proposal import gather_columns as gather
    Xs, Y = cube_slab.shape[2], cube_slab.shape[3]
    local = flat - x0 * Y
    own = (local >= 0) & (local < Xs * Y)
    cols = gather(cube_slab, torch.where(own, local, torch.zeros_like(local)))
    return torch.where(own[:, :, None, None], cols, torch.zeros((), dtype=cols.dtype, device=cols.device))


def columns_from_slab(cube_slab: torch.Tensor, flat: torch.Tensor, x0: int, group=None, gather=None) -> torch.Tensor:
    """feature_1d [B,K,J,Z] on every rank from each rank's owned_columns: one
    SUM all-reduce (exact: one non-zero term per element)."""
    cols = owned_columns(cube_slab, flat, x0, gather)
    dist.all_reduce(cols, op=dist.ReduceOp.SUM, group=group)
    return cols
