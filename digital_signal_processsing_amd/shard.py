"""Multi-GPU sharding of a long signal: one process per GPU, contiguous
frame-aligned shards, and a (k-1)-frame halo exchanged with point-to-point
send/recv over torch.distributed ("nccl" = RCCL over xGMI on MI355X; "gloo" on
CPU for tests).

The window is finite, so the only exchange step is the halo: shard r needs the
last (k-1)*C samples of shard r-1 (rank 0 uses zero history, the reference's
zero halo zone, gpu_utils.h:112-123).  There is no collective in the data
path; outputs stay sharded.  The message is (k-1)*C*elem bytes (4 KiB at
k=1024 fp32 mono), latency-bound on one xGMI link.  The reference has no
multi-GPU code at all; this is the north_star's sharding.
"""
from __future__ import annotations

from typing import Optional, Tuple


def shard_bounds(total_frames: int, world: int, rank: int) -> Tuple[int, int]:
    """[f0, f1) frames of `rank`: contiguous, balanced to within one frame."""
    base, rem = divmod(total_frames, world)
    f0 = rank * base + min(rank, rem)
    f1 = f0 + base + (1 if rank < rem else 0)
    return f0, f1


def exchange_halo(x_local, grade: int, channels: int = 1, group=None, recv_buf=None):
    """Send this shard's last (grade-1)*channels samples to rank+1 and receive
    rank-1's into the returned history tensor (None on rank 0 or when
    grade == 1).  Works for any backend whose tensors live where `x_local`
    lives.  Each shard must hold at least grade-1 frames.
    """
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    h = (grade - 1) * channels
    if h == 0 or world == 1:
        return None
    if x_local.numel() < h:
        raise ValueError(f"shard holds {x_local.numel()} samples < halo {h}: use fewer ranks or a smaller grade")
    ops = []
    if rank + 1 < world:
        tail = x_local[x_local.numel() - h:].contiguous()
        ops.append(dist.P2POp(dist.isend, tail, _peer(rank + 1, group), group))
    hist = None
    if rank > 0:
        hist = recv_buf if recv_buf is not None else torch.empty(h, dtype=x_local.dtype, device=x_local.device)
        ops.append(dist.P2POp(dist.irecv, hist, _peer(rank - 1, group), group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return hist


def _peer(group_rank: int, group) -> int:
    import torch.distributed as dist
    if group is None:
        return group_rank
    return dist.get_global_rank(group, group_rank)


def sharded_moving_average(x_local, grade: int, channels: int = 1, algo="auto", group=None,
                           out=None, recv_buf=None):
    """Moving average of the global signal whose shard this rank holds
    (device tensor); returns this rank's shard of the output."""
    from . import moving_average_into
    import torch

    hist = exchange_halo(x_local, grade, channels, group, recv_buf)
    if out is None:
        out = torch.empty_like(x_local)
    moving_average_into(x_local, out, grade, channels, algo, history=hist)
    return out
