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


def head_frames(grade: int, nframes: int) -> int:
    """Frames at the start of a shard whose window reaches into the previous
    shard: [0, grade-1), rounded up to 64 frames so the interior launch starts
    16-byte aligned."""
    if grade <= 1:
        return 0
    return min(nframes, (grade - 1 + 63) // 64 * 64)


def start_halo_exchange(x_local, grade: int, channels: int = 1, group=None, recv_buf=None, peers=None):
    """Post the halo send (this shard's last (grade-1)*channels samples to
    rank+1) and receive (rank-1's tail); returns (requests, history) where
    history is None on rank 0 / grade 1.  Wait on the requests before using
    history; with NCCL (= RCCL) the wait makes the current stream wait.
    `peers` = (receive-from, send-to) group ranks (None: no such peer) replaces
    rank - 1 / rank + 1: a one-rank communicator can then exchange with itself,
    which is how tests/test_rccl_one_device.py runs this RCCL path on a
    one-GPU box."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [], None
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    h = (grade - 1) * channels
    if peers is None:
        peers = (rank - 1 if rank > 0 else None, rank + 1 if rank + 1 < world else None)
    src, dst = peers
    if h == 0 or (src is None and dst is None):
        return [], None
    if x_local.numel() < h:
        raise ValueError(f"shard holds {x_local.numel()} samples < halo {h}: use fewer ranks or a smaller grade")
    # gloo cannot move device tensors: stage the halo through host memory
    # (rehearsal / CPU-only use; the measured multi-GPU path is NCCL = RCCL)
    staged = x_local.is_cuda and dist.get_backend(group) != "nccl"
    # RCCL's process group takes no int16 ("Short") tensors: the halo moves as its bytes (a uint8
    # view of the same memory, no copy) -- found by tests/test_rccl_one_device.py on MI355X
    as_bytes = (lambda t: t.view(torch.uint8)) if not staged and dist.get_backend(group) == "nccl" else (lambda t: t)
    ops = []
    if dst is not None:
        tail = x_local[x_local.numel() - h:]
        if staged:
            tail = tail.cpu()
        ops.append(dist.P2POp(dist.isend, as_bytes(tail), _peer(dst, group), group))
    hist = None
    wire = None
    if src is not None:
        hist = recv_buf if recv_buf is not None else torch.empty(h, dtype=x_local.dtype, device=x_local.device)
        wire = torch.empty(h, dtype=x_local.dtype) if staged else hist
        ops.append(dist.P2POp(dist.irecv, as_bytes(wire), _peer(src, group), group))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    if staged and wire is not None:
        reqs = [_StagedRecv(reqs, wire, hist)]
    return reqs, hist


class _StagedRecv:
    """Completes the host-staged receive: wait, then copy the halo to the device."""

    def __init__(self, reqs, wire, dst):
        self.reqs, self.wire, self.dst = reqs, wire, dst

    def wait(self):
        for r in self.reqs:
            r.wait()
        self.dst.copy_(self.wire)


def exchange_halo(x_local, grade: int, channels: int = 1, group=None, recv_buf=None):
    """Blocking form of start_halo_exchange: returns the history tensor."""
    reqs, hist = start_halo_exchange(x_local, grade, channels, group, recv_buf)
    for r in reqs:
        r.wait()
    return hist


def _peer(group_rank: int, group) -> int:
    import torch.distributed as dist
    if group is None:
        return group_rank
    return dist.get_global_rank(group, group_rank)


def split_moving_average_into(x_local, out, grade: int, channels: int = 1, algo="auto", history=None,
                              events=None, before_head=None, head_events=None) -> None:
    """out = moving average of x_local given `history` (the (grade-1)*channels
    samples before it, None = zeros) as two launches: the interior (frames >=
    head_frames(), history taken from inside x_local) first, then -- after
    `before_head()` (e.g. waiting for the halo) -- the head.  Same result as
    one launch with `history`; the split only lets the halo arrive late.
    `events` / `head_events`: optional (start, end) CUDA events recorded around
    the interior / the head launch (bench.py's per-rank timing)."""
    from . import moving_average_into

    C = channels
    nframes = x_local.numel() // C
    head = head_frames(grade, nframes)
    if head < nframes:
        if events is not None:
            events[0].record()
        interior_hist = x_local[(head - (grade - 1)) * C: head * C] if head > 0 else None
        moving_average_into(x_local[head * C:], out[head * C:], grade, C, algo, history=interior_hist)
        if events is not None:
            events[1].record()
    if before_head is not None:
        before_head()
    if head_events is not None:
        head_events[0].record()
    if head > 0:
        moving_average_into(x_local[: head * C], out[: head * C], grade, C, algo,
                            history=history() if callable(history) else history)
    if head_events is not None:
        head_events[1].record()


def sharded_moving_average(x_local, grade: int, channels: int = 1, algo="auto", group=None,
                           out=None, recv_buf=None, events=None, head_events=None):
    """Moving average of the global signal whose shard this rank holds
    (device tensor); returns this rank's shard of the output.  The halo
    send/recv is posted first and overlaps the interior launch; only the head
    launch waits for it.  `events` = optional (start, end) CUDA events around
    the interior launch (bench.py's roofline timing)."""
    import torch

    if out is None:
        out = torch.empty_like(x_local)
    reqs, hist = start_halo_exchange(x_local, grade, channels, group, recv_buf)

    def wait():
        for r in reqs:
            r.wait()

    split_moving_average_into(x_local, out, grade, channels, algo, history=hist, events=events, before_head=wait,
                              head_events=head_events)
    return out
