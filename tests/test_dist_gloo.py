"""Multi-GPU sharding logic on CPU (gloo): contiguous frame-aligned shards,
(k-1)-frame halo from rank r-1 by point-to-point send/recv, rank 0 zero
history.  Each rank checks that (halo ++ shard) filtered by the oracle equals
its slice of the whole-signal oracle output -- the property the GPU path
relies on (the GPU side of it is tests/test_gpu_parity.py::
test_history_equals_concatenation)."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, C, k, dtype, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import oracle
    from digital_signal_processsing_amd.shard import exchange_halo, shard_bounds
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        if dtype == "i16":
            x = oracle.synth_i16(frames * C, offset=5)
            full = oracle.mavg_i16(x, k, C)
        else:
            x = oracle.synth_f32(frames * C, offset=5, dist=1)
            full = oracle.mavg_f32(x, k, C)
        f0, f1 = shard_bounds(frames, world, rank)
        local = torch.from_numpy(x[f0 * C:f1 * C].copy())
        hist = exchange_halo(local, k, C)
        if rank == 0 or k == 1:
            assert hist is None
            ext = local.numpy()
        else:
            assert hist.numel() == (k - 1) * C
            assert np.array_equal(hist.numpy(), x[(f0 - (k - 1)) * C:f0 * C])
            ext = np.concatenate([hist.numpy(), local.numpy()])
        got = (oracle.mavg_i16 if dtype == "i16" else oracle.mavg_f32)(ext, k, C)[(ext.size - local.numel()):]
        want = full[f0 * C:f1 * C]
        if dtype == "i16":
            assert np.array_equal(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, f"{e!r}\n{traceback.format_exc()}"))


@pytest.mark.parametrize("world,frames,C,k,dtype", [
    (2, 100_000, 1, 1024, "f32"),
    (2, 50_001, 2, 41, "i16"),
    (3, 30_000, 2, 300, "i16"),
    (2, 10_000, 1, 1, "i16"),
    (4, 40_003, 1, 4096, "f32"),
])
def test_halo_exchange_gloo(world, frames, C, k, dtype):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, C, k, dtype, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in results.values()), results


def test_shard_bounds_cover_and_balance():
    from digital_signal_processsing_amd.shard import shard_bounds
    for total in (1, 7, 1000, 2 ** 33):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(total, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == total
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1
