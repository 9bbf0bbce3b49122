"""The RCCL (torch.distributed "nccl") path of the multi-GPU layer, run on the one GPU a test box
has: a one-rank NCCL communicator created the way bench.py creates it (init_process_group with
device_id and a timeout), its collectives (barrier, all_reduce MAX on a device tensor -- bench's
max-over-ranks timing -- and all_gather_object -- bench's device records), and the halo exchange
of digital_signal_processsing_amd/shard.py on device tensors: the shard's batch_isend_irecv with
the communicator's only rank as both peers (RCCL self send/receive), the receive's wait ordering
the head launch on the stream, and every output of the second shard against the oracle over the
whole signal (reference semantics: basics/profilable_moving_averager.cpp:14-37; the zeroed halo
zone it replaces: gpu_utils.h:112-123).  Ranks on distinct GPUs (the driver's 8-GPU run) use the
same calls with rank - 1 / rank + 1 as peers; they cannot share one device under RCCL.

The child runs in its own process under a time limit, so a communicator that never completes
ends the test instead of the session."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import datetime, os, sys, tempfile
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.getcwd())
import oracle
import digital_signal_processsing_amd as dsp
from digital_signal_processsing_amd.shard import start_halo_exchange, split_moving_average_into
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
store = dist.FileStore(os.path.join(tempfile.mkdtemp(), "rccl_store"), 1)
dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev,
                        timeout=datetime.timedelta(seconds=60))
assert dist.get_backend() == "nccl"
dist.barrier()
t = torch.tensor([2.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert t.item() == 2.5
rec = [None]
dist.all_gather_object(rec, {"pci": torch.cuda.get_device_properties(0).pci_bus_id})
assert rec[0]["pci"] == torch.cuda.get_device_properties(0).pci_bus_id
for dt, C, k in (("f32", 1, 1024), ("i16", 2, 44100), ("f32", 8, 3000)):
    na, nb = 70_001, 90_017  # frames of the previous shard and of this one
    if dt == "f32":
        x = oracle.synth_f32((na + nb) * C, seed=k + C, dist=0)  # int16-valued: fp32 outputs exact
        ref = oracle.mavg_f32(x, k, C)
    else:
        x = oracle.synth_i16((na + nb) * C, seed=k + C)
        ref = oracle.mavg_i16(x, k, C)
    xa = torch.from_numpy(x[: na * C]).to(dev)
    xb = torch.from_numpy(x[na * C:]).to(dev)
    # the previous shard's tail reaches this shard's history buffer through RCCL (self peers)
    reqs, hist = start_halo_exchange(xa, k, C, peers=(0, 0))
    assert len(reqs) > 0 and hist is not None and hist.is_cuda and hist.numel() == (k - 1) * C
    y = torch.empty_like(xb)
    def wait():
        for r in reqs:
            r.wait()
    split_moving_average_into(xb, y, k, C, "blelloch", history=hist, before_head=wait)
    torch.cuda.synchronize()
    assert torch.equal(hist.cpu(), xa[xa.numel() - (k - 1) * C:].cpu()), (dt, C, k, "halo")
    assert np.array_equal(y.cpu().numpy(), ref[na * C:]), (dt, C, k)
dist.destroy_process_group()
print("rccl one-device ok", torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else "")
'''


@pytest.mark.gpu
@pytest.mark.timeout(200)
def test_rccl_communicator_and_halo_exchange_on_one_device(gpu):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-u", "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=170)
    assert r.returncode == 0 and "rccl one-device ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_halo_exchange_without_peers_is_empty():
    """CPU: a one-rank gloo group with the default peers exchanges nothing (rank 0 uses zeros)."""
    import datetime
    import tempfile
    import torch
    import torch.distributed as dist
    from digital_signal_processsing_amd.shard import start_halo_exchange
    store = dist.FileStore(os.path.join(tempfile.mkdtemp(), "gloo_store"), 1)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1, timeout=datetime.timedelta(seconds=30))
    try:
        reqs, hist = start_halo_exchange(torch.arange(10, dtype=torch.float32), 4)
        assert reqs == [] and hist is None
        reqs, hist = start_halo_exchange(torch.arange(10, dtype=torch.float32), 4, peers=(None, None))
        assert reqs == [] and hist is None
    finally:
        dist.destroy_process_group()
