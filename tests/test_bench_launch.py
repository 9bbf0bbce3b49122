"""bench.py --gpus N launches its own ranks (the driver's command has no
torch.distributed.run in front of it): rank environment, failure
propagation, and -- on the GPU -- a 2-rank run through the sharded path
(halo exchange + interior/head launches of libmavg) with --check."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAUNCH_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
               "TORCHELASTIC_RUN_ID")


def _clean_env():
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env["PYTHONUNBUFFERED"] = "1"
    return env


def test_rank_env_is_what_torchrun_sets():
    import bench
    env = bench.rank_env({"PATH": "/bin"}, 3, 8, 29555)
    assert env["RANK"] == env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/bin"


def test_core_ranges():
    import bench
    assert bench._core_ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"
    assert bench._core_ranges([4]) == "4"
    assert bench._core_ranges([]) == ""


def test_self_launch_propagates_rank_failure_without_hanging():
    """Without a GPU every rank fails at set_device: the parent must return a
    non-zero status promptly instead of waiting on the surviving ranks."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], env=_clean_env(), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_gloo_check(gpu):
    """The driver's form `bench.py --gpus 2` with no launcher environment:
    two self-launched ranks (sharing GPU 0 over gloo) run the weak-scaling
    step and check their shards, including each shard head, against the
    oracle; rank 0 prints exactly one JSON line."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "3", "--warmup", "1", "--check"], env=_clean_env(), capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["n_samples_total"] == 2 * d["config"]["n_samples_per_gpu"]
    assert d["check"]["ranks"] == 2 and d["check"]["mismatches"] == 0 and d["check"]["slices"] > 0
    assert "interior launch" in d["roofline"]["scope"]
    assert d["value"] > 0 and d["scaling"] == "weak"
    sd = d["scaling_detail"]
    assert 0 < sd["weak_scaling_efficiency"] <= 1.2, sd
    assert [r["rank"] for r in sd["per_rank"]] == [0, 1]
    for r in sd["per_rank"]:
        assert r["halo_wait_ms"] >= 0 and r["head_ms"] > 0 and r["single_launch_gsamples_s"] > 0, r
    rc = d["rccl"]  # what the communicator saw (gloo rehearsal: both ranks may share GPU 0)
    assert rc["world_size"] == 2 and rc["backend"] == "gloo" and rc["halo_bytes"] == 1023 * 4, rc
    assert [r["rank"] for r in rc["devices"]] == [0, 1] and all(r["pci_bus_id"] for r in rc["devices"]), rc
    assert rc["distinct_devices"] == (len({r["uuid"] for r in rc["devices"]}) == 2), rc


def _rec(rank, uuid, host="h"):
    return {"rank": rank, "device": rank, "pci_bus_id": f"0000:{rank:02x}:00", "uuid": uuid, "host": host}


def test_rccl_block_requires_distinct_devices_under_nccl():
    """The N > 1 JSON line's `rccl` block proves by itself that N ranks held N
    devices: under nccl (RCCL) a shared device fails the run; gloo may share."""
    import bench
    ok = bench.rccl_block([_rec(0, "a"), _rec(1, "b")], "nccl", "2.27.7", 4092, 2)
    assert ok["distinct_devices"] and ok["world_size"] == 2 and ok["halo_bytes"] == 4092
    assert ok["rccl_version"] == "2.27.7" and [r["rank"] for r in ok["devices"]] == [0, 1]
    with pytest.raises(SystemExit, match="distinct devices"):
        bench.rccl_block([_rec(0, "a"), _rec(1, "a")], "nccl", "2.27.7", 4092, 2)
    assert not bench.rccl_block([_rec(0, "a"), _rec(1, "a")], "gloo", None, 4092, 2)["distinct_devices"]
    # the same UUID string on two hosts is two devices
    assert bench.rccl_block([_rec(0, "a", "h0"), _rec(1, "a", "h1")], "nccl", None, 8, 2)["distinct_devices"]
