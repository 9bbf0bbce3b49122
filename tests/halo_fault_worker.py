"""Fault-injection rank for tests/test_dist_bounds.py (a program, not a test
module): started N times by bench.self_launch, which sets the rank environment
and MAVG_BENCH_STATUS_DIR.  CPU only (gloo); argv: <mode> <phase budget s>.

  skip-send  rank 0 never posts its halo send and waits in a barrier; rank 1
             waits for the halo (shard.exchange_halo).  Both ranks' watchdogs
             must end them with status 124 and a line naming the phase.
  hang       every rank sleeps in a phase without a budget: only the parent's
             launch deadline can end the run.
  ok         the exchange completes; exit 0.
"""
import datetime
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    mode, budget = sys.argv[1], float(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    from digital_signal_processsing_amd.deadline import PhaseWatchdog
    from digital_signal_processsing_amd.shard import exchange_halo

    wd = PhaseWatchdog(rank, world, publish_after_s=0.2)
    with wd.phase("init (rendezvous)", 120):
        # the communicator's own timeout stays longer than the phase budget (as in bench.py)
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=budget + 60))
    x = torch.arange(4096, dtype=torch.float32) + 4096 * rank
    if mode == "skip-send":
        if rank == 0:  # never posts its send to rank 1
            with wd.phase("barrier", budget):
                dist.barrier()
        else:
            with wd.phase("halo wait", budget):
                exchange_halo(x, 64)
    elif mode == "hang":
        wd.set("sleeping without a budget", None)
        time.sleep(3600)
    elif mode == "ok":
        with wd.phase("halo wait", budget):
            h = exchange_halo(x, 64)
        if rank > 0:
            assert torch.equal(h, x[-63:] - 4096), "halo is the previous shard's tail"
        with wd.phase("barrier", budget):
            dist.barrier()
        dist.destroy_process_group()
    else:
        raise SystemExit(f"unknown mode {mode}")
    wd.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
