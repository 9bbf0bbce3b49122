"""Failure bounds of the N > 1 orchestration (CPU, gloo): a rank whose peer
never posts its halo send must end within its phase budget with status 124
and a line naming the rank and the phase; ranks that hang where no budget
applies are killed by bench.self_launch's deadline, which names every rank's
last phase.  (DESIGN.md "Multi-GPU": the first RCCL scaling run executes a
path that has not run on hardware; a hang there would leave no record.)"""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WORKER = os.path.join(ROOT, "tests", "halo_fault_worker.py")

LAUNCH_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
               "TORCHELASTIC_RUN_ID", "MAVG_BENCH_STATUS_DIR")


def _launch(mode, budget, world, timeout):
    """bench.self_launch(worker) in a child interpreter: (status, stderr, seconds)."""
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env["PYTHONUNBUFFERED"] = "1"
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.self_launch([{mode!r}, {str(budget)!r}], {world}, timeout={timeout!r}, "
            f"script={WORKER!r}))")
    t = time.monotonic()
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    return p.returncode, p.stderr, time.monotonic() - t


def test_missing_halo_send_exits_124_naming_rank_and_phase():
    budget = 4.0
    rc, err, secs = _launch("skip-send", budget, 2, timeout=240)
    assert rc == 124, err[-3000:]
    # the first watchdog to fire (a race between the two ranks) ends its rank; the launcher then
    # stops the other.  Its line names the rank and the phase and lists the other rank's phase
    # from the shared status directory, so the stuck halo wait is named either way
    lines = [l for l in err.splitlines() if "timed out in phase" in l]
    assert lines, err[-3000:]
    assert any(("rank 1/2 timed out in phase 'halo wait'" in l and "other ranks: rank 0: barrier" in l) or
               ("rank 0/2 timed out in phase 'barrier'" in l and "other ranks: rank 1: halo wait" in l)
               for l in lines), err[-3000:]
    # bounded: the budget plus interpreter and rendezvous start-up, far below the communicator's timeout
    assert secs < budget + 90, secs


def test_launch_deadline_kills_hung_ranks_and_names_their_phases():
    rc, err, secs = _launch("hang", 1.0, 2, timeout=20.0)
    assert rc == 124, err[-3000:]
    assert "launch deadline of 20 s expired with ranks [0, 1] still running" in err, err[-3000:]
    assert "rank 0: sleeping without a budget" in err and "rank 1: sleeping without a budget" in err, err[-3000:]
    assert secs < 20.0 + 30, secs


def test_completed_exchange_exits_zero():
    rc, err, _ = _launch("ok", 60.0, 3, timeout=240)
    assert rc == 0, err[-3000:]
    assert "timed out" not in err


def test_watchdog_fires_in_process_and_reports_detail(tmp_path):
    from digital_signal_processsing_amd.deadline import PhaseWatchdog, read_phases
    fired = []
    wd = PhaseWatchdog(3, 8, directory=str(tmp_path), poll_s=0.02, on_timeout=fired.append, stream=open(os.devnull, "w"),
                       publish_after_s=0.05)
    try:
        with wd.phase("fast phase", 5.0):
            time.sleep(0.1)
        assert not fired
        wd.set("barrier after the timed steps", 0.3, lambda: " -- halo wait of timed step 7")
        t = time.monotonic()
        while not fired and time.monotonic() - t < 10:
            time.sleep(0.02)
        assert fired, "the watchdog did not fire"
        assert fired[0].startswith("mavg-bench: rank 3/8 timed out in phase 'barrier after the timed steps'")
        assert "halo wait of timed step 7" in fired[0]
        assert read_phases(str(tmp_path))[3]["phase"] == "barrier after the timed steps"
    finally:
        wd.stop()
    assert not os.path.exists(tmp_path / "rank3.json")


def test_run_deadline_is_finite_and_grows_with_the_work():
    import bench
    a = bench.parse(["--gpus", "8"])
    d = bench.run_deadline(a)
    assert a.init_timeout + a.phase_timeout < d < 600, d  # inside the driver's limit by default
    b = bench.parse(["--gpus", "8", "--steps", "2000"])
    assert bench.run_deadline(b) > d
    c = bench.parse(["--gpus", "1"])  # the CPU baseline's reps count where it runs
    assert bench.run_deadline(c) > bench.run_deadline(bench.parse(["--gpus", "1", "--no-cpu-baseline"]))


@pytest.mark.parametrize("phases,want", [
    ({}, "no rank left a phase record"),
    ({0: {"phase": "barrier", "since": 90.0}, 2: {"phase": "halo wait", "since": 95.0}},
     "rank 0: barrier for 10.0 s; rank 2: halo wait for 5.0 s"),
])
def test_describe_phases(phases, want):
    from digital_signal_processsing_amd.deadline import describe_phases
    assert describe_phases(phases, now=100.0) == want
