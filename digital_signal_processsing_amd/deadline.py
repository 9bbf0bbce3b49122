"""Bounded phases for the multi-process (N > 1) orchestration.

The sharded step's only exchange is the halo send/recv (shard.py); the rest of
an N-rank run is rendezvous, barriers and small all-gathers.  Any of them can
wait forever on a peer that never arrives (a rank that died before its send, a
peer-access or IPC failure on the first RCCL run), and a hang produces no
record at all.  Each rank therefore names the phase it is in together with a
time budget; a daemon thread ends the process with status 124 and one line on
stderr naming the rank, the phase and how long it waited, once a phase outlives
its budget.  The reference has no multi-process path; its failure policy is
"print and exit" (`gpu_utils.h:10-18`, CUDA_CHECK), and its harness counts a
variant's non-zero return code as a failure (`basics/run_benchmarks.py:93-97`).

Ranks of one node also leave their current phase in a shared directory (a file
per rank, written by the watchdog thread only once a phase has lasted a
second, so the timed loop pays a tuple assignment per step and no I/O): the
timeout line lists every rank's phase, and a parent that launched the ranks
(bench.self_launch) can say where each one was when its own deadline expired.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import threading
import time
from contextlib import contextmanager
from typing import Callable, Optional

EXIT_TIMEOUT = 124  # timeout(1)'s status: the driver reads it as "timed out"


def status_dir(env=None) -> str:
    """The directory the ranks of one run share: MAVG_BENCH_STATUS_DIR, else
    one keyed by the rendezvous (MASTER_ADDR:MASTER_PORT and the elastic run
    id, which torch.distributed.run sets for every rank it starts)."""
    env = os.environ if env is None else env
    d = env.get("MAVG_BENCH_STATUS_DIR")
    if d:
        return d
    key = "_".join(str(env.get(v, "")) for v in ("MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID"))
    return os.path.join(tempfile.gettempdir(), "mavg_bench_" + "".join(c if c.isalnum() else "_" for c in key))


def read_phases(directory: str) -> dict:
    """{rank: {"phase", "since", "budget_s", "pid"}} of every rank that left
    a status file (missing or half-written files are skipped)."""
    out = {}
    try:
        names = os.listdir(directory)
    except OSError:
        return out
    for name in names:
        if not (name.startswith("rank") and name.endswith(".json")):
            continue
        try:
            with open(os.path.join(directory, name)) as f:
                rec = json.load(f)
            out[int(rec["rank"])] = rec
        except (OSError, ValueError, KeyError):
            continue
    return out


def describe_phases(phases: dict, now: Optional[float] = None) -> str:
    """'rank 0: barrier for 12.3 s; rank 1: halo wait (step 4) for 12.4 s'"""
    now = time.time() if now is None else now
    parts = []
    for r in sorted(phases):
        rec = phases[r]
        parts.append(f"rank {r}: {rec.get('phase', '?')} for {max(0.0, now - float(rec.get('since', now))):.1f} s")
    return "; ".join(parts) if parts else "no rank left a phase record"


class PhaseWatchdog:
    """Per-rank phase deadline.

        wd = PhaseWatchdog(rank, world)
        with wd.phase("init", 300):
            dist.init_process_group(...)
        wd.set("timed steps", 120)      # no context: lasts until the next set()/phase()
        wd.stop()

    `detail`: an optional callable returning extra text for the timeout line
    (e.g. which step's halo wait the launch stream has not passed); it runs on
    the watchdog thread and must not block.  `on_timeout` (tests) replaces
    the process exit."""

    def __init__(self, rank: int, world: int, directory: Optional[str] = None, poll_s: float = 0.2,
                 on_timeout: Optional[Callable[[str], None]] = None, stream=None, publish_after_s: float = 1.0):
        self.rank, self.world = rank, world
        self.dir = directory if directory is not None else status_dir()
        self.poll_s = poll_s
        self.publish_after_s = publish_after_s
        self.on_timeout = on_timeout
        self.stream = stream if stream is not None else sys.stderr
        self._cur = None          # (name, started monotonic, started wall, budget or None, detail)
        self._published = None    # the _cur tuple last written to the status file
        self._stop = threading.Event()
        self.fired = None         # the timeout line, once fired
        self._thread = threading.Thread(target=self._run, name=f"phase-watchdog-{rank}", daemon=True)
        self._thread.start()

    # -- the rank's side: cheap, no I/O -------------------------------------
    def set(self, name: str, budget_s: Optional[float], detail: Optional[Callable[[], str]] = None) -> None:
        self._cur = (name, time.monotonic(), time.time(), budget_s, detail)

    def clear(self) -> None:
        self._cur = None

    @contextmanager
    def phase(self, name: str, budget_s: Optional[float], detail: Optional[Callable[[], str]] = None):
        prev = self._cur
        self.set(name, budget_s, detail)
        try:
            yield self
        finally:
            self._cur = prev if prev is None else (prev[0], time.monotonic(), time.time(), prev[3], prev[4])

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2)
        try:
            os.unlink(self._path())
        except OSError:
            pass
        try:
            os.rmdir(self.dir)  # the last rank out removes the directory
        except OSError:
            pass

    # -- the watchdog thread -------------------------------------------------
    def _path(self) -> str:
        return os.path.join(self.dir, f"rank{self.rank}.json")

    def _publish(self, cur) -> None:
        name, _, wall, budget, _ = cur
        rec = {"rank": self.rank, "world": self.world, "phase": name, "since": wall, "budget_s": budget,
               "pid": os.getpid()}
        try:
            os.makedirs(self.dir, exist_ok=True)
            tmp = self._path() + f".{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                json.dump(rec, f)
            os.replace(tmp, self._path())
        except OSError:
            pass
        self._published = cur

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            cur = self._cur
            if cur is None:
                continue
            name, t_mono, _, budget, detail = cur
            waited = time.monotonic() - t_mono
            if waited >= self.publish_after_s and self._published is not cur:
                self._publish(cur)
            if budget is None or waited <= budget:
                continue
            extra = ""
            if detail is not None:
                try:
                    extra = detail() or ""
                except Exception as e:  # noqa: BLE001 - the line must still go out
                    extra = f" (detail unavailable: {e!r})"
            others = {r: v for r, v in read_phases(self.dir).items() if r != self.rank}
            line = (f"mavg-bench: rank {self.rank}/{self.world} timed out in phase '{name}' after {waited:.1f} s "
                    f"(budget {budget:g} s){extra}; other ranks: {describe_phases(others)}")
            self.fired = line
            try:
                print(line, file=self.stream, flush=True)
            except Exception:  # noqa: BLE001
                pass
            if self.on_timeout is not None:
                self.on_timeout(line)
                return
            # the main thread may be blocked inside a device synchronize or a
            # collective: leave without running Python's exit handlers
            os._exit(EXIT_TIMEOUT)
