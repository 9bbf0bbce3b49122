#!/usr/bin/env python3
"""North-star benchmark: Gsamples/s of the causal moving average on MI355X.

BASELINE.json metric: "Gsamples/s moving-average (N=2^30 fp32, k=1024);
achieved HBM GB/s vs peak".  A step is one pass of the hot path over one
batch: (N>1) the (k-1)-sample halo exchange with the neighbour rank over
RCCL, then one libmavg launch over this rank's 2^30-sample shard, inputs
already resident in HBM (generated on the device by the counter-based
synthetic generator).  Weak scaling: 2^30 samples per GPU.

    python bench.py                      # N=1, default K/W
    python bench.py --gpus N             # spawns N ranks itself (one process per GPU)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line (contract in the task statement), with
`roofline` (dominant kernel, algorithmic bytes / HIP-event kernel time vs
8 TB/s) and `cpu_baseline` (oracle restatement on a bounded sample, 1 core).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import signal
import socket
import statistics
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Gsamples/s moving-average (N=2^30 fp32, k=1024); achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
MALL_BYTES = 256 << 20  # MI355X Infinity Cache (memory-side, in front of HBM)

WORKLOADS = {
    # name: (samples per GPU, k, channels, dtype, default algo)
    "headline": (1 << 30, 1024, 1, "f32", "blelloch"),      # configs[4] per GPU / metric config
    "blelloch_2p26": (1 << 26, 64, 1, "f32", "blelloch"),   # configs[1]
    "direct_2p28": (1 << 28, 7, 1, "f32", "direct"),        # configs[2]
    "carry_2p30": (1 << 30, 4096, 1, "f32", "blelloch"),    # configs[3]
    # secondary lines (--all-workloads): the reference's own int16 PCM data path,
    # stereo as in its WAV harness, and the Hillis-Steele flavour of the scan
    "i16_2p30": (1 << 30, 1024, 1, "i16", "blelloch"),
    "i16_stereo_2p30": (1 << 30, 1024, 2, "i16", "blelloch"),
    "hillis_2p30": (1 << 30, 1024, 1, "f32", "hillis"),
    # a one-second window at 44.1 kHz: too long for an LDS-staged halo, so the
    # one-pass look-ahead scan (the inter-block carry path beyond config #4)
    "long_2p30": (1 << 30, 44100, 1, "f32", "blelloch"),
    # a window of two tiles past the LDS-staged halo: the look-ahead scan with
    # self-published records (no phase A)
    "mid_2p30": (1 << 30, 8192, 1, "f32", "blelloch"),
    # the same one-second window on the reference's int16 PCM path (mono, and
    # stereo as its WAV harness writes it)
    "i16_long": (1 << 30, 44100, 1, "i16", "blelloch"),
    "i16_stereo_long": (1 << 30, 44100, 2, "i16", "blelloch"),
    # the Hillis-Steele flavour past its LDS-staged halo (the look-ahead
    # record carry with the log-step in-tile scan), and very long windows
    "hillis_long": (1 << 30, 44100, 1, "f32", "hillis"),
    "long_1m": (1 << 30, 1_000_000, 1, "f32", "blelloch"),
    "long_2m": (1 << 30, 2_000_000, 1, "f32", "blelloch"),
    "long_4m": (1 << 30, 4_000_000, 1, "f32", "blelloch"),
    # fp32 multi-channel frames: stereo (the fp32 form of the reference's WAV
    # harness layout and of its only vectorized scan, longlong2 frames), 4 and 8
    "f32_stereo_2p30": (1 << 30, 1024, 2, "f32", "blelloch"),
    "f32_c4_2p30": (1 << 30, 1024, 4, "f32", "blelloch"),
    "f32_c8_2p30": (1 << 30, 1024, 8, "f32", "blelloch"),
    # multi-channel windows past the LDS-staged halo (the wide look-ahead scan) and at the edge of
    # the halo-only channel tile, and the reference's int16 PCM at the channel counts its WAV
    # reader accepts (wav_header.h:26-48)
    "f32_stereo_long": (1 << 30, 44100, 2, "f32", "blelloch"),
    "f32_c4_long": (1 << 30, 44100, 4, "f32", "blelloch"),
    "f32_c8_long": (1 << 30, 44100, 8, "f32", "blelloch"),
    "f32_c8_k2048": (1 << 30, 2048, 8, "f32", "blelloch"),
    # the in-place halo-only channel tile (fp32 C = 4) and the int16 dword-column look-ahead (C = 8,
    # self-published records) at a window of one tile
    "f32_c4_k2048": (1 << 30, 2048, 4, "f32", "blelloch"),
    "i16_c8_k2048": (1 << 30, 2048, 8, "i16", "blelloch"),
    "i16_c4_2p30": (1 << 30, 1024, 4, "i16", "blelloch"),
    "i16_c8_2p30": (1 << 30, 1024, 8, "i16", "blelloch"),
    "i16_c4_long": (1 << 30, 44100, 4, "i16", "blelloch"),
    "i16_c8_long": (1 << 30, 44100, 8, "i16", "blelloch"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="headline", choices=sorted(WORKLOADS))
    ap.add_argument("--algo", default=None, help="override the workload's algorithm")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-samples", type=int, default=1 << 30,
                    help="CPU-baseline sample (samples; default: the whole 2^30 headline signal, SURVEY.md 8d)")
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0),
                    help="threads of the multi-core CPU baseline (default: OMP_NUM_THREADS, else os.cpu_count())")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the measured path); gloo = rehearsal of the N>1 orchestration on a "
                         "box with fewer GPUs than ranks (halo staged through host memory, ranks share GPUs)")
    ap.add_argument("--check", action="store_true",
                    help="after timing, every rank checks sampled output slices (incl. its shard head) "
                         "against the CPU oracle")
    ap.add_argument("--all-workloads", action="store_true",
                    help="print one extra JSON line per secondary workload (rank 0, N=1 only)")
    # N > 1 failure bounds (DESIGN.md "Multi-GPU"): a peer that never arrives ends the run with
    # status 124 and a line naming the rank and the phase, instead of a hang past the driver's limit
    ap.add_argument("--init-timeout", type=float, default=300.0,
                    help="N>1: seconds a rank may wait in the rendezvous (init_process_group)")
    ap.add_argument("--phase-timeout", type=float, default=120.0,
                    help="N>1: seconds a rank may spend in any later phase (halo exchange, barrier, all-gather)")
    ap.add_argument("--launch-deadline", type=float, default=None,
                    help="--gpus N without a launcher: seconds before the parent kills its ranks "
                         "(default: derived from --steps/--warmup, the workloads and the timeouts)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    """Environment of one self-launched rank (what torch.distributed.run sets)."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return env


def run_deadline(args) -> float:
    """Seconds `bench.py --gpus N` (self-launched ranks) may run before the
    parent kills its ranks: the rendezvous and one stuck phase (each rank's
    own watchdog fires first), plus, per workload, its warm-up and timed steps
    twice over (the sharded steps, then shard_timing's single launches) at a
    generous 50 ms each, the copy calibration, the check and the all-gathers,
    plus the CPU baseline's repetitions where one runs (N = 1 only)."""
    n_work = len(WORKLOADS) if args.all_workloads else 1
    per_workload = 60.0 + (2 * args.steps + 2 * args.warmup) * 0.05
    cpu = 0.0 if (args.no_cpu_baseline or args.gpus > 1) else 30.0 * (args.cpu_reps + max(3, args.cpu_reps))
    return args.init_timeout + args.phase_timeout + n_work * per_workload + cpu


def self_launch(argv, world: int, timeout: float = None, script: str = None) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh child ranks (this
    process has not touched the GPU and never does), wait for all of them and
    return the exit status of the first rank that failed (0 if none did).  If
    one rank fails the others are stopped (they would wait forever in the next
    collective).  Past `timeout` seconds
    every rank still running is killed, stderr names each rank's last phase
    (the ranks' PhaseWatchdog records, deadline.py) and the status is 124.
    Rank 0's stdout is the one JSON line.  `script`: the program each rank
    runs (default this file; tests pass a fault-injection worker)."""
    from digital_signal_processsing_amd.deadline import EXIT_TIMEOUT, describe_phases, read_phases
    port = _free_port()
    me = os.path.abspath(script or __file__)
    sdir = tempfile.mkdtemp(prefix="mavg_bench_")
    procs = []
    for r in range(world):
        env = rank_env(os.environ, r, world, port)
        env["MAVG_BENCH_STATUS_DIR"] = sdir
        procs.append(subprocess.Popen([sys.executable, "-u", me] + list(argv), env=env))
    deadline = None if timeout is None else time.monotonic() + timeout
    first = 0  # the status of the first rank that failed: the cause, not the SIGTERMs that follow it
    live = list(procs)
    try:
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                rc = 128 - rc if rc < 0 else rc
                if rc != 0 and first == 0:
                    first = rc
                    for q in live:  # the exact child PIDs this function started
                        q.send_signal(signal.SIGTERM)
            if deadline is not None and live and time.monotonic() > deadline:
                ranks = [procs.index(q) for q in live]
                print(f"mavg-bench: launch deadline of {timeout:.0f} s expired with ranks {ranks} still running; "
                      f"{describe_phases(read_phases(sdir))}; killing them", file=sys.stderr, flush=True)
                for q in live:
                    q.kill()
                first = first or EXIT_TIMEOUT
                deadline = None
            time.sleep(0.05)
    finally:
        for q in live:
            if q.poll() is None:
                q.kill()
        shutil.rmtree(sdir, ignore_errors=True)
    return first


class _NoWatchdog:
    """N = 1: no peer to wait for, no watchdog thread beside the timed loop."""

    def set(self, *a, **kw):
        pass

    def phase(self, *a, **kw):
        return _nullcontext()

    def stop(self):
        pass


class _nullcontext:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def make_watchdog(world: int):
    if world <= 1:
        return _NoWatchdog()
    from digital_signal_processsing_amd.deadline import PhaseWatchdog
    return PhaseWatchdog(int(os.environ.get("RANK", "0")), world)


def init_dist(args, wd=None):
    import torch
    import torch.distributed as dist
    wd = wd or _NoWatchdog()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dist_backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # the communicator's own timeout (RCCL's watchdog, gloo's waits) backs up the
        # rank's PhaseWatchdog, whose budgets are shorter so that its line comes first
        tmo = datetime.timedelta(seconds=max(args.init_timeout, args.phase_timeout) + 60.0)
        with wd.phase("init (rendezvous)", args.init_timeout):
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
            else:
                dist.init_process_group("gloo", timeout=tmo)
            # the first collective: a communicator that cannot connect fails here, bounded
            dist.barrier()
    return rank, world, local


def barrier(world):
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()


def max_over_ranks(v: float, world: int) -> float:
    import torch
    import torch.distributed as dist
    if world == 1:
        return v
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_traffic(path, workload, algo):
    """HBM bytes per launch from the committed PMC summary (profiles/), or None."""
    try:
        with open(path) as f:
            data = json.load(f)
        ent = data.get(f"{workload}:{algo}")
        return None if ent is None else float(ent["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, n_total, k, C, seed):
    """Oracle restatement (profilable_moving_averager.cpp:14-37, fp64 running
    sum) over the benchmark's own synthetic signal -- by default all of it
    (2^30 samples at the headline, 3 reps) -- on one host core
    (the calling thread pinned to one allowed core), then the OpenMP
    restatement on `threads` cores pinned to the first allowed ones."""
    import oracle
    oracle.build()
    n = min(args.cpu_samples, n_total)
    x = oracle.synth_f32(n, seed=seed)
    allowed = os.sched_getaffinity(0)
    core = min(allowed)
    os.sched_setaffinity(0, {core})
    try:
        oracle.mavg_f32(x[: min(n, 1 << 20)], k, C)  # warm the code path
        times = []
        for _ in range(args.cpu_reps):
            t = time.perf_counter()
            oracle.mavg_f32(x, k, C)
            times.append(time.perf_counter() - t)
    finally:
        os.sched_setaffinity(0, allowed)
    med = statistics.median(times)
    threads = args.cpu_threads or len(allowed) or 1
    pinned = sorted(allowed)[:threads]
    # OpenMP creates its pool at the first parallel region (here), inheriting this mask
    os.sched_setaffinity(0, set(pinned))
    try:
        oracle.mavg_f32_mt(x[: min(n, 1 << 20)], k, C, threads)
        mt = []
        for _ in range(max(3, args.cpu_reps)):
            t = time.perf_counter()
            oracle.mavg_f32_mt(x, k, C, threads)
            mt.append(time.perf_counter() - t)
    finally:
        os.sched_setaffinity(0, allowed)
    mt_med = statistics.median(mt)
    what = "the whole benchmark signal" if n == n_total else f"the first {n} of the benchmark's {n_total}"
    multicore = {
        "value": round(n / mt_med / 1e9, 4),
        "unit": "Gsamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"same sample, OpenMP chunks with a k-frame halo each, {threads} threads pinned to cores "
                  f"{_core_ranges(pinned)} (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}), "
                  f"median of {len(mt)} reps, {mt_med * 1e3:.1f} ms/rep",
    }
    single = {
        "value": round(n / med / 1e9, 4),
        "unit": "Gsamples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n} fp32 samples ({what} synthetic samples), k={k}, C={C}, "
                  f"median of {args.cpu_reps} reps, {med * 1e3:.1f} ms/rep, single thread pinned to core {core}",
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "allowed_cpus": len(allowed),
    }
    return single, multicore


def _core_ranges(cores) -> str:
    """[0,1,2,5] -> '0-2,5'"""
    out, start, prev = [], None, None
    for c in sorted(cores):
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append(f"{start}-{prev}" if prev != start else str(start))
            start = prev = c
    if start is not None:
        out.append(f"{start}-{prev}" if prev != start else str(start))
    return ",".join(out)


def check_output(y, n, k, C, dt, seed, rank, samples=64, span=4096):
    """Compare slices of this rank's output shard with the oracle run on the
    same global synthetic stream (test leg: the oracle is only the checker)."""
    import numpy as np
    import oracle
    oracle.build()
    frames = n // C
    f_base = rank * frames                       # global frame of local frame 0
    rng = np.random.default_rng(rank)
    starts = [0, max(0, frames - span)] + list(rng.integers(0, max(1, frames - span), samples))
    ycpu = y.cpu().numpy()
    bad = 0
    for s in starts:
        s = int(s)
        e = min(frames, s + span)
        g0 = max(0, f_base + s - (k - 1))            # first global frame the window needs
        cnt = (f_base + e - g0) * C
        if dt == "f32":
            xs = oracle.synth_f32(cnt, seed=seed, offset=g0 * C)
            ref = oracle.mavg_f32(xs, k, C)[(f_base + s - g0) * C:]
            got = ycpu[s * C:e * C].astype(np.float64)
            bad += int(np.sum(np.abs(got - ref) > 1e-5 * np.maximum(np.abs(ref), 1e-30)))
        else:
            xs = oracle.synth_i16(cnt, seed=seed, offset=g0 * C)
            ref = oracle.mavg_i16(xs, k, C)[(f_base + s - g0) * C:]
            bad += int(np.sum(ycpu[s * C:e * C] != ref))
    return {"slices": len(starts), "span_frames": span, "mismatches": bad}


def shard_timing(args, x, y, k, C, algo, ev, hev, value, n, rank, world):
    """N > 1: what the sharded step costs each rank beyond one plain launch.
    Per rank, from the timed steps' events on the launch stream: the halo wait
    (interior end -> head start: the stream waits for the RCCL receive) and the
    head launch.  Then, in the same run, each rank times K whole-shard launches
    with no halo (the N=1 step on its own shard, wall clock between barriers),
    so the weak-scaling efficiency comes out of this one run:
        weak_scaling_efficiency = value / (N * mean per-rank single-launch rate)."""
    import torch
    import torch.distributed as dist
    import digital_signal_processsing_amd as dsp
    halo_ms = statistics.mean(b.elapsed_time(h[0]) for (_, b), h in zip(ev, hev))
    head_ms = statistics.mean(h[0].elapsed_time(h[1]) for h in hev)
    for _ in range(max(1, args.warmup)):
        dsp.moving_average_into(x, y, k, C, algo)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dsp.moving_average_into(x, y, k, C, algo)
    torch.cuda.synchronize()
    single_s = time.perf_counter() - t0
    rate = n * args.steps / single_s / 1e9
    mine = {"rank": rank, "halo_wait_ms": round(halo_ms, 4), "head_ms": round(head_ms, 4),
            "single_launch_gsamples_s": round(rate, 3)}
    every = [None] * world
    dist.all_gather_object(every, mine)
    mean_rate = statistics.mean(r["single_launch_gsamples_s"] for r in every)
    return {
        "weak_scaling_efficiency": round(value / (world * mean_rate), 4),
        "single_launch_gsamples_s_mean": round(mean_rate, 3),
        "per_rank": every,
        "method": "per rank: K whole-shard launches without halo in this run (wall clock between a barrier and "
                  "a synchronize); halo_wait = interior end -> head start on the launch stream; efficiency = "
                  "value / (N x mean single-launch rate)",
    }


def device_record(rank: int) -> dict:
    """This rank's device as the communicator sees it (N > 1 `rccl` block)."""
    import torch
    dev = torch.cuda.current_device()
    pr = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": dev,
            "pci_bus_id": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
            "uuid": str(pr.uuid), "name": pr.name, "host": socket.gethostname(),
            "visible_devices": torch.cuda.device_count()}


def rccl_block(every: list, backend: str, version, halo_bytes: int, world: int) -> dict:
    """The N > 1 line's `rccl` block: what the communicator saw -- its world
    size and backend, the RCCL version torch links, each rank's device (index,
    PCI bus id, UUID, host) and the halo bytes each exchange moves.  Under
    backend "nccl" (= RCCL) the N ranks must hold N distinct devices, or the
    run fails loudly (a scaling record that shares GPUs is not one); the gloo
    rehearsal may share a device and says so."""
    keys = {(r["host"], r["uuid"]) for r in every}
    distinct = len(keys) == len(every) == world
    if backend == "nccl" and not distinct:
        raise SystemExit(f"RCCL world of {world} ranks on {len(keys)} distinct devices: {every}")
    return {
        "world_size": world,
        "backend": backend,
        "rccl_version": version,
        "devices": every,
        "distinct_devices": distinct,
        "halo_bytes": halo_bytes,
        "exchange": "batch_isend_irecv: (k-1)*C samples from rank r to rank r+1, once per step",
    }


def comm_report(rank: int, world: int, halo_bytes: int) -> dict:
    import torch
    import torch.distributed as dist
    every = [None] * world
    dist.all_gather_object(every, device_record(rank))
    try:
        version = ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception:  # noqa: BLE001 - a build without RCCL: report it as absent
        version = None
    return rccl_block(every, dist.get_backend(), version, halo_bytes, dist.get_world_size())


def copy_ceiling(xs, ys, rot, steps, world, min_s=0.25):
    """Mean per-launch time (ms) of the library's calibration copy over the
    workload's buffers, at least `steps` launches and `min_s` seconds of them
    (max over ranks), and the number of launches timed."""
    import torch
    import digital_signal_processsing_amd as dsp
    for w in range(3):
        dsp.stream_copy(xs[w % rot], ys[w % rot])
    torch.cuda.synchronize()
    times, t0 = [], time.perf_counter()
    while len(times) < steps or time.perf_counter() - t0 < min_s:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for i, (a, b) in enumerate(ev):
            a.record()
            dsp.stream_copy(xs[i % rot], ys[i % rot])
            b.record()
        torch.cuda.synchronize()
        times += [a.elapsed_time(b) for a, b in ev]
    return max_over_ranks(statistics.mean(times), world), len(times), time.perf_counter() - t0


def halo_progress(hev):
    """Watchdog detail for a wait after the timed steps (RCCL: the halo receive
    is a stream wait, so a missing send shows up in the synchronize): the first
    timed step whose head launch the launch stream has not reached."""
    if not hev:
        return ""
    for i, (h0, _) in enumerate(hev):
        if not h0.query():
            return f" -- the launch stream has not passed the halo wait of timed step {i} (its head launch not started)"
    return " -- every timed step's halo wait has been passed on the launch stream"


def run_workload(args, name, rank, world, with_cpu, wd=None):
    import torch
    import digital_signal_processsing_amd as dsp
    from digital_signal_processsing_amd.shard import sharded_moving_average

    n, k, C, dt, algo = WORKLOADS[name]
    if args.algo and name == args.workload:
        algo = args.algo
    seed = 0x5EED
    dtype = torch.float32 if dt == "f32" else torch.int16
    elem = 4 if dt == "f32" else 2
    # A footprint the 256 MB MALL could partly hold across steps (config #2:
    # 512 MiB) is timed cold: the step cycles through R copies of (x, y) so
    # that >= 2 GiB of other traffic separates two uses of the same buffers
    # (SURVEY.md 8d asks for the MALL to be flushed between iterations).
    rot = max(1, -(-8 * MALL_BYTES // (2 * elem * n))) if world == 1 else 1
    # weak scaling: this rank holds global samples [rank*n, (rank+1)*n)
    xs = [dsp.fill_synthetic(n, dtype, seed=seed, offset=rank * n, device="cuda") for _ in range(rot)]
    ys = [torch.empty_like(xs[0]) for _ in range(rot)]
    x, y = xs[0], ys[0]
    hist_buf = torch.empty(max((k - 1) * C, 1), dtype=dtype, device="cuda")
    resolved = dsp.resolve_algo(n, k, C, dsp.F32 if dt == "f32" else dsp.I16, algo)
    launch_plan = dsp.plan(n, k, C, dsp.F32 if dt == "f32" else dsp.I16, algo)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    hev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] if world > 1 else None

    # Same-box streaming ceiling first: the library's flat non-temporal copy over
    # the same buffers, timed over at least --steps launches and at least 0.25 s
    # of them (a calibration measured over a duration, not a burst).  Measured
    # first, it also takes the device out of its idle power state before the
    # workload's own W warm-up steps: at W = 5 a 0.7-0.8 ms int16 launch was
    # otherwise still timed on the clock ramp (i16_c4_2p30 0.670 of peak after
    # 5 warm-up steps, 0.777 after 200; the headline 0.786 / 0.807;
    # profiles/r05_validation/warmup_ramp/).  The timed region is unchanged.
    wd = wd or _NoWatchdog()
    pt = args.phase_timeout
    with wd.phase(f"{name}: copy calibration (all-reduce)", pt):
        copy_ms, copy_launches, copy_s = copy_ceiling(xs, ys, rot, args.steps, world)

    def step(i=None, j=0):
        if world > 1:
            # halo send/recv posted first, interior launch overlaps it, head launch after it
            sharded_moving_average(x, k, C, algo, out=y, recv_buf=hist_buf[: (k - 1) * C],
                                   events=ev[i] if i is not None else None,
                                   head_events=hev[i] if i is not None else None)
            return
        if i is not None:
            j = i % rot
            ev[i][0].record()
        dsp.moving_average_into(xs[j], ys[j], k, C, algo)
        if i is not None:
            ev[i][1].record()

    with wd.phase(f"{name}: warm-up steps (halo exchange)", pt):
        for w in range(args.warmup):
            step(j=w % rot)
    with wd.phase(f"{name}: barrier before the timed steps", pt):
        barrier(world)
    wd.set(f"{name}: timed steps (halo exchange)", pt)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    wd.set(f"{name}: barrier after the timed steps (halo wait on the stream)", pt, lambda: halo_progress(hev))
    barrier(world)
    dt_s = time.perf_counter() - t0
    wd.set(f"{name}: all-reduce of the timings", pt)
    dt_s = max_over_ranks(dt_s, world)
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    kern_avg_ms = statistics.mean(kern_ms)
    kern_avg_ms = max_over_ranks(kern_avg_ms, world)
    alg_bytes = 2 * elem * n  # read x once, write y once
    if world > 1:  # events bracket the interior launch only (frames >= head_frames)
        from digital_signal_processsing_amd.shard import head_frames
        alg_bytes = 2 * elem * (n - head_frames(k, n // C) * C)
    achieved = alg_bytes / (kern_avg_ms * 1e-3) / 1e9
    total_samples = n * world * args.steps
    value = total_samples / dt_s / 1e9
    traffic = load_traffic(args.traffic_json, name, resolved)
    line = {
        "metric": METRIC if name == "headline" else f"Gsamples/s moving-average ({name})",
        "value": round(value, 3),
        "unit": "Gsamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_s * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dt,
        "accumulate": "f64" if dt == "f32" else ("i32" if k <= 65535 else "i64"),
        "data": "synthetic (device counter-based splitmix64, int16-valued samples)",
        "config": {
            "workload": f"{name}: {n} {dt} samples per GPU, k={k}, C={C}, algo={resolved}",
            "n_samples_per_gpu": n,
            "n_samples_total": n * world,
            "k": k,
            "channels": C,
            "algo": resolved,
            "parallelism": f"shard{world} (contiguous shards, (k-1)-sample RCCL halo)" if world > 1 else "single GPU",
        },
        "hbm_gbs_algorithmic": round(alg_bytes * world * args.steps / dt_s / 1e9, 1),
        "timing": "wall clock over the timed steps (barrier + synchronize on both sides)"
                  + (f"; steps rotate over {rot} input/output buffer pairs so no step finds its data in the "
                     f"256 MB MALL" if rot > 1 else ""),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": launch_plan,
            "kernel_avg_ms": round(kern_avg_ms, 4),
            "kernel_min_ms": round(min(kern_ms), 4),
            "kernel_median_ms": round(statistics.median(kern_ms), 4),
            "algorithmic_bytes_per_launch": alg_bytes,
            "statistic": "mean of the per-launch HIP-event durations of the timed steps",
            "scope": ("one launch over the whole signal" if world == 1 else
                      "the interior launch of this rank's shard (frames >= head_frames); the halo wait and "
                      "the head launch are outside it and only in value / ms_per_step"),
        },
    }
    if args.check:
        wd.set(f"{name}: check against the oracle", pt)
        res = check_output(y, n, k, C, dt, seed, rank)
        wd.set(f"{name}: all-gather of the checks", pt)
        if world > 1:
            import torch.distributed as dist
            allres = [None] * world
            dist.all_gather_object(allres, res)
            res = {"ranks": world, "slices": sum(r["slices"] for r in allres),
                   "mismatches": sum(r["mismatches"] for r in allres)}
        line["check"] = res
    if world > 1:
        wd.set(f"{name}: all-gather of the device records", pt)
        line["rccl"] = comm_report(rank, world, (k - 1) * C * elem)
    if world > 1:  # after --check: the single launches overwrite the output with a no-halo result
        wd.set(f"{name}: single-launch timing (barrier, all-gather)", pt)
        line["scaling_detail"] = shard_timing(args, x, y, k, C, algo, ev, hev, value, n, rank, world)
    wd.set(f"{name}: report", None)
    copy_gbs = 2 * elem * n / (copy_ms * 1e-3) / 1e9
    line["copy_ceiling"] = {
        "kernel": "mavg_stream_copy: flat grid, one 16-B non-temporal load + store per thread",
        "achieved": round(copy_gbs, 1),
        "unit": "GB/s",
        "frac": round(copy_gbs / HBM_PEAK_GBS, 4),
        "kernel_avg_ms": round(copy_ms, 4),
        "launches": copy_launches,
        "seconds": round(copy_s, 3),
        "when": "measured before the workload's warm-up steps, over at least --steps launches and 0.25 s",
    }
    # what ran on the device before the timed steps (bench lines from round 5 on: the copy
    # calibration first, which also takes the device out of its idle clocks; earlier rounds'
    # lines had only the W warm-up steps -- DESIGN.md "The start of a process")
    line["warmup_detail"] = {"copy_calibration_launches": copy_launches, "copy_calibration_s": round(copy_s, 3),
                             "workload_warmup_steps": args.warmup}
    line["roofline"]["frac_of_copy"] = round(achieved / copy_gbs, 4)
    if with_cpu and rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"], line["cpu_baseline_multicore"] = cpu_baseline(args, n, k, C, seed)
    del x, y, xs, ys
    torch.cuda.empty_cache()
    return line


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        deadline = args.launch_deadline if args.launch_deadline is not None else run_deadline(args)
        sys.exit(self_launch(sys.argv[1:], args.gpus, timeout=deadline))
    wd = make_watchdog(int(os.environ.get("WORLD_SIZE", "1")))
    rank, world, _ = init_dist(args, wd)
    line = run_workload(args, args.workload, rank, world, with_cpu=True, wd=wd)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if args.all_workloads and world == 1:
        for name in sorted(WORKLOADS):
            if name != args.workload:
                extra = run_workload(args, name, rank, world, with_cpu=False)
                print(json.dumps(extra), file=sys.stderr, flush=True)
    if world > 1:
        import torch.distributed as dist
        with wd.phase("destroy_process_group", args.phase_timeout):
            dist.destroy_process_group()
    wd.stop()


if __name__ == "__main__":
    main()
