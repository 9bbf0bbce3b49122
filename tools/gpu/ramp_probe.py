#!/usr/bin/env python3
"""Per-launch time series of a bench workload after the same-box copy, to see
whether (and for how long) its launches run slower at the start of a process.

    python tools/gpu/ramp_probe.py <workload> [launches=400] [bucket=20] [copy_s=0.25]

Prints, per bucket of launches, the mean fraction of 8 TB/s (algorithmic bytes
over the per-launch HIP-event duration) and, when torch can read it, the
graphics clock sampled after the bucket.
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import bench  # noqa: E402
import digital_signal_processsing_amd as dsp  # noqa: E402


def clock():
    try:
        return torch.cuda.clock_rate()
    except Exception:  # noqa: BLE001 - no SMI library on this box: omit the column
        return None


def main(name, launches=400, bucket=20, copy_s=0.25):
    n, k, C, dt, algo = bench.WORKLOADS[name]
    dtype = torch.float32 if dt == "f32" else torch.int16
    elem = 4 if dt == "f32" else 2
    x = dsp.fill_synthetic(n, dtype, seed=0x5EED, device="cuda")
    y = torch.empty_like(x)
    print(f"{name}: {dsp.plan(n, k, C, dsp.F32 if dt == 'f32' else dsp.I16, algo)}", flush=True)
    print(f"clock before copy: {clock()}", flush=True)
    if copy_s > 0:
        ms, cnt = bench.copy_ceiling([x], [y], 1, 20, 1, min_s=copy_s)
        print(f"copy: {cnt} launches, {2 * elem * n / ms / 1e6 / 8000:.4f} of peak, clock {clock()}", flush=True)
    for b in range(0, launches, bucket):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(bucket)]
        for a, e in ev:
            a.record()
            dsp.moving_average_into(x, y, k, C, algo)
            e.record()
        torch.cuda.synchronize()
        t = [a.elapsed_time(e) for a, e in ev]
        fr = [2 * elem * n / (v * 1e-3) / 1e9 / 8000 for v in t]
        print(f"launches {b:4d}-{b + bucket - 1:4d}: mean {statistics.mean(fr):.4f} first {fr[0]:.4f} "
              f"min {min(fr):.4f} max {max(fr):.4f} clock {clock()}", flush=True)
    # an idle gap, then again: does the device fall back?
    time.sleep(1.0)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(bucket)]
    for a, e in ev:
        a.record()
        dsp.moving_average_into(x, y, k, C, algo)
        e.record()
    torch.cuda.synchronize()
    fr = [2 * elem * n / (a.elapsed_time(e) * 1e-3) / 1e9 / 8000 for a, e in ev]
    print(f"after 1 s idle: mean {statistics.mean(fr):.4f} first {fr[0]:.4f} last {fr[-1]:.4f}", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(int(v) for v in a[1:3]), *(float(v) for v in a[3:4]))
