#!/usr/bin/env python3
"""Phase timeline of the row-band scan from a MAVG_BAND_TRACE build
(`make -C digital_signal_processsing_amd/csrc trace` -> abl/libmavg_trace.so).

Per workgroup, wave 0 stamps (100-MHz wall clock): 0 start, 1 rows staged,
2 its row sums published, 3 first window sum read, 4 end; 5 = XCC id.  Prints
the phase distributions, how long a band waits for its slowest member, and
how many workgroups were resident on average.

    python tools/tune/band_trace.py abl/libmavg_trace.so [--k 44100] [--c 1] [--dtype f32]
"""
import argparse
import ctypes
import os
import re
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import digital_signal_processsing_amd as dsp  # noqa: E402


def pct(d):
    return f"median {np.median(d):7.2f}  p10 {np.percentile(d, 10):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():8.2f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--k", type=int, default=44100)
    ap.add_argument("--c", type=int, default=1)
    ap.add_argument("--dtype", default="f32", choices=["f32", "i16"])
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--launches", type=int, default=4)
    a = ap.parse_args()
    n = 1 << a.log2n
    tdt = torch.float32 if a.dtype == "f32" else torch.int16
    code = dsp.F32 if a.dtype == "f32" else dsp.I16
    lib = ctypes.CDLL(a.lib)
    lib.mavg_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_int] * 5 + [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.mavg_plan.argtypes = [ctypes.c_size_t] + [ctypes.c_int] * 5 + [ctypes.c_char_p, ctypes.c_size_t]
    buf = ctypes.create_string_buffer(512)
    assert lib.mavg_plan(n, a.c, a.k, code, 0, 0, buf, 512) == 0
    plan = buf.value.decode()
    assert plan.startswith("band_scan<"), plan
    grid = int(re.search(r"grid=(\d+)", plan).group(1))
    S = int(re.search(r"columns=(\d+)", plan).group(1))
    Sp = (S + 7) // 8 * 8
    ws_bytes = int(re.search(r"ws=(\d+)", plan).group(1))
    x = dsp.fill_synthetic(n, tdt, dist=2 if a.dtype == "f32" else 0, device="cuda")
    y = torch.empty_like(x)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    for e0, e1 in ev:
        e0.record()
        assert lib.mavg_run(x.data_ptr(), y.data_ptr(), n, a.c, a.k, code, 0, 0, None, ws.data_ptr(), ws_bytes,
                            stream) == 0
        e1.record()
    torch.cuda.synchronize()
    ms = [e0.elapsed_time(e1) for e0, e1 in ev]
    tr = ws[ws_bytes - grid * 64:].cpu().numpy().view(np.uint64).reshape(grid, 8).astype(np.int64)
    cols = np.arange(grid) % Sp
    live = cols < S
    t = tr[live]
    t0 = t[:, 0].min()
    st = (t[:, :5] - t0) / 100.0  # us
    print(plan)
    print("launch ms:", " ".join(f"{m:.3f}" for m in ms), f" traced span {st[:, 4].max():.1f} us, WGs {live.sum()}")
    for nm, (i, j) in zip(["stage rows (start->A)", "row sums published", "first window sum (wait+read)",
                           "scan + stores (rest)", "lifetime"], [(0, 1), (1, 2), (2, 3), (3, 4), (0, 4)]):
        print(f"  {nm:30s} {pct(st[:, j] - st[:, i])} us")
    # per band: the spread of its members' starts and publishes, and how long
    # a member waits after its own publish for the band's last publish
    bands = (np.arange(grid) // Sp)[live]
    nb = bands.max() + 1
    first_start = np.full(nb, np.inf)
    last_pub = np.zeros(nb)
    np.minimum.at(first_start, bands, st[:, 0])
    np.maximum.at(last_pub, bands, st[:, 2])
    last_start = np.zeros(nb)
    np.maximum.at(last_start, bands, st[:, 0])
    print(f"  band start spread (last - first member start) {pct(last_start - first_start)} us")
    print(f"  own publish -> band's last publish            {pct(last_pub[bands] - st[:, 2])} us")
    print(f"  band's last publish -> first window sum read  {pct(st[:, 3] - last_pub[bands])} us")
    # residency: mean WGs alive over the middle 80% of the launch
    span = st[:, 4].max()
    ts = np.linspace(0.1 * span, 0.9 * span, 200)
    alive = [np.sum((st[:, 0] <= x) & (st[:, 4] > x)) for x in ts]
    print(f"  resident workgroups: mean {np.mean(alive):.0f} ({np.mean(alive) / 256:.2f} per CU)")
    xcc = tr[live, 5] & 0xF
    print("  WGs per XCC id:", np.bincount(xcc, minlength=8).tolist())


if __name__ == "__main__":
    main()
