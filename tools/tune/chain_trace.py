#!/usr/bin/env python3
"""Phase timeline of the chained look-back scan from a MAVG_CHAIN_TRACE build
(`make -C digital_signal_processsing_amd/csrc trace` -> abl/libmavg_trace.so).

Per tile the kernel stamps (100-MHz wall clock, s_memrealtime):
  0 start (tile waves)   1 barrier A passed (tile and shifted stage loaded)
  2 chain wave past B    3 L(t) published    4 barrier C passed   5 outputs issued
  6 look-back outcome: ls (distance to the inclusive used) | polls << 32
This prints, over the last of several launches, the distribution of each
phase, the per-run dispatch interval, how far behind the inclusive frontier
was, and the launch span.

    python tools/tune/chain_trace.py abl/libmavg_trace.so [--k 44100] [--c 1] [--dtype f32]
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
    assert plan.startswith("chain_scan<"), plan
    ntiles = int(re.search(r"grid=(\d+)", plan).group(1))
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
    tr = ws[ws_bytes - ntiles * 64:].cpu().numpy().view(np.uint64).reshape(ntiles, 8).astype(np.int64)
    print(plan)
    print("launch ms:", " ".join(f"{m:.3f}" for m in ms))
    t0 = tr[:, 0].min()
    st = (tr[:, :6] - t0) * 10  # ns
    span = (st[:, 5].max() - st[:, 0].min()) / 1e3
    print(f"tiles {ntiles}, traced span {span:.1f} us")
    names = ["load (start->A)", "scan (A->chain wave past B)", "look-back (->L(t) published)",
             "carry to tile waves (->C)", "outputs issued (C->end)", "lifetime (start->end)"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (0, 5)]
    for nm, (i, j) in zip(names, pairs):
        d = (st[:, j] - st[:, i]) / 1e3
        print(f"  {nm:32s} median {np.median(d):7.2f} us  p10 {np.percentile(d, 10):7.2f}  "
              f"p90 {np.percentile(d, 90):7.2f}  max {d.max():8.2f}")
    ls = tr[:, 6] & 0xFFFFFFFF
    polls = tr[:, 6] >> 32
    fast = ls < 64
    print(f"  inclusive found at distance ls: median {np.median(ls[fast]):.0f}  p90 {np.percentile(ls[fast], 90):.0f}"
          f"  max {ls[fast].max()}  (first-round hits {np.mean(polls == 0):.3f}, mean polls {polls.mean():.2f})")
    # per-run dispatch interval and concurrency (remap mode 1: 8 contiguous runs)
    q, r = ntiles // 8, ntiles % 8
    starts = [x * (q + 1) if x < r else r * (q + 1) + (x - r) * q for x in range(8)] + [ntiles]
    for x in (0, 3, 7):
        s = st[starts[x]:starts[x + 1]]
        mid = slice(len(s) // 4, 3 * len(s) // 4)
        dstart = np.median(np.diff(s[mid, 0]))
        life = np.median(s[mid, 5] - s[mid, 0])
        print(f"  run {x}: tiles {len(s)}, median start interval {dstart:.1f} ns, lifetime {life / 1e3:.2f} us, "
              f"tiles in flight ~{life / max(dstart, 1e-9):.0f}, run span {(s[:, 5].max() - s[:, 0].min()) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
