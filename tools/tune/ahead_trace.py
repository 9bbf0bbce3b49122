#!/usr/bin/env python3
"""Phase timeline of the look-ahead scan from a MAVG_AHEAD_TRACE build
(make -C digital_signal_processsing_amd/csrc OBJ=../../build/obj_atrace OUT=../../abl
 LIBNAME=libmavg_atrace.so HIPFLAGS="... -DMAVG_AHEAD_TRACE").

Per tile, thread 0 stamps (100-MHz wall clock, s_memrealtime):
  0 start   1 phase A summed (per-wave records: published)   2 first barrier passed
  3 in-tile scan done   4 wave 0's carry items read   5 second barrier passed   6 outputs issued
  7 wave 0's polls of untagged carry items
Prints, over the last of several launches, the distribution of each phase,
the per-run dispatch interval, the tiles in flight per XCD and the launch span.

    python tools/tune/ahead_trace.py abl/libmavg_atrace.so [--k 44100] [--c 1] [--dtype f32]
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
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--slots", default=None,
                    help="an experiment build's stamp order, e.g. 0,2,4,1,5,3,6: consecutive differences only")
    a = ap.parse_args()
    n = 1 << a.log2n
    tdt = torch.float32 if a.dtype == "f32" else torch.int16
    code = dsp.F32 if a.dtype == "f32" else dsp.I16
    lib = ctypes.CDLL(a.lib)
    lib.mavg_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_int] * 5 + [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.mavg_plan.argtypes = [ctypes.c_size_t] + [ctypes.c_int] * 5 + [ctypes.c_char_p, ctypes.c_size_t]
    lib.mavg_workspace_bytes.argtypes = [ctypes.c_size_t] + [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_size_t)]
    buf = ctypes.create_string_buffer(512)
    assert lib.mavg_plan(n, a.c, a.k, code, a.algo, 0, buf, 512) == 0
    plan = buf.value.decode()
    assert plan.startswith(("ahead_scan<", "wide_ahead<")), plan
    ntiles = int(re.search(r"grid=(\d+)", plan).group(1))
    plan_ws = int(re.search(r"ws=(\d+)", plan).group(1))  # this launch's need: the trace ends there
    need = ctypes.c_size_t(0)
    assert lib.mavg_workspace_bytes(n, a.c, a.k, code, a.algo, 0, ctypes.byref(need)) == 0
    ws_bytes = max(need.value, plan_ws)  # what the library demands for the problem (any view alignment)
    remap = int(re.search(r"remap=(\d+)", plan).group(1))
    x = dsp.fill_synthetic(n, tdt, dist=2 if a.dtype == "f32" else 0, device="cuda")
    y = torch.empty_like(x)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    for e0, e1 in ev:
        e0.record()
        rc = lib.mavg_run(x.data_ptr(), y.data_ptr(), n, a.c, a.k, code, a.algo, 0, None, ws.data_ptr(), ws_bytes,
                          stream)
        assert rc == 0, f"mavg_run returned {rc} (workspace {ws_bytes} B, plan {plan})"
        e1.record()
    torch.cuda.synchronize()
    ms = [e0.elapsed_time(e1) for e0, e1 in ev]
    tr = ws[plan_ws - ntiles * 64:plan_ws].cpu().numpy().view(np.uint64).reshape(ntiles, 8).astype(np.int64)
    print(plan)
    nbytes = 2 * n * x.element_size()
    print("launch ms:", " ".join(f"{m:.3f}" for m in ms), f" (last: {nbytes / ms[-1] / 8e9:.3f} of 8 TB/s)")
    t0 = tr[:, 0].min()
    st = (tr[:, :7] - t0) * 10  # ns
    span = (st[:, 6].max() - st[:, 0].min()) / 1e3
    print(f"tiles {ntiles}, traced span {span:.1f} us")
    if a.slots:
        order = [int(v) for v in a.slots.split(",")]
        for i, j in zip(order, order[1:]):
            d = (st[:, j] - st[:, i]) / 1e3
            print(f"  stamp {i} -> {j}: median {np.median(d):7.2f} us  mean {d.mean():7.2f}  p10 {np.percentile(d, 10):7.2f}  "
                  f"p90 {np.percentile(d, 90):7.2f}")
        return
    names = ["phase A (start->1)", "to first barrier (1->2)", "publish + in-tile scan (2->3)",
             "carry items (3->4)", "second barrier (4->5)", "outputs issued (5->6)", "lifetime (start->end)"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (0, 6)]
    life = st[:, 6] - st[:, 0]
    for nm, (i, j) in zip(names, pairs):
        d = (st[:, j] - st[:, i]) / 1e3
        print(f"  {nm:32s} median {np.median(d):7.2f} us  mean {d.mean():7.2f}  p10 {np.percentile(d, 10):7.2f}  "
              f"p90 {np.percentile(d, 90):7.2f}  share of lifetime {d.sum() / (life.sum() / 1e3):.3f}")
    polls = tr[:, 7]
    print(f"  wave-0 carry polls: tiles that polled {np.mean(polls > 0):.4f}, mean {polls.mean():.3f}, max {polls.max()}")
    if remap == 1:
        q, r = ntiles // 8, ntiles % 8
        starts = [xx * (q + 1) if xx < r else r * (q + 1) + (xx - r) * q for xx in range(8)] + [ntiles]
        for xx in (0, 3, 7):
            s = st[starts[xx]:starts[xx + 1]]
            mid = slice(len(s) // 4, 3 * len(s) // 4)
            dstart = np.median(np.diff(s[mid, 0]))
            lf = np.median(s[mid, 6] - s[mid, 0])
            print(f"  run {xx}: tiles {len(s)}, median start interval {dstart:.1f} ns, lifetime {lf / 1e3:.2f} us, "
                  f"tiles in flight ~{lf / max(dstart, 1e-9):.0f}, run span {(s[:, 6].max() - s[:, 0].min()) / 1e3:.1f} us")
    else:
        # window-matched runs (remap G): tile t runs on XCD (t // G) % 8 (tiles past the last whole
        # period map to themselves and are left out); per XCD, the start interval over the middle
        # half of its tiles (many tiles share a 10-ns stamp, so not the median of the differences)
        full = ntiles - ntiles % (8 * remap)
        for xx in (0, 3, 7):
            tiles = np.array([t for t in range(full) if (t // remap) % 8 == xx])
            s0 = np.sort(st[tiles, 0])
            lo, hi = len(s0) // 4, 3 * len(s0) // 4
            dstart = (s0[hi] - s0[lo]) / max(hi - lo, 1)
            lf = np.median(life[tiles])
            print(f"  XCD {xx}: tiles {len(tiles)}, mean start interval {dstart:.2f} ns (middle half), lifetime "
                  f"{lf / 1e3:.2f} us, tiles in flight ~{lf / max(dstart, 1e-9):.0f}")


if __name__ == "__main__":
    main()
