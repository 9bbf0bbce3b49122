#!/usr/bin/env python3
"""Look-ahead distance sweep in bench.py's environment: the library's own
dispatch with D (dispatch slots between a tile and the tile whose record it
publishes) forced through the test hook mavg_test_ahead_schedule (include/mavg_debug.h),
interleaved rounds, one HIP-event pair per launch on torch's current stream.
The hook exists only in builds with MAVG_TEST_HOOKS: this tool loads the
release-flag build with the hooks (`make -C digital_signal_processsing_amd/csrc hooks`
-> lib/libmavg_hooks.so; no device checks, so the timing is the release code's).
The forced D changes only the producer distance; the window-matched run length
stays the tuned schedule's (ahead_run_length of the default D).

    python tools/tune/d_sweep.py --k 4000000 --c 1 --dtype f32 --slots 256 512 768 1024
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import digital_signal_processsing_amd as dsp
from digital_signal_processsing_amd import _lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--c", type=int, default=1)
    ap.add_argument("--dtype", default="f32", choices=["i16", "f32"])
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--slots", type=int, nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    n = 1 << a.log2n
    tdt = torch.int16 if a.dtype == "i16" else torch.float32
    code = dsp.I16 if a.dtype == "i16" else dsp.F32
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libmavg_hooks.so")
    lib = _lib.load(path)
    x = dsp.fill_synthetic(n, tdt, seed=0x5EED, device="cuda")
    y = torch.empty_like(x)
    ref = None
    times = {d: [] for d in a.slots}
    plans = {}
    for rnd in range(a.rounds):
        for d in (a.slots if rnd % 2 == 0 else a.slots[::-1]):
            lib.mavg_test_ahead_schedule(d, -1)
            try:
                plans[d] = dsp.plan(n, a.k, a.c, code, library=path)
                dsp.moving_average_into(x, y, a.k, a.c, library=path)  # warm-up (and the workspace)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
                for e0, e1 in ev:
                    e0.record()
                    dsp.moving_average_into(x, y, a.k, a.c, library=path)
                    e1.record()
                torch.cuda.synchronize()
                times[d] += [e0.elapsed_time(e1) for e0, e1 in ev]
            finally:
                lib.mavg_test_ahead_schedule(-1, -1)
            if ref is None:
                ref = y.clone()
            else:
                assert torch.equal(ref.view(torch.uint8), y.view(torch.uint8)), f"D={d}: outputs differ"
    nbytes = 2 * n * x.element_size()
    print(f"n=2^{a.log2n} k={a.k} C={a.c} dtype={a.dtype} rounds={a.rounds} steps={a.steps}  outputs equal: True")
    for d in a.slots:
        m = statistics.mean(times[d])
        md = statistics.median(times[d])
        print(f"D={d:5d}  mean {m:.4f} ms ({nbytes / m / 8e9:.4f} of 8 TB/s)  median {md:.4f} "
              f"({nbytes / md / 8e9:.4f})  {plans[d]}")


if __name__ == "__main__":
    main()
