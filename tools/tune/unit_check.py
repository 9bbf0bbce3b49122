#!/usr/bin/env python3
"""Spot-check the library's non-default launch paths at full size against the
oracle on sampled slices (bench.py's --check): a reference block size (the
frame-unit tile and look-ahead kernels), the default dispatch, and a view one
frame into the buffer (not 16-B aligned for most shapes).

    python3 tools/tune/unit_check.py [--log2n 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import bench  # noqa: E402
import digital_signal_processsing_amd as dsp  # noqa: E402

CASES = [("f32", 2, 44100), ("i16", 4, 44100), ("f32", 2, 8192), ("i16", 2, 44100), ("f32", 4, 44100),
         ("f32", 1, 44100), ("f32", 8, 44100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=30)
    a = ap.parse_args()
    n = 1 << a.log2n
    for dt, C, k in CASES:
        dtype = torch.float32 if dt == "f32" else torch.int16
        code = dsp.F32 if dt == "f32" else dsp.I16
        x = dsp.fill_synthetic(n, dtype, seed=0x5EED, device="cuda")
        for what, block in (("default", 0), ("block=256", 256)):
            y = torch.empty_like(x)
            plan = dsp.plan(n, k, C, code, "blelloch", block_size=block) if block else dsp.plan(n, k, C, code, "blelloch")
            dsp.moving_average_into(x, y, k, C, "blelloch", block_size=block)
            torch.cuda.synchronize()
            r = bench.check_output(y, n, k, C, dt, 0x5EED, 0, samples=24, span=2048)
            print(f"{dt} C={C} k={k} {what:10s} mismatches {r['mismatches']:8d} / {r['slices']} slices  {plan}",
                  flush=True)
        del x


if __name__ == "__main__":
    main()
