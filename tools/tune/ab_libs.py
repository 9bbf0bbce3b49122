#!/usr/bin/env python3
"""A/B two builds of libmavg.so inside bench.py's environment (torch-allocated
buffers, one launch per HIP-event pair on torch's current stream, launches
back to back): the in-process tuner and bench.py disagreed on a tile rule,
and this separates the kernel from the harness.

    python tools/tune/ab_libs.py LIB_A LIB_B [--k 1024] [--c 1] [--dtype i16] [--rounds 6] [--steps 20]

Prints, per library, the mean / median of the per-launch times over all
rounds (rounds alternate A, B, A, B ...) and the same-stream copy for scale.
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import digital_signal_processsing_amd as dsp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+", help="two or more library builds")
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--c", type=int, default=1)
    ap.add_argument("--dtype", default="i16", choices=["i16", "f32"])
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--algo", type=int, default=0, help="mavg_algo (0 auto, 5 direct)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--dist", type=int, default=0, help="synthetic distribution (fp32: 0, 1, 2)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ypad", type=int, default=0, help="offset y by this many bytes inside a bigger buffer")
    ap.add_argument("--blocks", type=int, nargs="+", default=None,
                    help="block_size per library (0: the tuned dispatch; else the reference's block size)")
    a = ap.parse_args()
    a.blocks = a.blocks or [0] * len(a.libs)
    assert len(a.libs) >= 2 and len(a.blocks) == len(a.libs)
    n = 1 << a.log2n
    tdt = torch.int16 if a.dtype == "i16" else torch.float32
    code = dsp.I16 if a.dtype == "i16" else dsp.F32
    x = dsp.fill_synthetic(n, tdt, seed=0x5EED, dist=a.dist, device="cuda")
    pad = a.ypad // x.element_size()
    ybuf = torch.empty(n + pad, dtype=tdt, device="cuda")
    y = ybuf[pad:]
    libs = []
    blocks = {}
    for li, p in enumerate(a.libs):
        lib = ctypes.CDLL(p)
        lib.mavg_run.restype = ctypes.c_int
        lib.mavg_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_size_t, ctypes.c_void_p]
        buf = ctypes.create_string_buffer(512)
        lib.mavg_plan.restype = ctypes.c_int
        lib.mavg_plan(ctypes.c_size_t(n), a.c, a.k, code, a.algo, a.blocks[li], buf, ctypes.c_size_t(512))
        p = f"{p} block={a.blocks[li]}"
        libs.append((p, lib, buf.value.decode()))
        blocks[p] = a.blocks[li]
    stream = torch.cuda.current_stream().cuda_stream
    wsb = {}
    for p, lib, _ in libs:  # each library's own workspace (long-window scans)
        nb = ctypes.c_size_t(0)
        lib.mavg_workspace_bytes.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
        assert lib.mavg_workspace_bytes(n, a.c, a.k, code, a.algo, blocks[p], ctypes.byref(nb)) == 0
        wsb[p] = torch.empty(max(16, nb.value), dtype=torch.uint8, device="cuda") if nb.value else None

    def launch(lib, p):
        ws = wsb[p]
        st = lib.mavg_run(x.data_ptr(), y.data_ptr(), n, a.c, a.k, code, a.algo, blocks[p], None,
                          ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, stream)
        assert st == 0, st

    def copy():
        y.copy_(x)

    times = {p: [] for p, _, _ in libs}
    times["torch copy_"] = []
    for p, lib, _ in libs:  # warm-up
        for _ in range(5):
            launch(lib, p)
    torch.cuda.synchronize()
    outs = []
    for r in range(a.rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for p, lib, _ in order:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            for e0, e1 in ev:
                e0.record()
                launch(lib, p)
                e1.record()
            torch.cuda.synchronize()
            times[p] += [e0.elapsed_time(e1) for e0, e1 in ev]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        for e0, e1 in ev:
            e0.record()
            copy()
            e1.record()
        torch.cuda.synchronize()
        times["torch copy_"] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for p, lib, _ in libs:
        launch(lib, p)
        torch.cuda.synchronize()
        outs.append(y.clone())
    byt = 2 * x.element_size() * n
    print(f"n=2^{a.log2n} k={a.k} C={a.c} dtype={a.dtype} rounds={a.rounds} steps={a.steps} "
          f"y-x={y.data_ptr() - x.data_ptr():#x}  outputs equal: "
          f"{all(bool(torch.equal(outs[0], o)) for o in outs[1:])}  max |diff| "
          f"{max(float((outs[0].double() - o.double()).abs().max()) for o in outs[1:]):.3g}")
    for p, lib, plan in libs + [("torch copy_", None, "")]:
        t = times[p]
        mean, med = statistics.mean(t), statistics.median(t)
        print(f"{p:48s} mean {mean:.4f} ms ({byt / mean / 1e6 / 8000:.4f} of 8 TB/s)  median {med:.4f} "
              f"({byt / med / 1e6 / 8000:.4f})  min {min(t):.4f}  {plan}")


if __name__ == "__main__":
    main()
