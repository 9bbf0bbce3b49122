"""CPU oracle for the moving-average hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker or as the timed CPU
baseline.  The product (``digital_signal_processsing_amd``, ``libmavg.so``,
the ``bin_*`` CLIs) never imports it.

Parity status: **unpinned** against an executed reference -- the reference's
CPU averager does not compile as shipped and the reference holds no golden
vectors (see ``mavg_oracle.c`` header and DESIGN.md).  The C restatement
(``oracle_mavg_*``, following ``basics/profilable_moving_averager.cpp:14-37``)
is cross-checked against the independent numpy formulation below and against
closed-form known answers in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    """Compile the C restatement (gcc) into oracle/liboracle.so."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    p, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    lib.oracle_mavg_i16.argtypes = [p, p, sz, i, i]
    lib.oracle_mavg_f32.argtypes = [p, p, sz, i, i]
    lib.oracle_window_sum_i64.argtypes = [p, sz, i, i, sz, sz, p]
    lib.oracle_mavg_f32_mt.argtypes = [p, p, sz, i, i, i]
    lib.oracle_mavg_f32_mt.restype = ctypes.c_int
    lib.oracle_synth_i16.argtypes = [p, sz, u64, u64]
    lib.oracle_synth_f32.argtypes = [p, sz, u64, u64, i]
    for f in (lib.oracle_mavg_i16, lib.oracle_mavg_f32, lib.oracle_window_sum_i64):
        f.restype = ctypes.c_int
    pu = ctypes.POINTER(ctypes.c_uint64)
    pd = ctypes.POINTER(ctypes.c_double)
    lib.oracle_check_synth_f32.argtypes = [p, sz, i, i, u64, u64, i, ctypes.c_double, i, pu, pu, pd]
    lib.oracle_check_synth_f32.restype = ctypes.c_int
    lib.oracle_check_synth_i16.argtypes = [p, sz, i, i, u64, u64, i, pu, pu]
    lib.oracle_check_synth_f32_exact.argtypes = [p, sz, i, i, u64, u64, i, ctypes.c_double, i, p, p]
    lib.oracle_check_synth_f32_exact.restype = ctypes.c_int
    lib.oracle_check_synth_i16.restype = ctypes.c_int
    lib.oracle_synth_i16.restype = None
    lib.oracle_synth_f32.restype = None
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def mavg_i16(x: np.ndarray, k: int, channels: int = 1) -> np.ndarray:
    """int16 mode, bit-exact restatement of profilable_cpu_computations."""
    x = np.ascontiguousarray(x, dtype=np.int16)
    y = np.zeros_like(x)
    rc = _load().oracle_mavg_i16(_ptr(x), _ptr(y), x.size, channels, k)
    if rc != 0:
        raise ValueError(f"oracle_mavg_i16: bad arguments (n={x.size}, C={channels}, k={k})")
    return y


def mavg_f32(x: np.ndarray, k: int, channels: int = 1) -> np.ndarray:
    """fp32 mode: double running sum, float(sum / k)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros_like(x)
    rc = _load().oracle_mavg_f32(_ptr(x), _ptr(y), x.size, channels, k)
    if rc != 0:
        raise ValueError(f"oracle_mavg_f32: bad arguments (n={x.size}, C={channels}, k={k})")
    return y


def mavg_f32_mt(x: np.ndarray, k: int, channels: int = 1, threads: int = 8) -> np.ndarray:
    """Multi-core CPU baseline (OpenMP, per-chunk k-frame halo)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros_like(x)
    rc = _load().oracle_mavg_f32_mt(_ptr(x), _ptr(y), x.size, channels, k, threads)
    if rc != 0:
        raise ValueError("oracle_mavg_f32_mt: bad arguments")
    return y


def window_sum_i64(x: np.ndarray, k: int, channels: int, f0: int, f1: int) -> np.ndarray:
    """Exact int64 windowed sums for frames [f0, f1) (zero history)."""
    x = np.ascontiguousarray(x, dtype=np.int16)
    out = np.zeros((f1 - f0) * channels, dtype=np.int64)
    rc = _load().oracle_window_sum_i64(_ptr(x), x.size, channels, k, f0, f1, _ptr(out))
    if rc != 0:
        raise ValueError("oracle_window_sum_i64: bad arguments")
    return out


def synth_i16(n: int, seed: int = 0x5EED, offset: int = 0) -> np.ndarray:
    x = np.empty(n, dtype=np.int16)
    _load().oracle_synth_i16(_ptr(x), n, seed, offset)
    return x


def synth_f32(n: int, seed: int = 0x5EED, offset: int = 0, dist: int = 0) -> np.ndarray:
    x = np.empty(n, dtype=np.float32)
    _load().oracle_synth_f32(_ptr(x), n, seed, offset, dist)
    return x


# ---------------------------------------------------------------------------
# Independent numpy formulation (per-channel prefix sums).  Used only to
# cross-check the C restatement; it shares no code with it.
# ---------------------------------------------------------------------------
def numpy_window_sum(x: np.ndarray, k: int, channels: int = 1) -> np.ndarray:
    """S[f, c] = sum_{j<k} x[(f-j)C + c] with zero history, exact in int64 /
    float64 (float64 only approximately for non-integer float data)."""
    xf = x.reshape(-1, channels)
    acc = np.int64 if np.issubdtype(x.dtype, np.integer) else np.float64
    p = np.cumsum(xf.astype(acc), axis=0)
    s = p.copy()
    if k < p.shape[0]:
        s[k:] = p[k:] - p[:-k]
    return s.reshape(-1)


def numpy_mavg_i16(x: np.ndarray, k: int, channels: int = 1) -> np.ndarray:
    s = numpy_window_sum(x.astype(np.int16), k, channels)
    q = np.abs(s) // k  # C++ integer division truncates toward zero
    return (np.sign(s) * q).astype(np.int16)


def numpy_mavg_f32(x: np.ndarray, k: int, channels: int = 1) -> np.ndarray:
    return (numpy_window_sum(x.astype(np.float32), k, channels) / float(k)).astype(np.float32)


def check_synth(y: np.ndarray, k: int, channels: int = 1, seed: int = 0x5EED, offset: int = 0, dist: int = 0,
                rtol: float = 1e-5, threads: int = 0) -> dict:
    """Check EVERY sample of a device output ``y`` against the restatement over
    the counter-based synthetic stream (samples [offset, offset + y.size) of
    it, zero history before sample 0) without materialising the input: int16
    bit-exact, fp32 within ``rtol`` relative.  Chunked over ``threads`` cores;
    exact for these inputs (see oracle_check_synth_f32 in mavg_oracle.c).
    Returns {"checked", "mismatches", "first_bad" (sample index or None),
    "max_rel" (fp32)}.  fp32 dist 2 (whose fp64 sums round) goes to
    check_synth_exact."""
    threads = threads or min(16, len(os.sched_getaffinity(0)))
    y = np.ascontiguousarray(y)
    if y.dtype == np.float32 and dist == 2:
        return check_synth_exact(y, k, channels, seed, offset, dist, rtol, threads)
    bad, first = ctypes.c_uint64(0), ctypes.c_uint64(0)
    if y.dtype == np.int16:
        rc = _load().oracle_check_synth_i16(_ptr(y), y.size, channels, k, seed, offset, threads,
                                            ctypes.byref(bad), ctypes.byref(first))
        worst = None
    elif y.dtype == np.float32:
        mr = ctypes.c_double(0.0)
        rc = _load().oracle_check_synth_f32(_ptr(y), y.size, channels, k, seed, offset, dist, rtol, threads,
                                            ctypes.byref(bad), ctypes.byref(first), ctypes.byref(mr))
        worst = mr.value
    else:
        raise TypeError(f"check_synth: int16 or float32 output, got {y.dtype}")
    if rc != 0:
        raise ValueError(f"oracle_check_synth: bad arguments (n={y.size}, C={channels}, k={k}, offset={offset})")
    return {"checked": int(y.size), "mismatches": int(bad.value),
            "first_bad": None if bad.value == 0 else int(first.value), "max_rel": worst}


def check_synth_exact(y: np.ndarray, k: int, channels: int = 1, seed: int = 0x5EED, offset: int = 0,
                      dist: int = 2, rtol: float = 1e-5, threads: int = 0) -> dict:
    """fp32 check of EVERY sample against the EXACT window sum (__int128 fixed
    point, oracle_check_synth_f32_exact): pass when |y - S/k| <= rtol |S/k|, or
    on the floor |y - S/k| <= rtol * F with F = sum|x| / k, the window's mean
    absolute input (for |S/k| ~ 0).  Returns {"checked", "mismatches",
    "first_bad", "floor_used" (outputs that passed only on the floor),
    "not_correctly_rounded" (y != fl32(S/k)), "max_rel" (over S != 0),
    "max_cond" (max |y - S/k| / F; the fp32 output rounding alone is up to
    2^-24)}."""
    threads = threads or min(16, len(os.sched_getaffinity(0)))
    y = np.ascontiguousarray(y, dtype=np.float32)
    st = np.zeros(4, np.uint64)
    ds = np.zeros(2, np.float64)
    rc = _load().oracle_check_synth_f32_exact(_ptr(y), y.size, channels, k, seed, offset, dist, rtol, threads,
                                             _ptr(st), _ptr(ds))
    if rc == -2:
        raise ValueError("check_synth_exact: a sample is not a multiple of 2^-64 (not exactly representable)")
    if rc != 0:
        raise ValueError(f"check_synth_exact: bad arguments (n={y.size}, C={channels}, k={k}, offset={offset})")
    return {"checked": int(y.size), "mismatches": int(st[0]), "first_bad": None if st[0] == 0 else int(st[1]),
            "floor_used": int(st[2]), "not_correctly_rounded": int(st[3]), "max_rel": float(ds[0]),
            "max_cond": float(ds[1])}


def numpy_synth_f32_dist2(n: int, seed: int = 0x5EED, offset: int = 0) -> np.ndarray:
    """Independent numpy statement of the dist-2 generator (cross-check of
    synth_f32_dist2 in mavg_oracle.c; shares no code with it)."""
    z = np.arange(offset, offset + n, dtype=np.uint64) + np.uint64(seed)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    h = z ^ (z >> np.uint64(31))
    m = np.uint64(0x3FFF)
    i = sum(((h >> np.uint64(s)) & m).astype(np.int64) for s in (0, 14, 28, 42)) - 32766
    b = ((h >> np.uint64(56)) & np.uint64(31)).astype(np.int64)
    s = np.where(b < 8, 0, b - 8)
    v = i.astype(np.float64) * (1.0 / 3000.0)
    return (v * np.ldexp(1.0, -s)).astype(np.float32)
