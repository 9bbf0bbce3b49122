"""MI355X-native (gfx950) causal moving-average filter.

Host-side Python mirror of the reference's per-variant GPU drivers
(``<Variant>GpuLoad`` in ``basics/*.cu``): every call goes through the C ABI of
``libmavg.so`` (include/mavg.h) into hand-written HIP kernels.  PyTorch is used
only for device memory and streams.

    y = moving_average(x, grade=1024)                  # fp32 or int16 CUDA tensor
    y = moving_average(x, grade=32, channels=2, algo="hillis")

Semantics: ``basics/profilable_moving_averager.cpp:14-37`` -- interleaved
frames, window ``grade`` frames, zero history (or ``history``: the
(grade-1)*channels samples that precede ``x``), int16 output = exact
truncating ``S / grade``, fp32 output = ``S / grade`` with ``S`` in fp64.
"""
from __future__ import annotations

from typing import Optional

from . import _lib
from ._lib import (ALGOS, F32, I16, MavgError, MavgLibraryError, algo_name,  # noqa: F401
                   strerror)

__all__ = [
    "moving_average",
    "moving_average_into",
    "fill_synthetic",
    "workspace_bytes",
    "resolve_algo",
    "plan",
    "stream_copy",
    "ALGOS",
    "MavgError",
    "MavgLibraryError",
]


def _torch():
    import torch
    return torch


def _dtype_code(t) -> int:
    torch = _torch()
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.int16:
        return I16
    raise TypeError(f"moving_average supports float32 and int16 tensors, got {t.dtype}")


def _algo_code(algo) -> int:
    if isinstance(algo, int):
        return algo
    try:
        return ALGOS[algo]
    except KeyError:
        raise ValueError(f"unknown algo {algo!r}; one of {sorted(ALGOS)}") from None


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def _stream_handle(stream, device) -> int:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return stream.cuda_stream


def workspace_bytes(n: int, grade: int, channels: int = 1, dtype: int = F32, algo="auto",
                    block_size: int = 0, library: Optional[str] = None) -> int:
    import ctypes
    out = ctypes.c_size_t(0)
    _lib.check(_lib.load(library).mavg_workspace_bytes(n, channels, grade, dtype, _algo_code(algo), block_size,
                                                ctypes.byref(out)), "mavg_workspace_bytes")
    return out.value


def resolve_algo(n: int, grade: int, channels: int = 1, dtype: int = F32, algo="auto",
                 library: Optional[str] = None) -> str:
    lib = _lib.load(library)
    return lib.mavg_algo_name(lib.mavg_resolve_algo(n, channels, grade, dtype, _algo_code(algo))).decode()


def plan(n: int, grade: int, channels: int = 1, dtype: int = F32, algo="auto", block_size: int = 0,
         library: Optional[str] = None) -> str:
    """The kernel and launch geometry mavg_run would use (nothing is launched)."""
    import ctypes
    buf = ctypes.create_string_buffer(256)
    _lib.check(_lib.load(library).mavg_plan(n, channels, grade, dtype, _algo_code(algo), block_size, buf, len(buf)),
               "mavg_plan")
    return buf.value.decode()


def moving_average_into(x, out, grade: int, channels: int = 1, algo="auto", history=None,
                        block_size: int = 0, stream=None, workspace=None, library: Optional[str] = None) -> None:
    """Enqueue ``out = moving_average(x)`` on ``stream`` (default: current).

    ``workspace``: optional caller-owned device buffer (any dtype, contiguous)
    of at least ``workspace_bytes(...)`` bytes, like the reference's
    ``DspWorkspace`` scratch; without it the look-back scan (long windows)
    takes one from torch's caching allocator per call.
    ``library``: path of another build of the same ABI (the debug build,
    ``_lib.DEBUG_LIB_PATH``); default the release ``libmavg.so``."""
    torch = _torch()
    if not (x.is_cuda and out.is_cuda):
        raise ValueError("x and out must be device tensors (libmavg has no CPU path)")
    if not (x.is_contiguous() and out.is_contiguous()):
        raise ValueError("x and out must be contiguous")
    if x.dtype != out.dtype or x.numel() != out.numel():
        raise ValueError("x and out must have the same dtype and size")
    dt = _dtype_code(x)
    hist_ptr = None
    if history is not None:
        if history.dtype != x.dtype or not history.is_cuda or not history.is_contiguous():
            raise ValueError("history must be a contiguous device tensor of x's dtype")
        if history.numel() != (grade - 1) * channels:
            raise ValueError(f"history must hold (grade-1)*channels = {(grade - 1) * channels} samples")
        hist_ptr = history.data_ptr() if history.numel() else None
    # workspace (look-back scan only): from torch's caching allocator, tied to
    # the launch stream so it is not handed out again before the kernel ends
    ws_n = workspace_bytes(x.numel(), grade, channels, dt, algo, block_size, library)
    ws = None
    if ws_n and workspace is not None:
        if not (workspace.is_cuda and workspace.is_contiguous()):
            raise ValueError("workspace must be a contiguous device tensor")
        if workspace.numel() * workspace.element_size() < ws_n:
            raise ValueError(f"workspace holds {workspace.numel() * workspace.element_size()} bytes, "
                             f"the launch needs {ws_n}")
        ws, ws_n = workspace, workspace.numel() * workspace.element_size()
    elif ws_n:
        if torch.cuda.is_current_stream_capturing():
            # a workspace taken from the capture's private pool is freed again
            # before the capture ends; pass one that outlives the graph
            raise ValueError(f"grade={grade} uses the look-back scan, which needs a {ws_n}-byte workspace: "
                             "inside a graph capture pass workspace= (see workspace_bytes())")
        # allocated on the launch stream itself: a block the caching allocator
        # hands out there is free with respect to that stream's pending work
        # (one taken on another stream could still be in use by kernels queued
        # there, and record_stream only protects the free)
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            ws = torch.empty(ws_n, dtype=torch.uint8, device=x.device)
    st = _lib.load(library).mavg_run(x.data_ptr(), out.data_ptr(), x.numel(), channels, grade, dt,
                              _algo_code(algo), block_size, hist_ptr,
                              ws.data_ptr() if ws is not None else None, ws_n,
                              _stream_handle(stream, x.device))
    _lib.check(st, "mavg_run")


def moving_average(x, grade: int, channels: int = 1, algo="auto", history=None,
                   block_size: int = 0, stream=None, library: Optional[str] = None):
    """Causal ``grade``-frame moving average of an interleaved signal ``x``."""
    torch = _torch()
    if stream is not None and stream != torch.cuda.current_stream(x.device):
        # x (and history) come from the caller's current stream: the launch
        # stream waits for it, and `out` is allocated on the launch stream
        stream.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(stream):
            out = torch.empty_like(x)
        moving_average_into(x, out, grade, channels, algo, history, block_size, stream, library=library)
        # the kernel reads x and history on `stream`: keep the caching
        # allocator from handing their blocks out again before it ends
        x.record_stream(stream)
        if history is not None:
            history.record_stream(stream)
        return out
    out = torch.empty_like(x)
    moving_average_into(x, out, grade, channels, algo, history, block_size, stream, library=library)
    return out


def fill_synthetic(n: int, dtype=None, seed: int = 0x5EED, offset: int = 0, dist: int = 0,
                   device="cuda", stream=None, out=None):
    """Counter-based synthetic signal generated on the device:
    element i is splitmix64(seed + offset + i) >> 48 as int16 (dist 0), or a
    uniform [0,1) float (dist 1)."""
    torch = _torch()
    dtype = torch.float32 if dtype is None else dtype
    if out is None:
        out = torch.empty(n, dtype=dtype, device=device)
    st = _lib.load().mavg_fill_synthetic(out.data_ptr(), out.numel(), _dtype_code(out), seed, offset,
                                         dist, _stream_handle(stream, out.device))
    _lib.check(st, "mavg_fill_synthetic")
    return out


def stream_copy(src, dst, stream=None) -> None:
    """HBM calibration: dst = src with the library's flat non-temporal copy
    kernel (not part of the filter; bench.py's same-box streaming ceiling)."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes:
        raise ValueError("src and dst must have the same size in bytes")
    st = _lib.load().mavg_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, _stream_handle(stream, src.device))
    _lib.check(st, "mavg_stream_copy")
