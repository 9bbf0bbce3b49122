"""CPU tests of the drop-in boundary: libmavg.so loads, exports every symbol
include/mavg.h declares, and validates arguments without touching a GPU."""
import ctypes
import os
import re

import pytest

from digital_signal_processsing_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols(header="mavg.h"):
    text = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mavg_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert _header_symbols() == sorted(_lib.EXPORTED_SYMBOLS)
    assert _header_symbols("mavg_debug.h") == sorted(_lib.DEBUG_SYMBOLS)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in _header_symbols():
        assert hasattr(lib, name), name
    assert lib.mavg_abi_version() == _lib.ABI_VERSION == 4


def test_release_library_has_no_test_hook():
    """The schedule test hook (process-wide state) is exported by the debug
    build only (include/mavg_debug.h); the release build exports exactly
    include/mavg.h."""
    lib = _lib.load()
    for name in _lib.DEBUG_SYMBOLS:
        assert not hasattr(lib, name), name
    dbg = _lib.load(_lib.DEBUG_LIB_PATH)
    for name in _header_symbols() + _header_symbols("mavg_debug.h"):
        assert hasattr(dbg, name), name
    assert dbg.mavg_abi_version() == _lib.ABI_VERSION


def test_loaded_libraries_are_built_from_this_tree():
    """Every shipped build of the library carries the source id of csrc/ and
    include/ it was compiled from (mavg_build_id, build_id.py): a prebuilt
    library that does not match the tree's sources fails here."""
    from digital_signal_processsing_amd import build_id
    want = build_id.source_id()
    assert re.fullmatch(r"[0-9a-f]{16}", want)
    for path in (_lib.LIB_PATH, _lib.DEBUG_LIB_PATH, _lib.HOOKS_LIB_PATH):
        assert _lib.build_id(path) == want, (path, "stale library: rebuild with __graft_entry__.build()")


def _dynamic_flags(path):
    """DT_FLAGS of an ELF64 little-endian shared object (0 when absent)."""
    import struct
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2 and data[5] == 1, path
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    for i in range(shnum):
        sh_type, = struct.unpack_from("<I", data, shoff + i * shentsize + 4)
        if sh_type != 6:  # SHT_DYNAMIC
            continue
        off, size = struct.unpack_from("<QQ", data, shoff + i * shentsize + 0x18)
        flags = 0
        for j in range(0, size, 16):
            tag, val = struct.unpack_from("<qQ", data, off + j)
            if tag == 30:  # DT_FLAGS
                flags = val
        return flags
    return 0


def test_library_binds_its_own_kernels():
    """Every build is linked -Bsymbolic (DF_SYMBOLIC): a kernel template instance is a weak
    symbol, and without it a program instantiating the same kernel from other sources (a tuner
    built from an older tree) interposes its host stub, so the library's own launches would run
    that program's code object (round 5: an in-process A/B that compared nothing)."""
    for path in (_lib.LIB_PATH, _lib.DEBUG_LIB_PATH, _lib.HOOKS_LIB_PATH):
        assert _dynamic_flags(path) & 0x2, path  # DF_SYMBOLIC


def test_build_id_follows_the_sources(tmp_path):
    """The id changes with any byte of a source file, and only with the sources."""
    import shutil
    from digital_signal_processsing_amd import build_id
    for rel in ("digital_signal_processsing_amd/csrc", "include"):
        shutil.copytree(os.path.join(ROOT, rel), tmp_path / rel,
                        ignore=shutil.ignore_patterns("*.o", "*.so", "__pycache__"))
    base = build_id.source_id(str(tmp_path))
    assert base == build_id.source_id()
    (tmp_path / "README").write_text("not a source")
    assert build_id.source_id(str(tmp_path)) == base
    hpp = tmp_path / "digital_signal_processsing_amd" / "csrc" / "mavg_tile.hpp"
    hpp.write_bytes(hpp.read_bytes() + b"\n")
    assert build_id.source_id(str(tmp_path)) != base


def test_strerror_and_names():
    assert _lib.strerror(_lib.OK) == "ok"
    assert "invalid" in _lib.strerror(_lib.ERR_INVALID_ARG)
    for name, code in _lib.ALGOS.items():
        assert _lib.algo_name(code) == name


def _run(n, C, k, dtype=_lib.F32, algo=0, din=16, dout=16, hist=None, block=0):
    lib = _lib.load()
    return lib.mavg_run(din, dout, n, C, k, dtype, algo, block, hist, None, 0, None)


@pytest.mark.parametrize("args,status", [
    (dict(n=10, C=1, k=0), _lib.ERR_INVALID_ARG),        # k < 1 (reference divides by zero)
    (dict(n=10, C=0, k=3), _lib.ERR_INVALID_ARG),        # C < 1
    (dict(n=9, C=2, k=3), _lib.ERR_INVALID_ARG),         # partial frame
    (dict(n=16, C=9, k=3), _lib.ERR_INVALID_ARG),        # 16 % 9 != 0
    (dict(n=18, C=9, k=3, algo=1), _lib.ERR_UNSUPPORTED),  # C > 8 on a templated kernel
    (dict(n=10, C=1, k=3, dtype=7), _lib.ERR_INVALID_ARG),
    (dict(n=10, C=1, k=3, algo=99), _lib.ERR_INVALID_ARG),
    (dict(n=10, C=1, k=3, din=0), _lib.ERR_INVALID_ARG),  # null input
    (dict(n=8, C=1, k=3, din=18), _lib.ERR_MISALIGNED),   # fp32 view not 4-B aligned
    (dict(n=8, C=1, k=3, dout=22), _lib.ERR_MISALIGNED),
    (dict(n=8, C=1, k=3, dtype=_lib.I16, din=21), _lib.ERR_MISALIGNED),  # int16 view not 2-B aligned
    (dict(n=8, C=1, k=3, hist=19), _lib.ERR_MISALIGNED),  # history not sample-aligned
    (dict(n=8, C=1, k=3, block=48), _lib.ERR_INVALID_ARG),    # reference: a multiple of 32 in [32, 1024]
    (dict(n=8, C=1, k=3, block=2048), _lib.ERR_INVALID_ARG),
    (dict(n=8, C=1, k=3, block=16), _lib.ERR_INVALID_ARG),
    (dict(n=0, C=1, k=3, din=0, dout=0), _lib.OK),        # empty input is a no-op
])
def test_run_validates_before_launch(args, status):
    assert _run(**args) == status


def test_workspace_bytes():
    lib = _lib.load()
    out = ctypes.c_size_t(123)
    assert lib.mavg_workspace_bytes(1 << 20, 1, 1024, _lib.F32, _lib.ALGO_BLELLOCH, 0, ctypes.byref(out)) == _lib.OK
    assert out.value == 0
    assert lib.mavg_workspace_bytes(1 << 20, 1, 1024, _lib.F32, 0, 0, None) == _lib.ERR_INVALID_ARG


def test_resolve_algo_is_concrete():
    lib = _lib.load()
    for k in (1, 7, 64, 1024, 4096, 100000):
        a = lib.mavg_resolve_algo(1 << 20, 1, k, _lib.F32, _lib.ALGO_AUTO)
        assert a != _lib.ALGO_AUTO and _lib.algo_name(a) != "invalid"


def test_stream_copy_validates():
    lib = _lib.load()
    assert lib.mavg_stream_copy(None, None, 0, None) == _lib.OK
    assert lib.mavg_stream_copy(None, 16, 32, None) == _lib.ERR_INVALID_ARG
    assert lib.mavg_stream_copy(16, 32, 24, None) == _lib.ERR_INVALID_ARG   # not a multiple of 16
    assert lib.mavg_stream_copy(8, 32, 32, None) == _lib.ERR_MISALIGNED


def test_fill_synthetic_validates():
    lib = _lib.load()
    assert lib.mavg_fill_synthetic(None, 0, _lib.F32, 1, 0, 0, None) == _lib.OK
    assert lib.mavg_fill_synthetic(None, 8, _lib.F32, 1, 0, 0, None) == _lib.ERR_INVALID_ARG
    assert lib.mavg_fill_synthetic(16, 8, _lib.I16, 1, 0, 1, None) == _lib.ERR_INVALID_ARG
    assert lib.mavg_fill_synthetic(16, 8, _lib.I16, 1, 0, 2, None) == _lib.ERR_INVALID_ARG  # dist 2: fp32 only
    assert lib.mavg_fill_synthetic(16, 8, _lib.F32, 1, 0, 3, None) == _lib.ERR_INVALID_ARG


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_libs", {})
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.MavgLibraryError):
        _lib.load()


def test_plan_describes_launch_without_gpu():
    import digital_signal_processsing_amd as dsp
    p = dsp.plan(1 << 30, 1024)
    # fp32 mono: 512-thread tiles staged by LDS-DMA up to 16 KiB of halo
    assert p.startswith("tile_scan<f32,acc=f64,C=1,F=4,U=2,blelloch") and "grid=262144" in p, p
    assert "block=512" in p and "dma=1" in p, p
    # split cache policy (nt tile loads but the halo tail, nt halo, nt stores)
    assert "nt=13" in p and "nt=13" in dsp.plan(1 << 30, 4096) and "nt=13" in dsp.plan(1 << 30, 64), p
    assert "U=4" in dsp.plan(1 << 30, 4096) and "block=512" in dsp.plan(1 << 30, 4096)
    # multi-channel fp32 frames: the wide-frame tile (chunks of consecutive frames per lane)
    assert dsp.plan(1 << 30, 1024, channels=2).startswith("wide_tile<f32,acc=f64,C=2,P=16,U=1")
    assert dsp.plan(1 << 30, 1024, channels=4).startswith("wide_tile<f32,acc=f64,C=4,P=8,U=1")
    assert dsp.plan(1 << 30, 1024, channels=8).startswith("chan_tile<f32,acc=f64,C=8,Q=32")  # a channel per lane
    assert ",xg=1>" in dsp.plan(1 << 30, 1024, channels=8) and ",xg=1>" not in dsp.plan(1 << 30, 511, channels=8)
    # past the halo-only tile (8 channels k > 1536, 4 channels k > 3584): the halo-only channel-per-lane
    # look-ahead (x from global memory, only the shifted tile in LDS)
    # (round 6: with 16-B frames x comes as whole-frame loads turned into columns, xl=1)
    for C, k in ((8, 1537), (8, 44100), (4, 2561), (4, 3000), (4, 3088), (4, 8192), (4, 44100)):
        p = dsp.plan(1 << 30, k, channels=C)
        assert p.startswith(f"wide_ahead<f32,acc=f64,C={C},P=32") and ",ch=1,xg=1," in p, p
        # 4 channels: self-published records with the columns formed at once (xl=2), phase A with
        # XL at windows of whole 2048-frame tiles (xl=1); 8 channels: phase A, column loads
        want = ",xl=0>" if C == 8 else (",xl=1>" if k % 2048 == 0 else ",xl=2>")
        assert want in p and ((" self=1 " in p) == (want == ",xl=2>")), p
    assert ",xg=1>" in dsp.plan(1 << 30, 1536, channels=8)
    for k in (2048, 2544, 2560, 3072):  # the in-place chan tile (staged halo of exactly k frames),
        p = dsp.plan(1 << 30, k, channels=4)  # with XL while 4 workgroups per CU fit its LDS (160 KiB)
        want = ",xg=1,ip=1,xl=1>" if k <= 2544 else ",xg=1,ip=1>"
        assert p.startswith("chan_tile<f32,acc=f64,C=4,Q=32") and want in p, p
    # int16 8 channels: a dword column (two channels) per lane from a window of one tile on
    i16c8 = lambda k: dsp.plan(1 << 30, k, channels=8, dtype=dsp.I16)
    assert i16c8(1024).startswith("wide_tile<i16") and i16c8(2047).startswith("wide_tile<i16")
    assert i16c8(44100).startswith("wide_ahead<i16,acc=i32,C=8,P=32") and ",ch=1,xg=1," in i16c8(44100)
    for k in (2048, 2049, 3073, 8192, 44100):  # past the wide tile: self-published, columns formed at once
        assert i16c8(k).startswith("wide_ahead<i16,acc=i32,C=8,P=32") and ",xl=2>" in i16c8(k), i16c8(k)
        assert " self=1 " in i16c8(k), i16c8(k)
    # aggregate-first look-ahead records in 32-KiB tiles (round 6): int16 mono / stereo past a
    # 16-KiB halo, int16 4 channels past 64 KiB, fp32 stereo past the wide tile's 32 KiB, short of
    # the L2 reach (int16 mono: k <= 131072); fp32 mono and 8 channels keep their kernels
    agg = lambda p: p.startswith("ahead_scan<") and " self=1 " in p and ",U=8," in p
    i16 = lambda k, C: dsp.plan(1 << 30, k, channels=C, dtype=dsp.I16)
    assert i16(8192, 1).startswith("tile_scan<") and agg(i16(8193, 1)) and agg(i16(131072, 1))
    assert not agg(i16(131073, 1)) and i16(131073, 1).startswith("ahead_scan<")
    assert i16(4096, 2).startswith("tile_scan<") and agg(i16(4097, 2)) and agg(i16(500_000, 2))
    # past the L2 reach: window-matched runs of the same tiles, self-published (int16 mono past
    # k = 2^21: phase A), no run totals up to 1024 tiles per window
    far = lambda p: p.startswith("ahead_scan<") and ",U=8," in p and " remap=1 " not in p and "runs=1" not in p
    assert far(i16(600_000, 2)) and " self=1 " in i16(600_000, 2) and " ahead=320 " in i16(600_000, 2)
    assert far(i16(4_000_000, 2)) and " self=1 " in i16(4_000_000, 2) and " ahead=960 " in i16(4_000_000, 2)
    assert far(i16(1_500_000, 1)) and " self=1 " in i16(1_500_000, 1)
    assert far(i16(4_000_000, 1)) and " self=1 " not in i16(4_000_000, 1)
    for k in (600_000, 1_000_000, 4_000_000, 8_000_000):  # fp32 mono: phase A (bench.py's timing)
        assert far(dsp.plan(1 << 30, k)) and " self=1 " not in dsp.plan(1 << 30, k), k
    assert "runs=1" in dsp.plan(1 << 30, 9_000_000)  # past 1024 tiles: the run-total kernel
    assert i16(8192, 4).startswith("wide_ahead<") and agg(i16(8193, 4)) and agg(i16(100_000, 4))
    assert dsp.plan(1 << 30, 4096, channels=2).startswith("wide_tile<") and agg(dsp.plan(1 << 30, 4097, channels=2))
    assert not agg(dsp.plan(1 << 30, 300_000, channels=2)) and not agg(dsp.plan(1 << 30, 44100))
    assert not agg(i16(44100, 8)) and not agg(dsp.plan(1 << 30, 44100, channels=4))
    assert not agg(dsp.plan(1 << 30, 44100, channels=2, algo="hillis"))
    assert dsp.plan(3 << 28, 1024, channels=3).startswith("tile_scan<f32")  # 12-B frames: frame units
    assert dsp.plan(1 << 30, 1024, channels=2, algo="hillis").startswith("tile_scan<")
    # int16 keeps the register-staged tiles (bench.py's timing, tools/tune/ab_libs.py)
    i16 = lambda k, c=1: dsp.plan(1 << 30, k, channels=c, dtype=dsp.I16)
    for k, c in ((1024, 1), (1023, 1), (1024, 2), (512, 2)):
        assert "U=4" in i16(k, c) and "dma=0" in i16(k, c) and "block=256" in i16(k, c), i16(k, c)
    assert "U=2" in i16(64) and "dma=0" in i16(64), i16(64)
    assert dsp.plan(1 << 20, 70_000).startswith("ahead_scan<f32")
    # Hillis-Steele past its LDS-staged halo: the look-ahead record carry with the HS in-tile scan
    assert dsp.plan(1 << 20, 70_000, algo="hillis").startswith("ahead_scan<f32,acc=f64,C=1,F=4,U=4,hillis")
    assert dsp.plan(1 << 20, 7, algo="direct").startswith("direct<f32")
    assert dsp.plan(1 << 20, 7, algo="naive").startswith("naive<f32")
    assert "hillis" in dsp.plan(1 << 20, 7, algo="hillis_scalar")
    assert dsp.plan(1 << 20, 100_000, dtype=dsp.I16).startswith("ahead_scan<i16,acc=i64")
    assert dsp.plan(3 * 1000, 7, channels=3, dtype=dsp.I16, algo="blelloch").startswith("tile_scan<i16,acc=i32,C=3,F=1")
    with pytest.raises(dsp.MavgError):
        dsp.plan(10, 0)


def test_longest_plan_is_not_truncated():
    """The look-ahead plan with window-matched runs and run totals is the
    longest; its trailing ws= field (tools/tune/ahead_trace.py reads it) must
    be whole."""
    import digital_signal_processsing_amd as dsp
    p = dsp.plan(1 << 30, 10_000_000)  # fp32 mono past 1024 8192-frame tiles: the run-total kernel
    assert "runs=1" in p and re.search(r" ws=\d+$", p), p
    assert 0 < int(p.split(" ws=")[1]) <= dsp.workspace_bytes(1 << 30, 10_000_000), p


def test_workspace_only_for_ahead_scan():
    import digital_signal_processsing_amd as dsp
    # halo-staged tiles need none; the look-ahead scan needs its record
    # granules: 8 bytes per (record, channel, 32-bit word of the tile-sum
    # type), padded to 16 bytes, plus 16 bytes of statistics; a record per
    # whole tile, or per (whole tile, wave) -- 4 per tile -- for mono windows
    # whose records fit one round of loads (WREC)
    assert dsp.workspace_bytes(1 << 30, 1024) == 0
    assert dsp.workspace_bytes(1 << 30, 4096) == 0
    # fp32 halos past 16 KiB take the look-ahead scan (U=4: 4096-frame tiles);
    # the workspace is sized for the frame-unit form too (1024-frame tiles),
    # which a view that is not 16-B aligned may run
    tiles = (1 << 30) // 4096
    assert dsp.plan(1 << 30, 8192).startswith("ahead_scan<f32,acc=f64,C=1,F=4,U=4")
    assert "wrec=1" in dsp.plan(1 << 30, 20_000) and "ws=%d" % (tiles * 4 * 2 * 8 + 16) in dsp.plan(1 << 30, 20_000)
    assert "wrec=0" in dsp.plan(1 << 30, 300_000) and "ws=%d" % (tiles * 2 * 8 + 16) in dsp.plan(1 << 30, 300_000)
    # past the L2 reach (window-matched runs): 8192-frame tiles (U=8), one record per tile
    for k in (600_000, 4_000_000):
        p = dsp.plan(1 << 30, k)
        assert "U=8" in p and "wrec=0" in p and "ws=%d" % (tiles // 2 * 2 * 8 + 16) in p, p
    assert dsp.plan(1 << 30, 8192, algo="blelloch_scalar").startswith("ahead_scan<f32,acc=f64,C=1,F=1,U=4")
    assert dsp.workspace_bytes(1 << 30, 8192) == 4 * tiles * 4 * 2 * 8 + 16
    assert dsp.workspace_bytes(1 << 30, 8192, algo="blelloch_scalar") == 4 * tiles * 4 * 2 * 8 + 16
    assert dsp.plan(1 << 30, 8192, algo="hillis").startswith("ahead_scan<") and "hillis" in dsp.plan(
        1 << 30, 8192, algo="hillis")
    # int16 mono keeps the tiles up to 16 KiB of halo (past it: the aggregate-first look-ahead)
    assert dsp.workspace_bytes(1 << 30, 8192, dtype=dsp.I16) == 0
    n = 2 * 1_000_003
    st = (n // 2) // 1024     # int16 stereo, frame-unit tiles: one int32 word per (whole tile, channel)
    assert dsp.workspace_bytes(n, 44100, 2, dsp.I16) == (st * 2 * 8 + 15) // 16 * 16 + 16
    assert dsp.workspace_bytes(1 << 20, 70_000, algo="hillis") == dsp.workspace_bytes(1 << 20, 70_000)
    assert dsp.workspace_bytes(0, 70_000) == 0


def test_ahead_scan_without_workspace_is_an_error():
    lib = _lib.load()
    # plan mode is not used here: a real call with dummy aligned pointers must
    # refuse before touching the device when the workspace is missing
    st = lib.mavg_run(1 << 20, 1 << 21, 1 << 20, 1, 70_000, _lib.F32, _lib.ALGO_BLELLOCH, 0, None, None, 0, None)
    assert st == _lib.ERR_WORKSPACE


def test_auto_picks_the_tile_scan_at_every_window():
    import digital_signal_processsing_amd as dsp
    for k in (1, 7, 9, 10, 1024, 100_000):
        assert dsp.resolve_algo(1 << 20, k) == "blelloch", k
    assert dsp.plan(1 << 20, 7, algo="direct").startswith("direct<")


def test_many_channels_auto_resolves_to_naive():
    import digital_signal_processsing_amd as dsp
    assert dsp.resolve_algo(16 * 100, 5, channels=16) == "naive"
    assert dsp.plan(16 * 100, 5, channels=16).startswith("naive<")


@pytest.mark.parametrize("algo,block,want", [
    ("blelloch", 512, "block=512"), ("blelloch", 256, "block=256"), ("blelloch", 1024, "block=1024"),
    ("blelloch", 32, "block=64"), ("blelloch", 96, "block=128"), ("blelloch", 128, "block=128"),
    ("hillis", 64, "block=64"), ("blelloch_scalar", 512, "block=512"), ("hillis_scalar", 1024, "block=1024"),
    ("direct", 128, "block=128"), ("direct_vec2", 1024, "block=1024"), ("direct_scalar", 64, "block=64"),
    ("naive", 96, "block=96"), ("naive", 32, "block=32"), ("naive", 0, "block=256"),
])
def test_block_size_sets_the_workgroup(algo, block, want):
    """The reference launches its kernels with the argv block size
    (blelloch_scan_averager.cu:155,215-217); here the naive kernel runs it
    exactly and the tiled kernels run the next power of two >= one wave64."""
    import digital_signal_processsing_amd as dsp
    p = dsp.plan(1 << 20, 64, algo=algo, block_size=block)
    assert re.search(r"block=\d+", p).group(0) == want, p


def test_block_size_tuned_and_fallback_geometry():
    import digital_signal_processsing_amd as dsp
    assert dsp.plan(1 << 20, 1024, block_size=0) == dsp.plan(1 << 20, 1024)
    # U=2 tiles at the requested workgroup: 64 threads x 4 frames x 2
    assert "tile_frames=512" in dsp.plan(1 << 20, 64, algo="blelloch", block_size=64)
    # a window whose halo does not fit the requested workgroup's LDS keeps the tuned launch
    assert dsp.plan(1 << 20, 70_000, block_size=512) == dsp.plan(1 << 20, 70_000)
    assert dsp.plan(1 << 20, 70_000, block_size=512).startswith("ahead_scan<")
    with pytest.raises(dsp.MavgError):
        dsp.plan(1 << 20, 64, block_size=48)


def test_workspace_error_on_misaligned_view_queues_nothing():
    """A view 4 B past 16-B alignment peels a 3-frame head (frame-unit form)
    before the vector body.  A workspace that covers the head's look-ahead
    launch (32 B) but not the body's must be refused before anything is
    queued: both launches are planned first (mavg.h)."""
    lib = _lib.load()
    din, dout, ws = (1 << 20) + 4, (1 << 21) + 4, 1 << 22
    st = lib.mavg_run(din, dout, 1 << 20, 1, 70_000, _lib.F32, _lib.ALGO_BLELLOCH, 0, None, ws, 32, None)
    assert st == _lib.ERR_WORKSPACE


def test_direct_block_size_falls_back_when_the_halo_does_not_fit():
    import digital_signal_processsing_amd as dsp
    # fp32 mono k=13000: a 1024-thread direct tile would need > 64 KiB of LDS;
    # the tuned 2-unit x 256-thread launch runs instead
    p = dsp.plan(1 << 20, 13_000, algo="direct", block_size=1024)
    assert p == dsp.plan(1 << 20, 13_000, algo="direct") and "U=2" in p and "block=256" in p, p
    assert "block=1024" in dsp.plan(1 << 20, 1000, algo="direct", block_size=1024)
