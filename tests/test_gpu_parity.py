"""GPU parity: libmavg (HIP, gfx950) against the CPU oracle on the same seeded
inputs.  int16 results must be bit-exact with the serial reference semantics
(basics/profilable_moving_averager.cpp:14-37); fp32 results must be within
RTOL relative of the fp64 restatement (BASELINE.json north_star: 1e-5)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north_star: "within 1e-5 relative fp32"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

ALL_ALGOS = ["blelloch", "blelloch_scalar", "hillis", "hillis_scalar", "direct", "direct_vec2",
             "direct_scalar", "naive"]


def _dev(x, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(gpu)


def _run(x_np, k, C, algo, gpu, history=None, library=None):
    import digital_signal_processsing_amd as dsp
    x = _dev(x_np, gpu)
    h = _dev(history, gpu) if history is not None else None
    y = dsp.moving_average(x, k, channels=C, algo=algo, history=h, library=library)
    return y.cpu().numpy()


def assert_f32_close(y, r, what=""):
    err = np.abs(y.astype(np.float64) - r.astype(np.float64))
    tol = RTOL * np.maximum(np.abs(r.astype(np.float64)), 1e-30)
    bad = np.nonzero(err > tol)[0]
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first at {bad[:5]}: got {y[bad[:5]]} want {r[bad[:5]]}"


# ---------------------------------------------------------------------------
def test_device_synth_matches_oracle(oracle_mod, gpu):
    import digital_signal_processsing_amd as dsp
    import torch
    n = 100_003
    for dist in (0, 1, 2):
        y = dsp.fill_synthetic(n, torch.float32, seed=0x5EED, offset=999, dist=dist, device=gpu)
        assert np.array_equal(y.cpu().numpy().view(np.uint32),
                              oracle_mod.synth_f32(n, seed=0x5EED, offset=999, dist=dist).view(np.uint32)), dist
    y = dsp.fill_synthetic(n, torch.int16, seed=7, offset=3, device=gpu)
    assert np.array_equal(y.cpu().numpy(), oracle_mod.synth_i16(n, seed=7, offset=3))


@pytest.mark.parametrize("algo", ALL_ALGOS)
@pytest.mark.parametrize("C", [1, 2])
def test_golden_fixtures_i16(oracle_mod, gpu, algo, C):
    g = np.load(os.path.join(GOLDEN, "mavg_golden.npz"))
    x = oracle_mod.synth_i16(4096 * C, seed=0x5EED)
    for k in (1, 3, 7, 32, 41, 64, 1000, 1024):
        y = _run(x, k, C, algo, gpu)
        assert np.array_equal(y, g[f"i16_C{C}_k{k}"]), f"{algo} C={C} k={k}"


@pytest.mark.parametrize("algo", ALL_ALGOS)
@pytest.mark.parametrize("C", [1, 2])
def test_golden_fixtures_f32(oracle_mod, gpu, algo, C):
    g = np.load(os.path.join(GOLDEN, "mavg_golden.npz"))
    x = oracle_mod.synth_f32(4096 * C, seed=0x5EED, dist=1)
    for k in (1, 3, 7, 32, 41, 64, 1000, 1024):
        assert_f32_close(_run(x, k, C, algo, gpu), g[f"f32u_C{C}_k{k}"], f"{algo} C={C} k={k}")


# sizes: tiny, ragged (not multiples of any chunk / vector), multi-segment
SIZES = [1, 5, 63, 1000, 4097, 65_537, 1_000_003]
SCAN_ALGOS = ["blelloch", "blelloch_scalar", "hillis", "hillis_scalar"]


@pytest.mark.parametrize("algo", SCAN_ALGOS + ["direct", "naive"])
@pytest.mark.parametrize("frames", SIZES)
def test_ragged_sizes_i16(oracle_mod, gpu, algo, frames):
    for C, k in ((1, 1), (1, 7), (1, 1024), (2, 64), (2, 41)):
        if algo == "naive" and frames * k > 50_000_000:
            continue
        x = oracle_mod.synth_i16(frames * C, offset=frames + k)
        y = _run(x, k, C, algo, gpu)
        assert np.array_equal(y, oracle_mod.mavg_i16(x, k, C)), f"{algo} frames={frames} C={C} k={k}"


@pytest.mark.parametrize("algo", SCAN_ALGOS + ["direct"])
@pytest.mark.parametrize("frames", SIZES)
def test_ragged_sizes_f32(oracle_mod, gpu, algo, frames):
    for C, k, dist in ((1, 1, 0), (1, 7, 1), (1, 1024, 0), (1, 4096, 1), (2, 64, 1), (4, 3, 0)):
        x = oracle_mod.synth_f32(frames * C, offset=frames + k, dist=dist)
        assert_f32_close(_run(x, k, C, algo, gpu), oracle_mod.mavg_f32(x, k, C),
                         f"{algo} frames={frames} C={C} k={k} dist={dist}")


# fp32 rounding data (dist 2: zero-mean, mixed-scale, non-dyadic; its fp64
# window sums round) against the EXACT window sum, every algorithm and kernel
# family: the 1e-5 relative bar, with the floor 1e-5 * (window's mean |x|)
# for outputs whose sum cancels to ~0, and the error beyond the fp32 output
# rounding held under 1e-9 of that scale (oracle.check_synth_exact)
ROUNDING_CASES = [  # frames, C, k
    (1, 1, 1), (63, 1, 7), (4097, 2, 41), (65_537, 1, 1024), (100_003, 1, 4096), (300_007, 1, 20_000),
    (300_007, 2, 44_100), (200_003, 3, 333), (1_000_003, 1, 70_000)]


@pytest.mark.parametrize("algo", ALL_ALGOS)
def test_rounding_data_against_exact_sums(oracle_mod, gpu, algo):
    import digital_signal_processsing_amd as dsp
    import torch
    for frames, C, k in ROUNDING_CASES:
        if algo == "naive" and frames * k > 50_000_000:
            continue
        if algo.startswith("direct") and k > 5000:
            continue  # the direct kernel's LDS halo (its reference is a small-window path)
        x = dsp.fill_synthetic(frames * C, torch.float32, dist=2, device=gpu)
        y = dsp.moving_average(x, k, channels=C, algo=algo).cpu().numpy()
        r = oracle_mod.check_synth_exact(y, k, C, dist=2, rtol=RTOL)
        assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (algo, frames, C, k, r)


@pytest.mark.parametrize("C", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("dtype", ["i16", "f32"])
def test_all_channel_counts(oracle_mod, gpu, C, dtype):
    frames = 20_011
    for algo in ("blelloch", "hillis_scalar", "direct", "naive"):
        for k in (1, 5, 333):
            if dtype == "i16":
                x = oracle_mod.synth_i16(frames * C, offset=C * 1000 + k)
                assert np.array_equal(_run(x, k, C, algo, gpu), oracle_mod.mavg_i16(x, k, C)), (algo, C, k)
            else:
                x = oracle_mod.synth_f32(frames * C, offset=C * 1000 + k, dist=1)
                assert_f32_close(_run(x, k, C, algo, gpu), oracle_mod.mavg_f32(x, k, C), f"{algo} C={C} k={k}")


@pytest.mark.parametrize("k", [2, 3, 5, 6, 7, 9, 13, 4093, 4097, 20_000, 70_000])
def test_unaligned_and_large_windows(oracle_mod, gpu, k):
    """x[n-k] not 16-B aligned inside the LDS ring; k too large for the ring
    (global re-read path); int16 k > 65535 (int64 accumulation)."""
    frames = 300_007
    for C in (1, 2):
        x = oracle_mod.synth_i16(frames * C, offset=k)
        for algo in ("blelloch", "hillis"):
            assert np.array_equal(_run(x, k, C, algo, gpu), oracle_mod.mavg_i16(x, k, C)), (algo, C, k)
        xf = oracle_mod.synth_f32(frames * C, offset=k, dist=1)
        assert_f32_close(_run(xf, k, C, "blelloch", gpu), oracle_mod.mavg_f32(xf, k, C), f"C={C} k={k}")


@pytest.mark.parametrize("algo", ["blelloch", "blelloch_scalar", "hillis", "direct", "direct_scalar", "naive"])
@pytest.mark.parametrize("dtype", ["i16", "f32"])
def test_history_equals_concatenation(oracle_mod, gpu, algo, dtype):
    """Sharding contract: running on x[a:] with the (k-1)*C preceding samples
    as history equals the tail of running on the whole signal."""
    C, k, frames, cut = 2, 300, 50_000, 17_001
    if dtype == "i16":
        x = oracle_mod.synth_i16(frames * C, offset=11)
        full = oracle_mod.mavg_i16(x, k, C)
    else:
        x = oracle_mod.synth_f32(frames * C, offset=11, dist=1)
        full = oracle_mod.mavg_f32(x, k, C)
    hist = x[(cut - (k - 1)) * C: cut * C]
    y = _run(x[cut * C:], k, C, algo, gpu, history=hist)
    if dtype == "i16":
        assert np.array_equal(y, full[cut * C:])
    else:
        assert_f32_close(y, full[cut * C:], algo)


def test_properties_identity_constant_linearity(oracle_mod, gpu):
    import digital_signal_processsing_amd as dsp
    import torch
    n = 1 << 20
    x = dsp.fill_synthetic(n, torch.int16, seed=3, device=gpu)
    assert torch.equal(dsp.moving_average(x, 1), x)                                  # k=1 identity
    c = torch.full((n,), -1234, dtype=torch.int16, device=gpu)
    y = dsp.moving_average(c, 777)
    assert (y[776:] == -1234).all()                                                   # constant from k-1 on
    a = dsp.fill_synthetic(n, torch.float32, seed=4, device=gpu)
    b = dsp.fill_synthetic(n, torch.float32, seed=5, device=gpu)
    ya, yb, yab = dsp.moving_average(a, 100), dsp.moving_average(b, 100), dsp.moving_average(a + 2 * b, 100)
    torch.testing.assert_close(yab, ya + 2 * yb, rtol=1e-5, atol=1e-3)               # linearity


def test_checksum_of_checksums_repeatability(gpu):
    """Same input, repeated launches: the output is deterministic bit-for-bit."""
    import digital_signal_processsing_amd as dsp
    import torch
    x = dsp.fill_synthetic(1 << 26, torch.float32, seed=9, device=gpu)
    h = None
    for _ in range(3):
        y = dsp.moving_average(x, 64)
        d = torch.sum(y.view(torch.int32).to(torch.int64) * 2654435761 % (1 << 31)).item()
        assert h is None or d == h
        h = d


@pytest.mark.parametrize("C,k,dtype", [(1, 1024, "f32"), (2, 41, "i16"), (1, 1, "f32"), (1, 4096, "f32"),
                                       (2, 70, "f32"), (1, 9000, "f32"), (1, 30_000, "f32"), (2, 20_000, "i16")])
def test_sharded_split_launch_equals_whole_signal(oracle_mod, gpu, C, k, dtype):
    """The multi-GPU step on one GPU: every shard filtered as interior launch +
    head launch with the previous shard's tail as history (what rank r does
    after the RCCL halo arrives) reproduces the whole-signal output."""
    import torch
    from digital_signal_processsing_amd.shard import shard_bounds, split_moving_average_into
    frames, world = 300_001, 4
    if dtype == "i16":
        x = oracle_mod.synth_i16(frames * C, offset=k)
        full = oracle_mod.mavg_i16(x, k, C)
    else:
        x = oracle_mod.synth_f32(frames * C, offset=k, dist=1)
        full = oracle_mod.mavg_f32(x, k, C)
    xd = torch.from_numpy(x).to(gpu)
    out = torch.empty_like(xd)
    for r in range(world):
        f0, f1 = shard_bounds(frames, world, r)
        hist = xd[(f0 - (k - 1)) * C: f0 * C] if (r > 0 and k > 1) else None
        # views straight into the whole signal: shards cut at any frame, so
        # neither the shard nor its history is 16-B aligned in general
        split_moving_average_into(xd[f0 * C: f1 * C], out[f0 * C: f1 * C], k, C, "blelloch", history=hist)
    y = out.cpu().numpy()
    if dtype == "i16":
        assert np.array_equal(y, full)
    else:
        assert_f32_close(y, full, f"C={C} k={k}")


def test_graph_capture_and_stream_semantics(oracle_mod, gpu):
    """mavg_run only enqueues on the caller's stream: it can be captured into a
    HIP graph and replayed, and it runs on a non-default stream."""
    import torch
    import digital_signal_processsing_amd as dsp
    n, k = 1 << 22, 1024
    xf = oracle_mod.synth_f32(n, seed=21, dist=1)
    ref = oracle_mod.mavg_f32(xf, k, 1)
    x = torch.from_numpy(xf).to(gpu)
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        dsp.moving_average_into(x, y, k)          # warm-up on a side stream
    s.synchronize()
    assert_f32_close(y.cpu().numpy(), ref, "side stream")
    y.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dsp.moving_average_into(x, y, k)
    g.replay()
    torch.cuda.synchronize()
    assert_f32_close(y.cpu().numpy(), ref, "graph replay")
    x.copy_(torch.from_numpy(oracle_mod.synth_f32(n, seed=22, dist=1)).to(gpu))
    g.replay()                                     # replay reads the new input in place
    torch.cuda.synchronize()
    assert_f32_close(y.cpu().numpy(), oracle_mod.mavg_f32(oracle_mod.synth_f32(n, seed=22, dist=1), k, 1), "replay 2")


@pytest.mark.parametrize("dtype,C,k", [("f32", 1, 1024), ("i16", 1, 1024), ("i16", 2, 700), ("f32", 1, 4096),
                                       ("i16", 1, 3000)])
def test_grouped_xcd_remap_with_tail(oracle_mod, gpu, dtype, C, k):
    """Tile counts just past a multiple of 8*64: the grouped tile->XCD mapping
    covers the full groups and the tail maps to itself; every tile must be
    written exactly once with the right halo."""
    import digital_signal_processsing_amd as dsp
    plan = dsp.plan(1 << 20, k, C, dsp.F32 if dtype == "f32" else dsp.I16)
    tile = int(plan.split("tile_frames=")[1].split()[0])
    frames = tile * (2 * 512 + 37) + 5
    if dtype == "f32":
        x = oracle_mod.synth_f32(frames * C, offset=99, dist=1)
        assert_f32_close(_run(x, k, C, "auto", gpu), oracle_mod.mavg_f32(x, k, C), plan)
    else:
        x = oracle_mod.synth_i16(frames * C, offset=99)
        assert np.array_equal(_run(x, k, C, "auto", gpu), oracle_mod.mavg_i16(x, k, C)), plan


@pytest.mark.parametrize("dtype,C,k,algo", [("f32", 1, 600_000, "auto"), ("i16", 2, 1_000_000, "auto"),
                                            ("f32", 1, 4_000_000, "auto"), ("f32", 4, 300_000, "auto"),
                                            ("f32", 1, 700_000, "hillis"), ("f32", 1, 2_000_000, "auto"),
                                            ("i16", 2, 1_700_000, "auto"), ("i16", 1, 1_500_000, "auto"),
                                            ("f32", 1, 9_000_000, "auto"), ("i16", 1, 3_500_000, "auto")])
def test_period_remap_very_long_windows_with_tail(oracle_mod, gpu, dtype, C, k, algo):
    """Windows past the L2 reach: the look-ahead scan runs in window-matched
    runs of G tiles per XCD (remap mode G, 8JG ~ k/T, G not a power of two:
    remap_tile's divide path) and its carry reads run totals for the whole
    runs inside the window (runs=1); more than a window and three periods,
    and a ragged tail past them (blocks mapped to themselves), every output
    against the oracle, and bitwise the same output when every record and run
    total is recomputed by its consumer or the look-ahead is cut to 0 / 8."""
    import digital_signal_processsing_amd as dsp
    code = dsp.F32 if dtype == "f32" else dsp.I16
    plan = dsp.plan(1 << 30, k, C, code, algo)
    G = int(plan.split("remap=")[1].split()[0])
    tile = int(plan.split("tile_frames=")[1].split()[0])
    assert _is_long(plan) and G > 1, plan
    # run totals: the 4096-frame (int16 mono: 8192-frame) U=4 kernel past 384 tiles; fp32 mono and
    # int16 stereo take 8192-frame tiles (U=8) without them short of that kernel's range
    assert ("runs=1" in plan) == (C <= 2 and algo == "auto" and k > 384 * tile and plan.startswith("ahead_scan<")
                                  and "U=8" not in plan), plan
    frames = tile * max(3 * 8 * G + 37, k // tile + 8 * G + 37) + 5  # past one window, 3 periods, a ragged tail
    assert int(dsp.plan(frames * C, k, C, code, algo).split("remap=")[1].split()[0]) == G
    if dtype == "f32":
        x = oracle_mod.synth_f32(frames * C, dist=2)  # offset 0: the checker's stream starts at the signal's start
        base = _run(x, k, C, algo, gpu)
        r = oracle_mod.check_synth_exact(base, k, C, dist=2)
        assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (plan, r)
    else:
        x = oracle_mod.synth_i16(frames * C, offset=77)
        base = _run(x, k, C, algo, gpu)
        assert np.array_equal(base, oracle_mod.mavg_i16(x, k, C)), plan
    for sched in ({}, {"spin": 0}, {"slots": 0}, {"slots": 8, "spin": 0}):
        # the forced schedule keeps the plan's runs (G) and run-total grouping
        p = _with_schedule(sched, lambda lib: dsp.plan(frames * C, k, C, code, algo, library=lib))
        assert int(p.split("remap=")[1].split()[0]) == G and ("runs=1" in p) == ("runs=1" in plan), (sched, p)
        y = _with_schedule(sched, lambda lib: _run(x, k, C, algo, gpu, library=lib))
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), sched


def test_many_channels_auto(oracle_mod, gpu):
    """C > 8 (beyond the templated kernels): AUTO runs the naive any-C kernel."""
    for C, dtype in ((12, "i16"), (16, "f32")):
        if dtype == "i16":
            x = oracle_mod.synth_i16(3001 * C, offset=C)
            assert np.array_equal(_run(x, 37, C, "auto", gpu), oracle_mod.mavg_i16(x, 37, C))
        else:
            x = oracle_mod.synth_f32(3001 * C, offset=C, dist=1)
            assert_f32_close(_run(x, 37, C, "auto", gpu), oracle_mod.mavg_f32(x, 37, C), "C=16")


# ---------------------------------------------------------------------------
# the long-window scans: the look-ahead scan (mavg_lookback.hpp: whole-tile
# records published inside the launch) and, for multi-channel fp32 frames, the
# wide look-ahead scan (mavg_wide.hpp: the same record carry, the wide in-tile
# scan)
LONG_KERNELS = ("ahead_scan", "wide_ahead")


def _is_long(plan):
    return plan.split("<")[0] in LONG_KERNELS


def _lookback_tile(dsp, n, k, C, dt):
    plan = dsp.plan(n, k, C, dt)
    assert _is_long(plan), plan
    return int(plan.split("tile_frames=")[1].split()[0])


@pytest.mark.parametrize("C", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dtype", ["i16", "f32"])
def test_ahead_window_edges(oracle_mod, gpu, C, dtype):
    """k just below / at / above multiples of the tile (empty, one-frame and
    full partial pieces), windows spanning many tiles, int16 k > 65535, and a
    ragged tail tile."""
    import digital_signal_processsing_amd as dsp
    dt = dsp.F32 if dtype == "f32" else dsp.I16
    frames = 200_003
    T = _lookback_tile(dsp, frames * C, 70_001, C, dt)
    for k in sorted({16 * T - 1, 16 * T, 16 * T + 1, 20_000, 44_100, 70_001}):
        if not _is_long(dsp.plan(frames * C, k, C, dt)):
            continue
        if dtype == "i16":
            x = oracle_mod.synth_i16(frames * C, offset=k + C)
            assert np.array_equal(_run(x, k, C, "blelloch", gpu), oracle_mod.mavg_i16(x, k, C)), (C, k)
        else:
            x = oracle_mod.synth_f32(frames * C, offset=k + C, dist=1)
            assert_f32_close(_run(x, k, C, "blelloch", gpu), oracle_mod.mavg_f32(x, k, C), f"C={C} k={k}")


@pytest.mark.parametrize("frames", [1, 777, 44_099, 44_100, 44_101, 100_000])
def test_ahead_short_signals(oracle_mod, gpu, frames):
    """Signals shorter than (or about as long as) the window: every tile's
    window reaches before frame 0."""
    k, C = 44_100, 2
    x = oracle_mod.synth_i16(frames * C, offset=frames)
    assert np.array_equal(_run(x, k, C, "auto", gpu), oracle_mod.mavg_i16(x, k, C))
    xf = oracle_mod.synth_f32(frames * C, offset=frames, dist=1)
    assert_f32_close(_run(xf, k, C, "auto", gpu), oracle_mod.mavg_f32(xf, k, C), f"frames={frames}")


@pytest.mark.parametrize("dtype", ["i16", "f32"])
@pytest.mark.parametrize("cut", [5_000, 37_001])
def test_ahead_history_equals_concatenation(oracle_mod, gpu, dtype, cut):
    """History with a long window: the part of the window before frame 0 comes
    from the history buffer (cut < k: the window also reaches before it)."""
    C, k, frames = 2, 20_000, 120_000
    if dtype == "i16":
        x = oracle_mod.synth_i16(frames * C, offset=5)
        full = oracle_mod.mavg_i16(x, k, C)
    else:
        x = oracle_mod.synth_f32(frames * C, offset=5, dist=1)
        full = oracle_mod.mavg_f32(x, k, C)
    lo = max(0, cut - (k - 1))
    hist = np.zeros((k - 1) * C, dtype=x.dtype)
    hist[(k - 1 - (cut - lo)) * C:] = x[lo * C: cut * C]
    y = _run(x[cut * C:], k, C, "blelloch", gpu, history=hist)
    if dtype == "i16":
        assert np.array_equal(y, full[cut * C:])
    else:
        assert_f32_close(y, full[cut * C:], f"cut={cut}")


def test_int64_division_edges(oracle_mod, gpu):
    """k > 65535 (int64 window sums): extreme constant signals make k divide
    the window sum exactly in the steady state and at many warm-up frames --
    the case the fp64 quotient estimate has to correct."""
    for k in (65_536, 70_001, 131_072):
        for c in (-32768, 32767, -1, 12345):
            x = np.full(300_000, c, dtype=np.int16)
            y = _run(x, k, 1, "auto", gpu)
            assert np.array_equal(y, oracle_mod.mavg_i16(x, k, 1)), (k, c)
            assert (y[k - 1:] == c).all()
        x = oracle_mod.synth_i16(2 * 250_000, offset=k)
        assert np.array_equal(_run(x, k, 2, "auto", gpu), oracle_mod.mavg_i16(x, k, 2)), k


# the refused capture (own_workspace=False) ends an empty graph: torch warns
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
@pytest.mark.parametrize("own_workspace", [True, False])
def test_ahead_graph_capture(oracle_mod, gpu, own_workspace):
    """The granule reset and the look-ahead launch replay correctly from a
    captured HIP graph, repeatedly, with a caller-owned workspace; without one
    the binding refuses inside a capture (no workspace from the capture's
    private pool, which is freed again before the capture ends)."""
    import digital_signal_processsing_amd as dsp
    import torch
    n, k = 1_000_003, 30_000
    x = torch.from_numpy(oracle_mod.synth_f32(n, seed=23, dist=1)).to(gpu)
    y = torch.empty_like(x)
    assert _is_long(dsp.plan(n, k))
    ws = torch.empty(dsp.workspace_bytes(n, k), dtype=torch.uint8, device=gpu) if own_workspace else None
    s = torch.cuda.Stream(device=gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(s):
        dsp.moving_average_into(x, y, k, workspace=ws)  # warm-up outside capture
    torch.cuda.current_stream(gpu).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    if not own_workspace:
        # the binding refuses to take a workspace from the capture's pool
        with pytest.raises(ValueError, match="workspace="):
            with torch.cuda.graph(g):
                dsp.moving_average_into(x, y, k)
        return
    with torch.cuda.graph(g):
        dsp.moving_average_into(x, y, k, workspace=ws)
    ref = oracle_mod.mavg_f32(oracle_mod.synth_f32(n, seed=23, dist=1), k, 1)
    for i in range(3):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert_f32_close(y.cpu().numpy(), ref, f"replay {i}")


def test_ahead_large_stereo_slices(oracle_mod, gpu):
    """2^27 int16 stereo samples, one-second window at 44.1 kHz (k=44100):
    bit-exact at random slices, the first tiles and the tail."""
    import digital_signal_processsing_amd as dsp
    import torch
    C, k, seed = 2, 44_100, 0x5EED
    n = 1 << 27
    x = dsp.fill_synthetic(n, torch.int16, seed=seed, device=gpu)
    y = dsp.moving_average(x, k, channels=C).cpu().numpy()
    del x
    frames = n // C
    rng = np.random.default_rng(1)
    span = 3000
    starts = [0, 2048, 44_000, frames - span] + list(rng.integers(0, frames - span, 40))
    for s in starts:
        s = int(s)
        a = max(0, s - k + 1)
        xs = oracle_mod.synth_i16((s + span - a) * C, seed=seed, offset=a * C)
        ref = oracle_mod.mavg_i16(xs, k, C)[(s - a) * C:]
        assert np.array_equal(y[s * C:(s + span) * C], ref), f"slice at frame {s}"


def _with_schedule(sched, fn, debug=False):
    """fn(library) under a forced look-ahead schedule: the schedule hook
    (mavg_test_ahead_schedule, include/mavg_debug.h) is not in the release
    build, so fn runs on lib/libmavg_hooks.so (release flags + the hook: the
    release code's recompute and one-pass paths) or, with debug=True, on
    lib/libmavg_debug.so (the same hook with the device bounds checks); the
    callers compare its output bitwise with the release build's default
    schedule."""
    from digital_signal_processsing_amd import _lib
    path = _lib.DEBUG_LIB_PATH if debug else _lib.HOOKS_LIB_PATH
    lib = _lib.load(path)
    lib.mavg_test_ahead_schedule(sched.get("slots", -1), sched.get("spin", -1))
    try:
        return fn(path)
    finally:
        lib.mavg_test_ahead_schedule(-1, -1)


@pytest.mark.parametrize("dtype,C,k", [("f32", 1, 20_000), ("f32", 3, 9_000), ("i16", 2, 44_100),
                                       ("i16", 1, 100_000), ("f32", 1, 300_000), ("f32", 2, 600_000),
                                       ("f32", 1, 1_100_000), ("i16", 1, 2_200_000),
                                       ("i16", 8, 5_000), ("i16", 8, 44_100), ("i16", 4, 44_100),
                                       ("i16", 2, 600_000), ("i16", 1, 1_500_000)])
def test_ahead_records_bitwise_whatever_the_schedule(oracle_mod, gpu, dtype, C, k):
    """Every record is the same bits whether its producer published it (look-
    ahead D slots, head duty, own tile) or the consumer recomputed it after a
    bounded wait: forcing the recompute path (SPIN=0), the one-pass form
    (SLOTS=0: every tile publishes only its own records), minimal and absent
    look-ahead gives bitwise the same output as the default schedule, also for
    fp32 data whose sums round and cancel (dist 2), and it matches the exact
    window sums (fp32) / the oracle (int16).  Signal lengths give ragged XCD
    runs (tiles not a multiple of 8)."""
    import digital_signal_processsing_amd as dsp
    dt = dsp.F32 if dtype == "f32" else dsp.I16
    frames = 2_600_000 // C + 12_345  # > D = 512 tiles at C=1: the look-ahead producers run
    plan = dsp.plan(frames * C, k, C, dt)
    tf = int(plan.split("tile_frames=")[1].split()[0])
    D = int(plan.split(" ahead=")[1].split()[0])
    if frames < (D + 64) * tf:  # 8192-frame tiles: more than D + 64 of them
        frames = (D + 64) * tf + 12_345
        plan = dsp.plan(frames * C, k, C, dt)
    assert _is_long(plan), plan
    if plan.startswith("ahead_scan<"):
        # int16 mono windows whose per-wave records fit one round of loads take the
        # per-wave records (wrec=1); the others (fp32 mono 8192-frame tiles past
        # the self-published range, multi-channel) one record per tile
        assert ("wrec=1" in plan) == (C == 1 and "U=8" not in plan and k // tf + 1 <= 64), plan
    if dtype == "f32":
        x = oracle_mod.synth_f32(frames * C, seed=77, dist=2)
    else:
        x = oracle_mod.synth_i16(frames * C, seed=77)
    base = _run(x, k, C, "auto", gpu)
    for sched in ({}, {"spin": 0}, {"slots": 0}, {"slots": 8}, {"slots": 1 << 28}, {"slots": 8, "spin": 0}):
        y = _with_schedule(sched, lambda lib: _run(x, k, C, "auto", gpu, library=lib))
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), sched
    # one pass through the debug build: the recompute path under its device bounds checks
    y = _with_schedule({"slots": 8, "spin": 0}, lambda lib: _run(x, k, C, "auto", gpu, library=lib), debug=True)
    assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), "debug build"
    if dtype == "f32":
        r = oracle_mod.check_synth_exact(base, k, C, seed=77, dist=2, rtol=RTOL)
        assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, r
    else:
        assert np.array_equal(base, oracle_mod.mavg_i16(x, k, C))


@pytest.mark.parametrize("C,k,dt", [(1, 20_000, "f32"), (1, 70_000, "f32"), (2, 44_100, "i16"), (1, 100_000, "i16"),
                                    (3, 9_000, "f32")])
def test_hillis_long_windows_through_the_record_carry(oracle_mod, gpu, C, k, dt):
    """hillis / hillis_scalar past the LDS-staged halo run the look-ahead
    scan's record carry with the Hillis-Steele in-tile scan: int16 bit-exact,
    fp32 rounding data (dist 2) within the bar against the exact sums, and
    bitwise the same under a forced recompute schedule."""
    import digital_signal_processsing_amd as dsp
    import torch
    frames = 900_007
    dtc = dsp.F32 if dt == "f32" else dsp.I16
    for algo in ("hillis", "hillis_scalar"):
        plan = dsp.plan(frames * C, k, C, dtc, algo)
        assert plan.startswith("ahead_scan<") and "hillis" in plan, plan
        if dt == "f32":
            x = dsp.fill_synthetic(frames * C, torch.float32, seed=31, dist=2, device=gpu)
        else:
            x = dsp.fill_synthetic(frames * C, torch.int16, seed=31, device=gpu)
        y = dsp.moving_average(x, k, channels=C, algo=algo).cpu().numpy()
        y0 = _with_schedule({"spin": 0, "slots": 0},
                            lambda lib: dsp.moving_average(x, k, channels=C, algo=algo, library=lib).cpu().numpy())
        assert np.array_equal(y.view(np.uint8), y0.view(np.uint8)), algo
        r = oracle_mod.check_synth(y, k, C, seed=31, dist=2 if dt == "f32" else 0, rtol=RTOL)
        assert r["mismatches"] == 0, (algo, r)


@pytest.mark.parametrize("k", [4_097, 5_000, 8_191, 8_192, 8_193, 12_288])
def test_self_published_records(oracle_mod, gpu, k):
    """fp32 mono windows of at most 3 tiles run the look-ahead scan with
    self-published records (no phase A; every tile publishes its own record,
    the carry reads the records after the in-tile scan): every output of
    rounding data (dist 2) within the bar against the exact window sums,
    bitwise the same under forced recompute and absent look-ahead, with a
    ragged tail, and with a history (the window reaching before frame 0)."""
    import digital_signal_processsing_amd as dsp
    frames = 3_000_017  # > 700 tiles: ragged XCD runs, head duty, many consumers per record
    plan = dsp.plan(frames, k, 1, dsp.F32)
    assert plan.startswith("ahead_scan<") and "self=1" in plan and "wrec=1" in plan, plan
    assert "self=1" not in dsp.plan(frames, k, 1, dsp.F32, "hillis")
    x = oracle_mod.synth_f32(frames, seed=91, dist=2)
    base = _run(x, k, 1, "auto", gpu)
    for sched in ({}, {"spin": 0}, {"slots": 0}, {"slots": 8, "spin": 0}):
        y = _with_schedule(sched, lambda lib: _run(x, k, 1, "auto", gpu, library=lib))
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), sched
    r = oracle_mod.check_synth_exact(base, k, 1, seed=91, dist=2, rtol=RTOL)
    assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, r
    cut = 2 * k + 777
    xf = oracle_mod.synth_f32(400_000, offset=k, dist=1)
    full = oracle_mod.mavg_f32(xf, k, 1)
    hist = xf[cut - (k - 1): cut].copy()
    assert_f32_close(_run(xf[cut:], k, 1, "blelloch", gpu, history=hist), full[cut:], f"k={k} history")


@pytest.mark.parametrize("dtype,C,k", [("i16", 1, 8_193), ("i16", 1, 44_100), ("i16", 1, 131_072),
                                       ("i16", 2, 4_097), ("i16", 2, 200_000), ("i16", 4, 8_193),
                                       ("i16", 4, 100_000), ("f32", 2, 4_097), ("f32", 2, 100_000)])
def test_aggregate_first_records(oracle_mod, gpu, dtype, C, k):
    """int16 mono / stereo / 4 channels and fp32 stereo windows past their tiles' LDS
    halo run the look-ahead scan in 32-KiB tiles with aggregate-first records (no
    phase A: every tile publishes its own record as soon as its loads land, the
    carry reads the records after the in-tile scan): the first window past each
    range boundary and long ones, bitwise the same under a forced recompute, absent
    and minimal look-ahead (head duty only), int16 bit-exact against the oracle,
    fp32 rounding data (dist 2) within the bar against the exact sums, and a
    history (the window reaching before frame 0)."""
    import digital_signal_processsing_amd as dsp
    dt = dsp.F32 if dtype == "f32" else dsp.I16
    frames = 3_000_017 // C  # hundreds of tiles: ragged XCD runs, head duty
    plan = dsp.plan(frames * C, k, C, dt)
    assert plan.startswith("ahead_scan<") and "self=1" in plan and "U=8" in plan and "wrec=0" in plan, plan
    tf = int(plan.split("tile_frames=")[1].split()[0])
    assert tf * C * (4 if dtype == "f32" else 2) == 32768, plan
    if k in (4_097, 8_193):  # the first window of the range: the one before it keeps its kernel
        prev = dsp.plan(frames * C, k - 1, C, dt)
        assert "self=1" not in prev, prev
    if dtype == "f32":
        x = oracle_mod.synth_f32(frames * C, seed=93, dist=2)
    else:
        x = oracle_mod.synth_i16(frames * C, seed=93)
    base = _run(x, k, C, "auto", gpu)
    for sched in ({"spin": 0}, {"slots": 0}, {"slots": 8, "spin": 0}):
        y = _with_schedule(sched, lambda lib: _run(x, k, C, "auto", gpu, library=lib))
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), sched
    if dtype == "f32":
        r = oracle_mod.check_synth_exact(base, k, C, seed=93, dist=2, rtol=RTOL)
        assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, r
    else:
        assert np.array_equal(base, oracle_mod.mavg_i16(x, k, C))
    cut = k + 4_321  # a history: the concatenation property through the aggregate-first carry
    n2 = min(frames, cut + 300_000)
    xs = x[: n2 * C]
    full = _run(xs, k, C, "auto", gpu)
    hist = xs[(cut - (k - 1)) * C: cut * C].copy()
    tail = _run(xs[cut * C:], k, C, "auto", gpu, history=hist)
    if dtype == "f32":
        assert_f32_close(tail, full[cut * C:], f"k={k} C={C} history")
    else:
        assert np.array_equal(tail, full[cut * C:]), f"k={k} C={C} history"


def _wide_windows(dsp, C, dt=None):
    """Windows around every shape change of the wide tile (halo rows, tile
    length, the last window it takes) and a few inside each range."""
    n = 1 << 24
    dt = dsp.F32 if dt is None else dt

    def shape(k):
        p = dsp.plan(n, k, C, dt)
        return p.split(" grid")[0] + p.split("block=")[1].split()[0]
    ks = {1, 2, 3, 7, 8, 9, 63, 64, 65}
    row = (64 if dt == dsp.F32 else 128) // C  # frames per 256-B LDS row of the staged halo
    ks.update({row - 1, row, row + 1, 2 * row + 1, 5 * row - 1})
    for k in range(2, 9000):  # (k = 1 is a copy)
        if shape(k) != shape(k + 1):
            ks.update({k - 1, k, k + 1, k + 2})
    tf = int(dsp.plan(n, 2, C, dt).split("tile_frames=")[1].split()[0])
    ks.update({tf - 1, tf, tf + 1})
    return sorted(k for k in ks if k >= 1)


@pytest.mark.parametrize("C", [2, 4, 8])
def test_wide_tile_every_window_edge(oracle_mod, gpu, C):
    """fp32 multi-channel frames run the wide-frame tile scan (mavg_wide.hpp:
    chunks of P consecutive frames per lane, swizzled LDS stage, outputs through
    LDS; 8 channels: chan_tile_kernel, one channel of 32 frames per lane): every window where the plan changes (halo rows, tile shapes, the switch
    to the look-ahead scan) and one frame either side, odd windows (the
    half-granule x[n-k] shift at C=2), on rounding data (dist 2) against the
    exact window sums, with a ragged tail tile."""
    import digital_signal_processsing_amd as dsp
    frames = 3 * 4096 + 1237
    seen = set()
    for k in _wide_windows(dsp, C):
        plan = dsp.plan(frames * C, k, C, dsp.F32)
        seen.add(plan.split(" grid")[0])
        x = oracle_mod.synth_f32(frames * C, seed=k, dist=2)
        r = oracle_mod.check_synth_exact(_run(x, k, C, "blelloch", gpu), k, C, seed=k, dist=2, rtol=RTOL)
        assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (k, plan, r)
    tile = "chan_tile<" if C == 8 else "wide_tile<"  # 8 channels: one channel per lane
    # past the wide tile: stereo takes the aggregate-first unit look-ahead (round 6), 4 / 8 channels
    # the wide look-ahead
    ahead = "ahead_scan<" if C == 2 else "wide_ahead<"
    assert any(p.startswith(tile) for p in seen) and any(p.startswith(ahead) for p in seen), seen


@pytest.mark.parametrize("C", [4, 8])
def test_wide_int16_every_window_edge(oracle_mod, gpu, C):
    """int16 with 4 and 8 channels runs the wide tile (and the wide
    look-ahead scan past it): bit-exact with the oracle at every window where
    the plan changes, one frame either side, a ragged tail, with and without
    a history."""
    import digital_signal_processsing_amd as dsp
    frames = 3 * 4096 + 1237
    seen = set()
    for k in _wide_windows(dsp, C, dsp.I16) + [20_000, 70_001]:
        plan = dsp.plan(frames * C, k, C, dsp.I16)
        seen.add(plan.split("<")[0])
        x = oracle_mod.synth_i16((frames + k) * C, offset=k)
        full = oracle_mod.mavg_i16(x, k, C)
        assert np.array_equal(_run(x[: frames * C], k, C, "blelloch", gpu),
                              oracle_mod.mavg_i16(x[: frames * C], k, C)), (k, plan)
        y = _run(x[k * C:], k, C, "blelloch", gpu, history=x[C: k * C])
        assert np.array_equal(y, full[k * C:]), (k, plan, "history")
    assert "wide_tile" in seen and "wide_ahead" in seen, seen


@pytest.mark.parametrize("C,k", [(2, 2), (2, 7), (2, 1023), (2, 1024), (2, 4096), (4, 2), (4, 255), (4, 1024),
                                 (4, 2048), (8, 2), (8, 8), (8, 9), (8, 1000), (8, 1024)])
def test_wide_tile_short_signals_history_and_views(oracle_mod, gpu, C, k):
    """The wide tile's edge paths: signals shorter than a tile and than the
    window (every tile an edge tile), a history (the window reaching before
    frame 0, element-staged first tiles), views 16 B into an allocation (C=2: a
    peeled 2-frame head then the body with pre=2; C=4: 16-B aligned frames; C=8:
    32-B-aligned views), against the oracle."""
    import digital_signal_processsing_amd as dsp
    import torch
    assert dsp.plan(1 << 24, k, C, dsp.F32).split("<")[0] in ("wide_tile", "chan_tile"), dsp.plan(1 << 24, k, C,
                                                                                                   dsp.F32)
    for frames in (1, 5, k, 2 * k + 3, 100_003):
        x = oracle_mod.synth_f32(frames * C, offset=frames + k, dist=1)
        assert_f32_close(_run(x, k, C, "blelloch", gpu), oracle_mod.mavg_f32(x, k, C), f"frames={frames}")
    frames = 100_003
    x = oracle_mod.synth_f32(frames * C, offset=3, dist=1)
    full = oracle_mod.mavg_f32(x, k, C)
    cut = 3 * k + 11
    lo = max(0, cut - (k - 1))
    hist = np.zeros((k - 1) * C, dtype=np.float32)
    hist[(k - 1 - (cut - lo)) * C:] = x[lo * C: cut * C]
    assert_f32_close(_run(x[cut * C:], k, C, "blelloch", gpu, history=hist), full[cut * C:], "history")
    off = 8 if C == 8 else 4  # 32 B (C=8) or 16 B
    xb = torch.zeros(frames * C + off, dtype=torch.float32, device=gpu)
    xb[off:] = torch.from_numpy(x).to(gpu)
    yb = torch.zeros_like(xb)
    dsp.moving_average_into(xb[off:], yb[off:], k, C, "blelloch")
    assert_f32_close(yb[off:].cpu().numpy(), full, f"view +{off * 4} B")
    if C == 2:  # 8 B in: a one-frame head, then the 16-B aligned body (pre=1)
        xb = torch.zeros(frames * C + 2, dtype=torch.float32, device=gpu)
        xb[2:] = torch.from_numpy(x).to(gpu)
        yb = torch.zeros_like(xb)
        dsp.moving_average_into(xb[2:], yb[2:], k, C, "blelloch")
        assert_f32_close(yb[2:].cpu().numpy(), full, "view +8 B")


@pytest.mark.parametrize("C,k", [(8, 512), (8, 1000), (8, 1024), (8, 1501), (8, 1536), (4, 2048), (4, 2544),
                                 (4, 3072)])
def test_chan_tile_halo_only_stage(oracle_mod, gpu, C, k):
    """The channel-per-lane tile with only the halo staged (xg=1: x from global
    memory, outputs staged in the halo region): rounding data against the exact
    window sums with a ragged tail, signals shorter than a tile, a history and
    a 32-B (C=8) / 16-B (C=4) offset view, against the oracle."""
    import digital_signal_processsing_amd as dsp
    import torch
    frames = 9 * 1024 + 333
    plan = dsp.plan(frames * C, k, C, dsp.F32)
    assert plan.startswith("chan_tile<") and ",xg=1" in plan, plan
    # fp32 C = 4 with a halo of exactly k frames (whole 256-B rows) writes its outputs in place
    assert (",ip=1" in plan) == (C == 4 and (k * C) % 64 == 0), plan
    assert (",xl=1>" in plan) == (C == 4 and k <= 2544), plan  # x as whole 16-B frames (round 6)
    x = oracle_mod.synth_f32(frames * C, seed=k + C, dist=2)
    r = oracle_mod.check_synth_exact(_run(x, k, C, "blelloch", gpu), k, C, seed=k + C, dist=2, rtol=RTOL)
    assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (plan, r)
    for short in (1, 7, k - 1, k + 5):
        xs = oracle_mod.synth_f32(short * C, offset=short, dist=1)
        assert_f32_close(_run(xs, k, C, "blelloch", gpu), oracle_mod.mavg_f32(xs, k, C), f"frames={short}")
    x = oracle_mod.synth_f32(frames * C, offset=3, dist=1)
    full = oracle_mod.mavg_f32(x, k, C)
    cut = k + 1111
    hist = x[(cut - (k - 1)) * C: cut * C].copy()
    assert_f32_close(_run(x[cut * C:], k, C, "blelloch", gpu, history=hist), full[cut * C:], "history")
    off = 8 if C == 8 else 4
    xb = torch.zeros(frames * C + off, dtype=torch.float32, device=gpu)
    xb[off:] = torch.from_numpy(x).to(gpu)
    yb = torch.zeros_like(xb)
    dsp.moving_average_into(xb[off:], yb[off:], k, C, "blelloch")
    assert_f32_close(yb[off:].cpu().numpy(), full, f"view +{off * 4} B")


@pytest.mark.parametrize("C,k", [(4, 4097), (4, 44_100), (8, 1537), (8, 2049), (8, 44_100), (2, 4097)])
def test_f32_multichannel_long_windows_every_form(oracle_mod, gpu, C, k):
    """Past the wide tile's LDS-staged halo (the wide look-ahead scan):
    rounding data against the exact sums, a view 16 B (C=8: 32 B) into an
    allocation, and the frame-unit form (blelloch_scalar: the look-ahead scan
    in one-frame units) for comparison."""
    import digital_signal_processsing_amd as dsp
    import torch
    frames = 300_007
    plan = dsp.plan(frames * C, k, C, dsp.F32)
    # stereo: the aggregate-first unit look-ahead in 4096-frame tiles (round 6)
    assert plan.startswith("ahead_scan<" if C == 2 else "wide_ahead<"), plan
    assert C != 2 or ("self=1" in plan and "U=8" in plan), plan
    assert dsp.plan(frames * C, k, C, dsp.F32, "blelloch_scalar").startswith("ahead_scan<")
    x = oracle_mod.synth_f32(frames * C, seed=k, dist=2)
    r = oracle_mod.check_synth_exact(_run(x, k, C, "blelloch", gpu), k, C, seed=k, dist=2, rtol=RTOL)
    assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (plan, r)
    ref = oracle_mod.mavg_f32(x, k, C)
    off = 8 if C == 8 else 4
    xb = torch.zeros(frames * C + off, dtype=torch.float32, device=gpu)
    xb[off:] = torch.from_numpy(x).to(gpu)
    yb = torch.zeros_like(xb)
    dsp.moving_average_into(xb[off:], yb[off:], k, C, "blelloch")
    assert_f32_close(yb[off:].cpu().numpy(), ref, f"k={k} view")
    assert_f32_close(_run(x, k, C, "blelloch_scalar", gpu), ref, f"k={k} scalar")


@pytest.mark.parametrize("C,k", [(2, 300_000), (4, 3585), (4, 20_000), (4, 8192), (8, 2049), (8, 44_100),
                                 (8, 700_000)])
def test_wide_ahead_bitwise_whatever_the_schedule(oracle_mod, gpu, C, k):
    """Multi-channel fp32 windows past the wide tile run the wide look-ahead
    scan (stereo: past the L2 reach; shorter stereo windows take the
    aggregate-first unit look-ahead, test_aggregate_first_records): rounding data (dist 2) within the bar against the exact window sums,
    and bitwise the same output when every record is recomputed by its
    consumer (spin 0), under the one-pass (slots 0) and minimal look-ahead
    schedules (the debug build's schedule hook) as under the release build's
    default schedule; ragged XCD runs and a ragged tail tile.  fp32 4 channels
    (round 6) publish every record in one order from every producer -- the tile
    itself, head duty, a consumer's recompute -- so self-published fp64 records
    keep their bits too (k = 3585, 20000; k = 8192: phase A)."""
    import digital_signal_processsing_amd as dsp
    frames = max(2_600_000 // C, 3 * k) + 12_345
    plan = dsp.plan(frames * C, k, C, dsp.F32)
    assert plan.startswith("wide_ahead<"), plan
    x = oracle_mod.synth_f32(frames * C, seed=k + C, dist=2)
    base = _run(x, k, C, "auto", gpu)
    r = oracle_mod.check_synth_exact(base, k, C, seed=k + C, dist=2, rtol=RTOL)
    assert r["mismatches"] == 0 and r["max_cond"] <= 2.0 ** -24 + 1e-9, (plan, r)
    for sched in ({}, {"spin": 0}, {"slots": 0}, {"slots": 8, "spin": 0}):
        y = _with_schedule(sched, lambda lib: _run(x, k, C, "auto", gpu, library=lib))
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), sched
    if " self=1 " in plan:
        # the self-order recompute of every record under the debug build's device checks
        y = _with_schedule({"spin": 0}, lambda lib: _run(x, k, C, "auto", gpu, library=lib), debug=True)
        assert np.array_equal(y.view(np.uint8), base.view(np.uint8)), "debug build"


@pytest.mark.parametrize("C", [2, 4, 8])
def test_wide_ahead_edges_history_views(oracle_mod, gpu, C):
    """The wide look-ahead scan at windows one frame either side of whole
    tiles (empty, one-frame and full partial windows), signals shorter than the
    window, a history reaching before frame 0, and 16-B / 32-B offset views."""
    import digital_signal_processsing_amd as dsp
    import torch
    T = int(dsp.plan(1 << 24, 50_000, C, dsp.F32).split("tile_frames=")[1].split()[0])
    for k in (16 * T - 1, 16 * T, 16 * T + 1, 3 * T + 7):
        for frames in (k // 3 + 1, 200_003):
            plan = dsp.plan(frames * C, k, C, dsp.F32)
            if not plan.startswith("wide_ahead<"):
                continue
            x = oracle_mod.synth_f32(frames * C, offset=k + frames, dist=1)
            assert_f32_close(_run(x, k, C, "blelloch", gpu), oracle_mod.mavg_f32(x, k, C), f"k={k} frames={frames}")
    k, frames, cut = 20_000, 120_000, 37_001
    x = oracle_mod.synth_f32(frames * C, offset=5, dist=1)
    full = oracle_mod.mavg_f32(x, k, C)
    lo = max(0, cut - (k - 1))
    hist = np.zeros((k - 1) * C, dtype=np.float32)
    hist[(k - 1 - (cut - lo)) * C:] = x[lo * C: cut * C]
    assert_f32_close(_run(x[cut * C:], k, C, "blelloch", gpu, history=hist), full[cut * C:], "history")
    off = 8 if C == 8 else 4
    xb = torch.zeros(frames * C + off, dtype=torch.float32, device=gpu)
    xb[off:] = torch.from_numpy(x).to(gpu)
    yb = torch.zeros_like(xb)
    dsp.moving_average_into(xb[off:], yb[off:], k, C, "blelloch")
    assert_f32_close(yb[off:].cpu().numpy(), full, f"view +{off * 4} B")


@pytest.mark.parametrize("fill", [0xFF, "tags"])
def test_ahead_poisoned_workspace(oracle_mod, gpu, fill):
    """The granules are zeroed on the stream before every launch: a caller
    workspace holding garbage -- including words that look like valid tagged
    records -- does not leak into the carry."""
    import digital_signal_processsing_amd as dsp
    import torch
    n, k = 600_001, 33_333
    x = torch.from_numpy(oracle_mod.synth_f32(n, seed=5, dist=1)).to(gpu)
    y = torch.empty_like(x)
    nb = dsp.workspace_bytes(n, k)
    assert nb > 0
    if fill == 0xFF:
        ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=gpu)
    else:  # every 8-byte word = {tag 1, payload 0x3ff00000}: a plausible record
        ws = torch.full((nb // 8,), (1 << 32) | 0x3FF00000, dtype=torch.int64, device=gpu)
    dsp.moving_average_into(x, y, k, workspace=ws)
    assert_f32_close(y.cpu().numpy(), oracle_mod.mavg_f32(oracle_mod.synth_f32(n, seed=5, dist=1), k, 1), str(fill))


def test_ahead_deterministic_repeats(oracle_mod, gpu):
    """Repeated launches of the look-ahead scan on fp32 data whose sums round:
    bitwise identical outputs (records are summed in a fixed order)."""
    import digital_signal_processsing_amd as dsp
    import torch
    n, k = 1 << 24, 50_000
    x = dsp.fill_synthetic(n, torch.float32, seed=9, dist=1, device=gpu)
    y0 = dsp.moving_average(x, k)
    for _ in range(5):
        assert torch.equal(dsp.moving_average(x, k).view(torch.int32), y0.view(torch.int32))


# ---------------------------------------------------------------------------
# dispatch boundaries: windows one frame either side of every halo-size
# threshold of dispatch_scan_f (tile shapes, tile -> look-ahead scan)
def _boundary_windows(dsp, n, C, dt):
    """Every window where the plan (kernel, tile, workgroup) changes, found by
    bisection on mavg_plan (no GPU), as k-1, k, k+1."""
    def shape(k):
        p = dsp.plan(n, k, C, dt)
        return p.split(" grid")[0] + p.split("block=")[1].split()[0]
    grid = sorted(set(int(round(10 * 1.05 ** i)) for i in range(200) if 10 * 1.05 ** i <= 60_000))
    ks = set()
    for a, b in zip(grid, grid[1:]):
        if shape(a) != shape(b):
            lo, hi = a, b
            while hi - lo > 1:
                mid = (lo + hi) // 2
                lo, hi = (mid, hi) if shape(mid) == shape(a) else (lo, mid)
            ks.update({hi - 1, hi, hi + 1})
    return sorted(ks)


@pytest.mark.parametrize("C", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dtype", ["i16", "f32"])
def test_dispatch_boundaries(oracle_mod, gpu, C, dtype):
    import digital_signal_processsing_amd as dsp
    rng = np.random.default_rng(1000 * C + (dtype == "f32"))
    elem = 4 if dtype == "f32" else 2
    seen = set()
    dt = dsp.F32 if dtype == "f32" else dsp.I16
    for k in _boundary_windows(dsp, 100_000 * C, C, dt):
        frames = int(rng.integers(k // 2, 3 * k + 20_000))
        off = int(rng.integers(0, 1 << 20))
        plan = dsp.plan(frames * C, k, C, dt)
        seen.add(plan.split(" grid")[0])
        use_hist = bool(rng.integers(0, 2))
        if dtype == "i16":
            x = oracle_mod.synth_i16((frames + k - 1) * C, offset=off)
            full = oracle_mod.mavg_i16(x, k, C)
        else:
            x = oracle_mod.synth_f32((frames + k - 1) * C, offset=off, dist=1)
            full = oracle_mod.mavg_f32(x, k, C)
        if use_hist:  # run on the tail with the (k-1) preceding frames as history
            y = _run(x[(k - 1) * C:], k, C, "auto", gpu, history=x[: (k - 1) * C])
            ref = full[(k - 1) * C:]
        else:
            y = _run(x[: frames * C], k, C, "auto", gpu)
            ref = (oracle_mod.mavg_i16 if dtype == "i16" else oracle_mod.mavg_f32)(x[: frames * C], k, C)
        if dtype == "i16":
            assert np.array_equal(y, ref), (k, frames, use_hist, plan)
        else:
            assert_f32_close(y, ref, f"k={k} frames={frames} hist={use_hist} {plan}")
    assert len(seen) >= 2, seen  # the sweep crosses kernel shapes (fp32 C=8: tile, look-ahead)


MISALIGNED_CASES = [(dt, C, algo, k) for dt in ("f32", "i16") for C in (1, 2)
                    for algo, k in (("blelloch", 37), ("blelloch", 1024), ("hillis", 300), ("direct", 9),
                                    ("direct_vec2", 5), ("blelloch", 20_000))]


@pytest.mark.parametrize("dt,C,algo,k", MISALIGNED_CASES)
def test_misaligned_views(oracle_mod, gpu, dt, C, algo, k):
    """Views that start 1..7 samples into an allocation: the same offset for
    input and output (head peeled, vector body) and a fresh aligned output
    (frame-unit form, element IO when a frame straddles its alignment).
    Results equal the oracle's on the same samples: int16 bit-exact, fp32
    within 1e-5 relative (the same bar as aligned launches)."""
    import torch
    import digital_signal_processsing_amd as dsp
    frames = 40_003
    base_n = frames * C + 16
    xb = (oracle_mod.synth_i16(base_n, seed=31) if dt == "i16" else oracle_mod.synth_f32(base_n, seed=31, dist=1))
    xd = torch.from_numpy(xb).to(gpu)
    for off in range(1, 8):
        n = (base_n - off) // C * C
        xs = xb[off:off + n]
        ref = oracle_mod.mavg_i16(xs, k, C) if dt == "i16" else oracle_mod.mavg_f32(xs, k, C)
        # same offset for input and output
        yb = torch.zeros_like(xd)
        dsp.moving_average_into(xd[off:off + n], yb[off:off + n], k, C, algo)
        # fresh (aligned) output
        y2 = dsp.moving_average(xd[off:off + n], k, C, algo)
        for y, what in ((yb[off:off + n], "same offset"), (y2, "fresh output")):
            got = y.cpu().numpy()
            if dt == "i16":
                assert np.array_equal(got, ref), f"{what} off={off}"
            else:
                assert_f32_close(got, ref, f"{what} off={off}")
        assert not yb[:off].any() and not yb[off + n:].any(), f"wrote outside the view, off={off}"


@pytest.mark.parametrize("dt,C", [("f32", 1), ("i16", 2), ("f32", 2)])
def test_misaligned_views_with_history(oracle_mod, gpu, dt, C):
    """A misaligned shard whose history is a misaligned view too (what a shard
    cut at an odd frame gets): equal to the whole-signal oracle."""
    import torch
    import digital_signal_processsing_amd as dsp
    frames, k = 50_001, 777
    x = oracle_mod.synth_i16(frames * C, seed=3) if dt == "i16" else oracle_mod.synth_f32(frames * C, seed=3, dist=1)
    full = oracle_mod.mavg_i16(x, k, C) if dt == "i16" else oracle_mod.mavg_f32(x, k, C)
    xd = torch.from_numpy(x).to(gpu)
    out = torch.zeros_like(xd)
    for f0 in (k - 1, 1001, 2047, 3333):
        f1 = f0 + 9_999
        dsp.moving_average_into(xd[f0 * C:f1 * C], out[f0 * C:f1 * C], k, C, "blelloch",
                                history=xd[(f0 - k + 1) * C:f0 * C])
        got = out[f0 * C:f1 * C].cpu().numpy()
        if dt == "i16":
            assert np.array_equal(got, full[f0 * C:f1 * C]), f0
        else:
            assert_f32_close(got, full[f0 * C:f1 * C], f"f0={f0}")


BLOCK_ALGOS = ["blelloch", "blelloch_scalar", "hillis", "hillis_scalar", "direct", "direct_vec2", "direct_scalar",
               "naive"]


@pytest.mark.parametrize("dt,C", [("f32", 1), ("i16", 2), ("f32", 3)])
def test_every_block_size_every_algo(oracle_mod, gpu, dt, C):
    """Every reference block size (run_benchmarks.py:21, plus 96 and 160) on
    every algorithm: the workgroup changes (mavg_plan), the output does not."""
    import digital_signal_processsing_amd as dsp
    frames = 30_011
    x = oracle_mod.synth_i16(frames * C, seed=13) if dt == "i16" else oracle_mod.synth_f32(frames * C, seed=13, dist=1)
    xd = _dev(x, gpu)
    for k in (1, 7, 300, 3000):
        ref = oracle_mod.mavg_i16(x, k, C) if dt == "i16" else oracle_mod.mavg_f32(x, k, C)
        for algo in BLOCK_ALGOS:
            if algo == "naive" and k == 3000:
                continue
            for block in (32, 64, 96, 128, 160, 256, 512, 1024):
                got = dsp.moving_average(xd, k, C, algo, block_size=block).cpu().numpy()
                if dt == "i16":
                    assert np.array_equal(got, ref), (algo, block, k)
                else:
                    assert_f32_close(got, ref, f"{algo} block={block} k={k}")


def test_explicit_side_stream_long_window(oracle_mod, gpu):
    """stream= differing from the current stream, on the look-ahead scan (which
    takes a workspace from the caching allocator): the workspace and the
    output are allocated on the launch stream, which waits for the producer
    of x on the current stream."""
    import torch
    import digital_signal_processsing_amd as dsp
    n, k = 3_000_017, 50_000
    s = torch.cuda.Stream()
    for rep in range(3):
        x = dsp.fill_synthetic(n, torch.float32, seed=40 + rep, dist=1, device=gpu)  # on the current stream
        y = dsp.moving_average(x, k, stream=s)
        del x  # freed on the current stream while s may still read it (record_stream keeps it alive)
        s.synchronize()
        assert_f32_close(y.cpu().numpy(), oracle_mod.mavg_f32(oracle_mod.synth_f32(n, seed=40 + rep, dist=1), k, 1),
                         f"rep {rep}")


DYN_LDS_CHILD = r'''
import threading, numpy as np, torch
import oracle
import digital_signal_processsing_amd as dsp
oracle.build()
n, k, C = 2 * 300_007, 10_000, 2
# the reference block size 1024 (the tuned dispatch takes the look-ahead scan at this window)
plan = dsp.plan(n, k, C, dsp.I16, block_size=1024)
assert "block=1024" in plan and int(plan.split("lds=")[1].split()[0]) > 64 * 1024, plan
x = oracle.synth_i16(n, seed=91)
ref = oracle.mavg_i16(x, k, C)
out = {}
def launch(tag):
    torch.cuda.set_device(0)  # hipSetDevice re-issued on a thread that has not launched yet
    y = dsp.moving_average(torch.from_numpy(x).to("cuda:0"), k, channels=C, block_size=1024)
    torch.cuda.synchronize()
    out[tag] = bool(np.array_equal(y.cpu().numpy(), ref))
for tag in ("first", "second"):
    t = threading.Thread(target=launch, args=(tag,))
    t.start(); t.join()
assert out == {"first": True, "second": True}, out
print("dyn lds ok")
'''


def test_dynamic_lds_tile_from_fresh_threads(gpu):
    """The 1024-thread tile above the default 64 KiB dynamic-LDS limit (int16
    stereo k=10000 at the reference block size 1024, 73 KiB), first launched from a fresh thread after
    hipSetDevice(0) in a fresh process, then again from another thread: the
    limit is raised per (kernel, device) on the current device
    (mavg_launch.hpp raise_dyn_lds_limit), and both outputs match the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-c", DYN_LDS_CHILD], cwd=root, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "dyn lds ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
