"""CPU tests of the oracle (the checker): C restatement vs an independent numpy
formulation, closed-form known answers derived from the reference loop
(basics/profilable_moving_averager.cpp:14-37), and the committed fixtures."""
import hashlib
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("C", [1, 2, 3, 8])
@pytest.mark.parametrize("k", [1, 2, 3, 7, 32, 41, 64, 1000, 4096, 5000])
def test_c_restatement_matches_numpy_i16(oracle_mod, C, k):
    x = oracle_mod.synth_i16(3000 * C, offset=17 * C + k)
    assert np.array_equal(oracle_mod.mavg_i16(x, k, C), oracle_mod.numpy_mavg_i16(x, k, C))


@pytest.mark.parametrize("C", [1, 2, 5])
@pytest.mark.parametrize("k", [1, 7, 64, 1024])
@pytest.mark.parametrize("dist", [0, 1])
def test_c_restatement_matches_numpy_f32(oracle_mod, C, k, dist):
    x = oracle_mod.synth_f32(3000 * C, offset=5, dist=dist)
    a = oracle_mod.mavg_f32(x, k, C)
    b = oracle_mod.numpy_mavg_f32(x, k, C)
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6 * np.abs(b).max())


def test_known_answers_i16(oracle_mod):
    # constant input c: warm-up frames f < k give (c*(f+1))/k truncated; then c
    k, c = 5, 7
    y = oracle_mod.mavg_i16(np.full(20, c, np.int16), k)
    assert list(y[:5]) == [(c * (f + 1)) // k for f in range(5)]
    assert (y[4:] == c).all()
    # impulse: y = trunc(A / k) for k frames after the impulse, else 0
    x = np.zeros(30, np.int16)
    x[10] = 1000
    y = oracle_mod.mavg_i16(x, 7)
    assert (y[10:17] == 1000 // 7).all() and (y[:10] == 0).all() and (y[17:] == 0).all()
    # negative sums truncate toward zero (C++ int64 division), not floor
    x = np.array([-7, 0, 0, -1], np.int16)
    assert list(oracle_mod.mavg_i16(x, 2)) == [-3, -3, 0, 0]
    # k = 1 is the identity
    x = oracle_mod.synth_i16(1000)
    assert np.array_equal(oracle_mod.mavg_i16(x, 1), x)
    # stereo channels are independent
    x = np.zeros(20, np.int16)
    x[0::2] = 4
    x[1::2] = -8
    y = oracle_mod.mavg_i16(x, 2, 2)
    assert list(y[:4]) == [2, -4, 4, -8]


def test_known_answers_f32(oracle_mod):
    x = np.arange(1, 11, dtype=np.float32)
    y = oracle_mod.mavg_f32(x, 4)
    # frame i holds i+1; warm-up divides by k even before k frames were seen
    sums = [1, 3, 6, 10] + [(i - 2) + (i - 1) + i + (i + 1) for i in range(4, 10)]
    expect = np.array([s / 4 for s in sums], np.float32)
    np.testing.assert_array_equal(y, expect)


def test_window_sum_slices(oracle_mod):
    x = oracle_mod.synth_i16(10000 * 2, offset=3)
    full = oracle_mod.numpy_window_sum(x, 300, 2)
    for f0, f1 in [(0, 10), (299, 301), (4000, 6000), (9990, 10000)]:
        got = oracle_mod.window_sum_i64(x, 300, 2, f0, f1)
        assert np.array_equal(got, full[f0 * 2:f1 * 2])


def test_synth_matches_spec(oracle_mod):
    # splitmix64 reference values computed independently in Python
    def splitmix64(z):
        m = (1 << 64) - 1
        z = (z + 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        return z ^ (z >> 31)

    seed, off = 0x5EED, 123
    x = oracle_mod.synth_i16(64, seed=seed, offset=off)
    xf = oracle_mod.synth_f32(64, seed=seed, offset=off, dist=1)
    for i in range(64):
        h = splitmix64(seed + off + i)
        assert int(x[i]) == np.int16(np.uint16(h >> 48))
        assert float(xf[i]) == np.float32((h >> 40) / 16777216.0)


def test_invalid_args(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.mavg_i16(np.zeros(5, np.int16), 2, 2)  # n not a multiple of C
    with pytest.raises(ValueError):
        oracle_mod.mavg_i16(np.zeros(4, np.int16), 0, 1)  # k < 1


def test_golden_fixtures(oracle_mod):
    g = np.load(os.path.join(GOLDEN, "mavg_golden.npz"))
    for C in (1, 2):
        x = oracle_mod.synth_i16(4096 * C, seed=0x5EED)
        xf = oracle_mod.synth_f32(4096 * C, seed=0x5EED, dist=1)
        for k in (1, 3, 7, 32, 41, 64, 1000, 1024):
            assert np.array_equal(oracle_mod.mavg_i16(x, k, C), g[f"i16_C{C}_k{k}"])
            assert np.array_equal(oracle_mod.mavg_f32(xf, k, C), g[f"f32u_C{C}_k{k}"])
    digests = dict(line.split() for line in open(os.path.join(GOLDEN, "digests.txt")))
    x = oracle_mod.synth_i16(1 << 20, seed=0x5EED)
    assert hashlib.sha256(oracle_mod.mavg_i16(x, 32, 1).tobytes()).hexdigest() == digests["i16_n1048576_C1_k32"]


@pytest.mark.parametrize("C,k,threads", [(1, 1024, 8), (2, 7, 3), (1, 1, 4), (3, 5000, 16), (1, 64, 1)])
def test_multicore_baseline_equals_serial(oracle_mod, C, k, threads):
    x = oracle_mod.synth_f32(200_003 * C, offset=k, dist=1)
    np.testing.assert_allclose(oracle_mod.mavg_f32_mt(x, k, C, threads), oracle_mod.mavg_f32(x, k, C),
                               rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("C,k,dist,offset,threads", [
    (1, 1024, 0, 0, 7), (2, 41, 1, 0, 3), (1, 7, 0, 12345, 8), (3, 300, 1, 99 * 3, 5), (1, 5000, 0, 0, 1),
    (2, 1, 0, 2, 4), (1, 70_000, 0, 4096, 6)])
def test_full_signal_checker_equals_serial_loop(oracle_mod, C, k, dist, offset, threads):
    """check_synth (chunked, x regenerated from its counter) accepts exactly
    the serial restatement's output, at any offset into the stream, and
    reports the first corrupted sample."""
    n = 150_001 * C
    x = oracle_mod.synth_f32(n + offset, dist=dist)
    y = oracle_mod.mavg_f32(x, k, C)[offset:]
    r = oracle_mod.check_synth(y, k, C, offset=offset, dist=dist, threads=threads)
    assert r["mismatches"] == 0 and r["checked"] == n and r["max_rel"] == 0.0, r
    y[n // 3] = np.nextafter(y[n // 3], np.float32(np.inf)) * np.float32(1.0001)
    r = oracle_mod.check_synth(y, k, C, offset=offset, dist=dist, threads=threads)
    assert r["mismatches"] == 1 and r["first_bad"] == n // 3, r
    xi = oracle_mod.synth_i16(n + offset)
    yi = oracle_mod.mavg_i16(xi, k, C)[offset:]
    assert oracle_mod.check_synth(yi, k, C, offset=offset, threads=threads)["mismatches"] == 0
    yi[0] ^= 1
    yi[-1] ^= 1
    r = oracle_mod.check_synth(yi, k, C, offset=offset, threads=threads)
    assert r["mismatches"] == 2 and r["first_bad"] == 0, r


def test_full_signal_checker_rejects_bad_args(oracle_mod):
    y = np.zeros(10, np.float32)
    for kw in (dict(k=0), dict(k=3, channels=3), dict(k=3, channels=2, offset=1), dict(k=3, dist=3)):
        with pytest.raises(ValueError):
            oracle_mod.check_synth(y, **kw)
    with pytest.raises(TypeError):
        oracle_mod.check_synth(np.zeros(4, np.float64), 3)


def test_dist2_generator_matches_numpy_statement(oracle_mod):
    """The zero-mean, mixed-scale generator (fp32 rounding stress): C and an
    independent numpy statement agree bit for bit at any offset."""
    for off in (0, 12345, (1 << 40) + 7):
        a = oracle_mod.synth_f32(50_000, offset=off, dist=2)
        b = oracle_mod.numpy_synth_f32_dist2(50_000, offset=off)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), off
    x = oracle_mod.synth_f32(1 << 20, dist=2)
    assert abs(float(x.mean())) < 0.01 and 1.5 < float(x.std()) < 2.0          # zero-mean
    assert (x < 0).mean() > 0.45 and (np.abs(x) < 1e-3).mean() > 0.3           # both signs, mixed scale
    assert np.abs(x[x != 0]).min() > 2.0 ** -41                                # exact in 2^-64 fixed point


def test_dist2_fp64_window_sums_round(oracle_mod):
    """dist 2 exists to make fp64 accumulation round: sequential fp64 window
    sums differ from the exact (math.fsum) sums for a good share of windows,
    so a full-size fp32 check on it is not a bit-equality check in disguise."""
    import math
    x = oracle_mod.synth_f32(1 << 16, dist=2).astype(np.float64)
    k = 1024
    inexact = 0
    for s in range(0, len(x) - k, 257):
        w = x[s:s + k]
        acc = 0.0
        for v in w:
            acc += v
        inexact += acc != math.fsum(w)
    assert inexact > 50, inexact


@pytest.mark.parametrize("C,k,dist,offset,threads", [
    (1, 1024, 2, 0, 7), (2, 41, 2, 6, 3), (1, 7, 2, 12345, 8), (1, 44_100, 2, 0, 5), (3, 300, 1, 99 * 3, 4),
    (1, 64, 0, 0, 2)])
def test_exact_checker_accepts_restatement_and_flags_errors(oracle_mod, C, k, dist, offset, threads):
    """check_synth_exact (exact __int128 window sums) accepts the serial fp64
    restatement's output on every distribution -- its running-sum drift stays
    far inside 1e-5 -- and reports an output nudged by more than the bar."""
    n = 120_001 * C
    x = oracle_mod.synth_f32(n + offset, dist=dist)
    y = oracle_mod.mavg_f32(x, k, C)[offset:]
    r = oracle_mod.check_synth_exact(y, k, C, offset=offset, dist=dist, threads=threads)
    assert r["mismatches"] == 0 and r["checked"] == n, r
    assert r["max_cond"] <= 2.0 ** -24 + 1e-9, r
    i = n // 3
    y[i] = np.float32(y[i] + 1e-4 * (abs(float(y[i])) + float(np.abs(x).mean())))  # > both bars
    r = oracle_mod.check_synth_exact(y, k, C, offset=offset, dist=dist, threads=threads)
    assert r["mismatches"] == 1 and r["first_bad"] == i, r
    # NaN is a mismatch, never a pass
    y[0] = np.nan
    assert oracle_mod.check_synth_exact(y, k, C, offset=offset, dist=dist, threads=threads)["mismatches"] == 2


def test_exact_checker_floor_for_cancelling_windows(oracle_mod):
    """|S| ~ 0: an output off by less than 1e-5 of the window's mean absolute
    input passes on the floor (and is counted), a larger error fails."""
    k = 4
    x = oracle_mod.synth_f32(4000, dist=2)
    y = oracle_mod.mavg_f32(x, k, 1)
    s = np.array([math_fsum(x[max(0, f - k + 1):f + 1]) for f in range(len(x))])
    fl = np.array([np.abs(x[max(0, f - k + 1):f + 1].astype(np.float64)).sum() for f in range(len(x))]) / k
    f = int(np.argmin(np.abs(s) / k / fl))          # the most cancelling window
    y[f] = np.float32(s[f] / k + 0.5e-5 * fl[f])    # > 1e-5 |S/k|, < 1e-5 F
    r = oracle_mod.check_synth_exact(y, k, 1, dist=2, threads=2)
    assert r["mismatches"] == 0 and r["floor_used"] >= 1, r
    y[f] = np.float32(s[f] / k + 2e-5 * fl[f])
    assert oracle_mod.check_synth_exact(y, k, 1, dist=2, threads=2)["mismatches"] == 1


def math_fsum(a):
    import math
    return math.fsum(a.astype(np.float64))
