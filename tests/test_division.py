"""The int16 output division (csrc/mavg_device.hpp to_out_i16): the kernels
compute trunc(S / k) -- C++ integer division, as the reference's
profilable_moving_averager.cpp:27-33 does with int64 -- as
(int)(double(S) * inv_up), inv_up = fl(fl(1/k) * (1 + 2^-50)).  This file
checks that rule against exact integer division in numpy, with the same IEEE
fp64 operations the device performs (v_cvt_f64_i32, v_mul_f64 round to
nearest even, v_cvt_i32_f64 truncates), at every divisor the int32 path
takes and at the quotient boundaries where an estimate can fail: exact
multiples q*k and q*k +- 1, k-1 remainders, and the extreme window sums
+-32768*k (runs on the CPU)."""
import numpy as np
import pytest

# the window sum of k int16 samples lies in [-32768 k, 32767 k]
QS = np.array([-32768, -32767, -20000, -1025, -2, -1, 0, 1, 2, 3, 1024, 12345, 32766, 32767], dtype=np.int64)


def inv_up(k):
    return (1.0 / np.asarray(k, dtype=np.float64)) * (1.0 + 2.0 ** -50)


def device_rule(s, k):
    # (double)s exact (|s| < 2^53), one rounded product, truncation toward zero
    return np.trunc(s.astype(np.float64) * inv_up(k)).astype(np.int64)


def exact_trunc(s, k):
    q = np.abs(s) // k
    return np.where(s < 0, -q, q)


def sums_at_boundaries(k):
    k = np.asarray(k, dtype=np.int64)[:, None]
    q = QS[None, :]
    base = q * k
    s = np.concatenate([base, base + 1, base - 1, base + (k - 1), base - (k - 1)], axis=1)
    lo, hi = -32768 * k, 32767 * k
    return np.clip(s, lo, hi), np.broadcast_to(k, s.shape)


@pytest.mark.parametrize("chunk", range(8))
def test_int32_path_every_divisor(chunk):
    """every k in [1, 65535] (the int32 accumulator path), 70 sums each"""
    ks = np.arange(1 + chunk * 8192, min(65536, 1 + (chunk + 1) * 8192), dtype=np.int64)
    s, kk = sums_at_boundaries(ks)
    got = device_rule(s, kk)
    want = exact_trunc(s, kk)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"first failure: S={s[tuple(bad[0])]} k={kk[tuple(bad[0])]}"


def test_int64_path_long_windows():
    """k past 65535 (int64 sums up to 32768 k < 2^47), sampled up to 2^31 - 1"""
    rng = np.random.default_rng(7)
    ks = np.unique(np.concatenate([
        np.arange(65536, 65536 + 4096, dtype=np.int64),
        rng.integers(65536, 2 ** 31 - 1, 20000, dtype=np.int64),
        np.array([2 ** 20, 2 ** 24 - 1, 2 ** 24, 2 ** 24 + 1, 2 ** 30, 2 ** 31 - 1], dtype=np.int64),
    ]))
    s, kk = sums_at_boundaries(ks)
    assert np.abs(s).max() < 2 ** 47
    got = device_rule(s, kk)
    want = exact_trunc(s, kk)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"first failure: S={s[tuple(bad[0])]} k={kk[tuple(bad[0])]}"


def test_random_sums():
    """random window sums and divisors, both paths"""
    rng = np.random.default_rng(11)
    k = rng.integers(1, 2 ** 31 - 1, 200000, dtype=np.int64)
    k[:100000] = rng.integers(1, 65536, 100000)
    s = rng.integers(-32768, 32768, k.size, dtype=np.int64) * k + rng.integers(-(2 ** 40), 2 ** 40, k.size) % k
    s = np.clip(s, -32768 * k, 32767 * k)
    assert np.array_equal(device_rule(s, k), exact_trunc(s, k))
