"""The tile -> workgroup mappings of the look-ahead scan, restated on the host
(specification tests; the device code is digital_signal_processsing_amd/csrc/
mavg_lookback.hpp period_tile and mavg_device.hpp remap_tile, exercised on the
GPU by test_gpu_parity.py::test_period_remap_very_long_windows_with_tail and
test_grouped_xcd_remap_with_tail): bijective over every grid, and for
window-matched runs x[n-k]'s tile runs on the tile's own XCD."""
import re

import pytest

TF = 4096


def period_tile(b, k, pden, pfull):
    if b >= pfull:
        return b
    i, x = b >> 3, b & 7
    per = ((i + 1) * pden - 1) // k
    s0, s1 = per * k // pden, (per + 1) * k // pden
    return 8 * s0 + x * (s1 - s0) + (i - s0)


def period_params(k, J, nb):
    pden = 8 * J * TF
    P = ((nb // 8 + 1) * pden - 1) // k
    return pden, 8 * (P * k // pden)


def remap_group(b, nb, G):
    i, x = b >> 3, b & 7
    full = nb - nb % (8 * G)
    if b >= full:
        return b
    per = i // G
    return per * 8 * G + x * G + (i - per * G)


@pytest.mark.parametrize("k", [524_289, 600_000, 1_000_000, 2_222_222, 4_000_000])
@pytest.mark.parametrize("J", [1, 2, 3])
@pytest.mark.parametrize("nb", [8 * 1000 + 5, 262_144, 262_181])
def test_period_tile_is_a_bijection_with_same_xcd_shift(k, J, nb):
    pden, pfull = period_params(k, J, nb)
    tiles = [period_tile(b, k, pden, pfull) for b in range(nb)]
    assert sorted(tiles) == list(range(nb))
    assert pfull % 8 == 0 and pfull <= nb
    blk = {t: b for b, t in enumerate(tiles)}
    inside = [t for t in range(nb) if blk[t] < pfull and t * TF >= k and blk[(t * TF - k) // TF] < pfull]
    same = sum(blk[t] % 8 == blk[(t * TF - k) // TF] % 8 for t in inside)
    # a run of ~g = k/(8 J T) tiles holds the shifted tile except near a run
    # boundary: run x of a period starts x * (G_p - G_{p-J}) tiles (at most
    # x <= 7, the floor/ceil run lengths) off its place J periods back, so the
    # misses grow with J and shrink with g (J = 1, k = 10^6: 7 %)
    g = k / (8 * J * TF)
    assert same / len(inside) >= 1 - (J + 2.5) / g, (same / len(inside), g)


@pytest.mark.parametrize("G", [2, 3, 18, 31, 61, 64])
@pytest.mark.parametrize("nb", [7, 8 * 61 + 3, 262_144, 262_181])
def test_grouped_runs_are_a_bijection(G, nb):
    assert sorted(remap_group(b, nb, G) for b in range(nb)) == list(range(nb))


def test_plans_pick_window_matched_runs_past_the_l2_reach():
    import digital_signal_processsing_amd as dsp
    remap = lambda k, C, dt: re.search(r"remap=(\S+)", dsp.plan(1 << 30, k, C, dt)).group(1)
    assert remap(44_100, 1, dsp.F32) == "1" and remap(300_000, 1, dsp.F32) == "1"
    assert remap(1_000_000, 1, dsp.F32) == "period1"
    assert remap(4_000_000, 1, dsp.F32) == "period4"
    assert remap(1_000_000, 2, dsp.I16) == "period1"
    assert remap(1024, 1, dsp.F32) == "64"  # the tile kernel's grouped runs
