"""The tile -> workgroup mapping of the look-ahead scan for windows past an
XCD's L2 reach, restated on the host (specification tests; the device code is
digital_signal_processsing_amd/csrc/mavg_device.hpp remap_tile, exercised on
the GPU by test_gpu_parity.py::test_period_remap_very_long_windows_with_tail
and test_grouped_xcd_remap_with_tail): runs of G tiles per XCD, bijective over
every grid, and G matched to the window so that x[n-k]'s tile runs on the
tile's own XCD; the launcher's choice of G (ahead_run_length, mavg_launch.hpp)."""
import re

import pytest

TF = 4096


def remap_group(b, nb, G):
    i, x = b >> 3, b & 7
    full = nb - nb % (8 * G)
    if b >= full:
        return b
    per = i // G
    return per * 8 * G + x * G + (i - per * G)


def run_length(k, tf, ahead):
    """ahead_run_length (mavg_launch.hpp)."""
    gmax = max(2, min(48, ahead // 20))
    m = k / tf
    J = 1
    while m / (8.0 * J) > gmax + 0.5:
        J += 1
    best, best_miss = 0, 2.0
    for j in range(J, J + 8):
        G = max(2, int(m / (8.0 * j) + 0.5))
        miss = abs(m - 8.0 * j * G) / G
        if G <= gmax and miss < best_miss - 1e-9:
            best_miss, best = miss, G
    return best or gmax


@pytest.mark.parametrize("G", [2, 3, 18, 23, 31, 41, 64])
@pytest.mark.parametrize("nb", [7, 8 * 61 + 3, 262_144, 262_181])
def test_runs_are_a_bijection(G, nb):
    assert sorted(remap_group(b, nb, G) for b in range(nb)) == list(range(nb))


@pytest.mark.parametrize("k,ahead", [(524_289, 1024), (600_000, 1024), (1_000_000, 1024), (2_222_222, 1024),
                                     (4_000_000, 1024), (1_000_000, 768), (10_000_000, 1024)])
def test_matched_runs_put_the_shifted_tile_on_the_same_xcd(k, ahead):
    nb = 262_144
    G = run_length(k, TF, ahead)
    assert 2 <= G <= min(48, ahead // 20)
    blk = {remap_group(b, nb, G): b for b in range(nb)}
    full = nb - nb % (8 * G)
    inside = [t for t in range(nb) if t * TF >= k and blk[t] < full and blk[(t * TF - k) // TF] < full]
    same = sum(blk[t] % 8 == blk[(t * TF - k) // TF] % 8 for t in inside) / len(inside)
    m = k / TF
    J = max(1, round(m / (8 * G)))
    miss = abs(m - 8 * J * G) / G
    assert same >= 1 - miss - 1.5 / G, (G, J, same, miss)


def test_plans_pick_window_matched_runs_past_the_l2_reach():
    import digital_signal_processsing_amd as dsp
    plan = lambda k, C, dt: dsp.plan(1 << 30, k, C, dt)
    remap = lambda k, C, dt: int(re.search(r"remap=(\d+)", plan(k, C, dt)).group(1))
    assert remap(44_100, 1, dsp.F32) == 1 and remap(300_000, 1, dsp.F32) == 1
    # 32-KiB tiles (U=8) without run totals up to 1024 tiles per window (round 6): fp32 mono and
    # int16 stereo 8192-frame tiles, int16 mono 16384; D (320; int16 stereo past 2^21: 960) sets the
    # run length; past 1024 tiles the 4096-frame run-total kernel
    for k, C, dt, tf, ahead, runs in ((600_000, 1, dsp.F32, 8192, 320, False),
                                      (1_000_000, 1, dsp.F32, 8192, 320, False),
                                      (4_000_000, 1, dsp.F32, 8192, 320, False),
                                      (10_000_000, 1, dsp.F32, 4096, 1024, True),
                                      (1_000_000, 2, dsp.I16, 8192, 320, False),
                                      (4_000_000, 2, dsp.I16, 8192, 960, False),
                                      (10_000_000, 2, dsp.I16, 4096, 768, True),
                                      (1_500_000, 1, dsp.I16, 16384, 320, False),
                                      (4_000_000, 1, dsp.I16, 16384, 320, False),
                                      (20_000_000, 1, dsp.I16, 8192, 1024, True)):
        p = plan(k, C, dt)
        assert "tile_frames=%d " % tf in p and " ahead=%d " % ahead in p, (k, C, p)
        assert remap(k, C, dt) == run_length(k, tf, ahead), (k, C)
        assert ("runs=1" in p) == runs, (k, C, p)
    assert remap(1024, 1, dsp.F32) == 64  # the tile kernel's grouped runs
