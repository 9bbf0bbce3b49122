"""Full-size parity: EVERY output of the BASELINE.json configurations (and the
long-window / int16 bench lines) against the CPU restatement of
basics/profilable_moving_averager.cpp:14-37, not samples of it.

The input is the device counter-based generator; the oracle
regenerates each sample from its counter (oracle.check_synth), so a 2^30
launch is checked in a few seconds of host time without a host copy of x.
fp32: within RTOL = 1e-5 relative (north_star); int16: bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5
SEED = 0x5EED

CONFIGS = [
    # id, samples, k, C, dtype, algo
    ("headline_2p30_k1024", 1 << 30, 1024, 1, "f32", "blelloch"),   # BASELINE metric config (configs[4] per GPU)
    ("config2_2p26_k64", 1 << 26, 64, 1, "f32", "blelloch"),        # configs[1]
    ("config3_2p28_k7_direct", 1 << 28, 7, 1, "f32", "direct"),     # configs[2]
    ("config4_2p30_k4096", 1 << 30, 4096, 1, "f32", "blelloch"),    # configs[3]
    ("long_2p30_k44100", 1 << 30, 44100, 1, "f32", "blelloch"),     # look-ahead scan
    ("mid_2p30_k8192", 1 << 30, 8192, 1, "f32", "blelloch"),        # look-ahead scan, self-published records
    ("hillis_2p30_k1024", 1 << 30, 1024, 1, "f32", "hillis"),
    ("hillis_2p30_k44100", 1 << 30, 44100, 1, "f32", "hillis"),   # Hillis-Steele through the record carry
    ("i16_2p30_k1024", 1 << 30, 1024, 1, "i16", "blelloch"),
    ("i16_stereo_2p30_k44100", 1 << 30, 44100, 2, "i16", "blelloch"),  # 1 s windows on 44.1 kHz stereo PCM
    ("i16_mono_2p30_k44100", 1 << 30, 44100, 1, "i16", "blelloch"),  # look-ahead scan, int16 mono
    ("i16_stereo_2p30_k1024", 1 << 30, 1024, 2, "i16", "blelloch"),  # the reference's stereo PCM layout
    ("long_1m_k1000000", 1 << 30, 1_000_000, 1, "f32", "blelloch"),  # window-matched runs
    ("long_4m_k4000000", 1 << 30, 4_000_000, 1, "f32", "blelloch"),  # window-matched runs, 8192-frame tiles
    # int16 past the L2 reach: self-published records in window-matched runs (stereo), phase A (mono)
    ("i16_stereo_2p30_k2000000", 1 << 30, 2_000_000, 2, "i16", "blelloch"),
    ("i16_mono_2p30_k4000000", 1 << 30, 4_000_000, 1, "i16", "blelloch"),
    ("f32_stereo_2p30_k1024", 1 << 30, 1024, 2, "f32", "blelloch"),  # fp32 form of the stereo harness layout
    ("f32_c4_2p30_k1024", 1 << 30, 1024, 4, "f32", "blelloch"),
    ("f32_c8_2p30_k1024", 1 << 30, 1024, 8, "f32", "blelloch"),
    # multi-channel windows past the LDS-staged halo (wide look-ahead) and the halo-only chan tile's edge
    ("f32_stereo_2p30_k44100", 1 << 30, 44100, 2, "f32", "blelloch"),
    ("f32_c4_2p30_k44100", 1 << 30, 44100, 4, "f32", "blelloch"),
    ("f32_c8_2p30_k44100", 1 << 30, 44100, 8, "f32", "blelloch"),
    ("f32_c8_2p30_k2048", 1 << 30, 2048, 8, "f32", "blelloch"),
    # the in-place halo-only chan tile (fp32 C = 4, 2048 <= k <= 3584, k % 16 == 0: each output
    # written over the x[n-k] it last read) at full size: large grids and the XCD remap
    ("f32_c4_2p30_k2048", 1 << 30, 2048, 4, "f32", "blelloch"),
    # the reference's int16 PCM at 4 and 8 channels (wav_header.h:26-48)
    ("i16_c4_2p30_k1024", 1 << 30, 1024, 4, "i16", "blelloch"),
    ("i16_c8_2p30_k1024", 1 << 30, 1024, 8, "i16", "blelloch"),
    ("i16_c4_2p30_k44100", 1 << 30, 44100, 4, "i16", "blelloch"),
    ("i16_c8_2p30_k44100", 1 << 30, 44100, 8, "i16", "blelloch"),
    # int16 8 channels at a window of one tile: the dword-column look-ahead, self-published (round 6)
    ("i16_c8_2p30_k2048", 1 << 30, 2048, 8, "i16", "blelloch"),
    # the chunk-form wide look-ahead (fp32 stereo past the L2 reach, int16 8 channels past int32
    # sums) with a partial window (k mod tile != 0): the r05ad development build zeroed that part
    # of the carry in this form, which the k = 44100 configs above no longer
    # reach since those windows take the aggregate-first look-ahead
    ("f32_stereo_2p30_k300001", 1 << 30, 300_001, 2, "f32", "blelloch"),
    ("i16_c8_2p30_k70001", 1 << 30, 70_001, 8, "i16", "blelloch"),
]


@pytest.mark.parametrize("name,n,k,C,dt,algo", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_every_output_matches_oracle(oracle_mod, gpu, name, n, k, C, dt, algo):
    import torch
    import digital_signal_processsing_amd as dsp
    dtype = torch.float32 if dt == "f32" else torch.int16
    x = dsp.fill_synthetic(n, dtype, seed=SEED, device=gpu)
    y = dsp.moving_average(x, k, channels=C, algo=algo)
    del x
    yh = y.cpu().numpy()
    del y
    r = oracle_mod.check_synth(yh, k, C, seed=SEED, rtol=RTOL)
    assert r["checked"] == n
    assert r["mismatches"] == 0, f"{name}: {r}"
    if dt == "f32":
        # int16-valued input: every window sum is exact in fp64, so the output
        # is the correctly rounded quotient -- bit-equal, not merely 1e-5
        assert r["max_rel"] == 0.0, f"{name}: {r}"


# fp32 parity on rounding, cancelling data at full size (dist 2: zero-mean,
# mixed-scale, non-dyadic samples whose fp64 window sums round): every output
# against the EXACT window sum (__int128 fixed point, oracle.check_synth_exact).
# Bar (north_star, DESIGN.md "Parity bar"): |y - S/k| <= 1e-5 |S/k|, or, where
# the sum cancels to ~0, <= 1e-5 * F with F = sum|x|/k the window's mean
# absolute input (the count of such outputs is reported); and the error beyond
# the fp32 output rounding must stay under 1e-9 F (fp64 accumulation quality).
DIST2_CONFIGS = [c for c in CONFIGS if c[4] == "f32"]


@pytest.mark.parametrize("name,n,k,C,dt,algo", DIST2_CONFIGS, ids=[c[0] + "_dist2" for c in DIST2_CONFIGS])
def test_every_output_of_rounding_data_within_bar(oracle_mod, gpu, name, n, k, C, dt, algo):
    import torch
    import digital_signal_processsing_amd as dsp
    x = dsp.fill_synthetic(n, torch.float32, seed=SEED, dist=2, device=gpu)
    y = dsp.moving_average(x, k, channels=C, algo=algo)
    del x
    yh = y.cpu().numpy()
    del y
    r = oracle_mod.check_synth_exact(yh, k, C, seed=SEED, dist=2, rtol=RTOL)
    print(f"{name} dist2: {r}")
    assert r["checked"] == n
    assert r["mismatches"] == 0, f"{name}: {r}"
    assert r["max_cond"] <= 2.0 ** -24 + 1e-9, f"{name}: {r}"


@pytest.mark.parametrize("world", [2, 8])
def test_every_output_of_sharded_weak_scaling_signal(oracle_mod, gpu, world):
    """BASELINE config #5 on one GPU: the 2^30-sample shards of a world*2^30
    signal (what rank r holds under weak scaling, bench.py) filtered as
    interior + head launch with rank r-1's tail as history; every output of
    the first and a later shard is checked at its global offset."""
    import torch
    import digital_signal_processsing_amd as dsp
    from digital_signal_processsing_amd.shard import split_moving_average_into
    n, k = 1 << 30, 1024
    for r in (0, world - 1):
        x = dsp.fill_synthetic(n, torch.float32, seed=SEED, offset=r * n, device=gpu)
        hist = (dsp.fill_synthetic(k - 1, torch.float32, seed=SEED, offset=r * n - (k - 1), device=gpu)
                if r > 0 else None)
        y = torch.empty_like(x)
        split_moving_average_into(x, y, k, 1, "blelloch", history=hist)
        del x
        res = oracle_mod.check_synth(y.cpu().numpy(), k, 1, seed=SEED, offset=r * n, rtol=RTOL)
        del y
        assert res["mismatches"] == 0 and res["max_rel"] == 0.0, f"rank {r}/{world}: {res}"
