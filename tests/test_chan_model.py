"""The channel-per-lane tile (csrc/mavg_wide.hpp chan_tile_kernel), its index
math restated in numpy on the CPU: the swizzled stage (chan_slot), the halo
reduction, the per-lane in-channel sums over Q frames, the Kogge-Stone scan
across the NB lanes of a channel (steps of C, 2C, ... lanes: whole-wave
shifts, which is why the kernel uses ds_bpermute and not row_shr DPP), the
wave-segment carry, the rebuilt prefix and the readback of the outputs.  The
restatement must equal the oracle's moving average; the GPU kernel itself is
checked against the oracle in tests/test_gpu_parity.py."""
import numpy as np
import pytest

from test_lds_layout import chan_slot


def chan_tile_model(x, k, C, Q, WG):
    """eb = x's sample size: 4 (fp32, a lane owns one channel) or 2 (int16, a lane owns a dword
    column of two channels, E = 2 accumulators, exact integer sums and truncating division)."""
    eb = x.dtype.itemsize
    E = 4 // eb                      # channels per dword column
    CL = C // E                      # dword columns per frame
    nframes = len(x) // C
    NW, NB, GPF = WG // 64, 64 // CL, CL // 4
    WF, EPG = NB * Q, 16 // eb
    TF = NW * WF
    TG = TF * GPF
    Hg = ((k * C + EPG - 1) // EPG + 15) // 16 * 16
    Hf = Hg * EPG // C
    acc = np.float64 if eb == 4 else np.int64
    xs = x.reshape(-1, C).astype(acc)
    out = np.zeros(xs.shape, dtype=np.float64 if eb == 4 else np.int16)
    lanes = np.arange(64)
    col_of, b_of = lanes % CL, lanes // CL
    for tile in range((nframes + TF - 1) // TF):
        t0, h0 = tile * TF, tile * TF - Hf
        stage = np.zeros((Hg + TG) * EPG, dtype=acc)
        e = np.arange((Hg + TG) * EPG)
        f, c = h0 + e // C, e % C
        ok = (f >= 0) & (f < nframes)
        vals = np.where(ok, xs[np.clip(f, 0, nframes - 1), c], 0)
        slots = np.array([chan_slot(g, CL, Q) for g in range(Hg + TG)])
        stage[slots[e // EPG] * EPG + e % EPG] = vals  # logical granule g lives in slot chan_slot(g)

        def elem(ei):  # stage sample ei (frame * C + channel)
            return stage[slots[ei // EPG] * EPG + ei % EPG]

        W = np.zeros(C, dtype=acc)
        for ei in range((Hf - k) * C, Hf * C):
            W[ei % C] += elem(ei)
        for ee in range(E):
            ch = col_of * E + ee           # the channel each lane accumulates
            run = np.zeros((NW, 64), dtype=acc)
            for w in range(NW):
                f0 = Hf + w * WF + b_of * Q
                for i in range(Q):
                    run[w] += elem((f0 + i) * C + ch) - elem((f0 + i - k) * C + ch)
            incl, s = run.copy(), CL
            while s < 64:  # whole-wave shifts: lane l takes lane l - s
                t = np.zeros_like(incl)
                t[:, s:] = incl[:, :-s]
                incl += t
                s <<= 1
            tot = incl[:, 64 - CL:]  # [wave][column]: the last block's lanes
            for w in range(NW):
                base = W[ch] + sum(tot[i, col_of] for i in range(w)) + incl[w] - run[w]
                f0 = Hf + w * WF + b_of * Q
                for i in range(Q):
                    base = base + elem((f0 + i) * C + ch) - elem((f0 + i - k) * C + ch)
                    fr = t0 + w * WF + b_of * Q + i
                    m = fr < nframes
                    if eb == 4:
                        out[fr[m], ch[m]] = base[m] / k
                    else:  # C++ truncating division
                        q = np.abs(base[m]) // k
                        out[fr[m], ch[m]] = np.where(base[m] < 0, -q, q)
    return out.reshape(-1)


@pytest.mark.parametrize("C,Q,WG,k", [(8, 32, 256, 7), (8, 32, 256, 1024), (8, 32, 128, 100), (8, 16, 512, 513),
                                      (4, 16, 256, 37), (4, 32, 256, 700)])
def test_chan_tile_model_equals_the_oracle(oracle_mod, C, Q, WG, k):
    frames = (64 // C) * Q * (WG // 64) * 3 + 77  # three tiles and a ragged tail
    x = oracle_mod.synth_f32(frames * C, seed=C + k, dist=1)
    got = chan_tile_model(x, k, C, Q, WG)
    ref = oracle_mod.mavg_f32(x, k, C).astype(np.float64)
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-6), np.abs(got - ref).max()


@pytest.mark.parametrize("Q,WG,k", [(32, 256, 2048), (32, 256, 3000), (16, 256, 1024), (16, 128, 77)])
def test_chan_tile_model_int16_dword_columns(oracle_mod, Q, WG, k):
    """int16 with 8 channels: a lane owns a dword column (two channels), the fp32 C = 4
    addressing, bit-exact with the oracle."""
    C = 8
    frames = 16 * Q * (WG // 64) * 3 + 77
    x = oracle_mod.synth_i16(frames * C, seed=k)
    assert np.array_equal(chan_tile_model(x, k, C, Q, WG), oracle_mod.mavg_i16(x, k, C))


@pytest.mark.parametrize("CL,P", [(8, 32), (4, 32), (4, 16)])
def test_wide_ahead_offset_table_is_chan_slot(CL, P):
    """wide_ahead_kernel's CH addressing (ch_table / ch_idx): element (frame j0 + i, column cl) of a
    chan_slot stage at float index tb[i mod NBX] + (i / NBX) NBX 4 GPF, tb[r] = lb + (r ^ bq) 4 GPF --
    the same index as chan_slot for every lane, wave and frame of the lane's block."""
    NB, GPF = 64 // CL, CL // 4
    NBX = min(NB, P)
    for w in range(4):
        for lane in range(64):
            cl, bq = lane % CL, lane // CL
            j0 = w * NB * P + bq * P
            lb = (j0 * GPF + (cl >> 2)) * 4 + (cl & 3)
            tb = [lb + (r ^ bq) * 4 * GPF for r in range(NBX)]
            for i in range(P):
                d = (j0 + i) * CL + cl
                assert tb[i % NBX] + (i // NBX) * NBX * 4 * GPF == chan_slot(d >> 2, CL, P) * 4 + (d & 3)


def test_row_local_shifts_would_be_wrong(oracle_mod):
    """The first GPU build shifted by row_shr (inside 16-lane rows): every even
    frame block but the first lost its predecessor.  The model reproduces that
    failure, so the test above really exercises the cross-row steps."""
    C, s = 8, 8
    run = np.arange(64, dtype=np.float64)
    t = np.zeros(64)
    for l in range(64):
        if l % 16 >= s:
            t[l] = run[l - s]
    wrong = run + t
    right = run.copy()
    right[s:] += run[:-s]
    assert not np.array_equal(wrong, right) and np.array_equal(wrong[:16], right[:16])
