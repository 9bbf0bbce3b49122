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
    nframes = len(x) // C
    NW, NB, GPF = WG // 64, 64 // C, C // 4
    WF, EPG = NB * Q, 4
    TF = NW * WF
    TG = TF * GPF
    Hg = ((k * C + EPG - 1) // EPG + 15) // 16 * 16
    Hf = Hg * EPG // C
    xs = x.reshape(-1, C).astype(np.float64)
    out = np.zeros_like(xs)
    lanes = np.arange(64)
    c_of, b_of = lanes % C, lanes // C
    for tile in range((nframes + TF - 1) // TF):
        t0, h0 = tile * TF, tile * TF - Hf
        stage = np.zeros((Hg + TG) * EPG)
        e = np.arange((Hg + TG) * EPG)
        f, c = h0 + e // C, e % C
        ok = (f >= 0) & (f < nframes)
        vals = np.where(ok, xs[np.clip(f, 0, nframes - 1), c], 0.0)
        slots = np.array([chan_slot(g, C, Q) for g in range(Hg + TG)])
        stage[slots[e // EPG] * EPG + e % EPG] = vals  # logical granule g lives in slot chan_slot(g)

        def elem(ei):
            return stage[slots[ei >> 2] * 4 + (ei & 3)]

        W = np.zeros(C)
        for ei in range((Hf - k) * C, Hf * C):
            W[ei % C] += elem(ei)
        run = np.zeros((NW, 64))
        for w in range(NW):
            f0 = Hf + w * WF + b_of * Q
            for i in range(Q):
                run[w] += elem((f0 + i) * C + c_of) - elem((f0 + i - k) * C + c_of)
        incl, s = run.copy(), C
        while s < 64:  # whole-wave shifts: lane l takes lane l - s
            t = np.zeros_like(incl)
            t[:, s:] = incl[:, :-s]
            incl += t
            s <<= 1
        tot = incl[:, 64 - C:]  # [wave][channel]: the last block's lanes
        for w in range(NW):
            base = W[c_of] + sum(tot[i, c_of] for i in range(w)) + incl[w] - run[w]
            f0 = Hf + w * WF + b_of * Q
            for i in range(Q):
                base = base + elem((f0 + i) * C + c_of) - elem((f0 + i - k) * C + c_of)
                fr = t0 + w * WF + b_of * Q + i
                m = fr < nframes
                out[fr[m], c_of[m]] = base[m] / k
    return out.reshape(-1)


@pytest.mark.parametrize("C,Q,WG,k", [(8, 32, 256, 7), (8, 32, 256, 1024), (8, 32, 128, 100), (8, 16, 512, 513),
                                      (4, 16, 256, 37), (4, 32, 256, 700)])
def test_chan_tile_model_equals_the_oracle(oracle_mod, C, Q, WG, k):
    frames = (64 // C) * Q * (WG // 64) * 3 + 77  # three tiles and a ragged tail
    x = oracle_mod.synth_f32(frames * C, seed=C + k, dist=1)
    got = chan_tile_model(x, k, C, Q, WG)
    ref = oracle_mod.mavg_f32(x, k, C).astype(np.float64)
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-6), np.abs(got - ref).max()


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
