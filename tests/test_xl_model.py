"""The frame-piece loads of the halo-only channel-per-lane kernels (csrc/mavg_wide.hpp xl_load /
xl_transpose, csrc/mavg_device.hpp quad_transpose4; DESIGN.md "wide_ahead_kernel", XL) restated
in numpy on the CPU: which 16 bytes each lane loads, the two DPP quad_perm stages with the
kernel's value selects, and the column each lane must end with -- dword cl of frames
j0 .. j0 + P - 1 for lane b*CL + cl, the layout the 4-B column loads produce.  Also the bytes
each wave instruction touches: 64 (CL = 4) or 128 (CL = 8) contiguous per block of lanes instead
of one 16-/32-B piece.  The GPU kernels themselves are checked against the oracle in
tests/test_gpu_parity.py and tests/test_gpu_fullsize.py."""
import numpy as np
import pytest


def quad_perm(v, perm):
    """DPP quad_perm: lane 4j + i reads lane 4j + perm[i] (all lanes valid)."""
    lanes = np.arange(64)
    src = (lanes & ~3) + np.asarray(perm)[lanes & 3]
    return v[src]


def quad_transpose4(a):
    """a: [4][64] registers x lanes; the kernel's two stages, value selects only."""
    a = [r.copy() for r in a]
    q = np.arange(64) & 3
    for s, perm in ((1, (1, 0, 3, 2)), (2, (2, 3, 0, 1))):
        hi_lane = (q & s) != 0
        for e in range(4):
            if e & s:
                continue
            lo, hi = a[e], a[e | s]
            send = np.where(hi_lane, lo, hi)
            got = quad_perm(send, perm)
            a[e] = np.where(hi_lane, got, lo)
            a[e | s] = np.where(hi_lane, hi, got)
    return a


def xl_model(frames_dw, CL, P, f0_of_lane, nframes):
    """frames_dw: [nframes][CL] dwords.  Returns xr [P][64] after xl_load + xl_transpose."""
    lanes = np.arange(64)
    cl = lanes % CL
    last = nframes - 1
    xr = [None] * P
    for m in range(P // 4):
        f = np.minimum(f0_of_lane + 4 * m + (cl & 3), last)
        piece = [frames_dw[f, 4 * (cl >> 2) + q] for q in range(4)]  # the lane's 16 bytes
        t = quad_transpose4(piece)
        for q in range(4):
            xr[4 * m + q] = t[q]
    return xr


@pytest.mark.parametrize("CL,P", [(4, 16), (4, 32), (8, 32), (8, 16)])
def test_frame_pieces_transpose_into_columns(CL, P):
    NB = 64 // CL
    rng = np.random.default_rng(CL * 100 + P)
    WF = NB * P
    nframes = 3 * WF
    frames_dw = rng.integers(0, 2**32, size=(nframes, CL), dtype=np.uint64).astype(np.uint32)
    lanes = np.arange(64)
    for w in range(3):
        j0 = w * WF + (lanes // CL) * P
        xr = xl_model(frames_dw, CL, P, j0, nframes)
        for i in range(P):  # the 4-B column loads: lane b*CL + cl holds dword cl of frame j0 + i
            np.testing.assert_array_equal(xr[i], frames_dw[j0 + i, lanes % CL])


@pytest.mark.parametrize("CL,P", [(4, 32), (8, 32)])
def test_partial_tile_reads_stay_inside_the_signal(CL, P):
    """Frames past the end read the last frame (their outputs are not stored); the frames before
    it arrive exactly as the column loads would deliver them."""
    NB = 64 // CL
    nframes = NB * P - 37
    frames_dw = np.arange(nframes * CL, dtype=np.uint32).reshape(nframes, CL)
    lanes = np.arange(64)
    j0 = (lanes // CL) * P
    xr = xl_model(frames_dw, CL, P, j0, nframes)
    for i in range(P):
        f = j0 + i
        ok = f < nframes
        np.testing.assert_array_equal(xr[i][ok], frames_dw[f[ok], (lanes % CL)[ok]])


@pytest.mark.parametrize("CL,P", [(4, 32), (8, 32)])
def test_wave_instruction_touches_whole_pieces(CL, P):
    """Bytes of one load instruction (fixed m): each block's CL lanes read 4*CL contiguous dwords
    (64 or 128 B), the 4-B column loads one frame's CL dwords per instruction in 4-B pieces."""
    lanes = np.arange(64)
    cl, b = lanes % CL, lanes // CL
    for m in range(P // 4):
        f = b * P + 4 * m + (cl & 3)
        dw0 = f * CL + 4 * (cl >> 2)   # first dword of the lane's 16 bytes
        for blk in range(64 // CL):
            d = np.sort(np.concatenate([dw0[b == blk] + q for q in range(4)]))
            assert np.array_equal(d, np.arange(d[0], d[0] + 4 * CL)), (m, blk)
            assert d[0] % (4 * CL) == 0  # the piece starts on its own size (64 / 128 B)
