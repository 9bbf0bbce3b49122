// mavg_kernels.hpp -- hand-written HIP kernels for gfx950 (CDNA4, wave64).
//
// The hot path: causal k-frame moving average over interleaved C-channel
// signals, y[f,c] = S[f,c] / k with S[f,c] = sum_{j<k} x[(f-j)C + c]
// (reference semantics: basics/profilable_moving_averager.cpp:14-37).
// Every scan computes W[n] = W[n-1] + d[n], d[n] = x[n] - x[n-k], with a
// hierarchical scan (serial in-lane over F frames, 64-lane DPP scan, LDS
// exchange of wave-segment totals) and no inter-workgroup communication.
// They replace the reference's multi-launch recursive Blelloch / Hillis-Steele
// pipelines (blelloch_scan_averager.cu:40-186, hillis_steele_averager.cu:17-100).
//
//   mavg_tile.hpp      tile_scan_kernel: one short-lived workgroup per flat
//                      tile; the carry is rebuilt from a k-frame halo staged
//                      in LDS.  The default for windows up to ~16 KiB of halo.
//   mavg_wide.hpp      wide_tile_kernel: the tile scan for multi-channel
//                      frames, lanes own 64/128-B chunks of consecutive
//                      frames read from a swizzled LDS stage.
//   mavg_lookback.hpp  ahead_scan_kernel: one pass over HBM, carry from
//                      whole-tile records that tiles D slots ahead published
//                      inside the launch; windows past the LDS-staged halo,
//                      both flavours (Blelloch and Hillis-Steele in-tile scans).
//   mavg_direct.hpp    direct_kernel: small windows summed directly from LDS
//                      (replaces profilable_sm_*.cu).
//   mavg_misc.hpp      naive_kernel (profilable_parallel_averager.cu:14-23)
//                      and synth_kernel (counter-based synthetic input).
//   mavg_device.hpp    the shared building blocks.
//
// Arithmetic: fp32 data accumulates in fp64 (a global fp32 prefix loses
// 1e-4..1e-1 relative); int16 data accumulates exactly in
// int32 (k <= 65535) or int64, and divides exactly (C++ truncation) with a
// biased fp64 reciprocal product (to_out_i16, proof in its comment, checked by
// tests/test_division.py) -- NOT the reference's float reciprocal, which is
// off on exact multiples.
#pragma once

#include "mavg_device.hpp"
#include "mavg_direct.hpp"
#include "mavg_lookback.hpp"
#include "mavg_misc.hpp"
#include "mavg_tile.hpp"
#include "mavg_wide.hpp"
