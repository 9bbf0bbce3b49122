/*
 * mavg.h -- C ABI of libmavg, the MI355X-native (gfx950) causal moving-average
 * filter.  Plain pointers and sizes only; no HIP, torch or C++ types.
 *
 * This is the in-process replacement for the reference's per-variant
 * "<Variant>GpuLoad" drivers and their kernels:
 *
 *   reference                                              replaced by
 *   ---------------------------------------------------    -------------------------
 *   blellochAveragerGpuLoad  basics/blelloch_scan_averager.cu:189-232        mavg_run(.., MAVG_ALGO_BLELLOCH_SCALAR ..)
 *     recursive_blelloch :134-167, blelloch_scan_inclusive :40-131,
 *     blelloch_uniform_add :17-36, averager_kernel :171-186
 *   blellochAveragerGpuLoad  basics/blelloch_scan_vloaded_averager.cu:183-228 mavg_run(.., MAVG_ALGO_BLELLOCH ..)
 *   hillisSteeleAveragerGpuLoad basics/hillis_steele_averager.cu:221-249     mavg_run(.., MAVG_ALGO_HILLIS_SCALAR ..)
 *   (vloaded)                basics/hillis_steele_vloaded_averager.cu         mavg_run(.., MAVG_ALGO_HILLIS ..)
 *   vload4AveragerGpuLoad    basics/profilable_sm_vload4.cu:91-145            mavg_run(.., MAVG_ALGO_DIRECT ..)
 *   vload2AveragerGpuLoad    basics/profilable_sm_vload2.cu:65-92             mavg_run(.., MAVG_ALGO_DIRECT_VEC2 ..)
 *   sharedMemoryAveragerGpuLoad basics/profilable_sm_averager.cu:48-74       mavg_run(.., MAVG_ALGO_DIRECT_SCALAR ..)
 *   parallelAveragerGpuLoad  basics/profilable_parallel_averager.cu:26-51    mavg_run(.., MAVG_ALGO_NAIVE ..)
 *   DspWorkspace<T,Mode>     gpu_utils.h:67-160 (halo zone, scratch)         caller-owned buffers + d_history
 *                                                                             + mavg_workspace_bytes
 *
 * Semantics (all algorithms, both dtypes) follow the serial reference
 * basics/profilable_moving_averager.cpp:14-37: interleaved frames x[f*C + c],
 * window k ("grade"), frames before the first one read as zero -- or, when
 * d_history is given, as the (k-1)*C samples immediately preceding d_in
 * (the multi-GPU halo; gpu_utils.h:112-123 is the reference's zero halo).
 *   MAVG_I16: y = (int16)(S / k), S the exact int64 window sum, C++ truncating
 *             division.  Bit-exact with the serial reference (the reference's
 *             GPU variants use a float reciprocal and are not).
 *   MAVG_F32: y = (float)(S / k), S accumulated in fp64; within 1e-5 relative
 *             of the fp64 serial restatement.
 *
 * Ownership: the caller owns d_in, d_out, d_history and d_ws (device memory);
 * mavg_run never allocates, never synchronises, never exits, and only
 * enqueues work on `stream` (a hipStream_t; NULL = the legacy default
 * stream), so it can be captured into a HIP graph.  d_in is const (the
 * reference scans in place; this library does not).  Thread-safe and
 * re-entrant; the only process state is per DEVICE (keyed on hipGetDevice):
 * the CU count and, per kernel, whether its dynamic-LDS limit has been raised
 * on that device -- so one process may drive several devices.  (The test
 * hook that forces the look-ahead scan's schedule is process-wide state; it
 * lives in the debug build only, include/mavg_debug.h.)
 */
#ifndef MAVG_H
#define MAVG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAVG_ABI_VERSION 4  /* 2: mavg_plan takes block_size; 3: the schedule test hook moved to mavg_debug.h;
                               4: mavg_build_id */

typedef enum {
    MAVG_I16 = 0, /* int16 PCM in/out (the reference's WAV data path) */
    MAVG_F32 = 1  /* fp32 in/out (BASELINE.json north_star) */
} mavg_dtype;

typedef enum {
    MAVG_ALGO_AUTO = 0,            /* pick by (dtype, k, C): see DESIGN.md */
    MAVG_ALGO_BLELLOCH = 1,        /* single-pass streaming work-efficient scan, 16-B units */
    MAVG_ALGO_BLELLOCH_SCALAR = 2, /* same scan, one frame per lane */
    MAVG_ALGO_HILLIS = 3,          /* streaming Hillis-Steele (log-step) scan, 16-B units */
    MAVG_ALGO_HILLIS_SCALAR = 4,   /* Hillis-Steele, one frame per lane */
    MAVG_ALGO_DIRECT = 5,          /* direct LDS-tiled window sum, 16-B loads (vload4) */
    MAVG_ALGO_DIRECT_VEC2 = 6,     /* direct LDS-tiled, 8-B loads (vload2) */
    MAVG_ALGO_DIRECT_SCALAR = 7,   /* direct LDS-tiled, element loads (shared) */
    MAVG_ALGO_NAIVE = 8            /* one thread per sample, window from global memory */
} mavg_algo;

typedef enum {
    MAVG_OK = 0,
    MAVG_ERR_INVALID_ARG = 1, /* null pointer, k < 1, C < 1, n not a multiple of C, bad enum */
    MAVG_ERR_UNSUPPORTED = 2, /* valid but not implemented (C > 8 outside AUTO/NAIVE, k too large for algo) */
    MAVG_ERR_MISALIGNED = 3,  /* a pointer not aligned to the sample size (2 B int16, 4 B fp32) */
    MAVG_ERR_WORKSPACE = 4,   /* ws_bytes smaller than mavg_workspace_bytes() */
    MAVG_ERR_HIP = 5          /* a HIP runtime call or kernel launch failed */
} mavg_status;

/* Device workspace (bytes) mavg_run needs for this problem, whatever the
 * alignment of the views later passed to mavg_run.  0 for every launch
 * except the look-ahead scan that AUTO/BLELLOCH pick for windows too long
 * for an LDS-staged halo (fp32 halos > 16 KiB, e.g. mono k > 4096; int16 past
 * ~47 KiB): 8-B tagged records, one per (tile, channel, 32-bit word of the
 * tile sum), or one per (tile, wave, ...) for mono windows short enough for
 * per-wave records, padded to 16, + 16, sized for the smaller tiles of the
 * frame-unit form a misaligned view may run (2^30 fp32 mono samples: 64 MiB
 * at k=8192..44100 with per-wave records, 16 MiB at k=10^6 with per-tile
 * records; int16 stereo k=44100: 8 MiB), + the run totals of windows past
 * 384 tiles (8 B per run of G tiles per channel word: < 1 % more).
 * 16-B alignment; contents need no initialisation (mavg_run zeroes them on
 * the stream); one workspace must not serve two launches that may run
 * concurrently. */
int mavg_workspace_bytes(size_t n_samples, int channels, int grade, int dtype,
                         int algo, int block_size, size_t* out_bytes);

/*
 * y[0..n) = moving average of x[0..n), n = frames * channels samples.
 *   d_in/d_out any sample-aligned views (2 B int16, 4 B fp32): a vector
 *              algorithm on views that are not 16-B aligned peels a head of
 *              < 16 B in its one-frame-per-lane form when both views share
 *              the offset, else runs that form over the whole signal.
 *   d_history  NULL (zero history) or (grade-1)*channels samples that
 *              precede d_in (sample-aligned).
 *   block_size the reference's argv block size (a multiple of 32 in
 *              [32, 1024]) or 0 for the tuned geometry.  Non-zero: the naive
 *              kernel runs exactly block_size threads per workgroup; the tile
 *              scans and the direct kernel run the next power of two of at
 *              least one wave64 (64, 128, 256, 512, 1024), while the window's
 *              halo fits that workgroup's LDS (longer windows keep the tuned
 *              look-ahead scan).  mavg_plan() shows the result.
 *   stream     hipStream_t or NULL.
 * Returns a mavg_status.  Nothing is enqueued unless MAVG_OK is returned
 * (MAVG_ERR_HIP excepted, when the launch itself failed).
 */
int mavg_run(const void* d_in, void* d_out, size_t n_samples, int channels,
             int grade, int dtype, int algo, int block_size,
             const void* d_history, void* d_ws, size_t ws_bytes, void* stream);

/* Describe, without launching anything, the kernel and launch geometry
 * mavg_run would use for these arguments on 16-B-aligned views
 * (e.g. "tile_scan<f32,...> grid=... block=256 ..."). */
int mavg_plan(size_t n_samples, int channels, int grade, int dtype, int algo,
              int block_size, char* buf, size_t buflen);

/* The algorithm MAVG_ALGO_AUTO resolves to for these arguments. */
int mavg_resolve_algo(size_t n_samples, int channels, int grade, int dtype, int algo);

/* Counter-based synthetic signal on the device: x[i] for global index
 * offset+i, from splitmix64(seed + offset + i).  dist 0: int16-valued
 * (as int16 or as float); dist 1: uniform [0,1) floats; dist 2: zero-mean,
 * mixed-scale, non-dyadic floats whose fp64 window sums round (the fp32
 * rounding-stress input of the parity tests).  dist 1 and 2: MAVG_F32 only. */
int mavg_fill_synthetic(void* d_out, size_t n_samples, int dtype, uint64_t seed,
                        uint64_t offset, int dist, void* stream);

/* HBM calibration (not part of the filter): d_out = d_in with one flat,
 * non-temporal 16-B load + store per thread, the best copy measured on
 * MI355X.  bench.py times it beside the filter so a result can be
 * read against the same box's achievable streaming rate.  bytes a multiple
 * of 16, both pointers 16-B aligned. */
int mavg_stream_copy(const void* d_in, void* d_out, size_t bytes, void* stream);

const char* mavg_strerror(int status);
const char* mavg_algo_name(int algo);
int mavg_abi_version(void);
/* Source id the library was compiled from: 16 hex digits of a SHA-256 over
 * csrc/ and include/ (digital_signal_processsing_amd/build_id.py, linked in by
 * csrc/Makefile).  Lets a caller prove the loaded library is the tree's. */
const char* mavg_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* MAVG_H */
