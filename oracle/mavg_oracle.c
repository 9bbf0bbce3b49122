/*
 * mavg_oracle.c -- CPU restatement of the reference moving-average filter.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libmavg, the bin_* CLIs,
 * the Python package) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 * as the checker / the timed CPU baseline.
 *
 * PARITY STATUS: unpinned against an executed reference.  The reference's own
 * CPU averager (basics/profilable_moving_averager.cpp) does not compile as
 * shipped (no closing brace after :83; benchmark.h:5 and gpu_utils.h:2
 * include <cuda_runtime.h>, absent here) and the reference holds no tests,
 * golden vectors or fixtures.  This restatement follows
 * the reference loop statement by statement and is cross-checked against an
 * independent numpy formulation and closed-form known answers in tests/.
 *
 * Semantics (basics/profilable_moving_averager.cpp:14-37):
 *   samples are interleaved frames x[f*C + c]; window length k ("point");
 *   per channel a running int64 sum; warm-up loop :19-25 adds frames 0..k-1
 *   and divides by k (not by the number of frames seen); steady loop :27-35
 *   subtracts frame f-k then adds frame f; output = (int16)(sum / k) with
 *   C++ truncating int64 division.
 *
 * fp32 mode (BASELINE.json north_star): the same loop with a double running
 * sum over float inputs and output (float)(sum / k) -- SURVEY.md section 8c.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>

#define ORACLE_MAX_CH 64

/* Follows profilable_moving_averager.cpp:14-37.  Returns 0, or -1 on bad args.
 * Deviation (documented): the warm-up loop is clamped to the frame count; the
 * reference reads past the end when k > frames (:19-23, undefined behaviour). */
int oracle_mavg_i16(const int16_t* x, int16_t* y, size_t n, int C, int k)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || (n % (size_t)C) != 0) return -1;
    const size_t frames = n / (size_t)C;                 /* :16 */
    int64_t sum[ORACLE_MAX_CH];                          /* :17 */
    memset(sum, 0, sizeof(sum));
    const size_t warm = (size_t)k < frames ? (size_t)k : frames;
    for (size_t i = 0; i < warm; ++i) {                  /* :19 */
        for (int ch = 0; ch < C; ++ch) {                 /* :20 */
            sum[ch] += x[i * C + ch];                    /* :21-22 */
            y[i * C + ch] = (int16_t)(sum[ch] / k);      /* :23 */
        }
    }
    for (size_t i = (size_t)k; i < frames; ++i) {        /* :27 */
        for (int ch = 0; ch < C; ++ch) {                 /* :28 */
            sum[ch] -= x[(i - (size_t)k) * C + ch];      /* :30-31 */
            sum[ch] += x[i * C + ch];                    /* :29,32 */
            y[i * C + ch] = (int16_t)(sum[ch] / k);      /* :33 */
        }
    }
    return 0;
}

/* fp32 mode: same loop structure, double running sum, float(sum / k). */
int oracle_mavg_f32(const float* x, float* y, size_t n, int C, int k)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || (n % (size_t)C) != 0) return -1;
    const size_t frames = n / (size_t)C;
    double sum[ORACLE_MAX_CH];
    for (int ch = 0; ch < C; ++ch) sum[ch] = 0.0;
    const double dk = (double)k;
    const size_t warm = (size_t)k < frames ? (size_t)k : frames;
    for (size_t i = 0; i < warm; ++i)
        for (int ch = 0; ch < C; ++ch) {
            sum[ch] += (double)x[i * C + ch];
            y[i * C + ch] = (float)(sum[ch] / dk);
        }
    for (size_t i = (size_t)k; i < frames; ++i)
        for (int ch = 0; ch < C; ++ch) {
            sum[ch] -= (double)x[(i - (size_t)k) * C + ch];
            sum[ch] += (double)x[i * C + ch];
            y[i * C + ch] = (float)(sum[ch] / dk);
        }
    return 0;
}

/* Exact windowed sums (int64) for a sub-range of frames [f0, f1) of a signal
 * whose frames before 0 are zero: used by tests to check arbitrary slices
 * (e.g. shard boundaries) of a long signal without running the whole loop. */
int oracle_window_sum_i64(const int16_t* x, size_t n, int C, int k,
                          size_t f0, size_t f1, int64_t* out)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || (n % (size_t)C) != 0) return -1;
    const size_t frames = n / (size_t)C;
    if (f1 > frames || f0 > f1) return -1;
    for (int ch = 0; ch < C; ++ch) {
        int64_t s = 0;
        size_t lo = f0 + 1 > (size_t)k ? f0 + 1 - (size_t)k : 0;
        for (size_t j = lo; j <= f0 && f0 < f1; ++j) s += x[j * C + ch];
        for (size_t f = f0; f < f1; ++f) {
            if (f > f0) {
                s += x[f * C + ch];
                if (f >= (size_t)k) s -= x[(f - (size_t)k) * C + ch];
            }
            out[(f - f0) * C + ch] = s;
        }
    }
    return 0;
}

/* ---- counter-based synthetic input ----------------------
 * x[i] = (int16)(splitmix64(seed + i) >> 48); the GPU generator in
 * libmavg computes the identical sequence so any sub-range can be regenerated
 * on the host.  dist 0: int16-valued; dist 1: uniform [0,1) with 24-bit
 * mantissa (precision stress, parity tests only); dist 2: zero-mean,
 * mixed-scale, non-dyadic fp32 (synth_f32_dist2: rounding and cancellation
 * stress at full size). */
static inline uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* dist 2.  i = (sum of the four 14-bit fields of h) - 32766: an Irwin-Hall
 * integer in [-32766, 32766], symmetric about 0.  v = fl64(i * fl64(1/3000))
 * (a full 24-bit fp32 mantissa after rounding: the values are not dyadic
 * fractions with short expansions), scaled by 2^-s with s = max(0, b - 8), b
 * the 5 bits above the fields (a quarter of the samples at full scale, the rest
 * spread over 2^-1 .. 2^-23), then rounded to fp32.  Window sums then mix
 * magnitudes 2^3 .. 2^-35 and cancel towards 0, so fp64 accumulation rounds.
 * Every step is one correctly rounded IEEE operation (no fused or reassociated
 * arithmetic), so the device generator (synth_kernel) matches it bit for bit.
 * Smallest non-zero |x| is 2^-23/3000 > 2^-41: x * 2^64 is an integer (the
 * exact checker below relies on it). */
static inline float synth_f32_dist2(uint64_t h)
{
    const int64_t i = (int64_t)(h & 0x3fffu) + (int64_t)((h >> 14) & 0x3fffu) +
                      (int64_t)((h >> 28) & 0x3fffu) + (int64_t)((h >> 42) & 0x3fffu) - 32766;
    const int b = (int)((h >> 56) & 31u);
    const int s = b < 8 ? 0 : b - 8;
    uint64_t pbits = (uint64_t)(1023 - s) << 52;   /* 2^-s, exactly */
    double p;
    memcpy(&p, &pbits, sizeof p);
    const double v = (double)i * (1.0 / 3000.0);
    return (float)(v * p);
}

static inline float synth_f32_at(uint64_t seed, uint64_t i, int dist)
{
    uint64_t h = splitmix64(seed + i);
    if (dist == 1) return (float)(h >> 40) * (1.0f / 16777216.0f);
    if (dist == 2) return synth_f32_dist2(h);
    return (float)(int16_t)(uint16_t)(h >> 48);
}

void oracle_synth_i16(int16_t* x, size_t n, uint64_t seed, uint64_t offset)
{
    for (size_t i = 0; i < n; ++i)
        x[i] = (int16_t)(uint16_t)(splitmix64(seed + offset + i) >> 48);
}

void oracle_synth_f32(float* x, size_t n, uint64_t seed, uint64_t offset, int dist)
{
    for (size_t i = 0; i < n; ++i) x[i] = synth_f32_at(seed, offset + i, dist);
}

/* ---- multi-core CPU baseline --------------------------
 * Same arithmetic as oracle_mavg_f32, split into `threads` contiguous frame
 * chunks; each chunk seeds its running sums from the k frames before it
 * (the CPU analogue of the GPU tiles' halo).  Results equal the serial loop
 * up to fp64 summation order.  Reported beside the single-core baseline,
 * never used as a checker. */
#ifdef _OPENMP
#include <omp.h>
#endif
int oracle_mavg_f32_mt(const float* x, float* y, size_t n, int C, int k, int threads)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || (n % (size_t)C) != 0 || threads < 1) return -1;
    const size_t frames = n / (size_t)C;
    const double dk = (double)k;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int t = 0; t < threads; ++t) {
        const size_t f0 = frames * (size_t)t / (size_t)threads;
        const size_t f1 = frames * (size_t)(t + 1) / (size_t)threads;
        double sum[ORACLE_MAX_CH];
        for (int ch = 0; ch < C; ++ch) {
            double s = 0.0;
            /* the k frames before f0: the first step below subtracts x[f0-k] */
            const size_t lo = f0 > (size_t)k ? f0 - (size_t)k : 0;
            for (size_t j = lo; j < f0; ++j) s += (double)x[j * C + ch];
            sum[ch] = s;
        }
        for (size_t i = f0; i < f1; ++i)
            for (int ch = 0; ch < C; ++ch) {
                sum[ch] += (double)x[i * C + ch];
                if (i >= (size_t)k) sum[ch] -= (double)x[(i - (size_t)k) * C + ch];
                y[i * C + ch] = (float)(sum[ch] / dk);
            }
    }
    return 0;
}

/* ---- full-signal checkers over the synthetic stream ------------------------
 * Compare a device output y (frames [g0, g0 + n/C) of the global counter-based
 * stream, g0 = offset / C, zero history before global frame 0) against the
 * restatement above WITHOUT materialising x: each sample is regenerated from
 * its counter.  The frames are split into `threads` contiguous chunks, each
 * seeded with the window sum of the k-1 frames before it.  This equals the
 * serial loop (oracle_mavg_f32 / oracle_mavg_i16) exactly: int16 sums are
 * integers, and every fp64 partial sum of dist-0 (int16-valued) or dist-1
 * (multiples of 2^-24 below 1) samples is a multiple of 2^-24 below 2^29 in
 * magnitude for k < 2^29, so fp64 adds them without rounding in any order.
 * Used by the -m gpu full-size parity tests (every output of a 2^30 launch).
 * dist 2 (inexact in fp64) has its own checker: oracle_check_synth_f32_exact. */
int oracle_check_synth_f32(const float* y, size_t n, int C, int k, uint64_t seed, uint64_t offset,
                           int dist, double rtol, int threads,
                           uint64_t* n_bad, uint64_t* first_bad, double* max_rel)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || k >= (1 << 29) || (n % (size_t)C) != 0 ||
        (offset % (uint64_t)C) != 0 || threads < 1 || (dist != 0 && dist != 1))
        return -1;
    const size_t frames = n / (size_t)C;
    const uint64_t g0 = offset / (uint64_t)C;
    const double dk = (double)k;
    uint64_t bad_total = 0, first = UINT64_MAX;
    double worst = 0.0;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad_total) \
    reduction(min : first) reduction(max : worst)
    for (int t = 0; t < threads; ++t) {
        const size_t f0 = frames * (size_t)t / (size_t)threads;
        const size_t f1 = frames * (size_t)(t + 1) / (size_t)threads;
        for (int ch = 0; ch < C; ++ch) {
            /* window sum of the k global frames [g-k, g-1] before g = g0 + f0:
             * the first step below adds frame g and subtracts frame g-k */
            const uint64_t g = g0 + f0;
            const uint64_t lo = g >= (uint64_t)k ? g - (uint64_t)k : 0;
            double s = 0.0;
            for (uint64_t j = lo; j < g; ++j) s += (double)synth_f32_at(seed, j * C + ch, dist);
            for (size_t f = f0; f < f1; ++f) {
                const uint64_t gf = g0 + f;
                s += (double)synth_f32_at(seed, gf * C + ch, dist);
                if (gf >= (uint64_t)k) s -= (double)synth_f32_at(seed, (gf - k) * C + ch, dist);
                const double want = (double)(float)(s / dk);
                const double got = (double)y[f * C + ch];
                const double err = fabs(got - want);
                const double den = fabs(want) > 1e-30 ? fabs(want) : 1e-30;
                const double rel = err / den;
                if (!(err <= rtol * den)) {   /* NaN-safe */
                    ++bad_total;
                    if ((uint64_t)(f * C + ch) < first) first = (uint64_t)(f * C + ch);
                }
                if (rel > worst || rel != rel) worst = rel != rel ? INFINITY : rel;
            }
        }
    }
    *n_bad = bad_total;
    *first_bad = first;
    *max_rel = worst;
    return 0;
}

/* ---- exact fp32 checker (any dist) -----------------------------------------
 * The reference loop (profilable_moving_averager.cpp:27-35) keeps a running
 * sum; in fp32 mode its fp64 running sum rounds once the samples are not
 * small integers (dist 2), and over 2^30 steps that drift is not a usable
 * yardstick.  This checker uses the EXACT window sum instead: every sample is
 * an integer multiple of 2^-64 below 2^32 in magnitude (checked: the function
 * returns -2 otherwise), so S = sum of x * 2^64 is exact in __int128 (|S| <
 * 2^96 * 2^27 for k < 2^27).  want = S / k (one fp64 rounding of S, one of the
 * quotient: relative error < 2^-52).  For each output:
 *   err <= rtol * |want|                  passes (relative bar, north_star)
 *   else err <= rtol * F, F = sum|x| / k  passes on the floor (|want| ~ 0:
 *                                         the window's mean absolute input),
 *                                         counted in stats[2]
 *   else                                  a mismatch (stats[0], first in stats[1]).
 * stats[3] counts outputs that are not the correctly rounded fp32 of want.
 * dstats[0] = max err / |want| over want != 0; dstats[1] = max err / F (the
 * error against the summation's condition scale: fp32 output rounding alone
 * contributes up to 2^-24). */
static inline int fx64(float x, __int128* out)
{
    uint32_t u;
    memcpy(&u, &x, sizeof u);
    const int e = (int)((u >> 23) & 0xffu);
    if (e == 255) return -1;                             /* inf / NaN */
    const int64_t m = e ? (int64_t)((u & 0x7fffffu) | 0x800000u) : (int64_t)(u & 0x7fffffu);
    const int sh = (e ? e : 1) - 150 + 64;               /* x = m 2^(e-150): x 2^64 = m 2^sh */
    __int128 v;
    if (m == 0) { *out = 0; return 0; }
    if (sh >= 0) {
        if (sh > 72) return -1;                          /* |x| >= 2^32: the window sums could overflow */
        v = (__int128)m << sh;
    } else {
        if (sh < -24 || (m & ((INT64_C(1) << -sh) - 1)) != 0) return -1;   /* not a multiple of 2^-64 */
        v = (__int128)(m >> -sh);
    }
    *out = (u >> 31) ? -v : v;
    return 0;
}
/* (double) of an __int128 without the library call: the magnitude's two
 * halves, one rounding each, then the sum (relative error < 2^-51 for either
 * sign) */
static inline double i128_to_double(__int128 s)
{
    /* magnitude first, then the sign: (double)hi * 2^64 + (double)lo with a
     * negative hi cancels catastrophically for small |s| (s = -5: hi = -1,
     * lo = 2^64 - 5 rounds to 2^64, the sum to 0) */
    const int neg = s < 0;
    const unsigned __int128 u = neg ? -(unsigned __int128)s : (unsigned __int128)s;
    const double d = (double)(uint64_t)(u >> 64) * 0x1p64 + (double)(uint64_t)u;
    return neg ? -d : d;
}

int oracle_check_synth_f32_exact(const float* y, size_t n, int C, int k, uint64_t seed, uint64_t offset,
                                 int dist, double rtol, int threads, uint64_t* stats, double* dstats)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || k >= (1 << 27) || (n % (size_t)C) != 0 ||
        (offset % (uint64_t)C) != 0 || threads < 1 || dist < 0 || dist > 2)
        return -1;
    const size_t frames = n / (size_t)C;
    const uint64_t g0 = offset / (uint64_t)C;
    const double dk = (double)k;
    uint64_t bad_total = 0, first = UINT64_MAX, floor_total = 0, ncr_total = 0;
    double worst_rel = 0.0, worst_cond = 0.0;
    int failed = 0;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad_total, floor_total, ncr_total) \
    reduction(min : first) reduction(max : worst_rel, worst_cond, failed)
    for (int t = 0; t < threads; ++t) {
        const size_t f0 = frames * (size_t)t / (size_t)threads;
        const size_t f1 = frames * (size_t)(t + 1) / (size_t)threads;
        int fail_t = 0;
        for (int ch = 0; ch < C && !fail_t; ++ch) {
            const uint64_t g = g0 + f0;
            const uint64_t lo = g >= (uint64_t)k ? g - (uint64_t)k : 0;
            __int128 s = 0, sa = 0, v;
            for (uint64_t j = lo; j < g; ++j) {
                if (fx64(synth_f32_at(seed, j * C + ch, dist), &v)) { fail_t = 1; break; }
                s += v;
                sa += v < 0 ? -v : v;
            }
            for (size_t f = f0; f < f1 && !fail_t; ++f) {
                const uint64_t gf = g0 + f;
                if (fx64(synth_f32_at(seed, gf * C + ch, dist), &v)) { fail_t = 1; break; }
                s += v;
                sa += v < 0 ? -v : v;
                if (gf >= (uint64_t)k) {
                    if (fx64(synth_f32_at(seed, (gf - k) * C + ch, dist), &v)) { fail_t = 1; break; }
                    s -= v;
                    sa -= v < 0 ? -v : v;
                }
                const double want = i128_to_double(s) * 0x1p-64 / dk;
                const double fl = i128_to_double(sa) * 0x1p-64 / dk;
                const double got = (double)y[f * C + ch];
                const double err = fabs(got - want);
                const uint64_t idx = (uint64_t)(f * C + ch);
                if (err <= rtol * fabs(want)) {
                    /* relative bar */
                } else if (err <= rtol * fl) {
                    ++floor_total;
                } else {            /* also NaN */
                    ++bad_total;
                    if (idx < first) first = idx;
                }
                if ((float)want != (float)got) ++ncr_total;
                if (want != 0.0) {
                    const double r = err / fabs(want);
                    if (r > worst_rel || r != r) worst_rel = r != r ? INFINITY : r;
                }
                if (fl > 0.0) {
                    const double r = err / fl;
                    if (r > worst_cond || r != r) worst_cond = r != r ? INFINITY : r;
                } else if (err != 0.0) {
                    worst_cond = INFINITY;
                }
            }
        }
        if (fail_t) failed = 1;
    }
    if (failed > 0) return -2;
    stats[0] = bad_total;
    stats[1] = first;
    stats[2] = floor_total;
    stats[3] = ncr_total;
    dstats[0] = worst_rel;
    dstats[1] = worst_cond;
    return 0;
}

int oracle_check_synth_i16(const int16_t* y, size_t n, int C, int k, uint64_t seed, uint64_t offset,
                           int threads, uint64_t* n_bad, uint64_t* first_bad)
{
    if (C < 1 || C > ORACLE_MAX_CH || k < 1 || (n % (size_t)C) != 0 || (offset % (uint64_t)C) != 0 ||
        threads < 1)
        return -1;
    const size_t frames = n / (size_t)C;
    const uint64_t g0 = offset / (uint64_t)C;
    uint64_t bad_total = 0, first = UINT64_MAX;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad_total) reduction(min : first)
    for (int t = 0; t < threads; ++t) {
        const size_t f0 = frames * (size_t)t / (size_t)threads;
        const size_t f1 = frames * (size_t)(t + 1) / (size_t)threads;
        for (int ch = 0; ch < C; ++ch) {
            const uint64_t g = g0 + f0;
            const uint64_t lo = g >= (uint64_t)k ? g - (uint64_t)k : 0;
            int64_t s = 0;
            for (uint64_t j = lo; j < g; ++j) s += (int16_t)(uint16_t)(splitmix64(seed + j * C + ch) >> 48);
            for (size_t f = f0; f < f1; ++f) {
                const uint64_t gf = g0 + f;
                s += (int16_t)(uint16_t)(splitmix64(seed + gf * C + ch) >> 48);
                if (gf >= (uint64_t)k) s -= (int16_t)(uint16_t)(splitmix64(seed + (gf - k) * C + ch) >> 48);
                if (y[f * C + ch] != (int16_t)(s / k)) {
                    ++bad_total;
                    if ((uint64_t)(f * C + ch) < first) first = (uint64_t)(f * C + ch);
                }
            }
        }
    }
    *n_bad = bad_total;
    *first_bad = first;
    return 0;
}
