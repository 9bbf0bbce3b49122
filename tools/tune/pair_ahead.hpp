// pair_ahead.hpp -- round-6 experiment, tuner only (tools/tune/wide_ab.hip "pair"): the paired
// look-ahead scan (pair_ahead_kernel), the halo-only channel-per-lane look-ahead of
// mavg_wide.hpp (wide_ahead_kernel, CH + XG) with TWO consecutive tiles per workgroup, whose
// bytes are all in flight at once.  Not in the library: it measured a tie at best against the
// one-tile kernel in 2048-frame tiles (profiles/r06_tuning/pair/, xl/).
#pragma once

#include "../../digital_signal_processsing_amd/csrc/mavg_launch.hpp"

namespace mavg {

// ----------------------------------------------------------------------------
// Why (round 6).  The phase trace of the one-tile look-ahead (profiles/r05_tuning/trace/) puts a
// tile's life at 11-15 us, a third of it phase A's HBM read and another quarter the output issue,
// with 4-5 workgroups per CU: each CU keeps only a few tiles' bytes in flight, and every tile
// pays one HBM latency and one record wait of its own.  Here a workgroup takes the two
// consecutive dispatch slots of its XCD's run that hold tiles t and t + 1 and issues every load
// of both before its first barrier -- both tiles' x (registers), both shifted stages (LDS-DMA,
// two buffers) and both phase-A tiles -- so one HBM latency and one record wait serve two tiles:
//   tile t      the one-tile kernel's carry: the records of the whole tiles inside its window,
//               plus the partial window, plus the history;
//   tile t + 1  no records at all: its carry is tile t's window sum at its last frame, which
//               pass 2 of tile t has just formed (W[t0 + T - 1] = W[t0 - 1] + sum of d over
//               tile t), handed over in LDS.
// The records stay per tile and per virtual slot: slot v = 8 (2 i + s) + x for workgroup
// b = 8 i + x (XCD x = b mod 8) and s = 0, 1 -- the same slot -> tile map (remap mode 1), the
// same producer for each record (the workgroup holding slot v - D), own records for v < D and
// head duty, as the one-tile kernel, so records keep their bits (and the recompute path its
// order) whatever the schedule.  Tile t + 1's carry is a fixed function of tile t's (the pairs
// are fixed by the grid): bitwise the same output under every schedule (forced-schedule tests).
// fp32 tile t + 1 sums differently from the one-tile kernel (one chained carry instead of
// records); within the parity bar like any other decomposition.
// Windows short of the L2 reach only (remap mode 1: consecutive slots of a run hold consecutive
// tiles).
// ----------------------------------------------------------------------------
// XL: x as 16-B frame loads plus quad transposes (mavg_wide.hpp xl_load; 16-B frames)
template <typename T, typename A, int C, int P, int WG, int NT, int DV, int U, int XL = 0>
__global__ __launch_bounds__(WG) void pair_ahead_kernel(AheadParams p) {
  constexpr int F = 1;
  constexpr int NW = WG / 64;
  constexpr int EPG = 16 / (int)sizeof(T);
  using CEl = ChanElem<T>;
  constexpr int E = CEl::E;
  constexpr int CL = C / E;  // dword columns per frame (a lane owns one)
  static_assert(C % E == 0 && (CL == 4 || CL == 8), "16- or 32-B frames");
  constexpr int NB = 64 / CL;   // frame blocks per wave
  constexpr int WF = NB * P;    // frames per wave
  constexpr int TF = NW * WF;   // frames per tile
  static_assert(TF == WG * F * U, "the record units tile the same frames as the columns");
  constexpr int TG = TF * C / EPG;  // tile granules
  constexpr int SG = TG + 1;        // shifted-stage granules
  constexpr int VE = F * C;
  using IO = UnitIO<T, VE>;
  using GIO = UnitIO<T, EPG>;
  using Gr = Unit<T, EPG>;
  using SA = typename ScanAcc<T, A>::type;
  constexpr int NG = GranCount<SA>::n;
  constexpr int NSRC = 6;  // per tile: phase A, own record, head duty

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* sst[2] = {smem, smem + SG * 16};                     // shifted stages (then the outputs)
  A* hsum = reinterpret_cast<A*>(smem + 2 * SG * 16);                 // [NW][C] tile t's carry shares
  A* carry2 = hsum + NW * C;                                          // [C] W at tile t's last frame
  SA* tot = reinterpret_cast<SA*>(carry2 + C);                        // [2][NW][C] wave totals of d
  SA* shares = tot + 2 * NW * C;                                      // [NSRC][NW][C]

  const T* __restrict__ in = static_cast<const T*>(p.in);
  T* __restrict__ out = static_cast<T*>(p.out);
  const T* __restrict__ hist = static_cast<const T*>(p.hist);
  gran_t* gran = (gran_t*)p.gran;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  const int k = p.k;
  const long long nframes = p.nframes;
  const int pre = p.pre;

  // virtual slots: workgroup b = 8 i + x holds slots 8 (2 i + s) + x, s = 0, 1 (XCD x, consecutive
  // positions 2 i, 2 i + 1 of its run)
  const unsigned nbv = (unsigned)((nframes + TF - 1) / TF);
  const unsigned vs0 = ((blockIdx.x >> 3) * 2u) * 8u + (blockIdx.x & 7u);
  if (vs0 >= nbv) return;  // the whole workgroup: no slot, no record duty
  const unsigned vs1 = vs0 + 8u;
  const bool has2 = vs1 < nbv;
  const long long tile0 = remap_tile(vs0, nbv, 1);
  const long long t00 = tile0 * TF;
  const long long t01 = t00 + TF;  // tile t + 1 (mode 1: the next slot of the run is the next tile)
  MAVG_DCHECK(!has2 || remap_tile(vs1, nbv, 1) == tile0 + 1, "pair: consecutive tiles", tile0, vs1);
  MAVG_DCHECK(t00 < nframes && (!has2 || t01 < nframes), "pair tile index", tile0, nbv);
  const bool full0 = t00 + TF <= nframes;
  const bool full1 = t01 + TF <= nframes;
  const long long a = t00 - k;
  const long long jlo = a >= 0 ? (a + TF - 1) / TF : 0;
  const long long qlo = jlo, qhi = tile0;  // per-tile records of the whole tiles [jlo, tile t)
  const int pcount = a >= 0 ? (int)(jlo * TF - a) : 0;
  const long long nitem = qhi - qlo;

  // ---- 1. every load of both tiles: x (registers), the shifted tiles (LDS-DMA), phase A ----
  const int cl = lane & (CL - 1);
  const int j0 = w * WF + (lane / CL) * P;
  uint32_t xr0[P], xr1[P];
  auto load_x = [&](long long t0, bool full, uint32_t (&xr)[P]) {
    if constexpr (XL == 1) {
      xl_load<P, CL>(in, t0 + j0, cl, nframes, xr);
    } else if (full) {
      const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
#pragma unroll
      for (int i = 0; i < P; ++i) xr[i] = in32[(t0 + j0 + i) * CL + cl];
    } else {
#pragma unroll
      for (int i = 0; i < P; ++i) {
        T v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = load_elem(in, hist, t0 + j0 + i, cl * E + e, C, nframes, k, pre);
        xr[i] = CEl::put(v);
      }
    }
  };
  load_x(t00, full0, xr0);
  if (has2) load_x(t01, full1, xr1);
  auto stage = [&](long long t0, unsigned char* sstage) {
    const long long h0 = t0 - k;  // F = 1: the shifted stage starts exactly k frames before the tile
    if (h0 >= 0 && (h0 * C + (long long)SG * EPG) <= nframes * C) {
      const T* src = in + h0 * C;
      for (int s0 = 0; s0 < SG; s0 += WG) {
        const int s = s0 + tid;
        if (s < SG) glds16<(NT & kNtHalo) != 0>(src + (long long)chan_slot<CL, P>(s) * EPG, sstage + (s0 + wq * 64) * 16);
      }
    } else {
#pragma unroll 1
      for (int gl = tid; gl < SG; gl += WG) {
        Gr u;
#pragma unroll
        for (int i = 0; i < EPG; ++i) {
          const int e = gl * EPG + i;
          u.e[i] = load_elem(in, hist, h0 + e / C, e % C, C, nframes, k, pre);
        }
        GIO::store(reinterpret_cast<T*>(sstage + chan_slot<CL, P>(gl) * 16), u);
      }
    }
  };
  stage(t00, sst[0]);
  if (has2) stage(t01, sst[1]);
  auto share = [&](int src, const SA (&r)[C]) {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) shares[(src * NW + w) * C + c] = r[c];
    }
  };
  // phase A of both slots: the tiles of slots v + D (default policy: their own later loads hit L2)
  const unsigned bd0 = vs0 + (unsigned)p.ahead, bd1 = vs1 + (unsigned)p.ahead;
  const long long ja0 = bd0 < nbv ? remap_tile(bd0, nbv, 1) : -1;
  const long long ja1 = has2 && bd1 < nbv ? remap_tile(bd1, nbv, 1) : -1;
  const bool prod0 = ja0 >= 0 && ja0 < p.nfull, prod1 = ja1 >= 0 && ja1 < p.nfull;
  {
    Unit<T, VE> xa0[U], xa1[U];
    if (prod0) {
#pragma unroll
      for (int u = 0; u < U; ++u) xa0[u] = IO::gload(in + (ja0 * TF + (long long)(u * WG + tid) * F) * C, false);
    }
    if (prod1) {
#pragma unroll
      for (int u = 0; u < U; ++u) xa1[u] = IO::gload(in + (ja1 * TF + (long long)(u * WG + tid) * F) * C, false);
    }
    if (prod0) {
      SA r[C];
      wave_record<T, SA, C, F, U>(xa0, r);
      share(0, r);
    }
    if (prod1) {
      SA r[C];
      wave_record<T, SA, C, F, U>(xa1, r);
      share(3, r);
    }
  }
  // own records (slots v < D: no producer D slots earlier) and head duty, per slot
  const bool own0 = vs0 < (unsigned)p.ahead && tile0 < p.nfull;
  const bool own1 = has2 && vs1 < (unsigned)p.ahead && tile0 + 1 < p.nfull;
  if (own0) {
    SA r[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, tile0, w, lane, false, r);
    share(1, r);
  }
  if (own1) {
    SA r[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, tile0 + 1, w, lane, false, r);
    share(4, r);
  }
  auto head_tile = [&](unsigned v) -> long long {
    const unsigned xr = v & 7u, s = v >> 3;
    if (xr >= 1u && s < (unsigned)p.head) {
      const long long j = run_start(xr, nbv) - p.head + s;
      if (j >= 0 && j < p.nfull) return j;
    }
    return -1;
  };
  const long long jh0 = head_tile(vs0), jh1 = has2 ? head_tile(vs1) : -1;
  if (jh0 >= 0) {
    SA r[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, jh0, w, lane, false, r);
    share(2, r);
  }
  if (jh1 >= 0) {
    SA r[C];
    wave_record_lean<T, SA, C, F, U, WG>(in, jh1, w, lane, false, r);
    share(5, r);
  }
  // tile t's carry reads one (record, channel) pair per thread: slot s = q*C + c
  const long long nslot = nitem * C;
  const int cc = tid % C;
  unsigned long long rv[NG];
  auto slot_load = [&](long long sl, unsigned long long (&v)[NG]) {
#pragma unroll
    for (int h = 0; h < NG; ++h) v[h] = gran_load(gran + (qlo * C + sl) * NG + h);
  };
  MAVG_DCHECK(qhi <= p.nfull, "pair record read range", qhi, p.nfull);
  if (tid < nslot) {
    slot_load(tid, rv);
  } else {
#pragma unroll
    for (int h = 0; h < NG; ++h) rv[h] = 0ull;
  }
  __syncthreads();
  for (int src = wq; src < NSRC; src += NW) {
    long long j = -1;
    switch (src) {
      case 0: j = prod0 ? ja0 : -1; break;
      case 1: j = own0 ? tile0 : -1; break;
      case 2: j = jh0; break;
      case 3: j = prod1 ? ja1 : -1; break;
      case 4: j = own1 ? tile0 + 1 : -1; break;
      default: j = jh1; break;
    }
    if (j >= 0) publish_record_lds<SA, C, NW>(gran, j, shares + (src * NW) * C, lane);
  }

  // ---- 2. tile t's partial window before frame 0 (history / peeled head): channel cc ----
  A hp = (A)0;
  if (a < 0 && (hist != nullptr || pre > 0)) {
#pragma unroll 1
    for (long long e = tid; e < -a * C; e += WG) hp += to_acc<A>(load_elem(in, hist, a + e / C, cc, C, nframes, k, pre));
  }

  // ---- 3. the in-tile scans of both tiles (pass 1) ----
  // stage addressing as wide_ahead_kernel's CH form (F = 1: x[n-k] of tile frame f is shifted-
  // stage frame f): element (j0 + i, cl) at float index tb[i mod NBX] + (i / NBX) NBX 4 GPF
  constexpr int GPFc = CL >= 4 ? CL / 4 : 1;
  constexpr int NBX = NB < P ? NB : P;
  static_assert(NBX * (P / NBX) == P && P >= NB, "whole address-table rounds; chan_slot keys inside a lane's frames");
  constexpr int kFS = 4 * GPFc;  // floats per frame of the stage
  auto ch_table = [&](int lb, int bq, int (&tb)[NBX]) {
#pragma unroll
    for (int r = 0; r < NBX; ++r) tb[r] = lb + (r ^ bq) * kFS;
  };
  auto ch_idx = [&](const int (&tb)[NBX], int i) -> int { return tb[i % NBX] + (i / NBX) * NBX * kFS; };
  const int ch_lb = (j0 * GPFc + (cl >> 2)) * 4 + (cl & 3);
  const int ch_bq = lane / CL;
  constexpr int kGrp = 8;
  SA crun0[E], cincl0[E], crun1[E], cincl1[E];
  A hpo[E];
#pragma unroll
  for (int e = 0; e < E; ++e) crun0[e] = cincl0[e] = crun1[e] = cincl1[e] = (SA)0, hpo[e] = (A)0;
  auto pass1 = [&](const uint32_t (&xr)[P], const unsigned char* sstage, SA (&crun)[E], SA (&cincl)[E], SA* totw,
                   auto pw) {
    constexpr bool PW = decltype(pw)::value;
    const uint32_t* ssf = reinterpret_cast<const uint32_t*>(sstage);
    int tb[NBX];
    ch_table(ch_lb, ch_bq, tb);
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i % kGrp == 0 && i > 0) __builtin_amdgcn_sched_barrier(0);
      const int ix = ch_idx(tb, i);
      MAVG_DCHECK((ix == (chan_slot<CL, P>(((j0 + i) * CL + cl) >> 2) * 4 + (cl & 3))), "pair stage index", ix, i);
      const uint32_t xk = ssf[ix];
      const uint32_t xv = xr[i];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if constexpr (PW)
          if (j0 + i < pcount) hpo[e] += to_acc<A>(CEl::get(xk, e));
        crun[e] += to_acc<SA>(CEl::get(xv, e)) - to_acc<SA>(CEl::get(xk, e));
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      cincl[e] = crun[e];
#pragma unroll
      for (int sh = CL; sh < 64; sh <<= 1) {
        SA t = shfl_up(cincl[e], sh);
        t = lane >= sh ? t : (SA)0;
        cincl[e] += t;
      }
      if (lane >= 64 - CL) totw[w * C + cl * E + e] = cincl[e];
    }
  };
  if constexpr (XL == 1) {
    xl_transpose<P>(xr0, cl);
    if (has2) xl_transpose<P>(xr1, cl);
  }
  if (pcount > wq * WF) pass1(xr0, sst[0], crun0, cincl0, tot, std::true_type{});
  else pass1(xr0, sst[0], crun0, cincl0, tot, std::false_type{});
  if (has2) pass1(xr1, sst[1], crun1, cincl1, tot + NW * C, std::false_type{});

  // ---- 4. tile t's whole-tile carry from the records, WG (record, channel) slots per round ----
  A hq = (A)0;  // channel cc
#pragma unroll 1
  for (long long sb0 = 0; sb0 < nslot; sb0 += WG) {
    const long long sl = sb0 + tid;
    const bool act = sl < nslot;
    if (sb0 != 0) {
      if (act) {
        slot_load(sl, rv);
      } else {
#pragma unroll
        for (int h = 0; h < NG; ++h) rv[h] = 0ull;
      }
    }
    bool miss = false;
#pragma unroll
    for (int h = 0; h < NG; ++h) miss |= act && (rv[h] >> 32) != 1ull;
#pragma unroll 1
    for (int it = 0; __any(miss) && it < p.spin; ++it) {
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats) + 1, 1u);
#endif
      __builtin_amdgcn_s_sleep(2);
      if (miss) slot_load(sl, rv);
      miss = false;
#pragma unroll
      for (int h = 0; h < NG; ++h) miss |= act && (rv[h] >> 32) != 1ull;
    }
    // still untagged: the wave recomputes each such record with the producer's sequence
    unsigned long long mask = __ballot(miss);
#pragma unroll 1
    while (mask != 0ull) {
      const int l = __builtin_ctzll(mask);
      const long long ql = __shfl(sl, l, 64) / C;
      SA v = (SA)0;
#pragma unroll 1
      for (int c = 0; c < C; ++c) {
        const SA rc = tile_record_chan_lean<T, SA, C, F, U, WG>(in, qlo + ql, c, lane);
        if (cc == c) v = rc;
      }
      const bool mine = miss && sl / C == ql;
      if (mine) {
#pragma unroll
        for (int h = 0; h < NG; ++h) rv[h] = kGranTag | gran_word(v, h);
      }
#ifdef MAVG_AHEAD_STATS
      if (lane == 0) atomicAdd(reinterpret_cast<unsigned int*>(p.stats), 1u);
#endif
      mask &= ~__ballot(mine);
    }
    if (act) {
      uint32_t wd[NG];
#pragma unroll
      for (int h = 0; h < NG; ++h) wd[h] = (uint32_t)rv[h];
      hq += (A)gran_value<SA>(wd);
    }
  }
  {
    // the wave's per-channel carry shares by butterflies over the lanes of one channel (lane mod C)
    // and, for the partial window's column sums, of one column (lane mod CL)
    static_assert(64 % C == 0 && 64 % CL == 0 && CL * E == C, "channel = lane mod C; column = lane mod CL");
    A v = hp + hq;
    if constexpr (E == 1) v += hpo[0];
#pragma unroll
    for (int sh = C; sh < 64; sh <<= 1) v += __shfl_xor(v, sh, 64);
    if constexpr (E > 1) {
      A hv[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        hv[e] = hpo[e];
#pragma unroll
        for (int sh = CL; sh < 64; sh <<= 1) hv[e] += __shfl_xor(hv[e], sh, 64);
      }
      A add = (A)0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const A t = __shfl(hv[e], lane / E, 64);
        if (lane % E == e) add = t;
      }
      v += add;
    }
    if (lane < C) hsum[w * C + lane] = v;
  }
  __syncthreads();

  // ---- 5. pass 2 and the outputs of a tile: each output over the x[n-k] it last read (same lane,
  //         same address: no barrier), then the wave's frames read back slot-contiguous ----
  auto pass2 = [&](long long t0, bool full, uint32_t (&xr)[P], unsigned char* sstage, const A (&base)[E],
                   A (&run)[E]) {
    int lb2 = ch_lb, bq2 = ch_bq;
    asm volatile("" : "+v"(lb2), "+v"(bq2));
#pragma unroll
    for (int i = 0; i < P; ++i) asm volatile("" : "+v"(xr[i]));
    int tb[NBX];
    ch_table(lb2, bq2, tb);
    uint32_t* sw = reinterpret_cast<uint32_t*>(sstage);
#pragma unroll
    for (int e = 0; e < E; ++e) run[e] = base[e];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (i % kGrp == 0 && i > 0) __builtin_amdgcn_sched_barrier(0);
      const int ix = ch_idx(tb, i);
      const uint32_t xk = sw[ix];
      const uint32_t xv = xr[i];
      T y[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        run[e] += (A)(to_acc<SA>(CEl::get(xv, e)) - to_acc<SA>(CEl::get(xk, e)));
        y[e] = to_out<T, A, DV>(run[e], p.o);
      }
      if (full) {
        sw[ix] = CEl::put(y);
      } else if (t0 + j0 + i < nframes) {
#pragma unroll
        for (int e = 0; e < E; ++e) out[(t0 + j0 + i) * C + cl * E + e] = y[e];
      }
    }
    if (!full) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int WGR = WF * C / EPG;  // the wave's granules
    const int rg = wq * WGR;
    T* ob = out + (t0 + (long long)wq * WF) * C;
#pragma unroll
    for (int r = 0; r < WGR / 64; ++r) {
      const int s2 = rg + r * 64 + lane;
      const Gr g = GIO::load(reinterpret_cast<const T*>(sstage + s2 * 16));
      GIO::template store<(NT & kNtStore) != 0>(ob + (long long)(chan_slot<CL, P>(s2) - rg) * EPG, g);
    }
  };
  A run[E];
  {
    A base[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int ch = cl * E + e;
      base[e] = (A)0;
#pragma unroll
      for (int i = 0; i < NW; ++i) base[e] += hsum[i * C + ch];
#pragma unroll
      for (int i = 0; i < NW - 1; ++i)
        if (i < wq) base[e] += (A)tot[i * C + ch];
      base[e] += (A)(cincl0[e] - crun0[e]);
    }
    pass2(t00, full0, xr0, sst[0], base, run);
  }
  if (!has2) return;
  // tile t + 1's carry: tile t's window sum at its last frame (frame TF - 1: the last wave's lanes
  // of block NB - 1, one per column)
  if (wq == NW - 1 && lane >= 64 - CL) {
#pragma unroll
    for (int e = 0; e < E; ++e) carry2[cl * E + e] = run[e];
  }
  __syncthreads();
  {
    A base[E];
    const SA* tot1 = tot + NW * C;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int ch = cl * E + e;
      base[e] = carry2[ch];
#pragma unroll
      for (int i = 0; i < NW - 1; ++i)
        if (i < wq) base[e] += (A)tot1[i * C + ch];
      base[e] += (A)(cincl1[e] - crun1[e]);
    }
    pass2(t01, full1, xr1, sst[1], base, run);
  }
}

// paired look-ahead scan (pair_ahead_kernel above): the halo-only channel-per-lane look-ahead with two
// consecutive tiles per workgroup (tile t + 1 chains tile t's carry); windows short of the L2
// reach (remap mode 1), 16- or 32-B frames, 16-B-aligned views.  The records and their
// workspace are the one-tile kernel's (per tile, per virtual slot); the grid is 8 workgroups per
// pair of run positions.
template <typename T, typename A, int C, int P, int WG, int NT, int DV, int U, int XL = 0>
int launch_pair_ahead(const Sig& sg, int k, hipStream_t st, Workspace ws, int ahead) {
  constexpr int NW = WG / 64;
  constexpr int EPG = 16 / (int)sizeof(T);
  constexpr int CL = C * (int)sizeof(T) / 4;
  constexpr int TF = NW * (64 / CL) * P;
  static_assert(TF == WG * U, "F = 1 record units");
  constexpr int TG = TF * C / EPG;
  using SA = typename ScanAcc<T, A>::type;
  const long long nframes = sg.nframes;
  if (ahead_past_l2(k, C, sizeof(T), TF) || (long long)k < TF) return MAVG_ERR_UNSUPPORTED;
  ahead &= ~7;
  int spin = kAheadSpin;
#ifdef MAVG_TEST_HOOKS
  {
    const int t = g_test_ahead_slots.load(std::memory_order_relaxed);
    if (t >= 0) ahead = t & ~7;
  }
  {
    const int t = g_test_ahead_spin.load(std::memory_order_relaxed);
    if (t >= 0) spin = t;
  }
#endif
  const long long ntiles = (nframes + TF - 1) / TF;
  const long long nfull = nframes / TF;
  if (ntiles > 0x7fffffffLL) return MAVG_ERR_UNSUPPORTED;
  const long long q8 = (ntiles + 7) / 8;               // run positions of the longest run
  const long long grid = 8 * ((q8 + 1) / 2);           // a workgroup per pair of positions per XCD
  const size_t need = ahead_granule_bytes<T, A, C, 1, U>(nfull);
  const size_t lds = (size_t)2 * (TG + 1) * 16 + (size_t)(NW * C + C) * sizeof(A) + (size_t)(2 + 6) * NW * C * sizeof(SA);
  if (lds > 64 * 1024) return MAVG_ERR_UNSUPPORTED;
  if (g_plan) {
    snprintf(g_plan->text, sizeof(g_plan->text),
             "pair_ahead<%s,acc=%s,C=%d,P=%d,nt=%d,dv=%d,FU=%d,xl=%d> grid=%lld block=%d lds=%zu tile_frames=%d "
             "ahead=%d remap=1 tiles=%lld ws=%zu",
             type_name<T>(), type_name<A>(), C, P, NT, DV, U, XL, grid, WG, lds, TF, ahead, ntiles, need);
    g_plan->ws_bytes = need;
    return MAVG_OK;
  }
  if (ws.ptr == nullptr || ws.bytes < need) return MAVG_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(ws.ptr) & 15u) != 0) return MAVG_ERR_MISALIGNED;
  if (hipMemsetAsync(ws.ptr, 0, need, st) != hipSuccess) return MAVG_ERR_HIP;
  AheadParams p{};
  p.in = sg.in;
  p.out = sg.out;
  p.hist = sg.hist;
  p.nframes = nframes;
  p.pre = sg.pre;
  p.eio = 0;
  p.nfull = nfull;
  p.k = k;
  p.o = make_out_params(k);
  p.halo_units = k;
  p.xk_off = 0;
  p.xcd_remap = 1;
  p.runs_done = 0;
  p.ahead = ahead;
  p.head = (int)std::min<long long>((long long)k / TF, nfull);
  p.spin = spin;
  p.self = 0;
  p.gran = static_cast<unsigned long long*>(ws.ptr);
  p.runs = nullptr;
  p.stats = static_cast<unsigned char*>(ws.ptr) + need - 16;
  hipLaunchKernelGGL((pair_ahead_kernel<T, A, C, P, WG, NT, DV, U, XL>), dim3((unsigned)grid), dim3(WG), lds, st, p);
  return hipGetLastError() == hipSuccess ? MAVG_OK : MAVG_ERR_HIP;
}

}  // namespace mavg
