// group.hip -- bucket grouping of MSM entries (msm.hpp step 2): a stable LSD
// counting sort written for gfx950 (round 6; replaced a separate digit-key
// kernel + rocPRIM's onesweep radix sort + its passes).
//
// An entry is one (point, digit window) pair: its key is the bucket (shared
// plans: segment base + |digit| - 1, a zero digit the segment's bucket 0
// with the dummy entry; per-window plans: window base + |digit| - 1, a zero
// digit key G, which sorts after every bucket), its value the base index
// with the digit's sign in bit 31.  The accumulate needs the entries grouped
// by key and off[] (the first entry of every bucket).  The key bits split
// into P digits of rb <= 8 bits (16-bit keys 2 x 8, the A+B1 batch's 17 bits
// 3 x 6), least significant first; each pass is
//   count    one workgroup per tile of GS_TE entries: an LDS histogram of the
//            pass digit, written as column `tile` of a bin-major count matrix;
//   scan     exclusive scan of the matrix (two kernels: chunk sums, then
//            each chunk's prefix + its own scan): the output position of the
//            first entry of every (bin, tile);
//   scatter  the same tile again: every wave ranks its own contiguous part of
//            the tile by digit (per-wave LDS counts, prefixed over the waves;
//            inside a round of 64 entries the lane's rank among the lanes
//            with its digit comes from ballots over the digit bits), stages
//            the tile in LDS in output order and writes it out as one
//            contiguous run per bin.
// Ranks follow input order, so every pass is stable and the result is the
// same bytes on every run (the XYZZ bucket sums, and the partials that
// zk_groth16_prove_partial returns, are reproducible; no atomics decide an
// order).  Pass 0 computes its entries from the scalars (in the count and
// the scatter kernel: 8 B read per point, nothing materialised before the
// first scatter); later passes read the previous pass's output.  Every pass
// is load-balanced by construction (fixed-size tiles), whatever the digit
// distribution (a witness of mostly 0 / 1 puts most entries in a few
// buckets).  off[] then comes from the sorted keys (k_msm_offsets).
// Digits of <= 8 bits (not the 9-10 of onesweep) keep a tile's run per bin
// at >= 32 entries (128 B) of each array: same box, serial 2^20 prove, the
// three MSM sorts 0.62 ms against onesweep's 0.70 (2 x 9 / 2 x 8 bits) and
// 0.79 with 9-10-bit digits here (profiles/r06_ab_grouping.txt).
#include "msm.hpp"

namespace zk {

// tile shape (A/B builds: -DZK_GS_THREADS, -DZK_GS_IPT)
#ifndef ZK_GS_THREADS
#define ZK_GS_THREADS 512
#endif
#ifndef ZK_GS_IPT
#define ZK_GS_IPT 16
#endif
constexpr uint32_t GS_THREADS = ZK_GS_THREADS;
constexpr uint32_t GS_WAVES = GS_THREADS / 64;
constexpr uint32_t GS_IPT = ZK_GS_IPT;              // entries per lane per tile
constexpr uint32_t GS_TE = GS_THREADS * GS_IPT;     // entries per tile (8192)
constexpr uint32_t GS_WR = GS_IPT;                  // rounds of 64 entries per wave
// most digit bits per pass (A/B builds: -DZK_GS_RB)
#ifndef ZK_GS_RB
#define ZK_GS_RB 8
#endif
constexpr uint32_t GS_MAXRB = ZK_GS_RB;
constexpr uint32_t GS_MAXNB = 1u << GS_MAXRB;
constexpr uint32_t GS_SCAN_ITEMS = 8;               // scan: counters per thread
constexpr uint32_t GS_SCAN_THREADS = 1024;
constexpr uint32_t GS_SCAN_CHUNK = GS_SCAN_ITEMS * GS_SCAN_THREADS;

struct GsArgs {
  const uint64_t* sc[MSM_MAXSEG];
  uint32_t n[MSM_MAXSEG], wstride[MSM_MAXSEG], ioff[MSM_MAXSEG], kbase[MSM_MAXSEG];
  uint32_t tile0[MSM_MAXSEG + 1];   // first pass-0 tile of segment k
  uint32_t boff[MSM_MAXWIN];
  uint32_t nseg, nwin, c, bits, shared, G, M, rb;
};

// Digit of window w of a scalar, given the carry out of window w - 1 (signed
// windows, the top one unsigned), one window at a time.
template <int SW>
ZK_DI uint32_t gs_digit(const GsArgs& a, uint32_t w, const uint64_t (&s)[SW], uint32_t& carry, bool& neg) {
  const bool top = w == a.nwin - 1;
  const int width = top ? (int)(a.bits - a.c * w) : (int)a.c;
  const uint32_t v = scal_window<SW>(s, (int)(a.c * w), width) + carry;
  if (!top && v > (1u << (a.c - 1))) {
    carry = 1;
    neg = true;
    return (1u << a.c) - v;
  }
  carry = 0;
  neg = false;
  return v;
}

// The entry of (segment k, point i, window w) with digit magnitude mag.
ZK_DI void gs_entry(const GsArgs& a, uint32_t k, uint32_t i, uint32_t w, uint32_t mag, bool neg, uint32_t& key,
                    uint32_t& ent) {
  if (a.shared) {
    key = a.kbase[k] + (mag ? mag - 1 : 0u);
    ent = mag ? ((w * a.wstride[k] + a.ioff[k] + i) | (neg ? 0x80000000u : 0u)) : MSM_DUMMY;
  } else {
    key = mag ? a.boff[w] + mag - 1 : a.G;
    ent = i | (neg ? 0x80000000u : 0u);
  }
}

ZK_DI uint32_t gs_seg(const GsArgs& a, uint32_t tile) {
  uint32_t k = 0;
#pragma unroll
  for (uint32_t j = 1; j < MSM_MAXSEG; j++)
    if (j < a.nseg && tile >= a.tile0[j]) k = j;
  return k;
}

// The GS_IPT entries of this lane in tile `tile`, in input order.  Pass 0
// (SRC): the tile is GS_TE / 64 units of segment k's (point round, window)
// sequence, point-major (unit u = point round u / nwin, window u mod nwin);
// wave v takes units [v GS_WR, (v + 1) GS_WR) and lane l point 64 pr + l of
// a unit.  Consecutive units of one point round are consecutive windows, so
// the signed-digit carry runs along them (the first unit of a wave recomputes
// the carry of the windows below it).  Later passes: entries
// tile GS_TE + v GS_WR 64 + 64 r + l of the input arrays.
template <int SW, bool SRC>
ZK_DI void gs_load(const GsArgs& a, uint32_t tile, const uint32_t* __restrict__ kin, const uint32_t* __restrict__ ein,
                   uint32_t (&key)[GS_IPT], uint32_t (&ent)[GS_IPT], uint32_t& valid) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  valid = 0;
  if constexpr (SRC) {
    const uint32_t k = gs_seg(a, tile);
    const uint32_t u0 = (tile - a.tile0[k]) * (GS_TE / 64) + wave * GS_WR;
    const uint32_t nk = a.n[k];
    uint32_t pr = u0 / a.nwin, w = u0 - pr * a.nwin;
    uint32_t i = pr * 64 + lane;
    uint64_t s[SW];
    uint32_t carry = 0;
    bool neg = false;
#pragma unroll
    for (int j = 0; j < SW; j++) s[j] = i < nk ? a.sc[k][(size_t)i * SW + j] : 0ull;
    for (uint32_t q = 0; q < w; q++) (void)gs_digit<SW>(a, q, s, carry, neg);
#pragma unroll
    for (uint32_t r = 0; r < GS_IPT; r++) {
      key[r] = ent[r] = 0;
      if (i < nk) {
        const uint32_t mag = gs_digit<SW>(a, w, s, carry, neg);
        gs_entry(a, k, i, w, mag, neg, key[r], ent[r]);
        valid |= 1u << r;
      }
      if (++w == a.nwin) {   // next point round
        w = 0;
        carry = 0;
        i += 64;
#pragma unroll
        for (int j = 0; j < SW; j++) s[j] = (r + 1 < GS_IPT && i < nk) ? a.sc[k][(size_t)i * SW + j] : 0ull;
      }
    }
  } else {
    const size_t e0 = (size_t)tile * GS_TE + wave * GS_WR * 64 + lane;
#pragma unroll
    for (uint32_t r = 0; r < GS_IPT; r++) {
      const size_t e = e0 + 64 * r;
      const bool ok = e < a.M;
      key[r] = ok ? kin[e] : 0u;
      ent[r] = ok ? ein[e] : 0u;
      if (ok) valid |= 1u << r;
    }
  }
}

// count: column `tile` of the bin-major matrix cnt[b ntiles + tile]
template <int SW, bool SRC>
__global__ void __launch_bounds__(GS_THREADS) k_gs_count(GsArgs a, uint32_t shift, uint32_t ntiles,
                                                         const uint32_t* __restrict__ kin,
                                                         uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[GS_MAXNB];
  const uint32_t NB = 1u << a.rb, tile = blockIdx.x;
  for (uint32_t b = threadIdx.x; b < NB; b += GS_THREADS) h[b] = 0;
  __syncthreads();
  uint32_t key[GS_IPT], ent[GS_IPT], valid;
  if constexpr (SRC) {
    gs_load<SW, true>(a, tile, nullptr, nullptr, key, ent, valid);
  } else {   // keys only
    const size_t e0 = (size_t)tile * GS_TE + (threadIdx.x >> 6) * GS_WR * 64 + (threadIdx.x & 63);
    valid = 0;
#pragma unroll
    for (uint32_t r = 0; r < GS_IPT; r++) {
      const size_t e = e0 + 64 * r;
      key[r] = e < a.M ? kin[e] : 0u;
      if (e < a.M) valid |= 1u << r;
    }
  }
  (void)ent;
#pragma unroll
  for (uint32_t r = 0; r < GS_IPT; r++)
    if (valid >> r & 1u) atomicAdd(&h[(key[r] >> shift) & (NB - 1)], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < NB; b += GS_THREADS) cnt[(size_t)b * ntiles + tile] = h[b];
}

// scan, kernel 1: the sum of every GS_SCAN_CHUNK counters
__global__ void __launch_bounds__(GS_SCAN_THREADS) k_gs_scan_sums(const uint32_t* __restrict__ cnt, size_t L,
                                                                  uint32_t* __restrict__ sums) {
  __shared__ uint32_t ws[GS_SCAN_THREADS / 64];
  const size_t base = (size_t)blockIdx.x * GS_SCAN_CHUNK;
  uint32_t s = 0;
#pragma unroll
  for (uint32_t j = 0; j < GS_SCAN_ITEMS; j++) {
    const size_t i = base + j * GS_SCAN_THREADS + threadIdx.x;
    if (i < L) s += cnt[i];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t v = 0; v < GS_SCAN_THREADS / 64; v++) t += ws[v];
    sums[blockIdx.x] = t;
  }
}

// Exclusive scan of one value per thread over the workgroup (wave shuffles,
// then the wave totals); returns the thread's exclusive prefix, total in *tot.
template <uint32_t THREADS>
ZK_DI uint32_t gs_block_scan(uint32_t v, uint32_t* ws, uint32_t* tot) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t x = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += x;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (uint32_t w = 0; w < THREADS / 64; w++) {
      const uint32_t t = ws[w];
      ws[w] = s;
      s += t;
    }
    ws[THREADS / 64] = s;
  }
  __syncthreads();
  const uint32_t ex = ws[wave] + incl - v;
  if (tot) *tot = ws[THREADS / 64];
  __syncthreads();   // ws reusable
  return ex;
}

// scan, kernel 2: chunk b's offset (the sums of the chunks before it) plus
// the exclusive scan of its own counters, in place
__global__ void __launch_bounds__(GS_SCAN_THREADS) k_gs_scan_apply(uint32_t* __restrict__ cnt, size_t L,
                                                                   const uint32_t* __restrict__ sums) {
  __shared__ uint32_t ws[GS_SCAN_THREADS / 64 + 1];
  __shared__ uint32_t red[GS_SCAN_THREADS / 64];
  // offset of this chunk
  uint32_t o = 0;
  for (uint32_t j = threadIdx.x; j < blockIdx.x; j += GS_SCAN_THREADS) o += sums[j];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) o += __shfl_xor(o, d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = o;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t v = 0; v < GS_SCAN_THREADS / 64; v++) off += red[v];
  // thread t scans counters [t ITEMS, (t + 1) ITEMS) of the chunk (contiguous)
  const size_t base = (size_t)blockIdx.x * GS_SCAN_CHUNK + (size_t)threadIdx.x * GS_SCAN_ITEMS;
  uint32_t c[GS_SCAN_ITEMS], s = 0;
#pragma unroll
  for (uint32_t j = 0; j < GS_SCAN_ITEMS; j++) {
    c[j] = base + j < L ? cnt[base + j] : 0u;
    s += c[j];
  }
  uint32_t ex = gs_block_scan<GS_SCAN_THREADS>(s, ws, nullptr) + off;
#pragma unroll
  for (uint32_t j = 0; j < GS_SCAN_ITEMS; j++) {
    if (base + j < L) cnt[base + j] = ex;
    ex += c[j];
  }
}

// scatter: rank, stage, write out (see the file comment)
template <int SW, bool SRC>
__global__ void __launch_bounds__(GS_THREADS) k_gs_scatter(GsArgs a, uint32_t shift, uint32_t ntiles,
                                                           const uint32_t* __restrict__ kin,
                                                           const uint32_t* __restrict__ ein,
                                                           const uint32_t* __restrict__ pos,
                                                           uint32_t* __restrict__ kout, uint32_t* __restrict__ eout) {
  __shared__ uint32_t sk[GS_TE], se[GS_TE];
  __shared__ uint32_t wh[GS_WAVES][GS_MAXNB];   // per-wave counts -> per-wave running slot
  __shared__ uint32_t tb[GS_MAXNB];             // output position of local slot 0 of bin b
  __shared__ uint32_t ws[GS_THREADS / 64 + 1];
  const uint32_t NB = 1u << a.rb, tile = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t j = threadIdx.x; j < GS_WAVES * GS_MAXNB; j += GS_THREADS) (&wh[0][0])[j] = 0;
  uint32_t key[GS_IPT], ent[GS_IPT], valid;
  gs_load<SW, SRC>(a, tile, kin, ein, key, ent, valid);
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < GS_IPT; r++)
    if (valid >> r & 1u) atomicAdd(&wh[wave][(key[r] >> shift) & (NB - 1)], 1u);
  __syncthreads();
  // per bin: the waves' exclusive prefix (in wh) and the tile count, then
  // the local slot of the bin's first entry (scan over bins, GS_BPT
  // consecutive bins per thread)
  constexpr uint32_t GS_BPT = GS_MAXNB > GS_THREADS ? GS_MAXNB / GS_THREADS : 1;
  uint32_t tc[GS_BPT], tsum = 0;
#pragma unroll
  for (uint32_t h = 0; h < GS_BPT; h++) {
    const uint32_t b = GS_BPT * threadIdx.x + h;
    tc[h] = 0;
    if (b < NB) {
      uint32_t s = 0;
      for (uint32_t v = 0; v < GS_WAVES; v++) {
        const uint32_t c = wh[v][b];
        wh[v][b] = s;
        s += c;
      }
      tc[h] = s;
    }
    tsum += tc[h];
  }
  uint32_t lb = gs_block_scan<GS_THREADS>(tsum, ws, nullptr);
#pragma unroll
  for (uint32_t h = 0; h < GS_BPT; h++) {
    const uint32_t b = GS_BPT * threadIdx.x + h;
    if (b < NB) {
      tb[b] = pos[(size_t)b * ntiles + tile] - lb;
      for (uint32_t v = 0; v < GS_WAVES; v++) wh[v][b] += lb;
    }
    lb += tc[h];
  }
  __syncthreads();
  // rank in input order: rounds in order, lanes in order inside a round
  const uint64_t lt_mask = (1ull << lane) - 1;
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t r = 0; r < GS_IPT; r++) {
    const bool ok = valid >> r & 1u;
    const uint32_t d = (key[r] >> shift) & (NB - 1);
    uint64_t m = __ballot(ok);
    for (uint32_t bit = 0; bit < a.rb; bit++) {
      const uint64_t bb = __ballot((d >> bit) & 1u);
      m &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    if (ok) {
      const uint32_t base = wh[wave][d];
      const uint32_t slot = base + __popcll(m & lt_mask);
      sk[slot] = key[r];
      se[slot] = ent[r];
      if ((m & lt_mask) == 0) wh[wave][d] = base + __popcll(m);   // the lowest lane of the digit
      cnt++;
    }
  }
  // tile total
  uint32_t tot = 0;
  (void)gs_block_scan<GS_THREADS>(cnt, ws, &tot);
  // contiguous runs per bin: local slot j of bin b lands at tb[b] + j
  for (uint32_t j = threadIdx.x; j < tot; j += GS_THREADS) {
    const uint32_t k = sk[j];
    const uint32_t g = tb[(k >> shift) & (NB - 1)] + j;
    kout[g] = k;
    eout[g] = se[j];
  }
}

// off[g] = first sorted position with key >= g, for g in [0, G].
// ctl (MsmWork::nbig): the merge's control words, zeroed here so that no
// memset launch is needed.
__global__ void __launch_bounds__(256) k_msm_offsets(const uint32_t* __restrict__ key, uint32_t M, uint32_t G,
                                                     uint32_t* __restrict__ off, uint32_t* __restrict__ ctl) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2) ctl[i] = 0;
  if (i > M) return;
  const uint32_t lo = i ? min(key[i - 1], G) + 1 : 0;     // keys in (key[i-1], key[i]] start at i
  const uint32_t hi = i < M ? min(key[i], G) : G;
  for (uint32_t g = lo; g <= hi; g++) off[g] = i;
}

void msm_offsets(MsmWork& w, uint32_t M, hipStream_t st) {
  w.nbig.ensure(2 * sizeof(uint32_t));
  k_msm_offsets<<<ceil_div((uint64_t)M + 1, 256), 256, 0, st>>>(w.key.as<uint32_t>(), M, w.plan.G,
                                                                 w.off.as<uint32_t>(), w.nbig.as<uint32_t>());
  ZK_LAUNCH_CHECK();
}

template <int SW>
static void gs_run(MsmWork& w, const GsArgs& a, uint32_t ntiles0, hipStream_t st) {
  const MsmPlan& p = w.plan;
  const uint32_t M = a.M;
  uint32_t maxkey = p.shared ? p.G - 1 : p.G;
  uint32_t kb = 1;
  while (kb < 32 && (maxkey >> kb)) kb++;
  const uint32_t P = (kb + GS_MAXRB - 1) / GS_MAXRB;
  GsArgs g = a;
  g.rb = (kb + P - 1) / P;
  const uint32_t NB = 1u << g.rb;
  const uint32_t ntiles1 = ceil_div(M, GS_TE);
  const size_t L = (size_t)NB * std::max(ntiles0, ntiles1);
  w.gcnt.ensure(sizeof(uint32_t) * std::max<size_t>(L, 1));
  w.gcnt_sums.ensure(sizeof(uint32_t) * (L / GS_SCAN_CHUNK + 2));
  uint32_t* cnt = w.gcnt.as<uint32_t>();
  uint32_t* sums = w.gcnt_sums.as<uint32_t>();
  // ping-pong so that the last pass writes w.key / w.ent
  uint32_t* kbuf[2] = {w.key.as<uint32_t>(), w.key_in.as<uint32_t>()};
  uint32_t* ebuf[2] = {w.ent.as<uint32_t>(), w.ent_in.as<uint32_t>()};
  const uint32_t* kin = nullptr;
  const uint32_t* ein = nullptr;
  for (uint32_t pass = 0; pass < P; pass++) {
    const uint32_t shift = pass * g.rb;
    const uint32_t nt = pass == 0 ? ntiles0 : ntiles1;
    const size_t Lp = (size_t)NB * nt;
    if (pass == 0)
      k_gs_count<SW, true><<<nt, GS_THREADS, 0, st>>>(g, shift, nt, nullptr, cnt);
    else
      k_gs_count<SW, false><<<nt, GS_THREADS, 0, st>>>(g, shift, nt, kin, cnt);
    ZK_LAUNCH_CHECK();
    const uint32_t nchunk = ceil_div(Lp, GS_SCAN_CHUNK);
    k_gs_scan_sums<<<nchunk, GS_SCAN_THREADS, 0, st>>>(cnt, Lp, sums);
    ZK_LAUNCH_CHECK();
    k_gs_scan_apply<<<nchunk, GS_SCAN_THREADS, 0, st>>>(cnt, Lp, sums);
    ZK_LAUNCH_CHECK();
    const uint32_t out = (P - 1 - pass) & 1u;
    if (pass == 0)
      k_gs_scatter<SW, true><<<nt, GS_THREADS, 0, st>>>(g, shift, nt, nullptr, nullptr, cnt, kbuf[out], ebuf[out]);
    else
      k_gs_scatter<SW, false><<<nt, GS_THREADS, 0, st>>>(g, shift, nt, kin, ein, cnt, kbuf[out], ebuf[out]);
    ZK_LAUNCH_CHECK();
    kin = kbuf[out];
    ein = ebuf[out];
  }
}

void msm_group(MsmWork& w, const MsmSeg* segs, int nseg, int sw, hipStream_t st) {
  const MsmPlan& p = w.plan;
  GsArgs a{};
  a.nseg = (uint32_t)nseg;
  a.nwin = (uint32_t)p.nwin;
  a.c = (uint32_t)p.c;
  a.bits = (uint32_t)p.bits;
  a.shared = p.shared ? 1u : 0u;
  a.G = p.G;
  for (int k = 0; k < p.nwin && k < MSM_MAXWIN; k++) a.boff[k] = p.boff[k];
  uint32_t tiles = 0;
  size_t M = 0;
  for (int k = 0; k < nseg; k++) {
    a.sc[k] = segs[k].scalars;
    a.n[k] = segs[k].n;
    a.wstride[k] = segs[k].wstride ? segs[k].wstride : segs[k].n;
    a.ioff[k] = segs[k].ioff;
    a.kbase[k] = (p.shared && nseg > 1) ? (uint32_t)k << (p.segshift & 31) : 0u;
    a.tile0[k] = tiles;
    const uint64_t rounds = (uint64_t)ceil_div(segs[k].n, 64) * (uint64_t)p.nwin;
    tiles += (uint32_t)((rounds + GS_TE / 64 - 1) / (GS_TE / 64));
    M += (size_t)segs[k].n * p.nwin;
  }
  for (int k = nseg; k <= MSM_MAXSEG; k++) a.tile0[k] = tiles;
  a.M = (uint32_t)M;
  if (M) {
    w.key_in.ensure(sizeof(uint32_t) * M);
    w.ent_in.ensure(sizeof(uint32_t) * M);
    if (sw == 1) gs_run<1>(w, a, tiles, st);
    else gs_run<4>(w, a, tiles, st);
  }
  msm_offsets(w, (uint32_t)M, st);
}

}  // namespace zk
