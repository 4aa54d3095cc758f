// msm.hip -- Pippenger bucket MSM kernels for gfx950 (see msm.hpp for the
// pipeline).  Wave64 throughout; no MFMA (big-integer modular arithmetic).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "msm.hpp"

namespace zk {

// ---------------------------------------------------------------- plan ---
MsmPlan msm_make_plan(uint32_t n, int bits, int sw, int force_c) {
  MsmPlan p{};
  p.n = n;
  p.bits = bits;
  p.sw = sw;
  // balanced windows only: for each window count the smallest c that covers
  // the bits (a tiny top window would pile every point into a few huge buckets)
  int best_c = 4;
  double best = 1e300;
  for (int nw = (bits + 15) / 16; nw <= std::min(MSM_MAXWIN, bits); nw++) {
    const int c = (bits + nw - 1) / nw;
    if (c < 4) break;
    const int nwin = (bits + c - 1) / c;
    const int top = bits - c * (nwin - 1);
    const double nbuck = (double)(nwin - 1) * (1u << (c - 1)) + (double)(1u << top);
    // accumulate: one mixed add per (point, window); reduce: ~2.5 full adds per bucket
    const double cost = (double)n * nwin + 3.5 * nbuck;
    if (cost < best) { best = cost; best_c = c; }
  }
  if (force_c) best_c = force_c;
  p.c = best_c;
  p.nwin = (bits + p.c - 1) / p.c;

  uint32_t G = 0, rc = 0, q = 0;
  for (int w = 0; w < p.nwin; w++) {
    const int width = (w == p.nwin - 1) ? bits - p.c * w : p.c;
    const int k = (w == p.nwin - 1) ? width : p.c - 1;   // nb = 2^k
    p.nb[w] = 1u << k;
    p.kr[w] = (uint8_t)(k / 2);
    p.kc[w] = (uint8_t)(k - k / 2);
    p.boff[w] = G;
    p.rcoff[w] = rc;
    p.qoff[w] = q;
    G += p.nb[w];
    rc += (1u << p.kr[w]) + (1u << p.kc[w]);
    q += p.kr[w] + p.kc[w] + 1;
  }
  p.boff[p.nwin] = G;
  p.rcoff[p.nwin] = rc;
  p.qoff[p.nwin] = q;
  p.G = G;
  p.nrc = rc;
  p.nq = q;
  p.nred = p.nwin;
  p.shared = 0;
  p.nseg = 1;
  p.segshift = 31;
  return p;
}

MsmPlan msm_make_plan_shared(uint32_t n, int bits, int sw, int c) {
  MsmPlan p{};
  p.n = n;
  p.bits = bits;
  p.sw = sw;
  p.c = c;
  p.nwin = (bits + c - 1) / c;
  const int top = bits - c * (p.nwin - 1);
  const int k = std::max(c - 1, top);   // signed digits <= 2^(c-1); the top window unsigned <= 2^top
  p.shared = 1;
  p.nred = 1;
  p.nb[0] = 1u << k;
  p.kr[0] = (uint8_t)(k / 2);
  p.kc[0] = (uint8_t)(k - k / 2);
  p.boff[0] = 0;
  p.boff[1] = p.G = p.nb[0];
  p.rcoff[0] = 0;
  p.rcoff[1] = p.nrc = (1u << p.kr[0]) + (1u << p.kc[0]);
  p.qoff[0] = 0;
  p.qoff[1] = p.nq = p.kr[0] + p.kc[0] + 1;
  p.nseg = 1;
  p.segshift = 31;
  return p;
}

// Batch plan: segment k = one MSM with its own 2^k buckets [k 2^k, (k+1) 2^k)
// and its own reduction window.
static MsmPlan msm_make_plan_batch(const MsmSeg* segs, int nseg, int bits, int c) {
  uint32_t total = 0;
  for (int k = 0; k < nseg; k++) total += segs[k].n;
  MsmPlan p = msm_make_plan_shared(total, bits, 1, c);
  const int kb = p.kr[0] + p.kc[0];
  p.nseg = nseg;
  p.nred = nseg;
  p.segshift = kb;
  for (int k = 0; k < nseg; k++) {
    p.nb[k] = 1u << kb;
    p.kr[k] = p.kr[0];
    p.kc[k] = p.kc[0];
    p.boff[k] = (uint32_t)k << kb;
    p.rcoff[k] = k * ((1u << p.kr[0]) + (1u << p.kc[0]));
    p.qoff[k] = k * (p.kr[0] + p.kc[0] + 1);
  }
  p.boff[nseg] = p.G = (uint32_t)nseg << kb;
  p.rcoff[nseg] = p.nrc = nseg * ((1u << p.kr[0]) + (1u << p.kc[0]));
  p.qoff[nseg] = p.nq = nseg * (p.kr[0] + p.kc[0] + 1);
  return p;
}

// --------------------------------------------------------- accumulate ---

// Chunk length: the M grouped entries (known on device only) split evenly
// over the T accumulate threads, T = one full-occupancy wave set of the
// chip, so every launch is exactly one balanced round whatever the digit
// distribution.
// K is a multiple of 4: EntQ's 16-byte loads stay aligned.
__device__ __forceinline__ uint32_t chunk_len(uint32_t M, uint32_t T) {
  return M ? ((M + T - 1) / T + 3) / 4 * 4 : 4u;
}

// The sorted (key, entry) pairs of a chunk, fetched ENTQ at a time with
// 16-byte loads into the lane's own column of an LDS slab (no sharing, so
// no barriers: LDS only extends the registers, which the accumulate has
// none of to spare at 3 waves/SIMD).  A chunk is contiguous but a wave's 64
// lanes are K entries apart, so one 4-byte load per entry touches 64 lines
// per wave per entry, and the lines a full-occupancy round keeps open per
// XCD (~6 MB) outgrow its 4 MB L2: each line came back from the fabric up to
// 32 times; now at most 128 B / (4 B x ENTQ) = 2.  Reads may run ENTQ - 1
// entries past the chunk (the arrays carry that slack).
constexpr uint32_t ENTQ = 16;
constexpr uint32_t ENTQ_LDS_WORDS = 2 * ENTQ * 64;   // per wave
struct EntQ {
  uint32_t* col;   // this lane's column: keys at col[64 j], entries at col[64 (ENTQ + j)]
  ZK_DI explicit EntQ(uint32_t* lds) : col(lds + (threadIdx.x >> 6) * ENTQ_LDS_WORDS + (threadIdx.x & 63)) {}
  // entry i = start, start + 1, ... in order (the refill is uniform across the wave)
  ZK_DI void next(const uint32_t* __restrict__ key, const uint32_t* __restrict__ ent, uint32_t start, uint32_t i,
                  uint32_t& g, uint32_t& en) {
    const uint32_t j = (i - start) & (ENTQ - 1);
    if (j == 0) {
      const uint4* kp = reinterpret_cast<const uint4*>(key + i);
      const uint4* ep = reinterpret_cast<const uint4*>(ent + i);
#pragma unroll
      for (uint32_t q = 0; q < ENTQ / 4; q++) {
        const uint4 a = kp[q], b = ep[q];
        col[64 * (4 * q + 0)] = a.x; col[64 * (4 * q + 1)] = a.y;
        col[64 * (4 * q + 2)] = a.z; col[64 * (4 * q + 3)] = a.w;
        col[64 * (ENTQ + 4 * q + 0)] = b.x; col[64 * (ENTQ + 4 * q + 1)] = b.y;
        col[64 * (ENTQ + 4 * q + 2)] = b.z; col[64 * (ENTQ + 4 * q + 3)] = b.w;
      }
    }
    g = col[64 * j];
    en = col[64 * (ENTQ + j)];
  }
};

// Thread t owns sorted entries [tK, tK+K).  One mixed add per entry (uniform
// across the wave); at a bucket change the finished run is flushed:
//   complete bucket                        -> buckets[g]
//   run begun by an earlier thread (head)   -> partials[2t]
//   run continued by a later thread (tail)  -> partials[2t+1]
// tuning builds: -DZK_ACCUM_WPE=w asks for >= w waves per SIMD (register cap)
#ifdef ZK_ACCUM_WPE
#define ZK_ACCUM_ATTR __attribute__((amdgpu_waves_per_eu(ZK_ACCUM_WPE)))
#else
#define ZK_ACCUM_ATTR
#endif
// A/B builds: register caps on the accumulates (ZK_ACCUM_G1_WPE /
// ZK_ACCUM_G2_WPE waves per SIMD worth of registers) with the launch sized
// for ZK_ACCUM_G1_WAVES / ZK_ACCUM_G2_WAVES waves per SIMD, so that a full
// accumulate round leaves registers for other streams' kernels (quotient,
// sorts) on every SIMD
#ifdef ZK_ACCUM_G1_WPE
#define ZK_ACCUM_G1_ATTR __attribute__((amdgpu_waves_per_eu(ZK_ACCUM_G1_WPE)))
#else
#define ZK_ACCUM_G1_ATTR ZK_ACCUM_ATTR
#endif
#ifdef ZK_ACCUM_G2_WPE
#define ZK_ACCUM_G2_ATTR __attribute__((amdgpu_waves_per_eu(ZK_ACCUM_G2_WPE)))
#else
#define ZK_ACCUM_G2_ATTR ZK_ACCUM_ATTR
#endif
template <class A>
struct SegBases {
  const char* p[MSM_MAXSEG];
  uint32_t stride;   // bytes between consecutive bases (packed or padded to 128-B lines)
};
// Base i of batch segment `seg` (the MSM owning the bucket).
template <class A>
ZK_DI const A* seg_base(const SegBases<A>& sb, uint32_t seg, uint32_t i) {
  const char* b = sb.p[0];
#pragma unroll
  for (int k = 1; k < MSM_MAXSEG; k++)
    if (seg == (uint32_t)k) b = sb.p[k];
  return reinterpret_cast<const A*>(b + (size_t)i * sb.stride);
}

template <class C>
__global__ void __launch_bounds__(128) ZK_ACCUM_G1_ATTR k_msm_accum(SegBases<typename C::A> sb, uint32_t segshift,
                                                   const uint32_t* __restrict__ ent,
                                                   const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ off, uint32_t G, uint32_t T,
                                                   typename C::X* __restrict__ buckets,
                                                   typename C::X* __restrict__ partials) {
  using X = typename C::X;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t M = off[G];  // grouped entries (known on device only)
  const uint32_t K = chunk_len(M, T);
  const uint32_t start = t * K;
  if (t >= T || start >= M) return;
  const uint32_t end = min(start + K, M);
  X acc;
  xyzz_set_inf(acc);
  uint32_t cur = key[start], run_start = start;
  __shared__ uint32_t entq_lds[2 * ENTQ_LDS_WORDS];   // 128 threads = 2 waves
  EntQ q(entq_lds);
  for (uint32_t e = start; e < end; e++) {
    uint32_t g, en;
    q.next(key, ent, start, e, g, en);
    if (g != cur) {
      const bool head = (run_start == start) && (off[cur] < start);
      if (head) st_vec(&partials[2 * (size_t)t], acc);
      else st_vec(&buckets[cur], acc);
      xyzz_set_inf(acc);
      cur = g;
      run_start = e;
    }
    if (en == MSM_DUMMY) continue;   // zero digit (shared-bucket plans)
    // batch: bucket g >> segshift names the MSM whose bases entry en indexes
    typename C::A a = ld_vec(seg_base(sb, g >> segshift, en & 0x7fffffffu));
    if (en & 0x80000000u) a.y = f_neg(a.y);
    if (!aff_is_inf(a)) acc = xyzz_madd(acc, a);
  }
  const bool head = (run_start == start) && (off[cur] < start);
  const bool tail = off[cur + 1] > end;
  if (head) st_vec(&partials[2 * (size_t)t], acc);
  else if (tail) st_vec(&partials[2 * (size_t)t + 1], acc);
  else st_vec(&buckets[cur], acc);
}

// G2 accumulate over lane pairs (Fq2h, ff.hpp): chunk t is owned by lanes
// 2t, 2t+1, each holding one Fq coefficient of every Fq2 coordinate.  The
// loop, its branches and the flushes are those of k_msm_accum; the pair's
// two lanes read and write the two 48-byte halves of each point.
ZK_DI void st_pair(G2X* p, const XYZZ<Fq2h>& a) {
  Fq* q = reinterpret_cast<Fq*>(p) + pair_half();
  st_vec(q + 0, a.X.v);
  st_vec(q + 2, a.Y.v);
  st_vec(q + 4, a.ZZ.v);
  st_vec(q + 6, a.ZZZ.v);
}
__global__ void __launch_bounds__(128) ZK_ACCUM_G2_ATTR k_msm_accum_pair(SegBases<G2A> sb, uint32_t segshift,
                                                                      const uint32_t* __restrict__ ent,
                                                                      const uint32_t* __restrict__ key,
                                                                      const uint32_t* __restrict__ off, uint32_t G,
                                                                      uint32_t T, G2X* __restrict__ buckets,
                                                                      G2X* __restrict__ partials) {
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  const uint32_t h = pair_half();
  const uint32_t M = off[G];
  const uint32_t K = chunk_len(M, T);
  const uint32_t start = t * K;
  if (t >= T || start >= M) return;   // uniform over the pair
  const uint32_t end = min(start + K, M);
  XYZZ<Fq2h> acc;
  xyzz_set_inf(acc);
  uint32_t cur = key[start], run_start = start;
  __shared__ uint32_t entq_lds[2 * ENTQ_LDS_WORDS];   // 128 threads = 2 waves
  EntQ q(entq_lds);
  for (uint32_t e = start; e < end; e++) {
    uint32_t g, en;
    q.next(key, ent, start, e, g, en);
    if (g != cur) {
      const bool head = (run_start == start) && (off[cur] < start);
      if (head) st_pair(&partials[2 * (size_t)t], acc);
      else st_pair(&buckets[cur], acc);
      xyzz_set_inf(acc);
      cur = g;
      run_start = e;
    }
    if (en == MSM_DUMMY) continue;
    const Fq* bp = reinterpret_cast<const Fq*>(seg_base(sb, g >> segshift, en & 0x7fffffffu)) + h;
    Affine<Fq2h> a{{ld_vec(bp)}, {ld_vec(bp + 2)}};
    if (en & 0x80000000u) a.y = f_neg(a.y);
    if (!aff_is_inf(a)) acc = xyzz_madd(acc, a);
  }
  const bool head = (run_start == start) && (off[cur] < start);
  const bool tail = off[cur + 1] > end;
  if (head) st_pair(&partials[2 * (size_t)t], acc);
  else if (tail) st_pair(&partials[2 * (size_t)t + 1], acc);
  else st_pair(&buckets[cur], acc);
}

// Buckets whose entries span several accumulate chunks.  A bucket over
// P = t1 - t0 + 1 chunks is tail(t0) + head(t0+1) + ... + head(t1):
//  * P <= fix_max (the common case: ~1-2): one thread sums the pieces
//    serially (k_msm_fixup), all such buckets at once;
//  * larger P (skewed scalars: a witness of mostly ones puts ~n entries in
//    one bucket) goes through a log-depth segmented merge (k_msm_merge):
//    level l covers entry ranges ("groups") of W = K 4^l; a group's children
//    are the 4 groups of level l-1 (level 0 = the chunks), and each leaves at
//    most two open pieces of a large bucket --
//      first slot  the bucket holding entry s, if it began before s
//      last slot   the bucket holding entry e-1, if it began in [s, e) and
//                  continues past e
//    both decidable from the sorted keys and bucket offsets alone.  A level
//    reads its children's <= 8 slots in key order, writes buckets that are
//    now complete and passes the rest up: log4(M/K) levels of <= 7 adds.
// MSM_MERGE_FAN children per group: log_FAN(T) merge launches per MSM,
// which are no-ops unless some bucket spans more than fix_max chunks
// (skewed scalars).  Fan-out 8 (6 instead of 9 launches) measured 0.36 ms
// SLOWER in the overlapped prove (profiles/r03_ab_batchq_fan8_rcw4_rejected.txt).
#ifndef ZK_MERGE_FAN_LOG
#define ZK_MERGE_FAN_LOG 2
#endif
constexpr int MSM_MERGE_FAN = 1 << ZK_MERGE_FAN_LOG;

// The latency-bound G1 reductions (fixup, row/column sums, quantities, the
// tree merge) run their adds without the scheduling barriers
// (xyzz_add_ilp), so independent products overlap; ZK_TAIL_ILP=0 (build
// flag) restores them (A/B).  The one-lane G2 path keeps them (its 96-VGPR
// points would spill).
#ifndef ZK_TAIL_ILP
#define ZK_TAIL_ILP 1
#endif
template <class F>
ZK_DI XYZZ<F> tail_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  return xyzz_add(p, q);
}
ZK_DI XYZZ<Fq> tail_add(const XYZZ<Fq>& p, const XYZZ<Fq>& q) {
  if constexpr (ZK_TAIL_ILP != 0) return xyzz_add_ilp(p, q);
  else return xyzz_add(p, q);
}
// G2 lane-pair sums (row/column sums, fixup) as well: prove 9.61 -> 9.55 ms
// (median of 5 alternating pairs, profiles/r02_ab_g2_ilp.txt; the 408 B of
// scratch are the out-of-line doubling call, with or without); ZK_TAIL_ILP_G2=0
// (build flag) keeps their barriers

#ifndef ZK_TAIL_ILP_G2
#define ZK_TAIL_ILP_G2 1
#endif
ZK_DI XYZZ<Fq2h> tail_add(const XYZZ<Fq2h>& p, const XYZZ<Fq2h>& q) {
  if constexpr (ZK_TAIL_ILP_G2 != 0) return xyzz_add_ilp(p, q);
  else return xyzz_add(p, q);
}

__device__ __forceinline__ bool big_bucket(const uint32_t* off, uint32_t b, uint32_t K, uint32_t fix_max) {
  return (off[b + 1] - 1) / K - off[b] / K + 1 > fix_max;
}

// One thread per bucket, or -- when there are more buckets than chunks
// (by_boundary: the 2^19-bucket full-width MSM, where most buckets lie inside
// one chunk and most per-bucket lanes would idle) one thread per chunk
// boundary u, which takes the bucket holding entry u K if u is the first
// boundary inside it.
template <class C>
__global__ void __launch_bounds__(128) k_msm_fixup(const uint32_t* __restrict__ key, const uint32_t* __restrict__ off,
                                                   uint32_t G, uint32_t T, uint32_t fix_max, bool by_boundary,
                                                   uint32_t* __restrict__ nbig, typename C::X* __restrict__ buckets,
                                                   const typename C::X* __restrict__ partials) {
  using X = typename C::X;
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t K = chunk_len(off[G], T);
  uint32_t g = u;
  if (by_boundary) {
    if (u == 0 || u >= T || (uint64_t)u * K >= off[G]) return;
    g = key[u * K];
    if (off[g] / K != u - 1) return;   // not split here, or not its first boundary
  } else if (g >= G) {
    return;
  }
  const uint32_t bs = off[g], be = off[g + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  if (t1 - t0 + 1 > fix_max) {   // left to the merge levels, which skip themselves when none exist
    atomicAdd(nbig, 1u);
    return;
  }
  X acc = ld_vec(&partials[2 * (size_t)t0 + 1]);
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = tail_add(acc, ld_vec(&partials[2 * (size_t)t]));
  st_vec(&buckets[g], acc);
}

template <class X>
__device__ __forceinline__ X shfl_xor_point(const X& v, int d) {
  constexpr int NW = sizeof(X) / 4;
  X o;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int k = 0; k < NW; k++) dst[k] = __shfl_xor(src[k], d);
  return o;
}

// All merge levels in ONE launch (round 5; was one launch per level, 8-9
// per MSM at ~5 us each although they exit at once unless some bucket spans
// more than fix_max chunks).  ctl[0] = buckets left to the merge (the
// fixup's count), ctl[1] = the grid barrier's arrivals.  Level l's groups
// are spread over the grid (grid-stride); the blocks meet at a counting
// barrier between levels (agent-scope release before arriving, acquire after
// leaving: the out[] slots of level l are read by other blocks, on other
// XCDs, at level l + 1).
// Forward progress without a cooperative launch: the grid is capped on the
// host (msm_back_impl) at min(64, the blocks of this kernel the chip holds at
// once), so every block fits on the device together; a block waiting at the
// barrier holds only its own slot, and nothing any other kernel waits on
// depends on this one, so the other streams' kernels retire and the blocks
// not yet placed are dispatched -- co-residency is reached, not assumed.
// The wait costs latency only when the merge runs at all (ctl[0] > 0:
// skewed scalars).
ZK_DI void merge_grid_barrier(uint32_t* bar, uint32_t target) {
  __threadfence();   // every thread's out[] stores, device-wide, before its block arrives
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(2);
  }
  __syncthreads();
  __threadfence();   // acquire for every thread: the next level reads other blocks' slots
}

template <class C>
__global__ void __launch_bounds__(128) k_msm_merge(const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ off, uint32_t G, uint32_t T,
                                                   uint32_t fix_max, uint32_t nlevels, uint32_t* __restrict__ ctl,
                                                   typename C::X* __restrict__ buckets,
                                                   typename C::X* __restrict__ pa, typename C::X* __restrict__ pb) {
  using X = typename C::X;
  if (__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;   // nothing at any level
  const uint32_t M = off[G];
  const uint32_t K = chunk_len(M, T);
  for (uint32_t level = 1; level <= nlevels; level++) {
  const X* in = (level & 1) ? pa : pb;
  X* out = (level & 1) ? pb : pa;
  const uint64_t W = (uint64_t)K << (ZK_MERGE_FAN_LOG * level);
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;; u += gridDim.x * blockDim.x) {
  const uint64_t s64 = (uint64_t)u * W;
  if (s64 >= M) break;
  const uint32_t s = (uint32_t)s64, e = (uint32_t)min<uint64_t>(s64 + W, M);
  const uint32_t cw = (uint32_t)(W / MSM_MERGE_FAN);
  // the children's open slots of large buckets, in key order
  uint32_t sb[2 * MSM_MERGE_FAN];
  size_t si[2 * MSM_MERGE_FAN];
  int ns = 0;
#pragma unroll
  for (int c = 0; c < MSM_MERGE_FAN; c++) {
    const uint32_t cs = s + c * cw;
    if (cs < e) {
      const uint32_t ce = min(cs + cw, e);
      const size_t v = (size_t)MSM_MERGE_FAN * u + c;
      uint32_t b = key[cs];
      if (off[b] < cs && big_bucket(off, b, K, fix_max)) { sb[ns] = b; si[ns] = 2 * v; ns++; }
      b = key[ce - 1];
      if (off[b + 1] > ce && off[b] >= cs && big_bucket(off, b, K, fix_max)) { sb[ns] = b; si[ns] = 2 * v + 1; ns++; }
    }
  }
  int k = 0;
  while (k < ns) {
    const uint32_t b = sb[k];
    X acc = ld_vec(&in[si[k]]);
    for (k++; k < ns && sb[k] == b; k++) acc = tail_add(acc, ld_vec(&in[si[k]]));
    if (off[b] >= s && off[b + 1] <= e) st_vec(&buckets[b], acc);   // complete
    else if (off[b] < s) st_vec(&out[2 * (size_t)u], acc);           // open at the start
    else st_vec(&out[2 * (size_t)u + 1], acc);                       // open at the end
  }
  }
  if (level < nlevels) merge_grid_barrier(&ctl[1], level * gridDim.x);
  }
}

// ------------------------------------------------------------- reduce ---
// One wave64 per sum: lane l folds terms l, l+64, ... serially (all lanes
// busy), then a 6-step butterfly over __shfl_xor (no LDS, so occupancy is
// set by VGPRs alone; a G2 point is 96 dwords -- 96 cross-lane moves per
// step against ~20K instructions per add).  Both phases run through ONE
// xyzz_add call site: the loop is not unrolled, so the kernel's code stays
// a single add (I-cache) instead of 1 + 6 inlined copies.

constexpr int MSM_RED_WAVES = 4;   // sums per 256-thread workgroup

// Partial row/column sum b of the plan: its window, and the buckets it folds
// (len buckets from g0 at stride).  Row i's partial s covers columns
// [s len, (s + 1) len), column j's partial s rows [s len, (s + 1) len).
struct SumSpan {
  uint32_t len, g0, stride;
};
ZK_DI SumSpan rowcol_span(const MsmPlan& p, uint32_t b) {
  int w = 0;
  while (b >= p.rcoff[w + 1]) w++;
  const uint32_t i = b - p.rcoff[w];
  const uint32_t kr = p.kr[w], kc = p.kc[w], lsr = p.lsr[w], lsc = p.lsc[w];
  const uint32_t nr = 1u << (kr + lsr);
  if (i < nr) {
    const uint32_t len = 1u << (kc - lsr);
    return {len, p.boff[w] + ((i >> lsr) << kc) + (i & ((1u << lsr) - 1)) * len, 1u};
  }
  const uint32_t j = i - nr, len = 1u << (kr - lsc);
  return {len, p.boff[w] + (j >> lsc) + (((j & ((1u << lsc) - 1)) * len) << kc), 1u << kc};
}

// Quantity q of the plan: U^C_b (row partials whose row has bit b), U^D_b
// (column partials whose column has bit b) or P (all column partials).
struct QuantSpan {
  uint32_t len, src, bit, shift;   // bit 32: every term
  uint32_t cnt;                    // terms in the quantity
};
ZK_DI QuantSpan quant_span(const MsmPlan& p, uint32_t b) {
  int w = 0;
  while (b >= p.qoff[w + 1]) w++;
  const uint32_t q = b - p.qoff[w];
  const uint32_t kr = p.kr[w], kc = p.kc[w], lsr = p.lsr[w], lsc = p.lsc[w];
  const uint32_t nr = 1u << (kr + lsr), nc = 1u << (kc + lsc);
  if (q < kr) return {nr, p.rcoff[w], q, lsr, nr / 2};
  if (q < kr + kc) return {nc, p.rcoff[w] + nr, q - kr, lsc, nc / 2};
  return {nc, p.rcoff[w] + nr, 32u, 0u, nc};
}
// The k-th term of the quantity (k < cnt): the k-th partial whose row /
// column has the bit (exactly half of them), so the loops visit only the
// terms (round 5: U^C_b, U^D_b took twice the serial steps they needed).
ZK_DI uint32_t quant_term(const QuantSpan& s, uint32_t k) {
  if (s.bit == 32) return k;
  const uint32_t bb = s.bit + s.shift;
  return ((k >> bb) << (bb + 1)) | (1u << bb) | (k & ((1u << bb) - 1));
}

template <class X>
__device__ __forceinline__ X shfl_point(const X& v, int src) {
  constexpr int NW = sizeof(X) / 4;
  X o;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* d = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int k = 0; k < NW; k++) d[k] = __shfl(s[k], src);
  return o;
}

// The wave's 64 lane points summed by lane-quad adds (curve.hpp): the 32
// sums of lanes l and l + 32 (the caller's last single-lane step) are folded
// in 5 quad rounds -- 16 adds (quad j: lanes 2j, 2j + 1), then 8, 4, 2, 1 --
// instead of 5 more single-lane butterfly steps; a quad add issues about a
// third of a single-lane add's instructions, and these steps are the
// latency-bound tail of every sum.  The total is in lanes 0-3.
#ifndef ZK_ROWCOL_QTAIL
#define ZK_ROWCOL_QTAIL 1
#endif
template <class X>
ZK_DI X wave_tail_quad(const X& v) {
  const int j = (threadIdx.x & 63) >> 2;
  X t;
#pragma unroll 1
  for (int it = 0; it < 5; it++) {
    X a, b;
    if (it == 0) {
      a = shfl_point(v, 2 * j);
      b = shfl_point(v, 2 * j + 1);
    } else {
      a = t;
      b = shfl_xor_point(t, 64 >> it);
    }
    t = xyzz_add_quad(a, b);
  }
  return t;
}

// Row sums C_hi (2^kc contiguous buckets) and column sums D_lo (2^kr buckets
// at stride 2^kc) of every window, one wave each.
template <class C>
__global__ void __launch_bounds__(64 * MSM_RED_WAVES) k_msm_rowcol(MsmPlan p, const uint32_t* __restrict__ off,
                                                                  const typename C::X* __restrict__ buckets,
                                                                  typename C::X* __restrict__ rc) {
  using X = typename C::X;
  const uint32_t b = blockIdx.x * MSM_RED_WAVES + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (b >= p.nrc) return;   // whole waves
  const SumSpan sp = rowcol_span(p, b);
  const uint32_t len = sp.len, g0 = sp.g0, stride = sp.stride;
  const uint32_t niter = (len + 63) >> 6;
  constexpr uint32_t NB = ZK_ROWCOL_QTAIL ? 1 : 6;   // single-lane butterfly steps
  X v;
  xyzz_set_inf(v);
#pragma unroll 1
  for (uint32_t it = 0; it < niter + NB; it++) {
    X o;
    if (it < niter) {
      const uint32_t t = it * 64 + lane, g = g0 + t * stride;
      if (t < len && (p.all_valid || off[g + 1] != off[g])) o = ld_vec(&buckets[g]);
      else xyzz_set_inf(o);
    } else {
      o = shfl_xor_point(v, ZK_ROWCOL_QTAIL ? 32 : 1 << (it - niter));
    }
    v = tail_add(v, o);
  }
  if constexpr (ZK_ROWCOL_QTAIL) v = wave_tail_quad(v);
  if (lane == 0) st_vec(&rc[b], v);
}

// ---- lane-quad reductions (xyzz_add_quad) ------------------------------
// The same sums with each add split over the 4 lanes of a quad (curve.hpp):
// one sum per workgroup of RW waves = 16 RW quads.  Quad j folds terms j,
// j + 16 RW, ... serially, a 4-step __shfl_xor butterfly (lane distances
// 4..32 keep each lane's quad position) combines a wave, then a log2(RW)-step
// tree over LDS combines the waves (wave w + 2^k hands its total to wave w
// in step k).  One xyzz_add_quad call site.  The G1 quantities (tens of
// sums) run on quads, ZK_QUANT_WAVES_G1 waves per sum (4: one wave per SIMD,
// 2 terms per quad before the butterfly; round 5: prove 9.173 vs 9.252 ms
// with 8, median of 4 alternating processes, profiles/r05_ab_quant_waves.txt);
// the G2 ones on lane pairs (k_msm_quant_pair).
#ifndef ZK_QUANT_WAVES_G1
#define ZK_QUANT_WAVES_G1 4
#endif

constexpr int ilog2_c(int x) { return x <= 1 ? 0 : 1 + ilog2_c(x / 2); }

template <class X, int RW>
__device__ __forceinline__ X quad_sum_step(X v, uint32_t it, uint32_t niter, X* xs, bool have, const X& term) {
  X o;
  if (it < niter) {
    if (have) o = term;
    else xyzz_set_inf(o);
  } else if (it < niter + 4) {
    o = shfl_xor_point(v, 4 << (it - niter));
  } else {
    const uint32_t k = it - niter - 4, wave = threadIdx.x >> 6, m = 1u << k;
    __syncthreads();   // the previous step's reads are done
    if ((wave & (2 * m - 1)) == m && (threadIdx.x & 63) == 0) xs[wave >> (k + 1)] = v;
    __syncthreads();
    if ((wave & (2 * m - 1)) == 0) o = xs[wave >> (k + 1)];
    else xyzz_set_inf(o);
  }
  return o;
}

template <class C, int RW>
__global__ void __launch_bounds__(64 * RW) k_msm_quant_q(MsmPlan p, const typename C::X* __restrict__ rc,
                                                        typename C::X* __restrict__ res) {
  using X = typename C::X;
  __shared__ X xs[RW > 1 ? RW / 2 : 1];
  constexpr uint32_t NQ = 16 * RW;
  const uint32_t b = blockIdx.x;
  if (b >= p.nq) return;
  const QuantSpan qs = quant_span(p, b);
  const X* src = rc + qs.src;
  const uint32_t j = threadIdx.x >> 2;
  const uint32_t niter = (qs.cnt + NQ - 1) / NQ;
  X v;
  xyzz_set_inf(v);
#pragma unroll 1
  for (uint32_t it = 0; it < niter + 4 + ilog2_c(RW); it++) {
    X term;
    bool have = false;
    if (it < niter) {
      const uint32_t k = it * NQ + j;
      have = k < qs.cnt;
      if (have) term = ld_vec(&src[quant_term(qs, k)]);
    }
    const X o = quad_sum_step<X, RW>(v, it, niter, xs, have, term);
    v = xyzz_add_quad(v, o);
  }
  if (threadIdx.x == 0) st_vec(&res[b], v);
}

// ---- lane-pair G2 reductions (Fq2h) -------------------------------------
// G2 row/column sums and fixup with each add split over a lane pair: half the
// registers (two waves per SIMD) and half the multiply chain per add on the
// few hundred latency-bound sums.  Pair j of a wave folds terms j, j + 32,
// ...; the butterfly's lane distances 2..32 keep each lane's half.
ZK_DI XYZZ<Fq2h> ld_pair(const G2X* p) {
  const Fq* q = reinterpret_cast<const Fq*>(p) + pair_half();
  return {{ld_vec(q + 0)}, {ld_vec(q + 2)}, {ld_vec(q + 4)}, {ld_vec(q + 6)}};
}

// G2 reduction tails on lane duos (curve.hpp xyzz_add_duo: two lane pairs
// per add, half the pair add's dependent products).  ZK_G2_DUO=0: A/B build
// with the lane-pair butterflies.
#ifndef ZK_G2_DUO
#define ZK_G2_DUO 1
#endif
template <int K>
ZK_DI XYZZ<Fq2h> duo_bcast_point(const XYZZ<Fq2h>& v) {
  return {duo_bcast<K>(v.X), duo_bcast<K>(v.Y), duo_bcast<K>(v.ZZ), duo_bcast<K>(v.ZZZ)};
}
// The wave's 32 lane-pair points summed on duos: duo j first adds pairs 2j
// and 2j + 1 (its own two pairs), then 8, 4, 2, 1 duo adds across lanes
// 32 .. 4 apart.  The total is in lanes 0-3.
ZK_DI XYZZ<Fq2h> wave_tail_duo(const XYZZ<Fq2h>& v) {
  XYZZ<Fq2h> t;
#pragma unroll 1
  for (int it = 0; it < 5; it++) {
    XYZZ<Fq2h> a, b;
    if (it == 0) {
      a = duo_bcast_point<0>(v);
      b = duo_bcast_point<1>(v);
    } else {
      a = t;
      b = shfl_xor_point(t, 64 >> it);
    }
    t = xyzz_add_duo(a, b);
  }
  return t;
}

__global__ void __launch_bounds__(64 * MSM_RED_WAVES) k_msm_rowcol_pair(MsmPlan p, const uint32_t* __restrict__ off,
                                                                       const G2X* __restrict__ buckets,
                                                                       G2X* __restrict__ rc) {
  const uint32_t b = blockIdx.x * MSM_RED_WAVES + (threadIdx.x >> 6);
  const uint32_t pr = (threadIdx.x & 63) >> 1;
  if (b >= p.nrc) return;   // whole waves
  const SumSpan sp = rowcol_span(p, b);
  const uint32_t len = sp.len, g0 = sp.g0, stride = sp.stride;
  const uint32_t niter = (len + 31) >> 5;
  constexpr uint32_t NB = ZK_G2_DUO ? 0 : 5;   // lane-pair butterfly steps
  XYZZ<Fq2h> v;
  xyzz_set_inf(v);
#pragma unroll 1
  for (uint32_t it = 0; it < niter + NB; it++) {
    XYZZ<Fq2h> o;
    if (it < niter) {
      const uint32_t t = it * 32 + pr, g = g0 + t * stride;
      if (t < len && (p.all_valid || off[g + 1] != off[g])) o = ld_pair(&buckets[g]);
      else xyzz_set_inf(o);
    } else {
      o = shfl_xor_point(v, 2 << (it - niter));
    }
    v = tail_add(v, o);
  }
  if constexpr (ZK_G2_DUO) v = wave_tail_duo(v);
  if ((threadIdx.x & 63) < 2) st_pair(&rc[b], v);
}

// G2 quantities on lane pairs over ZK_QUANT_WAVES_G2 waves: pair j of the
// workgroup folds terms j, j + 32 RW, ..., a 5-step __shfl_xor butterfly
// (lane distances 2..32 keep each lane's half) combines a wave, then a
// log2(RW)-step tree over LDS combines the waves.  Round 5: was the lane-quad
// kernel on the full Fq2 point, which spills (792 B per lane) at one wave
// per SIMD.
#ifndef ZK_QUANT_WAVES_G2
#define ZK_QUANT_WAVES_G2 4
#endif
template <int RW>
__global__ void __launch_bounds__(64 * RW) k_msm_quant_pair(MsmPlan p, const G2X* __restrict__ rc,
                                                           G2X* __restrict__ res) {
  __shared__ XYZZ<Fq2h> xs[RW > 1 ? RW : 2];   // [slot][half]
  constexpr uint32_t NP = 32 * RW;
  constexpr uint32_t LR = ilog2_c(RW);
  const uint32_t b = blockIdx.x;
  if (b >= p.nq) return;   // whole workgroup
  const QuantSpan qs = quant_span(p, b);
  const G2X* src = rc + qs.src;
  const uint32_t j = threadIdx.x >> 1, wave = threadIdx.x >> 6;
  const uint32_t niter = (qs.cnt + NP - 1) / NP;
  XYZZ<Fq2h> v;
  xyzz_set_inf(v);
#pragma unroll 1
  for (uint32_t it = 0; it < niter + 5 + LR; it++) {
    XYZZ<Fq2h> o;
    if (it < niter) {
      const uint32_t k = it * NP + j;
      if (k < qs.cnt) o = ld_pair(&src[quant_term(qs, k)]);
      else xyzz_set_inf(o);
    } else if (it < niter + 5) {
      o = shfl_xor_point(v, 2 << (it - niter));
    } else {
      const uint32_t k = it - niter - 5, m = 1u << k;
      __syncthreads();   // the previous step's reads are done
      if ((wave & (2 * m - 1)) == m && (threadIdx.x & 63) < 2) xs[2 * (wave >> (k + 1)) + pair_half()] = v;
      __syncthreads();
      if ((wave & (2 * m - 1)) == 0) o = xs[2 * (wave >> (k + 1)) + pair_half()];
      else xyzz_set_inf(o);
    }
    v = tail_add(v, o);
  }
  if (threadIdx.x < 2) st_pair(&res[b], v);
}

// The G2 quantities on lane duos (ZK_G2_DUO): duo j of the workgroup folds
// terms j, j + 16 RW, ..., a 4-step __shfl_xor butterfly (lane distances
// 4 .. 32 keep each lane's duo position), then a log2(RW)-step LDS tree.
template <int RW>
__global__ void __launch_bounds__(64 * RW) k_msm_quant_duo(MsmPlan p, const G2X* __restrict__ rc,
                                                          G2X* __restrict__ res) {
  __shared__ XYZZ<Fq2h> xs[RW > 1 ? 2 * RW : 4];   // [slot][lane of the duo]
  constexpr uint32_t NU = 16 * RW;
  constexpr uint32_t LR = ilog2_c(RW);
  const uint32_t b = blockIdx.x;
  if (b >= p.nq) return;   // whole workgroup
  const QuantSpan qs = quant_span(p, b);
  const G2X* src = rc + qs.src;
  const uint32_t j = threadIdx.x >> 2, wave = threadIdx.x >> 6;
  const uint32_t niter = (qs.cnt + NU - 1) / NU;
  XYZZ<Fq2h> v;
  xyzz_set_inf(v);
#pragma unroll 1
  for (uint32_t it = 0; it < niter + 4 + LR; it++) {
    XYZZ<Fq2h> o;
    if (it < niter) {
      const uint32_t k = it * NU + j;
      if (k < qs.cnt) o = ld_pair(&src[quant_term(qs, k)]);
      else xyzz_set_inf(o);
    } else if (it < niter + 4) {
      o = shfl_xor_point(v, 4 << (it - niter));
    } else {
      const uint32_t k = it - niter - 4, m = 1u << k;
      __syncthreads();   // the previous step's reads are done
      if ((wave & (2 * m - 1)) == m && (threadIdx.x & 63) < 4) xs[4 * (wave >> (k + 1)) + (threadIdx.x & 3)] = v;
      __syncthreads();
      if ((wave & (2 * m - 1)) == 0) o = xs[4 * (wave >> (k + 1)) + (threadIdx.x & 3)];
      else xyzz_set_inf(o);
    }
    v = xyzz_add_duo(v, o);
  }
  if (threadIdx.x < 2) st_pair(&res[b], v);
}

// G2 fixup on lane pairs, per bucket or (by_boundary, more buckets than
// chunks: c = 22 at 2^24, 2^21 buckets over 65 K chunks) per chunk boundary as
// k_msm_fixup<G1> (round 5; one pair per bucket cost 1.15 ms per 2^24 proof).
__global__ void __launch_bounds__(128) k_msm_fixup_pair(const uint32_t* __restrict__ key,
                                                        const uint32_t* __restrict__ off, uint32_t G, uint32_t T,
                                                        uint32_t fix_max, bool by_boundary,
                                                        uint32_t* __restrict__ nbig, G2X* __restrict__ buckets,
                                                        const G2X* __restrict__ partials) {
  const uint32_t u = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;   // pair-uniform from here on
  const uint32_t K = chunk_len(off[G], T);
  uint32_t g = u;
  if (by_boundary) {
    if (u == 0 || u >= T || (uint64_t)u * K >= off[G]) return;
    g = key[u * K];
    if (off[g] / K != u - 1) return;   // not split here, or not its first boundary
  } else if (g >= G) {
    return;
  }
  const uint32_t bs = off[g], be = off[g + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  if (t1 - t0 + 1 > fix_max) {
    if (!pair_half()) atomicAdd(nbig, 1u);
    return;
  }
  XYZZ<Fq2h> acc = ld_pair(&partials[2 * (size_t)t0 + 1]);
#pragma unroll 1
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = tail_add(acc, ld_pair(&partials[2 * (size_t)t]));
  st_pair(&buckets[g], acc);
}

// Two parts of one split MSM (msm_batch_back COMBINE): bucket g = this
// part's bucket + the earlier part's, each only where its part had entries,
// written for EVERY bucket (infinity where both are empty), so the reduction
// reads them all (MsmPlan::all_valid).
// prev_all: the earlier part's every bucket holds a value (it combined
// with a part before it).
template <class C>
__global__ void __launch_bounds__(128) k_msm_combine(const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ off_prev, bool prev_all, uint32_t G,
                                                     typename C::X* __restrict__ buckets,
                                                     const typename C::X* __restrict__ prev) {
  using X = typename C::X;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  X a, b;
  if (off[g + 1] != off[g]) a = ld_vec(&buckets[g]);
  else xyzz_set_inf(a);
  if (prev_all || off_prev[g + 1] != off_prev[g]) b = ld_vec(&prev[g]);
  else xyzz_set_inf(b);
  st_vec(&buckets[g], tail_add(a, b));
}
__global__ void __launch_bounds__(128) k_msm_combine_pair(const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ off_prev, bool prev_all,
                                                          uint32_t G, G2X* __restrict__ buckets,
                                                          const G2X* __restrict__ prev) {
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (g >= G) return;   // pair-uniform
  XYZZ<Fq2h> a, b;
  if (off[g + 1] != off[g]) a = ld_pair(&buckets[g]);
  else xyzz_set_inf(a);
  if (prev_all || off_prev[g + 1] != off_prev[g]) b = ld_pair(&prev[g]);
  else xyzz_set_inf(b);
  st_pair(&buckets[g], tail_add(a, b));
}

// ------------------------------------------------------------ driver -----

// Accumulate threads: one full-occupancy round of the chip (blocks per CU
// from the occupancy calculator x CUs x 128; G2 runs two lanes per chunk).
template <class C>
static uint32_t accum_threads() {
  static const uint32_t T = [] {
    int dev = 0, cus = 0, per_cu = 0;
    ZK_HIP(hipGetDevice(&dev));
    ZK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    constexpr bool pair = std::is_same<C, G2>::value;
    if constexpr (pair)
      ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_msm_accum_pair, 128, 0));
    else
      ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_msm_accum<C>, 128, 0));
#ifdef ZK_ACCUM_G1_WAVES
    if constexpr (!pair) per_cu = std::min(per_cu, ZK_ACCUM_G1_WAVES * 2);   // 128-thread blocks: 2 waves
#endif
#ifdef ZK_ACCUM_G2_WAVES
    if constexpr (pair) per_cu = std::min(per_cu, ZK_ACCUM_G2_WAVES * 2);
#endif
    return (uint32_t)std::max(1, per_cu * cus * (pair ? 64 : 128));
  }();
  return T;
}

// Blocks of the merge kernel the chip holds at once (its occupancy x CUs):
// the upper bound of its grid-barrier launch.
template <class C>
static uint32_t merge_max_blocks() {
  static const uint32_t B = [] {
    int dev = 0, cus = 0, per_cu = 0;
    ZK_HIP(hipGetDevice(&dev));
    ZK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_msm_merge<C>, 128, 0));
    return (uint32_t)std::max(0, per_cu * cus);
  }();
  return B;
}

// Waves of one row/column-sum launch that the chip holds at once (the
// kernel's occupancy x CUs), for msm_split_sums.
template <class C>
static uint32_t rowcol_waves() {
  static const uint32_t W = [] {
    int dev = 0, cus = 0, per_cu = 0;
    ZK_HIP(hipGetDevice(&dev));
    ZK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if constexpr (std::is_same<C, G2>::value)
      ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_msm_rowcol_pair, 64 * MSM_RED_WAVES, 0));
    else
      ZK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_msm_rowcol<C>, 64 * MSM_RED_WAVES, 0));
    return (uint32_t)std::max(1, per_cu * cus * MSM_RED_WAVES);
  }();
  return W;
}

// Split row/column sums into partial sums (MsmPlan::lsr/lsc) while the
// launch stays within `target` waves and every partial keeps >= 2 terms per
// lane group (`lanes` terms per wave step): each wave then runs fewer serial
// adds before its butterfly, and the waves fill the SIMDs evenly instead of
// a few long row waves setting the time.  Always the side whose partials are
// longest first.  The quantities fold the partials with their row's or
// column's weight.
// Measured (profiles/r03_ab_split_sums.txt): the standalone 2^20 255-bit G1
// MSM 3.75 -> 3.64 ms (2^19 buckets: 1536 waves of 22 / 14 steps -> 2048 of
// 14); the overlapped prove is unchanged by the G1 split (9.62 vs 9.60 ms)
// and 0.3-0.4 ms SLOWER with the G2 split (its 1024 lane-pair waves crowd the
// quotient and the A+B1+IC sort, which gate the critical path), so G2 keeps
// whole sums (ZK_SPLIT_G2=1: A/B build flag).
#ifndef ZK_SPLIT_G1
#define ZK_SPLIT_G1 1
#endif
#ifndef ZK_SPLIT_G2
#define ZK_SPLIT_G2 0
#endif
// Partials keep >= ZK_SPLIT_MIN terms per lane: the prove plans' 256-term
// rows and columns stay whole (4 per lane; their quantities then fold 128
// terms instead of 256-512), the standalone plans' 512-1024-term sums split
// to 256.  Round 6 (2 -> 4, profiles/r06_ab_split_min.txt): serial A+B1
// bucket sum 0.298 -> 0.245 ms, overlapped prove median 8.626 -> 8.511 ms,
// configs[1] MSM unchanged (3.27-3.29 ms); no split at all cost that MSM
// 0.1 ms.
#ifndef ZK_SPLIT_MIN
#define ZK_SPLIT_MIN 4
#endif
static void msm_split_sums(MsmPlan& p, uint32_t target, uint32_t lanes) {
  auto recount = [&]() {
    uint32_t rc = 0;
    for (uint32_t w = 0; w < p.nred; w++) {
      p.rcoff[w] = rc;
      rc += (1u << (p.kr[w] + p.lsr[w])) + (1u << (p.kc[w] + p.lsc[w]));
    }
    p.rcoff[p.nred] = p.nrc = rc;
  };
  for (;;) {
    int bw = -1;
    bool brow = false;
    uint32_t blen = 0;
    for (uint32_t w = 0; w < p.nred; w++) {
      const uint32_t rlen = 1u << (p.kc[w] - p.lsr[w]), clen = 1u << (p.kr[w] - p.lsc[w]);
      if (rlen > blen) { blen = rlen; bw = (int)w; brow = true; }
      if (clen > blen) { blen = clen; bw = (int)w; brow = false; }
    }
    if (bw < 0 || blen / 2 < ZK_SPLIT_MIN * lanes) break;
    const uint32_t add = brow ? 1u << (p.kr[bw] + p.lsr[bw]) : 1u << (p.kc[bw] + p.lsc[bw]);
    if ((uint64_t)p.nrc + add > target) break;
    (brow ? p.lsr : p.lsc)[bw]++;
    recount();
  }
}

// Buckets spread over at most this many accumulate chunks are summed by the
// serial fixup; larger ones go through the log-depth merge.
constexpr uint32_t MSM_FIX_MAX = 8;

// One MSM (nseg = 1) or a batch of MSMs sharing every phase: segment k's
// keys start at bucket k << segshift and its entries at sum_{j<k} nwin n_j.
template <class C>
static void msm_front_impl(MsmWork& w, const MsmSeg* segs, int nseg, int sw, hipStream_t st) {
  using X = typename C::X;
  constexpr bool g2 = std::is_same<C, G2>::value;
  MsmPlan& p = w.plan;
  if (nseg < 1 || nseg > MSM_MAXSEG || (nseg > 1 && (!p.shared || sw != 1)))
    throw Error(ZK_ERR_ARG, "msm: bad batch");
  size_t M = 0;
  for (int k = 0; k < nseg; k++) M += (size_t)segs[k].n * p.nwin;
  if (M >= 0x80000000ull) throw Error(ZK_ERR_ARG, "msm: too many (point, window) entries");
  const uint32_t n = p.n;   // all points of the batch (profiling units)
  w.off.ensure(sizeof(uint32_t) * (p.G + 1));
  w.ent.ensure(sizeof(uint32_t) * (M + ENTQ));   // EntQ reads up to ENTQ - 1 past the end
  w.key.ensure(sizeof(uint32_t) * (M + ENTQ));
  w.buckets.ensure(sizeof(X) * p.G);
  p.T = accum_threads<C>();
  p.fix_max = MSM_FIX_MAX;
  // row/column sums: G2 on lane pairs, G1 one lane per add (lane-quad tail),
  // split to fill the chip.  Round 5: the H MSM's 512 sums moved from lane
  // quads (4 waves per sum) to this form, bucket sum 0.285 -> 0.246 ms serial
  // (profiles/r05_ab_qtail_slowbox.txt)
  if (g2 ? ZK_SPLIT_G2 : ZK_SPLIT_G1) msm_split_sums(p, rowcol_waves<C>(), g2 ? 32u : 64u);
  w.partials.ensure(sizeof(X) * 2 * (size_t)p.T);
  w.partials2.ensure(sizeof(X) * ((size_t)p.T / 2 + 2));
  w.rc.ensure(sizeof(X) * p.nrc);
  w.res.ensure(sizeof(X) * p.nq);
  SegBases<typename C::A> sb{};
  sb.stride = segs[0].stride ? segs[0].stride : (uint32_t)sizeof(typename C::A);
  for (int k = 0; k < nseg; k++) {
    sb.p[k] = static_cast<const char*>(segs[k].bases);
    if ((segs[k].stride ? segs[k].stride : (uint32_t)sizeof(typename C::A)) != sb.stride)
      throw Error(ZK_ERR_ARG, "msm: batch segments with different base strides");
  }

  Prof* pf = w.prof;
  int ph = pf ? pf->begin(st, (w.tag + "msm_sort").c_str(), n) : -1;
  // group the (point, window) entries by bucket: stable counting sort (group.hip)
  msm_group(w, segs, nseg, sw, st);
  if (pf) pf->end(st, ph);
  // The number of non-zero digits M' <= M is known on device only: the T
  // accumulate threads split it evenly there (chunk_len), no host sync.
  if (M) {
    ph = pf ? pf->begin(st, (w.tag + (g2 ? "msm_accum_g2" : "msm_accum_g1")).c_str(), n) : -1;
    if constexpr (g2)
      k_msm_accum_pair<<<ceil_div(2 * (size_t)p.T, 128), 128, 0, st>>>(sb, p.segshift, w.ent.as<uint32_t>(),
                                                                        w.key.as<uint32_t>(), w.off.as<uint32_t>(),
                                                                        p.G, p.T, w.buckets.as<X>(),
                                                                        w.partials.as<X>());
    else
      k_msm_accum<C><<<ceil_div(p.T, 128), 128, 0, st>>>(sb, p.segshift, w.ent.as<uint32_t>(), w.key.as<uint32_t>(),
                                                          w.off.as<uint32_t>(), p.G, p.T, w.buckets.as<X>(),
                                                          w.partials.as<X>());
    ZK_LAUNCH_CHECK();
    if (pf) pf->end(st, ph);
  }
}

template <class C>
static void msm_back_impl(MsmWork& w, hipStream_t st, int mode, const MsmWork* prev) {
  using X = typename C::X;
  constexpr bool g2 = std::is_same<C, G2>::value;
  MsmPlan& p = w.plan;
  Prof* pf = w.prof;
  const uint32_t n = p.n;
  (void)n;
  int ph = pf ? pf->begin(st, (w.tag + "msm_merge").c_str(), p.G) : -1;   // buckets split across chunks
  // ctl (w.nbig, zeroed by the front's k_msm_offsets): [0] buckets left to
  // the merge, [1] its grid barrier
  const bool by_boundary = p.G > p.T;
  const size_t fix_n = by_boundary ? p.T : p.G;
  if constexpr (g2)
    k_msm_fixup_pair<<<ceil_div(2 * fix_n, 128), 128, 0, st>>>(
        w.key.as<uint32_t>(), w.off.as<uint32_t>(), p.G, p.T, p.fix_max, by_boundary, w.nbig.as<uint32_t>(),
        reinterpret_cast<G2X*>(w.buckets.p), reinterpret_cast<const G2X*>(w.partials.p));
  else
    k_msm_fixup<C><<<ceil_div(fix_n, 128), 128, 0, st>>>(w.key.as<uint32_t>(), w.off.as<uint32_t>(), p.G, p.T,
                                                          p.fix_max, by_boundary, w.nbig.as<uint32_t>(),
                                                          w.buckets.as<X>(), w.partials.as<X>());
  ZK_LAUNCH_CHECK();
  {
    // level l merges groups of FAN^l chunks; T chunks at most.  The levels
    // ping-pong between partials (level 0 = the chunks) and partials2.
    uint32_t nlevels = 0;
    while ((1ull << (ZK_MERGE_FAN_LOG * nlevels)) < p.T) nlevels++;
    const uint32_t groups1 = (uint32_t)(((uint64_t)p.T + MSM_MERGE_FAN - 1) >> ZK_MERGE_FAN_LOG);
    if (nlevels) {
      // a small grid-stride grid: the common case exits at once and should
      // not queue hundreds of blocks behind other streams' long kernels; at
      // most the blocks the chip holds at once (the grid barrier's bound)
      const uint32_t grid = std::min<uint32_t>(std::min<uint32_t>(ceil_div(groups1, 128), 64), merge_max_blocks<C>());
      if (grid < 1 || grid > merge_max_blocks<C>()) throw Error(ZK_ERR_DEVICE, "msm: merge grid exceeds residency");
      k_msm_merge<C><<<grid, 128, 0, st>>>(
          w.key.as<uint32_t>(), w.off.as<uint32_t>(), p.G, p.T, p.fix_max, nlevels, w.nbig.as<uint32_t>(),
          w.buckets.as<X>(), w.partials.as<X>(), w.partials2.as<X>());
      ZK_LAUNCH_CHECK();
    }
  }
  p.all_valid = 0;
  if (mode == MSM_BACK_COMBINE || mode == MSM_BACK_ACCUM) {
    if (!prev || prev->plan.G != p.G || prev->plan.nseg != p.nseg) throw Error(ZK_ERR_ARG, "msm: combine plans differ");
    const bool prev_all = prev->plan.all_valid != 0;
    if constexpr (g2)
      k_msm_combine_pair<<<ceil_div(2 * (size_t)p.G, 128), 128, 0, st>>>(
          w.off.as<uint32_t>(), prev->off.as<uint32_t>(), prev_all, p.G, reinterpret_cast<G2X*>(w.buckets.p),
          reinterpret_cast<const G2X*>(prev->buckets.p));
    else
      k_msm_combine<C><<<ceil_div(p.G, 128), 128, 0, st>>>(w.off.as<uint32_t>(), prev->off.as<uint32_t>(), prev_all,
                                                            p.G, w.buckets.as<X>(), prev->buckets.as<X>());
    ZK_LAUNCH_CHECK();
    p.all_valid = 1;
  }
  if (pf) pf->end(st, ph);
  if (mode == MSM_BACK_FIXUP || mode == MSM_BACK_ACCUM) return;
  ph = pf ? pf->begin(st, (w.tag + "msm_bucket_sum").c_str(), p.G) : -1;   // row/col sums + quantities
  if constexpr (g2)
    k_msm_rowcol_pair<<<ceil_div(p.nrc, MSM_RED_WAVES), 64 * MSM_RED_WAVES, 0, st>>>(
        p, w.off.as<uint32_t>(), reinterpret_cast<const G2X*>(w.buckets.p), reinterpret_cast<G2X*>(w.rc.p));
  else
    k_msm_rowcol<C><<<ceil_div(p.nrc, MSM_RED_WAVES), 64 * MSM_RED_WAVES, 0, st>>>(p, w.off.as<uint32_t>(),
                                                                                  w.buckets.as<X>(), w.rc.as<X>());
  ZK_LAUNCH_CHECK();
  if constexpr (g2) {
    if constexpr (ZK_G2_DUO)
      k_msm_quant_duo<ZK_QUANT_WAVES_G2><<<p.nq, 64 * ZK_QUANT_WAVES_G2, 0, st>>>(
          p, reinterpret_cast<const G2X*>(w.rc.p), reinterpret_cast<G2X*>(w.res.p));
    else
      k_msm_quant_pair<ZK_QUANT_WAVES_G2><<<p.nq, 64 * ZK_QUANT_WAVES_G2, 0, st>>>(
          p, reinterpret_cast<const G2X*>(w.rc.p), reinterpret_cast<G2X*>(w.res.p));
  }
  else
    k_msm_quant_q<C, ZK_QUANT_WAVES_G1><<<p.nq, 64 * ZK_QUANT_WAVES_G1, 0, st>>>(p, w.rc.as<X>(), w.res.as<X>());
  ZK_LAUNCH_CHECK();
  if (pf) pf->end(st, ph);
}

template <class C>
void msm_launch(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw, uint32_t n,
                int bits, hipStream_t st, uint32_t stride) {
  w.plan = msm_make_plan(n, bits, sw);
  const MsmSeg seg{d_bases, d_scalars, n, stride};
  msm_front_impl<C>(w, &seg, 1, sw, st);
  msm_back_impl<C>(w, st, MSM_BACK_FULL, nullptr);
}

template <class C>
void msm_launch_shared(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw, uint32_t n,
                       int bits, int c, hipStream_t st, uint32_t stride) {
  w.plan = msm_make_plan_shared(n, bits, sw, c);
  if ((uint64_t)n * w.plan.nwin >= MSM_DUMMY) throw Error(ZK_ERR_ARG, "msm: too many window bases");
  const MsmSeg seg{d_bases, d_scalars, n, stride};
  msm_front_impl<C>(w, &seg, 1, sw, st);
  msm_back_impl<C>(w, st, MSM_BACK_FULL, nullptr);
}

template <class C>
void msm_launch_batch(MsmWork& w, const MsmSeg* segs, int nseg, int bits, int c, hipStream_t st) {
  if (nseg < 1 || nseg > MSM_MAXSEG) throw Error(ZK_ERR_ARG, "msm: batch of 1..4 MSMs");
  w.plan = msm_make_plan_batch(segs, nseg, bits, c);
  for (int k = 0; k < nseg; k++)
    if ((uint64_t)segs[k].n * w.plan.nwin >= MSM_DUMMY) throw Error(ZK_ERR_ARG, "msm: too many window bases");
  msm_front_impl<C>(w, segs, nseg, 1, st);
  msm_back_impl<C>(w, st, MSM_BACK_FULL, nullptr);
}

template <class C>
void msm_batch_front(MsmWork& w, const MsmSeg* segs, int nseg, int bits, int c, hipStream_t st) {
  if (nseg < 1 || nseg > MSM_MAXSEG) throw Error(ZK_ERR_ARG, "msm: batch of 1..4 MSMs");
  w.plan = msm_make_plan_batch(segs, nseg, bits, c);
  for (int k = 0; k < nseg; k++) {
    const uint64_t ws = segs[k].wstride ? segs[k].wstride : segs[k].n;
    if ((uint64_t)segs[k].ioff + segs[k].n > ws || ws * w.plan.nwin >= MSM_DUMMY)
      throw Error(ZK_ERR_ARG, "msm: bad window-base range");
  }
  msm_front_impl<C>(w, segs, nseg, 1, st);
}

template <class C>
void msm_batch_back(MsmWork& w, hipStream_t st, int mode, const MsmWork* prev) {
  msm_back_impl<C>(w, st, mode, prev);
}

// ------------------------------------------- precomputed window bases -----
constexpr int NORM_CHUNK = 16;
template <class C>
__global__ void __launch_bounds__(128) k_normalize(const typename C::X* __restrict__ in, size_t n,
                                                   typename C::F* __restrict__ pre,
                                                   typename C::A* __restrict__ out) {
  using F = typename C::F;
  const size_t c0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * NORM_CHUNK;
  if (c0 >= n) return;
  const size_t c1 = min(c0 + NORM_CHUNK, n);
  F run;
  f_set_one(run);
  for (size_t j = c0; j < c1; j++) {
    pre[j] = run;
    const F z = ld_vec(&in[j]).ZZZ;
    if (!f_is_zero(z)) run = f_mul(run, z);
  }
  F inv = f_inv(run);
  for (size_t j = c1; j-- > c0;) {
    const typename C::X q = ld_vec(&in[j]);
    typename C::A a;
    if (f_is_zero(q.ZZZ)) {
      f_set_zero(a.x);
      f_set_zero(a.y);
    } else {
      const F i3 = f_mul(inv, pre[j]);   // ZZZ^-1 = Z^-3
      inv = f_mul(inv, q.ZZZ);
      const F zi = f_mul(q.ZZ, i3);      // Z^-1
      a.x = f_mul(q.X, f_sqr(zi));
      a.y = f_mul(q.Y, i3);
    }
    st_vec(&out[j], a);
  }
}

template <class C>
void batch_normalize(const typename C::X* d_in, size_t n, typename C::F* d_pre, typename C::A* d_out,
                     hipStream_t st) {
  if (!n) return;
  k_normalize<C><<<ceil_div(ceil_div(n, NORM_CHUNK), 128), 128, 0, st>>>(d_in, n, d_pre, d_out);
  ZK_LAUNCH_CHECK();
}

// out[i] = 2^c in[i] (XYZZ)
template <class C>
__global__ void __launch_bounds__(128) k_shift_bases(const typename C::A* __restrict__ in, size_t n, int c,
                                                     typename C::X* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const typename C::A a = ld_vec(&in[i]);
  typename C::X q;
  if (aff_is_inf(a)) {
    xyzz_set_inf(q);
  } else {
    q = aff_dbl(a);
    for (int k = 1; k < c; k++) q = xyzz_dbl(q);
  }
  st_vec(&out[i], q);
}

template <class C>
void msm_precompute_windows(typename C::A* d_bases, size_t n, int W, int c, hipStream_t st) {
  if (!n || W < 2) return;
  DevBuf xs, pre;
  xs.ensure(sizeof(typename C::X) * n);
  pre.ensure(sizeof(typename C::F) * n);
  for (int w = 1; w < W; w++) {
    k_shift_bases<C><<<ceil_div(n, 128), 128, 0, st>>>(d_bases + (size_t)(w - 1) * n, n, c,
                                                        xs.as<typename C::X>());
    ZK_LAUNCH_CHECK();
    batch_normalize<C>(xs.as<typename C::X>(), n, pre.as<typename C::F>(), d_bases + (size_t)w * n, st);
  }
  ZK_HIP(hipStreamSynchronize(st));   // xs / pre die here
}

// out element i (ow 16-B words) = in element i (iw words) followed by zeros
__global__ void __launch_bounds__(256) k_pad_copy(const uint4* __restrict__ in, size_t n, uint32_t iw, uint32_t ow,
                                                  uint4* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * ow) return;
  const size_t i = t / ow;
  const uint32_t k = (uint32_t)(t - i * ow);
  out[t] = k < iw ? in[i * iw + k] : make_uint4(0, 0, 0, 0);
}

template <class C>
uint32_t msm_pad_bases(DevBuf& d, size_t n, hipStream_t st) {
  constexpr uint32_t sz = sizeof(typename C::A), padded = (sz + 127) / 128 * 128;
  if (padded == sz) return 0;
  DevBuf out;
  out.ensure((size_t)padded * std::max<size_t>(n, 1));
  if (n) {
    k_pad_copy<<<ceil_div(n * (padded / 16), 256), 256, 0, st>>>(d.as<uint4>(), n, sz / 16, padded / 16,
                                                                  out.as<uint4>());
    ZK_LAUNCH_CHECK();
  }
  ZK_HIP(hipStreamSynchronize(st));   // the packed copy dies here
  d = std::move(out);
  return padded;
}

template <class C>
void msm_download(MsmWork& w, hipStream_t st) {
  using X = typename C::X;
  const size_t bytes = sizeof(X) * w.plan.nq;
  w.host_res.ensure(bytes);
  ZK_HIP(hipMemcpyAsync(w.host_res.p, w.res.p, bytes, hipMemcpyDeviceToHost, st));
}

// Device XYZZ (32-bit limbs) and host XYZZ (64-bit limbs) share their bytes.
// Every quantity is a point times a power of two:
//   U^C_b : 2^(c w + kc + b),  U^D_b : 2^(c w + b),  P : 2^(c w)
// so one Horner pass over exponents from the top combines everything.
// seg < 0: every reduction window (one MSM); seg = k: window k alone (MSM k
// of a batch, weight 1).
template <class C>
static host::X<typename C::HF> msm_finish_impl(const MsmWork& w, int seg) {
  using HF = typename C::HF;
  using HX = host::X<HF>;
  static_assert(sizeof(HX) == sizeof(typename C::X), "layout");
  const MsmPlan& p = w.plan;
  const HX* r = w.host_res.as<const HX>();
  // reduction window `win` carries weight 2^(c win); a shared plan has one
  // window of weight 1 (the shifts live in the precomputed bases), a batch
  // one window of weight 1 per MSM
  auto wexp = [&](int win) { return p.shared ? 0 : p.c * win; };
  const int w0 = seg < 0 ? 0 : seg, w1 = seg < 0 ? (int)p.nred : seg + 1;
  int maxe = 0;
  for (int win = w0; win < w1; win++)
    maxe = std::max(maxe, wexp(win) + std::max<int>(p.kc[win] + p.kr[win] - 1, p.kc[win]));
  std::vector<std::vector<const HX*>> at(maxe + 1);
  for (int win = w0; win < w1; win++) {
    const int kr = p.kr[win], kc = p.kc[win];
    for (int q = 0; q < kr + kc + 1; q++) {
      int e = q < kr ? wexp(win) + kc + q : q < kr + kc ? wexp(win) + (q - kr) : wexp(win);
      at[e].push_back(&r[p.qoff[win] + q]);
    }
  }
  HX acc = host::inf<HF>();
  auto host_form = [](const HX& d) {   // device Montgomery radix -> host radix, per coordinate
    return HX{host::to_host(d.X_), host::to_host(d.Y), host::to_host(d.ZZ), host::to_host(d.ZZZ)};
  };
  for (int e = maxe; e >= 0; e--) {
    acc = host::dbl(acc);
    for (const HX* t : at[e]) acc = host::addp(acc, host_form(*t));
  }
  return acc;
}

template <class C>
host::X<typename C::HF> msm_finish(const MsmWork& w) {
  if (w.plan.nseg > 1) throw Error(ZK_ERR_ARG, "msm: batch results are per segment");
  return msm_finish_impl<C>(w, -1);
}

template <class C>
host::X<typename C::HF> msm_finish_seg(const MsmWork& w, int seg) {
  if (seg < 0 || seg >= w.plan.nseg) throw Error(ZK_ERR_ARG, "msm: no such batch segment");
  return msm_finish_impl<C>(w, seg);
}

// --------------------------------------------------- base conversion -----
__device__ __forceinline__ Fq load_canon_fq(const uint64_t* w) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    r.v[2 * i] = (uint32_t)w[i];
    r.v[2 * i + 1] = (uint32_t)(w[i] >> 32);
  }
  return fp_to_mont(r);
}
__device__ __forceinline__ void load_abi(const uint64_t* w, G1A& a) {
  if (w[12] & 0xff) { a.x = fp_zero<FqParams>(); a.y = fp_zero<FqParams>(); return; }
  a.x = load_canon_fq(w);
  a.y = load_canon_fq(w + 6);
}
__device__ __forceinline__ void load_abi(const uint64_t* w, G2A& a) {
  if (w[24] & 0xff) { a.x = fq2_zero(); a.y = fq2_zero(); return; }
  a.x.c0 = load_canon_fq(w);
  a.x.c1 = load_canon_fq(w + 6);
  a.y.c0 = load_canon_fq(w + 12);
  a.y.c1 = load_canon_fq(w + 18);
}
template <class C>
__global__ void __launch_bounds__(256) k_convert_bases(const uint64_t* __restrict__ in,
                                                       const uint32_t* __restrict__ idx,
                                                       typename C::A* __restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  size_t src = idx ? idx[i] : i;
  typename C::A a;
  load_abi(in + src * C::ABI_WORDS, a);
  st_vec(&out[i], a);
}
template <class C>
void convert_bases(const uint64_t* d_abi, typename C::A* d_out, size_t n, hipStream_t st) {
  if (!n) return;
  k_convert_bases<C><<<ceil_div(n, 256), 256, 0, st>>>(d_abi, nullptr, d_out, n);
  ZK_LAUNCH_CHECK();
}
template <class C>
void convert_bases_gather(const uint64_t* d_abi, const uint32_t* d_idx, typename C::A* d_out, size_t n,
                          hipStream_t st) {
  if (!n) return;
  k_convert_bases<C><<<ceil_div(n, 256), 256, 0, st>>>(d_abi, d_idx, d_out, n);
  ZK_LAUNCH_CHECK();
}

// ------------------------------------------------- host -> ABI words -----
static void fq_out(const host::Fq& m, uint64_t* w) {
  host::Fq c = host::from_mont(m);
  std::memcpy(w, c.l, 48);
}
template <>
void host_to_abi<G1>(const host::X<host::Fq>& p, uint64_t* w) {
  std::memset(w, 0, 13 * 8);
  host::Fq x, y;
  if (!host::to_affine(p, x, y)) { w[12] = 1; return; }
  fq_out(x, w);
  fq_out(y, w + 6);
}
template <>
void host_to_abi<G2>(const host::X<host::Fq2>& p, uint64_t* w) {
  std::memset(w, 0, 25 * 8);
  host::Fq2 x, y;
  if (!host::to_affine(p, x, y)) { w[24] = 1; return; }
  fq_out(x.c0, w);
  fq_out(x.c1, w + 6);
  fq_out(y.c0, w + 12);
  fq_out(y.c1, w + 18);
}

#define ZK_MSM_INST(C)                                                                               \
  template void msm_launch<C>(MsmWork&, const C::A*, const uint64_t*, int, uint32_t, int, hipStream_t,  \
                              uint32_t);                                                              \
  template void msm_launch_shared<C>(MsmWork&, const C::A*, const uint64_t*, int, uint32_t, int, int,   \
                                     hipStream_t, uint32_t);                                          \
  template uint32_t msm_pad_bases<C>(DevBuf&, size_t, hipStream_t);                                  \
  template void msm_precompute_windows<C>(C::A*, size_t, int, int, hipStream_t);                       \
  template void batch_normalize<C>(const C::X*, size_t, C::F*, C::A*, hipStream_t);                    \
  template void msm_download<C>(MsmWork&, hipStream_t);                                              \
  template host::X<C::HF> msm_finish<C>(const MsmWork&);                                            \
  template host::X<C::HF> msm_finish_seg<C>(const MsmWork&, int);                                   \
  template void msm_launch_batch<C>(MsmWork&, const MsmSeg*, int, int, int, hipStream_t);            \
  template void msm_batch_front<C>(MsmWork&, const MsmSeg*, int, int, int, hipStream_t);             \
  template void msm_batch_back<C>(MsmWork&, hipStream_t, int, const MsmWork*);                       \
  template void convert_bases<C>(const uint64_t*, C::A*, size_t, hipStream_t);                       \
  template void convert_bases_gather<C>(const uint64_t*, const uint32_t*, C::A*, size_t, hipStream_t);
ZK_MSM_INST(G1)
ZK_MSM_INST(G2)

}  // namespace zk
