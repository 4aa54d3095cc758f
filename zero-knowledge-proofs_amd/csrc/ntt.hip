// ntt.hip -- LDS-tiled radix-2 NTT passes over Fr (see ntt.hpp).
#include <algorithm>
#include <vector>

#include "ntt.hpp"

namespace zk {

// 2^NTT_TILE_LOG elements per tile: 1024 x 32 B = 32 KiB of LDS per
// workgroup (ZK_NTT_TILE_LOG: A/B builds only).  Round 3: 1024-element tiles
// (256 threads, 5 workgroups per CU instead of 2 x 512 threads) beat 2048
// once the tile arithmetic went to [0, 2r): 2^22 0.506 -> 0.499 ms with 3
// passes instead of 2, 2^24 2.35 -> 2.17 ms, 2^20 0.154 -> 0.156 ms
// (profiles/r03_ab_ntt_tile_radix2.txt)
#ifndef ZK_NTT_TILE_LOG
#define ZK_NTT_TILE_LOG 10
#endif
constexpr int NTT_TILE_LOG = ZK_NTT_TILE_LOG;
// Radix of the register rounds (2^NTT_R elements per thread) and threads per
// tile: one group per thread for a full tile.
#ifndef ZK_NTT_R
#define ZK_NTT_R 2
#endif
constexpr int NTT_R = ZK_NTT_R;
constexpr int NTT_THREADS = (1 << NTT_TILE_LOG) >> NTT_R;
// Tile arithmetic in [0, 2r) (ZK_NTT_LAZY, default on): products skip their
// final subtraction (a Montgomery product of inputs < 2^256 is < 2r with
// R = 2^261), and the butterflies' sums and differences reduce modulo 2r
// instead of r, which costs the same as the canonical fp_add / fp_sub.  2r <
// 2^256, so tile values keep the 8-word layout; every pass canonicalises on
// its store.
#ifndef ZK_NTT_LAZY
#define ZK_NTT_LAZY 1
#endif
ZK_DI Fr fr_mul_lz(const Fr& a, const Fr& b) { return fp_mul<FrParams, !ZK_NTT_LAZY>(a, b); }
ZK_DI Fr fr_add_lz(const Fr& a, const Fr& b) {
  if constexpr (!ZK_NTT_LAZY) return fp_add(a, b);
  Fr s, t;
  uint32_t c = 0, bw = 0, k2 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t m2 = (FrParams::MOD[i] << 1) | k2;   // 2r, word i (constant-folded)
    k2 = FrParams::MOD[i] >> 31;
    t.v[i] = __builtin_subc(s.v[i], m2, bw, &bw);
  }
  const bool take_t = c || !bw;   // a + b >= 2r (a carry out means >= 2^256 > 2r)
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = take_t ? t.v[i] : s.v[i];
  return s;
}
ZK_DI Fr fr_sub_lz(const Fr& a, const Fr& b) {
  if constexpr (!ZK_NTT_LAZY) return fp_sub(a, b);
  Fr d;
  uint32_t br = 0, c = 0, k2 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t m2 = (FrParams::MOD[i] << 1) | k2;
    k2 = FrParams::MOD[i] >> 31;
    d.v[i] = __builtin_addc(d.v[i], m2 & mask, c, &c);
  }
  return d;
}
// [0, 2r) -> canonical
ZK_DI Fr fr_canon_lz(const Fr& a) {
  if constexpr (!ZK_NTT_LAZY) return a;
  return fp_reduce_once(a);
}

// v * w for a pre-cut twiddle
ZK_DI Fr fr_mul_wu(const Fr& v, const FrU& w) {
  uint32_t x[FrParams::NL];
  unpack28<8, FrParams::NL, FrParams::LB>(v.v, x);
  return fp_mul_limbs<FrParams, !ZK_NTT_LAZY>(x, w.l);
}

// One radix-2^R round of a tile's sub-transform: local stages
// [lsb, lsb + R).  Each thread owns whole groups of 2^R elements (rows
// r0 + m 2^lsb, one column), keeps them in registers for all R stages and
// touches LDS once per round (16-byte accesses), so a 10-stage tile costs 5
// LDS round trips and 5 barriers instead of 10.  Twiddle of local stage t
// for row r: omega_(2^(t+1))^(r mod 2^t) = omega_2048^((r mod 2^t) 2^(10-t)).
template <int R, int Q, bool DIT, bool LSB0>
__device__ __forceinline__ void ntt_stage(Fr (&x)[1 << R], const FrU* __restrict__ sm, uint32_t rlow, uint32_t lsb) {
  constexpr int G = 1 << R;
  const uint32_t t = lsb + Q;
  // LSB0 (the round over local stages 0 .. R-1): rlow = 0, so twiddle k of
  // stage Q is omega_2048^(k 2^(10-Q)) and k = 0 is 1 -- those butterflies
  // skip their multiply (all of stage 0, half of stage 1, ...).
  FrU w[1 << Q];
#pragma unroll
  for (int k = 0; k < (1 << Q); k++)
    if (!(LSB0 && k == 0)) w[k] = ld_vec(&sm[(rlow + ((uint32_t)k << lsb)) << (NTT_SM_LOG - 1 - t)]);
#pragma unroll
  for (int i = 0; i < G / 2; i++) {
    const int m = ((i >> Q) << (Q + 1)) | (i & ((1 << Q) - 1));
    const int k = m & ((1 << Q) - 1);
    Fr u = x[m], v = x[m + (1 << Q)];
    if (LSB0 && k == 0) {
      x[m] = fr_add_lz(u, v);
      x[m + (1 << Q)] = fr_sub_lz(u, v);
    } else if (DIT) {
      v = fr_mul_wu(v, w[k]);
      x[m] = fr_add_lz(u, v);
      x[m + (1 << Q)] = fr_sub_lz(u, v);
    } else {
      x[m] = fr_add_lz(u, v);
      x[m + (1 << Q)] = fr_mul_wu(fr_sub_lz(u, v), w[k]);
    }
  }
}

template <int R, bool DIT, bool LSB0 = false>
__device__ __forceinline__ void ntt_round(Fr* sh, const FrU* __restrict__ sm, uint32_t ns, uint32_t logC,
                                          uint32_t lsb) {
  constexpr int G = 1 << R;
  const uint32_t C = 1u << logC;
  const uint32_t ngroups = (1u << (ns + logC)) >> R;
  for (uint32_t g = threadIdx.x; g < ngroups; g += NTT_THREADS) {
    const uint32_t c = g & (C - 1), rg = g >> logC;
    const uint32_t rlow = rg & ((1u << lsb) - 1);
    const uint32_t r0 = ((rg >> lsb) << (lsb + R)) | rlow;
    Fr x[G];
#pragma unroll
    for (int m = 0; m < G; m++) x[m] = ld_vec(&sh[((r0 + ((uint32_t)m << lsb)) << logC) | c]);
    if (DIT) {
      ntt_stage<R, 0, DIT, LSB0>(x, sm, rlow, lsb);
      if constexpr (R > 1) ntt_stage<R, (R > 1 ? 1 : 0), DIT, LSB0>(x, sm, rlow, lsb);
      if constexpr (R > 2) ntt_stage<R, (R > 2 ? 2 : 0), DIT, LSB0>(x, sm, rlow, lsb);
    } else {
      if constexpr (R > 2) ntt_stage<R, (R > 2 ? 2 : 0), DIT, LSB0>(x, sm, rlow, lsb);
      if constexpr (R > 1) ntt_stage<R, (R > 1 ? 1 : 0), DIT, LSB0>(x, sm, rlow, lsb);
      ntt_stage<R, 0, DIT, LSB0>(x, sm, rlow, lsb);
    }
#pragma unroll
    for (int m = 0; m < G; m++) st_vec(&sh[((r0 + ((uint32_t)m << lsb)) << logC) | c], x[m]);
  }
}

// The rounds of a tile's 2^ns-point sub-transform: DIF top-down (the last
// round, over local stages 0 .., is the LSB0 one), DIT bottom-up (LSB0 first).
template <bool DIT>
__device__ __forceinline__ void ntt_rounds(Fr* sh, const FrU* __restrict__ sm, uint32_t ns, uint32_t logC) {
  const uint32_t full = ns / NTT_R, rem = ns % NTT_R;
  if (DIT) {
    uint32_t lsb = 0;
    if (rem == 1) {
      ntt_round<1, true, true>(sh, sm, ns, logC, 0);
      lsb = 1;
      __syncthreads();
    } else if (rem == 2) {
      ntt_round<2, true, true>(sh, sm, ns, logC, 0);
      lsb = 2;
      __syncthreads();
    }
    for (uint32_t i = 0; i < full; i++, lsb += NTT_R) {
      if (lsb == 0) ntt_round<NTT_R, true, true>(sh, sm, ns, logC, 0);
      else ntt_round<NTT_R, true>(sh, sm, ns, logC, lsb);
      __syncthreads();
    }
  } else {
    uint32_t lsb = ns;
    for (uint32_t i = 0; i < full; i++) {
      lsb -= NTT_R;
      if (lsb == 0) ntt_round<NTT_R, false, true>(sh, sm, ns, logC, 0);
      else ntt_round<NTT_R, false>(sh, sm, ns, logC, lsb);
      __syncthreads();
    }
    if (rem == 2) ntt_round<2, false, true>(sh, sm, ns, logC, 0);
    if (rem == 1) ntt_round<1, false, true>(sh, sm, ns, logC, 0);
    __syncthreads();
  }
}

// Where a pass reads and writes.  Default: in place on `dst`.  IO_GATHER
// (first DIT pass only: s_lo = 0, one column per tile) reads element p of
// the pass from src[bitrev(p)] -- natural-order input of a DIT transform,
// so no separate permutation pass -- and orders its tiles so that the 4
// tiles whose gathers share 128-byte lines run back to back on one XCD.
// ltab: factor on load (indexed like the source); stab / scale: factor on
// store (indexed like the destination).
constexpr uint32_t IO_GATHER = 1, IO_SCALE = 2;
struct PassIO {
  const Fr* src;
  Fr* dst;
  const Fr* ltab;
  const Fr* stab;
  Fr scale;
  uint32_t flags;
  uint32_t* chk = nullptr;   // first pass of an API transform: *chk |= 1 on a non-canonical input
  uint64_t bstride = 0;      // batch: transform k of the launch works on src / dst + k bstride
};

// One pass = one four-step level.  The block of N = 2^(s_lo+ns) elements
// at hi is a 2^ns x 2^s_lo matrix (row r, column lo); the pass runs the
// 2^ns-point sub-transform down every column of its tile (C columns), whose
// twiddles are powers of omega_(2^ns) only, and the inter-level twiddle
// omega_N^(lo * bitrev(r)) is applied to the whole tile once: after the
// columns for DIF (natural -> bit-reversed), before them for DIT (the
// transpose).  With n = n1 n2, X[k1 + n1 k2] = sum_b w_n2^(b k2) w_n^(b k1)
// sum_a x[a n2 + b] w_n1^(a k1); sub-transforms in place leave element k at
// bitrev(k1) n2 + bitrev(k2) = bitrev_(log n)(k): exactly radix-2 DIF order.
template <bool DIT>
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_pass(PassIO io, NttTabs tabs, uint32_t log_n, uint32_t s_lo,
                                                          uint32_t ns, uint32_t logC) {
  extern __shared__ uint4 sh_raw[];
  Fr* sh = reinterpret_cast<Fr*>(sh_raw);
  const uint32_t C = 1u << logC;
  const uint32_t tile_elems = (1u << ns) << logC;
  const uint32_t lo_blocks = (1u << s_lo) >> logC;      // column blocks per hi
  // XCD-aware order: workgroups go round-robin to the 8 XCDs, so XCD x gets
  // the contiguous tile range [x G/8, (x+1) G/8) -- neighbouring column
  // blocks (which share 128-byte lines when tiles are 1-2 columns wide) meet
  // in one XCD's L2
  const uint32_t G = gridDim.x;
  const uint32_t ntiles = (uint32_t)((1ull << log_n) >> (ns + logC));   // per transform
  uint32_t tile = (G & 7) ? blockIdx.x : (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const uint32_t bi = tile / ntiles;   // transform of a batched launch
  tile -= bi * ntiles;
  const Fr* __restrict__ src = io.src + bi * io.bstride;
  Fr* __restrict__ dst = io.dst + bi * io.bstride;
  const bool gather = io.flags & IO_GATHER;
  if (gather && log_n > ns) tile = bitrev32(tile, log_n - ns);   // gathers of neighbouring tiles share lines
  const uint32_t hi = tile / lo_blocks;
  const uint32_t lo0 = (tile % lo_blocks) << logC;
  const size_t base = ((size_t)hi << (s_lo + ns)) + lo0;

  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) {
    const uint32_t r = k >> logC, c = k & (C - 1);
    const size_t gi = base + ((size_t)r << s_lo) + c;
    const size_t si = gather ? bitrev32((uint32_t)gi, log_n) : gi;
    Fr v = ld_vec(&src[si]);
    if (io.chk && !fr_lt_r(v)) atomicOr(io.chk, 1u);
    if (io.ltab) v = fp_mul(v, ld_vec(&io.ltab[si]));
    if (DIT && s_lo) v = fr_mul_lz(v, tw_pass<!ZK_NTT_LAZY>(tabs, (lo0 + c) * bitrev32(r, ns), s_lo + ns, log_n));
    st_vec(&sh[k], v);
  }
  __syncthreads();
  ntt_rounds<DIT>(sh, tabs.smu, ns, logC);
  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) {
    const uint32_t r = k >> logC, c = k & (C - 1);
    const size_t go = base + ((size_t)r << s_lo) + c;
    Fr v = ld_vec(&sh[k]);
    if (!DIT && s_lo) v = fp_mul(v, tw_pass<!ZK_NTT_LAZY>(tabs, (lo0 + c) * bitrev32(r, ns), s_lo + ns, log_n));
    if (io.stab) v = fp_mul(v, ld_vec(&io.stab[go]));
    else if (io.flags & IO_SCALE) v = fp_mul(v, io.scale);
    else if (DIT || !s_lo) v = fr_canon_lz(v);   // no canonical product above
    st_vec(&dst[go], v);
  }
}

static void run_pass_io(bool dit, const PassIO& io, const NttTabs& t, uint32_t log_n, uint32_t s_lo, uint32_t ns,
                        hipStream_t st, uint32_t nb = 1) {
  const uint32_t logC = std::min<uint32_t>(s_lo, NTT_TILE_LOG - ns);
  const uint32_t tiles = (uint32_t)((1ull << log_n) >> (ns + logC)) * nb;
  const size_t lds = sizeof(Fr) << (ns + logC);
  if (dit)
    k_ntt_pass<true><<<tiles, NTT_THREADS, lds, st>>>(io, t, log_n, s_lo, ns, logC);
  else
    k_ntt_pass<false><<<tiles, NTT_THREADS, lds, st>>>(io, t, log_n, s_lo, ns, logC);
  ZK_LAUNCH_CHECK();
}

static void run_pass(bool dit, Fr* d, const NttTabs& t, uint32_t log_n, uint32_t s_lo, uint32_t ns,
                     hipStream_t st, const Fr* src = nullptr, const Fr* ltab = nullptr, uint32_t nb = 1) {
  PassIO io{src ? src : d, d, ltab, nullptr, Fr{}, 0u};
  io.bstride = (uint64_t)1 << log_n;
  run_pass_io(dit, io, t, log_n, s_lo, ns, st, nb);
}

// Pass plan, top (first DIF pass) to bottom: the contiguous pass (s_lo = 0)
// takes up to NTT_TILE_LOG stages; the rest are split evenly into strided
// passes of <= NTT_TILE_LOG stages (round 2, 2048-element tiles: at 2^22 two
// passes instead of three, 0.580 vs 0.609 ms with
// depth 9, profiles/r02_ntt_sweep.txt; a one-column tile's 32-byte rows share
// lines with its neighbours, which the XCD-aware tile order keeps in one L2).
static uint32_t max_strided() { return NTT_TILE_LOG; }
static std::vector<uint32_t> pass_plan(uint32_t L) {
  const uint32_t last = std::min<uint32_t>(L, NTT_TILE_LOG);
  const uint32_t rest = L - last;
  std::vector<uint32_t> ns;
  if (rest) {
    const uint32_t ms = max_strided();
    const uint32_t np = (rest + ms - 1) / ms;
    for (uint32_t i = 0; i < np; i++) ns.push_back(rest / np + (i < rest % np ? 1 : 0));
  }
  ns.push_back(last);
  return ns;
}


void ntt_dif(Fr* d, const NttDomain& dom, bool inv, hipStream_t st, Prof* pf, const Fr* src, const Fr* ltab,
             uint32_t nb) {
  const uint32_t L = dom.log_n;
  if (L == 0) return;
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)nb << L) : -1;
  const NttTabs t = tabs_of(dom, inv);
  uint32_t s_hi = L;
  bool first = true;
  for (uint32_t ns : pass_plan(L)) {
    run_pass(false, d, t, L, s_hi - ns, ns, st, first ? src : nullptr, first ? ltab : nullptr, nb);
    first = false;
    s_hi -= ns;
  }
  if (pf) pf->end(st, ph);
}

void ntt_dit(Fr* d, const NttDomain& dom, bool inv, hipStream_t st, Prof* pf, uint32_t nb) {
  const uint32_t L = dom.log_n;
  if (L == 0) return;
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)nb << L) : -1;
  const NttTabs t = tabs_of(dom, inv);
  const std::vector<uint32_t> plan = pass_plan(L);
  uint32_t s_lo = 0;
  for (auto it = plan.rbegin(); it != plan.rend(); ++it) {
    run_pass(true, d, t, L, s_lo, *it, st, nullptr, nullptr, nb);
    s_lo += *it;
  }
  if (pf) pf->end(st, ph);
}

// Natural order in and out (the reference's fft / ifft): DIT passes, the
// first gathering its tiles from the bit-reversed positions of src (times
// ltab[i] when given), the last writing dst (times stab[i] or *scale).  No
// standalone permutation pass: at 2^22, 2 HBM round trips instead of 3
// passes plus a bit reversal.  With more than one pass the intermediate
// levels live in tmp (n elements), so src may equal dst.
void ntt_natural(Fr* dst, const Fr* src, Fr* tmp, const NttDomain& dom, bool inv, hipStream_t st, Prof* pf,
                 const Fr* ltab, const Fr* stab, const Fr* scale, uint32_t* chk) {
  const uint32_t L = dom.log_n;
  if (L == 0) return;
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)1 << L) : -1;
  const NttTabs t = tabs_of(dom, inv);
  const std::vector<uint32_t> plan = pass_plan(L);
  const size_t P = plan.size();
  uint32_t s_lo = 0;
  for (size_t i = 0; i < P; i++) {
    const uint32_t ns = plan[P - 1 - i];
    PassIO io{i == 0 ? src : tmp, i + 1 == P ? dst : tmp, nullptr, nullptr, Fr{}, 0u};
    if (i == 0) {
      io.flags |= IO_GATHER;
      io.ltab = ltab;
      io.chk = chk;
    }
    if (i + 1 == P) {
      io.stab = stab;
      if (scale) {
        io.scale = *scale;
        io.flags |= IO_SCALE;
      }
    }
    run_pass_io(true, io, t, L, s_lo, ns, st);
    s_lo += ns;
  }
  if (pf) pf->end(st, ph);
}

// iNTT -> coset shift -> NTT (the quotient's per-polynomial round trip):
// the last DIF pass and the first DIT pass both work on the same contiguous
// 2^ns-element tiles, so ONE kernel runs the DIF stages with the inverse
// twiddles, multiplies each element p by tab_br[p] = n^-1 g^bitrev(p) (a
// contiguous read: gathering tab[bitrev(p)] from an n-entry table touched a
// new 128-B line and, beyond the MALL, a new page per element) and runs
// the DIT stages with the forward twiddles while the tile stays in LDS: two
// HBM round trips and the separate scale pass disappear.
// Batched: the launch covers nb transforms of 2^log_n elements back to back
// in data (block b works on tile b mod tiles of transform b / tiles).
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_tile_shift(Fr* __restrict__ data, const FrU* __restrict__ ism,
                                                               const FrU* __restrict__ sm,
                                                               const Fr* __restrict__ tab_br, uint32_t ns,
                                                               uint32_t log_n) {
  extern __shared__ uint4 sh_raw[];
  Fr* sh = reinterpret_cast<Fr*>(sh_raw);
  const uint32_t tile_elems = 1u << ns;
  const size_t base = (size_t)blockIdx.x << ns;
  const size_t tbase = base & (((size_t)1 << log_n) - 1);   // position within its transform
  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) st_vec(&sh[k], ld_vec(&data[base + k]));
  __syncthreads();
  ntt_rounds<false>(sh, ism, ns, 0);
  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) {
    st_vec(&sh[k], fp_mul(ld_vec(&sh[k]), ld_vec(&tab_br[tbase + k])));
  }
  __syncthreads();
  ntt_rounds<true>(sh, sm, ns, 0);
  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS)
    st_vec(&data[base + k], fr_canon_lz(ld_vec(&sh[k])));
}

void ntt_coset_shift(Fr* d, const NttDomain& dom, const Fr* tab_br, hipStream_t st, Prof* pf, uint32_t nb) {
  const uint32_t L = dom.log_n;
  if (L == 0) {
    fr_scale_table(d, tab_br, 0, false, st, nb);
    return;
  }
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)(2 * nb) << L) : -1;
  const NttTabs ti = tabs_of(dom, true), tf = tabs_of(dom, false);
  const std::vector<uint32_t> plan = pass_plan(L);
  // inverse transform: every DIF pass but the last (contiguous) one
  uint32_t s_hi = L;
  for (size_t i = 0; i + 1 < plan.size(); i++) {
    run_pass(false, d, ti, L, s_hi - plan[i], plan[i], st, nullptr, nullptr, nb);
    s_hi -= plan[i];
  }
  const uint32_t ns = plan.back();   // s_hi == ns here: the contiguous pass
  k_ntt_tile_shift<<<(uint32_t)(((uint64_t)nb << L) >> ns), NTT_THREADS, sizeof(Fr) << ns, st>>>(d, ti.smu, tf.smu,
                                                                                                tab_br, ns, L);
  ZK_LAUNCH_CHECK();
  // forward transform: every DIT pass but the first (contiguous) one
  uint32_t s_lo = ns;
  for (size_t i = plan.size() - 1; i-- > 0;) {
    run_pass(true, d, tf, L, s_lo, plan[i], st, nullptr, nullptr, nb);
    s_lo += plan[i];
  }
  if (pf) pf->end(st, ph);
}

// ------------------------------------------------------------ tables -----
__device__ __forceinline__ Fr fr_pow_u64(Fr b, uint64_t e) {
  Fr acc = fp_one<FrParams>();
  while (e) {
    if (e & 1) acc = fp_mul(acc, b);
    b = fp_mul(b, b);
    e >>= 1;
  }
  return acc;
}

constexpr int POW_CHUNK = 64;
__global__ void __launch_bounds__(256) k_powers(Fr* __restrict__ out, Fr base, Fr scale, size_t n) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i0 = t * POW_CHUNK;
  if (i0 >= n) return;
  Fr x = fp_mul(scale, fr_pow_u64(base, i0));
  const size_t e = min(i0 + POW_CHUNK, n);
  for (size_t i = i0; i < e; i++) {
    st_vec(&out[i], x);
    x = fp_mul(x, base);
  }
}

void fr_powers(Fr* d_out, const Fr& base, const Fr& scale, size_t n, hipStream_t st) {
  if (!n) return;
  const size_t thr = (n + POW_CHUNK - 1) / POW_CHUNK;
  k_powers<<<ceil_div(thr, 256), 256, 0, st>>>(d_out, base, scale, n);
  ZK_LAUNCH_CHECK();
}

static Fr fr_const(const uint32_t (&c)[8]) {
  Fr r;
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
  return r;
}

// Z(g w^i) = g^n - 1 on the whole coset; Fermat inverse, one thread, once per domain.
__global__ void k_coset_zinv(Fr* out, uint32_t log_n) {
  Fr g;
#pragma unroll
  for (int i = 0; i < 8; i++) g.v[i] = FR_GEN[i];
  for (uint32_t k = 0; k < log_n; k++) g = fp_mul(g, g);
  g = fp_sub(g, fp_one<FrParams>());
  uint32_t e[8];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = __builtin_subc(FrParams::MOD[i], i == 0 ? 2u : 0u, br, &br);
  Fr acc = fp_one<FrParams>();
#pragma unroll
  for (int i = 7; i >= 0; i--)
    for (int k = 31; k >= 0; k--) {
      acc = fp_mul(acc, acc);
      if ((e[i] >> k) & 1) acc = fp_mul(acc, g);
    }
  *out = acc;
}

__global__ void __launch_bounds__(256) k_cut_limbs(const Fr* __restrict__ in, FrU* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  FrU u;
  unpack28<8, FrParams::NL, FrParams::LB>(ld_vec(&in[i]).v, u.l);
#pragma unroll
  for (int k = 0; k < 12 - FrParams::NL; k++) u.pad[k] = 0;
  st_vec(&out[i], u);
}

void ntt_domain_init(NttDomain& d, uint32_t log_n, hipStream_t st) {
  d.log_n = log_n;
  const size_t n = (size_t)1 << log_n;
  const size_t nsm = (size_t)1 << (NTT_SM_LOG - 1);
  const size_t ntl = std::min<size_t>(n, (size_t)1 << NTT_TL_LOG);
  const size_t nth = std::max<size_t>(n >> NTT_TL_LOG, 1);
  d.sm.ensure(sizeof(Fr) * nsm);
  d.ism.ensure(sizeof(Fr) * nsm);
  d.tl.ensure(sizeof(Fr) * ntl);
  d.itl.ensure(sizeof(Fr) * ntl);
  d.th.ensure(sizeof(Fr) * nth);
  d.ith.ensure(sizeof(Fr) * nth);
  Fr one = fr_const(FrParams::ONE);
  fr_powers(d.sm.as<Fr>(), fr_const(FR_ROOTS[NTT_SM_LOG]), one, nsm, st);
  fr_powers(d.ism.as<Fr>(), fr_const(FR_ROOTS_INV[NTT_SM_LOG]), one, nsm, st);
  fr_powers(d.tl.as<Fr>(), fr_const(FR_ROOTS[log_n]), one, ntl, st);
  fr_powers(d.itl.as<Fr>(), fr_const(FR_ROOTS_INV[log_n]), one, ntl, st);
  if (log_n > NTT_TL_LOG) {   // omega_n^4096 = omega_(n / 4096)
    fr_powers(d.th.as<Fr>(), fr_const(FR_ROOTS[log_n - NTT_TL_LOG]), one, nth, st);
    fr_powers(d.ith.as<Fr>(), fr_const(FR_ROOTS_INV[log_n - NTT_TL_LOG]), one, nth, st);
  }
  if (log_n > NTT_TL_LOG && NTT_TS_LOG > NTT_TL_LOG) {
    // direct twiddles for the passes over blocks of <= 2^16 (round 3): one
    // L2-resident load instead of TL x TH, a load and a product less per
    // element (2^22 API NTT: the first strided pass)
    d.ts_log = std::min<uint32_t>(log_n, NTT_TS_LOG);
    const size_t nts = (size_t)1 << d.ts_log;
    d.ts.ensure(sizeof(Fr) * nts);
    d.its.ensure(sizeof(Fr) * nts);
    fr_powers(d.ts.as<Fr>(), fr_const(FR_ROOTS[d.ts_log]), one, nts, st);
    fr_powers(d.its.as<Fr>(), fr_const(FR_ROOTS_INV[d.ts_log]), one, nts, st);
  }
  d.smu.ensure(sizeof(FrU) * nsm);
  d.ismu.ensure(sizeof(FrU) * nsm);
  k_cut_limbs<<<ceil_div(nsm, 256), 256, 0, st>>>(d.sm.as<Fr>(), d.smu.as<FrU>(), nsm);
  ZK_LAUNCH_CHECK();
  k_cut_limbs<<<ceil_div(nsm, 256), 256, 0, st>>>(d.ism.as<Fr>(), d.ismu.as<FrU>(), nsm);
  ZK_LAUNCH_CHECK();
  d.zinv.ensure(sizeof(Fr));
  k_coset_zinv<<<1, 1, 0, st>>>(d.zinv.as<Fr>(), log_n);
  ZK_LAUNCH_CHECK();
}

const Fr* domain_gpow(NttDomain& d, hipStream_t st) {
  if (!d.gpow.p) {
    const size_t n = (size_t)1 << d.log_n;
    d.gpow.ensure(sizeof(Fr) * n);
    fr_powers(d.gpow.as<Fr>(), fr_const(FR_GEN), fr_const(FR_INV_2K[d.log_n]), n, st);
  }
  return d.gpow.as<Fr>();
}

const Fr* domain_gipow(NttDomain& d, hipStream_t st) {
  if (!d.gipow.p) {
    const size_t n = (size_t)1 << d.log_n;
    d.gipow.ensure(sizeof(Fr) * n);
    fr_powers(d.gipow.as<Fr>(), fr_const(FR_GEN_INV), fr_const(FR_INV_2K[d.log_n]), n, st);
  }
  return d.gipow.as<Fr>();
}

const Fr* domain_gpow_br(NttDomain& d, hipStream_t st) {
  if (!d.gpow_br.p) {
    const size_t n = (size_t)1 << d.log_n;
    d.gpow_br.ensure(sizeof(Fr) * n);
    if (d.gpow.p) {
      fr_bitrev_scale(d.gpow.as<Fr>(), d.gpow_br.as<Fr>(), d.log_n, nullptr, nullptr, st);
    } else {   // natural-order table only as scratch
      DevBuf tmp;
      tmp.ensure(sizeof(Fr) * n);
      fr_powers(tmp.as<Fr>(), fr_const(FR_GEN), fr_const(FR_INV_2K[d.log_n]), n, st);
      fr_bitrev_scale(tmp.as<Fr>(), d.gpow_br.as<Fr>(), d.log_n, nullptr, nullptr, st);
      ZK_HIP(hipStreamSynchronize(st));   // tmp dies here
    }
  }
  return d.gpow_br.as<Fr>();
}

// -------------------------------------------------------- elementwise ---
__global__ void __launch_bounds__(256) k_to_mont(const uint64_t* __restrict__ in, Fr* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr a = ld_vec(reinterpret_cast<const Fr*>(in) + i);
  st_vec(&out[i], fp_to_mont(a));
}
__global__ void __launch_bounds__(256) k_from_mont(const Fr* __restrict__ in, uint64_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_vec(reinterpret_cast<Fr*>(out) + i, fp_from_mont(ld_vec(&in[i])));
}
__global__ void __launch_bounds__(256) k_scale_table(Fr* __restrict__ d, const Fr* __restrict__ tab,
                                                     uint32_t log_n, bool bitrev, uint32_t nb) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((q >> log_n) >= nb) return;
  const size_t p = q & (((size_t)1 << log_n) - 1);   // batched: the same table for every transform
  const size_t j = bitrev ? bitrev32((uint32_t)p, log_n) : p;
  st_vec(&d[q], fp_mul(ld_vec(&d[q]), ld_vec(&tab[j])));
}
__global__ void __launch_bounds__(256) k_bitrev_copy(const Fr* __restrict__ in, Fr* __restrict__ out, uint32_t log_n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >> log_n) return;
  st_vec(&out[i], ld_vec(&in[bitrev32((uint32_t)i, log_n)]));
}
__global__ void __launch_bounds__(256) k_scale_const(Fr* __restrict__ d, Fr c, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_vec(&d[i], fp_mul(ld_vec(&d[i]), c));
}

// Bit-reversal permutation through 32 x 32 LDS tiles: with i = x 2^(L-5) +
// mid 2^5 + y, bitrev(i) = rev5(y) 2^(L-5) + rev(mid) 2^5 + rev5(x), so for a
// fixed mid the 32 x 32 block (x, y) lands transposed at (rev5(y), rev5(x)):
// both the 32-element rows read and the 32-element rows written are
// contiguous (1 KiB).  Optional factor per output element.
constexpr int BR_T = 5;
__device__ __forceinline__ uint32_t rev5(uint32_t v) { return __builtin_bitreverse32(v) >> 27; }
__global__ void __launch_bounds__(256) k_bitrev_tiled(const Fr* __restrict__ in, Fr* __restrict__ out, uint32_t L,
                                                      const Fr* __restrict__ tab, Fr c, int mode) {
  __shared__ Fr t[32 * 33];
  const uint32_t mid = blockIdx.x, midbits = L - 2 * BR_T;
  const uint32_t rmid = midbits ? (__builtin_bitreverse32(mid) >> (32 - midbits)) : 0;
  for (uint32_t k = threadIdx.x; k < 1024; k += 256) {
    const uint32_t x = k >> 5, y = k & 31;
    const size_t i = ((size_t)x << (L - BR_T)) | ((size_t)mid << BR_T) | y;
    t[x * 33 + y] = ld_vec(&in[i]);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < 1024; k += 256) {
    const uint32_t yr = k >> 5, xr = k & 31;
    const size_t j = ((size_t)yr << (L - BR_T)) | ((size_t)rmid << BR_T) | xr;
    Fr v = t[rev5(xr) * 33 + rev5(yr)];
    if (mode == 1) v = fp_mul(v, ld_vec(&tab[j]));
    else if (mode == 2) v = fp_mul(v, c);
    st_vec(&out[j], v);
  }
}
__global__ void __launch_bounds__(256) k_bitrev_small(const Fr* __restrict__ in, Fr* __restrict__ out, uint32_t L,
                                                      const Fr* __restrict__ tab, Fr c, int mode) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >> L) return;
  const uint32_t j = bitrev32(i, L);
  Fr v = ld_vec(&in[i]);
  if (mode == 1) v = fp_mul(v, ld_vec(&tab[j]));
  else if (mode == 2) v = fp_mul(v, c);
  st_vec(&out[j], v);
}
void fr_bitrev_scale(const Fr* in, Fr* out, uint32_t log_n, const Fr* tab, const Fr* c, hipStream_t st) {
  const int mode = tab ? 1 : c ? 2 : 0;
  const Fr cv = c ? *c : Fr{};
  if (log_n >= 2 * BR_T)
    k_bitrev_tiled<<<1u << (log_n - 2 * BR_T), 256, 0, st>>>(in, out, log_n, tab, cv, mode);
  else
    k_bitrev_small<<<ceil_div((size_t)1 << log_n, 256), 256, 0, st>>>(in, out, log_n, tab, cv, mode);
  ZK_LAUNCH_CHECK();
}

void fr_to_mont(const uint64_t* d_canon, Fr* d_out, size_t n, hipStream_t st) {
  if (!n) return;
  k_to_mont<<<ceil_div(n, 256), 256, 0, st>>>(d_canon, d_out, n);
  ZK_LAUNCH_CHECK();
}
void fr_from_mont(const Fr* d_in, uint64_t* d_canon, size_t n, hipStream_t st) {
  if (!n) return;
  k_from_mont<<<ceil_div(n, 256), 256, 0, st>>>(d_in, d_canon, n);
  ZK_LAUNCH_CHECK();
}
void fr_scale_table(Fr* d, const Fr* tab, uint32_t log_n, bool bitrev, hipStream_t st, uint32_t nb) {
  k_scale_table<<<ceil_div((size_t)nb << log_n, 256), 256, 0, st>>>(d, tab, log_n, bitrev, nb);
  ZK_LAUNCH_CHECK();
}
void fr_bitrev_copy(const Fr* in, Fr* out, uint32_t log_n, hipStream_t st) {
  k_bitrev_copy<<<ceil_div((size_t)1 << log_n, 256), 256, 0, st>>>(in, out, log_n);
  ZK_LAUNCH_CHECK();
}
void fr_scale_const(Fr* d, const Fr& c, size_t n, hipStream_t st) {
  if (!n) return;
  k_scale_const<<<ceil_div(n, 256), 256, 0, st>>>(d, c, n);
  ZK_LAUNCH_CHECK();
}

}  // namespace zk
