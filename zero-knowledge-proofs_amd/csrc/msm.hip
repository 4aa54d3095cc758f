// msm.hip -- Pippenger bucket MSM kernels for gfx950 (see msm.hpp for the
// pipeline).  Wave64 throughout; no MFMA (big-integer modular arithmetic).
#include <algorithm>
#include <cstring>
#include <vector>

#include "msm.hpp"

namespace zk {

// ---------------------------------------------------------------- plan ---
MsmPlan msm_make_plan(uint32_t n, int bits, int sw, int force_c) {
  MsmPlan p{};
  p.n = n;
  p.bits = bits;
  p.sw = sw;
  int best_c = 4;
  double best = 1e300;
  for (int c = 4; c <= 16; c++) {
    int nwin = (bits + c - 1) / c;
    if (nwin > MSM_MAXWIN) continue;
    int top = bits - c * (nwin - 1);
    double nbuck = (double)(nwin - 1) * (1u << (c - 1)) + (double)(1u << top);
    // accumulate: one mixed add per (point, window); reduce: ~3 full adds per bucket
    double cost = (double)n * nwin + 4.0 * nbuck;
    if (cost < best) { best = cost; best_c = c; }
  }
  if (force_c) best_c = force_c;
  p.c = best_c;
  p.nwin = (bits + p.c - 1) / p.c;
  p.L = 8;
  p.K = 16;
  uint32_t G = 0, T = 0;
  int maxT = 1;
  for (int w = 0; w < p.nwin; w++) {
    int width = (w == p.nwin - 1) ? bits - p.c * w : p.c;
    p.nb[w] = (w == p.nwin - 1) ? (1u << width) : (1u << (p.c - 1));
    p.boff[w] = G;
    p.segoff[w] = T;
    G += p.nb[w];
    uint32_t t = ceil_div(p.nb[w], p.L);
    T += t;
    maxT = std::max<int>(maxT, (int)t);
  }
  p.boff[p.nwin] = G;
  p.segoff[p.nwin] = T;
  p.G = G;
  p.T = T;
  int qb = 0;
  while ((1 << qb) < maxT) qb++;
  p.Q = 1 + qb;
  return p;
}

// ------------------------------------------------------------- digits ---
template <int SW>
__device__ __forceinline__ uint32_t scal_window(const uint64_t (&s)[SW], int off, int width) {
  int wd = off >> 6, sh = off & 63;
  uint64_t lo = 0;
#pragma unroll
  for (int k = 0; k < SW; k++)
    if (k == wd) lo = s[k] >> sh;
  if (sh + width > 64) {
#pragma unroll
    for (int k = 0; k < SW; k++)
      if (k == wd + 1) lo |= s[k] << (64 - sh);
  }
  return (uint32_t)(lo & ((1ull << width) - 1));
}

// Signed recoding: windows 0..nwin-2 give digits in [-(2^(c-1)-1), 2^(c-1)]
// with a carry into the next window; the top window absorbs the final carry
// unsigned (digit in [0, 2^top]), so no extra carry window is needed.
template <int SW, bool SCATTER>
__global__ void __launch_bounds__(256) k_msm_digits(const uint64_t* __restrict__ sc, MsmPlan p,
                                                    uint32_t* __restrict__ counts,
                                                    uint32_t* __restrict__ cursor,
                                                    uint32_t* __restrict__ ent,
                                                    uint32_t* __restrict__ key) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  uint64_t s[SW];
#pragma unroll
  for (int k = 0; k < SW; k++) s[k] = sc[(size_t)i * SW + k];
  uint32_t carry = 0;
  const uint32_t half = 1u << (p.c - 1);
  for (int w = 0; w < p.nwin; w++) {
    const bool top = (w == p.nwin - 1);
    const int width = top ? p.bits - p.c * w : p.c;
    uint32_t v = scal_window<SW>(s, p.c * w, width) + carry;
    uint32_t mag;
    bool neg = false;
    if (!top && v > half) {
      mag = (1u << p.c) - v;  // digit = v - 2^c < 0
      neg = true;
      carry = 1;
    } else {
      mag = v;
      carry = 0;
    }
    if (mag) {
      uint32_t g = p.boff[w] + mag - 1;
      if (!SCATTER) {
        atomicAdd(&counts[g], 1u);
      } else {
        uint32_t pos = atomicAdd(&cursor[g], 1u);
        ent[pos] = i | (neg ? 0x80000000u : 0u);
        key[pos] = g;
      }
    }
  }
}

// Exclusive scan of G counts by one 1024-thread workgroup.
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t* __restrict__ counts, uint32_t G,
                                                   uint32_t* __restrict__ off, uint32_t* __restrict__ cur) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (G + 1023) / 1024;
  const uint32_t b = min(t * per, G), e = min(b + per, G);
  uint32_t s = 0;
  for (uint32_t i = b; i < e; i++) s += counts[i];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    uint32_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t base = t ? part[t - 1] : 0;
  for (uint32_t i = b; i < e; i++) {
    off[i] = base;
    cur[i] = base;
    base += counts[i];
  }
  if (t == 1023) off[G] = part[1023];
}

// --------------------------------------------------------- accumulate ---
template <class C>
__device__ __forceinline__ typename C::A load_point(const typename C::A* __restrict__ bases, uint32_t e) {
  typename C::A a = ld_vec(&bases[e & 0x7fffffffu]);
  if (e & 0x80000000u) a.y = f_neg(a.y);
  return a;
}

// Thread t owns sorted entries [tK, tK+K).  One mixed add per entry (uniform
// across the wave); at a bucket change the finished run is flushed:
//   complete bucket        -> buckets[g]
//   run begun by an earlier thread (head) -> partials[2t]
//   run continued by a later thread (tail) -> partials[2t+1]
template <class C>
__global__ void __launch_bounds__(128) k_msm_accum(const typename C::A* __restrict__ bases,
                                                   const uint32_t* __restrict__ ent,
                                                   const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ off, uint32_t G, int K,
                                                   typename C::X* __restrict__ buckets,
                                                   typename C::X* __restrict__ partials) {
  using X = typename C::X;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t M = off[G];  // non-zero digits (known on device only)
  const uint32_t start = t * (uint32_t)K;
  if (start >= M) return;
  const uint32_t end = min(start + (uint32_t)K, M);
  X acc;
  xyzz_set_inf(acc);
  uint32_t cur = key[start], run_start = start;
  for (uint32_t e = start; e < end; e++) {
    const uint32_t g = key[e];
    if (g != cur) {
      const bool head = (run_start == start) && (off[cur] < start);
      if (head) st_vec(&partials[2 * (size_t)t], acc);
      else st_vec(&buckets[cur], acc);
      xyzz_set_inf(acc);
      cur = g;
      run_start = e;
    }
    typename C::A a = load_point<C>(bases, ent[e]);
    if (!aff_is_inf(a)) acc = xyzz_madd(acc, a);
  }
  const bool head = (run_start == start) && (off[cur] < start);
  const bool tail = off[cur + 1] > end;
  if (head) st_vec(&partials[2 * (size_t)t], acc);
  else if (tail) st_vec(&partials[2 * (size_t)t + 1], acc);
  else st_vec(&buckets[cur], acc);
}

// Buckets whose entries span several threads: tail(t0) + head(t0+1..t1).
template <class C>
__global__ void __launch_bounds__(128) k_msm_fixup(const uint32_t* __restrict__ off, uint32_t G, int K,
                                                   typename C::X* __restrict__ buckets,
                                                   const typename C::X* __restrict__ partials) {
  using X = typename C::X;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const uint32_t bs = off[g], be = off[g + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  X acc = ld_vec(&partials[2 * (size_t)t0 + 1]);
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = xyzz_add(acc, ld_vec(&partials[2 * (size_t)t]));
  st_vec(&buckets[g], acc);
}

// Per (window, segment of L buckets): running sum from the top bucket down.
//   S_j = sum of the segment's buckets, W_j = sum_m (m+1) B_{jL+m}.
template <class C>
__global__ void __launch_bounds__(128) k_msm_reduce1(MsmPlan p, const uint32_t* __restrict__ off,
                                                     const typename C::X* __restrict__ buckets,
                                                     typename C::X* __restrict__ segS,
                                                     typename C::X* __restrict__ segW) {
  using X = typename C::X;
  const uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x;
  if (sid >= p.T) return;
  int w = 0;
  while (sid >= p.segoff[w + 1]) w++;
  const uint32_t j = sid - p.segoff[w];
  const uint32_t lo = p.boff[w] + j * p.L;
  const uint32_t hi = min(lo + (uint32_t)p.L, p.boff[w] + p.nb[w]);
  X run, sum;
  xyzz_set_inf(run);
  xyzz_set_inf(sum);
  for (uint32_t g = hi; g-- > lo;) {
    if (off[g + 1] != off[g]) run = xyzz_add(run, ld_vec(&buckets[g]));
    sum = xyzz_add(sum, run);
  }
  st_vec(&segS[sid], run);
  st_vec(&segW[sid], sum);
}

// One workgroup per (window, quantity q): q = 0 -> sum_j W_j;
// q = 1 + b -> U_b = sum over segments j with bit b set of S_j.
template <class C, int NT>
__global__ void __launch_bounds__(NT) k_msm_reduce2(MsmPlan p, const typename C::X* __restrict__ segS,
                                                    const typename C::X* __restrict__ segW,
                                                    typename C::X* __restrict__ res) {
  using X = typename C::X;
  __shared__ X sh[NT];
  const int w = blockIdx.x / p.Q, q = blockIdx.x % p.Q;
  const uint32_t T = p.segoff[w + 1] - p.segoff[w];
  const X* src = (q == 0 ? segW : segS) + p.segoff[w];
  X acc;
  xyzz_set_inf(acc);
  for (uint32_t j = threadIdx.x; j < T; j += NT)
    if (q == 0 || ((j >> (q - 1)) & 1)) acc = xyzz_add(acc, ld_vec(&src[j]));
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int d = NT / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) sh[threadIdx.x] = xyzz_add(sh[threadIdx.x], sh[threadIdx.x + d]);
    __syncthreads();
  }
  if (threadIdx.x == 0) st_vec(&res[blockIdx.x], sh[0]);
}

// ------------------------------------------------------------ driver -----
template <class C>
void msm_launch(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw, uint32_t n,
                int bits, hipStream_t st) {
  using X = typename C::X;
  MsmPlan& p = w.plan;
  p = msm_make_plan(n, bits, sw);
  const size_t M = (size_t)n * p.nwin;
  w.counts.ensure(sizeof(uint32_t) * (p.G + 1));
  w.off.ensure(sizeof(uint32_t) * (p.G + 1));
  w.cursor.ensure(sizeof(uint32_t) * (p.G + 1));
  w.ent.ensure(sizeof(uint32_t) * std::max<size_t>(M, 1));
  w.key.ensure(sizeof(uint32_t) * std::max<size_t>(M, 1));
  w.buckets.ensure(sizeof(X) * p.G);
  const size_t nthr_max = (M + p.K - 1) / p.K + 1;
  w.partials.ensure(sizeof(X) * 2 * nthr_max);
  w.segS.ensure(sizeof(X) * p.T);
  w.segW.ensure(sizeof(X) * p.T);
  w.res.ensure(sizeof(X) * p.nwin * p.Q);

  ZK_HIP(hipMemsetAsync(w.counts.p, 0, sizeof(uint32_t) * (p.G + 1), st));
  if (n) {
    const uint32_t nb = ceil_div(n, 256);
    if (sw == 1)
      k_msm_digits<1, false><<<nb, 256, 0, st>>>(d_scalars, p, w.counts.as<uint32_t>(), nullptr, nullptr, nullptr);
    else
      k_msm_digits<4, false><<<nb, 256, 0, st>>>(d_scalars, p, w.counts.as<uint32_t>(), nullptr, nullptr, nullptr);
    ZK_LAUNCH_CHECK();
  }
  k_msm_scan<<<1, 1024, 0, st>>>(w.counts.as<uint32_t>(), p.G, w.off.as<uint32_t>(), w.cursor.as<uint32_t>());
  ZK_LAUNCH_CHECK();
  if (n) {
    const uint32_t nb = ceil_div(n, 256);
    if (sw == 1)
      k_msm_digits<1, true><<<nb, 256, 0, st>>>(d_scalars, p, nullptr, w.cursor.as<uint32_t>(),
                                                w.ent.as<uint32_t>(), w.key.as<uint32_t>());
    else
      k_msm_digits<4, true><<<nb, 256, 0, st>>>(d_scalars, p, nullptr, w.cursor.as<uint32_t>(),
                                                w.ent.as<uint32_t>(), w.key.as<uint32_t>());
    ZK_LAUNCH_CHECK();
  }
  // The number of non-zero digits M' <= M is only known on device: launch for
  // M threads' worth of chunks; chunks beyond off[G] exit immediately.  To
  // avoid a host sync we bound M' by M.
  const uint32_t Mtot = (uint32_t)M;
  if (Mtot) {
    const uint32_t nthr = ceil_div(Mtot, p.K);
    k_msm_accum<C><<<ceil_div(nthr, 128), 128, 0, st>>>(d_bases, w.ent.as<uint32_t>(), w.key.as<uint32_t>(),
                                                           w.off.as<uint32_t>(), p.G, p.K, w.buckets.as<X>(),
                                                           w.partials.as<X>());
    ZK_LAUNCH_CHECK();
  }
  k_msm_fixup<C><<<ceil_div(p.G, 128), 128, 0, st>>>(w.off.as<uint32_t>(), p.G, p.K, w.buckets.as<X>(),
                                                      w.partials.as<X>());
  ZK_LAUNCH_CHECK();
  k_msm_reduce1<C><<<ceil_div(p.T, 128), 128, 0, st>>>(p, w.off.as<uint32_t>(), w.buckets.as<X>(),
                                                        w.segS.as<X>(), w.segW.as<X>());
  ZK_LAUNCH_CHECK();
  k_msm_reduce2<C, 128><<<p.nwin * p.Q, 128, 0, st>>>(p, w.segS.as<X>(), w.segW.as<X>(), w.res.as<X>());
  ZK_LAUNCH_CHECK();
}


template <class C>
void msm_download(MsmWork& w, hipStream_t st) {
  using X = typename C::X;
  const size_t bytes = sizeof(X) * w.plan.nwin * w.plan.Q;
  w.host_res.resize(bytes);
  ZK_HIP(hipMemcpyAsync(w.host_res.data(), w.res.p, bytes, hipMemcpyDeviceToHost, st));
}

// Device XYZZ (32-bit limbs) and host XYZZ (64-bit limbs) share their bytes.
template <class C>
host::X<typename C::HF> msm_finish(const MsmWork& w) {
  using HF = typename C::HF;
  using HX = host::X<HF>;
  static_assert(sizeof(HX) == sizeof(typename C::X), "layout");
  const MsmPlan& p = w.plan;
  const HX* r = reinterpret_cast<const HX*>(w.host_res.data());
  // Every partial is a point times a power of two:
  //   window w, q = 0     : 2^(c w)              * W-sum
  //   window w, q = 1 + b : 2^(c w + log2 L + b) * U_b
  // One Horner pass over exponents from the top.
  int lgL = 0;
  while ((1 << lgL) < p.L) lgL++;
  int maxe = 0;
  for (int w = 0; w < p.nwin; w++) maxe = std::max(maxe, p.c * w + lgL + p.Q - 2);
  std::vector<std::vector<const HX*>> at(maxe + 1);
  for (int w = 0; w < p.nwin; w++)
    for (int q = 0; q < p.Q; q++) {
      int e = q == 0 ? p.c * w : p.c * w + lgL + (q - 1);
      at[e].push_back(&r[w * p.Q + q]);
    }
  HX acc = host::inf<HF>();
  for (int e = maxe; e >= 0; e--) {
    acc = host::dbl(acc);
    for (const HX* t : at[e]) acc = host::addp(acc, *t);
  }
  return acc;
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
  template void msm_launch<C>(MsmWork&, const C::A*, const uint64_t*, int, uint32_t, int, hipStream_t); \
  template void msm_download<C>(MsmWork&, hipStream_t);                                              \
  template host::X<C::HF> msm_finish<C>(const MsmWork&);                                            \
  template void convert_bases<C>(const uint64_t*, C::A*, size_t, hipStream_t);                       \
  template void convert_bases_gather<C>(const uint64_t*, const uint32_t*, C::A*, size_t, hipStream_t);
ZK_MSM_INST(G1)
ZK_MSM_INST(G2)

}  // namespace zk
