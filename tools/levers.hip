// levers.hip -- measured prototypes of the two untried arithmetic levers of
// the G1 bucket accumulate (k_msm_accum<G1>, msm.hip), as isolated kernels
// with the accumulate's work per add: one chain of mixed additions per lane,
// each addend gathered at random from a 2^20-point table in HBM (96 B per
// affine point, as the accumulate gathers its window-shifted bases).
//
//   madd        the product's XYZZ mixed add (curve.hpp xyzz_madd, 8M + 2S)
//   madd_nc     the same add over FqNC: every Fq product with its column
//               carries replaced by one 32-bit fold (WRONG values): an upper
//               bound on what any carry-saving product form (2-column Comba)
//               can gain
//   aff<K,inv>  batch-affine accumulation: K independent chains per lane,
//               one Fq inversion per lane per step shared by the K adds
//               through Montgomery's trick (prefix products, then 2 products
//               per add back), affine add lambda = dy / dx: 6 products per
//               add + inversion / K.  inv = fermat (ff.hpp fq_inv), bgcd
//               (binary-GCD divsteps, below) or free (no inversion: the
//               arithmetic bound)
//   inv_*       one inversion chain per lane: the inversion's own cost
//
// Correctness: the batch-affine chains must equal the madd chains over the
// same index sequence after normalising (x = X / ZZ, y = Y / ZZZ); the bgcd
// inversion must equal fq_inv.  Timing: best of 3 launches at full occupancy
// (occupancy from hipOccupancyMaxActiveBlocksPerMultiprocessor).  With
// --pmc FILE every kernel runs once, in the order written to FILE
// (for SQ_INSTS_VALU per add under rocprofv3 --pmc; tools/levers.sh).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -pragma-unroll-threshold=2000000 \
//         tools/levers.hip -o tools/levers
// (the threshold lets the per-chain loops unroll, so the K chains stay in
// registers instead of scratch)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../zero-knowledge-proofs_amd/csrc/curve.hpp"

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

// ------------------------------------------------------------ FqNC -------
// Fq whose products drop the column carry (acc >> 28 into the next column):
// the high word of each column sum is XOR-folded into one register instead,
// so the 64-bit column sums stay observable (no narrowing to 32-bit
// multiplies).  Values are garbage; only the instruction stream matters.
struct FqNC {
  Fq v;
};
ZK_DI Fq nc_redc(const uint32_t (&x)[14], const uint32_t (&y)[14]) {
  constexpr int M = 14;
  uint32_t m[M], r[M], sink = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (j >= 0 && j < M) acc += (uint64_t)x[i] * y[j];
    }
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < M) acc += (uint64_t)m[i] * FqParams::MOD28[j];
    }
    if (k < M) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & 0x0fffffffu;
      acc += (uint64_t)m[k] * FqParams::MOD28[0];
    } else {
      r[k - M] = (uint32_t)acc & 0x0fffffffu;
    }
    sink ^= (uint32_t)(acc >> 32);
  }
  r[M - 1] = sink & 0x0fffffffu;
  Fq o;
  pack28<12, M>(r, o.v);
  return fp_reduce_once(o);
}
ZK_DI Fq nc_sqr(const Fq& a) {
  constexpr int M = 14;
  uint32_t x[M], m[M], r[M], sink = 0;
  unpack28<12, M>(a.v, x);
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    uint64_t cross = 0;
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < j && j < M) cross += (uint64_t)x[i] * x[j];
    }
    uint64_t acc = cross << 1;
    if ((k & 1) == 0 && k / 2 < M) acc += (uint64_t)x[k / 2] * x[k / 2];
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < M) acc += (uint64_t)m[i] * FqParams::MOD28[j];
    }
    if (k < M) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & 0x0fffffffu;
      acc += (uint64_t)m[k] * FqParams::MOD28[0];
    } else {
      r[k - M] = (uint32_t)acc & 0x0fffffffu;
    }
    sink ^= (uint32_t)(acc >> 32);
  }
  r[M - 1] = sink & 0x0fffffffu;
  Fq o;
  pack28<12, M>(r, o.v);
  return fp_reduce_once(o);
}
// a b - c d with one reduction (fq_redc2<true> without the carries)
ZK_DI Fq nc_mul_sub(const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
  constexpr int M = 14;
  uint32_t xa[M], xb[M], xc[M], xd[M], m[M], r[M], sink = 0;
  unpack28<12, M>(a.v, xa);
  unpack28<12, M>(b.v, xb);
  unpack28<12, M>(c.v, xc);
  unpack28<12, M>(d.v, xd);
  int32_t nc[M];
#pragma unroll
  for (int i = 0; i < M; i++) nc[i] = -(int32_t)xc[i];
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    int64_t acc = (int64_t)FqParams::P4SQ28[k];
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (j >= 0 && j < M) {
        acc += (int64_t)((uint64_t)xa[i] * xb[j]);
        acc += (int64_t)nc[i] * (int64_t)(int32_t)xd[j];
      }
    }
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < M) acc += (int64_t)((uint64_t)m[i] * FqParams::MOD28[j]);
    }
    if (k < M) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & 0x0fffffffu;
      acc += (int64_t)((uint64_t)m[k] * FqParams::MOD28[0]);
    } else {
      r[k - M] = (uint32_t)acc & 0x0fffffffu;
    }
    sink ^= (uint32_t)((uint64_t)acc >> 32);
  }
  r[M - 1] = sink & 0x0fffffffu;
  Fq o;
  pack28<12, M>(r, o.v);
  return fp_reduce_once(o);
}
ZK_DI FqNC f_mul(const FqNC& a, const FqNC& b) {
  uint32_t x[14], y[14];
  unpack28<12, 14>(a.v.v, x);
  unpack28<12, 14>(b.v.v, y);
  return {nc_redc(x, y)};
}
ZK_DI FqNC f_sqr(const FqNC& a) { return {nc_sqr(a.v)}; }
ZK_DI FqNC f_mul_sub(const FqNC& a, const FqNC& b, const FqNC& c, const FqNC& d) {
  return {nc_mul_sub(a.v, b.v, c.v, d.v)};
}
ZK_DI FqNC f_add(const FqNC& a, const FqNC& b) { return {fp_add(a.v, b.v)}; }
ZK_DI FqNC f_sub(const FqNC& a, const FqNC& b) { return {fp_sub(a.v, b.v)}; }
ZK_DI FqNC f_neg(const FqNC& a) { return {fp_neg(a.v)}; }
ZK_DI bool f_is_zero(const FqNC& a) { return fp_is_zero(a.v); }
ZK_DI void f_set_zero(FqNC& a) { a.v = fp_zero<FqParams>(); }
ZK_DI void f_set_one(FqNC& a) { a.v = fp_one<FqParams>(); }

// ------------------------------------------------------ bgcd inversion ---
// Constant-time binary GCD in the Bernstein-Yang divstep form over 32-bit
// words of the canonical value: each round runs 30 divsteps on the low words
// of (f, g) with a 2x2 transition matrix (entries |.| <= 2^30), then applies
// it to the full f, g (13 signed 30-bit limbs) and to d, e (tracked mod p,
// made divisible by 2^30 by adding a multiple of p).  ceil(1101 / 30) = 37
// rounds bound 381-bit inputs.  Input / output in Montgomery form (R = 2^392):
// the canonical inverse is mapped back with two products.
constexpr int BG_L = 13;                  // 13 x 30 bits >= 390 bits
constexpr uint32_t BG_M30 = 0x3fffffffu;
struct Sig { int32_t v[BG_L]; };          // signed 30-bit limbs, top limb signed
// p in 30-bit limbs, and p^-1 mod 2^30
struct BgConst {
  int32_t p30[BG_L];
  uint32_t pinv30;   // p^-1 mod 2^30
};
__constant__ BgConst BG;

ZK_DI int32_t bg_divsteps30(int32_t zeta, uint32_t f0, uint32_t g0, int32_t (&t)[4]) {
  // libsecp256k1-style variable-free formulation (zeta = -(delta + 1/2))
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0;
#pragma unroll 2
  for (int i = 0; i < 30; i++) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);                  // -1 if zeta < 0
    const uint32_t c2 = 0u - (g & 1u);                           // -1 if g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2; q += y & c2; r += z & c2;
    const uint32_t c3 = c1 & c2;
    zeta = (zeta ^ (int32_t)c3) - 1;
    f += g & c3; u += q & c3; v += r & c3;
    g >>= 1; u <<= 1; v <<= 1;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return zeta;
}
// (f, g) <- (u f + v g, q f + r g) / 2^30   (exact)
ZK_DI void bg_update_fg(Sig& f, Sig& g, const int32_t (&t)[4]) {
  int64_t cf = (int64_t)t[0] * f.v[0] + (int64_t)t[1] * g.v[0];
  int64_t cg = (int64_t)t[2] * f.v[0] + (int64_t)t[3] * g.v[0];
  cf >>= 30; cg >>= 30;
#pragma unroll
  for (int i = 1; i < BG_L; i++) {
    cf += (int64_t)t[0] * f.v[i] + (int64_t)t[1] * g.v[i];
    cg += (int64_t)t[2] * f.v[i] + (int64_t)t[3] * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & BG_M30); cf >>= 30;
    g.v[i - 1] = (int32_t)((uint32_t)cg & BG_M30); cg >>= 30;
  }
  f.v[BG_L - 1] = (int32_t)cf;
  g.v[BG_L - 1] = (int32_t)cg;
}
// (d, e) <- (u d + v e, q d + r e) / 2^30 mod p, inputs in (-2p, p), outputs too
ZK_DI void bg_update_de(Sig& d, Sig& e, const int32_t (&t)[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d.v[BG_L - 1] >> 31, se = e.v[BG_L - 1] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((BG.pinv30 * (uint32_t)cd + (uint32_t)md) & BG_M30);
  me -= (int32_t)((BG.pinv30 * (uint32_t)ce + (uint32_t)me) & BG_M30);
  cd += (int64_t)BG.p30[0] * md;
  ce += (int64_t)BG.p30[0] * me;
  cd >>= 30; ce >>= 30;
#pragma unroll
  for (int i = 1; i < BG_L; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)BG.p30[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)BG.p30[i] * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & BG_M30); cd >>= 30;
    e.v[i - 1] = (int32_t)((uint32_t)ce & BG_M30); ce >>= 30;
  }
  d.v[BG_L - 1] = (int32_t)cd;
  e.v[BG_L - 1] = (int32_t)ce;
}
// canonical 12-word x -> 30-bit limbs
ZK_DI Sig bg_from_words(const uint32_t (&w)[12]) {
  Sig s;
#pragma unroll
  for (int i = 0; i < BG_L; i++) {
    const int bit = 30 * i, k = bit >> 5, sh = bit & 31;
    const uint32_t lo = k < 12 ? w[k] : 0u, hi = k + 1 < 12 ? w[k + 1] : 0u;
    const uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
    s.v[i] = (int32_t)(v & BG_M30);
  }
  return s;
}
// normalise d (in (-2p, p)) to [0, p) times sign, to 12 words
ZK_DI void bg_to_words(Sig d, int32_t fsign, uint32_t (&w)[12]) {
  // d <- d + p if d < 0; negate if fsign < 0; d <- d + p if d < 0 again
  for (int pass = 0; pass < 3; pass++) {
    int32_t sg = d.v[BG_L - 1] >> 31;
    if (pass == 1) sg = fsign;   // negate step
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < BG_L; i++) {
      if (pass == 1) c += (int64_t)((d.v[i] ^ sg) - sg);
      else c += (int64_t)d.v[i] + (int64_t)(BG.p30[i] & sg);
      d.v[i] = (int32_t)((uint32_t)c & BG_M30);
      c >>= 30;
    }
    d.v[BG_L - 1] += (int32_t)(c << 30);
  }
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const int bit = 32 * k, i = bit / 30, sh = bit - 30 * i;
    uint32_t v = (uint32_t)d.v[i] >> sh;
    if (i + 1 < BG_L) v |= (uint32_t)d.v[i + 1] << (30 - sh);
    if (sh > 28 && i + 2 < BG_L) v |= (uint32_t)d.v[i + 2] << (60 - sh);
    w[k] = v;
  }
}
// Montgomery-form inverse: a R -> a^-1 R.  canonical(aR)^-1 = a^-1 R^-1, so
// the result is that times R^3 (two products with R^2).  0 -> 0.
ZK_DI Fq fq_inv_bgcd(const Fq& a) {
  Sig f, g, d, e;
#pragma unroll
  for (int i = 0; i < BG_L; i++) { f.v[i] = BG.p30[i]; d.v[i] = 0; e.v[i] = i == 0; }
  g = bg_from_words(a.v);
  int32_t zeta = -1;
  for (int round = 0; round < 37; round++) {
    int32_t t[4];
    zeta = bg_divsteps30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    bg_update_de(d, e, t);
    bg_update_fg(f, g, t);
  }
  // f = +-1 now; d = +-a^-1
  Fq o;
  bg_to_words(d, f.v[BG_L - 1] >> 31, o.v);
  const Fq r2 = fp_from_const<FqParams>(FqParams::R2);
  return fq_mul(fq_mul(o, r2), r2);
}

// ------------------------------------------------------------ kernels ----
ZK_DI uint32_t hidx(uint32_t c, uint32_t s, uint32_t mask) {
  uint32_t h = (c * 0x9E3779B1u) ^ (s * 0x85EBCA77u + 0x165667B1u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & mask;
}

template <class F, int W = 0>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(W ? W : 1))) k_chain_madd(const Affine<F>* __restrict__ pts, uint32_t mask, uint32_t steps,
                                                    uint32_t nchain, XYZZ<F>* __restrict__ out) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchain) return;
  XYZZ<F> acc = xyzz_from_aff(ld_vec(&pts[hidx(c, 0, mask)]));
  for (uint32_t s = 1; s <= steps; s++) acc = xyzz_madd(acc, ld_vec(&pts[hidx(c, s, mask)]));
  st_vec(&out[c], acc);
}

enum { INV_FREE = 0, INV_FERMAT = 1, INV_BGCD = 2 };
template <int MODE>
ZK_DI Fq inv_mode(const Fq& x) {
  if constexpr (MODE == INV_FERMAT) return fq_inv(x);
  else if constexpr (MODE == INV_BGCD) return fq_inv_bgcd(x);
  else return x;
}

// PL: the prefix products live in LDS (word-major per lane, conflict-free)
// instead of registers
// W: waves per SIMD the register allocation must allow (0: compiler's choice)
template <int K, int MODE, bool PL = false, int W = 0>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(W ? W : 1))) k_chain_affine(const G1A* __restrict__ pts, uint32_t mask, uint32_t steps,
                                                      uint32_t nthr, G1A* __restrict__ out, uint32_t* __restrict__ bad) {
  __shared__ uint32_t pre_lds[PL ? K * 12 * 128 : 1];
  auto pst = [&](int k, const Fq& v) {
#pragma unroll
    for (int w = 0; w < 12; w++) pre_lds[(k * 12 + w) * 128 + threadIdx.x] = v.v[w];
  };
  auto pld = [&](int k) {
    Fq v;
#pragma unroll
    for (int w = 0; w < 12; w++) v.v[w] = pre_lds[(k * 12 + w) * 128 + threadIdx.x];
    return v;
  };
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthr) return;
  G1A acc[K];
#pragma unroll
  for (int k = 0; k < K; k++) acc[k] = ld_vec(&pts[hidx(t * K + k, 0, mask)]);
  uint32_t z = 0;
  for (uint32_t s = 1; s <= steps; s++) {
    Fq pre[PL ? 1 : K], run;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const Fq x2 = ld_vec(&pts[hidx(t * K + k, s, mask)].x);
      const Fq d = fp_sub(x2, acc[k].x);
      z |= fp_is_zero(d) ? 1u : 0u;   // x1 == x2: the product would route this add elsewhere
      run = k ? fq_mul(run, d) : d;
      if constexpr (PL) { if (k < K - 1) pst(k, run); }
      else pre[k] = run;
      ZK_SB();
    }
    Fq inv = inv_mode<MODE>(run);
#pragma unroll
    for (int k = K - 1; k >= 0; k--) {
      const G1A p = ld_vec(&pts[hidx(t * K + k, s, mask)]);
      const Fq d = fp_sub(p.x, acc[k].x);
      Fq dinv = inv;
      if (k) {
        if constexpr (PL) dinv = fq_mul(inv, pld(k - 1));
        else dinv = fq_mul(inv, pre[k - 1]);
        ZK_SB();
        inv = fq_mul(inv, d);
        ZK_SB();
      }
      const Fq lam = fq_mul(fp_sub(p.y, acc[k].y), dinv);
      ZK_SB();
      const Fq x3 = fp_sub(fp_sub(fp_sqr(lam), acc[k].x), p.x);
      ZK_SB();
      acc[k].y = fp_sub(fq_mul(lam, fp_sub(acc[k].x, x3)), acc[k].y);
      ZK_SB();
      acc[k].x = x3;
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) st_vec(&out[t * K + k], acc[k]);
  bad[t] = z;
}

// one inversion chain per lane: x <- inv(x) + x  (the add keeps it from cycling)
template <int MODE>
__global__ void __launch_bounds__(128) k_inv_chain(const G1A* __restrict__ pts, uint32_t mask, uint32_t iters,
                                                   uint32_t nthr, Fq* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthr) return;
  Fq x = ld_vec(&pts[hidx(t, 0, mask)].x);
  for (uint32_t i = 0; i < iters; i++) x = fp_add(inv_mode<MODE>(x), x);
  st_vec(&out[t], x);
}
// the two inversions side by side, for the check
__global__ void k_inv_check(const G1A* __restrict__ pts, uint32_t mask, uint32_t n, Fq* __restrict__ o1,
                            Fq* __restrict__ o2) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const Fq x = t == 0 ? fp_zero<FqParams>() : ld_vec(&pts[hidx(t, 7, mask)].x);
  st_vec(&o1[t], fq_inv(x));
  st_vec(&o2[t], fq_inv_bgcd(x));
}
// normalise madd chain c and compare with affine chain c
__global__ void k_compare(const G1X* __restrict__ xs, const G1A* __restrict__ as, uint32_t n, uint32_t* __restrict__ ok) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const G1X p = ld_vec(&xs[c]);
  const G1A a = ld_vec(&as[c]);
  const Fq x = fq_mul(p.X, fq_inv(p.ZZ)), y = fq_mul(p.Y, fq_inv(p.ZZZ));
  ok[c] = (fp_eq(x, a.x) && fp_eq(y, a.y)) ? 1u : 0u;
}

// s P + r Q on ONE wave (the pi_C term s pi_A + r B1 moved to the GPU, as a
// latency measurement): 4-bit Straus, 2 x 15 table adds, 256 doublings and
// up to 128 adds, tables in global memory per lane (each lane computes the
// same term)
__global__ void __launch_bounds__(64) k_straus(const G1A* __restrict__ pts, uint4 ka, uint4 kb, uint4 kc, uint4 kd,
                                               G1X* __restrict__ tab, G1X* __restrict__ out) {
  const uint32_t lane = threadIdx.x;
  G1X* tp = tab + lane * 32;
  G1X* tq = tp + 16;
  const G1A P = ld_vec(&pts[1]), Q = ld_vec(&pts[2]);
  G1X t;
  xyzz_set_inf(t);
  st_vec(&tp[0], t);
  st_vec(&tq[0], t);
  t = xyzz_from_aff(P);
  st_vec(&tp[1], t);
  for (int i = 2; i < 16; i++) { t = xyzz_madd(t, P); st_vec(&tp[i], t); }
  t = xyzz_from_aff(Q);
  st_vec(&tq[1], t);
  for (int i = 2; i < 16; i++) { t = xyzz_madd(t, Q); st_vec(&tq[i], t); }
  const uint32_t k1[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
  const uint32_t k2[8] = {kc.x, kc.y, kc.z, kc.w, kd.x, kd.y, kd.z, kd.w};
  G1X acc;
  xyzz_set_inf(acc);
  for (int w = 63; w >= 0; w--) {
    for (int d = 0; d < 4; d++) acc = xyzz_dbl(acc);
    const uint32_t d1 = (k1[w >> 3] >> ((w & 7) * 4)) & 15u, d2 = (k2[w >> 3] >> ((w & 7) * 4)) & 15u;
    if (d1) acc = xyzz_add(acc, ld_vec(&tp[d1]));
    if (d2) acc = xyzz_add(acc, ld_vec(&tq[d2]));
  }
  st_vec(&out[lane], acc);
}

// ------------------------------------------------------------- host ------
static int g_cus = 0;
static FILE* g_adds = nullptr;
static bool g_pmc = false;

template <class Kern>
static uint32_t full_threads(Kern k, int* wps, int* vgpr) {
  int per_cu = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 128, 0));
  hipFuncAttributes fa;
  CHK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k)));
  *wps = per_cu * 2 / 4;   // 128 threads = 2 waves, 4 SIMDs per CU
  *vgpr = fa.numRegs;
  return (uint32_t)per_cu * g_cus * 128;
}

struct Result {
  std::string name;
  double ms, gadds;
  int wps, vgpr;
};

template <class Launch>
static double time_launch(Launch L) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  double best = 1e30;
  for (int rep = 0; rep < (g_pmc ? 1 : 3); rep++) {
    CHK(hipEventRecord(a));
    L();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return best;
}

static void note(const char* name, double adds) {
  if (g_adds) fprintf(g_adds, "%s %.0f\n", name, adds);
}

int main(int argc, char** argv) {
  const char* adds_path = nullptr;
  for (int i = 1; i + 1 < argc; i++)
    if (!strcmp(argv[i], "--pmc")) { g_pmc = true; adds_path = argv[i + 1]; }
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  g_cus = prop.multiProcessorCount;
  const uint32_t LOGB = 20, NB = 1u << LOGB, MASK = NB - 1;
  // random table "points": field elements < p (top word < 2^28); the chord
  // formulas do not use the curve equation
  std::vector<uint32_t> h(NB * 24);
  uint64_t s = 0x1e7e45ull;
  for (size_t i = 0; i < h.size(); i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)(s >> 11);
    if (i % 12 == 11) h[i] &= 0x0fffffffu;
  }
  // bgcd constants: p in 30-bit limbs, p^-1 mod 2^30
  BgConst bc;
  for (int i = 0; i < BG_L; i++) {
    const int bit = 30 * i, k = bit >> 5, sh = bit & 31;
    uint64_t lo = FqParams::MOD[k];
    if (k + 1 < 12) lo |= (uint64_t)FqParams::MOD[k + 1] << 32;
    bc.p30[i] = (int32_t)((lo >> sh) & BG_M30);
  }
  uint32_t x = 1;
  for (int k = 0; k < 6; k++) x *= 2 - FqParams::MOD[0] * x;
  bc.pinv30 = x & BG_M30;
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(BG), &bc, sizeof bc));
  G1A* pts;
  CHK(hipMalloc(&pts, (size_t)NB * sizeof(G1A)));
  CHK(hipMemcpy(pts, h.data(), (size_t)NB * sizeof(G1A), hipMemcpyHostToDevice));
  const size_t OUTN = 8u << 20;
  G1X* ox;
  G1A* oa;
  uint32_t *bad, *ok;
  Fq *f1, *f2;
  CHK(hipMalloc(&ox, OUTN * sizeof(G1X)));
  CHK(hipMalloc(&oa, OUTN * sizeof(G1A)));
  CHK(hipMalloc(&bad, OUTN * 4));
  CHK(hipMalloc(&ok, OUTN * 4));
  CHK(hipMalloc(&f1, OUTN * sizeof(Fq)));
  CHK(hipMalloc(&f2, OUTN * sizeof(Fq)));
  if (g_pmc) g_adds = fopen(adds_path, "w");

  // ---- correctness: bgcd == fermat; affine chains == madd chains
  if (!g_pmc) {
    const uint32_t n = 4096;
    k_inv_check<<<n / 128, 128>>>(pts, MASK, n, f1, f2);
    CHK(hipDeviceSynchronize());
    std::vector<uint32_t> a(n * 12), b(n * 12);
    CHK(hipMemcpy(a.data(), f1, n * 48, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(b.data(), f2, n * 48, hipMemcpyDeviceToHost));
    int bad_inv = 0;
    for (uint32_t i = 0; i < n; i++) bad_inv += memcmp(&a[i * 12], &b[i * 12], 48) != 0;
    printf("check bgcd inversion == fermat (incl. 0): %s (%d of %u differ)\n", bad_inv ? "FAIL" : "ok", bad_inv, n);
    const uint32_t S = 9, T = 1024, K = 4;
    k_chain_madd<Fq><<<T * K / 128, 128>>>(pts, MASK, S, T * K, ox);
    k_chain_affine<4, INV_BGCD><<<T / 128, 128>>>(pts, MASK, S, T, oa, bad);
    k_compare<<<T * K / 128, 128>>>(ox, oa, T * K, ok);
    CHK(hipDeviceSynchronize());
    std::vector<uint32_t> okh(T * K);
    CHK(hipMemcpy(okh.data(), ok, T * K * 4, hipMemcpyDeviceToHost));
    int good = 0;
    for (auto v : okh) good += v;
    printf("check batch-affine (K=4, bgcd) chains == madd chains: %s (%d of %u)\n", good == (int)(T * K) ? "ok" : "FAIL",
           good, T * K);
    k_chain_affine<4, INV_FERMAT><<<T / 128, 128>>>(pts, MASK, S, T, oa, bad);
    k_compare<<<T * K / 128, 128>>>(ox, oa, T * K, ok);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(okh.data(), ok, T * K * 4, hipMemcpyDeviceToHost));
    good = 0;
    for (auto v : okh) good += v;
    printf("check batch-affine (K=4, fermat) chains == madd chains: %s (%d of %u)\n", good == (int)(T * K) ? "ok" : "FAIL",
           good, T * K);
  }

  std::vector<Result> res;
  int wps, vg;
  // ---- madd (product add) and the carry-free bound
  {
    const uint32_t S = 96;
    uint32_t T = full_threads(k_chain_madd<Fq>, &wps, &vg);
    double ms = time_launch([&] { k_chain_madd<Fq><<<T / 128, 128>>>(pts, MASK, S, T, ox); });
    note("k_chain_madd<Fq>", (double)T * S);
    res.push_back({"madd (xyzz_madd, product)", ms, (double)T * S / ms / 1e6, wps, vg});
    const Affine<FqNC>* pn = reinterpret_cast<const Affine<FqNC>*>(pts);
    XYZZ<FqNC>* on = reinterpret_cast<XYZZ<FqNC>*>(ox);
    T = full_threads(k_chain_madd<FqNC>, &wps, &vg);
    ms = time_launch([&] { k_chain_madd<FqNC><<<T / 128, 128>>>(pn, MASK, S, T, on); });
    note("k_chain_madd<FqNC>", (double)T * S);
    res.push_back({"madd, no column carries (bound)", ms, (double)T * S / ms / 1e6, wps, vg});
    T = full_threads(k_chain_madd<FqNC, 3>, &wps, &vg);
    ms = time_launch([&] { k_chain_madd<FqNC, 3><<<T / 128, 128>>>(pn, MASK, S, T, on); });
    note("k_chain_madd<FqNC, 3>", (double)T * S);
    res.push_back({"madd, no column carries, 3 waves (bound)", ms, (double)T * S / ms / 1e6, wps, vg});
  }
  // ---- batch affine
#define AFF(KK, MODE, NAME, S)                                                              \
  {                                                                                         \
    uint32_t T = full_threads(k_chain_affine<KK, MODE>, &wps, &vg);                         \
    double ms = time_launch([&] { k_chain_affine<KK, MODE><<<T / 128, 128>>>(pts, MASK, S, T, oa, bad); }); \
    note("k_chain_affine<" #KK ", " #MODE ">", (double)T * S * KK);                        \
    res.push_back({NAME, ms, (double)T * S * KK / ms / 1e6, wps, vg});                      \
  }
#define AFFL(KK, MODE, NAME, S)                                                             \
  {                                                                                         \
    uint32_t T = full_threads(k_chain_affine<KK, MODE, true>, &wps, &vg);                   \
    double ms = time_launch([&] { k_chain_affine<KK, MODE, true><<<T / 128, 128>>>(pts, MASK, S, T, oa, bad); }); \
    note("k_chain_affine<" #KK ", " #MODE ", true>", (double)T * S * KK);                  \
    res.push_back({NAME, ms, (double)T * S * KK / ms / 1e6, wps, vg});                      \
  }
#define AFFW(KK, MODE, WW, NAME, S)                                                         \
  {                                                                                         \
    uint32_t T = full_threads(k_chain_affine<KK, MODE, true, WW>, &wps, &vg);               \
    double ms = time_launch([&] { k_chain_affine<KK, MODE, true, WW><<<T / 128, 128>>>(pts, MASK, S, T, oa, bad); }); \
    note("k_chain_affine<" #KK ", " #MODE ", true, " #WW ">", (double)T * S * KK);         \
    res.push_back({NAME, ms, (double)T * S * KK / ms / 1e6, wps, vg});                      \
  }
  AFF(2, INV_FREE, "affine K=2, inversion free (bound)", 48)
  AFF(4, INV_FREE, "affine K=4, inversion free (bound)", 24)
  AFF(8, INV_FREE, "affine K=8, inversion free (bound)", 12)
  AFF(16, INV_FREE, "affine K=16, inversion free (bound)", 6)
  AFFL(4, INV_FREE, "affine K=4, LDS prefixes, inversion free", 24)
  AFFL(8, INV_FREE, "affine K=8, LDS prefixes, inversion free", 12)
  AFFW(4, INV_FREE, 2, "affine K=4, LDS prefixes, 2 waves, inv free", 24)
  AFFW(4, INV_BGCD, 2, "affine K=4, LDS prefixes, 2 waves, bgcd", 24)
  AFF(4, INV_BGCD, "affine K=4, bgcd inversion", 24)
  AFFL(4, INV_BGCD, "affine K=4, LDS prefixes, bgcd inversion", 24)
  AFFL(8, INV_BGCD, "affine K=8, LDS prefixes, bgcd inversion", 12)
  AFF(8, INV_BGCD, "affine K=8, bgcd inversion", 12)
  AFF(16, INV_BGCD, "affine K=16, bgcd inversion", 6)
  AFF(8, INV_FERMAT, "affine K=8, fermat inversion", 6)
  // ---- inversion alone (per lane): reported as inversions/s
  {
    uint32_t T = full_threads(k_inv_chain<INV_BGCD>, &wps, &vg);
    double ms = time_launch([&] { k_inv_chain<INV_BGCD><<<T / 128, 128>>>(pts, MASK, 8, T, f1); });
    note("k_inv_chain<2>", (double)T * 8);
    res.push_back({"inversion bgcd (G inv/s)", ms, (double)T * 8 / ms / 1e6, wps, vg});
    T = full_threads(k_inv_chain<INV_FERMAT>, &wps, &vg);
    ms = time_launch([&] { k_inv_chain<INV_FERMAT><<<T / 128, 128>>>(pts, MASK, 2, T, f1); });
    note("k_inv_chain<1>", (double)T * 2);
    res.push_back({"inversion fermat (G inv/s)", ms, (double)T * 2 / ms / 1e6, wps, vg});
  }
  // ---- the pi_C Straus term on one wave (latency, not throughput)
  if (!g_pmc) {
    G1X* tab;
    CHK(hipMalloc(&tab, 64 * 32 * sizeof(G1X)));
    const uint4 ka = {0x89abcdefu, 0x01234567u, 0xdeadbeefu, 0x8badf00du},
                kb = {0x13579bdfu, 0x2468ace0u, 0x0f1e2d3cu, 0x0a1b2c3du},
                kc = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u},
                kd = {0x55555555u, 0x66666666u, 0x77777777u, 0x08888888u};
    const double ms = time_launch([&] { k_straus<<<1, 64>>>(pts, ka, kb, kc, kd, tab, ox); });
    printf("pi_C Straus term s P + r Q (255-bit scalars, 4-bit windows) on one wave: %.3f ms per launch\n", ms);
    CHK(hipFree(tab));
  }
  const double base = res[0].gadds;
  printf("%-40s %8s %10s %8s %5s %5s\n", "variant", "ms", "G adds/s", "vs madd", "w/SIMD", "VGPR");
  for (auto& r : res)
    printf("%-40s %8.3f %10.3f %8.3f %5d %5d\n", r.name.c_str(), r.ms, r.gadds, r.gadds / base, r.wps, r.vgpr);
  if (g_adds) fclose(g_adds);
  return 0;
}
