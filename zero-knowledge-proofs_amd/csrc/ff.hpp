// ff.hpp -- device prime-field arithmetic for gfx950 (CDNA4).
//
// Mirrors ark-ff 0.4.2's Fp<MontBackend<_, N64>, N64> (the Fr / Fq behind
// groth16-field's `F`, crates/groth16-field/src/lib.rs:14-17): Montgomery form
// with R = 2^(64*N64), little-endian limbs.  On device the same bytes are
// handled as 2*N64 32-bit limbs so that every limb product is one
// v_mad_u64_u32 (32x32+64 -> 64) -- the widest integer multiply CDNA4 has.
// No MFMA: this is carry-chained modular arithmetic, not a contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "constants.hpp"

#define ZK_DI __device__ __forceinline__

// 16-byte vector global loads / stores of whole field elements / points.
// __builtin_memcpy (not pointer punning into the destination) keeps arrays
// of elements promotable to registers.
template <class T>
ZK_DI T ld_vec(const T* p) {
  static_assert(sizeof(T) % 16 == 0, "16-byte multiple");
  T r;
  const uint4* s = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) {
    const uint4 u = s[i];
    __builtin_memcpy(reinterpret_cast<char*>(&r) + 16 * i, &u, 16);
  }
  return r;
}
template <class T>
ZK_DI void st_vec(T* p, const T& v) {
  static_assert(sizeof(T) % 16 == 0, "16-byte multiple");
  uint4* d = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) {
    uint4 u;
    __builtin_memcpy(&u, reinterpret_cast<const char*>(&v) + 16 * i, 16);
    d[i] = u;
  }
}

template <class P>
struct Fp {
  uint32_t v[P::N];
};

using Fq = Fp<FqParams>;
using Fr = Fp<FrParams>;

template <class P>
ZK_DI Fp<P> fp_zero() {
  Fp<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = 0;
  return r;
}
template <class P>
ZK_DI Fp<P> fp_one() {
  Fp<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = P::ONE[i];
  return r;
}
template <class P>
ZK_DI Fp<P> fp_from_const(const uint32_t (&c)[P::N]) {
  Fp<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = c[i];
  return r;
}
template <class P>
ZK_DI bool fp_is_zero(const Fp<P>& a) {
  uint32_t x = a.v[0];
#pragma unroll
  for (int i = 1; i < P::N; i++) x |= a.v[i];
  return x == 0;
}
template <class P>
ZK_DI bool fp_eq(const Fp<P>& a, const Fp<P>& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}

// r = a - m if a >= m else a   (a < 2m)
template <class P>
ZK_DI Fp<P> fp_reduce_once(const Fp<P>& a) {
  Fp<P> s;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) s.v[i] = __builtin_subc(a.v[i], P::MOD[i], br, &br);
  Fp<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = br ? a.v[i] : s.v[i];
  return r;
}

template <class P>
ZK_DI Fp<P> fp_add(const Fp<P>& a, const Fp<P>& b) {
  Fp<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  return fp_reduce_once(r);   // a + b < 2m < 2^(32N): no carry out
}
template <class P>
ZK_DI Fp<P> fp_dbl(const Fp<P>& a) { return fp_add(a, a); }

template <class P>
ZK_DI Fp<P> fp_sub(const Fp<P>& a, const Fp<P>& b) {
  Fp<P> r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  uint32_t mask = 0u - br, c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = __builtin_addc(r.v[i], P::MOD[i] & mask, c, &c);
  return r;
}
template <class P>
ZK_DI Fp<P> fp_neg(const Fp<P>& a) { return fp_sub(fp_zero<P>(), a); }

// Montgomery product a*b/R mod m by radix-2^LB product scanning.
// The 32-bit storage limbs are re-cut into NL limbs of LB bits (Fq 14 x 28,
// Fr 9 x 29) so that every limb product (< 2^(2 LB)) accumulates into a
// 64-bit column sum with a single v_mad_u64_u32 -- no carry flags, no carry
// chains: a column holds at most 2*NL products (Fq < 2^61, Fr < 2^62.2).
// Montgomery reduction is interleaved per column (m_k = low LB bits *
// -m^-1), so R = 2^(LB NL) (2^392 for Fq, 2^261 for Fr).  Inputs < 2^(32N);
// output < 2m, reduced once.  Measured 2.1x the 32-bit CIOS on gfx950
// (tools/mulbench.hip); Fr at 9 x 29 bits: 162 instead of 200 v_mad.
// Fr column sums in ONE dependency chain (ZK_MAD_CHAIN, default on): every
// limb product is an inline-asm v_mad whose addend is the running column
// sum.  Plain C lets LLVM re-associate each column into a chain from 0 plus
// one v_lshl_add_u64 of the previous column's carry -- a 64-bit add (~5 issue
// cycles, as many as a v_mad) per column, 17 per Fr product, bought for
// latency that the NTT's 4 waves/SIMD already hide: 2^22 API NTT 0.554 ->
// 0.533 ms.  Fq keeps the split columns: its 28-product chains at 3
// waves/SIMD lost (2^20 MSM 3.61 -> 3.85 ms, prove 9.68 -> 10.13 ms;
// profiles/r03_ab_mad_chain.txt).
#ifndef ZK_MAD_CHAIN
#define ZK_MAD_CHAIN 1
#endif
template <bool CH>
ZK_DI void mad_acc(uint64_t& acc, uint32_t a, uint32_t b) {
  if constexpr (CH) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
  else acc += (uint64_t)a * b;
}
// b a compile-time constant (modulus limbs): an SGPR operand
template <bool CH>
ZK_DI void mad_acc_k(uint64_t& acc, uint32_t a, uint32_t b) {
  if constexpr (CH) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "s"(b) : "vcc");
  else acc += (uint64_t)a * b;
}
template <class P>
constexpr bool mad_chain() { return ZK_MAD_CHAIN && P::NL <= 9; }
// Two chained v_mad per asm statement: the compiler pads every inline-asm
// statement with an s_nop (it cannot see inside), so pairs halve the pads
// (ZK_MAD_PAIR: A/B builds)
#ifndef ZK_MAD_PAIR
#define ZK_MAD_PAIR 0
#endif
ZK_DI void mad_acc2(uint64_t& acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %4, %0"
      : "+v"(acc) : "v"(a0), "v"(b0), "v"(a1), "v"(b1) : "vcc");
}
ZK_DI void mad_acc2_k(uint64_t& acc, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %4, %0"
      : "+v"(acc) : "v"(a0), "s"(b0), "v"(a1), "s"(b1) : "vcc");
}

template <int N, int M, int LB = 28>
ZK_DI void unpack28(const uint32_t (&a)[N], uint32_t (&o)[M]) {
  constexpr uint32_t MASK = (1u << LB) - 1;
#pragma unroll
  for (int i = 0; i < M; i++) {
    const int bit = LB * i, w = bit >> 5, s = bit & 31;
    const uint32_t lo = w < N ? a[w] : 0u;
    const uint32_t hi = (w + 1 < N) ? a[w + 1] : 0u;
    const uint32_t v = s ? __builtin_amdgcn_alignbit(hi, lo, s) : lo;
    o[i] = v & MASK;
  }
}
template <int N, int M, int LB = 28>
ZK_DI void pack28(const uint32_t (&r)[M], uint32_t (&o)[N]) {
#pragma unroll
  for (int w = 0; w < N; w++) {
    const int bit = 32 * w, i = bit / LB, s = bit - LB * i;   // 0 <= s < LB
    uint32_t v = r[i] >> s;
    if (i + 1 < M && LB - s < 32) v |= r[i + 1] << (LB - s);
    if (2 * LB - s < 32 && i + 2 < M) v |= r[i + 2] << (2 * LB - s);
    o[w] = v;
  }
}
// The product on operands already cut into limbs.  RED = false skips the
// final subtraction: the result is then < 2m (inputs < 2^(32N)), which the
// NTT's tile arithmetic keeps (ntt.hip, fr_*_lz).
template <class P, bool RED = true>
ZK_DI Fp<P> fp_mul_limbs(const uint32_t (&x)[P::NL], const uint32_t (&y)[P::NL]) {
  constexpr int N = P::N, M = P::NL, LB = P::LB;
  constexpr uint32_t MASK = (1u << LB) - 1;
  uint32_t m[M], r[M];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    uint64_t acc = carry;
    if constexpr (mad_chain<P>() && ZK_MAD_PAIR) {
#pragma unroll
      for (int i = 0; i < M; i += 2) {
        const int j0 = k - i, j1 = k - i - 1;
        const bool v0 = j0 >= 0 && j0 < M, v1 = i + 1 < M && j1 >= 0 && j1 < M;
        if (v0 && v1) mad_acc2(acc, x[i], y[j0], x[i + 1], y[j1]);
        else if (v0) mad_acc<true>(acc, x[i], y[j0]);
        else if (v1) mad_acc<true>(acc, x[i + 1], y[j1]);
      }
#pragma unroll
      for (int i = 0; i < M; i += 2) {
        const int j0 = k - i, j1 = k - i - 1;
        const bool v0 = i < k && j0 >= 1 && j0 < M, v1 = i + 1 < M && i + 1 < k && j1 >= 1 && j1 < M;
        if (v0 && v1) mad_acc2_k(acc, m[i], P::MODL[j0], m[i + 1], P::MODL[j1]);
        else if (v0) mad_acc_k<true>(acc, m[i], P::MODL[j0]);
        else if (v1) mad_acc_k<true>(acc, m[i + 1], P::MODL[j1]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < M; i++) {
        const int j = k - i;
        if (j >= 0 && j < M) mad_acc<mad_chain<P>()>(acc, x[i], y[j]);
      }
#pragma unroll
      for (int i = 0; i < M; i++) {
        const int j = k - i;
        if (i < k && j >= 1 && j < M) mad_acc_k<mad_chain<P>()>(acc, m[i], P::MODL[j]);
      }
    }
    if (k < M) {
      m[k] = ((uint32_t)acc * P::INVL) & MASK;
      acc += (uint64_t)m[k] * P::MODL[0];
    } else {
      r[k - M] = (uint32_t)acc & MASK;
    }
    carry = acc >> LB;
  }
  r[M - 1] = (uint32_t)carry;
  Fp<P> o;
  pack28<N, M, LB>(r, o.v);
  if constexpr (RED) return fp_reduce_once(o);
  else return o;
}
template <class P, bool RED = true>
ZK_DI Fp<P> fp_mul(const Fp<P>& a, const Fp<P>& b) {
  uint32_t x[P::NL], y[P::NL];
  unpack28<P::N, P::NL, P::LB>(a.v, x);
  unpack28<P::N, P::NL, P::LB>(b.v, y);
  return fp_mul_limbs<P, RED>(x, y);
}
// Squaring: column k of a^2 is 2 sum_{i<j} a_i a_j (+ a_{k/2}^2), so the
// product half needs M(M+1)/2 v_mad instead of M^2 (Fq: 105 vs 196); the
// interleaved Montgomery reduction is unchanged.
template <class P>
ZK_DI Fp<P> fp_sqr(const Fp<P>& a) {
  constexpr int N = P::N, M = P::NL, LB = P::LB;
  constexpr uint32_t MASK = (1u << LB) - 1;
  uint32_t x[M], m[M], r[M];
  unpack28<N, M, LB>(a.v, x);
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    uint64_t cross = 0;
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < j && j < M) mad_acc<mad_chain<P>()>(cross, x[i], x[j]);
    }
    uint64_t acc = carry + (cross << 1);
    if ((k & 1) == 0 && k / 2 < M) mad_acc<mad_chain<P>()>(acc, x[k / 2], x[k / 2]);
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < M) mad_acc_k<mad_chain<P>()>(acc, m[i], P::MODL[j]);
    }
    if (k < M) {
      m[k] = ((uint32_t)acc * P::INVL) & MASK;
      acc += (uint64_t)m[k] * P::MODL[0];
    } else {
      r[k - M] = (uint32_t)acc & MASK;
    }
    carry = acc >> LB;
  }
  r[M - 1] = (uint32_t)carry;
  Fp<P> o;
  pack28<N, M, LB>(r, o.v);
  return fp_reduce_once(o);
}

template <class P>
ZK_DI Fp<P> fp_to_mont(const Fp<P>& canon) { return fp_mul(canon, fp_from_const<P>(P::R2)); }
template <class P>
ZK_DI Fp<P> fp_from_mont(const Fp<P>& a) {
  Fp<P> one;
#pragma unroll
  for (int i = 0; i < P::N; i++) one.v[i] = i == 0 ? 1u : 0u;
  return fp_mul(a, one);
}
// a^(m-2): Fermat inversion (0 -> 0)
template <class P>
ZK_DI Fp<P> fp_inv(const Fp<P>& a) {
  uint32_t e[P::N];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) e[i] = __builtin_subc(P::MOD[i], i == 0 ? 2u : 0u, br, &br);
  Fp<P> acc = fp_one<P>();
  for (int i = P::N - 1; i >= 0; i--) {
    for (int k = 31; k >= 0; k--) {
      acc = fp_sqr(acc);
      if ((e[i] >> k) & 1) acc = fp_mul(acc, a);
    }
  }
  return acc;
}

ZK_DI Fq fq_mul(const Fq& a, const Fq& b) { return fp_mul(a, b); }

ZK_DI Fq fq_inv(const Fq& a) {
  uint32_t e[12];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) e[i] = __builtin_subc(FqParams::MOD[i], i == 0 ? 2u : 0u, br, &br);
  Fq acc = fp_one<FqParams>();
#pragma unroll
  for (int i = 11; i >= 0; i--) {
    for (int k = 31; k >= 0; k--) {
      acc = fq_mul(acc, acc);
      if ((e[i] >> k) & 1) acc = fq_mul(acc, a);
    }
  }
  return acc;
}

// ---------------------------------------------------------------- Fq2 -----
// Fq2 = Fq[u]/(u^2 + 1)  (ark-bls12-381 Fq2Config NONRESIDUE = -1)
struct Fq2 {
  Fq c0, c1;
};
ZK_DI Fq2 fq2_zero() { return {fp_zero<FqParams>(), fp_zero<FqParams>()}; }
ZK_DI Fq2 fq2_one() { return {fp_one<FqParams>(), fp_zero<FqParams>()}; }
ZK_DI bool fq2_is_zero(const Fq2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
ZK_DI Fq2 fq2_add(const Fq2& a, const Fq2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
ZK_DI Fq2 fq2_sub(const Fq2& a, const Fq2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
ZK_DI Fq2 fq2_neg(const Fq2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
// Schoolbook product with lazy reduction: each output coefficient is ONE
// product-scanning pass over two limb products and one Montgomery
// reduction,
//   c0 = REDC(a0 b0 - a1 b1 + 4p^2),   c1 = REDC(a0 b1 + a1 b0),
// the same 1176 v_mad as Karatsuba's three full products but without its
// five Fq additions / subtractions (12-limb carry chains, each link a VCC
// hazard) and with two packs / final subtractions instead of three.  The
// subtracted products go through v_mad_i64_i32 on negated 28-bit limbs; the
// 4p^2 column offset keeps the total non-negative (a1 b1 < 4 p^2 for inputs
// < 2p), so signed column sums and arithmetic carries give a value < 2p.
template <bool SUB>
ZK_DI Fq fq_redc2(const uint32_t (&x0)[14], const uint32_t (&y0)[14], const uint32_t (&x1)[14],
                  const uint32_t (&y1)[14]) {
  constexpr int M = 14;
  uint32_t m[M], r[M];
  int32_t nx1[M];
#pragma unroll
  for (int i = 0; i < M; i++) nx1[i] = SUB ? -(int32_t)x1[i] : (int32_t)x1[i];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    int64_t acc = carry;
    if (SUB) acc += (int64_t)FqParams::P4SQ28[k];
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (j >= 0 && j < M) {
        acc += (int64_t)((uint64_t)x0[i] * y0[j]);
        acc += (int64_t)nx1[i] * (int64_t)(int32_t)y1[j];
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
    carry = acc >> 28;   // arithmetic: floor division of a possibly negative column
  }
  r[M - 1] = (uint32_t)(carry + (SUB ? (int64_t)FqParams::P4SQ28[2 * M - 1] : 0));
  Fq o;
  pack28<12, M>(r, o.v);
  return fp_reduce_once(o);
}

ZK_DI Fq2 fq2_mul(const Fq2& a, const Fq2& b) {
  uint32_t a0[14], a1[14], b0[14], b1[14];
  unpack28<12, 14>(a.c0.v, a0);
  unpack28<12, 14>(a.c1.v, a1);
  unpack28<12, 14>(b.c0.v, b0);
  unpack28<12, 14>(b.c1.v, b1);
  Fq c0 = fq_redc2<true>(a0, b0, a1, b1);
  __builtin_amdgcn_sched_barrier(0);
  Fq c1 = fq_redc2<false>(a0, b1, a1, b0);
  __builtin_amdgcn_sched_barrier(0);
  return {c0, c1};
}
ZK_DI Fq2 fq2_sqr(const Fq2& a) {
  // (c0 + c1 u)^2 = (c0+c1)(c0-c1) + 2 c0 c1 u
  Fq m = fq_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  __builtin_amdgcn_sched_barrier(0);
  Fq t = fq_mul(a.c0, a.c1);
  __builtin_amdgcn_sched_barrier(0);
  return {m, fp_add(t, t)};
}
ZK_DI Fq2 fq2_inv(const Fq2& a) {
  Fq n = fp_add(fq_mul(a.c0, a.c0), fq_mul(a.c1, a.c1));
  n = fq_inv(n);
  return {fq_mul(a.c0, n), fp_neg(fq_mul(a.c1, n))};
}

// a*b - c*d with ONE Montgomery reduction (fq_redc2's signed columns and
// 4p^2 offset): 588 v_mad instead of 784 for two products and a subtraction.
ZK_DI Fq fq_mul_sub(const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
  uint32_t xa[14], xb[14], xc[14], xd[14];
  unpack28<12, 14>(a.v, xa);
  unpack28<12, 14>(b.v, xb);
  unpack28<12, 14>(c.v, xc);
  unpack28<12, 14>(d.v, xd);
  return fq_redc2<true>(xa, xb, xc, xd);
}

// Generic field-op shims so curve code is written once for Fq and Fq2.
ZK_DI Fq f_mul_sub(const Fq& a, const Fq& b, const Fq& c, const Fq& d) { return fq_mul_sub(a, b, c, d); }
ZK_DI Fq f_add(const Fq& a, const Fq& b) { return fp_add(a, b); }
ZK_DI Fq f_sub(const Fq& a, const Fq& b) { return fp_sub(a, b); }
ZK_DI Fq f_mul(const Fq& a, const Fq& b) { return fq_mul(a, b); }
ZK_DI Fq f_sqr(const Fq& a) { return fp_sqr(a); }
ZK_DI Fq f_neg(const Fq& a) { return fp_neg(a); }
ZK_DI bool f_is_zero(const Fq& a) { return fp_is_zero(a); }
ZK_DI Fq f_inv(const Fq& a) { return fq_inv(a); }
ZK_DI void f_set_zero(Fq& a) { a = fp_zero<FqParams>(); }
ZK_DI void f_set_one(Fq& a) { a = fp_one<FqParams>(); }

// ---------------------------------------------------- lane-pair Fq2 ------
// Fq2h: one Fq2 element spread over the two lanes of an aligned lane pair
// (lane 2j holds c0, lane 2j+1 holds c1).  Every Fq2 operation is split so
// both lanes do the same instruction stream on half the data: a product is
// one coefficient per lane,
//   lane 0: c0 = REDC(a0 b0 - a1 b1 + 4p^2)   lane 1: c1 = REDC(a1 b0 + a0 b1 + 4p^2)
// (4p^2 = 0 mod p, so lane 1 may add it too: one code path), with the
// partner's 28-bit limbs fetched by DPP quad_perm [1,0,3,2].  A G2 XYZZ point
// is then 48 VGPRs per lane instead of 96, so the G2 bucket accumulation fits
// two waves per SIMD instead of one.  Both lanes of a pair must be active and
// take the same branches (every predicate below is combined over the pair).
struct Fq2h {
  Fq v;
};
ZK_DI uint32_t pair_swap(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
}
ZK_DI uint32_t pair_half() { return threadIdx.x & 1u; }
// The pair's c0 / c1 on both lanes (DPP quad_perm [0,0,2,2] / [1,1,3,3]):
// the b operands of the products below, one move each instead of a swap and
// two per-lane selects (ZK_G2_BCAST=0: A/B build with the swap form)
#ifndef ZK_G2_BCAST
#define ZK_G2_BCAST 1
#endif
ZK_DI uint32_t pair_even(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xf, 0xf, false);   // quad_perm [0,0,2,2]
}
ZK_DI uint32_t pair_odd(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xf, 0xf, false);   // quad_perm [1,1,3,3]
}
ZK_DI Fq pair_swap(const Fq& a) {
  Fq o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.v[i] = pair_swap(a.v[i]);
  return o;
}
ZK_DI Fq2h f_add(const Fq2h& a, const Fq2h& b) { return {fp_add(a.v, b.v)}; }
ZK_DI Fq2h f_sub(const Fq2h& a, const Fq2h& b) { return {fp_sub(a.v, b.v)}; }
ZK_DI Fq2h f_neg(const Fq2h& a) { return {fp_neg(a.v)}; }
ZK_DI bool f_is_zero(const Fq2h& a) {
  const uint32_t z = fp_is_zero(a.v) ? 1u : 0u;
  return (z & pair_swap(z)) != 0;
}
ZK_DI void f_set_zero(Fq2h& a) { a.v = fp_zero<FqParams>(); }
ZK_DI void f_set_one(Fq2h& a) { a.v = pair_half() ? fp_zero<FqParams>() : fp_one<FqParams>(); }
ZK_DI Fq2h f_mul(const Fq2h& a, const Fq2h& b) {
  constexpr int M = 14;
  const bool h = pair_half();
  uint32_t xa[M], xb[M];
  unpack28<12, M>(a.v.v, xa);
  unpack28<12, M>(b.v.v, xb);
  // lane 0: a0*b0 - a1*b1;  lane 1: a1*b0 + a0*b1  (own a first, partner a second)
  uint32_t y0[M], y1[M];
  int32_t nx1[M];
  const uint32_t neg = h ? 0u : ~0u;
#pragma unroll
  for (int i = 0; i < M; i++) {
    const uint32_t pa = pair_swap(xa[i]);
    nx1[i] = (int32_t)((pa ^ neg) - neg);
    if constexpr (ZK_G2_BCAST) {   // lane 0: (b0, b1), lane 1: (b0, b1) = (partner, own)
      y0[i] = pair_even(xb[i]);
      y1[i] = pair_odd(xb[i]);
    } else {
      const uint32_t pb = pair_swap(xb[i]);
      y0[i] = h ? pb : xb[i];
      y1[i] = h ? xb[i] : pb;
    }
  }
  uint32_t m[M], r[M];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    int64_t acc = carry + (int64_t)FqParams::P4SQ28[k];
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (j >= 0 && j < M) {
        acc += (int64_t)((uint64_t)xa[i] * y0[j]);
        acc += (int64_t)nx1[i] * (int64_t)(int32_t)y1[j];
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
    carry = acc >> 28;
  }
  r[M - 1] = (uint32_t)(carry + (int64_t)FqParams::P4SQ28[2 * M - 1]);
  Fq o;
  pack28<12, M>(r, o.v);
  return {fp_reduce_once(o)};
}
#ifndef ZK_G2_SQR_BCAST
#define ZK_G2_SQR_BCAST 1
#endif
ZK_DI Fq2h f_sqr(const Fq2h& a) {
  const bool h = pair_half();
  if constexpr (ZK_G2_SQR_BCAST) {
    // lane 0: (a0 + a1)(a0 - a1);  lane 1: (a0 + a0) a1 -- the doubling moves
    // into the operand, so no doubled copy and no output select:
    //   x = partner (lane 0: a1, lane 1: a0), e = a0 on both lanes,
    //   u = e + x, w = own - (lane 0 ? x : 0)
    const Fq x = pair_swap(a.v);
    Fq e, xm;
    const uint32_t keep = h ? 0u : ~0u;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      e.v[i] = pair_even(a.v.v[i]);
      xm.v[i] = x.v[i] & keep;
    }
    return {fq_mul(fp_add(e, x), fp_sub(a.v, xm))};
  }
  // lane 0: (a0 + a1)(a0 - a1);  lane 1: 2 a1 a0
  const Fq p = pair_swap(a.v);
  const Fq s = fp_add(a.v, p), d = fp_sub(a.v, p);
  Fq u, w;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    u.v[i] = h ? p.v[i] : s.v[i];
    w.v[i] = h ? a.v.v[i] : d.v[i];
  }
  const Fq t = fq_mul(u, w);
  const Fq t2 = fp_add(t, t);
  Fq o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.v[i] = h ? t2.v[i] : t.v[i];
  return {o};
}

// a*b - c*d per lane with ONE reduction: four limb products per column,
//   lane 0: a0 b0 - a1 b1 - c0 d0 + c1 d1,  lane 1: a1 b0 + a0 b1 - c1 d0 - c0 d1,
// offset by 4p^2 (the sum is > -2p^2 for inputs < p).
ZK_DI Fq2h f_mul_sub(const Fq2h& a, const Fq2h& b, const Fq2h& c, const Fq2h& d) {
  constexpr int M = 14;
  const bool h = pair_half();
  uint32_t xa[M], xb[M], xc[M], xd[M];
  unpack28<12, M>(a.v.v, xa);
  unpack28<12, M>(b.v.v, xb);
  unpack28<12, M>(c.v.v, xc);
  unpack28<12, M>(d.v.v, xd);
  uint32_t y0[M], y1[M], z0[M], z1[M];
  int32_t na1[M], nc0[M], nc1[M];
  const uint32_t neg = h ? 0u : ~0u;
#pragma unroll
  for (int i = 0; i < M; i++) {
    const uint32_t pa = pair_swap(xa[i]), pc = pair_swap(xc[i]);
    na1[i] = (int32_t)((pa ^ neg) - neg);        // lane 0: -a1, lane 1: +a0
    nc0[i] = -(int32_t)xc[i];                    // -c_own
    nc1[i] = (int32_t)((pc ^ ~neg) - ~neg);      // lane 0: +c1, lane 1: -c0
    if constexpr (ZK_G2_BCAST) {
      y0[i] = pair_even(xb[i]);
      y1[i] = pair_odd(xb[i]);
      z0[i] = pair_even(xd[i]);
      z1[i] = pair_odd(xd[i]);
    } else {
      const uint32_t pb = pair_swap(xb[i]), pd = pair_swap(xd[i]);
      y0[i] = h ? pb : xb[i];
      y1[i] = h ? xb[i] : pb;
      z0[i] = h ? pd : xd[i];
      z1[i] = h ? xd[i] : pd;
    }
  }
  uint32_t m[M], r[M];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * M - 1; k++) {
    int64_t acc = carry + (int64_t)FqParams::P4SQ28[k];
#pragma unroll
    for (int i = 0; i < M; i++) {
      const int j = k - i;
      if (j >= 0 && j < M) {
        acc += (int64_t)((uint64_t)xa[i] * y0[j]);
        acc += (int64_t)na1[i] * (int64_t)(int32_t)y1[j];
        acc += (int64_t)nc0[i] * (int64_t)(int32_t)z0[j];
        acc += (int64_t)nc1[i] * (int64_t)(int32_t)z1[j];
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
    carry = acc >> 28;
  }
  r[M - 1] = (uint32_t)(carry + (int64_t)FqParams::P4SQ28[2 * M - 1]);
  Fq o;
  pack28<12, M>(r, o.v);
  return {fp_reduce_once(o)};
}

ZK_DI Fq2 f_add(const Fq2& a, const Fq2& b) { return fq2_add(a, b); }
ZK_DI Fq2 f_sub(const Fq2& a, const Fq2& b) { return fq2_sub(a, b); }
ZK_DI Fq2 f_mul(const Fq2& a, const Fq2& b) { return fq2_mul(a, b); }
ZK_DI Fq2 f_sqr(const Fq2& a) { return fq2_sqr(a); }
ZK_DI Fq2 f_neg(const Fq2& a) { return fq2_neg(a); }
ZK_DI bool f_is_zero(const Fq2& a) { return fq2_is_zero(a); }
ZK_DI Fq2 f_inv(const Fq2& a) { return fq2_inv(a); }
ZK_DI Fq2 f_mul_sub(const Fq2& a, const Fq2& b, const Fq2& c, const Fq2& d) {
  return fq2_sub(fq2_mul(a, b), fq2_mul(c, d));
}
ZK_DI void f_set_zero(Fq2& a) { a = fq2_zero(); }
ZK_DI void f_set_one(Fq2& a) { a = fq2_one(); }
