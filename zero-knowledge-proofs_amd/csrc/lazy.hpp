// lazy.hpp -- Fq in a redundant signed radix-2^28 form for the bucket
// accumulate (k_msm_accum<G1>).
//
// ff.hpp's fp_mul re-cuts its packed 12 x 32-bit operands into 14 x 28-bit
// limbs, runs the product-scanning Montgomery product, packs the result back
// and subtracts p once: ~110 of its ~500 VALU instructions are that
// unpack / pack / final subtraction, and every fp_add / fp_sub is a 12-link
// carry chain plus a conditional subtraction.  Inside one madd-2008-s the
// packed form is never needed, so here a field element stays as 14 signed
// 32-bit limbs (value = sum v_i 2^(28 i), same Montgomery domain R = 2^392 as
// ff.hpp's Fq):
//   * products take and return limbs (no unpack / pack), the columns are
//     signed (v_mad_i64_i32), so operands may be negative and no output is
//     reduced: for inputs |a|, |b| < 16p the output (T + m p) / 2^392 lies in
//     (-p/8, 9p/8) (|T| / 2^392 < 256 p^2 / 2^392 < p/8, m p < 2^392 p) with
//     limbs 0..12 in [0, 2^28) and a small signed top limb;
//   * additions / subtractions are limb-wise (one v_add / v_sub per limb, no
//     carries); fl_norm propagates carries where a limb could outgrow the
//     column bound below;
//   * a zero test screens limb 0 first: V = k p implies V = k p mod 2^28, so
//     v_0 p^-1 mod 2^28 must be a small k; only then (about 2^-24 of the
//     time) is the value canonicalised and compared.
// Column bound: a product column holds <= 14 limb products and <= 14 m_i p_j
// terms; operands with |limb| <= 2^29 keep it below 2^62.9 (fl_mul_sub:
// 28 products, operands |limb| < 2^28).  Every call site below states its
// operands' limb and value bounds.
// Host-and-device code so tools/lazy_check.hip can verify it on the CPU.
#pragma once
#include <math.h>
#include <stdint.h>

#include "ff.hpp"

#define ZK_HD __host__ __device__ __forceinline__
// scheduling barrier between products on the device (curve.hpp's ZK_SB: keeps
// independent products from overlapping and inflating the live set)
#if defined(__HIP_DEVICE_COMPILE__)
#define ZK_LSB() __builtin_amdgcn_sched_barrier(0)
#else
#define ZK_LSB()
#endif

namespace zk {

constexpr int FL_N = 14;
constexpr int32_t FL_MASK = (1 << 28) - 1;
constexpr uint32_t FL_PINV = 0x30003u;   // p^-1 mod 2^28

struct Fl {
  int32_t v[FL_N];
};
struct FlA {   // affine
  Fl x, y;
};
struct FlX {   // XYZZ
  Fl X, Y, ZZ, ZZZ;
};

// packed canonical (12 x 32) -> limbs in [0, 2^28)
ZK_HD Fl fl_from_fq(const Fq& a) {
  Fl r;
#pragma unroll
  for (int i = 0; i < FL_N; i++) {
    const int bit = 28 * i, w = bit >> 5, s = bit & 31;
    const uint64_t lo = w < 12 ? a.v[w] : 0u, hi = w + 1 < 12 ? a.v[w + 1] : 0u;
    r.v[i] = (int32_t)((uint32_t)((hi << 32 | lo) >> s) & (uint32_t)FL_MASK);
  }
  return r;
}
ZK_HD Fl fl_zero() {
  Fl r;
#pragma unroll
  for (int i = 0; i < FL_N; i++) r.v[i] = 0;
  return r;
}
ZK_HD Fl fl_one() {   // 2^392 mod p, the device Montgomery one
  Fq o;
#pragma unroll
  for (int i = 0; i < 12; i++) o.v[i] = FqParams::ONE[i];
  return fl_from_fq(o);
}
ZK_HD Fl fl_add(const Fl& a, const Fl& b) {
  Fl r;
#pragma unroll
  for (int i = 0; i < FL_N; i++) r.v[i] = (int32_t)((uint32_t)a.v[i] + (uint32_t)b.v[i]);
  return r;
}
ZK_HD Fl fl_sub(const Fl& a, const Fl& b) {
  Fl r;
#pragma unroll
  for (int i = 0; i < FL_N; i++) r.v[i] = (int32_t)((uint32_t)a.v[i] - (uint32_t)b.v[i]);
  return r;
}
ZK_HD Fl fl_neg(const Fl& a) { return fl_sub(fl_zero(), a); }
// carry propagation: limbs 0..12 into [0, 2^28), the sign in limb 13
ZK_HD Fl fl_norm(const Fl& a) {
  Fl r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < FL_N - 1; i++) {
    const int32_t t = a.v[i] + c;
    r.v[i] = t & FL_MASK;
    c = t >> 28;   // arithmetic
  }
  r.v[FL_N - 1] = a.v[FL_N - 1] + c;
  return r;
}
ZK_HD bool fl_is_exact_zero(const Fl& a) {
  int32_t x = 0;
#pragma unroll
  for (int i = 0; i < FL_N; i++) x |= a.v[i];
  return x == 0;
}

// Montgomery product a b / 2^392 (signed product scanning, interleaved REDC).
// Operands |limb| <= 2^29, |value| < 16p: result limbs 0..12 in [0, 2^28),
// value in (-p/8, 9p/8).
ZK_HD Fl fl_mul(const Fl& a, const Fl& b) {
  uint32_t m[FL_N];
  Fl r;
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * FL_N - 1; k++) {
    int64_t acc = carry;
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (j >= 0 && j < FL_N) acc += (int64_t)a.v[i] * (int64_t)b.v[j];
    }
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < FL_N) acc += (int64_t)((uint64_t)m[i] * FqParams::MOD28[j]);
    }
    if (k < FL_N) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & (uint32_t)FL_MASK;
      acc += (int64_t)((uint64_t)m[k] * FqParams::MOD28[0]);
    } else {
      r.v[k - FL_N] = (int32_t)((uint32_t)acc & (uint32_t)FL_MASK);
    }
    carry = acc >> 28;
  }
  r.v[FL_N - 1] = (int32_t)carry;
  return r;
}
// a^2: cross products once, doubled (105 instead of 196 limb products)
ZK_HD Fl fl_sqr(const Fl& a) {
  uint32_t m[FL_N];
  Fl r;
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * FL_N - 1; k++) {
    int64_t cross = 0;
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (i < j && j < FL_N) cross += (int64_t)a.v[i] * (int64_t)a.v[j];
    }
    int64_t acc = carry + 2 * cross;
    if ((k & 1) == 0 && k / 2 < FL_N) acc += (int64_t)a.v[k / 2] * (int64_t)a.v[k / 2];
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < FL_N) acc += (int64_t)((uint64_t)m[i] * FqParams::MOD28[j]);
    }
    if (k < FL_N) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & (uint32_t)FL_MASK;
      acc += (int64_t)((uint64_t)m[k] * FqParams::MOD28[0]);
    } else {
      r.v[k - FL_N] = (int32_t)((uint32_t)acc & (uint32_t)FL_MASK);
    }
    carry = acc >> 28;
  }
  r.v[FL_N - 1] = (int32_t)carry;
  return r;
}
// (a b - c d) / 2^392 with one reduction.  28 products per column: at most
// one of a, b above |limb| 2^28 (then <= 2^29), c, d below it; |value| < 16p
// (|ab| + |cd| < 256 p^2 keeps the result in (-p/8, 9p/8) as fl_mul's).
ZK_HD Fl fl_mul_sub(const Fl& a, const Fl& b, const Fl& c, const Fl& d) {
  uint32_t m[FL_N];
  Fl r;
  int32_t nc[FL_N];
#pragma unroll
  for (int i = 0; i < FL_N; i++) nc[i] = -c.v[i];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * FL_N - 1; k++) {
    int64_t acc = carry;
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (j >= 0 && j < FL_N) {
        acc += (int64_t)a.v[i] * (int64_t)b.v[j];
        acc += (int64_t)nc[i] * (int64_t)d.v[j];
      }
    }
#pragma unroll
    for (int i = 0; i < FL_N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < FL_N) acc += (int64_t)((uint64_t)m[i] * FqParams::MOD28[j]);
    }
    if (k < FL_N) {
      m[k] = ((uint32_t)acc * FqParams::INV28) & (uint32_t)FL_MASK;
      acc += (int64_t)((uint64_t)m[k] * FqParams::MOD28[0]);
    } else {
      r.v[k - FL_N] = (int32_t)((uint32_t)acc & (uint32_t)FL_MASK);
    }
    carry = acc >> 28;
  }
  r.v[FL_N - 1] = (int32_t)carry;
  return r;
}

// Canonical packed form [0, p) of a value |V| < 7p: k = floor(V / p)
// estimated from the top 56 bits (off by at most one), V - k p normalised,
// then one conditional add or subtract of p.
ZK_HD Fq fl_to_fq(const Fl& a) {
  Fl n = fl_norm(a);
  const int64_t top = (int64_t)n.v[FL_N - 1] * (1ll << 28) + n.v[FL_N - 2];   // V / 2^336, floored
  constexpr double PT = (double)((uint64_t)FqParams::MOD28[13] << 28 | FqParams::MOD28[12]);
  const int32_t k = (int32_t)floor((double)top / PT);
#pragma unroll
  for (int i = 0; i < FL_N; i++) n.v[i] -= k * (int32_t)FqParams::MOD28[i];
  n = fl_norm(n);   // V - k p in [-p, 2p)
  if (n.v[FL_N - 1] < 0) {
#pragma unroll
    for (int i = 0; i < FL_N; i++) n.v[i] += (int32_t)FqParams::MOD28[i];
    n = fl_norm(n);
  }
  // pack 14 x 28 -> 12 x 32 (value < 2p < 2^382), then subtract p if >= p
  Fq o;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    const int bit = 32 * w, i = bit / 28, s = bit - 28 * i;
    uint32_t v = (uint32_t)n.v[i] >> s;
    if (i + 1 < FL_N && 28 - s < 32) v |= (uint32_t)n.v[i + 1] << (28 - s);
    if (56 - s < 32 && i + 2 < FL_N) v |= (uint32_t)n.v[i + 2] << (56 - s);
    o.v[w] = v;
  }
  uint32_t s[12];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint64_t d = (uint64_t)o.v[i] - FqParams::MOD[i] - br;
    s[i] = (uint32_t)d;
    br = (d >> 32) & 1;
  }
  if (!br)
#pragma unroll
    for (int i = 0; i < 12; i++) o.v[i] = s[i];
  return o;
}
ZK_HD bool fl_is_zero_slow(const Fl& a) {
  const Fq c = fl_to_fq(a);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) x |= c.v[i];
  return x == 0;
}
// V = 0 mod p for |V| < 7p?  Limb 0 screens: V = k p forces
// v_0 p^-1 = k (mod 2^28) with |k| <= 8.
ZK_HD bool fl_maybe_zero(const Fl& a) {
  const uint32_t k = ((uint32_t)a.v[0] * FL_PINV + 8u) & (uint32_t)FL_MASK;
  return k <= 16u;
}
ZK_HD bool fl_is_zero(const Fl& a) { return fl_maybe_zero(a) && fl_is_zero_slow(a); }

ZK_HD void flx_set_inf(FlX& p) {
  p.X = fl_zero(); p.Y = fl_one(); p.ZZ = fl_zero(); p.ZZZ = fl_zero();
}
ZK_HD bool flx_is_inf(const FlX& p) { return fl_is_exact_zero(p.ZZ); }   // only set_inf makes ZZ = 0

// mdbl-2008-s-1: 2a, a affine (limbs in (-2^28, 2^28), |value| < p)
ZK_HD FlX fla_dbl(const FlA& a) {
  const Fl U = fl_add(a.y, a.y);   // |limb| < 2^29
  const Fl V = fl_sqr(U);
  ZK_LSB();
  const Fl W = fl_mul(U, V);
  ZK_LSB();
  const Fl S = fl_mul(a.x, V);
  ZK_LSB();
  const Fl X2 = fl_sqr(a.x);
  ZK_LSB();
  const Fl M = fl_norm(fl_add(fl_add(X2, X2), X2));   // (-3p/8, 27p/8)
  FlX r;
  r.X = fl_norm(fl_sub(fl_sqr(M), fl_add(S, S)));   // (-19p/8, 11p/8)
  ZK_LSB();
  r.Y = fl_mul_sub(M, fl_sub(S, r.X), W, a.y);
  ZK_LSB();
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + a (a affine, not infinity; limbs in (-2^28, 2^28), value
// in (-p, p)).  Invariants of p, true of every output: X normalised with
// value in (-7p/2, 3p/2); Y, ZZ, ZZZ with |limb| < 2^28 and value in
// (-p, 9p/8) (product outputs, or a.x / a.y / one after infinity).
ZK_HD FlX flx_madd(const FlX& p, const FlA& a) {
  if (flx_is_inf(p)) return {a.x, a.y, fl_one(), fl_one()};
  const Fl U2 = fl_mul(a.x, p.ZZ);
  ZK_LSB();
  const Fl S2 = fl_mul(a.y, p.ZZZ);
  ZK_LSB();
  const Fl P = fl_sub(U2, p.X);   // |limb| < 2^29, (-13p/8, 37p/8)
  const Fl R = fl_sub(S2, p.Y);   // |limb| < 2^29, (-9p/8, 17p/8)
  if (fl_maybe_zero(P) && fl_is_zero_slow(P)) {
    if (fl_is_zero_slow(R)) return fla_dbl(a);
    FlX r;
    flx_set_inf(r);
    return r;
  }
  // ZZ3 and ZZZ3 first: p.ZZ, p.ZZZ and PP die before X3 / Y3 (live set)
  const Fl PP = fl_sqr(P);
  ZK_LSB();
  const Fl PPP = fl_mul(P, PP);
  ZK_LSB();
  FlX r;
  r.ZZ = fl_mul(p.ZZ, PP);
  ZK_LSB();
  r.ZZZ = fl_mul(p.ZZZ, PPP);
  ZK_LSB();
  const Fl Q = fl_mul(p.X, PP);
  ZK_LSB();
  r.X = fl_norm(fl_sub(fl_sub(fl_sqr(R), PPP), fl_add(Q, Q)));   // (-7p/2, 11p/8)
  ZK_LSB();
  r.Y = fl_mul_sub(R, fl_sub(Q, r.X), p.Y, PPP);
  ZK_LSB();
  return r;
}

}  // namespace zk
