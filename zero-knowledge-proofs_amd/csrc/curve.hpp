// curve.hpp -- BLS12-381 G1 (over Fq) / G2 (over Fq2) group law on device.
//
// The reference's group is ark-ec's short-Weierstrass Projective (Jacobian)
// behind G1Projective / G2Projective (crates/groth16-core/src/lib.rs:16,
// 275-300).  Group elements are unique, so any coordinate system yields the
// same affine result; on device we use extended Jacobian "XYZZ" coordinates
// (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2) because the bucket-accumulate step is a
// stream of XYZZ += affine additions (madd-2008-s: 8M + 2S, no inversion)
// and the EFD formulas handle the degenerate cases with two branches.
//
// Device affine layout: Montgomery x then y, (0,0) = point at infinity
// (0 != 4 so (0,0) is off-curve for both groups).
#pragma once
#include <type_traits>

#include "ff.hpp"

// Scheduling barrier between field operations: keeps the scheduler from
// overlapping independent multiplies (each holds ~60 VGPRs of 28-bit limbs),
// which otherwise pushes G2 formulas past 512 VGPRs into scratch.
#define ZK_SB() __builtin_amdgcn_sched_barrier(0)

template <class F>
struct Affine {
  F x, y;
};
template <class F>
struct XYZZ {
  F X, Y, ZZ, ZZZ;
};

using G1A = Affine<Fq>;
using G2A = Affine<Fq2>;
using G1X = XYZZ<Fq>;
using G2X = XYZZ<Fq2>;

template <class F>
ZK_DI bool aff_is_inf(const Affine<F>& a) {
  return f_is_zero(a.x) && f_is_zero(a.y);
}
template <class F>
ZK_DI void xyzz_set_inf(XYZZ<F>& p) {
  f_set_zero(p.X); f_set_one(p.Y); f_set_zero(p.ZZ); f_set_zero(p.ZZZ);
}
template <class F>
ZK_DI bool xyzz_is_inf(const XYZZ<F>& p) { return f_is_zero(p.ZZ); }

template <class F>
ZK_DI XYZZ<F> xyzz_from_aff(const Affine<F>& a) {
  XYZZ<F> p;
  if (aff_is_inf(a)) { xyzz_set_inf(p); return p; }
  p.X = a.x; p.Y = a.y; f_set_one(p.ZZ); f_set_one(p.ZZZ);
  return p;
}

// dbl-2008-s-1 (a = 0)
template <class F>
ZK_DI XYZZ<F> xyzz_dbl(const XYZZ<F>& p) {
  F U = f_add(p.Y, p.Y);
  F V = f_sqr(U);
  ZK_SB();
  F W = f_mul(U, V);
  ZK_SB();
  F S = f_mul(p.X, V);
  ZK_SB();
  F X2 = f_sqr(p.X);
  ZK_SB();
  F M = f_add(f_add(X2, X2), X2);
  XYZZ<F> r;
  r.X = f_sub(f_sqr(M), f_add(S, S));
  ZK_SB();
  r.Y = f_sub(f_mul(M, f_sub(S, r.X)), f_mul(W, p.Y));
  ZK_SB();
  r.ZZ = f_mul(V, p.ZZ);
  ZK_SB();
  r.ZZZ = f_mul(W, p.ZZZ);
  ZK_SB();
  return r;   // p at infinity (ZZ = 0) stays at infinity
}

// Out-of-line doubling for the (rare) p == q branch of xyzz_add: inlined, its
// live set adds to the add's and pushes G2 into scratch.
template <class F>
__device__ __noinline__ XYZZ<F> xyzz_dbl_call(const XYZZ<F>& p) { return xyzz_dbl(p); }

// mdbl-2008-s-1: 2*a for affine a (not infinity)
template <class F>
ZK_DI XYZZ<F> aff_dbl(const Affine<F>& a) {
  F U = f_add(a.y, a.y);
  F V = f_sqr(U);
  ZK_SB();
  F W = f_mul(U, V);
  ZK_SB();
  F S = f_mul(a.x, V);
  ZK_SB();
  F X2 = f_sqr(a.x);
  ZK_SB();
  F M = f_add(f_add(X2, X2), X2);
  XYZZ<F> r;
  r.X = f_sub(f_sqr(M), f_add(S, S));
  ZK_SB();
  r.Y = f_sub(f_mul(M, f_sub(S, r.X)), f_mul(W, a.y));
  ZK_SB();
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + a, a affine (a must not be infinity)
template <class F>
ZK_DI XYZZ<F> xyzz_madd(const XYZZ<F>& p, const Affine<F>& a) {
  if (xyzz_is_inf(p)) return xyzz_from_aff(a);
  F U2 = f_mul(a.x, p.ZZ);
  ZK_SB();
  F S2 = f_mul(a.y, p.ZZZ);
  ZK_SB();
  F P = f_sub(U2, p.X);
  F R = f_sub(S2, p.Y);
  if (f_is_zero(P)) {
    if (f_is_zero(R)) return aff_dbl(a);
    XYZZ<F> r; xyzz_set_inf(r); return r;
  }
  F PP = f_sqr(P);
  ZK_SB();
  F PPP = f_mul(P, PP);
  ZK_SB();
  F Q = f_mul(p.X, PP);
  ZK_SB();
  XYZZ<F> r;
  r.X = f_sub(f_sub(f_sqr(R), PPP), f_add(Q, Q));
  ZK_SB();
  r.Y = f_mul_sub(R, f_sub(Q, r.X), p.Y, PPP);
  ZK_SB();
  r.ZZ = f_mul(p.ZZ, PP);
  ZK_SB();
  r.ZZZ = f_mul(p.ZZZ, PPP);
  ZK_SB();
  return r;
}

// add-2008-s: p + q.  Operations are ordered so that each input coordinate
// dies as early as possible (G2 points are 96 VGPRs each; the textbook order
// keeps both points and four products live at once and spills).
template <class F, bool SB>
ZK_DI XYZZ<F> xyzz_add_impl(const XYZZ<F>& p, const XYZZ<F>& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  F U1 = f_mul(p.X, q.ZZ);
  if constexpr (SB) ZK_SB();
  F P = f_sub(f_mul(q.X, p.ZZ), U1);
  if constexpr (SB) ZK_SB();
  F S1 = f_mul(p.Y, q.ZZZ);
  if constexpr (SB) ZK_SB();
  F R = f_sub(f_mul(q.Y, p.ZZZ), S1);
  if constexpr (SB) ZK_SB();
  if (f_is_zero(P)) {
    if (f_is_zero(R)) {
      // inline for the G1 reductions (no call frame: their kernels then need
      // no scratch); out of line elsewhere (live-set pressure)
      if constexpr (!SB && std::is_same<F, Fq>::value) return xyzz_dbl(p);
      else return xyzz_dbl_call(p);
    }
    XYZZ<F> r; xyzz_set_inf(r); return r;
  }
  XYZZ<F> r;
  F PP = f_sqr(P);
  if constexpr (SB) ZK_SB();
  r.ZZ = f_mul(p.ZZ, q.ZZ);
  if constexpr (SB) ZK_SB();
  r.ZZ = f_mul(r.ZZ, PP);
  if constexpr (SB) ZK_SB();
  F PPP = f_mul(P, PP);
  if constexpr (SB) ZK_SB();
  r.ZZZ = f_mul(p.ZZZ, q.ZZZ);
  if constexpr (SB) ZK_SB();
  r.ZZZ = f_mul(r.ZZZ, PPP);
  if constexpr (SB) ZK_SB();
  F Q = f_mul(U1, PP);
  if constexpr (SB) ZK_SB();
  r.X = f_sub(f_sub(f_sqr(R), PPP), f_add(Q, Q));
  if constexpr (SB) ZK_SB();
  r.Y = f_mul_sub(R, f_sub(Q, r.X), S1, PPP);
  if constexpr (SB) ZK_SB();
  return r;
}
template <class F>
ZK_DI XYZZ<F> xyzz_add(const XYZZ<F>& p, const XYZZ<F>& q) {
  return xyzz_add_impl<F, true>(p, q);
}
// The same add with the scheduler free to overlap its independent products
// (U1 / U2 / S1 / S2, the ZZ and ZZZ chains): for the latency-bound G1
// reduction kernels (fixup, row/column sums) that run one or two waves per
// SIMD, where the serial product chain, not the VGPR count, sets the time.
template <class F>
ZK_DI XYZZ<F> xyzz_add_ilp(const XYZZ<F>& p, const XYZZ<F>& q) {
  return xyzz_add_impl<F, false>(p, q);
}

// ---- lane-quad cooperative add (latency-bound reductions) --------------
// In the bucket-reduction trees a few hundred sums run at once, one or two
// waves per SIMD, so an add costs its full instruction latency (~14 products
// issued back to back).  Here the four lanes of a quad hold the same p and q
// and split each stage's independent products: add-2008-s is 4 stages of
// <= 4 products (U1 U2 S1 S2 | PP RR ZZ1ZZ2 ZZZ1ZZZ2 | PPP Q ZZ3 | ZZZ3 S1PPP
// R(Q-X3)), each lane computes one and the results are broadcast inside the
// quad by DPP moves.  Every lane of a quad must be active and hold the same
// operands (then every branch below is uniform within the quad).
template <int K, class F>
ZK_DI F quad_bcast(const F& v) {
  constexpr int NW = sizeof(F) / 4;
  F o;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* d = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int k = 0; k < NW; k++)
    d[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)s[k], K * 0x55, 0xf, 0xf, false);   // quad_perm [K,K,K,K]
  return o;
}
template <class F>
ZK_DI F quad_sel(const F& a0, const F& a1, const F& a2, const F& a3, uint32_t qi) {
  constexpr int NW = sizeof(F) / 4;
  F o;
  const uint32_t* s0 = reinterpret_cast<const uint32_t*>(&a0);
  const uint32_t* s1 = reinterpret_cast<const uint32_t*>(&a1);
  const uint32_t* s2 = reinterpret_cast<const uint32_t*>(&a2);
  const uint32_t* s3 = reinterpret_cast<const uint32_t*>(&a3);
  uint32_t* d = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int k = 0; k < NW; k++) {
    const uint32_t lo = (qi & 1) ? s1[k] : s0[k];
    const uint32_t hi = (qi & 1) ? s3[k] : s2[k];
    d[k] = (qi & 2) ? hi : lo;
  }
  return o;
}

template <class F>
ZK_DI XYZZ<F> xyzz_add_quad(const XYZZ<F>& p, const XYZZ<F>& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  const uint32_t qi = threadIdx.x & 3;
  F m = f_mul(quad_sel(p.X, q.X, p.Y, q.Y, qi), quad_sel(q.ZZ, p.ZZ, q.ZZZ, p.ZZZ, qi));
  ZK_SB();
  const F U1 = quad_bcast<0>(m), S1 = quad_bcast<2>(m);
  const F P = f_sub(quad_bcast<1>(m), U1);
  const F R = f_sub(quad_bcast<3>(m), S1);
  if (f_is_zero(P)) {
    if (f_is_zero(R)) return xyzz_dbl_call(p);
    XYZZ<F> r; xyzz_set_inf(r); return r;
  }
  m = f_mul(quad_sel(P, R, p.ZZ, p.ZZZ, qi), quad_sel(P, R, q.ZZ, q.ZZZ, qi));
  ZK_SB();
  const F PP = quad_bcast<0>(m), RR = quad_bcast<1>(m), ZZ12 = quad_bcast<2>(m), ZZZ12 = quad_bcast<3>(m);
  m = f_mul(quad_sel(P, U1, ZZ12, ZZ12, qi), PP);
  ZK_SB();
  XYZZ<F> r;
  const F PPP = quad_bcast<0>(m), Q = quad_bcast<1>(m);
  r.ZZ = quad_bcast<2>(m);
  r.X = f_sub(f_sub(RR, PPP), f_add(Q, Q));
  const F QX = f_sub(Q, r.X);
  m = f_mul(quad_sel(ZZZ12, S1, R, R, qi), quad_sel(PPP, PPP, QX, QX, qi));
  ZK_SB();
  r.ZZZ = quad_bcast<0>(m);
  r.Y = f_sub(quad_bcast<2>(m), quad_bcast<1>(m));
  return r;
}

// ---- lane-duo G2 add (latency-bound G2 reductions) ----------------------
// Four lanes = two lane pairs (units u = 0, 1) hold the same p and q (each
// lane its Fq2 half, ff.hpp Fq2h) and split every stage's Fq2 products: unit
// u computes one product of each independent pair, the two interleaved (no
// scheduling barriers), and the results are broadcast to both units by DPP
// quad_perm [2K, 2K+1, 2K, 2K+1].  add-2008-s in 4 stages of two products
// per lane (U1|U2 + S1|S2, PP|RR + ZZ12|ZZZ12, PPP|Q + ZZ3, ZZZ3|R(Q-X3) +
// S1 PPP) instead of the lane pair's 14 products.  All four lanes must be
// active and hold the same operands.
template <int K>
ZK_DI Fq2h duo_bcast(const Fq2h& v) {
  Fq2h o;
#pragma unroll
  for (int k = 0; k < 12; k++)
    o.v.v[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.v.v[k], K ? 0xEE : 0x44, 0xf, 0xf, false);
  return o;
}
ZK_DI Fq2h duo_sel(const Fq2h& a0, const Fq2h& a1, uint32_t u) {
  Fq2h o;
#pragma unroll
  for (int k = 0; k < 12; k++) o.v.v[k] = u ? a1.v.v[k] : a0.v.v[k];
  return o;
}
ZK_DI XYZZ<Fq2h> xyzz_add_duo(const XYZZ<Fq2h>& p, const XYZZ<Fq2h>& q) {
  if (xyzz_is_inf(p)) return q;
  if (xyzz_is_inf(q)) return p;
  const uint32_t u = (threadIdx.x >> 1) & 1;
  Fq2h ma = f_mul(duo_sel(p.X, q.X, u), duo_sel(q.ZZ, p.ZZ, u));     // U1 | U2
  Fq2h mb = f_mul(duo_sel(p.Y, q.Y, u), duo_sel(q.ZZZ, p.ZZZ, u));   // S1 | S2
  const Fq2h U1 = duo_bcast<0>(ma), S1 = duo_bcast<0>(mb);
  const Fq2h P = f_sub(duo_bcast<1>(ma), U1), R = f_sub(duo_bcast<1>(mb), S1);
  if (f_is_zero(P)) {
    if (f_is_zero(R)) return xyzz_dbl_call(p);
    XYZZ<Fq2h> r; xyzz_set_inf(r); return r;
  }
  ma = f_sqr(duo_sel(P, R, u));                                          // PP | RR
  mb = f_mul(duo_sel(p.ZZ, p.ZZZ, u), duo_sel(q.ZZ, q.ZZZ, u));        // ZZ12 | ZZZ12
  const Fq2h PP = duo_bcast<0>(ma), RR = duo_bcast<1>(ma);
  const Fq2h ZZ12 = duo_bcast<0>(mb), ZZZ12 = duo_bcast<1>(mb);
  ma = f_mul(duo_sel(P, U1, u), PP);                                     // PPP | Q
  mb = f_mul(ZZ12, PP);                                                  // ZZ3 (both units)
  const Fq2h PPP = duo_bcast<0>(ma), Q = duo_bcast<1>(ma);
  XYZZ<Fq2h> r;
  r.ZZ = mb;
  r.X = f_sub(f_sub(RR, PPP), f_add(Q, Q));
  ma = f_mul(duo_sel(ZZZ12, R, u), duo_sel(PPP, f_sub(Q, r.X), u));    // ZZZ3 | R (Q - X3)
  mb = f_mul(S1, PPP);                                                   // S1 PPP (both units)
  r.ZZZ = duo_bcast<0>(ma);
  r.Y = f_sub(duo_bcast<1>(ma), mb);
  return r;
}

template <class F>
ZK_DI Affine<F> aff_neg(const Affine<F>& a) { return {a.x, f_neg(a.y)}; }

