// host_pairing.hpp -- BLS12-381 pairing, square roots and point validation on
// the host, for the verifier (crates/groth16-core/src/lib.rs:308-432) and for
// compressed-point decoding (ark-serialize CanonicalDeserialize, core:28).
//
// Not on the prove hot path: one verification is 4 Miller loops and one
// final exponentiation, strictly sequential field arithmetic, so it runs on
// a host core (host_ec.hpp's 64-bit-limb Montgomery Fq / Fq2).
//
// Tower: Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi) with xi = 1 + u,
// Fq12 = Fq6[w]/(w^2 - v).  G2 lives on the M-type twist
// E': y^2 = x^3 + 4 xi, untwisted by psi(x', y') = (x' w^-2, y' w^-3).
// The pairing is the optimal ate pairing with loop parameter x =
// -0xd201000000010000; the final exponentiation is a plain
// square-and-multiply by (p^12 - 1)/r (constants.hpp) -- slow (tens of ms)
// but with no Frobenius tables to get wrong.  Only "product of pairings == 1"
// is observable (Bls12_381::multi_pairing(..).is_zero(), core:352-354), so
// any bilinear non-degenerate pairing gives the reference's verdicts.
#pragma once
#include <vector>

#include "host_ec.hpp"

namespace zk {
namespace host {

inline bool eq(const Fq& a, const Fq& b) { return memcmp(a.l, b.l, sizeof a.l) == 0; }
inline bool eq(const Fq2& a, const Fq2& b) { return eq(a.c0, b.c0) && eq(a.c1, b.c1); }
inline Fq2 fq2_zero() { return {zero(), zero()}; }
inline Fq2 fq2_one() { return {one(), zero()}; }
inline Fq2 mul_xi(const Fq2& a) { return {sub(a.c0, a.c1), add(a.c0, a.c1)}; }   // (1 + u) a
inline Fq2 mul_fq(const Fq2& a, const Fq& k) { return {mul(a.c0, k), mul(a.c1, k)}; }
inline Fq2 conj(const Fq2& a) { return {a.c0, neg(a.c1)}; }                     // a^p

// ---------------------------------------------------------------- Fq6 -----
struct Fq6 { Fq2 c0, c1, c2; };
inline Fq6 add(const Fq6& a, const Fq6& b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
inline Fq6 neg(const Fq6& a) { return {neg(a.c0), neg(a.c1), neg(a.c2)}; }
inline Fq6 mul(const Fq6& a, const Fq6& b) {
  // v^3 = xi
  const Fq2 c0 = add(mul(a.c0, b.c0), mul_xi(add(mul(a.c1, b.c2), mul(a.c2, b.c1))));
  const Fq2 c1 = add(add(mul(a.c0, b.c1), mul(a.c1, b.c0)), mul_xi(mul(a.c2, b.c2)));
  const Fq2 c2 = add(add(mul(a.c0, b.c2), mul(a.c1, b.c1)), mul(a.c2, b.c0));
  return {c0, c1, c2};
}
inline Fq6 mul_v(const Fq6& a) { return {mul_xi(a.c2), a.c0, a.c1}; }   // v a

// --------------------------------------------------------------- Fq12 -----
struct Fq12 { Fq6 c0, c1; };
inline Fq12 one12() {
  Fq12 r;
  r.c0 = {fq2_one(), fq2_zero(), fq2_zero()};
  r.c1 = {fq2_zero(), fq2_zero(), fq2_zero()};
  return r;
}
inline Fq12 mul(const Fq12& a, const Fq12& b) {
  // w^2 = v
  return {add(mul(a.c0, b.c0), mul_v(mul(a.c1, b.c1))), add(mul(a.c0, b.c1), mul(a.c1, b.c0))};
}
inline Fq12 conj(const Fq12& a) { return {a.c0, neg(a.c1)}; }   // a^(p^6)
inline bool is_one(const Fq12& a) {
  const Fq12 o = one12();
  const Fq2* x[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  const Fq2* y[6] = {&o.c0.c0, &o.c0.c1, &o.c0.c2, &o.c1.c0, &o.c1.c1, &o.c1.c2};
  for (int i = 0; i < 6; i++)
    if (!eq(*x[i], *y[i])) return false;
  return true;
}
template <int N>
inline Fq12 pow12(const Fq12& a, const uint64_t (&e)[N], int nbits) {
  Fq12 acc = one12();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = mul(acc, acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = mul(acc, a);
  }
  return acc;
}

// ------------------------------------------------------ affine points -----
struct A1 { Fq x, y; bool inf; };
struct A2 { Fq2 x, y; bool inf; };

// w^3 * (line through T with slope lambda, evaluated at P): the untwisted
// line l(P) = y_P - y_T - lambda_E (x_P - x_T) with x_T = x' w^-2,
// y_T = y' w^-3, lambda_E = lambda' w^-1 becomes
//   (lambda' x' - y') + (-lambda' x_P) v + (y_P) v w
// (w^3 is sent to 1 by the final exponentiation, so scaling every line by
// it changes nothing).
inline Fq12 line_eval(const Fq2& lambda, const Fq2& xT, const Fq2& yT, const A1& P) {
  Fq12 l;
  l.c0 = {sub(mul(lambda, xT), yT), neg(mul_fq(lambda, P.x)), fq2_zero()};
  l.c1 = {fq2_zero(), {P.y, zero()}, fq2_zero()};
  return l;
}

// f_{|x|, Q}(P), conjugated for the negative x (1/f and conj(f) agree after
// the final exponentiation, which also sends the dropped vertical lines to 1)
inline Fq12 miller_loop(const A1& P, const A2& Q) {
  Fq12 f = one12();
  if (P.inf || Q.inf) return f;
  Fq2 tx = Q.x, ty = Q.y;
  for (int i = 62; i >= 0; i--) {
    // doubling step: lambda = 3 x^2 / 2 y
    const Fq2 x2 = sqr(tx);
    const Fq2 lam = mul(add(add(x2, x2), x2), inv(add(ty, ty)));
    f = mul(mul(f, f), line_eval(lam, tx, ty, P));
    const Fq2 nx = sub(sub(sqr(lam), tx), tx);
    ty = sub(mul(lam, sub(tx, nx)), ty);
    tx = nx;
    if ((BLS_X_ABS >> i) & 1) {
      // addition step T + Q: lambda = (y_Q - y_T) / (x_Q - x_T)
      const Fq2 la = mul(sub(Q.y, ty), inv(sub(Q.x, tx)));
      f = mul(f, line_eval(la, tx, ty, P));
      const Fq2 ax = sub(sub(sqr(la), tx), Q.x);
      ty = sub(mul(la, sub(tx, ax)), ty);
      tx = ax;
    }
  }
  return conj(f);
}

inline Fq12 final_exp(const Fq12& f) { return pow12(f, FINAL_EXP, FINAL_EXP_BITS); }

// prod_i e(P_i, Q_i) == 1   (ark's multi_pairing(..).is_zero())
inline bool pairing_product_is_one(const std::vector<A1>& ps, const std::vector<A2>& qs) {
  Fq12 f = one12();
  for (size_t i = 0; i < ps.size(); i++) f = mul(f, miller_loop(ps[i], qs[i]));
  return is_one(final_exp(f));
}

// ------------------------------------------------------- square roots -----
template <int N>
inline Fq pow_fq(const Fq& a, const uint64_t (&e)[N]) {
  Fq acc = one();
  for (int i = 64 * N - 1; i >= 0; i--) {
    acc = sqr(acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = mul(acc, a);
  }
  return acc;
}
template <int N>
inline Fq2 pow_fq2(const Fq2& a, const uint64_t (&e)[N]) {
  Fq2 acc = fq2_one();
  for (int i = 64 * N - 1; i >= 0; i--) {
    acc = sqr(acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = mul(acc, a);
  }
  return acc;
}
// p = 3 mod 4: sqrt(a) = a^((p+1)/4) when a is a square
inline bool sqrt_fq(const Fq& a, Fq& out) {
  out = pow_fq(a, FQ_SQRT_EXP);
  return eq(sqr(out), a);
}
// Fq2 with p = 3 mod 4: the "complex method" (Adj and Rodriguez-Henriquez,
// "Square root computation over even extension fields", Algorithm 9)
inline bool sqrt_fq2(const Fq2& a, Fq2& out) {
  const Fq2 a1 = pow_fq2(a, FQ_PM3_DIV4);
  const Fq2 alpha = mul(a1, mul(a1, a));
  const Fq2 a0 = mul(conj(alpha), alpha);
  const Fq2 minus_one = neg(fq2_one());
  if (eq(a0, minus_one)) return false;
  const Fq2 x0 = mul(a1, a);
  if (eq(alpha, minus_one)) {
    out = {neg(x0.c1), x0.c0};   // u x0
  } else {
    out = mul(pow_fq2(add(fq2_one(), alpha), FQ_PM1_DIV2), x0);
  }
  return eq(sqr(out), a);
}

// ------------------------------------------------- subgroup / curve -----
inline Fq g1_b() { return add(add(one(), one()), add(one(), one())); }   // 4
inline Fq2 g2_b() { return {g1_b(), g1_b()}; }                           // 4 (1 + u)
inline bool on_curve(const A1& p) { return p.inf || eq(sqr(p.y), add(mul(sqr(p.x), p.x), g1_b())); }
inline bool on_curve(const A2& p) { return p.inf || eq(sqr(p.y), add(mul(sqr(p.x), p.x), g2_b())); }
template <class F>
inline X<F> from_affine(const F& x, const F& y, bool at_inf) {
  if (at_inf) return inf<F>();
  return {x, y, f_one<F>(), f_one<F>()};
}
// r P == O (ark's Validate::Yes subgroup check)
inline bool in_subgroup(const A1& p) { return p.inf || is_inf(mul_scalar(from_affine(p.x, p.y, false), FR_MOD64)); }
inline bool in_subgroup(const A2& p) { return p.inf || is_inf(mul_scalar(from_affine(p.x, p.y, false), FR_MOD64)); }

}  // namespace host
}  // namespace zk
