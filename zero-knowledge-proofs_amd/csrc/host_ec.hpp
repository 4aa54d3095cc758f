// host_ec.hpp -- host-side Fq / Fq2 / XYZZ arithmetic (64-bit limbs, u128).
//
// Used ONLY for the latency-bound O(windows) tail of each MSM (combining the
// per-window partial sums from the GPU with ~64..255 doublings), for the two
// variable-base full-width terms s*pi_A + r*B1 of pi_C
// (crates/groth16-core/src/lib.rs:239-259), and for affine normalisation of
// the five MSM results.  These are a few hundred strictly sequential group
// operations per proof: a host core runs one in ~0.4 us, a single GPU lane
// in ~15 us, so they belong here.  All data-parallel work is on the GPU.
// Same Montgomery representation (R = 2^384) and bytes as the device code.
#pragma once
#include <stdint.h>
#include <string.h>

#include "constants.hpp"

namespace zk {
namespace host {

typedef unsigned __int128 u128;

template <int N>
struct Mod64 {
  uint64_t m[N];
  uint64_t inv;     // -m^-1 mod 2^64
  uint64_t one[N];  // R mod m
  uint64_t r2[N];
};

template <class P, int N>
inline Mod64<N> make_mod() {
  Mod64<N> M;
  for (int i = 0; i < N; i++) {
    M.m[i] = (uint64_t)P::MOD[2 * i] | ((uint64_t)P::MOD[2 * i + 1] << 32);
    M.one[i] = (uint64_t)P::ONE[2 * i] | ((uint64_t)P::ONE[2 * i + 1] << 32);
    M.r2[i] = (uint64_t)P::R2[2 * i] | ((uint64_t)P::R2[2 * i + 1] << 32);
  }
  uint64_t x = 1;  // Newton: x = m^-1 mod 2^64
  for (int k = 0; k < 7; k++) x *= 2 - M.m[0] * x;
  M.inv = (uint64_t)0 - x;
  return M;
}

inline const Mod64<6>& FQ() {
  static const Mod64<6> M = make_mod<FqHostParams, 6>();
  return M;
}
inline const Mod64<4>& FR() {
  static const Mod64<4> M = make_mod<FrHostParams, 4>();
  return M;
}

// ---- generic N-limb Montgomery helpers (used for Fr on the host) ----
template <int N>
inline bool geq_n(const uint64_t* a, const uint64_t* m) {
  for (int i = N - 1; i >= 0; i--) { if (a[i] > m[i]) return true; if (a[i] < m[i]) return false; }
  return true;
}
template <int N>
inline void mont_mul_n(uint64_t* o, const uint64_t* a, const uint64_t* b, const Mod64<N>& M) {
  uint64_t t[N + 2] = {0};
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
    for (int j = 0; j < N; j++) { u128 s = (u128)a[j] * b[i] + t[j] + c; t[j] = (uint64_t)s; c = (uint64_t)(s >> 64); }
    u128 s = (u128)t[N] + c; t[N] = (uint64_t)s; t[N + 1] = (uint64_t)(s >> 64);
    uint64_t q = t[0] * M.inv;
    s = (u128)q * M.m[0] + t[0]; c = (uint64_t)(s >> 64);
    for (int j = 1; j < N; j++) { s = (u128)q * M.m[j] + t[j] + c; t[j - 1] = (uint64_t)s; c = (uint64_t)(s >> 64); }
    s = (u128)t[N] + c; t[N - 1] = (uint64_t)s; t[N] = t[N + 1] + (uint64_t)(s >> 64);
  }
  if (t[N] || geq_n<N>(t, M.m)) {
    uint64_t br = 0;
    for (int i = 0; i < N; i++) { u128 d = (u128)t[i] - M.m[i] - br; t[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
  }
  memcpy(o, t, sizeof(uint64_t) * N);
}

// Fr on the host: 4 x u64 Montgomery (R = 2^256)
struct Fr { uint64_t l[4]; };
inline Fr fr_mul(const Fr& a, const Fr& b) { Fr r; mont_mul_n<4>(r.l, a.l, b.l, FR()); return r; }
inline Fr fr_to_mont(const uint64_t* c) { Fr a, r2; memcpy(a.l, c, 32); memcpy(r2.l, FR().r2, 32); return fr_mul(a, r2); }
inline void fr_from_mont(const Fr& a, uint64_t* c) { Fr o{}; o.l[0] = 1; Fr r = fr_mul(a, o); memcpy(c, r.l, 32); }
inline Fr fr_one() { Fr r; memcpy(r.l, FR().one, 32); return r; }
inline bool fr_is_zero(const Fr& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }
inline Fr fr_sub(const Fr& a, const Fr& b) {
  Fr r; uint64_t br = 0;
  for (int i = 0; i < 4; i++) { u128 d = (u128)a.l[i] - b.l[i] - br; r.l[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
  if (br) { uint64_t c = 0; for (int i = 0; i < 4; i++) { u128 s = (u128)r.l[i] + FR().m[i] + c; r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64); } }
  return r;
}
inline Fr fr_pow(const Fr& a, const uint64_t* e, int nbits) {
  Fr acc = fr_one();
  for (int i = nbits - 1; i >= 0; i--) {
    acc = fr_mul(acc, acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = fr_mul(acc, a);
  }
  return acc;
}
inline Fr fr_inv(const Fr& a) {
  uint64_t e[4]; memcpy(e, FR().m, 32); e[0] -= 2;
  return fr_pow(a, e, 256);
}
inline Fr fr_from_u64(uint64_t v) { uint64_t c[4] = {v, 0, 0, 0}; return fr_to_mont(c); }
// host Montgomery (R = 2^256) -> device Montgomery (R = 2^261)
inline Fr fr_to_dev(const Fr& h) {
  Fr k;
  for (int i = 0; i < 4; i++) k.l[i] = (uint64_t)FrHostParams::TO_DEV[2 * i] | ((uint64_t)FrHostParams::TO_DEV[2 * i + 1] << 32);
  return fr_mul(h, k);
}

struct Fq { uint64_t l[6]; };
struct Fq2 { Fq c0, c1; };

// Fq modulus and -m^-1 mod 2^64 as compile-time constants, so the products
// below unroll with the modulus words as immediates (the s*pi_A + r*B1
// Straus term is ~400 sequential group operations per proof on one core)
constexpr uint64_t fq_m64(int i) {
  return (uint64_t)FqHostParams::MOD[2 * i] | ((uint64_t)FqHostParams::MOD[2 * i + 1] << 32);
}
constexpr uint64_t fq_inv64() {
  uint64_t x = 1;
  for (int k = 0; k < 7; k++) x *= 2 - fq_m64(0) * x;
  return (uint64_t)0 - x;
}
constexpr uint64_t FQ_M[6] = {fq_m64(0), fq_m64(1), fq_m64(2), fq_m64(3), fq_m64(4), fq_m64(5)};
constexpr uint64_t FQ_INV = fq_inv64();

inline bool is_zero(const Fq& a) {
  uint64_t x = 0;
  for (int i = 0; i < 6; i++) x |= a.l[i];
  return x == 0;
}
inline bool geq_m(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) { if (a[i] > FQ_M[i]) return true; if (a[i] < FQ_M[i]) return false; }
  return true;
}
inline void sub_m(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) { u128 d = (u128)a[i] - FQ_M[i] - br; a[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
}
inline Fq add(const Fq& a, const Fq& b) {
  Fq r; uint64_t c = 0;
  for (int i = 0; i < 6; i++) { u128 s = (u128)a.l[i] + b.l[i] + c; r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64); }
  if (c || geq_m(r.l)) sub_m(r.l);
  return r;
}
inline Fq sub(const Fq& a, const Fq& b) {
  Fq r; uint64_t br = 0;
  for (int i = 0; i < 6; i++) { u128 d = (u128)a.l[i] - b.l[i] - br; r.l[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) { u128 s = (u128)r.l[i] + FQ_M[i] + c; r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64); }
  }
  return r;
}
inline Fq mul(const Fq& a, const Fq& b) {
  uint64_t t[8] = {0};
#pragma GCC unroll 6
  for (int i = 0; i < 6; i++) {
    uint64_t c = 0;
#pragma GCC unroll 6
    for (int j = 0; j < 6; j++) { u128 s = (u128)a.l[j] * b.l[i] + t[j] + c; t[j] = (uint64_t)s; c = (uint64_t)(s >> 64); }
    u128 s = (u128)t[6] + c; t[6] = (uint64_t)s; t[7] = (uint64_t)(s >> 64);
    uint64_t q = t[0] * FQ_INV;
    s = (u128)q * FQ_M[0] + t[0]; c = (uint64_t)(s >> 64);
#pragma GCC unroll 5
    for (int j = 1; j < 6; j++) { s = (u128)q * FQ_M[j] + t[j] + c; t[j - 1] = (uint64_t)s; c = (uint64_t)(s >> 64); }
    s = (u128)t[6] + c; t[5] = (uint64_t)s; t[6] = t[7] + (uint64_t)(s >> 64);
  }
  Fq r; memcpy(r.l, t, 48);
  if (t[6] || geq_m(r.l)) sub_m(r.l);
  return r;
}
inline Fq sqr(const Fq& a) { return mul(a, a); }
inline Fq neg(const Fq& a) { Fq z{}; return sub(z, a); }
inline Fq one() { Fq r; memcpy(r.l, FQ().one, 48); return r; }
inline Fq zero() { Fq r{}; return r; }
// a^(m-2) (Fermat): 384 squarings + ~190 products, ~40 us on one core.
// Kept as the reference for inv() below.
inline Fq inv_fermat(const Fq& a) {
  uint64_t e[6]; memcpy(e, FQ_M, 48);
  e[0] -= 2;  // m is odd and > 2
  Fq acc = one();
  for (int i = 383; i >= 0; i--) {
    acc = sqr(acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = mul(acc, a);
  }
  return acc;
}

// Constant-time inversion by Bernstein-Yang divsteps (the safegcd form with
// zeta = -(delta + 1/2)), 62 divsteps per round on the low words of (f, g),
// each round's 2x2 transition matrix (entries |.| <= 2^62) then applied to the
// full f, g and to the Bezout coefficients d, e, which stay in (-2m, m) by
// adding the multiple of m that makes them divisible by 2^62.  Numbers are 7
// signed 62-bit limbs (434 bits; the top limb carries the sign).  A 381-bit
// modulus needs at most (49 * 381 + 57) / 17 = 1101 divsteps: 18 rounds.
// About 10x fewer cycles than Fermat; it sits on the proof's critical path
// (pi_C's affine conversion follows the last MSM).
namespace bgcd {
constexpr int L = 7, ROUNDS = 18;
constexpr uint64_t M62 = ~0ull >> 2;
typedef __int128 i128;
struct S62 { int64_t v[L]; };
inline S62 from_words(const uint64_t (&w)[6]) {
  S62 s;
  for (int i = 0; i < L; i++) {
    const int bit = 62 * i, k = bit >> 6, sh = bit & 63;
    uint64_t x = k < 6 ? w[k] >> sh : 0;
    if (sh > 2 && k + 1 < 6) x |= w[k + 1] << (64 - sh);
    s.v[i] = (int64_t)(x & M62);
  }
  return s;
}
struct Consts {
  S62 m;
  uint64_t minv62;   // m^-1 mod 2^62
};
inline const Consts& consts() {
  static const Consts c = [] {
    Consts k;
    uint64_t w[6];
    memcpy(w, FQ_M, 48);
    k.m = from_words(w);
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - FQ_M[0] * x;
    k.minv62 = x & M62;
    return k;
  }();
  return c;
}
inline int64_t divsteps62(int64_t zeta, uint64_t f, uint64_t g, int64_t (&t)[4]) {
  uint64_t u = 1, v = 0, q = 0, r = 1;
  for (int i = 0; i < 62; i++) {
    const uint64_t c1 = (uint64_t)(zeta >> 63);   // zeta < 0
    const uint64_t c2 = 0 - (g & 1);              // g odd
    const uint64_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2; q += y & c2; r += z & c2;
    const uint64_t c3 = c1 & c2;
    zeta = (zeta ^ (int64_t)c3) - 1;
    f += g & c3; u += q & c3; v += r & c3;
    g >>= 1; u <<= 1; v <<= 1;
  }
  t[0] = (int64_t)u; t[1] = (int64_t)v; t[2] = (int64_t)q; t[3] = (int64_t)r;
  return zeta;
}
// (f, g) <- (u f + v g, q f + r g) / 2^62, exact
inline void update_fg(S62& f, S62& g, const int64_t (&t)[4]) {
  i128 cf = (i128)t[0] * f.v[0] + (i128)t[1] * g.v[0];
  i128 cg = (i128)t[2] * f.v[0] + (i128)t[3] * g.v[0];
  cf >>= 62; cg >>= 62;
  for (int i = 1; i < L; i++) {
    cf += (i128)t[0] * f.v[i] + (i128)t[1] * g.v[i];
    cg += (i128)t[2] * f.v[i] + (i128)t[3] * g.v[i];
    f.v[i - 1] = (int64_t)((uint64_t)cf & M62); cf >>= 62;
    g.v[i - 1] = (int64_t)((uint64_t)cg & M62); cg >>= 62;
  }
  f.v[L - 1] = (int64_t)cf;
  g.v[L - 1] = (int64_t)cg;
}
// (d, e) <- (u d + v e, q d + r e) / 2^62 mod m, in (-2m, m) -> (-2m, m)
inline void update_de(S62& d, S62& e, const int64_t (&t)[4]) {
  const Consts& K = consts();
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int64_t sd = d.v[L - 1] >> 63, se = e.v[L - 1] >> 63;
  int64_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  i128 cd = (i128)u * d.v[0] + (i128)v * e.v[0];
  i128 ce = (i128)q * d.v[0] + (i128)r * e.v[0];
  md -= (int64_t)((K.minv62 * (uint64_t)cd + (uint64_t)md) & M62);
  me -= (int64_t)((K.minv62 * (uint64_t)ce + (uint64_t)me) & M62);
  cd += (i128)K.m.v[0] * md;
  ce += (i128)K.m.v[0] * me;
  cd >>= 62; ce >>= 62;
  for (int i = 1; i < L; i++) {
    cd += (i128)u * d.v[i] + (i128)v * e.v[i] + (i128)K.m.v[i] * md;
    ce += (i128)q * d.v[i] + (i128)r * e.v[i] + (i128)K.m.v[i] * me;
    d.v[i - 1] = (int64_t)((uint64_t)cd & M62); cd >>= 62;
    e.v[i - 1] = (int64_t)((uint64_t)ce & M62); ce >>= 62;
  }
  d.v[L - 1] = (int64_t)cd;
  e.v[L - 1] = (int64_t)ce;
}
// d in (-2m, m), times the sign of f (+-1) -> [0, m) as 6 words
inline void to_words(S62 d, int64_t fsign, uint64_t (&w)[6]) {
  const Consts& K = consts();
  for (int pass = 0; pass < 3; pass++) {
    const int64_t sg = pass == 1 ? fsign : d.v[L - 1] >> 63;
    i128 c = 0;
    for (int i = 0; i < L; i++) {
      if (pass == 1) c += (i128)((d.v[i] ^ sg) - sg);
      else c += (i128)d.v[i] + (i128)(K.m.v[i] & sg);
      d.v[i] = i + 1 < L ? (int64_t)((uint64_t)c & M62) : (int64_t)c;
      c >>= 62;
    }
  }
  for (int k = 0; k < 6; k++) {
    const int bit = 64 * k, i = bit / 62, sh = bit - 62 * i;
    uint64_t x = (uint64_t)d.v[i] >> sh;
    if (i + 1 < L) x |= (uint64_t)d.v[i + 1] << (62 - sh);
    if (sh > 60 && i + 2 < L) x |= (uint64_t)d.v[i + 2] << (124 - sh);
    w[k] = x;
  }
}
}  // namespace bgcd

// Montgomery form in and out: canonical(a R)^-1 = a^-1 R^-1, times R^2
// twice.  0 -> 0 (as Fermat).
inline Fq inv(const Fq& a) {
  using namespace bgcd;
  S62 f = consts().m, g = from_words(a.l), d{}, e{};
  e.v[0] = 1;
  int64_t zeta = -1;
  for (int k = 0; k < ROUNDS; k++) {
    int64_t t[4];
    zeta = divsteps62(zeta, (uint64_t)f.v[0], (uint64_t)g.v[0], t);
    update_de(d, e, t);
    update_fg(f, g, t);
  }
  Fq o, r2;
  to_words(d, f.v[L - 1] >> 63, o.l);
  memcpy(r2.l, FQ().r2, 48);
  return mul(mul(o, r2), r2);
}
inline Fq from_mont(const Fq& a) { Fq o{}; o.l[0] = 1; return mul(a, o); }
// host Montgomery (R = 2^384) <-> device Montgomery (R = 2^392), see constants.hpp
inline Fq fq_const(const uint32_t (&c)[12]) { Fq r; for (int i = 0; i < 6; i++) r.l[i] = (uint64_t)c[2 * i] | ((uint64_t)c[2 * i + 1] << 32); return r; }
inline Fq to_dev(const Fq& h) { return mul(h, fq_const(FqHostParams::TO_DEV)); }
inline Fq to_host(const Fq& d) { return mul(d, fq_const(FqHostParams::TO_HOST)); }
inline Fq to_mont(const Fq& a) { Fq r2; memcpy(r2.l, FQ().r2, 48); return mul(a, r2); }

inline bool is_zero(const Fq2& a) { return is_zero(a.c0) && is_zero(a.c1); }
inline Fq2 add(const Fq2& a, const Fq2& b) { return {add(a.c0, b.c0), add(a.c1, b.c1)}; }
inline Fq2 sub(const Fq2& a, const Fq2& b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
inline Fq2 mul(const Fq2& a, const Fq2& b) {
  Fq t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  Fq m = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return {sub(t0, t1), sub(sub(m, t0), t1)};
}
inline Fq2 sqr(const Fq2& a) { return mul(a, a); }
inline Fq2 neg(const Fq2& a) { return {neg(a.c0), neg(a.c1)}; }
inline Fq2 inv(const Fq2& a) {
  Fq n = inv(add(sqr(a.c0), sqr(a.c1)));
  return {mul(a.c0, n), neg(mul(a.c1, n))};
}
inline Fq2 to_dev(const Fq2& h) { return {to_dev(h.c0), to_dev(h.c1)}; }
inline Fq2 to_host(const Fq2& d) { return {to_host(d.c0), to_host(d.c1)}; }
template <class F> inline F f_one();
template <> inline Fq f_one<Fq>() { return one(); }
template <> inline Fq2 f_one<Fq2>() { return {one(), zero()}; }
template <class F> inline F f_zero() { F z; memset(&z, 0, sizeof z); return z; }

// ---- XYZZ group law (same EFD formulas as the device code) ----
template <class F>
struct X {
  F X_, Y, ZZ, ZZZ;
};
template <class F>
inline X<F> inf() { return {f_zero<F>(), f_one<F>(), f_zero<F>(), f_zero<F>()}; }
template <class F>
inline bool is_inf(const X<F>& p) { return is_zero(p.ZZ); }

template <class F>
inline X<F> dbl(const X<F>& p) {
  if (is_inf(p)) return p;
  F U = add(p.Y, p.Y), V = sqr(U), W = mul(U, V), S = mul(p.X_, V);
  F X2 = sqr(p.X_), M = add(add(X2, X2), X2);
  X<F> r;
  r.X_ = sub(sqr(M), add(S, S));
  r.Y = sub(mul(M, sub(S, r.X_)), mul(W, p.Y));
  r.ZZ = mul(V, p.ZZ);
  r.ZZZ = mul(W, p.ZZZ);
  return r;
}
template <class F>
inline X<F> addp(const X<F>& p, const X<F>& q) {
  if (is_inf(p)) return q;
  if (is_inf(q)) return p;
  F U1 = mul(p.X_, q.ZZ), U2 = mul(q.X_, p.ZZ), S1 = mul(p.Y, q.ZZZ), S2 = mul(q.Y, p.ZZZ);
  F P = sub(U2, U1), R = sub(S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl(p);
    return inf<F>();
  }
  F PP = sqr(P), PPP = mul(P, PP), Q = mul(U1, PP);
  X<F> r;
  r.X_ = sub(sub(sqr(R), PPP), add(Q, Q));
  r.Y = sub(mul(R, sub(Q, r.X_)), mul(S1, PPP));
  r.ZZ = mul(mul(p.ZZ, q.ZZ), PP);
  r.ZZZ = mul(mul(p.ZZZ, q.ZZZ), PPP);
  return r;
}
// k*p for a little-endian 4x64 scalar (left-to-right double-and-add)
template <class F>
inline X<F> mul_scalar(const X<F>& p, const uint64_t k[4]) {
  X<F> acc = inf<F>();
  for (int i = 255; i >= 0; i--) {
    acc = dbl(acc);
    if ((k[i >> 6] >> (i & 63)) & 1) acc = addp(acc, p);
  }
  return acc;
}
// k1*p + k2*q (Straus / Shamir, 4-bit windows): 256 doublings shared by both
// scalars and <= 2 additions per window -- the s*pi_A + r*B_1 term of pi_C.
template <class F>
inline X<F> mul2_scalar(const X<F>& p, const uint64_t k1[4], const X<F>& q, const uint64_t k2[4]) {
  X<F> tp[16], tq[16];
  tp[0] = inf<F>();
  tq[0] = inf<F>();
  for (int i = 1; i < 16; i++) {
    tp[i] = addp(tp[i - 1], p);
    tq[i] = addp(tq[i - 1], q);
  }
  X<F> acc = inf<F>();
  for (int w = 63; w >= 0; w--) {
    for (int d = 0; d < 4; d++) acc = dbl(acc);
    const int sh = (w & 15) * 4;
    const unsigned d1 = (unsigned)(k1[w >> 4] >> sh) & 15u, d2 = (unsigned)(k2[w >> 4] >> sh) & 15u;
    if (d1) acc = addp(acc, tp[d1]);
    if (d2) acc = addp(acc, tq[d2]);
  }
  return acc;
}

// affine (Montgomery) from XYZZ: x = X/ZZ, y = Y/ZZZ.  Returns false at infinity.
template <class F>
inline bool to_affine(const X<F>& p, F& x, F& y) {
  if (is_inf(p)) { x = f_zero<F>(); y = f_zero<F>(); return false; }
  F i = inv(p.ZZZ);                 // Z^-3
  F zi = mul(p.ZZ, i);              // Z^-1
  F zzi = sqr(zi);                  // Z^-2
  x = mul(p.X_, zzi);
  y = mul(p.Y, i);
  return true;
}

}  // namespace host
}  // namespace zk
