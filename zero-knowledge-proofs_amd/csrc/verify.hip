// verify.hip -- Groth16 Verifier / BatchVerifier (crates/groth16-core/src/lib.rs:
// 303-432), the pairing-product check behind them (Bls12_381::multi_pairing,
// core:352) and ark-serialize compressed decoding of Proof (core:28).
//
// Host code only (no kernels): a verification is four Miller loops and one
// final exponentiation of strictly sequential field arithmetic
// (host_pairing.hpp).  Every entry point works without a GPU.
#include <cstring>
#include <vector>

#include "common.hpp"
#include "host_pairing.hpp"

namespace zk {
bool fq_canonical_largest(const uint64_t* c);   // setup.hip: y > (p - 1) / 2
}

using namespace zk;
using namespace zk::host;

namespace {

Fq fq_in(const uint64_t* w) {
  Fq c;
  std::memcpy(c.l, w, 48);
  return to_mont(c);
}
void fq_out(const Fq& m, uint64_t* w) {
  const Fq c = from_mont(m);
  std::memcpy(w, c.l, 48);
}

// ABI point -> host affine; false when a coordinate is not canonical or the
// point is off the curve (no ark value looks like that)
bool load(const zk_g1_affine& a, A1& p) {
  p.inf = a.infinity != 0;
  p.x = zero();
  p.y = zero();
  if (p.inf) return true;
  if (geq_m(a.x) || geq_m(a.y)) return false;
  p.x = fq_in(a.x);
  p.y = fq_in(a.y);
  return on_curve(p);
}
bool load(const zk_g2_affine& a, A2& p) {
  p.inf = a.infinity != 0;
  p.x = fq2_zero();
  p.y = fq2_zero();
  if (p.inf) return true;
  for (int k = 0; k < 2; k++)
    if (geq_m(a.x + 6 * k) || geq_m(a.y + 6 * k)) return false;
  p.x = {fq_in(a.x), fq_in(a.x + 6)};
  p.y = {fq_in(a.y), fq_in(a.y + 6)};
  return on_curve(p);
}

X<Fq> to_x(const A1& p) { return from_affine(p.x, p.y, p.inf); }
X<Fq2> to_x(const A2& p) { return from_affine(p.x, p.y, p.inf); }
A1 to_a(const X<Fq>& p) {
  A1 a;
  a.inf = !to_affine(p, a.x, a.y);
  return a;
}
A2 to_a(const X<Fq2>& p) {
  A2 a;
  a.inf = !to_affine(p, a.x, a.y);
  return a;
}
A1 negate(const A1& p) {
  A1 r = p;
  if (!p.inf) r.y = neg(p.y);
  return r;
}

// [IC]_1 = ic_g1[0] + sum_i Fr::from(lo64(x_i)) ic_g1[i + 1] over the
// non-zero lo64(x_i) (core:322-338; the MSM's result is the unique group
// element, so a plain double-and-add gives the same point)
int ic_sum(const zk_vk& vk, const zk_fr* in, size_t n, X<Fq>& out) {
  if (!vk.ic_g1 || vk.ic_len < n + 1) return ZK_ERR_ARG;   // the reference would index out of range
  A1 p;
  if (!load(vk.ic_g1[0], p)) return ZK_ERR_ARG;
  X<Fq> acc = to_x(p);
  for (size_t i = 0; i < n; i++) {
    const uint64_t k[4] = {in[i].l[0], 0, 0, 0};
    if (!k[0]) continue;
    if (!load(vk.ic_g1[i + 1], p)) return ZK_ERR_ARG;
    acc = addp(acc, mul_scalar(to_x(p), k));
  }
  out = acc;
  return ZK_OK;
}

// e(A, B) e(-alpha, beta) e(-IC, gamma) e(-C, delta) == 1   (core:340-354)
int pairing_check(const zk_vk& vk, const A1& a, const A2& b, const A1& ic, const A1& c, int* valid) {
  A1 alpha;
  A2 beta, gamma, delta;
  if (!load(vk.alpha_g1, alpha) || !load(vk.beta_g2, beta) || !load(vk.gamma_g2, gamma) ||
      !load(vk.delta_g2, delta))
    return ZK_ERR_ARG;
  *valid = pairing_product_is_one({a, negate(alpha), negate(ic), negate(c)}, {b, beta, gamma, delta}) ? 1 : 0;
  return ZK_OK;
}

void rd48(const uint8_t* in, uint8_t flag_mask, uint64_t* l) {
  for (int i = 0; i < 6; i++) l[i] = 0;
  for (int i = 0; i < 48; i++) {
    const uint8_t b = i == 0 ? (uint8_t)(in[0] & flag_mask) : in[i];
    l[(47 - i) / 8] |= (uint64_t)b << (8 * ((47 - i) % 8));
  }
}
bool is_zero6(const uint64_t* c) {
  uint64_t x = 0;
  for (int i = 0; i < 6; i++) x |= c[i];
  return x == 0;
}

// zcash / ark-bls12-381 0.4 compressed point, validated like
// CanonicalDeserialize::deserialize_compressed (Validate::Yes): compression
// flag set, x < p, x^3 + b a square, the flagged root, the prime-order
// subgroup.  One DELIBERATE DEVIATION from ark 0.4: an infinity encoding must
// also have the sort flag clear and every x byte zero.  ark-bls12-381 0.4's
// read_g1/g2_compressed returns the identity as soon as the infinity flag is
// set without looking at the x bytes, so bytes it accepts (infinity with
// stray x bits) are rejected here: the zcash encoding has exactly one
// identity, and accepting others makes the proof encoding malleable.  The ark
// source is not in the reference tree, so this behaviour is parity-unpinned
// either way.
static bool x_bytes_zero(const uint8_t* in, size_t len) {
  uint8_t acc = in[0] & 0x1f;   // flag bits masked off
  for (size_t i = 1; i < len; i++) acc |= in[i];
  return acc == 0;
}
int decode_g1(const uint8_t* in, zk_g1_affine& out) {
  std::memset(&out, 0, sizeof out);
  const uint8_t f = in[0];
  if (!(f & 0x80)) return ZK_ERR_ARG;
  if (f & 0x40) {
    if ((f & 0x20) || !x_bytes_zero(in, 48)) return ZK_ERR_ARG;
    out.infinity = 1;
    return ZK_OK;
  }
  uint64_t x[6];
  rd48(in, 0x1f, x);
  if (geq_m(x)) return ZK_ERR_ARG;
  A1 p;
  p.inf = false;
  p.x = fq_in(x);
  if (!sqrt_fq(add(mul(sqr(p.x), p.x), g1_b()), p.y)) return ZK_ERR_ARG;
  uint64_t yc[6];
  fq_out(p.y, yc);
  if (fq_canonical_largest(yc) != ((f & 0x20) != 0)) p.y = neg(p.y);
  if (!in_subgroup(p)) return ZK_ERR_ARG;
  std::memcpy(out.x, x, 48);
  fq_out(p.y, out.y);
  return ZK_OK;
}
int decode_g2(const uint8_t* in, zk_g2_affine& out) {
  std::memset(&out, 0, sizeof out);
  const uint8_t f = in[0];
  if (!(f & 0x80)) return ZK_ERR_ARG;
  if (f & 0x40) {
    if ((f & 0x20) || !x_bytes_zero(in, 96)) return ZK_ERR_ARG;
    out.infinity = 1;
    return ZK_OK;
  }
  uint64_t x0[6], x1[6];   // bytes: x.c1 (with the flags), then x.c0
  rd48(in, 0x1f, x1);
  rd48(in + 48, 0xff, x0);
  if (geq_m(x0) || geq_m(x1)) return ZK_ERR_ARG;
  A2 p;
  p.inf = false;
  p.x = {fq_in(x0), fq_in(x1)};
  if (!sqrt_fq2(add(mul(sqr(p.x), p.x), g2_b()), p.y)) return ZK_ERR_ARG;
  uint64_t y0[6], y1[6];
  fq_out(p.y.c0, y0);
  fq_out(p.y.c1, y1);
  const bool big = is_zero6(y1) ? fq_canonical_largest(y0) : fq_canonical_largest(y1);
  if (big != ((f & 0x20) != 0)) p.y = neg(p.y);
  if (!in_subgroup(p)) return ZK_ERR_ARG;
  std::memcpy(out.x, x0, 48);
  std::memcpy(out.x + 6, x1, 48);
  fq_out(p.y.c0, out.y);
  fq_out(p.y.c1, out.y + 6);
  return ZK_OK;
}

}  // namespace

#define ZK_HOST_GUARD(...)                 \
  try {                                    \
    __VA_ARGS__                            \
  } catch (const std::exception&) {        \
    return ZK_ERR_ARG;                     \
  }

int zk_pairing_product_is_one(const zk_g1_affine* g1, const zk_g2_affine* g2, size_t n, int* result) {
  if (!result || (n && (!g1 || !g2))) return ZK_ERR_ARG;
  ZK_HOST_GUARD({
    *result = 0;
    std::vector<A1> ps(n);
    std::vector<A2> qs(n);
    for (size_t i = 0; i < n; i++)
      if (!load(g1[i], ps[i]) || !load(g2[i], qs[i])) return ZK_ERR_ARG;
    *result = pairing_product_is_one(ps, qs) ? 1 : 0;
    return ZK_OK;
  })
}

int zk_groth16_verify(const zk_vk* vk, const zk_proof* proof, const zk_fr* public_inputs, size_t n_inputs,
                      int* valid) {
  if (!vk || !proof || !valid || (n_inputs && !public_inputs)) return ZK_ERR_ARG;
  ZK_HOST_GUARD({
    *valid = 0;
    if (n_inputs != vk->num_public) return ZK_ERR_INVALID_WITNESS;   // core:315-320
    X<Fq> ic;
    const int rc = ic_sum(*vk, public_inputs, n_inputs, ic);
    if (rc) return rc;
    A1 a, c;
    A2 b;
    if (!load(proof->a, a) || !load(proof->b, b) || !load(proof->c, c)) return ZK_ERR_ARG;
    return pairing_check(*vk, a, b, to_a(ic), c, valid);
  })
}

int zk_groth16_verify_batch(const zk_vk* vk, const zk_proof* proofs, const zk_fr* const* public_inputs,
                            const size_t* n_inputs, size_t n_proofs, const zk_fr* coeffs, int* valid) {
  if (!vk || !valid || (n_proofs && (!proofs || !public_inputs || !n_inputs || !coeffs))) return ZK_ERR_ARG;
  ZK_HOST_GUARD({
    *valid = 0;
    if (n_proofs == 0) {   // core:373-375
      *valid = 1;
      return ZK_OK;
    }
    // core:384-419: the coefficient-weighted sums of A, B, C and IC, then ONE
    // pairing check on them (the reference's rule, kept as is)
    X<Fq> sa = inf<Fq>(), sc = inf<Fq>(), sic = inf<Fq>();
    X<Fq2> sb = inf<Fq2>();
    for (size_t k = 0; k < n_proofs; k++) {
      if (n_inputs[k] != vk->num_public) return ZK_ERR_INVALID_WITNESS;   // core:388-393
      if (n_inputs[k] && !public_inputs[k]) return ZK_ERR_ARG;
      A1 a, c;
      A2 b;
      if (!load(proofs[k].a, a) || !load(proofs[k].b, b) || !load(proofs[k].c, c)) return ZK_ERR_ARG;
      const uint64_t* w = coeffs[k].l;
      sa = addp(sa, mul_scalar(to_x(a), w));
      sb = addp(sb, mul_scalar(to_x(b), w));
      sc = addp(sc, mul_scalar(to_x(c), w));
      X<Fq> ic;
      const int rc = ic_sum(*vk, public_inputs[k], n_inputs[k], ic);
      if (rc) return rc;
      sic = addp(sic, mul_scalar(ic, w));
    }
    return pairing_check(*vk, to_a(sa), to_a(sb), to_a(sic), to_a(sc), valid);
  })
}

int zk_proof_deserialize_compressed(const uint8_t in[192], zk_proof* out) {
  if (!in || !out) return ZK_ERR_ARG;
  ZK_HOST_GUARD({
    int rc = decode_g1(in, out->a);
    if (!rc) rc = decode_g2(in + 48, out->b);
    if (!rc) rc = decode_g1(in + 144, out->c);
    if (rc) std::memset(out, 0, sizeof *out);
    return rc;
  })
}
