// host_san_check.cpp -- the host-side C++ of libzkp_amd.so (host_ec.hpp:
// Fq/Fq2/XYZZ and scalar multiplication used by the MSM tails and the
// s*pi_A + r*B1 term; host_pairing.hpp: the verifier's optimal-ate pairing)
// under AddressSanitizer + UndefinedBehaviorSanitizer, host only
// (tests/test_sanitizers.py builds it with g++).  Checks group-law and
// bilinearity identities so the run is meaningful without a report.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../zero-knowledge-proofs_amd/csrc/host_pairing.hpp"

using namespace zk::host;

static X<Fq> g1() {
  X<Fq> p;
  std::memcpy(p.X_.l, G1_GEN_HOSTM, 48);
  std::memcpy(p.Y.l, G1_GEN_HOSTM + 12, 48);
  p.ZZ = one();
  p.ZZZ = one();
  return p;
}
static X<Fq2> g2() {
  X<Fq2> p;
  std::memcpy(p.X_.c0.l, G2_GEN_HOSTM, 48);
  std::memcpy(p.X_.c1.l, G2_GEN_HOSTM + 12, 48);
  std::memcpy(p.Y.c0.l, G2_GEN_HOSTM + 24, 48);
  std::memcpy(p.Y.c1.l, G2_GEN_HOSTM + 36, 48);
  p.ZZ = f_one<Fq2>();
  p.ZZZ = f_one<Fq2>();
  return p;
}
template <class F>
static bool same(const X<F>& a, const X<F>& b) {
  F ax, ay, bx, by;
  const bool ia = !to_affine(a, ax, ay), ib = !to_affine(b, bx, by);
  if (ia || ib) return ia == ib;
  return std::memcmp(&ax, &bx, sizeof ax) == 0 && std::memcmp(&ay, &by, sizeof ay) == 0;
}

int main() {
  const uint64_t k1[4] = {0x1234567890abcdefull, 0x1111, 0, 0}, k2[4] = {0xfedcba987654321ull, 0, 7, 0};
  uint64_t k12[4] = {0};
  // (k1 + k2) P == k1 P + k2 P, in G1 and G2, and the Straus double multiplication
  unsigned __int128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (unsigned __int128)k1[i] + k2[i];
    k12[i] = (uint64_t)c;
    c >>= 64;
  }
  const auto P = g1();
  const auto Q = g2();
  if (!same(mul_scalar(P, k12), addp(mul_scalar(P, k1), mul_scalar(P, k2)))) return 1;
  if (!same(mul_scalar(Q, k12), addp(mul_scalar(Q, k1), mul_scalar(Q, k2)))) return 2;
  if (!same(mul2_scalar(P, k1, P, k2), mul_scalar(P, k12))) return 3;
  if (!same(dbl(P), addp(P, P))) return 4;
  // bilinearity: e(k1 P, Q) e(-P, k1 Q) == 1
  Fq px, py, qx0, qy0;
  Fq2 qx, qy, rx, ry;
  to_affine(mul_scalar(P, k1), px, py);
  to_affine(Q, qx, qy);
  to_affine(mul_scalar(Q, k1), rx, ry);
  Fq gx, gy;
  to_affine(P, gx, gy);
  std::vector<A1> ps = {A1{px, py, false}, A1{gx, neg(gy), false}};
  std::vector<A2> qs = {A2{qx, qy, false}, A2{rx, ry, false}};
  if (!pairing_product_is_one(ps, qs)) return 5;
  qs[1] = A2{qx, qy, false};
  if (pairing_product_is_one(ps, qs)) return 6;
  (void)qx0;
  (void)qy0;
  // divstep inversion == Fermat, on 0, 1, -1, the raw residues m - 1, m - 2,
  // 2^380, 2^380 - 1 (top-limb sign / carry boundaries of the signed limbs)
  // and 2000 residues uniform in [0, m) (381-bit rejection sampling)
  {
    uint64_t st = 0x9e3779b97f4a7c15ull;
    auto raw = [](uint64_t sub) {   // m - sub
      Fq a;
      std::memcpy(a.l, FQ_M, 48);
      a.l[0] -= sub;
      return a;
    };
    for (int k = 0; k < 2007; k++) {
      Fq a = zero();
      if (k == 1) a = one();
      else if (k == 2) a = neg(one());
      else if (k == 3) a = raw(1);
      else if (k == 4) a = raw(2);
      else if (k == 5) a.l[5] = 1ull << 60;                       // 2^380
      else if (k == 6) { for (int i = 0; i < 5; i++) a.l[i] = ~0ull; a.l[5] = (1ull << 60) - 1; }
      else if (k > 6) {
        do {
          for (int i = 0; i < 6; i++) {
            st ^= st << 13; st ^= st >> 7; st ^= st << 17;
            a.l[i] = st;
          }
          a.l[5] &= 0x1fffffffffffffffull;   // 381 bits, then reject >= m
        } while (geq_m(a.l));
      }
      const Fq x = inv(a), y = inv_fermat(a);
      if (std::memcmp(&x, &y, sizeof x) != 0) return 7;
      if (k) {
        const Fq o = mul(a, x), u = one();
        if (std::memcmp(&o, &u, sizeof o) != 0) return 8;
      }
    }
  }
  std::printf("host sanitizer check ok\n");
  return 0;
}
