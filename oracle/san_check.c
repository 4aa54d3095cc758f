/*
 * san_check.c -- drives the oracle (TEST INFRASTRUCTURE) under AddressSanitizer
 * and UndefinedBehaviorSanitizer (host only: oracle/Makefile `san` target,
 * run by tests/test_sanitizers.py).  Every exported routine runs on small
 * inputs, single- and multi-threaded, and the results are cross-checked so
 * the run also means something without a sanitizer report.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zk_oracle.h"

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main(void) {
  or_init();
  const uint64_t n = 1 << 7, V = 3 * n + 1, np = 1;
  uint64_t *rp = calloc(n + 1, 8), *vals = calloc(4 * n, 8);
  uint32_t *ac = calloc(n, 4), *bc = calloc(n, 4), *cc = calloc(n, 4);
  or_synthetic_circuit(n, rp, ac, bc, cc, vals);
  or_r1cs cs = {n, V, rp, ac, vals, rp, bc, vals, rp, cc, vals};
  uint64_t params[20];
  or_random_fr(params, 5, 11);
  or_pk pk;
  or_vk vk;
  memset(&pk, 0, sizeof pk);
  memset(&vk, 0, sizeof vk);
  pk.a_g1 = calloc(13 * V, 8);
  pk.b_g1 = calloc(13 * V, 8);
  pk.b_g2 = calloc(25 * V, 8);
  pk.ic_g1 = calloc(13 * V, 8);
  pk.h_g1 = calloc(13 * n, 8);
  vk.ic_g1 = calloc(13 * (np + 1), 8);
  CHECK(or_setup(&cs, params, np, &pk, &vk, 4) == OR_OK);
  uint64_t *z = calloc(4 * V, 8), rs[8], proof1[51], proof4[51];
  or_synthetic_witness(n, 12, z);
  or_random_fr(rs, 2, 13);
  or_set_threads(1);
  CHECK(or_prove(&pk, &cs, z, V, np, rs, rs + 4, proof1) == OR_OK);
  or_set_threads(4);
  CHECK(or_prove(&pk, &cs, z, V, np, rs, rs + 4, proof4) == OR_OK);
  CHECK(memcmp(proof1, proof4, sizeof proof1) == 0);
  uint8_t comp[48];
  or_g1_compress(comp, proof1);
  uint8_t comp2[96];
  or_g2_compress(comp2, proof1 + 13);
  /* sparse vs literal dense quotient, and a rejected witness */
  uint64_t *h = calloc(4 * n, 8), *hd = calloc(4 * n, 8);
  CHECK(or_quotient(&cs, z, h) == OR_OK);
  CHECK(or_quotient_dense(&cs, z, hd) == OR_OK);
  CHECK(memcmp(h, hd, 32 * n) == 0);
  z[4 * 6] ^= 1;
  CHECK(or_validate(&cs, z, V) == OR_ERR_INVALID_WITNESS);
  CHECK(or_quotient(&cs, z, h) == OR_ERR_QAP_DIVISION);
  /* MSMs and FFTs over every size 1 .. 2^13, both thread counts */
  const uint64_t m = 1 << 13;
  uint64_t *bases = calloc(13 * m, 8), *sc = calloc(4 * m, 8), *x = calloc(4 * m, 8), *y = calloc(4 * m, 8);
  uint64_t a[4] = {123, 0, 0, 0}, b[4] = {456, 0, 0, 0}, out1[13], out4[13];
  or_g1_lin_bases(bases, a, b, m);
  or_random_fr(sc, m, 14);
  for (uint64_t k = 1; k <= m; k <<= 2) {
    or_set_threads(1);
    or_msm_g1(out1, bases, sc, k);
    or_set_threads(4);
    or_msm_g1(out4, bases, sc, k);
    CHECK(memcmp(out1, out4, sizeof out1) == 0);
  }
  uint64_t g2[25], q[25];
  or_g2_generator(g2);
  or_g2_mul(q, g2, a);
  CHECK(or_g2_on_curve(q));
  or_msm_g2(g2, pk.b_g2, sc, V);
  or_random_fr(x, m, 15);
  for (uint32_t L = 0; L <= 13; L++) {
    memcpy(y, x, 32ull << L);
    or_fft(y, L, 0);
    or_fft(y, L, 1);
    CHECK(memcmp(x, y, 32ull << L) == 0);
    uint64_t g[4] = {7, 0, 0, 0};
    or_coset_fft(y, L, 0, g);
    or_coset_fft(y, L, 1, g);
    CHECK(memcmp(x, y, 32ull << L) == 0);
  }
  free(rp); free(vals); free(ac); free(bc); free(cc);
  free(pk.a_g1); free(pk.b_g1); free(pk.b_g2); free(pk.ic_g1); free(pk.h_g1); free(vk.ic_g1);
  free(z); free(h); free(hd); free(bases); free(sc); free(x); free(y);
  printf("oracle sanitizer check ok\n");
  return 0;
}
