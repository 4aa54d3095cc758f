/*
 * zk_oracle.c -- CPU restatement of the reference Groth16 prove() hot path.
 * TEST INFRASTRUCTURE ONLY (see zk_oracle.h for scope, citations and the
 * parity-pinning status).  Plain C11 + unsigned __int128.
 *
 * Field representation mirrors ark-ff 0.4.2 (upstream, Cargo.lock:118):
 * Fp<MontBackend<_, N>, N>, Montgomery form with R = 2^(64N), little-endian
 * u64 limbs.  Fr: N = 4, Fq: N = 6, Fq2 = Fq[u]/(u^2 + 1).
 */
#include "zk_oracle.h"
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* multi-precision helpers                                                  */
/* ------------------------------------------------------------------------ */
static inline u64 mp_add(u64 *o, const u64 *a, const u64 *b, int n) {
  u64 c = 0;
  for (int i = 0; i < n; i++) { u128 s = (u128)a[i] + b[i] + c; o[i] = (u64)s; c = (u64)(s >> 64); }
  return c;
}
static inline u64 mp_sub(u64 *o, const u64 *a, const u64 *b, int n) {
  u64 br = 0;
  for (int i = 0; i < n; i++) { u128 d = (u128)a[i] - b[i] - br; o[i] = (u64)d; br = (u64)(d >> 64) & 1; }
  return br;
}
static inline int mp_geq(const u64 *a, const u64 *b, int n) {
  for (int i = n - 1; i >= 0; i--) { if (a[i] > b[i]) return 1; if (a[i] < b[i]) return 0; }
  return 1;
}
static inline int mp_is_zero(const u64 *a, int n) {
  u64 x = 0; for (int i = 0; i < n; i++) x |= a[i]; return x == 0;
}
static inline void mod_add(u64 *o, const u64 *a, const u64 *b, const u64 *m, int n) {
  u64 c = mp_add(o, a, b, n);
  if (c || mp_geq(o, m, n)) mp_sub(o, o, m, n);
}
static inline void mod_sub(u64 *o, const u64 *a, const u64 *b, const u64 *m, int n) {
  if (mp_sub(o, a, b, n)) mp_add(o, o, m, n);
}
/* CIOS Montgomery multiplication, o = a*b/R mod m */
static inline void mont_mul(u64 *o, const u64 *a, const u64 *b, const u64 *m, u64 minv, int n) {
  u64 t[8] = {0};
  for (int i = 0; i < n; i++) {
    u64 c = 0;
    for (int j = 0; j < n; j++) { u128 s = (u128)a[j] * b[i] + t[j] + c; t[j] = (u64)s; c = (u64)(s >> 64); }
    u128 s = (u128)t[n] + c; t[n] = (u64)s; t[n + 1] = (u64)(s >> 64);
    u64 q = t[0] * minv;
    s = (u128)q * m[0] + t[0]; c = (u64)(s >> 64);
    for (int j = 1; j < n; j++) { s = (u128)q * m[j] + t[j] + c; t[j - 1] = (u64)s; c = (u64)(s >> 64); }
    s = (u128)t[n] + c; t[n - 1] = (u64)s; t[n] = t[n + 1] + (u64)(s >> 64);
  }
  if (t[n] || mp_geq(t, m, n)) mp_sub(t, t, m, n);
  memcpy(o, t, sizeof(u64) * n);
}

static int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  return ch - 'A' + 10;
}
/* big-endian hex string (no 0x) -> n little-endian limbs */
static void from_hex(u64 *o, const char *h, int n) {
  memset(o, 0, sizeof(u64) * n);
  int len = (int)strlen(h);
  for (int i = 0; i < len; i++) {
    int nib = hexval(h[len - 1 - i]);
    o[i / 16] |= (u64)nib << (4 * (i % 16));
  }
}

/* ------------------------------------------------------------------------ */
/* Fr (BLS12-381 scalar field), Fq (base field), Fq2                        */
/* ------------------------------------------------------------------------ */
typedef struct { u64 l[4]; } fr;
typedef struct { u64 l[6]; } fq;
typedef struct { fq c0, c1; } fq2;

static u64 FR_M[4], FQ_M[6];
static const u64 FR_INV = 0xfffffffeffffffffULL;   /* -r^-1 mod 2^64 */
static const u64 FQ_INV = 0x89f3fffcfffcfffdULL;   /* -p^-1 mod 2^64 */
static fr FR_ONE, FR_R2;
static fq FQ_ONE, FQ_R2;

static inline void fr_add(fr *o, const fr *a, const fr *b) { mod_add(o->l, a->l, b->l, FR_M, 4); }
static inline void fr_sub(fr *o, const fr *a, const fr *b) { mod_sub(o->l, a->l, b->l, FR_M, 4); }
static inline void fr_mul(fr *o, const fr *a, const fr *b) { mont_mul(o->l, a->l, b->l, FR_M, FR_INV, 4); }
static inline int fr_is_zero(const fr *a) { return mp_is_zero(a->l, 4); }
static inline int fr_eq(const fr *a, const fr *b) { return memcmp(a, b, sizeof(fr)) == 0; }
static void fr_to_mont(fr *o, const u64 *canon) { fr t; memcpy(t.l, canon, 32); fr_mul(o, &t, &FR_R2); }
static void fr_from_mont(u64 *canon, const fr *a) { fr one = {{1, 0, 0, 0}}; fr t; fr_mul(&t, a, &one); memcpy(canon, t.l, 32); }
static void fr_from_u64(fr *o, u64 v) { u64 c[4] = {v, 0, 0, 0}; fr_to_mont(o, c); }
static void fr_pow(fr *o, const fr *a, const u64 *e, int nl) {
  fr acc = FR_ONE;
  for (int i = 64 * nl - 1; i >= 0; i--) {
    fr_mul(&acc, &acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fr_mul(&acc, &acc, a);
  }
  *o = acc;
}
static void fr_inv(fr *o, const fr *a) {
  u64 e[4]; u64 two[4] = {2, 0, 0, 0}; mp_sub(e, FR_M, two, 4);
  fr_pow(o, a, e, 4);
}
/* lo64 idiom: Fr::from(x.into_bigint().as_ref()[0]) (core:156-161 etc.) */
static inline u64 fr_lo64(const fr *a) { u64 c[4]; fr_from_mont(c, a); return c[0]; }

static inline void fq_add(fq *o, const fq *a, const fq *b) { mod_add(o->l, a->l, b->l, FQ_M, 6); }
static inline void fq_sub(fq *o, const fq *a, const fq *b) { mod_sub(o->l, a->l, b->l, FQ_M, 6); }
static inline void fq_mul(fq *o, const fq *a, const fq *b) { mont_mul(o->l, a->l, b->l, FQ_M, FQ_INV, 6); }
static inline void fq_sqr(fq *o, const fq *a) { fq_mul(o, a, a); }
static inline int fq_is_zero(const fq *a) { return mp_is_zero(a->l, 6); }
static inline int fq_eq(const fq *a, const fq *b) { return memcmp(a, b, sizeof(fq)) == 0; }
static inline void fq_set_zero(fq *a) { memset(a, 0, sizeof(fq)); }
static inline void fq_set_one(fq *a) { *a = FQ_ONE; }
static inline void fq_neg(fq *o, const fq *a) {
  if (fq_is_zero(a)) { fq_set_zero(o); return; }
  mp_sub(o->l, FQ_M, a->l, 6);
}
static void fq_to_mont(fq *o, const u64 *canon) { fq t; memcpy(t.l, canon, 48); fq_mul(o, &t, &FQ_R2); }
static void fq_from_mont(u64 *canon, const fq *a) { fq one = {{1, 0, 0, 0, 0, 0}}; fq t; fq_mul(&t, a, &one); memcpy(canon, t.l, 48); }
static void fq_inv(fq *o, const fq *a) {
  u64 e[6]; u64 two[6] = {2, 0, 0, 0, 0, 0}; mp_sub(e, FQ_M, two, 6);
  fq acc = FQ_ONE;
  for (int i = 383; i >= 0; i--) {
    fq_mul(&acc, &acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fq_mul(&acc, &acc, a);
  }
  *o = acc;
}

static inline void fq2_add(fq2 *o, const fq2 *a, const fq2 *b) { fq_add(&o->c0, &a->c0, &b->c0); fq_add(&o->c1, &a->c1, &b->c1); }
static inline void fq2_sub(fq2 *o, const fq2 *a, const fq2 *b) { fq_sub(&o->c0, &a->c0, &b->c0); fq_sub(&o->c1, &a->c1, &b->c1); }
static inline void fq2_mul(fq2 *o, const fq2 *a, const fq2 *b) {
  fq t0, t1, s0, s1, m;
  fq_mul(&t0, &a->c0, &b->c0);
  fq_mul(&t1, &a->c1, &b->c1);
  fq_add(&s0, &a->c0, &a->c1);
  fq_add(&s1, &b->c0, &b->c1);
  fq_mul(&m, &s0, &s1);
  fq_sub(&o->c0, &t0, &t1);           /* u^2 = -1 */
  fq_sub(&m, &m, &t0);
  fq_sub(&o->c1, &m, &t1);
}
static inline void fq2_sqr(fq2 *o, const fq2 *a) { fq2_mul(o, a, a); }
static inline int fq2_is_zero(const fq2 *a) { return fq_is_zero(&a->c0) && fq_is_zero(&a->c1); }
static inline int fq2_eq(const fq2 *a, const fq2 *b) { return fq_eq(&a->c0, &b->c0) && fq_eq(&a->c1, &b->c1); }
static inline void fq2_set_zero(fq2 *a) { fq_set_zero(&a->c0); fq_set_zero(&a->c1); }
static inline void fq2_set_one(fq2 *a) { fq_set_one(&a->c0); fq_set_zero(&a->c1); }
static inline void fq2_neg(fq2 *o, const fq2 *a) { fq_neg(&o->c0, &a->c0); fq_neg(&o->c1, &a->c1); }
static void fq2_inv(fq2 *o, const fq2 *a) {
  fq t0, t1, n;
  fq_sqr(&t0, &a->c0); fq_sqr(&t1, &a->c1); fq_add(&n, &t0, &t1);
  fq_inv(&n, &n);
  fq_mul(&o->c0, &a->c0, &n);
  fq_mul(&t1, &a->c1, &n); fq_neg(&o->c1, &t1);
}

/* OpenMP threads for the MSM chunks, FFT butterflies and point loads.
 * 1 = the reference's single-threaded arkworks build (Cargo.lock:101-113,
 * 161-170: no `parallel` feature); or_set_threads raises it for tests and
 * the all-core CPU baseline.  Results never depend on it. */
static int g_nthreads = 1;
void or_set_threads(int n) { g_nthreads = n > 0 ? n : 1; }
int or_get_threads(void) { return g_nthreads; }
#define OMP_T(n, min_per) (g_nthreads > 1 && (n) >= (u64)(min_per) * 2 ? g_nthreads : 1)

/* ark_std::log2: exact for powers of two, else ceil */
static u64 ark_log2(u64 x) {
  if (x <= 1) return 0;
  if ((x & (x - 1)) == 0) return (u64)__builtin_ctzll(x);
  return 64 - (u64)__builtin_clzll(x - 1);
}

/* ark-ec 0.4.2 make_digits (upstream), restated */
static void make_digits(const u64 *s, int w, int num_bits, int32_t *dig) {
  u64 radix = 1ULL << w, mask = radix - 1, carry = 0;
  int cnt = (num_bits + w - 1) / w;
  for (int i = 0; i < cnt; i++) {
    int off = i * w, li = off / 64, bi = off % 64;
    u64 buf;
    if (bi < 64 - w || li == 3) buf = s[li] >> bi;
    else buf = (s[li] >> bi) | (s[li + 1] << (64 - bi));
    u64 coef = carry + (buf & mask);
    carry = (coef + radix / 2) >> w;
    dig[i] = (int32_t)((int64_t)coef - (int64_t)(carry << w));
  }
  dig[cnt - 1] += (int32_t)(carry << w);
}

/* ------------------------------------------------------------------------ */
/* curves                                                                   */
/* ------------------------------------------------------------------------ */
static fq G1_B;      /* 4 */
static fq2 G2_B;     /* 4(1+u) */

#define F fq
#define FP(op) fq_##op
#define G(op) g1_##op
#define CURVE_B (&G1_B)
#include "curve_impl.h"
#undef F
#undef FP
#undef G
#undef CURVE_B

#define F fq2
#define FP(op) fq2_##op
#define G(op) g2_##op
#define CURVE_B (&G2_B)
#include "curve_impl.h"
#undef F
#undef FP
#undef G
#undef CURVE_B

static g1_aff G1_GEN;
static g2_aff G2_GEN;

/* interface <-> internal conversions (13 / 25 word canonical layout) */
static void g1_load(g1_aff *o, const u64 *w) {
  o->inf = (int)(w[12] & 0xff);
  if (o->inf) { fq_set_zero(&o->x); fq_set_zero(&o->y); return; }
  fq_to_mont(&o->x, w); fq_to_mont(&o->y, w + 6);
}
static void g1_store(u64 *w, const g1_aff *a) {
  memset(w, 0, 13 * 8);
  if (a->inf) { w[12] = 1; return; }
  fq_from_mont(w, &a->x); fq_from_mont(w + 6, &a->y);
}
static void g2_load(g2_aff *o, const u64 *w) {
  o->inf = (int)(w[24] & 0xff);
  if (o->inf) { fq2_set_zero(&o->x); fq2_set_zero(&o->y); return; }
  fq_to_mont(&o->x.c0, w); fq_to_mont(&o->x.c1, w + 6);
  fq_to_mont(&o->y.c0, w + 12); fq_to_mont(&o->y.c1, w + 18);
}
static void g2_store(u64 *w, const g2_aff *a) {
  memset(w, 0, 25 * 8);
  if (a->inf) { w[24] = 1; return; }
  fq_from_mont(w, &a->x.c0); fq_from_mont(w + 6, &a->x.c1);
  fq_from_mont(w + 12, &a->y.c0); fq_from_mont(w + 18, &a->y.c1);
}

/* ------------------------------------------------------------------------ */
/* init                                                                     */
/* ------------------------------------------------------------------------ */
static int g_inited = 0;
static fr FR_TWO_ADIC_ROOT;   /* 7^((r-1)/2^32), ark FrConfig GENERATOR = 7 */
static fr FR_GEN;             /* 7 */

static void init_mont_consts(u64 *one, u64 *r2, const u64 *m, int n, int bits) {
  /* one = 2^bits mod m, r2 = 2^(2 bits) mod m, by doubling */
  u64 x[8] = {1};
  for (int i = 0; i < 2 * bits; i++) {
    mod_add(x, x, x, m, n);
    if (i == bits - 1) memcpy(one, x, sizeof(u64) * n);
  }
  memcpy(r2, x, sizeof(u64) * n);
}

void or_init(void) {
  if (g_inited) return;
  from_hex(FR_M, "73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001", 4);
  from_hex(FQ_M, "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 6);
  init_mont_consts(FR_ONE.l, FR_R2.l, FR_M, 4, 256);
  init_mont_consts(FQ_ONE.l, FQ_R2.l, FQ_M, 6, 384);
  u64 four[6] = {4, 0, 0, 0, 0, 0};
  fq_to_mont(&G1_B, four);
  fq_to_mont(&G2_B.c0, four);
  G2_B.c1 = G2_B.c0;
  u64 t[6];
  from_hex(t, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb", 6);
  fq_to_mont(&G1_GEN.x, t);
  from_hex(t, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1", 6);
  fq_to_mont(&G1_GEN.y, t);
  G1_GEN.inf = 0;
  from_hex(t, "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8", 6);
  fq_to_mont(&G2_GEN.x.c0, t);
  from_hex(t, "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e", 6);
  fq_to_mont(&G2_GEN.x.c1, t);
  from_hex(t, "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801", 6);
  fq_to_mont(&G2_GEN.y.c0, t);
  from_hex(t, "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be", 6);
  fq_to_mont(&G2_GEN.y.c1, t);
  G2_GEN.inf = 0;
  fr_from_u64(&FR_GEN, 7);
  u64 e[4]; u64 one[4] = {1, 0, 0, 0};
  mp_sub(e, FR_M, one, 4);                 /* (r-1) >> 32 */
  for (int i = 0; i < 4; i++) e[i] = (e[i] >> 32) | (i < 3 ? (e[i + 1] << 32) : 0);
  fr_pow(&FR_TWO_ADIC_ROOT, &FR_GEN, e, 4);
  g_inited = 1;
}

/* omega_n for n = 2^log_n: two_adic_root^(2^(32-log_n)) (ark get_root_of_unity) */
static void fr_root(fr *o, uint32_t log_n) {
  fr w = FR_TWO_ADIC_ROOT;
  for (uint32_t i = log_n; i < 32; i++) fr_mul(&w, &w, &w);
  *o = w;
}

/* ------------------------------------------------------------------------ */
/* exported field / curve helpers                                           */
/* ------------------------------------------------------------------------ */
void or_fr_mul(u64 out[4], const u64 a[4], const u64 b[4]) { fr x, y; fr_to_mont(&x, a); fr_to_mont(&y, b); fr_mul(&x, &x, &y); fr_from_mont(out, &x); }
void or_fr_add(u64 out[4], const u64 a[4], const u64 b[4]) { fr x, y; fr_to_mont(&x, a); fr_to_mont(&y, b); fr_add(&x, &x, &y); fr_from_mont(out, &x); }
void or_fr_sub(u64 out[4], const u64 a[4], const u64 b[4]) { fr x, y; fr_to_mont(&x, a); fr_to_mont(&y, b); fr_sub(&x, &x, &y); fr_from_mont(out, &x); }
int or_fr_inv(u64 out[4], const u64 a[4]) {
  fr x; fr_to_mont(&x, a);
  if (fr_is_zero(&x)) { memset(out, 0, 32); return -1; }
  fr_inv(&x, &x); fr_from_mont(out, &x); return 0;
}
void or_fr_from_u64(u64 out[4], u64 v) { memset(out, 0, 32); out[0] = v; }
void or_fr_root_of_unity(u64 out[4], uint32_t log_n) { fr w; fr_root(&w, log_n); fr_from_mont(out, &w); }
void or_fq_mul(u64 out[6], const u64 a[6], const u64 b[6]) { fq x, y; fq_to_mont(&x, a); fq_to_mont(&y, b); fq_mul(&x, &x, &y); fq_from_mont(out, &x); }
void or_fq_inv(u64 out[6], const u64 a[6]) { fq x; fq_to_mont(&x, a); fq_inv(&x, &x); fq_from_mont(out, &x); }

void or_g1_generator(u64 out[13]) { g1_store(out, &G1_GEN); }
void or_g2_generator(u64 out[25]) { g2_store(out, &G2_GEN); }
int or_g1_on_curve(const u64 p[13]) { g1_aff a; g1_load(&a, p); return g1_aff_on_curve(&a); }
int or_g2_on_curve(const u64 p[25]) { g2_aff a; g2_load(&a, p); return g2_aff_on_curve(&a); }
void or_g1_add(u64 out[13], const u64 a[13], const u64 b[13]) {
  g1_aff x, y; g1_jac j; g1_load(&x, a); g1_load(&y, b);
  g1_from_aff(&j, &x); g1_madd(&j, &j, &y); g1_to_aff(&x, &j); g1_store(out, &x);
}
void or_g2_add(u64 out[25], const u64 a[25], const u64 b[25]) {
  g2_aff x, y; g2_jac j; g2_load(&x, a); g2_load(&y, b);
  g2_from_aff(&j, &x); g2_madd(&j, &j, &y); g2_to_aff(&x, &j); g2_store(out, &x);
}
void or_g1_mul(u64 out[13], const u64 p[13], const u64 k[4]) {
  g1_aff a; g1_jac j; g1_load(&a, p); g1_from_aff(&j, &a); g1_mul_bits(&j, &j, k, 256); g1_to_aff(&a, &j); g1_store(out, &a);
}
void or_g2_mul(u64 out[25], const u64 p[25], const u64 k[4]) {
  g2_aff a; g2_jac j; g2_load(&a, p); g2_from_aff(&j, &a); g2_mul_bits(&j, &j, k, 256); g2_to_aff(&a, &j); g2_store(out, &a);
}

/* bases[i] = (a + i b) G1 for i < n (the closed-form MSM KAT of SURVEY
 * 8(d): sum_i s_i bases[i] = (a sum s_i + b sum i s_i) G1).  Each of
 * g_nthreads chunks starts from (a + lo b) G1 and steps by b G1; one batch
 * inversion per chunk. */
void or_g1_lin_bases(u64 *out, const u64 a[4], const u64 b[4], u64 n) {
  if (n == 0) return;
  fr am, bm; fr_to_mont(&am, a); fr_to_mont(&bm, b);
  g1_jac gj; g1_from_aff(&gj, &G1_GEN);
  g1_jac bj; g1_aff bstep;
  g1_mul_bits(&bj, &gj, b, 256); g1_to_aff(&bstep, &bj);
  int T = OMP_T(n, 4096);
#pragma omp parallel for schedule(static) num_threads(T)
  for (int t = 0; t < T; t++) {
    u64 lo = n * (u64)t / (u64)T, hi = n * (u64)(t + 1) / (u64)T;
    if (lo >= hi) continue;
    fr k, lo_m; fr_from_u64(&lo_m, lo); fr_mul(&k, &lo_m, &bm); fr_add(&k, &k, &am);
    u64 kc[4]; fr_from_mont(kc, &k);
    g1_jac *J = (g1_jac *)malloc(sizeof(g1_jac) * (hi - lo));
    g1_aff *A = (g1_aff *)malloc(sizeof(g1_aff) * (hi - lo));
    g1_jac p; g1_mul_bits(&p, &gj, kc, 256);
    for (u64 i = lo; i < hi; i++) { J[i - lo] = p; g1_madd(&p, &p, &bstep); }
    g1_batch_to_aff(A, J, hi - lo);
    for (u64 i = lo; i < hi; i++) g1_store(out + 13 * i, &A[i - lo]);
    free(J); free(A);
  }
}

/* zcash / ark-bls12-381 0.4 compressed encoding: big-endian x with flags in the
 * top bits of byte 0: 0x80 compressed, 0x40 infinity, 0x20 y lexicographically
 * largest (y > (p-1)/2; for Fq2 compare c1 first, then c0). */
static void be48(uint8_t *o, const u64 *l) {
  for (int i = 0; i < 48; i++) o[i] = (uint8_t)(l[(47 - i) / 8] >> (8 * ((47 - i) % 8)));
}
static int fq_canon_largest(const u64 *c) {
  u64 half[6]; memcpy(half, FQ_M, 48);
  for (int i = 0; i < 6; i++) half[i] = (half[i] >> 1) | (i < 5 ? (half[i + 1] << 63) : 0);
  /* (p-1)/2 == p >> 1 for odd p */
  return !mp_geq(half, c, 6);
}
void or_g1_compress(uint8_t out[48], const u64 p[13]) {
  memset(out, 0, 48);
  if (p[12] & 0xff) { out[0] = 0xc0; return; }
  be48(out, p);
  out[0] |= 0x80;
  if (fq_canon_largest(p + 6)) out[0] |= 0x20;
}
void or_g2_compress(uint8_t out[96], const u64 p[25]) {
  memset(out, 0, 96);
  if (p[24] & 0xff) { out[0] = 0xc0; return; }
  be48(out, p + 6);       /* x.c1 first */
  be48(out + 48, p);      /* then x.c0 */
  out[0] |= 0x80;
  const u64 *yc0 = p + 12, *yc1 = p + 18;
  int largest = mp_is_zero(yc1, 6) ? fq_canon_largest(yc0) : fq_canon_largest(yc1);
  if (largest) out[0] |= 0x20;
}

/* ------------------------------------------------------------------------ */
/* MSM                                                                      */
/* ------------------------------------------------------------------------ */
int or_msm_g1(u64 out[13], const u64 *bases, const u64 *scalars, u64 n) {
  g1_aff *b = (g1_aff *)malloc(sizeof(g1_aff) * (n ? n : 1));
  for (u64 i = 0; i < n; i++) g1_load(&b[i], bases + 13 * i);
  g1_jac acc; g1_msm_ark(&acc, b, scalars, n);
  g1_aff a; g1_to_aff(&a, &acc); g1_store(out, &a);
  free(b); return OR_OK;
}
int or_msm_g2(u64 out[25], const u64 *bases, const u64 *scalars, u64 n) {
  g2_aff *b = (g2_aff *)malloc(sizeof(g2_aff) * (n ? n : 1));
  for (u64 i = 0; i < n; i++) g2_load(&b[i], bases + 25 * i);
  g2_jac acc; g2_msm_ark(&acc, b, scalars, n);
  g2_aff a; g2_to_aff(&a, &acc); g2_store(out, &a);
  free(b); return OR_OK;
}

/* ------------------------------------------------------------------------ */
/* FFT (ark-poly Radix2EvaluationDomain semantics, natural order in/out)    */
/* ------------------------------------------------------------------------ */
/* tw[k] = w^k for k < m, in chunks that start from w^lo */
static void pow_table(fr *tw, const fr *w, u64 m) {
  int T = OMP_T(m, 4096);
#pragma omp parallel for schedule(static) num_threads(T)
  for (int t = 0; t < T; t++) {
    u64 lo = m * (u64)t / (u64)T, hi = m * (u64)(t + 1) / (u64)T;
    if (lo >= hi) continue;
    u64 e[1] = {lo};
    fr p; fr_pow(&p, w, e, 1);
    for (u64 k = lo; k < hi; k++) { tw[k] = p; fr_mul(&p, &p, w); }
  }
}
static inline u64 bitrev(u64 x, uint32_t bits) {
  u64 r = 0;
  for (uint32_t i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}
static void fft_mont(fr *a, uint32_t log_n, int inverse) {
  u64 n = 1ULL << log_n;
  int T = OMP_T(n, 4096);
#pragma omp parallel for schedule(static) num_threads(T)
  for (long long i = 0; i < (long long)n; i++) {      /* bit reversal */
    u64 j = bitrev((u64)i, log_n);
    if ((u64)i < j) { fr t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  fr *tw = (fr *)malloc(sizeof(fr) * (n > 1 ? n / 2 : 1));
  for (uint32_t s = 1; s <= log_n; s++) {
    u64 len = 1ULL << s, half = len >> 1;
    fr wl; fr_root(&wl, s);
    if (inverse) fr_inv(&wl, &wl);
    pow_table(tw, &wl, half);
#pragma omp parallel for schedule(static) num_threads(T)
    for (long long b = 0; b < (long long)(n / 2); b++) {
      u64 k = (u64)b & (half - 1), i = ((u64)b >> (s - 1)) * len + k;
      fr u = a[i], v;
      fr_mul(&v, &a[i + half], &tw[k]);
      fr_add(&a[i], &u, &v);
      fr_sub(&a[i + half], &u, &v);
    }
  }
  free(tw);
  if (inverse) {
    fr ninv; fr_from_u64(&ninv, n); fr_inv(&ninv, &ninv);
#pragma omp parallel for schedule(static) num_threads(T)
    for (long long i = 0; i < (long long)n; i++) fr_mul(&a[i], &a[i], &ninv);
  }
}
static void coset_scale(fr *a, u64 n, const fr *g) {
  int T = OMP_T(n, 4096);
#pragma omp parallel for schedule(static) num_threads(T)
  for (int t = 0; t < T; t++) {
    u64 lo = n * (u64)t / (u64)T, hi = n * (u64)(t + 1) / (u64)T;
    if (lo >= hi) continue;
    u64 e[1] = {lo};
    fr p; fr_pow(&p, g, e, 1);
    for (u64 i = lo; i < hi; i++) { fr_mul(&a[i], &a[i], &p); fr_mul(&p, &p, g); }
  }
}

void or_fft(u64 *data, uint32_t log_n, int inverse) {
  u64 n = 1ULL << log_n;
  fr *a = (fr *)malloc(sizeof(fr) * n);
  for (u64 i = 0; i < n; i++) fr_to_mont(&a[i], data + 4 * i);
  fft_mont(a, log_n, inverse);
  for (u64 i = 0; i < n; i++) fr_from_mont(data + 4 * i, &a[i]);
  free(a);
}
void or_coset_fft(u64 *data, uint32_t log_n, int inverse, const u64 g[4]) {
  u64 n = 1ULL << log_n;
  fr *a = (fr *)malloc(sizeof(fr) * n);
  fr gm; fr_to_mont(&gm, g);
  for (u64 i = 0; i < n; i++) fr_to_mont(&a[i], data + 4 * i);
  if (!inverse) { coset_scale(a, n, &gm); fft_mont(a, log_n, 0); }
  else { fr gi; fr_inv(&gi, &gm); fft_mont(a, log_n, 1); coset_scale(a, n, &gi); }
  for (u64 i = 0; i < n; i++) fr_from_mont(data + 4 * i, &a[i]);
  free(a);
}

/* ------------------------------------------------------------------------ */
/* R1CS / QAP                                                               */
/* ------------------------------------------------------------------------ */
/* Rust usize::next_power_of_two (0 -> 1) as used by qap:100 */
u64 or_domain_size(u64 nc) {
  u64 n = 1;
  while (n < nc) n <<= 1;
  return n;
}
static uint32_t log2_exact(u64 n) { return (uint32_t)__builtin_ctzll(n); }

static void csr_coeff(fr *o, const u64 *val, u64 k) {
  if (!val) { *o = FR_ONE; return; }
  fr_to_mont(o, val + 4 * k);
}
/* (Mz)_row for one matrix, cols >= V dropped (qap:122-124) */
static void csr_row_dot(fr *o, const u64 *rp, const uint32_t *col, const u64 *val,
                        u64 row, const fr *zm, u64 V) {
  fr acc = {{0}};
  for (u64 k = rp[row]; k < rp[row + 1]; k++) {
    if (col[k] >= V) continue;
    fr c, t; csr_coeff(&c, val, k);
    fr_mul(&t, &c, &zm[col[k]]);
    fr_add(&acc, &acc, &t);
  }
  *o = acc;
}

static fr *load_z(const u64 *z, u64 V) {
  fr *zm = (fr *)malloc(sizeof(fr) * (V ? V : 1));
#pragma omp parallel for schedule(static) num_threads(OMP_T(V, 4096))
  for (long long i = 0; i < (long long)V; i++) fr_to_mont(&zm[i], z + 4 * i);
  return zm;
}

int or_validate(const or_r1cs *cs, const u64 *z, u64 zlen) {
  if (zlen != cs->num_variables) return OR_ERR_INVALID_WITNESS;
  u64 n = or_domain_size(cs->num_constraints);
  u64 row = n > 1 ? 1 : 0;      /* evaluate_at(omega) picks domain point omega^1 */
  if (row >= cs->num_constraints) return OR_OK;   /* padded zero row: 0*0 == 0 */
  fr *zm = load_z(z, zlen);
  fr a, b, c, ab;
  csr_row_dot(&a, cs->a_rowptr, cs->a_col, cs->a_val, row, zm, zlen);
  csr_row_dot(&b, cs->b_rowptr, cs->b_col, cs->b_val, row, zm, zlen);
  csr_row_dot(&c, cs->c_rowptr, cs->c_col, cs->c_val, row, zm, zlen);
  free(zm);
  fr_mul(&ab, &a, &b);
  return fr_eq(&ab, &c) ? OR_OK : OR_ERR_INVALID_WITNESS;
}

/* H = (A*B - C)/(x^n - 1) via iFFT -> coset FFT -> divide -> coset iFFT.
 * Output: n canonical coefficients (coefficient n-1 is always 0). */
static int quotient_mont(const or_r1cs *cs, const fr *zm, u64 V, fr *h) {
  u64 nc = cs->num_constraints, n = or_domain_size(nc);
  uint32_t ln = log2_exact(n);
  fr *a = (fr *)calloc(n, sizeof(fr)), *b = (fr *)calloc(n, sizeof(fr)), *c = (fr *)calloc(n, sizeof(fr));
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad) num_threads(OMP_T(nc, 4096))
  for (long long jj = 0; jj < (long long)nc; jj++) {
    u64 j = (u64)jj;
    csr_row_dot(&a[j], cs->a_rowptr, cs->a_col, cs->a_val, j, zm, V);
    csr_row_dot(&b[j], cs->b_rowptr, cs->b_col, cs->b_val, j, zm, V);
    csr_row_dot(&c[j], cs->c_rowptr, cs->c_col, cs->c_val, j, zm, V);
    fr ab; fr_mul(&ab, &a[j], &b[j]);
    if (!fr_eq(&ab, &c[j])) bad = 1;
  }
  if (bad) { free(a); free(b); free(c); return OR_ERR_QAP_DIVISION; }
  fr *v[3] = {a, b, c};
  for (int k = 0; k < 3; k++) {
    fft_mont(v[k], ln, 1);
    coset_scale(v[k], n, &FR_GEN);
    fft_mont(v[k], ln, 0);
  }
  /* Z(g w^i) = g^n - 1 */
  fr gn = FR_ONE, zinv;
  for (u64 i = 0; i < n; i++) fr_mul(&gn, &gn, &FR_GEN);
  fr_sub(&zinv, &gn, &FR_ONE); fr_inv(&zinv, &zinv);
#pragma omp parallel for schedule(static) num_threads(OMP_T(n, 4096))
  for (long long i = 0; i < (long long)n; i++) {
    fr t; fr_mul(&t, &a[i], &b[i]); fr_sub(&t, &t, &c[i]); fr_mul(&h[i], &t, &zinv);
  }
  fft_mont(h, ln, 1);
  fr gi; fr_inv(&gi, &FR_GEN);
  coset_scale(h, n, &gi);
  free(a); free(b); free(c);
  return OR_OK;
}

int or_quotient(const or_r1cs *cs, const u64 *z, u64 *h_out) {
  u64 V = cs->num_variables, n = or_domain_size(cs->num_constraints);
  fr *zm = load_z(z, V);
  fr *h = (fr *)malloc(sizeof(fr) * n);
  int rc = quotient_mont(cs, zm, V, h);
  if (rc == OR_OK) for (u64 i = 0; i < n; i++) fr_from_mont(h_out + 4 * i, &h[i]);
  free(zm); free(h);
  return rc;
}

/* Literal restatement of QAP::from_r1cs (qap:95-187) + compute_quotient_polynomial
 * (qap:225-271): dense columns, per-variable iFFT, dense scaled sums,
 * schoolbook A*B - C, long division by x^n - 1.  O(V n + n^2): small n only. */
int or_quotient_dense(const or_r1cs *cs, const u64 *z, u64 *h_out) {
  u64 nc = cs->num_constraints, V = cs->num_variables, n = or_domain_size(nc);
  uint32_t ln = log2_exact(n);
  fr *zm = load_z(z, V);
  fr *A = (fr *)calloc(n, sizeof(fr)), *B = (fr *)calloc(n, sizeof(fr)), *C = (fr *)calloc(n, sizeof(fr));
  fr *col = (fr *)malloc(sizeof(fr) * n);
  const u64 *rps[3] = {cs->a_rowptr, cs->b_rowptr, cs->c_rowptr};
  const uint32_t *cols[3] = {cs->a_col, cs->b_col, cs->c_col};
  const u64 *vals[3] = {cs->a_val, cs->b_val, cs->c_val};
  fr *acc[3] = {A, B, C};
  for (int m = 0; m < 3; m++) {
    for (u64 i = 0; i < V; i++) {
      if (fr_is_zero(&zm[i])) continue;               /* qap:238 */
      memset(col, 0, sizeof(fr) * n);
      for (u64 j = 0; j < nc; j++)
        for (u64 k = rps[m][j]; k < rps[m][j + 1]; k++)
          if (cols[m][k] == i) csr_coeff(&col[j], vals[m], k);
      fft_mont(col, ln, 1);                               /* qap:167-169 */
      for (u64 j = 0; j < n; j++) { fr t; fr_mul(&t, &col[j], &zm[i]); fr_add(&acc[m][j], &acc[m][j], &t); }
    }
  }
  /* numerator = A*B - C, degree <= 2n-2 */
  u64 nn = 2 * n;
  fr *N = (fr *)calloc(nn, sizeof(fr));
  for (u64 i = 0; i < n; i++)
    for (u64 j = 0; j < n; j++) { fr t; fr_mul(&t, &A[i], &B[j]); fr_add(&N[i + j], &N[i + j], &t); }
  for (u64 i = 0; i < n; i++) fr_sub(&N[i], &N[i], &C[i]);
  /* divide by x^n - 1: q[i-n] += N[i], N[i-n] += N[i], from the top */
  fr *q = (fr *)calloc(n, sizeof(fr));
  for (u64 i = nn; i-- > n;) {
    q[i - n] = N[i];
    fr_add(&N[i - n], &N[i - n], &N[i]);
    memset(&N[i], 0, sizeof(fr));
  }
  int bad = 0;
  for (u64 i = 0; i < n; i++) if (!fr_is_zero(&N[i])) bad = 1;
  if (!bad) for (u64 i = 0; i < n; i++) fr_from_mont(h_out + 4 * i, &q[i]);
  free(zm); free(A); free(B); free(C); free(col); free(N); free(q);
  return bad ? OR_ERR_QAP_DIVISION : OR_OK;
}

/* Lagrange basis of the size-n domain at t: L_j(t) = w^j (t^n - 1) / (n (t - w^j)) */
static void lagrange_at(fr *L, u64 n, const fr *t) {
  fr w; fr_root(&w, log2_exact(n));
  fr tn = *t;
  for (u64 i = 1; i < n; i <<= 1) fr_mul(&tn, &tn, &tn);
  fr zt; fr_sub(&zt, &tn, &FR_ONE);
  fr wj = FR_ONE;
  if (fr_is_zero(&zt)) {                               /* t is a domain point */
    for (u64 j = 0; j < n; j++) { L[j] = fr_eq(&wj, t) ? FR_ONE : (fr){{0}}; fr_mul(&wj, &wj, &w); }
    return;
  }
  fr *den = (fr *)malloc(sizeof(fr) * n), *pre = (fr *)malloc(sizeof(fr) * n);
  fr *wp = (fr *)malloc(sizeof(fr) * n);
  for (u64 j = 0; j < n; j++) { wp[j] = wj; fr_sub(&den[j], t, &wj); fr_mul(&wj, &wj, &w); }
  fr run = FR_ONE;
  for (u64 j = 0; j < n; j++) { pre[j] = run; fr_mul(&run, &run, &den[j]); }
  fr inv; fr_inv(&inv, &run);
  fr nn; fr_from_u64(&nn, n); fr_inv(&nn, &nn);
  fr k; fr_mul(&k, &zt, &nn);
  for (u64 j = n; j-- > 0;) {
    fr di; fr_mul(&di, &inv, &pre[j]); fr_mul(&inv, &inv, &den[j]);
    fr_mul(&L[j], &di, &wp[j]); fr_mul(&L[j], &L[j], &k);
  }
  free(den); free(pre); free(wp);
}

static void qap_eval_mont(const or_r1cs *cs, const fr *t, fr *av, fr *bv, fr *cv) {
  u64 nc = cs->num_constraints, V = cs->num_variables, n = or_domain_size(nc);
  fr *L = (fr *)malloc(sizeof(fr) * n);
  lagrange_at(L, n, t);
  memset(av, 0, sizeof(fr) * V); memset(bv, 0, sizeof(fr) * V); memset(cv, 0, sizeof(fr) * V);
  const u64 *rps[3] = {cs->a_rowptr, cs->b_rowptr, cs->c_rowptr};
  const uint32_t *cols[3] = {cs->a_col, cs->b_col, cs->c_col};
  const u64 *vals[3] = {cs->a_val, cs->b_val, cs->c_val};
  fr *out[3] = {av, bv, cv};
  for (int m = 0; m < 3; m++)
    for (u64 j = 0; j < nc; j++)
      for (u64 k = rps[m][j]; k < rps[m][j + 1]; k++) {
        if (cols[m][k] >= V) continue;
        fr c, x; csr_coeff(&c, vals[m], k);
        fr_mul(&x, &c, &L[j]);
        fr_add(&out[m][cols[m][k]], &out[m][cols[m][k]], &x);
      }
  free(L);
}

void or_qap_eval_at(const or_r1cs *cs, const u64 t[4], u64 *a_vals, u64 *b_vals, u64 *c_vals) {
  u64 V = cs->num_variables;
  fr tm; fr_to_mont(&tm, t);
  fr *a = (fr *)malloc(sizeof(fr) * V), *b = (fr *)malloc(sizeof(fr) * V), *c = (fr *)malloc(sizeof(fr) * V);
  qap_eval_mont(cs, &tm, a, b, c);
  for (u64 i = 0; i < V; i++) { fr_from_mont(a_vals + 4 * i, &a[i]); fr_from_mont(b_vals + 4 * i, &b[i]); fr_from_mont(c_vals + 4 * i, &c[i]); }
  free(a); free(b); free(c);
}

/* ------------------------------------------------------------------------ */
/* setup: CRS::generate_from_qap (crates/groth16-setup/src/lib.rs:141-268)  */
/* ------------------------------------------------------------------------ */
static void lo64_fr(fr *o, const fr *a) { fr_from_u64(o, fr_lo64(a)); }

int or_setup(const or_r1cs *cs, const u64 params[20], u64 num_public, or_pk *pk, or_vk *vk, int nthreads) {
  (void)nthreads;
  u64 V = cs->num_variables, n = or_domain_size(cs->num_constraints);
  fr P[5];
  for (int i = 0; i < 5; i++) fr_to_mont(&P[i], params + 4 * i);
  /* SetupParams::validate (setup:128-136): alpha, beta, gamma, delta non-zero */
  for (int i = 0; i < 4; i++) if (fr_is_zero(&P[i])) return OR_ERR_SETUP_PARAMS;
  if (num_public >= V) return OR_ERR_SETUP_PARAMS;    /* setup:148-152 */
  fr al, be, ga, de, ta;                               /* setup:155-159 (lo64) */
  lo64_fr(&al, &P[0]); lo64_fr(&be, &P[1]); lo64_fr(&ga, &P[2]); lo64_fr(&de, &P[3]); lo64_fr(&ta, &P[4]);
  /* reference unwraps inverse(delta~), inverse(gamma~): a zero there panics */
  if (fr_is_zero(&de) || fr_is_zero(&ga)) return OR_ERR_SETUP_PARAMS;

  /* full-width generator multiples (setup:166-171) */
  u64 k[4];
  g1_jac g1; g1_from_aff(&g1, &G1_GEN);
  g2_jac g2; g2_from_aff(&g2, &G2_GEN);
  g1_jac j1; g2_jac j2; g1_aff a1; g2_aff a2;
#define G1_FULL(dst, idx) do { fr_from_mont(k, &P[idx]); g1_mul_bits(&j1, &g1, k, 256); g1_to_aff(&a1, &j1); g1_store(dst, &a1); } while (0)
#define G2_FULL(dst, idx) do { fr_from_mont(k, &P[idx]); g2_mul_bits(&j2, &g2, k, 256); g2_to_aff(&a2, &j2); g2_store(dst, &a2); } while (0)
  G1_FULL(pk->alpha_g1, 0); G1_FULL(pk->beta_g1, 1); G2_FULL(pk->beta_g2, 1);
  G1_FULL(pk->delta_g1, 3); G2_FULL(pk->delta_g2, 3);
  memcpy(vk->alpha_g1, pk->alpha_g1, sizeof(pk->alpha_g1));
  memcpy(vk->beta_g2, pk->beta_g2, sizeof(pk->beta_g2));
  G2_FULL(vk->gamma_g2, 2);
  memcpy(vk->delta_g2, pk->delta_g2, sizeof(pk->delta_g2));
#undef G1_FULL
#undef G2_FULL

  /* A_i(tau~), B_i(tau~), C_i(tau~) (setup:174-182) */
  fr *av = (fr *)malloc(sizeof(fr) * V), *bv = (fr *)malloc(sizeof(fr) * V), *cv = (fr *)malloc(sizeof(fr) * V);
  qap_eval_mont(cs, &ta, av, bv, cv);

  g1_aff *t1 = (g1_aff *)malloc(sizeof(g1_aff) * 2048);
  g2_aff *t2 = (g2_aff *)malloc(sizeof(g2_aff) * 2048);
  g1_fb_table(t1, &g1); g2_fb_table(t2, &g2);

  u64 cnt1 = 2 * V + (V - num_public - 1) + (num_public + 1) + n;
  u64 *sc1 = (u64 *)malloc(sizeof(u64) * cnt1);
  u64 *sc2 = (u64 *)malloc(sizeof(u64) * (V ? V : 1));
  u64 p = 0;
  for (u64 i = 0; i < V; i++) sc1[p++] = fr_lo64(&av[i]);                    /* a_g1 setup:185-191 */
  for (u64 i = 0; i < V; i++) { sc1[p++] = fr_lo64(&bv[i]); sc2[i] = fr_lo64(&bv[i]); } /* b_g1, b_g2 setup:194-207 */
  fr dinv, ginv; fr_inv(&dinv, &de); fr_inv(&ginv, &ga);
  for (u64 i = num_public + 1; i < V; i++) {                                 /* pk ic setup:210-218 */
    fr t, u; fr_mul(&t, &be, &av[i]); fr_mul(&u, &al, &bv[i]); fr_add(&t, &t, &u); fr_add(&t, &t, &cv[i]);
    fr_mul(&t, &t, &dinv); sc1[p++] = fr_lo64(&t);
  }
  for (u64 i = 0; i <= num_public; i++) {                                    /* vk ic setup:221-229 */
    fr t, u; fr_mul(&t, &be, &av[i]); fr_mul(&u, &al, &bv[i]); fr_add(&t, &t, &u); fr_add(&t, &t, &cv[i]);
    fr_mul(&t, &t, &ginv); sc1[p++] = fr_lo64(&t);
  }
  fr tp = FR_ONE;                                                             /* h setup:232-241 */
  for (u64 i = 0; i < n; i++) { fr t; fr_mul(&t, &tp, &dinv); sc1[p++] = fr_lo64(&t); fr_mul(&tp, &tp, &ta); }

  g1_jac *J1 = (g1_jac *)malloc(sizeof(g1_jac) * cnt1);
  g1_aff *A1 = (g1_aff *)malloc(sizeof(g1_aff) * cnt1);
  g2_jac *J2 = (g2_jac *)malloc(sizeof(g2_jac) * (V ? V : 1));
  g2_aff *A2 = (g2_aff *)malloc(sizeof(g2_aff) * (V ? V : 1));
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (long long i = 0; i < (long long)cnt1; i++) g1_fb_mul(&J1[i], t1, sc1[i]);
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (long long i = 0; i < (long long)V; i++) g2_fb_mul(&J2[i], t2, sc2[i]);
  g1_batch_to_aff(A1, J1, cnt1);
  g2_batch_to_aff(A2, J2, V);
  p = 0;
  for (u64 i = 0; i < V; i++) g1_store(pk->a_g1 + 13 * i, &A1[p++]);
  for (u64 i = 0; i < V; i++) g1_store(pk->b_g1 + 13 * i, &A1[p++]);
  for (u64 i = 0; i < V - num_public - 1; i++) g1_store(pk->ic_g1 + 13 * i, &A1[p++]);
  for (u64 i = 0; i <= num_public; i++) g1_store(vk->ic_g1 + 13 * i, &A1[p++]);
  for (u64 i = 0; i < n; i++) g1_store(pk->h_g1 + 13 * i, &A1[p++]);
  for (u64 i = 0; i < V; i++) g2_store(pk->b_g2 + 25 * i, &A2[i]);
  pk->a_len = V; pk->b_len = V; pk->b2_len = V; pk->ic_len = V - num_public - 1; pk->h_len = n;
  pk->num_public = num_public;
  vk->ic_len = num_public + 1; vk->num_public = num_public;
  free(av); free(bv); free(cv); free(t1); free(t2); free(sc1); free(sc2);
  free(J1); free(A1); free(J2); free(A2);
  return OR_OK;
}

/* Sampled entries of the same key, for checking a setup too large to
 * restate whole (the sharded 2^24 GPU setup): the base of each listed
 * variable v in a_g1 / b_g1 / b_g2 (setup:185-207) and ic (setup:210-229:
 * pk ic_g1[v - num_public - 1] for v > num_public, the vk's ic_g1[v]
 * otherwise), and of each listed coefficient index i < n in h_g1
 * (setup:232-241), by exactly or_setup's arithmetic: A_i(tau~) etc. from the
 * whole sparse Lagrange pass, lo64 scalars, fixed-base multiples.  Outputs
 * 13 (G1) / 25 (G2) words per sample; NULL outputs are skipped. */
int or_setup_sample(const or_r1cs *cs, const u64 params[20], u64 num_public, const u64 *vars, u64 nv,
                    const u64 *hidx, u64 nh, u64 *a_g1, u64 *b_g1, u64 *b_g2, u64 *ic_g1, u64 *h_g1) {
  u64 V = cs->num_variables, n = or_domain_size(cs->num_constraints);
  fr P[5];
  for (int i = 0; i < 5; i++) fr_to_mont(&P[i], params + 4 * i);
  for (int i = 0; i < 4; i++) if (fr_is_zero(&P[i])) return OR_ERR_SETUP_PARAMS;
  if (num_public >= V) return OR_ERR_SETUP_PARAMS;
  for (u64 k = 0; k < nv; k++) if (vars[k] >= V) return OR_ERR_SETUP_PARAMS;
  for (u64 k = 0; k < nh; k++) if (hidx[k] >= n) return OR_ERR_SETUP_PARAMS;
  fr al, be, ga, de, ta;
  lo64_fr(&al, &P[0]); lo64_fr(&be, &P[1]); lo64_fr(&ga, &P[2]); lo64_fr(&de, &P[3]); lo64_fr(&ta, &P[4]);
  if (fr_is_zero(&de) || fr_is_zero(&ga)) return OR_ERR_SETUP_PARAMS;
  fr *av = (fr *)malloc(sizeof(fr) * V), *bv = (fr *)malloc(sizeof(fr) * V), *cv = (fr *)malloc(sizeof(fr) * V);
  qap_eval_mont(cs, &ta, av, bv, cv);
  g1_jac g1; g1_from_aff(&g1, &G1_GEN);
  g2_jac g2; g2_from_aff(&g2, &G2_GEN);
  g1_aff *t1 = (g1_aff *)malloc(sizeof(g1_aff) * 2048);
  g2_aff *t2 = (g2_aff *)malloc(sizeof(g2_aff) * 2048);
  g1_fb_table(t1, &g1); g2_fb_table(t2, &g2);
  fr dinv, ginv; fr_inv(&dinv, &de); fr_inv(&ginv, &ga);
  for (u64 k = 0; k < nv; k++) {
    const u64 v = vars[k];
    g1_jac j; g1_aff a; g2_jac j2; g2_aff a2;
    if (a_g1) { g1_fb_mul(&j, t1, fr_lo64(&av[v])); g1_to_aff(&a, &j); g1_store(a_g1 + 13 * k, &a); }
    if (b_g1) { g1_fb_mul(&j, t1, fr_lo64(&bv[v])); g1_to_aff(&a, &j); g1_store(b_g1 + 13 * k, &a); }
    if (b_g2) { g2_fb_mul(&j2, t2, fr_lo64(&bv[v])); g2_to_aff(&a2, &j2); g2_store(b_g2 + 25 * k, &a2); }
    if (ic_g1) {
      fr t, u; fr_mul(&t, &be, &av[v]); fr_mul(&u, &al, &bv[v]); fr_add(&t, &t, &u); fr_add(&t, &t, &cv[v]);
      fr_mul(&t, &t, v > num_public ? &dinv : &ginv);
      g1_fb_mul(&j, t1, fr_lo64(&t)); g1_to_aff(&a, &j); g1_store(ic_g1 + 13 * k, &a);
    }
  }
  for (u64 k = 0; k < nh && h_g1; k++) {
    u64 e[4] = {hidx[k], 0, 0, 0};
    fr tp, t; fr_pow(&tp, &ta, e, 1); fr_mul(&t, &tp, &dinv);
    g1_jac j; g1_aff a; g1_fb_mul(&j, t1, fr_lo64(&t)); g1_to_aff(&a, &j); g1_store(h_g1 + 13 * k, &a);
  }
  free(av); free(bv); free(cv); free(t1); free(t2);
  return OR_OK;
}

/* ------------------------------------------------------------------------ */
/* prove: Prover::prove (crates/groth16-core/src/lib.rs:139-272)            */
/* ------------------------------------------------------------------------ */
typedef struct { u64 *sc; g1_aff *pt; u64 n; } g1_terms;
typedef struct { u64 *sc; g2_aff *pt; u64 n; } g2_terms;
static void t1_push(g1_terms *t, const u64 *s, const g1_aff *p) { memcpy(t->sc + 4 * t->n, s, 32); t->pt[t->n++] = *p; }
static void t2_push(g2_terms *t, const u64 *s, const g2_aff *p) { memcpy(t->sc + 4 * t->n, s, 32); t->pt[t->n++] = *p; }
/* Append the terms (w_i, bases[i - off]) for lo <= i < hi with w_i != 0 and
 * i - off < len, in index order (the filter of core:169-175 / 187-193 /
 * 226-233 / 250-252); the selection is one sequential pass, the Montgomery
 * loads of the selected points run on g_nthreads threads. */
static u64 *g_sel;                                   /* scratch: selected indices */
static u64 select_terms(const u64 *w, u64 lo, u64 hi, u64 off, u64 len) {
  u64 m = 0;
  for (u64 i = lo; i < hi; i++)
    if (w[4 * i] && i - off < len) g_sel[m++] = i;
  return m;
}
static void t1_append(g1_terms *t, const u64 *w, u64 lo, u64 hi, const u64 *bases, u64 off, u64 len) {
  u64 m = select_terms(w, lo, hi, off, len), base = t->n;
#pragma omp parallel for schedule(static) num_threads(OMP_T(m, 4096))
  for (long long j = 0; j < (long long)m; j++) {
    u64 i = g_sel[j];
    memcpy(t->sc + 4 * (base + (u64)j), w + 4 * i, 32);
    g1_load(&t->pt[base + (u64)j], bases + 13 * (i - off));
  }
  t->n += m;
}
static void t2_append(g2_terms *t, const u64 *w, u64 lo, u64 hi, const u64 *bases, u64 off, u64 len) {
  u64 m = select_terms(w, lo, hi, off, len), base = t->n;
#pragma omp parallel for schedule(static) num_threads(OMP_T(m, 4096))
  for (long long j = 0; j < (long long)m; j++) {
    u64 i = g_sel[j];
    memcpy(t->sc + 4 * (base + (u64)j), w + 4 * i, 32);
    g2_load(&t->pt[base + (u64)j], bases + 25 * (i - off));
  }
  t->n += m;
}
/* multi_scalar_mult_g1 (core:275-286): empty -> identity, else msm().into_affine() */
static void msm1(g1_aff *o, const g1_terms *t) { g1_jac j; g1_msm_ark(&j, t->pt, t->sc, t->n); g1_to_aff(o, &j); }
static void msm2(g2_aff *o, const g2_terms *t) { g2_jac j; g2_msm_ark(&j, t->pt, t->sc, t->n); g2_to_aff(o, &j); }

int or_prove(const or_pk *pk, const or_r1cs *cs, const u64 *z, u64 zlen, u64 num_public,
             const u64 r[4], const u64 s[4], u64 proof[51]) {
  /* Witness::new (core:81-99) */
  if (num_public >= zlen) return OR_ERR_INVALID_WITNESS;
  if (!(z[0] == 1 && z[1] == 0 && z[2] == 0 && z[3] == 0)) return OR_ERR_INVALID_WITNESS;
  /* witness.validate (core:112-131) */
  int rc = or_validate(cs, z, zlen);
  if (rc) return rc;
  u64 V = zlen, n = or_domain_size(cs->num_constraints);
  const u64 one[4] = {1, 0, 0, 0};
  /* assignment_fr = lo64 (core:156-161); canonical z -> low limb */
  u64 *w = (u64 *)malloc(sizeof(u64) * 4 * V);
  for (u64 i = 0; i < V; i++) { w[4 * i] = z[4 * i]; w[4 * i + 1] = w[4 * i + 2] = w[4 * i + 3] = 0; }
  u64 cap = V + n + 8;
  g_sel = (u64 *)malloc(sizeof(u64) * (V > n ? V : n));
  g1_terms T1 = {(u64 *)malloc(32 * cap), (g1_aff *)malloc(sizeof(g1_aff) * cap), 0};
  g2_terms T2 = {(u64 *)malloc(32 * (V + 4)), (g2_aff *)malloc(sizeof(g2_aff) * (V + 4)), 0};
  g1_aff P, pi_a, pi_c, h1, b1; g2_aff Q, pi_b;
  u64 *hw = NULL;

  /* pi_A (core:164-179) */
  T1.n = 0;
  g1_load(&P, pk->alpha_g1); t1_push(&T1, one, &P);
  t1_append(&T1, w, 0, V, pk->a_g1, 0, pk->a_len);
  g1_load(&P, pk->delta_g1); t1_push(&T1, r, &P);
  msm1(&pi_a, &T1);

  /* pi_B (core:182-197) */
  T2.n = 0;
  g2_load(&Q, pk->beta_g2); t2_push(&T2, one, &Q);
  t2_append(&T2, w, 0, V, pk->b_g2, 0, pk->b2_len);
  g2_load(&Q, pk->delta_g2); t2_push(&T2, s, &Q);
  msm2(&pi_b, &T2);

  /* H (core:200-221) */
  fr *zm = load_z(z, V);
  fr *h = (fr *)malloc(sizeof(fr) * n);
  rc = quotient_mont(cs, zm, V, h);
  free(zm);
  if (rc) goto done;
  /* h_coeffs = lo64 (core:203-208), zipped with h_g1 (core:211-219) */
  hw = (u64 *)calloc(4 * n, sizeof(u64));
#pragma omp parallel for schedule(static) num_threads(OMP_T(n, 4096))
  for (long long i = 0; i < (long long)n; i++) hw[4 * i] = fr_lo64(&h[i]);
  T1.n = 0;
  t1_append(&T1, hw, 0, n, pk->h_g1, 0, pk->h_len);
  if (T1.n == 0) { h1.inf = 1; fq_set_zero(&h1.x); fq_set_zero(&h1.y); }
  else msm1(&h1, &T1);

  /* B1 (core:246-255) */
  T1.n = 0;
  g1_load(&P, pk->beta_g1); t1_push(&T1, one, &P);
  t1_append(&T1, w, 0, V, pk->b_g1, 0, pk->b_len);
  msm1(&b1, &T1);

  /* pi_C (core:224-265) */
  T1.n = 0;
  t1_append(&T1, w, pk->num_public + 1, V, pk->ic_g1, pk->num_public + 1, pk->ic_len);
  if (!h1.inf) t1_push(&T1, one, &h1);
  if (!pi_a.inf) t1_push(&T1, s, &pi_a);
  if (!b1.inf) t1_push(&T1, r, &b1);
  if (T1.n == 0) { pi_c.inf = 1; fq_set_zero(&pi_c.x); fq_set_zero(&pi_c.y); }
  else msm1(&pi_c, &T1);

  g1_store(proof, &pi_a);
  g2_store(proof + 13, &pi_b);
  g1_store(proof + 38, &pi_c);
done:
  free(w); free(h); free(hw); free(g_sel); g_sel = NULL;
  free(T1.sc); free(T1.pt); free(T2.sc); free(T2.pt);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* deterministic generators                                                 */
/* ------------------------------------------------------------------------ */
u64 or_splitmix64(u64 *state) {
  u64 z = (*state += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static void rand_fr_state(u64 *o, u64 *st) {
  for (;;) {
    for (int i = 0; i < 4; i++) o[i] = or_splitmix64(st);
    o[3] &= 0x7fffffffffffffffULL;
    if (!mp_geq(o, FR_M, 4)) return;
  }
}
void or_random_fr(u64 *out, u64 count, u64 seed) {
  u64 st = seed;
  for (u64 i = 0; i < count; i++) rand_fr_state(out + 4 * i, &st);
}
void or_synthetic_circuit(u64 n, u64 *rowptr, uint32_t *a_col, uint32_t *b_col, uint32_t *c_col, u64 *vals) {
  for (u64 j = 0; j <= n; j++) rowptr[j] = j;
  for (u64 j = 0; j < n; j++) {
    a_col[j] = (uint32_t)(1 + 3 * j); b_col[j] = (uint32_t)(2 + 3 * j); c_col[j] = (uint32_t)(3 + 3 * j);
    if (vals) { vals[4 * j] = 1; vals[4 * j + 1] = vals[4 * j + 2] = vals[4 * j + 3] = 0; }
  }
}
void or_synthetic_witness(u64 n, u64 seed, u64 *z) {
  u64 st = seed;
  memset(z, 0, 32); z[0] = 1;
  for (u64 j = 0; j < n; j++) {
    u64 *x = z + 4 * (1 + 3 * j), *y = z + 4 * (2 + 3 * j), *p = z + 4 * (3 + 3 * j);
    rand_fr_state(x, &st); rand_fr_state(y, &st);
    or_fr_mul(p, x, y);
  }
}
