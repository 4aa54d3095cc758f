/*
 * curve_impl.h -- short-Weierstrass (a = 0) group law in Jacobian coordinates,
 * included once per curve by zk_oracle.c (TEST INFRASTRUCTURE, see zk_oracle.h).
 *
 * Restates ark-ec 0.4.2 short_weierstrass::Projective (x = X/Z^2, y = Y/Z^3),
 * the group used by G1Projective/G2Projective in
 * crates/groth16-core/src/lib.rs:275-300 and crates/groth16-setup/src/lib.rs:162-241.
 *
 * Required macros: F (field type), FP(op) (field op name), G(op) (curve op
 * name), CURVE_B (pointer to the Montgomery-form constant b).
 */

typedef struct { F x, y; int inf; } G(aff);
typedef struct { F X, Y, Z; } G(jac);

static void G(set_inf)(G(jac) *p) {
  FP(set_zero)(&p->X); FP(set_one)(&p->Y); FP(set_zero)(&p->Z);
}
static int G(is_inf)(const G(jac) *p) { return FP(is_zero)(&p->Z); }

static void G(from_aff)(G(jac) *o, const G(aff) *a) {
  if (a->inf) { G(set_inf)(o); return; }
  o->X = a->x; o->Y = a->y; FP(set_one)(&o->Z);
}

/* dbl-2009-l */
static void G(dbl)(G(jac) *o, const G(jac) *p) {
  if (G(is_inf)(p)) { G(set_inf)(o); return; }
  F A, B, C, D, E, Fv, t, X3, Y3, Z3;
  FP(sqr)(&A, &p->X);
  FP(sqr)(&B, &p->Y);
  FP(sqr)(&C, &B);
  FP(add)(&t, &p->X, &B); FP(sqr)(&t, &t); FP(sub)(&t, &t, &A); FP(sub)(&t, &t, &C);
  FP(add)(&D, &t, &t);
  FP(add)(&E, &A, &A); FP(add)(&E, &E, &A);
  FP(sqr)(&Fv, &E);
  FP(add)(&t, &D, &D); FP(sub)(&X3, &Fv, &t);
  FP(sub)(&t, &D, &X3); FP(mul)(&Y3, &E, &t);
  FP(add)(&C, &C, &C); FP(add)(&C, &C, &C); FP(add)(&C, &C, &C);
  FP(sub)(&Y3, &Y3, &C);
  FP(mul)(&Z3, &p->Y, &p->Z); FP(add)(&Z3, &Z3, &Z3);
  o->X = X3; o->Y = Y3; o->Z = Z3;
}

/* add-2007-bl */
static void G(add)(G(jac) *o, const G(jac) *p, const G(jac) *q) {
  if (G(is_inf)(p)) { *o = *q; return; }
  if (G(is_inf)(q)) { *o = *p; return; }
  F Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, r, V, t, X3, Y3, Z3;
  FP(sqr)(&Z1Z1, &p->Z);
  FP(sqr)(&Z2Z2, &q->Z);
  FP(mul)(&U1, &p->X, &Z2Z2);
  FP(mul)(&U2, &q->X, &Z1Z1);
  FP(mul)(&S1, &p->Y, &q->Z); FP(mul)(&S1, &S1, &Z2Z2);
  FP(mul)(&S2, &q->Y, &p->Z); FP(mul)(&S2, &S2, &Z1Z1);
  FP(sub)(&H, &U2, &U1);
  FP(sub)(&r, &S2, &S1);
  if (FP(is_zero)(&H)) {
    if (FP(is_zero)(&r)) { G(dbl)(o, p); return; }
    G(set_inf)(o); return;
  }
  FP(add)(&I, &H, &H); FP(sqr)(&I, &I);
  FP(mul)(&J, &H, &I);
  FP(add)(&r, &r, &r);
  FP(mul)(&V, &U1, &I);
  FP(sqr)(&X3, &r); FP(sub)(&X3, &X3, &J); FP(add)(&t, &V, &V); FP(sub)(&X3, &X3, &t);
  FP(sub)(&t, &V, &X3); FP(mul)(&Y3, &r, &t);
  FP(mul)(&t, &S1, &J); FP(add)(&t, &t, &t); FP(sub)(&Y3, &Y3, &t);
  FP(add)(&Z3, &p->Z, &q->Z); FP(sqr)(&Z3, &Z3); FP(sub)(&Z3, &Z3, &Z1Z1);
  FP(sub)(&Z3, &Z3, &Z2Z2); FP(mul)(&Z3, &Z3, &H);
  o->X = X3; o->Y = Y3; o->Z = Z3;
}

/* madd-2007-bl (Jacobian + affine) */
static void G(madd)(G(jac) *o, const G(jac) *p, const G(aff) *q) {
  if (q->inf) { *o = *p; return; }
  if (G(is_inf)(p)) { G(from_aff)(o, q); return; }
  F Z1Z1, U2, S2, H, HH, I, J, r, V, t, X3, Y3, Z3;
  FP(sqr)(&Z1Z1, &p->Z);
  FP(mul)(&U2, &q->x, &Z1Z1);
  FP(mul)(&S2, &q->y, &p->Z); FP(mul)(&S2, &S2, &Z1Z1);
  FP(sub)(&H, &U2, &p->X);
  FP(sub)(&r, &S2, &p->Y);
  if (FP(is_zero)(&H)) {
    if (FP(is_zero)(&r)) { G(dbl)(o, p); return; }
    G(set_inf)(o); return;
  }
  FP(sqr)(&HH, &H);
  FP(add)(&I, &HH, &HH); FP(add)(&I, &I, &I);
  FP(mul)(&J, &H, &I);
  FP(add)(&r, &r, &r);
  FP(mul)(&V, &p->X, &I);
  FP(sqr)(&X3, &r); FP(sub)(&X3, &X3, &J); FP(add)(&t, &V, &V); FP(sub)(&X3, &X3, &t);
  FP(sub)(&t, &V, &X3); FP(mul)(&Y3, &r, &t);
  FP(mul)(&t, &p->Y, &J); FP(add)(&t, &t, &t); FP(sub)(&Y3, &Y3, &t);
  FP(add)(&Z3, &p->Z, &H); FP(sqr)(&Z3, &Z3); FP(sub)(&Z3, &Z3, &Z1Z1); FP(sub)(&Z3, &Z3, &HH);
  o->X = X3; o->Y = Y3; o->Z = Z3;
}

static void G(neg_aff)(G(aff) *o, const G(aff) *a) {
  *o = *a;
  if (!a->inf) FP(neg)(&o->y, &a->y);
}

static void G(to_aff)(G(aff) *o, const G(jac) *p) {
  if (G(is_inf)(p)) { FP(set_zero)(&o->x); FP(set_zero)(&o->y); o->inf = 1; return; }
  F zi, zi2;
  FP(inv)(&zi, &p->Z);
  FP(sqr)(&zi2, &zi);
  FP(mul)(&o->x, &p->X, &zi2);
  FP(mul)(&zi2, &zi2, &zi);
  FP(mul)(&o->y, &p->Y, &zi2);
  o->inf = 0;
}

/* Montgomery batch inversion over the Z coordinates. */
static void G(batch_to_aff)(G(aff) *o, const G(jac) *p, size_t n) {
  if (n == 0) return;
  F *acc = (F *)malloc(sizeof(F) * n);
  F run; FP(set_one)(&run);
  for (size_t i = 0; i < n; i++) {
    acc[i] = run;
    if (!G(is_inf)(&p[i])) FP(mul)(&run, &run, &p[i].Z);
  }
  F inv; FP(inv)(&inv, &run);
  for (size_t i = n; i-- > 0;) {
    if (G(is_inf)(&p[i])) {
      FP(set_zero)(&o[i].x); FP(set_zero)(&o[i].y); o[i].inf = 1; continue;
    }
    F zi, zi2;
    FP(mul)(&zi, &inv, &acc[i]);
    FP(mul)(&inv, &inv, &p[i].Z);
    FP(sqr)(&zi2, &zi);
    FP(mul)(&o[i].x, &p[i].X, &zi2);
    FP(mul)(&zi2, &zi2, &zi);
    FP(mul)(&o[i].y, &p[i].Y, &zi2);
    o[i].inf = 0;
  }
  free(acc);
}

static int G(aff_on_curve)(const G(aff) *a) {
  if (a->inf) return 1;
  F l, r;
  FP(sqr)(&l, &a->y);
  FP(sqr)(&r, &a->x); FP(mul)(&r, &r, &a->x); FP(add)(&r, &r, CURVE_B);
  return FP(eq)(&l, &r);
}

/* left-to-right double-and-add over an nbits-bit little-endian scalar */
static void G(mul_bits)(G(jac) *o, const G(jac) *p, const uint64_t *k, int nbits) {
  G(jac) acc; G(set_inf)(&acc);
  for (int i = nbits - 1; i >= 0; i--) {
    G(dbl)(&acc, &acc);
    if ((k[i >> 6] >> (i & 63)) & 1) G(add)(&acc, &acc, p);
  }
  *o = acc;
}

/*
 * ark-ec 0.4.2 VariableBaseMSM::msm_bigint_wnaf, restated (upstream, not
 * vendored): window c = 3 if n < 32 else ln_without_floats(n) + 2; signed
 * digits recentred into [-2^(c-1), 2^(c-1)) with the final carry folded into
 * the top digit; 2^c buckets per window reduced by a running sum; windows
 * combined high to low with c doublings each.  Single-threaded (the reference
 * builds ark-ec without the `parallel` feature, Cargo.lock:101-113).
 * scalars: canonical 4-limb integers.
 */
static void G(msm_ark_serial)(G(jac) *out, const G(aff) *bases, const uint64_t *scalars, size_t n) {
  G(set_inf)(out);
  if (n == 0) return;
  int c = n < 32 ? 3 : (int)(ark_log2(n) * 69 / 100) + 2;
  const int num_bits = 255;
  int ndig = (num_bits + c - 1) / c;
  int32_t *dig = (int32_t *)malloc(sizeof(int32_t) * (size_t)ndig * n);
  for (size_t j = 0; j < n; j++) make_digits(scalars + 4 * j, c, num_bits, dig + (size_t)ndig * j);
  size_t nb = (size_t)1 << c;
  G(jac) *bk = (G(jac) *)malloc(sizeof(G(jac)) * nb);
  G(jac) *wsum = (G(jac) *)malloc(sizeof(G(jac)) * ndig);
  for (int w = 0; w < ndig; w++) {
    for (size_t b = 0; b < nb; b++) G(set_inf)(&bk[b]);
    for (size_t j = 0; j < n; j++) {
      int32_t d = dig[(size_t)ndig * j + w];
      if (d > 0) G(madd)(&bk[d - 1], &bk[d - 1], &bases[j]);
      else if (d < 0) {
        G(aff) nbse; G(neg_aff)(&nbse, &bases[j]);
        G(madd)(&bk[-d - 1], &bk[-d - 1], &nbse);
      }
    }
    G(jac) run, res; G(set_inf)(&run); G(set_inf)(&res);
    for (size_t b = nb; b-- > 0;) {
      G(add)(&run, &run, &bk[b]);
      G(add)(&res, &res, &run);
    }
    wsum[w] = res;
  }
  G(jac) tot; G(set_inf)(&tot);
  for (int w = ndig - 1; w >= 1; w--) {
    G(add)(&tot, &tot, &wsum[w]);
    for (int k = 0; k < c; k++) G(dbl)(&tot, &tot);
  }
  G(add)(out, &wsum[0], &tot);
  free(dig); free(bk); free(wsum);
}

/*
 * The MSM the oracle runs.  With g_nthreads == 1 it IS msm_ark_serial (the
 * reference's single-threaded arkworks build).  With more threads the points
 * are cut into g_nthreads contiguous chunks, each chunk runs the same serial
 * algorithm (its own window size) and the chunk sums are added in order --
 * the result is the same group element, so the affine output is unchanged.
 * Chunks below 4096 points are not worth a thread.
 */
static void G(msm_ark)(G(jac) *out, const G(aff) *bases, const uint64_t *scalars, size_t n) {
  int T = g_nthreads;
  if (T > 1 && n / (size_t)T < 4096) T = (int)(n / 4096);
  if (T <= 1) { G(msm_ark_serial)(out, bases, scalars, n); return; }
  G(jac) *part = (G(jac) *)malloc(sizeof(G(jac)) * (size_t)T);
#pragma omp parallel for schedule(dynamic, 1) num_threads(T)
  for (int t = 0; t < T; t++) {
    size_t lo = n * (size_t)t / (size_t)T, hi = n * (size_t)(t + 1) / (size_t)T;
    G(msm_ark_serial)(&part[t], bases + lo, scalars + 4 * lo, hi - lo);
  }
  G(set_inf)(out);
  for (int t = 0; t < T; t++) G(add)(out, out, &part[t]);
  free(part);
}

/* Jacobian -> affine for n points, batch-inverted in g_nthreads chunks. */
static void G(batch_to_aff_par)(G(aff) *o, const G(jac) *p, size_t n) {
  int T = g_nthreads;
  if (T > 1 && n / (size_t)T < 1024) T = (int)(n / 1024);
  if (T <= 1) { G(batch_to_aff)(o, p, n); return; }
#pragma omp parallel for schedule(static) num_threads(T)
  for (int t = 0; t < T; t++) {
    size_t lo = n * (size_t)t / (size_t)T, hi = n * (size_t)(t + 1) / (size_t)T;
    G(batch_to_aff)(o + lo, p + lo, hi - lo);
  }
}

/* fixed-base table: 8-bit windows over a 64-bit scalar, tab[w*256 + d] = d*2^(8w)*P */
static void G(fb_table)(G(aff) *tab, const G(jac) *P) {
  G(jac) *tj = (G(jac) *)malloc(sizeof(G(jac)) * 8 * 256);
  G(jac) base = *P;
  for (int w = 0; w < 8; w++) {
    G(set_inf)(&tj[w * 256]);
    for (int d = 1; d < 256; d++) G(add)(&tj[w * 256 + d], &tj[w * 256 + d - 1], &base);
    for (int k = 0; k < 8; k++) G(dbl)(&base, &base);
  }
  G(batch_to_aff)(tab, tj, 8 * 256);
  free(tj);
}
static void G(fb_mul)(G(jac) *o, const G(aff) *tab, uint64_t k) {
  G(set_inf)(o);
  for (int w = 0; w < 8; w++) {
    unsigned d = (unsigned)(k >> (8 * w)) & 255u;
    if (d) G(madd)(o, o, &tab[w * 256 + d]);
  }
}
