/*
 * zk_oracle.h -- CPU restatement of the reference Groth16 prover hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * or as the timed CPU baseline.  The product (libzkp_amd.so) never links it.
 *
 * What it restates (reference = vats98754/zero-knowledge-proofs, Rust, which
 * cannot be built in this image -- no cargo/rustc, arkworks sources absent):
 *   - Prover::prove            crates/groth16-core/src/lib.rs:139-272
 *   - multi_scalar_mult_g1/g2  crates/groth16-core/src/lib.rs:275-300
 *       -> ark-ec 0.4.2 VariableBaseMSM::msm / msm_bigint_wnaf (upstream,
 *          not vendored; restated from its published algorithm)
 *   - QAP::from_r1cs / compute_quotient_polynomial / evaluate_at /
 *     verify_evaluation / degree
 *                              crates/groth16-qap/src/lib.rs:95-294
 *       -> ark-poly 0.4.2 Radix2EvaluationDomain fft/ifft (upstream)
 *   - CRS::generate_from_qap   crates/groth16-setup/src/lib.rs:141-268
 *   - Witness::new / validate  crates/groth16-core/src/lib.rs:81-131
 *   - the synthetic n x (x*y=z) circuit of groth16-cli
 *                              crates/groth16-cli/src/lib.rs:55-77
 *
 * Parity status: PARTIALLY PINNED.  The reference's own tests pin only toy
 * identities (field KATs crates/groth16-field/src/lib.rs:180-234, x*y=z
 * accept/reject crates/groth16-qap/src/lib.rs:356-448, pk lengths
 * crates/groth16-setup/src/lib.rs:376-401); no reference test or fixture pins
 * a proof, MSM or FFT value.  This oracle is pinned by those KATs, by
 * mathematical KATs (curve/field constants, r*G = O, roots of unity, the
 * zcash-format compressed G1 generator) and by an independent pure-Python
 * big-integer restatement of the LITERAL dense reference algorithm
 * (oracle/pyref.py -> tests/golden/ JSON).
 *
 * Encoding at this interface (same as include/zkp.h): canonical (NOT
 * Montgomery) little-endian u64 limbs.  Fr = 4 limbs, Fq = 6 limbs,
 * Fq2 = c0 limbs then c1 limbs.  G1 affine = 13 u64 words (x[6], y[6],
 * word 12 = infinity flag in its low byte), G2 affine = 25 u64 words
 * (x.c0, x.c1, y.c0, y.c1, flag word).
 */
#ifndef ZK_ORACLE_H
#define ZK_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OR_OK = 0,
  OR_ERR_MSM_LEN = 1,
  OR_ERR_INVALID_WITNESS = 2,
  OR_ERR_QAP_DIVISION = 3,
  OR_ERR_DOMAIN = 4,
  OR_ERR_SETUP_PARAMS = 5,
};

/* Sparse constraint matrices (rows = constraints).  *_val are canonical Fr. */
typedef struct {
  uint64_t num_constraints;
  uint64_t num_variables;
  const uint64_t *a_rowptr; const uint32_t *a_col; const uint64_t *a_val;
  const uint64_t *b_rowptr; const uint32_t *b_col; const uint64_t *b_val;
  const uint64_t *c_rowptr; const uint32_t *c_col; const uint64_t *c_val;
} or_r1cs;

/* Proving key (crates/groth16-setup/src/lib.rs:27-52); arrays caller-owned. */
typedef struct {
  uint64_t alpha_g1[13], beta_g1[13], delta_g1[13];
  uint64_t beta_g2[25], delta_g2[25];
  uint64_t *a_g1; uint64_t a_len;     /* V */
  uint64_t *b_g1; uint64_t b_len;     /* V */
  uint64_t *b_g2; uint64_t b2_len;    /* V */
  uint64_t *ic_g1; uint64_t ic_len;   /* V - num_public - 1 */
  uint64_t *h_g1; uint64_t h_len;     /* qap.degree() = n */
  uint64_t num_public;
} or_pk;

/* Verification key (crates/groth16-setup/src/lib.rs:56-69). */
typedef struct {
  uint64_t alpha_g1[13];
  uint64_t beta_g2[25], gamma_g2[25], delta_g2[25];
  uint64_t *ic_g1; uint64_t ic_len;   /* num_public + 1 */
  uint64_t num_public;
} or_vk;

void or_init(void);

/* ---- field helpers (canonical in/out) ---- */
void or_fr_mul(uint64_t out[4], const uint64_t a[4], const uint64_t b[4]);
void or_fr_add(uint64_t out[4], const uint64_t a[4], const uint64_t b[4]);
void or_fr_sub(uint64_t out[4], const uint64_t a[4], const uint64_t b[4]);
int  or_fr_inv(uint64_t out[4], const uint64_t a[4]);
void or_fr_from_u64(uint64_t out[4], uint64_t v);
void or_fr_root_of_unity(uint64_t out[4], uint32_t log_n);
void or_fq_mul(uint64_t out[6], const uint64_t a[6], const uint64_t b[6]);
void or_fq_inv(uint64_t out[6], const uint64_t a[6]);

/* ---- curve helpers ---- */
void or_g1_generator(uint64_t out[13]);
void or_g2_generator(uint64_t out[25]);
int  or_g1_on_curve(const uint64_t p[13]);
int  or_g2_on_curve(const uint64_t p[25]);
void or_g1_add(uint64_t out[13], const uint64_t a[13], const uint64_t b[13]);
void or_g2_add(uint64_t out[25], const uint64_t a[25], const uint64_t b[25]);
void or_g1_mul(uint64_t out[13], const uint64_t p[13], const uint64_t k[4]);
void or_g2_mul(uint64_t out[25], const uint64_t p[25], const uint64_t k[4]);
/* zcash-format compressed encoding, as ark-bls12-381 0.4 CanonicalSerialize */
void or_g1_compress(uint8_t out[48], const uint64_t p[13]);
void or_g2_compress(uint8_t out[96], const uint64_t p[25]);

/* ---- threads: 1 (default) = the reference's single-threaded arkworks build;
 * more run the MSM over contiguous point chunks and the FFT butterflies /
 * point loads in parallel (OpenMP).  Outputs never depend on it. ---- */
void or_set_threads(int n);
int  or_get_threads(void);
/* bases[i] = (a + i b) G1, i < n (13 words each): closed-form MSM KAT */
void or_g1_lin_bases(uint64_t *out, const uint64_t a[4], const uint64_t b[4], uint64_t n);

/* ---- MSM: ark-ec 0.4 msm_bigint_wnaf restated (chunked over threads) ---- */
int or_msm_g1(uint64_t out[13], const uint64_t *bases, const uint64_t *scalars, uint64_t n);
int or_msm_g2(uint64_t out[25], const uint64_t *bases, const uint64_t *scalars, uint64_t n);

/* ---- radix-2 FFT over Fr, natural order in/out (ark-poly Radix2) ---- */
void or_fft(uint64_t *data, uint32_t log_n, int inverse);
void or_coset_fft(uint64_t *data, uint32_t log_n, int inverse, const uint64_t g[4]);

/* ---- QAP ---- */
uint64_t or_domain_size(uint64_t num_constraints);
/* validate (core:112-131 + qap:190-220,274-282): OR_OK / OR_ERR_INVALID_WITNESS */
int or_validate(const or_r1cs *cs, const uint64_t *z, uint64_t zlen);
/* H coefficients (n of them, zero padded), sparse O(n log n) restatement */
int or_quotient(const or_r1cs *cs, const uint64_t *z, uint64_t *h_out);
/* literal dense restatement of qap:95-187 + qap:225-271 (small n only) */
int or_quotient_dense(const or_r1cs *cs, const uint64_t *z, uint64_t *h_out);
/* A_i(t), B_i(t), C_i(t) for all variables i (sparse Lagrange form) */
void or_qap_eval_at(const or_r1cs *cs, const uint64_t t[4], uint64_t *a_vals,
                    uint64_t *b_vals, uint64_t *c_vals);

/* ---- setup / prove ---- */
/* params = alpha,beta,gamma,delta,tau (5 x 4 limbs, canonical). */
int or_setup(const or_r1cs *cs, const uint64_t params[20], uint64_t num_public,
             or_pk *pk, or_vk *vk, int nthreads);
/* Sampled key entries by or_setup's arithmetic: bases of variables vars[k]
 * in a_g1 / b_g1 / b_g2 / ic (pk ic for v > num_public, else vk ic) and of
 * coefficients hidx[k] in h_g1; NULL outputs skipped. */
int or_setup_sample(const or_r1cs *cs, const uint64_t params[20], uint64_t num_public,
                    const uint64_t *vars, uint64_t nv, const uint64_t *hidx, uint64_t nh,
                    uint64_t *a_g1, uint64_t *b_g1, uint64_t *b_g2, uint64_t *ic_g1, uint64_t *h_g1);
/* proof = a (13) | b (25) | c (13) words */
int or_prove(const or_pk *pk, const or_r1cs *cs, const uint64_t *z, uint64_t zlen,
             uint64_t num_public, const uint64_t r[4], const uint64_t s[4],
             uint64_t proof[51]);

/* ---- deterministic generators (shared with pyref.py / bench.py) ---- */
uint64_t or_splitmix64(uint64_t *state);
void or_random_fr(uint64_t *out, uint64_t count, uint64_t seed);
/* synthetic circuit (crates/groth16-cli/src/lib.rs:60-70): fills CSR arrays
 * (each *_rowptr has n+1 entries, *_col / *_val n entries) */
void or_synthetic_circuit(uint64_t n, uint64_t *rowptr, uint32_t *a_col,
                          uint32_t *b_col, uint32_t *c_col, uint64_t *vals);
/* witness: z = [1, x0, y0, x0*y0, x1, ...] from seed */
void or_synthetic_witness(uint64_t n, uint64_t seed, uint64_t *z);

#ifdef __cplusplus
}
#endif
#endif
