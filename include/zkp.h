/*
 * zkp.h -- C ABI of the MI355X-native Groth16 prover hot path
 *          (BLS12-381; G1/G2 Pippenger MSM + radix-2 Fr NTT on gfx950).
 *
 * Drop-in boundary for vats98754/zero-knowledge-proofs (Rust, arkworks 0.4):
 * every entry point below names the reference interface it replaces.  The
 * Rust-side binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions
 *   - Field elements cross the ABI in CANONICAL (non-Montgomery) form,
 *     little-endian u64 limbs: Fr = 4 limbs, Fq = 6, Fq2 = c0 then c1.
 *     (ark's in-memory BigInt layout; Montgomery conversion is internal.)
 *   - Affine points carry an explicit infinity byte, like ark's
 *     G1Affine{x, y, infinity}.  x = y = 0 when infinity is set.
 *   - All host buffers are caller-owned.  A zk_ctx owns its device memory
 *     and any uploaded proving key; calls on one ctx are serialised by the
 *     caller; distinct ctxs are independent.  No callbacks, no exceptions.
 *   - Every function returns a zk_status; zk_last_error() gives detail.
 */
#ifndef ZKP_H
#define ZKP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error kinds map 1:1 onto the reference's error enums:
 *   GrothError::MSMError            crates/groth16-core/src/lib.rs:75-76,282-283
 *   GrothError::InvalidWitness      crates/groth16-core/src/lib.rs:63-64,83-98,113-128
 *   QAPError::PolynomialDivisionFailed crates/groth16-qap/src/lib.rs:76-77,266-268
 *   QAPError::DomainTooSmall        crates/groth16-qap/src/lib.rs:67-73,101-105
 *   SetupError::InvalidParams       crates/groth16-setup/src/lib.rs:107-108,128-152 */
typedef enum {
  ZK_OK = 0,
  ZK_ERR_MSM_LEN = 1,
  ZK_ERR_INVALID_WITNESS = 2,
  ZK_ERR_QAP_DIVISION = 3,
  ZK_ERR_DOMAIN = 4,
  ZK_ERR_SETUP_PARAMS = 5,
  ZK_ERR_DEVICE = 6,
  ZK_ERR_RCCL = 7,
  ZK_ERR_ARG = 8,          /* bad argument: NULL, out of range, non-canonical field element */
  ZK_ERR_DIMENSION = 9     /* FieldError::DimensionMismatch (crates/groth16-field/src/lib.rs:127-129),
                              as returned by QAP::evaluate_at (crates/groth16-qap/src/lib.rs:190-198) */
} zk_status;

typedef struct { uint64_t l[4]; } zk_fr;                                   /* 32 B  */
typedef struct { uint64_t x[6], y[6]; uint8_t infinity, _pad[7]; } zk_g1_affine;   /* 104 B */
typedef struct { uint64_t x[12], y[12]; uint8_t infinity, _pad[7]; } zk_g2_affine; /* 200 B */

/* Proof (crates/groth16-core/src/lib.rs:27-36) */
typedef struct { zk_g1_affine a; zk_g2_affine b; zk_g1_affine c; } zk_proof;

/* Constraint system in CSR form, rows = constraints.  Replaces the dense
 * a/b/c_evals matrices of QAP::from_r1cs (crates/groth16-qap/src/lib.rs:114-140)
 * and the per-variable polynomials of struct QAP (qap:31-46): the same
 * matrices, never materialised densely.  Columns >= num_variables are
 * ignored (qap:122-124).  *_val == NULL means every coefficient is 1. */
typedef struct {
  uint64_t num_constraints;
  uint64_t num_variables;
  const uint64_t *a_rowptr; const uint32_t *a_col; const zk_fr *a_val;
  const uint64_t *b_rowptr; const uint32_t *b_col; const zk_fr *b_val;
  const uint64_t *c_rowptr; const uint32_t *c_col; const zk_fr *c_val;
} zk_r1cs_csr;

/* SetupParams (crates/groth16-setup/src/lib.rs:82-93); tau is the field
 * the reference calls `s`. */
typedef struct { zk_fr alpha, beta, gamma, delta, tau; } zk_setup_params;

/* ProvingKey (crates/groth16-setup/src/lib.rs:27-52) minus the embedded
 * QAP, which is passed as a zk_r1cs_csr.  Arrays are caller-allocated:
 * a_g1, b_g1, b_g2: num_variables; ic_g1: num_variables - num_public - 1;
 * h_g1: qap.degree() = domain size n. */
typedef struct {
  zk_g1_affine alpha_g1, beta_g1, delta_g1;
  zk_g2_affine beta_g2, delta_g2;
  zk_g1_affine *a_g1;  uint64_t a_len;
  zk_g1_affine *b_g1;  uint64_t b_len;
  zk_g2_affine *b_g2;  uint64_t b2_len;
  zk_g1_affine *ic_g1; uint64_t ic_len;
  zk_g1_affine *h_g1;  uint64_t h_len;
  uint64_t num_public;
} zk_pk;

/* VerificationKey (crates/groth16-setup/src/lib.rs:56-69); ic_g1: num_public + 1 */
typedef struct {
  zk_g1_affine alpha_g1;
  zk_g2_affine beta_g2, gamma_g2, delta_g2;
  zk_g1_affine *ic_g1; uint64_t ic_len;
  uint64_t num_public;
} zk_vk;

typedef struct zk_ctx zk_ctx;          /* one GPU, its streams and workspaces */
typedef struct zk_pk_dev zk_pk_dev;    /* proving key resident in HBM        */

/* ---------------------------------------------------------------- ctx --- */
/* device: HIP ordinal.  NULL on failure (no GPU, HIP error). */
zk_ctx *zk_ctx_create(int device);
void zk_ctx_destroy(zk_ctx *ctx);
const char *zk_last_error(const zk_ctx *ctx);
int zk_ctx_synchronize(zk_ctx *ctx);
/* Live kernel timing: HIP events recorded on the launching stream around
 * each kernel phase (msm_sort, msm_accum_g1, msm_accum_g2, msm_merge,
 * msm_bucket_sum, ntt, quotient_eval, quotient_misc).  enable: 0 off (and
 * clear), 1 on, 2 on plus a per-launch stream timeline.  No reference
 * counterpart (measurement). */
int zk_ctx_profile(zk_ctx *ctx, int enable);
/* names: '\0'-separated phase names; per phase: total ms, launches, work
 * units (scalar-point pairs for msm_*, elements for ntt/quotient). */
int zk_ctx_profile_read(zk_ctx *ctx, char *names, size_t names_cap, double *ms,
                        uint64_t *launches, uint64_t *units, size_t max_phases,
                        size_t *nphases);
/* The timeline of zk_ctx_profile(ctx, 2): one text line per profiled launch
 * ("phase stream start_ms end_ms", times from the start of its proof) and
 * "--" after each proof.  *len = its length; with buf (cap > len) the text is
 * copied NUL-terminated and the timeline cleared. */
int zk_ctx_timeline_read(zk_ctx *ctx, char *buf, size_t cap, size_t *len);

/* Build provenance: "<git HEAD>[-dirty] src:<16 hex of sha256 over the
 * sources in zero-knowledge-proofs_amd/csrc/ *.hip and *.hpp (sorted) and
 * include/zkp.h>".  __graft_entry__.smoke() recomputes the source hash from
 * the tree it runs in and refuses a library built from other sources.  No
 * reference counterpart. */
const char *zk_build_id(void);
/* Prove stream schedule (measurement): -1 or 0 the overlapped four-stream
 * schedule (default), 3 every kernel in order on one stream (isolated kernel
 * durations).  Results never depend on it.  ZK_ERR_ARG for anything else.
 * No reference counterpart. */
int zk_ctx_set_schedule(zk_ctx *ctx, int schedule);

/* Explicit path choices of a ctx, for tests and A/B measurement.  The
 * library reads nothing from the environment; without these calls it picks
 * by size.  No value changes a result: each is covered by a bit-exact GPU
 * test.  ZK_ERR_ARG for an unknown option or value.  No reference
 * counterpart.
 *   ZK_OPT_QUOTIENT_PATH  -1 by domain size (default: small-domain below
 *                         2^23), 0 small-domain (fused iNTT/coset/NTT tile
 *                         kernel, gathered final), 1 large-domain (separate
 *                         passes, natural-order final coset iNTT)
 *   ZK_OPT_PROVE_WIN_C    0 by size (default: 16, or 22 from 2^24 constraints
 *                         per key shard), 16 or 22: digit window width of
 *                         the prove MSMs of keys uploaded / set up after the
 *                         call
 *   ZK_OPT_EXCHANGE_TIMEOUT_MS  watchdog of the attached exchange (default
 *                         60000, >= 1): a distributed-quotient proof whose
 *                         peers do not answer within it fails with
 *                         ZK_ERR_RCCL and aborts the exchange
 *   ZK_OPT_DIST_QUOTIENT  -1 (default): a sharded key's quotient is
 *                         distributed whenever the ctx has an exchange of the
 *                         key's (shard, nshards) attached; 0: never -- every
 *                         rank computes the whole quotient and reads the
 *                         whole witness (the replicated alternative, for
 *                         measuring one against the other on one node)
 *   ZK_OPT_EXCHANGE_FIRST 0 (default): a distributed-quotient proof starts
 *                         its G2 and A+B1+IC MSMs with the witness, beside
 *                         the quotient and its three all-to-alls; 1: those
 *                         MSMs wait until the quotient (all-to-alls
 *                         included) is done, so the collectives never queue
 *                         behind a full-occupancy accumulate (for measuring
 *                         one order against the other on one node; no
 *                         effect without a distributed quotient or under
 *                         schedule 3, where everything runs in order)
 * (Test hooks -- the virtual-rank prove, the bare exchange, fault injection
 * -- live in a separate library, include/zkp_test.h.) */
enum { ZK_OPT_QUOTIENT_PATH = 1, ZK_OPT_PROVE_WIN_C = 2, ZK_OPT_EXCHANGE_TIMEOUT_MS = 3,
       ZK_OPT_DIST_QUOTIENT = 5, ZK_OPT_EXCHANGE_FIRST = 6 };
int zk_ctx_set_option(zk_ctx *ctx, int option, int64_t value);

/* ---------------------------------------------------------------- MSM --- */
/* Sum_i scalars[i] * bases[i], normalised to affine.  Replaces
 * Prover::multi_scalar_mult_g1 -> G1Projective::msm (ark-ec 0.4.2
 * VariableBaseMSM::msm), crates/groth16-core/src/lib.rs:275-286.
 * nbases != nscalars -> ZK_ERR_MSM_LEN (ark's Err(min_len)).
 * scalar_bits: 64 when every scalar is < 2^64 (the prove path's lo64
 * scalars), else 255.  Infinity bases and zero scalars are allowed.
 * A scalar >= r (ark's Fr is always reduced) or wider than scalar_bits is
 * ZK_ERR_ARG -- checked on the host for host scalars, by a device flag for
 * the *_dev entry points. */
int zk_msm_g1(zk_ctx *ctx, const zk_g1_affine *bases, size_t nbases,
              const zk_fr *scalars, size_t nscalars, uint32_t scalar_bits,
              zk_g1_affine *out);
/* Same for G2: crates/groth16-core/src/lib.rs:289-300. */
int zk_msm_g2(zk_ctx *ctx, const zk_g2_affine *bases, size_t nbases,
              const zk_fr *scalars, size_t nscalars, uint32_t scalar_bits,
              zk_g2_affine *out);

/* Device-resident MSM (benchmarks, and callers that keep bases in HBM).
 * zk_msm_g1_upload converts bases once into the device layout; the scalars
 * pointer of zk_msm_g1_dev is DEVICE memory holding n canonical zk_fr. */
typedef struct zk_msm_bases zk_msm_bases;
int zk_msm_g1_upload(zk_ctx *ctx, const zk_g1_affine *bases, size_t n, zk_msm_bases **out);
int zk_msm_g2_upload(zk_ctx *ctx, const zk_g2_affine *bases, size_t n, zk_msm_bases **out);
/* Same, plus ceil(scalar_bits / c) window-shifted copies 2^(c w) P of every
 * base (c = 16 up to 64-bit scalars, else 20; scalar_bits = 0 -> 255):
 * later zk_msm_*_dev calls with scalars of at most scalar_bits bits sum every
 * digit window into ONE bucket set (one bucket reduction, no per-window
 * Horner).  Costs ceil(scalar_bits / c) x the base memory (points padded to
 * whole 128-byte lines) and a one-time precomputation.  No reference counterpart
 * (fixed-base preprocessing of bases reused across MSMs, as in the prover). */
int zk_msm_g1_upload_windows(zk_ctx *ctx, const zk_g1_affine *bases, size_t n, uint32_t scalar_bits,
                             zk_msm_bases **out);
int zk_msm_g2_upload_windows(zk_ctx *ctx, const zk_g2_affine *bases, size_t n, uint32_t scalar_bits,
                             zk_msm_bases **out);
void zk_msm_bases_free(zk_msm_bases *b);
int zk_msm_g1_dev(zk_ctx *ctx, const zk_msm_bases *bases, const void *d_scalars, size_t n,
                  uint32_t scalar_bits, zk_g1_affine *out);
int zk_msm_g2_dev(zk_ctx *ctx, const zk_msm_bases *bases, const void *d_scalars, size_t n,
                  uint32_t scalar_bits, zk_g2_affine *out);

/* ---------------------------------------------------------------- NTT --- */
/* In-place radix-2 transform over Fr of size 2^log_n, natural order in and
 * out.  Replaces Radix2EvaluationDomain::{fft, ifft, coset_fft, coset_ifft}
 * (ark-poly 0.4.2) as used at crates/groth16-qap/src/lib.rs:101,167-169,260.
 * dir: +1 forward (evaluations X_k = sum_j x_j w^jk), -1 inverse (scaled by
 * n^-1).  coset: NULL, or the shift g (forward evaluates on g*<w>; inverse
 * undoes it).  log_n <= 32 else ZK_ERR_DOMAIN (Fr 2-adicity is 32). */
int zk_ntt_fr(zk_ctx *ctx, zk_fr *data, uint32_t log_n, int dir, const zk_fr *coset);
/* Same on DEVICE memory holding canonical zk_fr. */
int zk_ntt_fr_dev(zk_ctx *ctx, void *d_data, uint32_t log_n, int dir, const zk_fr *coset);

/* -------------------------------------------------------------- setup --- */
/* CRS::generate_from_qap (crates/groth16-setup/src/lib.rs:141-268) with the
 * reference's exact semantics (low-64-bit truncation of every derived scalar,
 * h_g1 = [lo64(tau~^i / delta~)]_1 for i < n).  Fills caller-allocated pk / vk
 * arrays (sizes as documented on zk_pk / zk_vk). */
int zk_groth16_setup(zk_ctx *ctx, const zk_r1cs_csr *qap, const zk_setup_params *params,
                     uint64_t num_public, zk_pk *pk, zk_vk *vk);
/* Same, but the proving key stays in HBM (no host round trip); vk may be NULL. */
int zk_groth16_setup_dev(zk_ctx *ctx, const zk_r1cs_csr *qap, const zk_setup_params *params,
                         uint64_t num_public, zk_pk_dev **pk_out, zk_vk *vk);

/* -------------------------------------------------------------- prove --- */
/* Upload a proving key + its constraint system once; it stays resident.
 * The CSR is required because the reference's ProvingKey embeds the QAP as
 * dense per-variable polynomials (pk.qap, crates/groth16-setup/src/lib.rs:51,
 * built by QAP::from_r1cs, crates/groth16-qap/src/lib.rs:143-170): a Rust
 * caller passes the R1CS it built the QAP from (its A/B/C rows, the same
 * matrices the polynomials interpolate) instead of those polynomials, which
 * are infeasible beyond ~2^12 constraints.  This is the one
 * change to the drop-in contract of prove(pk, witness, rng). */
int zk_pk_upload(zk_ctx *ctx, const zk_pk *pk, const zk_r1cs_csr *qap, zk_pk_dev **out);
void zk_pk_free(zk_pk_dev *pk);

/* Prover::prove (crates/groth16-core/src/lib.rs:139-272), bit-exact:
 * z = full assignment [1 | public | witness] (Witness::assignment), zlen its
 * length, num_public = Witness::num_public.  r and s are the two Fr::rand
 * draws of core:152-153, made explicit so proofs are reproducible.
 * Errors: ZK_ERR_INVALID_WITNESS (Witness::new / validate), ZK_ERR_QAP_DIVISION;
 * ZK_ERR_ARG when r, s or some z_i is >= r (a device flag over z). */
int zk_groth16_prove(zk_ctx *ctx, const zk_pk_dev *pk, const zk_fr *z, size_t zlen,
                     size_t num_public, const zk_fr *r, const zk_fr *s, zk_proof *out);
/* Same with z in DEVICE memory (zlen canonical zk_fr). */
int zk_groth16_prove_dev(zk_ctx *ctx, const zk_pk_dev *pk, const void *d_z, size_t zlen,
                         size_t num_public, const zk_fr *r, const zk_fr *s, zk_proof *out);

/* ---- multi-GPU: MSM sharded by base range (one process per GPU) ---- */
/* Upload only shard `shard` of `nshards` contiguous ranges of every base
 * vector (and the H bases i = shard mod nshards).  The constraint system
 * stays whole on every rank: each computes the whole quotient unless its ctx
 * is attached to an exchange of the key's (shard, nshards), in which case
 * the quotient is distributed (zk_ctx_attach_rccl below). */
int zk_pk_upload_shard(zk_ctx *ctx, const zk_pk *pk, const zk_r1cs_csr *qap,
                       uint32_t shard, uint32_t nshards, zk_pk_dev **out);
int zk_groth16_setup_dev_shard(zk_ctx *ctx, const zk_r1cs_csr *qap, const zk_setup_params *params,
                               uint64_t num_public, uint32_t shard, uint32_t nshards,
                               zk_pk_dev **pk_out);
/* Opaque per-GPU partial accumulators (Montgomery XYZZ), exchanged by ONE
 * all-gather over RCCL/xGMI and folded by zk_groth16_prove_combine. */
#define ZK_PARTIAL_BYTES 1536
typedef struct { uint8_t bytes[ZK_PARTIAL_BYTES]; } zk_prove_partial;
int zk_groth16_prove_partial(zk_ctx *ctx, const zk_pk_dev *pk_shard, const void *d_z, size_t zlen,
                             size_t num_public, const zk_fr *r, const zk_fr *s,
                             zk_prove_partial *out);
/* The witness entries a key shard reads on this ctx: *nranges half-open
 * index ranges [ranges[2k], ranges[2k+1]) of z, ascending and disjoint (at
 * most cap are written).  With a distributed quotient (an exchange of the
 * key's shape attached) that is z_0, the variables of the shard's MSM bases
 * and those its quotient rows reference, plus the variables var_owner gives
 * the shard (so every z entry is read, and checked canonical, by some rank)
 * -- 1/N of the witness plus z_0 for the synthetic circuit (3n/N + 1
 * entries), since a shard's MSM variables are those its quotient rows first
 * reference; otherwise all of [0, zlen).  No reference counterpart. */
int zk_groth16_witness_ranges(zk_ctx *ctx, const zk_pk_dev *pk_shard, uint64_t *ranges, size_t cap,
                              size_t *nranges);
/* zk_groth16_prove_partial from a HOST witness slice -- the sharded form of
 * the drop-in prove(pk, witness, rng) (crates/groth16-core/src/lib.rs:139-147),
 * each rank receiving only its part: z_slice holds z[lo..hi) of every range
 * of zk_groth16_witness_ranges, concatenated in order (slice_len entries in
 * all, else ZK_ERR_ARG -- with a distributed quotient on every rank at once,
 * through the ranks' status agreement, so no peer is left waiting in an
 * all-to-all); zlen is the length of the whole witness (the
 * Witness::validate length check, core:113-118). */
int zk_groth16_prove_partial_host(zk_ctx *ctx, const zk_pk_dev *pk_shard, const zk_fr *z_slice,
                                  size_t slice_len, size_t zlen, size_t num_public, const zk_fr *r,
                                  const zk_fr *s, zk_prove_partial *out);
int zk_groth16_prove_combine(const zk_prove_partial *parts, size_t nparts,
                             const zk_fr *r, const zk_fr *s, zk_proof *out);

/* The quotient of a sharded key, distributed: ranks attached to one RCCL
 * communicator split every transform of compute_quotient_polynomial
 * (crates/groth16-qap/src/lib.rs:225-271) four-step over xGMI -- three
 * all-to-alls per proof -- instead of each recomputing it; shard k's H
 * bases are the coefficients i = k mod nshards.  Used by
 * zk_groth16_prove_partial when the ctx's communicator matches the key's
 * (shard, nshards) and nshards is 2, 4 or 8; otherwise every rank computes
 * the whole quotient.  No reference counterpart (multi-GPU). */
int zk_rccl_unique_id(uint8_t out[128]);   /* one rank makes it, all attach with it */
/* The communicator is created non-blocking and polled under the ctx's
 * exchange watchdog (ZK_OPT_EXCHANGE_TIMEOUT_MS): a peer that never attaches
 * makes this return ZK_ERR_RCCL after the timeout instead of hanging. */
int zk_ctx_attach_rccl(zk_ctx *ctx, const uint8_t unique_id[128], int rank, int world);
/* The same distributed quotient over a host-staged exchange: each of the
 * three all-to-alls brings this rank's world chunks of chunk_bytes (chunk k
 * for rank k) to pinned host memory and calls all_to_all, which must fill
 * recv (chunk s from rank s) through the caller's transport -- e.g.
 * torch.distributed over gloo, or any network -- and return 0;
 * all_reduce_max replaces *value by its maximum over the ranks (the status
 * agreement before the first exchange).  Non-zero from either callback ->
 * ZK_ERR_RCCL.  abort (may be NULL) is called when this rank fails after
 * the ranks agreed to start, so the caller can make its peers' pending
 * transfers fail (e.g. by tearing the process group down).  Callbacks run on
 * the thread that called the prove.  No reference counterpart. */
typedef struct {
  int (*all_to_all)(void *user, const void *send, void *recv, size_t chunk_bytes);
  int (*all_reduce_max)(void *user, int32_t *value);
  void (*abort)(void *user);
  void *user;
} zk_exchange_ops;
int zk_ctx_attach_exchange(zk_ctx *ctx, const zk_exchange_ops *ops, int rank, int world);
/* Drop the ctx's exchange (RCCL: ncclCommAbort, local -- every rank is
 * expected to detach too); later proofs of sharded keys compute the whole
 * quotient on every rank.  A caller whose attach or first distributed proof
 * failed on some rank detaches everywhere and carries on replicated.  No-op
 * without an exchange.  No reference counterpart. */
int zk_ctx_detach_exchange(zk_ctx *ctx);
/* ---------------------------------------------------------------- QAP --- */
/* QAP::evaluate_at (crates/groth16-qap/src/lib.rs:190-220): out[0..2] =
 * A(point), B(point), C(point) = sum_i z_i A_i(point) etc., out[3] = Z(point)
 * = point^n - 1, from the sparse matrices (sum_j (Az)_j L_j(point) with the
 * domain's Lagrange basis -- the value the dense interpolants give).
 * zlen != num_variables -> ZK_ERR_DIMENSION (FieldError::DimensionMismatch).
 * QAP::verify_evaluation (qap:274-282) is a*b == c on these values. */
int zk_qap_evaluate_at(zk_ctx *ctx, const zk_r1cs_csr *qap, const zk_fr *point, const zk_fr *z, size_t zlen,
                       zk_fr out[4]);
/* utils::batch_evaluate (crates/groth16-qap/src/lib.rs:315-322): out[p] =
 * poly_p(point) for npolys dense polynomials in coefficient form, poly p's
 * coefficients (lowest degree first) at coeffs[offsets[p] .. offsets[p+1]). */
int zk_poly_evaluate_batch(zk_ctx *ctx, const zk_fr *coeffs, const uint64_t *offsets, size_t npolys,
                           const zk_fr *point, zk_fr *out);

/* Synthetic data for benchmarks: the witness of the groth16-cli circuit
 * n x (x*y = z) (crates/groth16-cli/src/lib.rs:57-70), z = [1, x_0, y_0,
 * x_0 y_0, ...], 3n+1 canonical zk_fr written to DEVICE memory d_z, with
 * x_j, y_j < 2^254 drawn from a counter-based splitmix64 stream of `seed`. */
int zk_synthetic_witness_dev(zk_ctx *ctx, uint64_t n, uint64_t seed, void *d_z);

/* ------------------------------------------------------ serialization --- */
/* ark-serialize CanonicalSerialize, compressed (zcash flag bits), for
 * Proof (crates/groth16-core/src/lib.rs:28): a(48) | b(96) | c(48). */
int zk_proof_serialize_compressed(const zk_proof *proof, uint8_t out[192]);
/* CanonicalDeserialize, compressed, with ark's Validate::Yes checks: the
 * compression flag, infinity without the sort flag, x < p, a point on the
 * curve with the flagged root, in the prime-order subgroup.  Anything else
 * -> ZK_ERR_ARG (ark's SerializationError). */
int zk_proof_deserialize_compressed(const uint8_t in[192], zk_proof *out);

/* -------------------------------------------------------------- verify --- */
/* Host-only (no GPU): a handful of sequential pairings per call. */
/* Verifier::verify (crates/groth16-core/src/lib.rs:308-355): *valid = 1 iff
 * e(A,B) e(-alpha,beta) e(-IC,gamma) e(-C,delta) == 1 with
 * IC = ic_g1[0] + sum_i lo64(public_inputs[i]) ic_g1[i+1] (core:322-338).
 * n_inputs != vk->num_public -> ZK_ERR_INVALID_WITNESS (core:315-320).  The
 * reference's own proofs fail this check unless every derived setup scalar is
 * below 2^64 (lo64 truncation) -- mirrored, not fixed. */
int zk_groth16_verify(const zk_vk *vk, const zk_proof *proof, const zk_fr *public_inputs,
                      size_t n_inputs, int *valid);
/* BatchVerifier::verify_batch (core:360-432) with its Fr::rand coefficients
 * made explicit (coeffs[k] for proof k, canonical): ONE pairing check on
 * sum c_k A_k, sum c_k B_k, sum c_k IC_k, sum c_k C_k -- the reference's rule
 * as written.  n_proofs == 0 -> *valid = 1. */
int zk_groth16_verify_batch(const zk_vk *vk, const zk_proof *proofs, const zk_fr *const *public_inputs,
                            const size_t *n_inputs, size_t n_proofs, const zk_fr *coeffs, int *valid);
/* prod_i e(g1[i], g2[i]) == 1 -> *result = 1 (Bls12_381::multi_pairing(..)
 * .is_zero(), core:352).  Points must be canonical and on their curves. */
int zk_pairing_product_is_one(const zk_g1_affine *g1, const zk_g2_affine *g2, size_t n, int *result);

#ifdef __cplusplus
}
#endif
#endif /* ZKP_H */
