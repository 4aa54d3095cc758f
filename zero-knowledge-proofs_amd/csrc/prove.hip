// prove.hip -- Groth16 prove() orchestration on one GPU.
//
// Restates Prover::prove (crates/groth16-core/src/lib.rs:139-272) with the
// reference's arithmetic, quirks included:
//   w_i = lo64(z_i)                                         core:156-161
//   pi_A = alpha_1 + sum w_i a_g1[i] + r delta_1            core:164-179
//   pi_B = beta_2  + sum w_i b_g2[i] + s delta_2            core:182-197
//   H    = (A B - C) / (x^n - 1), h_i = lo64(H_i)           core:200-208, qap:225-271
//   H_1  = sum h_i h_g1[i]                                  core:211-221
//   B_1  = beta_1  + sum w_i b_g1[i]                        core:246-255
//   pi_C = sum_{i>l} w_i ic_g1[i-l-1] + H_1 + s pi_A + r B_1  core:224-265
// Every sum is one device MSM with 64-bit scalars: the full-width terms
// r*delta_1 and s*delta_2 are split as sum_k r_k (2^(64k) delta) over four
// precomputed bases (appended at pk upload), identity bases are compacted
// away at upload (they contribute nothing), and only s*pi_A + r*B_1 -- which
// depend on this proof's own MSM outputs -- are formed on the host.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "ctx.hpp"
#include "dist.hpp"
#include "quotient.hpp"

namespace zk {

// ------------------------------------------------------------------ CSR ---
__global__ void __launch_bounds__(256) k_u64_to_fr_mont(const uint64_t* __restrict__ in, Fr* __restrict__ out,
                                                        size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_vec(&out[i], fp_to_mont(ld_vec(reinterpret_cast<const Fr*>(in) + i)));
}

void csr_upload(CsrDev& d, const zk_r1cs_csr* q, hipStream_t st) {
  d.nc = q->num_constraints;
  d.V = q->num_variables;
  const uint64_t* rps[3] = {q->a_rowptr, q->b_rowptr, q->c_rowptr};
  const uint32_t* cols[3] = {q->a_col, q->b_col, q->c_col};
  const zk_fr* vals[3] = {q->a_val, q->b_val, q->c_val};
  for (int m = 0; m < 3; m++) {
    const uint64_t nnz = d.nc ? rps[m][d.nc] : 0;
    d.rp[m].ensure(sizeof(uint64_t) * (d.nc + 1));
    ZK_HIP(hipMemcpyAsync(d.rp[m].p, rps[m], sizeof(uint64_t) * (d.nc + 1), hipMemcpyHostToDevice, st));
    d.col[m].ensure(sizeof(uint32_t) * std::max<uint64_t>(nnz, 1));
    if (nnz) ZK_HIP(hipMemcpyAsync(d.col[m].p, cols[m], sizeof(uint32_t) * nnz, hipMemcpyHostToDevice, st));
    d.unit[m] = vals[m] == nullptr;
    if (!d.unit[m] && nnz) {
      DevBuf tmp;
      tmp.ensure(sizeof(zk_fr) * nnz);
      ZK_HIP(hipMemcpyAsync(tmp.p, vals[m], sizeof(zk_fr) * nnz, hipMemcpyHostToDevice, st));
      d.val[m].ensure(sizeof(Fr) * nnz);
      k_u64_to_fr_mont<<<ceil_div(nnz, 256), 256, 0, st>>>(tmp.as<uint64_t>(), d.val[m].as<Fr>(), nnz);
      ZK_LAUNCH_CHECK();
      ZK_HIP(hipStreamSynchronize(st));  // tmp dies here
    }
  }
}

// (Az)_j, (Bz)_j, (Cz)_j for every domain row (rows >= nc are zero padding,
// qap:155-164) plus the witness checks:
//   flags bit 0: row vrow unsatisfied      -> InvalidWitness (core:121-128: the
//                reference checks A(w)B(w) = C(w) at w = omega, i.e. row 1,
//                or row 0 when n == 1)
//   flags bit 1: some row unsatisfied      -> PolynomialDivisionFailed (qap:266)
//   flags bit 2: z_0 != 1                  -> InvalidWitness (core:89-93)
__global__ void __launch_bounds__(256) k_csr_eval(CsrArgs m, const Fr* __restrict__ zc, uint64_t nc, uint64_t V,
                                                  uint64_t n, uint64_t vrow, Fr* __restrict__ qa,
                                                  Fr* __restrict__ qb, Fr* __restrict__ qc,
                                                  uint32_t* __restrict__ flags) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) {
    Fr z0 = ld_vec(&zc[0]);
    bool one = z0.v[0] == 1;
#pragma unroll
    for (int i = 1; i < 8; i++) one = one && z0.v[i] == 0;
    if (!one) atomicOr(flags, 4u);
  }
  if (j >= n) return;
  Fr a = fp_zero<FrParams>(), b = a, c = a;
  if (j < nc) {
    a = row_dot(m.rp[0], m.col[0], m.val[0], j, zc, V);
    b = row_dot(m.rp[1], m.col[1], m.val[1], j, zc, V);
    c = row_dot(m.rp[2], m.col[2], m.val[2], j, zc, V);
    if (!fp_eq(fp_mul(a, b), c)) atomicOr(flags, j == vrow ? 3u : 2u);
  }
  st_vec(&qa[j], a);
  st_vec(&qb[j], b);
  st_vec(&qc[j], c);
}

__global__ void __launch_bounds__(256) k_quot_pointwise(Fr* __restrict__ qa, const Fr* __restrict__ qb,
                                                        const Fr* __restrict__ qc, const Fr* __restrict__ zinv,
                                                        size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr t = fp_sub(fp_mul(ld_vec(&qa[i]), ld_vec(&qb[i])), ld_vec(&qc[i]));
  st_vec(&qa[i], fp_mul(t, ld_vec(zinv)));
}

__device__ __forceinline__ uint32_t brev(uint32_t x, uint32_t log_n) {
  return log_n ? (__builtin_bitreverse32(x) >> (32 - log_n)) : 0;
}

// H_i = n^-1 g^-i * (bit-reversed iNTT output)[i], then lo64 (core:203-208):
// the element-wise gather path for domains that stay in the MALL
__global__ void __launch_bounds__(256) k_h_final(const Fr* __restrict__ hb, const Fr* __restrict__ gipow,
                                                 uint32_t log_n, uint64_t* __restrict__ hlo) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >> log_n) return;
  Fr h = fp_from_mont(fp_mul(ld_vec(&hb[brev((uint32_t)i, log_n)]), ld_vec(&gipow[i])));
  hlo[i] = (uint64_t)h.v[0] | ((uint64_t)h.v[1] << 32);
}

// H_i (Montgomery, natural order, n^-1 g^-i already applied) -> lo64 of the
// canonical value (core:203-208)
__global__ void __launch_bounds__(256) k_h_lo64(const Fr* __restrict__ h, size_t n, uint64_t* __restrict__ hlo) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr c = fp_from_mont(ld_vec(&h[i]));
  hlo[i] = (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
}

// out[k] = low word of src[idx[k] / div] (div > 1: a distributed-quotient
// rank holds H_(rank + div d) at position d)
__global__ void __launch_bounds__(256) k_gather_lo64(const uint64_t* __restrict__ src, int stride_words,
                                                     const uint32_t* __restrict__ idx, uint32_t div,
                                                     uint32_t count, uint64_t* __restrict__ out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  out[k] = src[(size_t)(idx[k] / div) * stride_words];
}

struct Extras {
  uint64_t v[5];
};
__global__ void k_set_extras(uint64_t* __restrict__ dst, Extras e, uint32_t n) {
  if (threadIdx.x < n) dst[threadIdx.x] = e.v[threadIdx.x];
}

// flags bit 3: some z_i >= r.  The reference's assignment is a vector of
// reduced Fr (core:40-44), so a non-canonical limb vector has no reference
// meaning (its lo64 would differ from the reduced value's): ZK_ERR_ARG.
__global__ void __launch_bounds__(256) k_check_canonical(const Fr* __restrict__ z, uint64_t n,
                                                         uint32_t* __restrict__ flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr a = ld_vec(&z[i]);
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) (void)__builtin_subc(a.v[k], FrParams::MOD[k], br, &br);
  if (!br) atomicOr(flags, 8u);   // a - r did not borrow: a >= r
}

void check_canonical(const void* d_z, uint64_t n, uint32_t* d_flags, hipStream_t st) {
  if (!n) return;
  k_check_canonical<<<ceil_div(n, 256), 256, 0, st>>>(reinterpret_cast<const Fr*>(d_z), n, d_flags);
  ZK_LAUNCH_CHECK();
}

bool fr_canonical(const zk_fr& a) {
  static const uint64_t R[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                0x73eda753299d7d48ull};
  for (int i = 3; i >= 0; i--)
    if (a.l[i] != R[i]) return a.l[i] < R[i];
  return false;
}

// ------------------------------------------------------------- pk upload ---
static uint64_t shard_lo(uint64_t len, uint32_t k, uint32_t ns) { return len * k / ns; }

// host XYZZ from canonical ABI affine words
static host::X<host::Fq> g1_from_abi(const zk_g1_affine& a) {
  if (a.infinity) return host::inf<host::Fq>();
  host::X<host::Fq> p;
  std::memcpy(p.X_.l, a.x, 48);
  std::memcpy(p.Y.l, a.y, 48);
  p.X_ = host::to_mont(p.X_);
  p.Y = host::to_mont(p.Y);
  p.ZZ = host::one();
  p.ZZZ = host::one();
  return p;
}
static host::X<host::Fq2> g2_from_abi(const zk_g2_affine& a) {
  if (a.infinity) return host::inf<host::Fq2>();
  host::X<host::Fq2> p;
  std::memcpy(p.X_.c0.l, a.x, 48);
  std::memcpy(p.X_.c1.l, a.x + 6, 48);
  std::memcpy(p.Y.c0.l, a.y, 48);
  std::memcpy(p.Y.c1.l, a.y + 6, 48);
  p.X_ = {host::to_mont(p.X_.c0), host::to_mont(p.X_.c1)};
  p.Y = {host::to_mont(p.Y.c0), host::to_mont(p.Y.c1)};
  p.ZZ = host::f_one<host::Fq2>();
  p.ZZZ = host::f_one<host::Fq2>();
  return p;
}

// [P, 2^64 P, 2^128 P, 2^192 P] in ABI form
template <class C, class ABI>
static void pow64_chain(const host::X<typename C::HF>& P, ABI* out) {
  host::X<typename C::HF> q = P;
  for (int k = 0; k < 4; k++) {
    host_to_abi<C>(q, reinterpret_cast<uint64_t*>(&out[k]));
    for (int d = 0; d < 64; d++) q = host::dbl(q);
  }
}

// Upload one base vector range [lo, hi): compact non-identity entries, append extras.
// Positions lo, lo + stride, ... < hi (stride > 1: the H coefficients of a
// shard, i = shard mod nshards, which is where the distributed quotient
// leaves them).
template <class C, class ABI>
static void upload_vector(zk_pk_dev& pk, int slot, const ABI* v, uint64_t lo, uint64_t hi, uint64_t idx_offset,
                          const std::vector<ABI>& extras, hipStream_t st, uint64_t stride = 1) {
  std::vector<uint32_t> idx;
  idx.reserve((hi - lo) / stride + 1);
  for (uint64_t i = lo; i < hi; i += stride)
    if (!v[i].infinity) idx.push_back((uint32_t)(i - lo));
  const uint32_t cnt = (uint32_t)idx.size();
  const uint32_t nex = (uint32_t)extras.size();
  pk.count[slot] = cnt;
  pk.extras[slot] = nex;
  pk.bases[slot].ensure(sizeof(typename C::A) * std::max<uint64_t>(cnt + nex, 1));
  pk.idx[slot].ensure(sizeof(uint32_t) * std::max<uint32_t>(cnt, 1));
  DevBuf raw, didx;
  raw.ensure(sizeof(ABI) * std::max<uint64_t>(hi - lo, 1));
  didx.ensure(sizeof(uint32_t) * std::max<uint32_t>(cnt, 1));
  if (hi > lo) ZK_HIP(hipMemcpyAsync(raw.p, v + lo, sizeof(ABI) * (hi - lo), hipMemcpyHostToDevice, st));
  if (cnt) ZK_HIP(hipMemcpyAsync(didx.p, idx.data(), sizeof(uint32_t) * cnt, hipMemcpyHostToDevice, st));
  convert_bases_gather<C>(raw.as<uint64_t>(), didx.as<uint32_t>(), pk.bases[slot].as<typename C::A>(), cnt, st);
  // scalar index = variable / coefficient index
  std::vector<uint32_t> gidx(cnt);
  for (uint32_t k = 0; k < cnt; k++) gidx[k] = (uint32_t)(idx[k] + lo + idx_offset);
  if (cnt) ZK_HIP(hipMemcpyAsync(pk.idx[slot].p, gidx.data(), sizeof(uint32_t) * cnt, hipMemcpyHostToDevice, st));
  if (nex) {
    DevBuf ex;
    ex.ensure(sizeof(ABI) * nex);
    ZK_HIP(hipMemcpyAsync(ex.p, extras.data(), sizeof(ABI) * nex, hipMemcpyHostToDevice, st));
    convert_bases<C>(ex.as<uint64_t>(), pk.bases[slot].as<typename C::A>() + cnt, nex, st);
    ZK_HIP(hipStreamSynchronize(st));
  }
  ZK_HIP(hipStreamSynchronize(st));  // host vectors / staging die here
}

zk_pk_dev* pk_upload(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* q, uint32_t shard, uint32_t nshards) {
  hipStream_t st = ctx->stream;
  std::unique_ptr<zk_pk_dev> d(new zk_pk_dev());
  d->device = ctx->device;
  d->V = q->num_variables;
  d->nc = q->num_constraints;
  d->n = 1;
  while (d->n < d->nc) d->n <<= 1;
  d->log_n = (uint32_t)__builtin_ctzll(d->n);
  d->num_public = pk->num_public;
  d->shard = shard;
  d->nshards = nshards;
  csr_upload(d->csr, q, st);
  const bool first = shard == 0;
  // extras: pi_A gets alpha_1 (scalar 1) and 2^(64k) delta_1 (scalar r_k);
  // pi_B gets beta_2 and 2^(64k) delta_2 (s_k); B_1 gets beta_1.
  std::vector<zk_g1_affine> exA, exB1, none1;
  std::vector<zk_g2_affine> exB2;
  if (first) {
    exA.resize(5);
    exA[0] = pk->alpha_g1;
    pow64_chain<G1>(g1_from_abi(pk->delta_g1), &exA[1]);
    exB2.resize(5);
    exB2[0] = pk->beta_g2;
    pow64_chain<G2>(g2_from_abi(pk->delta_g2), &exB2[1]);
    exB1.push_back(pk->beta_g1);
  }
  const uint64_t V = d->V;
  {
    const uint64_t L = std::min<uint64_t>(pk->a_len, V);  // core:171 i < a_g1.len()
    uint64_t lo = shard_lo(L, shard, nshards), hi = shard_lo(L, shard + 1, nshards);
    upload_vector<G1>(*d, MSM_A, pk->a_g1, lo, hi, 0, exA, st);
  }
  {
    const uint64_t L = std::min<uint64_t>(pk->b2_len, V);  // core:189
    uint64_t lo = shard_lo(L, shard, nshards), hi = shard_lo(L, shard + 1, nshards);
    upload_vector<G2>(*d, MSM_B2, pk->b_g2, lo, hi, 0, exB2, st);
  }
  {
    const uint64_t L = std::min<uint64_t>(pk->b_len, V);  // core:250
    uint64_t lo = shard_lo(L, shard, nshards), hi = shard_lo(L, shard + 1, nshards);
    upload_vector<G1>(*d, MSM_B1, pk->b_g1, lo, hi, 0, exB1, st);
  }
  {
    // ic_g1[k] pairs with variable k + num_public + 1 (core:227-231)
    uint64_t L = std::min<uint64_t>(pk->ic_len, V > pk->num_public + 1 ? V - pk->num_public - 1 : 0);
    uint64_t lo = shard_lo(L, shard, nshards), hi = shard_lo(L, shard + 1, nshards);
    upload_vector<G1>(*d, MSM_IC, pk->ic_g1, lo, hi, pk->num_public + 1, none1, st);
  }
  {
    // h_g1[i] pairs with H coefficient i (zip, core:211-215); H has n
    // coefficients; shard k takes i = k mod nshards
    uint64_t L = std::min<uint64_t>(pk->h_len, d->n);
    upload_vector<G1>(*d, MSM_H, pk->h_g1, std::min<uint64_t>(shard, L), L, 0, none1, st, nshards);
  }
  // the a/b vectors may be shorter than V (core:171 `i < pk.a_g1.len()`): indices stay < V.
  pk_precompute_windows(ctx, *d);
  return d.release();
}

// The prove MSMs all take 64-bit scalars (lo64, core:156-161 / 203-208, and
// the u64 limbs of r, s against 2^(64k) delta): c = 16 gives 4 windows whose
// shifted bases 2^16 P, 2^32 P, 2^48 P are computed once here, so each MSM
// sums into one set of 2^16 buckets instead of 3 x 2^15 + 2^16.
// c = 22 gives 3 windows over 2^21 buckets per MSM instead: 25 % fewer
// accumulate adds against a 32x larger bucket reduction (~12 ms per proof).
// Measured (window sweep): 2x slower at 2^20 constraints, 7 %
// faster at 2^24 -- so 22 from 2^24 constraints per key shard up.
// ZK_PROVE_WIN_C overrides (8..22).
static int prove_win_c(const zk_pk_dev& pk) {
  static const int env = [] {
    const char* e = getenv("ZK_PROVE_WIN_C");
    const int v = e ? atoi(e) : 0;
    return v >= 8 && v <= 22 ? v : 0;
  }();
  if (env) return env;
  return pk.n / std::max<uint64_t>(pk.nshards, 1) >= (1ull << 24) ? 22 : 16;
}

void pk_precompute_windows(zk_ctx* ctx, zk_pk_dev& pk) {
  const char* e = getenv("ZK_MSM_PRECOMP");
  if (e && std::strcmp(e, "0") == 0) return;
  const int PROVE_WIN_C = prove_win_c(pk), PROVE_WIN = (64 + PROVE_WIN_C - 1) / PROVE_WIN_C;
  hipStream_t st = ctx->stream;
  for (int slot = 0; slot < NUM_MSM; slot++) {
    const size_t n = (size_t)pk.count[slot] + pk.extras[slot];
    const size_t asz = slot == MSM_B2 ? sizeof(G2A) : sizeof(G1A);
    DevBuf big;
    big.ensure(asz * std::max<size_t>(n * PROVE_WIN, 1));
    if (n) ZK_HIP(hipMemcpyAsync(big.p, pk.bases[slot].p, asz * n, hipMemcpyDeviceToDevice, st));
    if (slot == MSM_B2) msm_precompute_windows<G2>(big.as<G2A>(), n, PROVE_WIN, PROVE_WIN_C, st);
    else msm_precompute_windows<G1>(big.as<G1A>(), n, PROVE_WIN, PROVE_WIN_C, st);
    ZK_HIP(hipStreamSynchronize(st));
    pk.stride[slot] = slot == MSM_B2 ? msm_pad_bases<G2>(big, n * PROVE_WIN, st)
                                     : msm_pad_bases<G1>(big, n * PROVE_WIN, st);
    pk.bases[slot] = std::move(big);
  }
  pk.win = PROVE_WIN;
  pk.win_c = PROVE_WIN_C;
}

// ---------------------------------------------------------------- prove ---
// Partial accumulators of one shard (host XYZZ, Montgomery).  SC = s A + r B1
// of this shard's A / B1 sums: by linearity the shards' SC add up to the
// s pi_A + r B_1 of pi_C (core:224-265), so each rank pays for its own two
// scalar multiplications while its H MSM is still running.
struct Partial {
  host::X<host::Fq> A, B1, IC, H, SC;
  host::X<host::Fq2> B2;
  int32_t status;
};
static_assert(sizeof(Partial) <= ZK_PARTIAL_BYTES, "partial size");

static void quotient(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, hipStream_t st) {
  const uint64_t n = pk->n;
  NttDomain& dom = ctx->domain(pk->log_n);
  ctx->qa.ensure(sizeof(Fr) * n);
  ctx->qb.ensure(sizeof(Fr) * n);
  ctx->qc.ensure(sizeof(Fr) * n);
  CsrArgs m;
  for (int k = 0; k < 3; k++) {
    m.rp[k] = pk->csr.rp[k].as<uint64_t>();
    m.col[k] = pk->csr.col[k].as<uint32_t>();
    m.val[k] = pk->csr.unit[k] ? nullptr : pk->csr.val[k].as<Fr>();
  }
  const uint64_t vrow = n > 1 ? 1 : 0;
  Prof* pf = &ctx->prof;
  int ph = pf->begin(st, "quotient_eval", n);
  k_csr_eval<<<ceil_div(n, 256), 256, 0, st>>>(m, reinterpret_cast<const Fr*>(d_z), pk->nc, pk->V, n, vrow,
                                                ctx->qa.as<Fr>(), ctx->qb.as<Fr>(), ctx->qc.as<Fr>(),
                                                ctx->flags.as<uint32_t>());
  ZK_LAUNCH_CHECK();
  pf->end(st, ph);
  Fr* v[3] = {ctx->qa.as<Fr>(), ctx->qb.as<Fr>(), ctx->qc.as<Fr>()};
  // per polynomial: iNTT (coefficients * n, bit-reversed), * n^-1 g^i, NTT
  // (evaluations on the coset g<w>, natural order).  Fused into one tile
  // kernel below 2^LARGE_Q_LOG; from there the three steps run as separate
  // passes, and the final coset iNTT runs in natural order (ntt_natural)
  // instead of a DIF plus an element-wise bit-reversed gather.  Same-box
  // A/B, overlapped prove: 2^24 fused 122.8 / separate 118.6 ms; 2^20 the
  // gather path 9.89 / natural 10.01 ms (profiles/r02_ab_quot.txt).
  // ZK_NTT_FUSE=0/1 and ZK_H_NATURAL=0/1 force either choice.
  constexpr uint32_t LARGE_Q_LOG = 23;
  auto env_or = [](const char* name) {
    const char* e = getenv(name);
    return e ? (std::strcmp(e, "0") == 0 ? 0 : 1) : -1;
  };
  static const int fuse_env = env_or("ZK_NTT_FUSE"), nat_env = env_or("ZK_H_NATURAL");
  const bool large = pk->log_n >= LARGE_Q_LOG;
  const bool fuse = fuse_env >= 0 ? fuse_env == 1 : !large;
  const bool natural = nat_env >= 0 ? nat_env == 1 : large;
  for (int k = 0; k < 3; k++) {
    if (fuse) {
      ntt_coset_shift(v[k], dom, dom.gpow_br.as<Fr>(), st, pf);
      continue;
    }
    ntt_dif(v[k], dom, /*inverse twiddles*/ true, st, pf);
    ph = pf->begin(st, "quotient_misc", n);
    fr_scale_table(v[k], dom.gpow_br.as<Fr>(), pk->log_n, false, st);
    pf->end(st, ph);
    ntt_dit(v[k], dom, false, st, pf);
  }
  ph = pf->begin(st, "quotient_misc", n);
  k_quot_pointwise<<<ceil_div(n, 256), 256, 0, st>>>(v[0], v[1], v[2], dom.zinv.as<Fr>(), n);
  ZK_LAUNCH_CHECK();
  pf->end(st, ph);
  // coset iNTT: small domains run a DIF and gather its bit-reversed output
  // element by element (k_h_final, all in the MALL); large ones run it in
  // natural order (the bit reversal is the first pass's tiled gather,
  // n^-1 g^-i fused into the last pass's store) into v[1], v[2] as scratch,
  // since beyond the MALL every gathered 32-B element was its own line/page
  ctx->scal[MSM_H].ensure(sizeof(uint64_t) * n);
  ctx->tmp_scal.ensure(sizeof(uint64_t) * n);
  if (!natural) {
    ntt_dif(v[0], dom, true, st, pf);
    ph = pf->begin(st, "quotient_misc", n);
    k_h_final<<<ceil_div(n, 256), 256, 0, st>>>(v[0], dom.gipow.as<Fr>(), pk->log_n, ctx->tmp_scal.as<uint64_t>());
    ZK_LAUNCH_CHECK();
    pf->end(st, ph);
    return;
  }
  Fr* h = v[1];
  if (pk->log_n == 0) {   // a size-1 transform is the identity: only the factor
    fr_scale_table(v[0], dom.gipow.as<Fr>(), 0, false, st);
    h = v[0];
  } else {
    ntt_natural(v[1], v[0], v[2], dom, true, st, pf, nullptr, dom.gipow.as<Fr>(), nullptr);
  }
  ph = pf->begin(st, "quotient_misc", n);
  k_h_lo64<<<ceil_div(n, 256), 256, 0, st>>>(h, n, ctx->tmp_scal.as<uint64_t>());
  ZK_LAUNCH_CHECK();
  pf->end(st, ph);
}

static bool dist_quotient_enabled() {
  const char* e = getenv("ZK_DIST_QUOTIENT");
  return !(e && std::strcmp(e, "0") == 0);
}

// A sharded key whose ctx is attached to the matching RCCL communicator
// computes its quotient distributed (three all-to-alls per proof).
static bool uses_dist_quotient(const zk_ctx* ctx, const zk_pk_dev* pk) {
  return pk->nshards > 1 && ctx->exch && ctx->exch->world == (int)pk->nshards &&
         ctx->exch->rank == (int)pk->shard && dist_quotient_ok(pk->n, (int)pk->nshards) &&
         dist_quotient_enabled();
}

// h_given (virtual-rank tests): this shard's lo64(H_(shard + nshards d)) is
// already on the device, with the witness-check flags of all ranks.
static Partial prove_partial(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, const zk_fr* r,
                             const zk_fr* s, const uint64_t* h_given = nullptr, uint32_t given_flags = 0) {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  const auto t_start = clk::now();
  hipStream_t st = ctx->stream;
  ctx->flags.ensure(16);
  ctx->prof.mark_origin(st);
  const int ph_span = ctx->prof.begin(st, "prove_gpu_span", pk->n);   // first kernel .. last MSM done
  ZK_HIP(hipMemsetAsync(ctx->flags.p, 0, 16, st));
  check_canonical(d_z, pk->V, ctx->flags.as<uint32_t>(), st);   // every z_i < r, else ZK_ERR_ARG
  // The five MSMs are independent.  Streams (<= GPU_MAX_HW_QUEUES = 4, so no
  // two share a hardware queue): main (high priority) runs the quotient and
  // then the H MSM that depends on it; side[0] (high priority) the G2 MSM,
  // the longest chain; side[1] the IC MSM (3n bases); side[2] A then B1.
  // Latency-bound phases (scan, bucket reduction) of one MSM overlap the
  // throughput-bound accumulation of another.
  ZK_HIP(hipEventRecord(ctx->ev_scal, st));           // z (and flags reset) ready
  static const int sched_env = [] {
    const char* e = getenv("ZK_PROVE_SCHED");
    return e ? atoi(e) : 0;
  }();
  const int sched = ctx->sched >= 0 ? ctx->sched : sched_env;   // zk_ctx_set_schedule overrides
  auto stream_of = [&](int slot) {
    if (sched == 3) return st;   // fully serial (per-phase profiling)
    return slot == MSM_H ? st : slot == MSM_B2 ? ctx->side[0] : slot == MSM_IC ? ctx->side[1] : ctx->side[2];
  };
  // The quotient: local (every coefficient), distributed over the RCCL
  // ranks of a sharded key (this rank's coefficients i = shard mod N), or
  // given (virtual-rank tests).
  const bool dist = !h_given && uses_dist_quotient(ctx, pk);
  const uint64_t* h_src = h_given ? h_given : ctx->tmp_scal.as<uint64_t>();
  const uint32_t h_div = (h_given || dist) ? pk->nshards : 1;
  auto run_quotient = [&]() {
    if (h_given) return;
    if (dist) {
      ctx->tmp_scal.ensure(sizeof(uint64_t) * (pk->n / pk->nshards));
      h_src = ctx->tmp_scal.as<uint64_t>();
      dist_quotient(ctx, pk, d_z, *ctx->exch, ctx->dq, ctx->flags.as<uint32_t>(), ctx->tmp_scal.as<uint64_t>(), st);
    } else {
      quotient(ctx, pk, d_z, st);   // (Az, Bz, Cz) -> lo64(H) in tmp_scal
      h_src = ctx->tmp_scal.as<uint64_t>();
    }
  };
  // scalars of one MSM: lo64 of its variables (or H coefficients), then the
  // extras' scalars (1 for alpha_1 / beta_2 / beta_1, the u64 limbs of r or s)
  auto prep_scalars = [&](int slot, hipStream_t ss) {
    const uint32_t cnt = pk->count[slot], nex = pk->extras[slot];
    ctx->scal[slot].ensure(sizeof(uint64_t) * std::max<uint32_t>(cnt + nex, 1));
    if (cnt) {
      const uint64_t* src = slot == MSM_H ? h_src : d_z;
      const int stride = slot == MSM_H ? 1 : 4;
      k_gather_lo64<<<ceil_div(cnt, 256), 256, 0, ss>>>(src, stride, pk->idx[slot].as<uint32_t>(),
                                                         slot == MSM_H ? h_div : 1u, cnt,
                                                         ctx->scal[slot].as<uint64_t>());
      ZK_LAUNCH_CHECK();
    }
    if (nex) {
      Extras ex{};
      ex.v[0] = 1;
      const zk_fr* full = slot == MSM_A ? r : slot == MSM_B2 ? s : nullptr;
      if (full) for (int k = 0; k < 4; k++) ex.v[1 + k] = full->l[k];
      k_set_extras<<<1, 64, 0, ss>>>(ctx->scal[slot].as<uint64_t>() + cnt, ex, nex);
      ZK_LAUNCH_CHECK();
    }
  };
  auto launch_slot = [&](int slot, hipStream_t ss) {
    prep_scalars(slot, ss);
    const uint32_t n = pk->count[slot] + pk->extras[slot];
    if (slot == MSM_B2) {
      if (pk->win > 1)
        msm_launch_shared<G2>(ctx->msm[slot], pk->bases[slot].as<G2A>(), ctx->scal[slot].as<uint64_t>(), 1, n, 64,
                              pk->win_c, ss, pk->stride[slot]);
      else
        msm_launch<G2>(ctx->msm[slot], pk->bases[slot].as<G2A>(), ctx->scal[slot].as<uint64_t>(), 1, n, 64, ss,
                       pk->stride[slot]);
      msm_download<G2>(ctx->msm[slot], ss);
    } else {
      if (pk->win > 1)
        msm_launch_shared<G1>(ctx->msm[slot], pk->bases[slot].as<G1A>(), ctx->scal[slot].as<uint64_t>(), 1, n, 64,
                              pk->win_c, ss, pk->stride[slot]);
      else
        msm_launch<G1>(ctx->msm[slot], pk->bases[slot].as<G1A>(), ctx->scal[slot].as<uint64_t>(), 1, n, 64, ss,
                       pk->stride[slot]);
      msm_download<G1>(ctx->msm[slot], ss);
    }
  };
  static const char* const tags[NUM_MSM] = {"A/", "B2/", "B1/", "IC/", "H/"};
  for (int slot = 0; slot < NUM_MSM; slot++) ctx->msm[slot].tag = sched == 3 ? tags[slot] : "";
  // Batched G1 (default with window-shifted keys): the G1 MSMs run in groups,
  // each group ONE msm_launch_batch (one sort, accumulate, merge and bucket
  // reduction, so the latency-bound tails cost one tree depth per group) in
  // the workspace of its first slot.  ZK_G1_GROUPS lists the groups, letters
  // A (pi_A), B (B_1), I (IC), H (H), comma-separated; default "ABI,H": A, B1
  // and IC start on side[1] with the witness, H follows the quotient on the
  // main stream, the G2 MSM runs on side[0].  ZK_PROVE_SCHED: 0 G2 starts
  // with the witness, 1 G2 waits for the quotient, 3 everything serial on
  // main.  ZK_MSM_BATCH=0 keeps one MSM per slot on four streams (below).
  static const bool batch_env = [] {
    const char* e = getenv("ZK_MSM_BATCH");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  static const std::vector<std::vector<int>> groups = [] {
    const char* e = getenv("ZK_G1_GROUPS");
    std::string spec = e ? e : "ABI,H";
    std::vector<std::vector<int>> g(1);
    for (char ch : spec) {
      if (ch == ',') { if (!g.back().empty()) g.emplace_back(); continue; }
      const int slot = ch == 'A' ? MSM_A : ch == 'B' ? MSM_B1 : ch == 'I' ? MSM_IC : ch == 'H' ? MSM_H : -1;
      if (slot >= 0) g.back().push_back(slot);
    }
    if (g.back().empty()) g.pop_back();
    int seen = 0;
    for (auto& grp : g) for (int sl : grp) seen |= 1 << sl;
    if (seen != ((1 << MSM_A) | (1 << MSM_B1) | (1 << MSM_IC) | (1 << MSM_H)))
      g = {{MSM_A, MSM_B1, MSM_IC}, {MSM_H}};
    return g;
  }();
  const bool batch = batch_env && pk->win > 1;
  std::vector<int> waits;   // slots whose ev_done the host tail waits for
  if (batch) {
    hipStream_t s2 = sched == 3 ? st : ctx->side[0];
    auto launch_group = [&](const std::vector<int>& grp, hipStream_t gs) {
      MsmSeg segs[MSM_MAXSEG];
      for (size_t k = 0; k < grp.size(); k++) {
        const int slot = grp[k];
        prep_scalars(slot, gs);
        segs[k] = MsmSeg{pk->bases[slot].p, ctx->scal[slot].as<uint64_t>(), pk->count[slot] + pk->extras[slot],
                         pk->stride[slot]};
      }
      MsmWork& w = ctx->msm[grp[0]];
      if (sched == 3) {
        w.tag.clear();
        for (int sl : grp) w.tag += tags[sl][0];
        w.tag += "/";
      }
      msm_launch_batch<G1>(w, segs, (int)grp.size(), 64, pk->win_c, gs);
      msm_download<G1>(w, gs);
      ZK_HIP(hipEventRecord(ctx->ev_done[grp[0]], gs));
      waits.push_back(grp[0]);
    };
    auto has_h = [](const std::vector<int>& grp) { return std::find(grp.begin(), grp.end(), (int)MSM_H) != grp.end(); };
    // ZK_PROVE_SCHED=4: the quotient's kernels are queued first (host launch
    // order only, no waits), then the G2 MSM and the groups.  5: the same,
    // and the side streams' accumulate kernels wait for the quotient (their
    // key and sort passes still overlap it): a full-occupancy accumulate
    // round otherwise holds every SIMD's registers and starves the
    // quotient's LDS-tiled NTT passes, which delays the H MSM behind it.
    // 6: the H group's key and sort passes also go ahead (queued right
    // after the quotient on the main stream) and every accumulate waits for
    // them -- sorts and the quotient share the chip, the accumulates start
    // together once every MSM's entries are grouped.  7: as 6, but the G2
    // accumulate starts with the witness; only the batched G1 accumulates
    // wait for the H group's sort.
    for (int sl = 0; sl < NUM_MSM; sl++) {
      ctx->msm[sl].accum_wait = nullptr;
      ctx->msm[sl].sort_done = nullptr;
      ctx->msm[sl].accum_done = nullptr;
    }
    if (sched >= 4 && sched <= 8) run_quotient();
    // 8: the quotient first, then the accumulates one after another in
    // ZK_ACCUM_ORDER ('H' the H group, '2' the G2 MSM, 'A' the other G1
    // groups; default "H2A"): every sort still starts with the witness, and
    // each MSM's latency-bound tail (merge, bucket sums) overlaps the next
    // accumulate instead of three full-occupancy rounds fighting for the chip.
    if (sched == 8) {
      static const std::string order = [] {
        const char* e = getenv("ZK_ACCUM_ORDER");
        std::string o = e ? e : "H2A";
        std::string s = o;
        std::sort(s.begin(), s.end());
        return s == "2AH" ? o : std::string("H2A");
      }();
      ZK_HIP(hipEventRecord(ctx->ev_quot, st));
      ctx->flags_host.ensure(16);
      ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
      hipEvent_t prev = ctx->ev_quot;
      int side = 1;
      for (char u : order) {
        if (u == '2') {
          MsmWork& w = ctx->msm[MSM_B2];
          w.accum_wait = prev;
          w.accum_done = prev = ctx->ev_acc[MSM_B2];
          ZK_HIP(hipStreamWaitEvent(s2, ctx->ev_scal, 0));
          launch_slot(MSM_B2, s2);
          continue;
        }
        for (const auto& grp : groups) {
          if (has_h(grp) != (u == 'H')) continue;
          MsmWork& w = ctx->msm[grp[0]];
          w.accum_wait = (u == 'H' && prev == ctx->ev_quot) ? nullptr : prev;   // H: same stream as the quotient
          w.accum_done = prev = ctx->ev_acc[grp[0]];
          hipStream_t gs = st;
          if (u != 'H') {
            gs = ctx->side[side];
            side = side + 1 < NUM_SIDE ? side + 1 : 1;
            ZK_HIP(hipStreamWaitEvent(gs, ctx->ev_scal, 0));
          }
          launch_group(grp, gs);
        }
      }
    }
    if (sched == 5) {
      ZK_HIP(hipEventRecord(ctx->ev_quot, st));
      for (int sl = 0; sl < NUM_MSM; sl++) ctx->msm[sl].accum_wait = sl == MSM_H ? nullptr : ctx->ev_quot;
    }
    if (sched == 6 || sched == 7) {
      ctx->flags_host.ensure(16);
      ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
      for (const auto& grp : groups)
        if (has_h(grp)) {
          ctx->msm[grp[0]].sort_done = ctx->ev_hsort;
          launch_group(grp, st);
        }
      for (int sl = 0; sl < NUM_MSM; sl++) ctx->msm[sl].accum_wait = ctx->ev_hsort;
      for (const auto& grp : groups)
        if (has_h(grp)) ctx->msm[grp[0]].accum_wait = nullptr;
      if (sched == 7) ctx->msm[MSM_B2].accum_wait = nullptr;
    }
    // the G2 MSM starts with the witness (ZK_PROVE_SCHED=1: after the quotient, below)
    if (sched == 3) {
      launch_slot(MSM_B2, st);
    } else if (sched != 1 && sched != 8 && sched != 9) {
      ZK_HIP(hipStreamWaitEvent(s2, ctx->ev_scal, 0));
      launch_slot(MSM_B2, s2);
    }
    // groups without H start with the witness on side[1], side[2], ...
    // 9: as 0, but the G2 accumulate waits until these groups' entries are
    // sorted, so its full-occupancy round cannot starve their sorts (and
    // with them the start of the largest accumulate).
    int side = 1;
    std::vector<hipStream_t> used;
    hipEvent_t g1_sorted = nullptr;
    for (const auto& grp : groups) {
      if (has_h(grp) || sched == 8) continue;
      hipStream_t gs = st;
      if (sched != 3) {
        gs = ctx->side[side];
        side = side + 1 < NUM_SIDE ? side + 1 : 1;
        ZK_HIP(hipStreamWaitEvent(gs, ctx->ev_scal, 0));
        used.push_back(gs);
      }
      if (sched == 9) ctx->msm[grp[0]].sort_done = g1_sorted = ctx->ev_acc[grp[0]];
      launch_group(grp, gs);
    }
    if (sched == 9) {
      ZK_HIP(hipStreamWaitEvent(s2, ctx->ev_scal, 0));
      ctx->msm[MSM_B2].accum_wait = g1_sorted;
      launch_slot(MSM_B2, s2);
    }
    if (sched < 4 || sched > 8) run_quotient();
    if (sched == 1) {
      ZK_HIP(hipEventRecord(ctx->ev_quot, st));
      ZK_HIP(hipStreamWaitEvent(s2, ctx->ev_quot, 0));
      launch_slot(MSM_B2, s2);
    }
    ZK_HIP(hipEventRecord(ctx->ev_done[MSM_B2], s2));
    waits.push_back(MSM_B2);
    if (sched != 6 && sched != 7 && sched != 8) {
      ctx->flags_host.ensure(16);
      ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
      for (const auto& grp : groups)
        if (has_h(grp)) launch_group(grp, st);
    }
    if (ph_span >= 0) {
      for (int sl : waits) ZK_HIP(hipStreamWaitEvent(st, ctx->ev_done[sl], 0));
      ctx->prof.end(st, ph_span);
    }
  } else {
    // ZK_PROVE_SCHED=3: everything on the main stream, in order, with per-MSM
    // phase names.  Default: the four independent MSMs start on the side
    // streams, the quotient and then H on the main one.
    for (int k = 0; k < NUM_SIDE; k++) ZK_HIP(hipStreamWaitEvent(ctx->side[k], ctx->ev_scal, 0));
    for (int slot : {MSM_B2, MSM_IC, MSM_A, MSM_B1}) {
      launch_slot(slot, stream_of(slot));
      ZK_HIP(hipEventRecord(ctx->ev_done[slot], stream_of(slot)));
    }
    run_quotient();
    ctx->flags_host.ensure(16);
    ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
    launch_slot(MSM_H, st);
    ZK_HIP(hipEventRecord(ctx->ev_done[MSM_H], st));
    waits = {MSM_A, MSM_B2, MSM_B1, MSM_IC, MSM_H};
    if (ph_span >= 0) {
      for (int slot : {MSM_B2, MSM_IC, MSM_A, MSM_B1}) ZK_HIP(hipStreamWaitEvent(st, ctx->ev_done[slot], 0));
      ctx->prof.end(st, ph_span);
    }
  }

  // Host tails (Horner over each MSM's partials, then s A + r B1) run as
  // each MSM's stream reaches its event, overlapping the MSMs still on the
  // GPU.
  ctx->prof.add_host("host_launch", ms_since(t_start));
  double t_fin = 0;
  Partial p{};
  std::vector<bool> done(waits.size(), false);
  bool sc_done = false, a_done = false, b1_done = false;
  for (size_t left = waits.size(); left > 0;) {
    bool progressed = false;
    for (size_t wi = 0; wi < waits.size(); wi++) {
      if (done[wi]) continue;
      const int slot = waits[wi];
      const hipError_t q = hipEventQuery(ctx->ev_done[slot]);
      if (q == hipErrorNotReady) continue;
      ZK_HIP(q);
      const auto t_f = clk::now();
      auto take = [&](int sl, const host::X<host::Fq>& v) {
        switch (sl) {
          case MSM_A: p.A = v; a_done = true; break;
          case MSM_B1: p.B1 = v; b1_done = true; break;
          case MSM_IC: p.IC = v; break;
          case MSM_H: p.H = v; break;
        }
      };
      if (slot == MSM_B2) {
        p.B2 = msm_finish<G2>(ctx->msm[slot]);
      } else if (batch) {
        for (const auto& grp : groups)
          if (grp[0] == slot)
            for (size_t k = 0; k < grp.size(); k++) take(grp[k], msm_finish_seg<G1>(ctx->msm[slot], (int)k));
      } else {
        take(slot, msm_finish<G1>(ctx->msm[slot]));
      }
      done[wi] = progressed = true;
      left--;
      if (!sc_done && a_done && b1_done) {
        p.SC = host::mul2_scalar(p.A, s->l, p.B1, r->l);
        sc_done = true;
      }
      t_fin += ms_since(t_f);
      if (left == 0) ctx->prof.add_host("host_tail_after_last", ms_since(t_f));
    }
    if (!progressed) std::this_thread::yield();
  }
  for (int k = 0; k < NUM_SIDE; k++) ZK_HIP(hipStreamSynchronize(ctx->side[k]));
  ZK_HIP(hipStreamSynchronize(st));
  for (int sl = 0; sl < NUM_MSM; sl++) {
    ctx->msm[sl].accum_wait = nullptr;
    ctx->msm[sl].sort_done = nullptr;
    ctx->msm[sl].accum_done = nullptr;
  }
  ctx->prof.add_host("host_finish", t_fin);
  ctx->prof.collect();
  const uint32_t flags = h_given ? given_flags : *ctx->flags_host.as<uint32_t>();
  p.status = ZK_OK;
  if (flags & 8u) p.status = ZK_ERR_ARG;
  else if (flags & 5u) p.status = ZK_ERR_INVALID_WITNESS;
  else if (flags & 2u) p.status = ZK_ERR_QAP_DIVISION;
  return p;
}

static int combine(const Partial* parts, size_t k, zk_proof* out) {
  // the witness checks are spread over the ranks' rows: a non-canonical
  // input (ZK_ERR_ARG) first, then InvalidWitness (core:83-98, 124-128)
  // wins over the division failure (qap:266)
  for (size_t i = 0; i < k; i++)
    if (parts[i].status == ZK_ERR_ARG) return ZK_ERR_ARG;
  for (size_t i = 0; i < k; i++)
    if (parts[i].status == ZK_ERR_INVALID_WITNESS) return ZK_ERR_INVALID_WITNESS;
  for (size_t i = 0; i < k; i++)
    if (parts[i].status != ZK_OK) return parts[i].status;
  auto A = host::inf<host::Fq>(), C = A;
  auto B2 = host::inf<host::Fq2>();
  for (size_t i = 0; i < k; i++) {
    A = host::addp(A, parts[i].A);
    B2 = host::addp(B2, parts[i].B2);
    // pi_C = IC + H_1 + s pi_A + r B_1 (core:224-265; identity terms add nothing)
    C = host::addp(C, host::addp(host::addp(parts[i].IC, parts[i].H), parts[i].SC));
  }
  host_to_abi<G1>(A, reinterpret_cast<uint64_t*>(&out->a));
  host_to_abi<G2>(B2, reinterpret_cast<uint64_t*>(&out->b));
  host_to_abi<G1>(C, reinterpret_cast<uint64_t*>(&out->c));
  return ZK_OK;
}

int prove_impl(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, size_t zlen, size_t num_public,
               const zk_fr* r, const zk_fr* s, zk_proof* out) {
  // Witness::new (core:81-99) and the length check of validate (core:113-118)
  if (!fr_canonical(*r) || !fr_canonical(*s)) return ZK_ERR_ARG;   // Fr::rand draws are reduced
  if (num_public >= zlen) return ZK_ERR_INVALID_WITNESS;
  if (zlen != pk->V) return ZK_ERR_INVALID_WITNESS;
  if (pk->nshards != 1) return ZK_ERR_ARG;
  Partial p = prove_partial(ctx, pk, reinterpret_cast<const uint64_t*>(d_z), r, s);
  return combine(&p, 1, out);
}

int prove_partial_impl(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, size_t zlen, size_t num_public,
                       const zk_fr* r, const zk_fr* s, zk_prove_partial* out) {
  std::memset(out, 0, sizeof *out);
  Partial p{};
  int local = ZK_OK;
  if (!fr_canonical(*r) || !fr_canonical(*s)) local = ZK_ERR_ARG;
  else if (num_public >= zlen || zlen != pk->V) local = ZK_ERR_INVALID_WITNESS;
  // Ranks of a distributed quotient agree on the host-side checks before
  // the first all-to-all: a rank that bailed out alone would leave its
  // peers blocked in the collective.
  if (uses_dist_quotient(ctx, pk)) {
    const int agreed = ctx->exch->agree_max(local, ctx->stream);
    if (local == ZK_OK) local = agreed;
  }
  if (local != ZK_OK) {
    p.status = local;
  } else {
    p = prove_partial(ctx, pk, reinterpret_cast<const uint64_t*>(d_z), r, s);
  }
  std::memcpy(out->bytes, &p, sizeof p);
  return p.status;
}

// N virtual ranks of a sharded key on ONE device: the distributed quotient's
// stages run rank by rank, its three all-to-alls become device copies, then
// each rank's MSMs and the fold.  Exercises exactly the per-rank code and
// index maps the RCCL path runs (tests; the RCCL path needs N devices).
int prove_virtual_shards_impl(zk_ctx* ctx, const zk_pk_dev* const* pks, uint32_t N, const void* d_z, size_t zlen,
                              size_t num_public, const zk_fr* r, const zk_fr* s, zk_proof* out) {
  if (N < 2) return ZK_ERR_ARG;
  for (uint32_t k = 0; k < N; k++)
    if (!pks[k] || pks[k]->shard != k || pks[k]->nshards != N || pks[k]->n != pks[0]->n) return ZK_ERR_ARG;
  const zk_pk_dev* pk0 = pks[0];
  if (!fr_canonical(*r) || !fr_canonical(*s)) return ZK_ERR_ARG;
  if (num_public >= zlen || zlen != pk0->V) return ZK_ERR_INVALID_WITNESS;
  if (!dist_quotient_ok(pk0->n, (int)N)) return ZK_ERR_ARG;
  hipStream_t st = ctx->stream;
  const uint64_t* z = reinterpret_cast<const uint64_t*>(d_z);
  const uint64_t m = pk0->n / N;
  std::vector<DistQ> dq(N);
  std::vector<DevBuf> hb(N);
  DevBuf flags;
  flags.ensure(sizeof(uint32_t) * N);
  ZK_HIP(hipMemsetAsync(flags.p, 0, sizeof(uint32_t) * N, st));
  check_canonical(d_z, zlen, flags.as<uint32_t>(), st);
  auto exchange = [&](int which) {
    const size_t chunk = dq_chunk_bytes(pk0, (int)N, which);
    for (uint32_t a = 0; a < N; a++)
      for (uint32_t b = 0; b < N; b++) {
        const DevBuf& src = which == 1 ? dq[b].s1 : which == 2 ? dq[b].s2 : dq[b].s3;
        DevBuf& dst = which == 1 ? dq[a].r1 : which == 2 ? dq[a].r2 : dq[a].r3;
        ZK_HIP(hipMemcpyAsync(static_cast<char*>(dst.p) + b * chunk, static_cast<const char*>(src.p) + a * chunk,
                              chunk, hipMemcpyDeviceToDevice, st));
      }
  };
  for (uint32_t k = 0; k < N; k++) dq_stage_a(ctx, pks[k], z, (int)k, (int)N, dq[k], flags.as<uint32_t>() + k, st);
  exchange(1);
  for (uint32_t k = 0; k < N; k++) dq_stage_b(ctx, pks[k], (int)k, (int)N, dq[k], st);
  exchange(2);
  for (uint32_t k = 0; k < N; k++) dq_stage_c(ctx, pks[k], (int)k, (int)N, dq[k], st);
  exchange(3);
  for (uint32_t k = 0; k < N; k++) {
    hb[k].ensure(sizeof(uint64_t) * m);
    dq_stage_d(ctx, pks[k], (int)k, (int)N, dq[k], hb[k].as<uint64_t>(), st);
  }
  std::vector<uint32_t> hf(N);
  ZK_HIP(hipMemcpyAsync(hf.data(), flags.p, sizeof(uint32_t) * N, hipMemcpyDeviceToHost, st));
  ZK_HIP(hipStreamSynchronize(st));
  uint32_t all = 0;
  for (uint32_t f : hf) all |= f;
  if (all & 8u) return ZK_ERR_ARG;
  std::vector<Partial> parts(N);
  for (uint32_t k = 0; k < N; k++) parts[k] = prove_partial(ctx, pks[k], z, r, s, hb[k].as<uint64_t>(), all);
  return combine(parts.data(), N, out);
}

int combine_impl(const zk_prove_partial* parts, size_t k, const zk_fr* r, const zk_fr* s, zk_proof* out) {
  std::vector<Partial> ps(k);
  for (size_t i = 0; i < k; i++) std::memcpy(&ps[i], parts[i].bytes, sizeof(Partial));
  (void)r;
  (void)s;
  return combine(ps.data(), k, out);
}

}  // namespace zk
