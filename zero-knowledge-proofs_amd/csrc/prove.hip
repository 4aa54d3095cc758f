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
  if (!fr_lt_r(ld_vec(&z[i]))) atomicOr(flags, 8u);
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

// Upload the non-identity entries at positions lo, lo + stride, ... < hi of
// one base vector that `take` accepts, compacted, and append the extras.
// stride > 1: the H coefficients of a shard, i = shard mod nshards, which is
// where the distributed quotient leaves them.  The scalar of position i is
// z_(i + idx_offset) (H: coefficient i).
template <class C, class ABI, class Take>
static void upload_vector(zk_pk_dev& pk, int slot, const ABI* v, uint64_t lo, uint64_t hi, uint64_t idx_offset,
                          const std::vector<ABI>& extras, hipStream_t st, uint64_t stride, Take take) {
  std::vector<uint32_t> gidx;
  std::vector<ABI> pts;
  for (uint64_t i = lo; i < hi; i += stride)
    if (!v[i].infinity && take(i)) {
      gidx.push_back((uint32_t)(i + idx_offset));
      pts.push_back(v[i]);
    }
  const uint32_t cnt = (uint32_t)gidx.size();
  const uint32_t nex = (uint32_t)extras.size();
  if (slot == MSM_H) {
    pk.h_ident = true;
    for (uint32_t k = 0; k < cnt; k++) pk.h_ident = pk.h_ident && gidx[k] == k;
  }
  pk.count[slot] = cnt;
  pk.extras[slot] = nex;
  pk.bases[slot].ensure(sizeof(typename C::A) * std::max<uint64_t>(cnt + nex, 1));
  pk.idx[slot].ensure(sizeof(uint32_t) * std::max<uint32_t>(cnt, 1));
  DevBuf raw;
  raw.ensure(sizeof(ABI) * std::max<uint64_t>(cnt, 1));
  if (cnt) ZK_HIP(hipMemcpyAsync(raw.p, pts.data(), sizeof(ABI) * cnt, hipMemcpyHostToDevice, st));
  convert_bases<C>(raw.as<uint64_t>(), pk.bases[slot].as<typename C::A>(), cnt, st);
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

// Positions [0, L) of a base vector whose position i pairs with variable
// i + off: this shard's variables (var_owner), or its contiguous range.
template <class C, class ABI>
static void vector_shard(zk_pk_dev& d, int slot, const ABI* v, uint64_t L, uint64_t off, const std::vector<ABI>& extras,
                         const std::vector<uint8_t>& own, hipStream_t st) {
  const uint32_t k = d.shard, N = d.nshards;
  if (own.empty())
    upload_vector<C>(d, slot, v, shard_lo(L, k, N), shard_lo(L, k + 1, N), off, extras, st, 1,
                     [](uint64_t) { return true; });
  else
    upload_vector<C>(d, slot, v, 0, L, off, extras, st, 1, [&](uint64_t i) { return own[i + off] == k; });
}

zk_pk_dev* pk_upload(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* q, uint32_t shard, uint32_t nshards) {
  hipStream_t st = ctx->stream;
  std::unique_ptr<zk_pk_dev> d(new zk_pk_dev());
  d->device = ctx->device;
  d->V = q->num_variables;
  d->nc = q->num_constraints;
  if (d->nc > (1ull << 32)) throw Error(ZK_ERR_DOMAIN, "more than 2^32 constraints (Fr 2-adicity 32)");
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
  const std::vector<uint8_t> own = var_owner(q, d->n, nshards);
  vector_shard<G1>(*d, MSM_A, pk->a_g1, std::min<uint64_t>(pk->a_len, V), 0, exA, own, st);     // core:171
  vector_shard<G2>(*d, MSM_B2, pk->b_g2, std::min<uint64_t>(pk->b2_len, V), 0, exB2, own, st);  // core:189
  vector_shard<G1>(*d, MSM_B1, pk->b_g1, std::min<uint64_t>(pk->b_len, V), 0, exB1, own, st);   // core:250
  // ic_g1[k] pairs with variable k + num_public + 1 (core:227-231)
  vector_shard<G1>(*d, MSM_IC, pk->ic_g1,
                   std::min<uint64_t>(pk->ic_len, V > pk->num_public + 1 ? V - pk->num_public - 1 : 0),
                   pk->num_public + 1, none1, own, st);
  {
    // h_g1[i] pairs with H coefficient i (zip, core:211-215); H has n
    // coefficients; shard k takes i = k mod nshards
    uint64_t L = std::min<uint64_t>(pk->h_len, d->n);
    upload_vector<G1>(*d, MSM_H, pk->h_g1, std::min<uint64_t>(shard, L), L, 0, none1, st, nshards,
                      [](uint64_t) { return true; });
  }
  // the a/b vectors may be shorter than V (core:171 `i < pk.a_g1.len()`): indices stay < V.
  pk_precompute_windows(ctx, *d);
  pk_witness_ranges(*d, q, own, st);
  pk_part_cuts(*d, st);
  return d.release();
}

// out[k] = first position of idx[0, count) holding a value >= key (the idx
// vectors ascend: compaction keeps variable order)
__global__ void k_lower_bound(const uint32_t* __restrict__ idx, uint32_t count, uint64_t key, uint32_t* __restrict__ out) {
  uint32_t lo = 0, hi = count;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if ((uint64_t)idx[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

// The parts of a host witness grow geometrically, ZK_HOST_PART_RATIO times
// each (2 parts, ratio 2: the first third, then the rest): the MSM work of
// the parts already on the device outlasts the copy of the next one.  Every
// part costs its own sort, bucket fixup and combine on the G2 and A+B1+IC
// streams, so more, smaller parts lose what the smaller exposed first copy
// saves.  Host-witness minus device-witness prove at 2^20 (tools/pcie_ab.py,
// medians of 4 alternating processes, profiles/r05_ab_host_parts.txt): 2
// parts +0.864 ms, 3 parts (ratio 3) +1.042, 4 parts (ratio 2.5) +1.231;
// round 4 with 2 parts, first part 1/2 +1.33, 1/3 +0.84, 1/4 +0.86, 1/6 +1.29
// (profiles/r04_ab_host_split.txt).  (ZK_HOST_PARTS / ZK_HOST_PART_RATIO:
// A/B builds only.)
#ifndef ZK_HOST_PART_RATIO
#define ZK_HOST_PART_RATIO 2
#endif
void pk_part_cuts(zk_pk_dev& pk, hipStream_t st) {
  double w = 1, tot = 0;
  double f[HOST_PARTS];
  for (int k = 0; k < HOST_PARTS; k++, w *= ZK_HOST_PART_RATIO) tot += (f[k] = w);
  double acc = 0;
  pk.vcut[0] = 0;
  for (int k = 1; k < HOST_PARTS; k++) {
    acc += f[k - 1] / tot;
    pk.vcut[k] = std::max<uint64_t>(pk.vcut[k - 1], (uint64_t)(acc * (double)pk.V));
  }
  pk.vcut[HOST_PARTS] = pk.V;
  DevBuf d;
  d.ensure(sizeof(uint32_t) * NUM_MSM * (HOST_PARTS + 1));
  ZK_HIP(hipMemsetAsync(d.p, 0, sizeof(uint32_t) * NUM_MSM * (HOST_PARTS + 1), st));
  for (int k = 1; k < HOST_PARTS; k++)
    for (int slot : {MSM_A, MSM_B2, MSM_B1, MSM_IC})
      if (pk.count[slot]) {
        k_lower_bound<<<1, 1, 0, st>>>(pk.idx[slot].as<uint32_t>(), pk.count[slot], pk.vcut[k],
                                       d.as<uint32_t>() + k * NUM_MSM + slot);
        ZK_LAUNCH_CHECK();
      }
  ZK_HIP(hipMemcpyAsync(pk.pcut, d.p, sizeof(uint32_t) * NUM_MSM * (HOST_PARTS + 1), hipMemcpyDeviceToHost, st));
  ZK_HIP(hipStreamSynchronize(st));
  for (int slot = 0; slot < NUM_MSM; slot++) pk.pcut[HOST_PARTS][slot] = pk.count[slot];
}

std::vector<uint8_t> var_owner(const zk_r1cs_csr* q, uint64_t n, uint32_t N) {
  std::vector<uint8_t> own;
  if (N < 2 || !dist_quotient_ok(n, (int)N)) return own;
  const uint64_t V = q->num_variables, nc = q->num_constraints, m = n / N, qq = m / N;
  own.assign(V, 0xff);
  const uint64_t* rps[3] = {q->a_rowptr, q->b_rowptr, q->c_rowptr};
  const uint32_t* cols[3] = {q->a_col, q->b_col, q->c_col};
  for (uint64_t j = 0; j < nc; j++) {   // rank of row j: its column b = j mod m lies in [rank q, rank q + q)
    const uint8_t rk = (uint8_t)((j % m) / qq);
    for (int mtx = 0; mtx < 3; mtx++)
      for (uint64_t e = rps[mtx][j]; e < rps[mtx][j + 1]; e++) {
        const uint32_t c = cols[mtx][e];
        if (c < V && own[c] == 0xff) own[c] = rk;
      }
  }
  for (uint64_t v = 0; v < V; v++)
    if (own[v] == 0xff) own[v] = (uint8_t)(v * N / V);
  return own;
}

// Exactly the z entries a shard reads when its quotient is distributed:
// z_0 (the constant check, core:89-93), the variables behind its compacted
// A / B2 / B1 / IC bases (the idx vectors) and the columns of the rows its
// column slice evaluates (dist.hip stage A: rows a m + rank q + b', a < N,
// b' < q), plus the variables var_owner gives this shard: a variable no row
// references and whose bases are all the identity is read by no stage, but
// it must still be checked canonical by some rank (the one-GPU prove rejects
// z_i >= r anywhere).  For a variable rows do reference, its owner's rows
// read it anyway.  Sorted, merged into ranges.
void pk_witness_ranges(zk_pk_dev& pk, const zk_r1cs_csr* q, const std::vector<uint8_t>& own, hipStream_t st) {
  pk.wr_dist.clear();
  if (pk.nshards < 2 || !dist_quotient_ok(pk.n, (int)pk.nshards)) return;
  std::vector<uint32_t> vars;
  for (int slot : {MSM_A, MSM_B2, MSM_B1, MSM_IC}) {
    const size_t k = vars.size();
    vars.resize(k + pk.count[slot]);
    if (pk.count[slot])
      ZK_HIP(hipMemcpyAsync(vars.data() + k, pk.idx[slot].p, sizeof(uint32_t) * pk.count[slot],
                            hipMemcpyDeviceToHost, st));
  }
  ZK_HIP(hipStreamSynchronize(st));
  vars.push_back(0);
  for (uint64_t v = 0; v < own.size(); v++)
    if (own[v] == pk.shard) vars.push_back((uint32_t)v);
  const uint64_t N = pk.nshards, m = pk.n / N, qq = m / N;
  const uint64_t* rps[3] = {q->a_rowptr, q->b_rowptr, q->c_rowptr};
  const uint32_t* cols[3] = {q->a_col, q->b_col, q->c_col};
  for (uint64_t a = 0; a < N; a++)
    for (uint64_t b = 0; b < qq; b++) {
      const uint64_t j = a * m + pk.shard * qq + b;
      if (j >= pk.nc) continue;
      for (int mtx = 0; mtx < 3; mtx++)
        for (uint64_t e = rps[mtx][j]; e < rps[mtx][j + 1]; e++)
          if (cols[mtx][e] < pk.V) vars.push_back(cols[mtx][e]);   // columns >= V are ignored (qap:122-124)
    }
  std::sort(vars.begin(), vars.end());
  vars.erase(std::unique(vars.begin(), vars.end()), vars.end());
  for (uint32_t v : vars) {
    if (!pk.wr_dist.empty() && pk.wr_dist.back() == v) pk.wr_dist.back() = (uint64_t)v + 1;
    else {
      pk.wr_dist.push_back(v);
      pk.wr_dist.push_back((uint64_t)v + 1);
    }
  }
}

// The prove MSMs all take 64-bit scalars (lo64, core:156-161 / 203-208, and
// the u64 limbs of r, s against 2^(64k) delta): c = 16 gives 4 windows whose
// shifted bases 2^16 P, 2^32 P, 2^48 P are computed once here, so each MSM
// sums into one set of 2^16 buckets instead of 3 x 2^15 + 2^16.
// c = 22 gives 3 windows over 2^21 buckets per MSM instead: 25 % fewer
// accumulate adds against a 32x larger bucket reduction (~12 ms per proof).
// Measured (window sweep): 2x slower at 2^20 constraints, 7 %
// faster at 2^24 -- so 22 from 2^24 constraints per key shard up.
// zk_ctx_set_option(ZK_OPT_PROVE_WIN_C) forces 16 or 22 (tests).
static int prove_win_c(const zk_ctx* ctx, const zk_pk_dev& pk) {
  if (ctx->prove_win_c) return ctx->prove_win_c;
  return pk.n / std::max<uint64_t>(pk.nshards, 1) >= (1ull << 24) ? 22 : 16;
}

void pk_precompute_windows(zk_ctx* ctx, zk_pk_dev& pk) {
  const int PROVE_WIN_C = prove_win_c(ctx, pk), PROVE_WIN = (64 + PROVE_WIN_C - 1) / PROVE_WIN_C;
  hipStream_t st = ctx->stream;
  for (int slot = 0; slot < NUM_MSM; slot++) {
    if (slot == MSM_IC) continue;   // windowed together with H (zk_pk_dev::ich_tot)
    const size_t n = slot == MSM_H ? pk.ich_tot() : (size_t)pk.count[slot] + pk.extras[slot];
    const size_t asz = slot == MSM_B2 ? sizeof(G2A) : sizeof(G1A);
    DevBuf big;
    big.ensure(asz * std::max<size_t>(n * PROVE_WIN, 1));
    if (slot == MSM_H) {   // [IC | H]
      const size_t nic = (size_t)pk.count[MSM_IC] + pk.extras[MSM_IC], nh = n - nic;
      if (nic) ZK_HIP(hipMemcpyAsync(big.p, pk.bases[MSM_IC].p, asz * nic, hipMemcpyDeviceToDevice, st));
      if (nh)
        ZK_HIP(hipMemcpyAsync(static_cast<char*>(big.p) + asz * nic, pk.bases[MSM_H].p, asz * nh,
                              hipMemcpyDeviceToDevice, st));
      ZK_HIP(hipStreamSynchronize(st));
      pk.bases[MSM_IC].release();
    } else if (n) {
      ZK_HIP(hipMemcpyAsync(big.p, pk.bases[slot].p, asz * n, hipMemcpyDeviceToDevice, st));
    }
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

static void quotient(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, hipStream_t st, uint64_t* h_out) {
  const uint64_t n = pk->n;
  NttDomain& dom = ctx->domain(pk->log_n);
  ctx->qabc.ensure(sizeof(Fr) * 3 * n);
  Fr* v[3] = {ctx->qabc.as<Fr>(), ctx->qabc.as<Fr>() + n, ctx->qabc.as<Fr>() + 2 * n};
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
                                                v[0], v[1], v[2], ctx->flags.as<uint32_t>());
  ZK_LAUNCH_CHECK();
  pf->end(st, ph);
  // per polynomial: iNTT (coefficients * n, bit-reversed), * n^-1 g^i, NTT
  // (evaluations on the coset g<w>, natural order).  Fused into one tile
  // kernel below 2^LARGE_Q_LOG; from there the three steps run as separate
  // passes, and the final coset iNTT runs in natural order (ntt_natural)
  // instead of a DIF plus an element-wise bit-reversed gather.  Same-box
  // A/B, overlapped prove: 2^24 fused 122.8 / separate 118.6 ms; 2^20 the
  // gather path 9.89 / natural 10.01 ms (profiles/r02_ab_quot.txt).  One
  // launch per pass for all three polynomials (nb = 3) lost 0.2 ms in the
  // overlapped prove (profiles/r03_ab_batchq_fan8_rcw4_rejected.txt).
  // zk_ctx_set_option(ZK_OPT_QUOTIENT_PATH) forces either path (tests).
  constexpr uint32_t LARGE_Q_LOG = 23;
  const bool large = ctx->quot_path >= 0 ? ctx->quot_path == 1 : pk->log_n >= LARGE_Q_LOG;
  for (int k = 0; k < 3; k++) {
    if (!large) {
      ntt_coset_shift(v[k], dom, domain_gpow_br(dom, st), st, pf);
      continue;
    }
    ntt_dif(v[k], dom, /*inverse twiddles*/ true, st, pf);
    ph = pf->begin(st, "quotient_misc", n);
    fr_scale_table(v[k], domain_gpow_br(dom, st), pk->log_n, false, st);
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
  ctx->tmp_scal.ensure(sizeof(uint64_t) * n);
  if (!large) {
    ntt_dif(v[0], dom, true, st, pf);
    ph = pf->begin(st, "quotient_misc", n);
    k_h_final<<<ceil_div(n, 256), 256, 0, st>>>(v[0], domain_gipow(dom, st), pk->log_n, h_out);
    ZK_LAUNCH_CHECK();
    pf->end(st, ph);
    return;
  }
  Fr* h = v[1];
  if (pk->log_n == 0) {   // a size-1 transform is the identity: only the factor
    fr_scale_table(v[0], domain_gipow(dom, st), 0, false, st);
    h = v[0];
  } else {
    ntt_natural(v[1], v[0], v[2], dom, true, st, pf, nullptr, domain_gipow(dom, st), nullptr);
  }
  ph = pf->begin(st, "quotient_misc", n);
  k_h_lo64<<<ceil_div(n, 256), 256, 0, st>>>(h, n, h_out);
  ZK_LAUNCH_CHECK();
  pf->end(st, ph);
}

// A sharded key whose ctx is attached to the matching exchange (an RCCL
// communicator, or a host-staged one) computes its quotient distributed
// (three all-to-alls per proof).
// zk_ctx_set_option(ZK_OPT_DIST_QUOTIENT, 0) turns it off: every rank then
// computes the whole quotient (bench.py's replicated-quotient comparison).
// exchange_matches: such an exchange is attached, whatever the option -- the
// ranks then agree on the mode before every proof (prove_partial_common).
static bool exchange_matches(const zk_ctx* ctx, const zk_pk_dev* pk) {
  return pk->nshards > 1 && ctx->exch && ctx->exch->world == (int)pk->nshards &&
         ctx->exch->rank == (int)pk->shard && dist_quotient_ok(pk->n, (int)pk->nshards);
}
static bool uses_dist_quotient(const zk_ctx* ctx, const zk_pk_dev* pk) {
  return ctx->dist_quotient != 0 && exchange_matches(ctx, pk);
}

// The G1 MSMs run as two pipelines (msm_launch_batch: one sort, accumulate,
// merge and bucket reduction each, so the latency-bound tails cost one tree
// depth per pipeline): A and B1, a batch of two MSMs that need only z, start
// with the witness; IC and H -- both terms of pi_C = IC + H_1 + s pi_A +
// r B_1 (core:224-265), so ONE MSM over the bases [ic_g1 | h_g1] with the
// scalars [lo64(z_i) | lo64(H_i)] -- follows the quotient.  One bucket set
// for IC and H: a bucket reduction fewer per proof than IC in the first batch
// and H alone.
static const int G1_AB[2] = {MSM_A, MSM_B1};

// h_given (virtual-rank tests): this shard's lo64(H_(shard + nshards d)) is
// already on the device, with the witness-check flags of all ranks.
// ranges: only these [lo, hi) entries of d_z are valid (a witness slice),
// else all of [0, V).
// early (the one-GPU prove): pi_A and pi_B in their affine ABI form as soon
// as those MSMs are done, while H is still on the GPU -- each conversion is
// a field inversion (~40 us on one core) that would otherwise follow the
// last MSM.
// z_host (the drop-in host-witness prove): d_z is the ctx's device copy,
// filled here in HOST_PARTS parts (pk_part_cuts) -- and the G2 and A+B1+IC
// MSMs run split the same way: part k's keys, sort and accumulate start as
// soon as its slice of z has landed, while the next slice is still crossing
// PCIe; each later part adds the previous part's completed buckets
// (msm_batch_back ACCUM / COMBINE) and the last one reduces once.
static Partial prove_partial(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, const zk_fr* r,
                             const zk_fr* s, const uint64_t* h_given = nullptr, uint32_t given_flags = 0,
                             const std::vector<uint64_t>* ranges = nullptr, zk_proof* early = nullptr,
                             const zk_fr* z_host = nullptr) {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  const auto t_start = clk::now();
  Range range_prove("zk_prove");
  hipStream_t st = ctx->stream;
  ctx->flags.ensure(16);
  ctx->flags_host.ensure(16);
  ctx->prof.mark_origin(st);
  const int ph_span = ctx->prof.begin(st, "prove_gpu_span", pk->n);   // first kernel .. last MSM done
  ZK_HIP(hipMemsetAsync(ctx->flags.p, 0, 16, st));
  const bool split = z_host != nullptr;
  // part k of a host witness: variables [vcut[k], vcut[k+1]) to the device,
  // every z_i < r, else ZK_ERR_ARG (the host thread waits for a pageable copy)
  auto upload_part = [&](int k) {
    const uint64_t lo = pk->vcut[k], hi = pk->vcut[k + 1];
    if (hi > lo)
      ZK_HIP(hipMemcpyAsync(const_cast<uint64_t*>(d_z) + 4 * lo, z_host + lo, sizeof(zk_fr) * (hi - lo),
                            hipMemcpyHostToDevice, st));
    check_canonical(d_z + 4 * lo, hi - lo, ctx->flags.as<uint32_t>(), st);
  };
  if (split) {
    upload_part(0);
  } else if (ranges) {   // every z_i < r, else ZK_ERR_ARG
    for (size_t k = 0; k + 1 < ranges->size(); k += 2)
      check_canonical(reinterpret_cast<const Fr*>(d_z) + (*ranges)[k], (*ranges)[k + 1] - (*ranges)[k],
                      ctx->flags.as<uint32_t>(), st);
  } else {
    check_canonical(d_z, pk->V, ctx->flags.as<uint32_t>(), st);
  }
  ZK_HIP(hipEventRecord(ctx->ev_scal, st));                     // z (and flags reset) ready
  // Streams (<= GPU_MAX_HW_QUEUES = 4, so no two share a hardware queue):
  // main (high priority) runs the quotient and then the H batch that depends
  // on it; side[0] (high) the G2 MSM, the longest chain; side[1] the A+B1+IC
  // batch.  The latency-bound phases of one MSM overlap the throughput-bound
  // accumulation of another.  Schedule 3 runs everything in order on main.
  const bool serial = ctx->sched == 3;
  hipStream_t s_g2 = serial ? st : ctx->side[0];
  hipStream_t s_abi = serial ? st : ctx->side[1];
  // The quotient: local (every coefficient), distributed over the ranks of
  // a sharded key (this rank's coefficients i = shard mod N), or given
  // (virtual-rank tests).
  const bool dist = !h_given && uses_dist_quotient(ctx, pk);
  const uint64_t* h_src = h_given ? h_given : ctx->tmp_scal.as<uint64_t>();
  const uint32_t h_div = (h_given || dist) ? pk->nshards : 1;
  // scalars of one MSM: lo64 of its variables (or H coefficients), then the
  // extras' scalars (1 for alpha_1 / beta_2 / beta_1, the u64 limbs of r or s)
  // IC's scalars need only z: gathered ahead of the quotient on the A+B1
  // stream (ev_ic), so that the IC+H grouping starts right after the quotient
  bool ic_ready = false;
  // the IC+H scalar vector, sized once before any stream writes it (IC's
  // gather on the A+B1 stream, H's lo64 from the quotient when h_direct)
  const uint32_t nic = pk->count[MSM_IC];
  const bool h_direct = pk->h_ident && !dist && !h_given;
  ctx->scal[MSM_H].ensure(sizeof(uint64_t) * std::max<uint64_t>({(uint64_t)pk->ich_tot(), (uint64_t)nic + pk->n, 1}));
  auto prep_ic = [&](hipStream_t ss) {
    if (nic) {
      k_gather_lo64<<<ceil_div(nic, 256), 256, 0, ss>>>(d_z, 4, pk->idx[MSM_IC].as<uint32_t>(), 1u, nic,
                                                        ctx->scal[MSM_H].as<uint64_t>());
      ZK_LAUNCH_CHECK();
    }
  };
  auto prep_scalars = [&](int slot, hipStream_t ss) {
    const uint32_t cnt = pk->count[slot], nex = pk->extras[slot];
    if (slot == MSM_H) {   // the IC + H MSM: [lo64(z_i) of IC's variables | lo64(H_i)]
      if (!ic_ready) prep_ic(ss);
      if (cnt && !h_direct) {
        k_gather_lo64<<<ceil_div(cnt, 256), 256, 0, ss>>>(h_src, 1, pk->idx[MSM_H].as<uint32_t>(), h_div, cnt,
                                                          ctx->scal[MSM_H].as<uint64_t>() + nic);
        ZK_LAUNCH_CHECK();
      }
      return;
    }
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
  // split parts: scalars of compacted positions [lo, hi) (+ the extras with
  // the second part), and the segment of positions [lo, hi_with_extras)
  auto prep_range = [&](int slot, uint32_t lo, uint32_t hi, bool extras, hipStream_t ss) {
    const uint32_t cnt = pk->count[slot], nex = pk->extras[slot];
    ctx->scal[slot].ensure(sizeof(uint64_t) * std::max<uint32_t>(cnt + nex, 1));
    if (hi > lo) {
      k_gather_lo64<<<ceil_div(hi - lo, 256), 256, 0, ss>>>(d_z, 4, pk->idx[slot].as<uint32_t>() + lo, 1u, hi - lo,
                                                           ctx->scal[slot].as<uint64_t>() + lo);
      ZK_LAUNCH_CHECK();
    }
    if (extras && nex) {
      Extras ex{};
      ex.v[0] = 1;
      const zk_fr* full = slot == MSM_A ? r : slot == MSM_B2 ? s : nullptr;
      if (full) for (int k = 0; k < 4; k++) ex.v[1 + k] = full->l[k];
      k_set_extras<<<1, 64, 0, ss>>>(ctx->scal[slot].as<uint64_t>() + cnt, ex, nex);
      ZK_LAUNCH_CHECK();
    }
  };
  auto seg_range = [&](int slot, uint32_t lo, uint32_t hi) {
    MsmSeg sg{pk->bases[slot].p, ctx->scal[slot].as<uint64_t>() + lo, hi - lo, pk->stride[slot]};
    sg.wstride = pk->count[slot] + pk->extras[slot];
    sg.ioff = lo;
    return sg;
  };
  // part k: compacted positions [pcut[k], pcut[k+1]) of every slot, the
  // extras with the last part.  Part 0 completes its buckets (FIXUP), every
  // later part adds the previous part's (ACCUM), and the last one reduces
  // (COMBINE).
  auto launch_part = [&](int part, hipStream_t gs2, hipStream_t gsa) {
    const bool last = part == HOST_PARTS - 1;
    const int mode = part == 0 ? MSM_BACK_FIXUP : last ? MSM_BACK_COMBINE : MSM_BACK_ACCUM;
    {
      Range range("msm_g2_part");
      const uint32_t lo = pk->pcut[part][MSM_B2], hi = pk->pcut[part + 1][MSM_B2];
      MsmWork& w = last ? ctx->msm[MSM_B2] : ctx->part_g2[part];
      w.tag = serial ? (last ? "B2/" : "B2p/") : "";
      prep_range(MSM_B2, lo, hi, last, gs2);
      const MsmSeg sg = seg_range(MSM_B2, lo, last ? hi + pk->extras[MSM_B2] : hi);
      msm_batch_front<G2>(w, &sg, 1, 64, pk->win_c, gs2);
      msm_batch_back<G2>(w, gs2, mode, part ? &ctx->part_g2[part - 1] : nullptr);
      if (last) {
        msm_download<G2>(w, gs2);
        ZK_HIP(hipEventRecord(ctx->ev_done[MSM_B2], gs2));
      }
    }
    {
      Range range("msm_g1_a_b1_part");
      MsmSeg segs[2];
      for (int i = 0; i < 2; i++) {
        const int sl = G1_AB[i];
        const uint32_t lo = pk->pcut[part][sl], hi = pk->pcut[part + 1][sl];
        prep_range(sl, lo, hi, last, gsa);
        segs[i] = seg_range(sl, lo, last ? hi + pk->extras[sl] : hi);
      }
      MsmWork& w = last ? ctx->msm[MSM_A] : ctx->part_abi[part];
      w.tag = serial ? (last ? "AB/" : "ABp/") : "";
      msm_batch_front<G1>(w, segs, 2, 64, pk->win_c, gsa);
      msm_batch_back<G1>(w, gsa, mode, part ? &ctx->part_abi[part - 1] : nullptr);
      if (last) {
        msm_download<G1>(w, gsa);
        ZK_HIP(hipEventRecord(ctx->ev_done[MSM_A], gsa));
      }
    }
  };
  static const char* const tags[NUM_MSM] = {"A/", "B2/", "B1/", "IC/", "H/"};
  auto launch_batch = [&](const int* slots, int k, const char* tag, hipStream_t gs) {
    Range range(k == 1 ? "msm_g1_ic_h" : "msm_g1_a_b1");
    MsmSeg segs[MSM_MAXSEG];
    for (int i = 0; i < k; i++) {
      prep_scalars(slots[i], gs);
      const uint32_t np = slots[i] == MSM_H ? pk->ich_tot() : pk->count[slots[i]] + pk->extras[slots[i]];
      segs[i] = MsmSeg{pk->bases[slots[i]].p, ctx->scal[slots[i]].as<uint64_t>(), np, pk->stride[slots[i]]};
    }
    MsmWork& w = ctx->msm[slots[0]];
    w.tag = serial ? tag : "";
    msm_launch_batch<G1>(w, segs, k, 64, pk->win_c, gs);
    msm_download<G1>(w, gs);
    ZK_HIP(hipEventRecord(ctx->ev_done[slots[0]], gs));
  };
  // G2 (pi_B), then A + B1 + IC, both starting with the witness
  auto launch_msms = [&]() {
    if (!serial) ZK_HIP(hipStreamWaitEvent(s_g2, ctx->ev_scal, 0));
    {
      Range range("msm_g2");
      MsmWork& w = ctx->msm[MSM_B2];
      w.tag = serial ? tags[MSM_B2] : "";
      prep_scalars(MSM_B2, s_g2);
      msm_launch_shared<G2>(w, pk->bases[MSM_B2].as<G2A>(), ctx->scal[MSM_B2].as<uint64_t>(), 1,
                            pk->count[MSM_B2] + pk->extras[MSM_B2], 64, pk->win_c, s_g2, pk->stride[MSM_B2]);
      msm_download<G2>(w, s_g2);
      ZK_HIP(hipEventRecord(ctx->ev_done[MSM_B2], s_g2));
    }
    if (!serial) ZK_HIP(hipStreamWaitEvent(s_abi, ctx->ev_scal, 0));
    if (!serial) {
      prep_ic(s_abi);
      ZK_HIP(hipEventRecord(ctx->ev_ic, s_abi));
      ic_ready = true;
    }
    launch_batch(G1_AB, 2, "AB/", s_abi);
  };
  // the quotient, then H on the main stream
  auto run_quotient = [&]() {
    if (h_given) return;
    Range range(dist ? "quotient_distributed" : "quotient");
    if (dist) {
      ctx->tmp_scal.ensure(sizeof(uint64_t) * (pk->n / pk->nshards));
      h_src = ctx->tmp_scal.as<uint64_t>();
      dist_quotient(ctx, pk, d_z, *ctx->exch, ctx->dq, ctx->flags.as<uint32_t>(), ctx->tmp_scal.as<uint64_t>(), st);
    } else {
      // (Az, Bz, Cz) -> lo64(H): in place in the IC+H scalars, else in
      // tmp_scal (sized here, before its pointer is taken)
      ctx->tmp_scal.ensure(sizeof(uint64_t) * pk->n);
      quotient(ctx, pk, d_z, st, h_direct ? ctx->scal[MSM_H].as<uint64_t>() + nic : ctx->tmp_scal.as<uint64_t>());
      h_src = ctx->tmp_scal.as<uint64_t>();
    }
  };
  // MSMs first, then the quotient (enqueueing the quotient first measured
  // 0.37 ms slower: profiles/r03_ab_quotient_first_rejected.txt).  With
  // ZK_OPT_EXCHANGE_FIRST a distributed quotient goes first and the side
  // streams wait for it, so its all-to-alls find free CUs on every rank.
  // (Split uploads are single-GPU only: the quotient needs all of z.)
  const bool xfirst = dist && ctx->exchange_first == 1 && !serial && !split;
  if (xfirst) {
    run_quotient();
    ZK_HIP(hipEventRecord(ctx->ev_quot, st));
    ZK_HIP(hipStreamWaitEvent(s_g2, ctx->ev_quot, 0));
    ZK_HIP(hipStreamWaitEvent(s_abi, ctx->ev_quot, 0));
  }
  if (split) {
    // part k's MSMs, then part k+1 of z (the host thread waits for the
    // pageable copy while the GPU runs the parts already there)
    for (int k = 0; k < HOST_PARTS; k++) {
      if (k) {
        upload_part(k);
        ZK_HIP(hipEventRecord(ctx->ev_scal, st));
      }
      if (!serial) {
        ZK_HIP(hipStreamWaitEvent(s_g2, ctx->ev_scal, 0));
        ZK_HIP(hipStreamWaitEvent(s_abi, ctx->ev_scal, 0));
        if (k == HOST_PARTS - 1) {   // all of z is here: IC's scalars off the critical path too
          prep_ic(s_abi);
          ZK_HIP(hipEventRecord(ctx->ev_ic, s_abi));
          ic_ready = true;
        }
      }
      launch_part(k, s_g2, s_abi);
    }
  } else {
    launch_msms();
  }
  if (!xfirst) run_quotient();
  // the exchange watchdog below counts from here: a host-staged exchange has
  // finished its all-to-alls inside run_quotient, and only local GPU work
  // (RCCL: the enqueued collectives) is left
  const auto t_quot = clk::now();
  // A distributed proof's witness checks are spread over the ranks (each
  // checks its slice and its quotient rows): every rank takes the max of the
  // flag words, so all return the status combine() would give -- flags are
  // ORs of 8 (z_i >= r), 4 / 3 (InvalidWitness) and 2 (division), and the
  // max keeps that precedence.  RCCL: on the stream, no host round trip.
  const bool flags_agreed = dist && ctx->exch->agree_max_dev(ctx->flags.as<uint32_t>(), st);
  ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
  {
    const int h_slot[1] = {MSM_H};
    if (ic_ready) ZK_HIP(hipStreamWaitEvent(st, ctx->ev_ic, 0));
    launch_batch(h_slot, 1, "ICH/", st);
  }
  const int waits[3] = {MSM_B2, MSM_A, MSM_H};   // MSM_A: the A+B1 batch, MSM_H: IC + H
  if (ph_span >= 0) {
    for (int sl : waits) ZK_HIP(hipStreamWaitEvent(st, ctx->ev_done[sl], 0));
    ctx->prof.end(st, ph_span);
  }

  // Host tails (Horner over each MSM's partials, then s A + r B1) run as
  // each MSM's stream reaches its event, overlapping the MSMs still on the
  // GPU.
  ctx->prof.add_host("host_launch", ms_since(t_start));
  Range range_tail("host_tail");
  double t_fin = 0;
  Partial p{};
  bool done[3] = {false, false, false};
  bool sc_done = false, ab_done = false;
  for (int left = 3; left > 0;) {
    // the H MSM waits for the peers' quotient stages: a dead peer must end
    // this proof (ZK_ERR_RCCL, the exchange aborted) instead of hanging it
    if (dist && (ctx->exch->async_error() || ms_since(t_quot) > ctx->exch->timeout_ms))
      throw Error(ZK_ERR_RCCL, "distributed quotient: a peer did not answer within the exchange timeout");
    bool progressed = false;
    for (int wi = 0; wi < 3; wi++) {
      if (done[wi]) continue;
      const int slot = waits[wi];
      const hipError_t q = hipEventQuery(ctx->ev_done[slot]);
      if (q == hipErrorNotReady) continue;
      ZK_HIP(q);
      const auto t_f = clk::now();
      if (slot == MSM_B2) {
        p.B2 = msm_finish<G2>(ctx->msm[slot]);
        if (early) host_to_abi<G2>(p.B2, reinterpret_cast<uint64_t*>(&early->b));
      } else if (slot == MSM_A) {
        p.A = msm_finish_seg<G1>(ctx->msm[slot], 0);
        p.B1 = msm_finish_seg<G1>(ctx->msm[slot], 1);
        ab_done = true;
      } else {
        p.IC = msm_finish_seg<G1>(ctx->msm[slot], 0);   // IC + H_1
        p.H = host::inf<host::Fq>();
      }
      done[wi] = progressed = true;
      left--;
      if (!sc_done && ab_done) {
        p.SC = host::mul2_scalar(p.A, s->l, p.B1, r->l);
        if (early) host_to_abi<G1>(p.A, reinterpret_cast<uint64_t*>(&early->a));
        sc_done = true;
      }
      t_fin += ms_since(t_f);
      if (left == 0) ctx->prof.add_host("host_tail_after_last", ms_since(t_f));
    }
    if (!progressed) std::this_thread::yield();
  }
  for (int k = 0; k < NUM_SIDE; k++) ZK_HIP(hipStreamSynchronize(ctx->side[k]));
  ZK_HIP(hipStreamSynchronize(st));
  ctx->prof.add_host("host_finish", t_fin);
  // host wall time of the whole call up to here, against prove_gpu_span
  ctx->prof.add_host("host_prove_total", ms_since(t_start));
  ctx->prof.collect();
  uint32_t flags = h_given ? given_flags : *ctx->flags_host.as<uint32_t>();
  if (dist && !flags_agreed) flags = (uint32_t)ctx->exch->agree_max((int)flags, st);
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
               const zk_fr* r, const zk_fr* s, zk_proof* out, const zk_fr* z_host) {
  // Witness::new (core:81-99) and the length check of validate (core:113-118)
  if (!fr_canonical(*r) || !fr_canonical(*s)) return ZK_ERR_ARG;   // Fr::rand draws are reduced
  if (num_public >= zlen) return ZK_ERR_INVALID_WITNESS;
  if (zlen != pk->V) return ZK_ERR_INVALID_WITNESS;
  if (pk->nshards != 1) return ZK_ERR_ARG;
  zk_proof ab{};
  Partial p = prove_partial(ctx, pk, reinterpret_cast<const uint64_t*>(d_z), r, s, nullptr, 0, nullptr, &ab, z_host);
  if (p.status != ZK_OK) return p.status;
  // combine() for one part: pi_A, pi_B already converted; pi_C = IC + H + s A + r B1
  out->a = ab.a;
  out->b = ab.b;
  host_to_abi<G1>(host::addp(host::addp(p.IC, p.H), p.SC), reinterpret_cast<uint64_t*>(&out->c));
  return ZK_OK;
}

// z_host / ranges: a host witness slice (zk_groth16_prove_partial_host) to
// upload first, after the ranks agreed, instead of the device witness d_z.
// bad_slice: the host slice does not match the ranges (ZK_ERR_ARG) -- with a
// distributed quotient it goes into the status agreement like every other
// input error, so the peers return with this rank instead of waiting in the
// first all-to-all.
static int prove_partial_common(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, const zk_fr* z_host,
                                const std::vector<uint64_t>* ranges, size_t zlen, size_t num_public,
                                const zk_fr* r, const zk_fr* s, zk_prove_partial* out, bool bad_slice = false) {
  std::memset(out, 0, sizeof *out);
  Partial p{};
  int local = ZK_OK;
  if (bad_slice || !fr_canonical(*r) || !fr_canonical(*s)) local = ZK_ERR_ARG;
  else if (num_public >= zlen || zlen != pk->V) local = ZK_ERR_INVALID_WITNESS;
  const bool attached = exchange_matches(ctx, pk);
  const bool dist = uses_dist_quotient(ctx, pk);
  if (attached && ctx->exch->broken) {
    ctx->err = "the exchange was aborted by an earlier failed proof; attach a new one (or detach it)";
    return ZK_ERR_RCCL;
  }
  hipStream_t st = ctx->stream;
  auto upload = [&]() {
    if (!z_host) return;
    ctx->z_canon.ensure(sizeof(zk_fr) * std::max<size_t>(pk->V, 1));
    size_t off = 0;
    for (size_t k = 0; k + 1 < ranges->size(); k += 2) {
      const uint64_t lo = (*ranges)[k], len = (*ranges)[k + 1] - lo;
      ZK_HIP(hipMemcpyAsync(static_cast<zk_fr*>(ctx->z_canon.p) + lo, z_host + off, sizeof(zk_fr) * len,
                            hipMemcpyHostToDevice, st));
      off += len;
    }
    d_z = ctx->z_canon.p;
  };
  if (!attached) {
    if (local == ZK_OK) {
      upload();
      p = prove_partial(ctx, pk, reinterpret_cast<const uint64_t*>(d_z), r, s, nullptr, 0, ranges);
    } else {
      p.status = local;
    }
    std::memcpy(out->bytes, &p, sizeof p);
    return p.status;
  }
  // An exchange of the key's shape is attached.  Every allocation a
  // distributed quotient needs is made first, then the ranks agree on the
  // host-side checks and on the quotient mode before the first all-to-all (a
  // rank that bailed out alone, or one set to ZK_OPT_DIST_QUOTIENT 0 while
  // its peers are not, would leave them blocked in the collective): one
  // all-reduce of {any rank distributed, 2 status + any rank replicated}.
  // A failure after the agreement -- a transport error, a device error, a
  // peer that stopped answering -- aborts the exchange, so the peers'
  // pending transfers fail too, and marks it dead.  A replicated proof after
  // the agreement uses no exchange: its failures leave the exchange alone.
  bool in_exchange = true;
  try {
    if (local == ZK_OK && dist) {
      try {
        dq_prepare(ctx, pk, (int)pk->nshards, ctx->dq, st);
        ctx->tmp_scal.ensure(sizeof(uint64_t) * (pk->n / pk->nshards));
        if (z_host) ctx->z_canon.ensure(sizeof(zk_fr) * std::max<size_t>(pk->V, 1));
      } catch (const Error& e) {
        local = e.code;
        ctx->err = e.what();
      }
    }
    int32_t v[2] = {dist ? 1 : 0, local * 2 + (dist ? 0 : 1)};
    ctx->exch->agree_max2(v, st);
    if (local == ZK_OK) local = v[1] >> 1;
    if (local == ZK_OK && v[0] == 1 && (v[1] & 1)) {
      local = ZK_ERR_ARG;
      ctx->err = "ranks disagree on ZK_OPT_DIST_QUOTIENT: set it identically on every rank";
    }
    if (local != ZK_OK) {
      p.status = local;
    } else {
      in_exchange = dist;
      upload();
      p = prove_partial(ctx, pk, reinterpret_cast<const uint64_t*>(d_z), r, s, nullptr, 0, ranges);
    }
  } catch (...) {
    if (in_exchange) {
      ctx->exch->broken = true;
      ctx->exch->abort();
    }
    throw;
  }
  std::memcpy(out->bytes, &p, sizeof p);
  return p.status;
}

int prove_partial_impl(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, size_t zlen, size_t num_public,
                       const zk_fr* r, const zk_fr* s, zk_prove_partial* out) {
  return prove_partial_common(ctx, pk, d_z, nullptr, nullptr, zlen, num_public, r, s, out);
}

// The ranges a shard reads on this ctx: wr_dist with a distributed quotient,
// else the whole witness.
std::vector<uint64_t> witness_ranges(const zk_ctx* ctx, const zk_pk_dev* pk) {
  if (uses_dist_quotient(ctx, pk)) return pk->wr_dist;
  return {0, pk->V};
}

int prove_partial_host_impl(zk_ctx* ctx, const zk_pk_dev* pk, const zk_fr* z_slice, size_t slice_len, size_t zlen,
                            size_t num_public, const zk_fr* r, const zk_fr* s, zk_prove_partial* out) {
  const std::vector<uint64_t> ranges = witness_ranges(ctx, pk);
  size_t want = 0;
  for (size_t k = 0; k + 1 < ranges.size(); k += 2) want += ranges[k + 1] - ranges[k];
  const bool bad = slice_len != want || (want && !z_slice);
  if (bad)
    ctx->err = "witness slice length " + std::to_string(slice_len) + " != " + std::to_string(want) +
               " (zk_groth16_witness_ranges)";
  return prove_partial_common(ctx, pk, nullptr, z_slice, &ranges, zlen, num_public, r, s, out, bad);
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
