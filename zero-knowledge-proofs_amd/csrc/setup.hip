// setup.hip -- CRS::generate_from_qap (crates/groth16-setup/src/lib.rs:141-268)
// on the GPU, with the reference's exact scalar semantics:
//   a~,b~,g~,d~,t~ = lo64(alpha..tau)                         setup:155-159
//   alpha_1 .. delta_2 = generator * FULL param               setup:166-171
//   A_i(t~), B_i(t~), C_i(t~)                                 setup:174-182
//   a_g1[i] = G1 lo64(A_i), b_g1/b_g2[i] = G lo64(B_i)        setup:185-207
//   pk ic[i-l-1] = G1 lo64((b~A_i + a~B_i + C_i)/d~), i > l    setup:210-218
//   vk ic[i]     = G1 lo64((b~A_i + a~B_i + C_i)/g~), i <= l   setup:221-229
//   h[i] = G1 lo64(t~^i / d~), i < qap.degree() = n           setup:232-241
// A_i(t) is evaluated from the sparse matrices as sum_j M[j][i] L_j(t) with
// the Lagrange basis of the size-n domain -- the same value as evaluating the
// interpolated polynomial of qap:143-170, without materialising it.
// The per-point work (64-bit fixed-base multiplications on 8-bit window
// tables, batch affine normalisation) is data-parallel on the GPU; the six
// full-width generator multiples are a few hundred sequential group ops and
// run on the host (host_ec.hpp).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "ctx.hpp"
#include "quotient.hpp"

namespace zk {

zk_pk_dev* pk_upload(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* q, uint32_t shard, uint32_t nshards);
void csr_upload(CsrDev& d, const zk_r1cs_csr* q, hipStream_t st);

// ---------------------------------------------------- fixed-base tables ---
// T[w][d] = d * 2^(8w) * G, w < 8, d < 256 (affine, Montgomery); T[w][0] unused.
template <class C>
struct FbTable {
  std::vector<typename C::A> host;
  DevBuf dev;
};

static host::X<host::Fq> g1_gen_host() {
  host::X<host::Fq> p;
  std::memcpy(p.X_.l, G1_GEN_HOSTM, 48);
  std::memcpy(p.Y.l, G1_GEN_HOSTM + 12, 48);
  p.ZZ = host::one();
  p.ZZZ = host::one();
  return p;
}
static host::X<host::Fq2> g2_gen_host() {
  host::X<host::Fq2> p;
  std::memcpy(p.X_.c0.l, G2_GEN_HOSTM, 48);
  std::memcpy(p.X_.c1.l, G2_GEN_HOSTM + 12, 48);
  std::memcpy(p.Y.c0.l, G2_GEN_HOSTM + 24, 48);
  std::memcpy(p.Y.c1.l, G2_GEN_HOSTM + 36, 48);
  p.ZZ = host::f_one<host::Fq2>();
  p.ZZZ = host::f_one<host::Fq2>();
  return p;
}

template <class HF, class DA>
static void build_table(const host::X<HF>& G, std::vector<DA>& out) {
  using HX = host::X<HF>;
  std::vector<HX> pts(2048);
  HX base = G;
  for (int w = 0; w < 8; w++) {
    pts[w * 256] = host::inf<HF>();
    for (int d = 1; d < 256; d++) pts[w * 256 + d] = host::addp(pts[w * 256 + d - 1], base);
    for (int k = 0; k < 8; k++) base = host::dbl(base);
  }
  out.resize(2048);
  for (int i = 0; i < 2048; i++) {
    HF x, y;
    if (!host::to_affine(pts[i], x, y)) { x = host::f_zero<HF>(); y = host::f_zero<HF>(); }
    x = host::to_dev(x);   // device Montgomery radix (constants.hpp)
    y = host::to_dev(y);
    static_assert(sizeof(HF) * 2 == sizeof(DA), "layout");
    std::memcpy(&out[i], &x, sizeof(HF));
    std::memcpy(reinterpret_cast<char*>(&out[i]) + sizeof(HF), &y, sizeof(HF));
  }
}

// ------------------------------------------------------------- kernels ---
// Lagrange basis at t over the size-n domain, per-thread batch inversion:
// L_j = w^j (t^n - 1) / (n (t - w^j)); k = (t^n - 1)/n precomputed.
constexpr int LAG_CHUNK = 32;
__global__ void __launch_bounds__(256) k_lagrange(const Fr* __restrict__ wpow, Fr t, Fr k, size_t n,
                                                  Fr* __restrict__ L) {
  const size_t c0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * LAG_CHUNK;
  if (c0 >= n) return;
  const size_t c1 = min(c0 + LAG_CHUNK, n);
  Fr run = fp_one<FrParams>();
  for (size_t j = c0; j < c1; j++) {               // L[j] <- prefix product
    st_vec(&L[j], run);
    run = fp_mul(run, fp_sub(t, ld_vec(&wpow[j])));
  }
  // Fermat inverse of the chunk product
  uint32_t e[8];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = __builtin_subc(FrParams::MOD[i], i == 0 ? 2u : 0u, br, &br);
  Fr inv = fp_one<FrParams>();
#pragma unroll
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      inv = fp_mul(inv, inv);
      if ((e[i] >> b) & 1) inv = fp_mul(inv, run);
    }
  for (size_t j = c1; j-- > c0;) {
    const Fr wj = ld_vec(&wpow[j]);
    const Fr d = fp_sub(t, wj);
    const Fr dinv = fp_mul(inv, ld_vec(&L[j]));
    inv = fp_mul(inv, d);
    st_vec(&L[j], fp_mul(fp_mul(dinv, wj), k));
  }
}
// t is a domain point (t^n = 1): L_j = [w^j == t]
__global__ void __launch_bounds__(256) k_lagrange_point(const Fr* __restrict__ wpow, Fr t, size_t n,
                                                        Fr* __restrict__ L) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  st_vec(&L[j], fp_eq(ld_vec(&wpow[j]), t) ? fp_one<FrParams>() : fp_zero<FrParams>());
}

// Column sums over CSC: out[i] = sum_k val_k L[row_k] (cols >= V dropped by construction)
__global__ void __launch_bounds__(256) k_colsum(const uint64_t* __restrict__ cp, const uint32_t* __restrict__ row,
                                                const Fr* __restrict__ val, const Fr* __restrict__ L, uint64_t V,
                                                Fr* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V) return;
  Fr acc = fp_zero<FrParams>();
  for (uint64_t k = cp[i]; k < cp[i + 1]; k++) {
    Fr x = ld_vec(&L[row[k]]);
    if (val) x = fp_mul(x, ld_vec(&val[k]));
    acc = fp_add(acc, x);
  }
  st_vec(&out[i], acc);
}

__device__ __forceinline__ uint64_t lo64_of(const Fr& m) {
  Fr c = fp_from_mont(m);
  return (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
}

struct SetupConsts {
  Fr al, be, dinv, ginv;  // Montgomery: a~, b~, d~^-1, g~^-1
  uint64_t V, num_public;
};
// per variable i: lo64 scalars for a_g1, b_g1 (= b_g2), pk ic (i > l) / vk ic (i <= l)
__global__ void __launch_bounds__(256) k_setup_scalars(const Fr* __restrict__ av, const Fr* __restrict__ bv,
                                                       const Fr* __restrict__ cv, SetupConsts k,
                                                       uint64_t* __restrict__ sa, uint64_t* __restrict__ sb,
                                                       uint64_t* __restrict__ sic, uint64_t* __restrict__ svk) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k.V) return;
  const Fr a = ld_vec(&av[i]), b = ld_vec(&bv[i]), c = ld_vec(&cv[i]);
  sa[i] = lo64_of(a);
  sb[i] = lo64_of(b);
  const Fr t = fp_add(fp_add(fp_mul(k.be, a), fp_mul(k.al, b)), c);
  if (i > k.num_public) sic[i - k.num_public - 1] = lo64_of(fp_mul(t, k.dinv));
  else svk[i] = lo64_of(fp_mul(t, k.ginv));
}
__global__ void __launch_bounds__(256) k_lo64(const Fr* __restrict__ in, size_t n, uint64_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = lo64_of(ld_vec(&in[i]));
}

// XYZZ = sum_w T[w][byte_w(k)]  (<= 8 mixed additions), k = scal[idx ? idx[i] : i]
template <class C>
__global__ void __launch_bounds__(128) k_fixed_base(const typename C::A* __restrict__ T,
                                                    const uint64_t* __restrict__ scal,
                                                    const uint32_t* __restrict__ idx, size_t n,
                                                    typename C::X* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = scal[idx ? idx[i] : i];
  typename C::X acc;
  xyzz_set_inf(acc);
  for (int w = 0; w < 8; w++) {
    const uint32_t d = (uint32_t)(k >> (8 * w)) & 255u;
    if (d) acc = xyzz_madd(acc, ld_vec(&T[w * 256 + d]));
  }
  st_vec(&out[i], acc);
}

// device affine (Montgomery, (0,0) = infinity) -> canonical ABI words
__device__ __forceinline__ void st_canon(uint64_t* w, const Fq& m) {
  Fq c = fp_from_mont(m);
#pragma unroll
  for (int i = 0; i < 6; i++) w[i] = (uint64_t)c.v[2 * i] | ((uint64_t)c.v[2 * i + 1] << 32);
}
__global__ void __launch_bounds__(256) k_to_abi_g1(const G1A* __restrict__ in, size_t n, uint64_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1A a = ld_vec(&in[i]);
  uint64_t* w = out + i * 13;
  if (aff_is_inf(a)) {
    for (int k = 0; k < 12; k++) w[k] = 0;
    w[12] = 1;
    return;
  }
  st_canon(w, a.x);
  st_canon(w + 6, a.y);
  w[12] = 0;
}
__global__ void __launch_bounds__(256) k_to_abi_g2(const G2A* __restrict__ in, size_t n, uint64_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G2A a = ld_vec(&in[i]);
  uint64_t* w = out + i * 25;
  if (aff_is_inf(a)) {
    for (int k = 0; k < 24; k++) w[k] = 0;
    w[24] = 1;
    return;
  }
  st_canon(w, a.x.c0);
  st_canon(w + 6, a.x.c1);
  st_canon(w + 12, a.y.c0);
  st_canon(w + 18, a.y.c1);
  w[24] = 0;
}

// ------------------------------------------------------------- helpers ---
template <class C>
static FbTable<C>& fb_table(int device, hipStream_t st);

static std::mutex g_tab_mu;
template <>
FbTable<G1>& fb_table<G1>(int device, hipStream_t st) {
  static std::map<int, FbTable<G1>> tabs;
  std::lock_guard<std::mutex> lk(g_tab_mu);
  FbTable<G1>& t = tabs[device];
  if (t.host.empty()) {
    build_table(g1_gen_host(), t.host);
    t.dev.ensure(sizeof(G1A) * 2048);
    ZK_HIP(hipMemcpyAsync(t.dev.p, t.host.data(), sizeof(G1A) * 2048, hipMemcpyHostToDevice, st));
    ZK_HIP(hipStreamSynchronize(st));
  }
  return t;
}
template <>
FbTable<G2>& fb_table<G2>(int device, hipStream_t st) {
  static std::map<int, FbTable<G2>> tabs;
  std::lock_guard<std::mutex> lk(g_tab_mu);
  FbTable<G2>& t = tabs[device];
  if (t.host.empty()) {
    build_table(g2_gen_host(), t.host);
    t.dev.ensure(sizeof(G2A) * 2048);
    ZK_HIP(hipMemcpyAsync(t.dev.p, t.host.data(), sizeof(G2A) * 2048, hipMemcpyHostToDevice, st));
    ZK_HIP(hipStreamSynchronize(st));
  }
  return t;
}

// out[i] = G * scal[idx ? idx[i] : i], affine Montgomery
template <class C>
static void fixed_base(zk_ctx* ctx, const uint64_t* d_scal, const uint32_t* d_idx, size_t n,
                       typename C::A* d_out, hipStream_t st) {
  if (!n) return;
  FbTable<C>& T = fb_table<C>(ctx->device, st);
  DevBuf xs, pre;
  xs.ensure(sizeof(typename C::X) * n);
  pre.ensure(sizeof(typename C::F) * n);
  k_fixed_base<C><<<ceil_div(n, 128), 128, 0, st>>>(T.dev.template as<typename C::A>(), d_scal, d_idx, n,
                                                     xs.template as<typename C::X>());
  ZK_LAUNCH_CHECK();
  batch_normalize<C>(xs.template as<typename C::X>(), n, pre.template as<typename C::F>(), d_out, st);
  ZK_HIP(hipStreamSynchronize(st));  // xs / pre die here
}

template <class C>
static void to_abi(const typename C::A* d_in, size_t n, void* host_out, hipStream_t st) {
  if (!n) return;
  DevBuf w;
  w.ensure(sizeof(uint64_t) * C::ABI_WORDS * n);
  if (C::ABI_WORDS == 13)
    k_to_abi_g1<<<ceil_div(n, 256), 256, 0, st>>>(reinterpret_cast<const G1A*>(d_in), n, w.as<uint64_t>());
  else
    k_to_abi_g2<<<ceil_div(n, 256), 256, 0, st>>>(reinterpret_cast<const G2A*>(d_in), n, w.as<uint64_t>());
  ZK_LAUNCH_CHECK();
  ZK_HIP(hipMemcpyAsync(host_out, w.p, sizeof(uint64_t) * C::ABI_WORDS * n, hipMemcpyDeviceToHost, st));
  ZK_HIP(hipStreamSynchronize(st));
}

// n device affine points (Montgomery) `stride` bytes apart (0 = packed) ->
// canonical ABI words in host memory (the test library's key readback)
void bases_to_abi_host(bool g2, const void* d_in, uint32_t stride, size_t n, uint64_t* host_out, hipStream_t st) {
  if (!n) return;
  const size_t asz = g2 ? sizeof(G2A) : sizeof(G1A);
  DevBuf packed;
  const void* src = d_in;
  if (stride && stride != asz) {
    packed.ensure(asz * n);
    ZK_HIP(hipMemcpy2DAsync(packed.p, asz, d_in, stride, asz, n, hipMemcpyDeviceToDevice, st));
    src = packed.p;
  }
  if (g2) to_abi<G2>(static_cast<const G2A*>(src), n, host_out, st);
  else to_abi<G1>(static_cast<const G1A*>(src), n, host_out, st);
}

// host-side generator multiple by a full-width canonical scalar -> ABI
template <class C, class HX>
static void gen_mul_abi(const HX& G, const zk_fr& k, void* out) {
  host_to_abi<C>(host::mul_scalar(G, k.l), reinterpret_cast<uint64_t*>(out));
}

static bool fr_canon_zero(const zk_fr& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }

// CSR (rows) -> CSC (columns < V) for one matrix
static void csr_to_csc(uint64_t nc, uint64_t V, const uint64_t* rp, const uint32_t* col, const zk_fr* val,
                       std::vector<uint64_t>& cp, std::vector<uint32_t>& row, std::vector<zk_fr>& cval) {
  cp.assign(V + 1, 0);
  const uint64_t nnz = nc ? rp[nc] : 0;
  for (uint64_t k = 0; k < nnz; k++)
    if (col[k] < V) cp[col[k] + 1]++;
  for (uint64_t i = 0; i < V; i++) cp[i + 1] += cp[i];
  row.resize(std::max<uint64_t>(cp[V], 1));
  if (val) cval.resize(std::max<uint64_t>(cp[V], 1));
  std::vector<uint64_t> cur(cp.begin(), cp.end() - 1);
  for (uint64_t j = 0; j < nc; j++)
    for (uint64_t k = rp[j]; k < rp[j + 1]; k++) {
      if (col[k] >= V) continue;
      const uint64_t p = cur[col[k]]++;
      row[p] = (uint32_t)j;
      if (val) cval[p] = val[k];
    }
}

// ---------------------------------------------------------------- setup ---
int setup_impl(zk_ctx* ctx, const zk_r1cs_csr* q, const zk_setup_params* P, uint64_t num_public, uint32_t shard,
               uint32_t nshards, zk_pk* pk_host, zk_pk_dev** pk_dev, zk_vk* vk) {
  Range range("zk_setup");
  hipStream_t st = ctx->stream;
  const uint64_t V = q->num_variables, nc = q->num_constraints;
  // SetupParams::validate (setup:128-136) and num_public < V (setup:148-152)
  if (fr_canon_zero(P->alpha) || fr_canon_zero(P->beta) || fr_canon_zero(P->gamma) || fr_canon_zero(P->delta))
    return ZK_ERR_SETUP_PARAMS;
  if (num_public >= V) return ZK_ERR_SETUP_PARAMS;
  // truncated copies (setup:155-159); the reference unwraps inverse(d~), inverse(g~)
  const uint64_t al = P->alpha.l[0], be = P->beta.l[0], ga = P->gamma.l[0], de = P->delta.l[0], ta = P->tau.l[0];
  if (de == 0 || ga == 0) return ZK_ERR_SETUP_PARAMS;
  if (nc > (1ull << 32)) return ZK_ERR_DOMAIN;
  uint64_t n = 1;
  while (n < nc) n <<= 1;
  const uint32_t log_n = (uint32_t)__builtin_ctzll(n);
  if (log_n > 32) return ZK_ERR_DOMAIN;
  if (V >= 0x80000000ull || n >= 0x80000000ull) return ZK_ERR_ARG;

  auto to_dev = [](const host::Fr& h) { Fr d; const host::Fr v = host::fr_to_dev(h); std::memcpy(d.v, v.l, 32); return d; };
  const host::Fr t = host::fr_from_u64(ta);
  host::Fr tn = t;
  for (uint32_t i = 0; i < log_n; i++) tn = host::fr_mul(tn, tn);
  const host::Fr zt = host::fr_sub(tn, host::fr_one());
  const host::Fr kk = host::fr_mul(zt, host::fr_inv(host::fr_from_u64(n)));
  const host::Fr dinv = host::fr_inv(host::fr_from_u64(de)), ginv = host::fr_inv(host::fr_from_u64(ga));

  // ---- Lagrange basis at tau~ and A_i, B_i, C_i (device) ----
  DevBuf wpow, L, abc[3];
  wpow.ensure(sizeof(Fr) * n);
  L.ensure(sizeof(Fr) * n);
  Fr one_d;
  for (int i = 0; i < 8; i++) one_d.v[i] = FrParams::ONE[i];
  Fr w_d;
  for (int i = 0; i < 8; i++) w_d.v[i] = FR_ROOTS[log_n][i];
  fr_powers(wpow.as<Fr>(), w_d, one_d, n, st);
  if (host::fr_is_zero(zt)) {
    k_lagrange_point<<<ceil_div(n, 256), 256, 0, st>>>(wpow.as<Fr>(), to_dev(t), n, L.as<Fr>());
  } else {
    k_lagrange<<<ceil_div(ceil_div(n, LAG_CHUNK), 256), 256, 0, st>>>(wpow.as<Fr>(), to_dev(t), to_dev(kk), n,
                                                                      L.as<Fr>());
  }
  ZK_LAUNCH_CHECK();
  const uint64_t* rps[3] = {q->a_rowptr, q->b_rowptr, q->c_rowptr};
  const uint32_t* cols[3] = {q->a_col, q->b_col, q->c_col};
  const zk_fr* vals[3] = {q->a_val, q->b_val, q->c_val};
  for (int m = 0; m < 3; m++) {
    std::vector<uint64_t> cp;
    std::vector<uint32_t> row;
    std::vector<zk_fr> cval;
    csr_to_csc(nc, V, rps[m], cols[m], vals[m], cp, row, cval);
    DevBuf dcp, drow, draw, dval;
    dcp.ensure(sizeof(uint64_t) * (V + 1));
    drow.ensure(sizeof(uint32_t) * row.size());
    ZK_HIP(hipMemcpyAsync(dcp.p, cp.data(), sizeof(uint64_t) * (V + 1), hipMemcpyHostToDevice, st));
    ZK_HIP(hipMemcpyAsync(drow.p, row.data(), sizeof(uint32_t) * row.size(), hipMemcpyHostToDevice, st));
    if (vals[m]) {
      draw.ensure(sizeof(zk_fr) * cval.size());
      dval.ensure(sizeof(Fr) * cval.size());
      ZK_HIP(hipMemcpyAsync(draw.p, cval.data(), sizeof(zk_fr) * cval.size(), hipMemcpyHostToDevice, st));
      fr_to_mont(draw.as<uint64_t>(), dval.as<Fr>(), cval.size(), st);
    }
    abc[m].ensure(sizeof(Fr) * std::max<uint64_t>(V, 1));
    k_colsum<<<ceil_div(V, 256), 256, 0, st>>>(dcp.as<uint64_t>(), drow.as<uint32_t>(),
                                               vals[m] ? dval.as<Fr>() : nullptr, L.as<Fr>(), V, abc[m].as<Fr>());
    ZK_LAUNCH_CHECK();
    ZK_HIP(hipStreamSynchronize(st));  // host vectors / staging die here
  }

  // ---- lo64 scalars ----
  const uint64_t nic = V - num_public - 1, nvk = num_public + 1;
  DevBuf sa, sb, sic, svk, sh, tp;
  sa.ensure(8 * V);
  sb.ensure(8 * V);
  sic.ensure(8 * std::max<uint64_t>(nic, 1));
  svk.ensure(8 * nvk);
  sh.ensure(8 * n);
  tp.ensure(sizeof(Fr) * n);
  SetupConsts K;
  K.al = to_dev(host::fr_from_u64(al));
  K.be = to_dev(host::fr_from_u64(be));
  K.dinv = to_dev(dinv);
  K.ginv = to_dev(ginv);
  K.V = V;
  K.num_public = num_public;
  k_setup_scalars<<<ceil_div(V, 256), 256, 0, st>>>(abc[0].as<Fr>(), abc[1].as<Fr>(), abc[2].as<Fr>(), K,
                                                    sa.as<uint64_t>(), sb.as<uint64_t>(), sic.as<uint64_t>(),
                                                    svk.as<uint64_t>());
  ZK_LAUNCH_CHECK();
  fr_powers(tp.as<Fr>(), to_dev(t), to_dev(dinv), n, st);   // t~^i / d~
  k_lo64<<<ceil_div(n, 256), 256, 0, st>>>(tp.as<Fr>(), n, sh.as<uint64_t>());
  ZK_LAUNCH_CHECK();

  // ---- full-width generator multiples (host; setup:166-171) ----
  const auto G1h = g1_gen_host();
  const auto G2h = g2_gen_host();
  zk_g1_affine alpha_g1, beta_g1, delta_g1;
  zk_g2_affine beta_g2, gamma_g2, delta_g2;
  gen_mul_abi<G1>(G1h, P->alpha, &alpha_g1);
  gen_mul_abi<G1>(G1h, P->beta, &beta_g1);
  gen_mul_abi<G1>(G1h, P->delta, &delta_g1);
  gen_mul_abi<G2>(G2h, P->beta, &beta_g2);
  gen_mul_abi<G2>(G2h, P->delta, &delta_g2);
  gen_mul_abi<G2>(G2h, P->gamma, &gamma_g2);

  if (vk) {
    vk->alpha_g1 = alpha_g1;
    vk->beta_g2 = beta_g2;
    vk->gamma_g2 = gamma_g2;
    vk->delta_g2 = delta_g2;
    vk->num_public = num_public;
    vk->ic_len = nvk;
    DevBuf o;
    o.ensure(sizeof(G1A) * nvk);
    fixed_base<G1>(ctx, svk.as<uint64_t>(), nullptr, nvk, o.as<G1A>(), st);
    to_abi<G1>(o.as<G1A>(), nvk, vk->ic_g1, st);
  }

  if (pk_host) {
    // full vectors, canonical, into caller arrays
    pk_host->alpha_g1 = alpha_g1;
    pk_host->beta_g1 = beta_g1;
    pk_host->delta_g1 = delta_g1;
    pk_host->beta_g2 = beta_g2;
    pk_host->delta_g2 = delta_g2;
    pk_host->num_public = num_public;
    pk_host->a_len = V;
    pk_host->b_len = V;
    pk_host->b2_len = V;
    pk_host->ic_len = nic;
    pk_host->h_len = n;
    DevBuf o;
    o.ensure(sizeof(G2A) * std::max<uint64_t>(V, n));
    fixed_base<G1>(ctx, sa.as<uint64_t>(), nullptr, V, o.as<G1A>(), st);
    to_abi<G1>(o.as<G1A>(), V, pk_host->a_g1, st);
    fixed_base<G1>(ctx, sb.as<uint64_t>(), nullptr, V, o.as<G1A>(), st);
    to_abi<G1>(o.as<G1A>(), V, pk_host->b_g1, st);
    fixed_base<G2>(ctx, sb.as<uint64_t>(), nullptr, V, o.as<G2A>(), st);
    to_abi<G2>(o.as<G2A>(), V, pk_host->b_g2, st);
    fixed_base<G1>(ctx, sic.as<uint64_t>(), nullptr, nic, o.as<G1A>(), st);
    to_abi<G1>(o.as<G1A>(), nic, pk_host->ic_g1, st);
    fixed_base<G1>(ctx, sh.as<uint64_t>(), nullptr, n, o.as<G1A>(), st);
    to_abi<G1>(o.as<G1A>(), n, pk_host->h_g1, st);
    return ZK_OK;
  }

  // ---- device-resident (optionally sharded) proving key ----
  std::unique_ptr<zk_pk_dev> d(new zk_pk_dev());
  d->device = ctx->device;
  d->V = V;
  d->nc = nc;
  d->n = n;
  d->log_n = log_n;
  d->num_public = num_public;
  d->shard = shard;
  d->nshards = nshards;
  csr_upload(d->csr, q, st);
  // host copies of the scalar vectors decide which bases are the identity
  // (scalar 0 <=> identity, since every scalar is < 2^64 < r)
  std::vector<uint64_t> ha(V), hb(V), hic(nic), hh(n);
  ZK_HIP(hipMemcpyAsync(ha.data(), sa.p, 8 * V, hipMemcpyDeviceToHost, st));
  ZK_HIP(hipMemcpyAsync(hb.data(), sb.p, 8 * V, hipMemcpyDeviceToHost, st));
  if (nic) ZK_HIP(hipMemcpyAsync(hic.data(), sic.p, 8 * nic, hipMemcpyDeviceToHost, st));
  ZK_HIP(hipMemcpyAsync(hh.data(), sh.p, 8 * n, hipMemcpyDeviceToHost, st));
  ZK_HIP(hipStreamSynchronize(st));

  // this shard's variables (var_owner: those its quotient rows first read),
  // contiguous shard ranges, or (stride = nshards) positions i = shard mod nshards
  const std::vector<uint8_t> own = var_owner(q, n, nshards);
  auto build_slot = [&](int slot, bool g2, const std::vector<uint64_t>& hs, const DevBuf& ds, uint64_t len,
                        uint64_t idx_offset, const std::vector<uint64_t>& extra_words, uint32_t nextra,
                        bool strided = false) {
    const bool by_owner = !strided && !own.empty();
    const uint64_t lo = strided ? std::min<uint64_t>(shard, len) : by_owner ? 0 : len * shard / nshards;
    const uint64_t hi = strided || by_owner ? len : len * (shard + 1) / nshards;
    const uint64_t stride = strided ? nshards : 1;
    std::vector<uint32_t> loc, glob;
    for (uint64_t i = lo; i < hi; i += stride)
      if (hs[i] && (!by_owner || own[i + idx_offset] == shard)) {
        loc.push_back((uint32_t)i);
        glob.push_back((uint32_t)(i + idx_offset));
      }
    const uint32_t cnt = (uint32_t)loc.size();
    const size_t asz = g2 ? sizeof(G2A) : sizeof(G1A);
    if (slot == MSM_H) {
      d->h_ident = true;
      for (uint32_t k = 0; k < cnt; k++) d->h_ident = d->h_ident && glob[k] == k;
    }
    d->count[slot] = cnt;
    d->extras[slot] = nextra;
    d->bases[slot].ensure(asz * std::max<uint64_t>(cnt + nextra, 1));
    d->idx[slot].ensure(sizeof(uint32_t) * std::max<uint32_t>(cnt, 1));
    DevBuf dloc;
    dloc.ensure(sizeof(uint32_t) * std::max<uint32_t>(cnt, 1));
    if (cnt) {
      ZK_HIP(hipMemcpyAsync(dloc.p, loc.data(), 4 * cnt, hipMemcpyHostToDevice, st));
      ZK_HIP(hipMemcpyAsync(d->idx[slot].p, glob.data(), 4 * cnt, hipMemcpyHostToDevice, st));
      if (g2) fixed_base<G2>(ctx, ds.as<uint64_t>(), dloc.as<uint32_t>(), cnt, d->bases[slot].as<G2A>(), st);
      else fixed_base<G1>(ctx, ds.as<uint64_t>(), dloc.as<uint32_t>(), cnt, d->bases[slot].as<G1A>(), st);
    }
    if (nextra) {
      DevBuf ex;
      ex.ensure(8 * extra_words.size());
      ZK_HIP(hipMemcpyAsync(ex.p, extra_words.data(), 8 * extra_words.size(), hipMemcpyHostToDevice, st));
      if (g2) convert_bases<G2>(ex.as<uint64_t>(), d->bases[slot].as<G2A>() + cnt, nextra, st);
      else convert_bases<G1>(ex.as<uint64_t>(), d->bases[slot].as<G1A>() + cnt, nextra, st);
    }
    ZK_HIP(hipStreamSynchronize(st));
  };
  // extras on shard 0 (see prove.hip): alpha_1 + 2^(64k) delta_1; beta_2 + 2^(64k) delta_2; beta_1
  std::vector<uint64_t> exA, exB2, exB1, none;
  uint32_t nA = 0, nB2 = 0, nB1 = 0;
  if (shard == 0) {
    auto push = [](std::vector<uint64_t>& v, const void* p, int words) {
      const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
      v.insert(v.end(), w, w + words);
    };
    push(exA, &alpha_g1, 13);
    auto dA = host::mul_scalar(G1h, P->delta.l);
    for (int k = 0; k < 4; k++) {
      uint64_t w[13];
      host_to_abi<G1>(dA, w);
      exA.insert(exA.end(), w, w + 13);
      for (int b = 0; b < 64; b++) dA = host::dbl(dA);
    }
    push(exB2, &beta_g2, 25);
    auto dB = host::mul_scalar(G2h, P->delta.l);
    for (int k = 0; k < 4; k++) {
      uint64_t w[25];
      host_to_abi<G2>(dB, w);
      exB2.insert(exB2.end(), w, w + 25);
      for (int b = 0; b < 64; b++) dB = host::dbl(dB);
    }
    push(exB1, &beta_g1, 13);
    nA = 5;
    nB2 = 5;
    nB1 = 1;
  }
  build_slot(MSM_A, false, ha, sa, V, 0, exA, nA);
  build_slot(MSM_B2, true, hb, sb, V, 0, exB2, nB2);
  build_slot(MSM_B1, false, hb, sb, V, 0, exB1, nB1);
  build_slot(MSM_IC, false, hic, sic, nic, num_public + 1, none, 0);
  build_slot(MSM_H, false, hh, sh, n, 0, none, 0, /*strided*/ true);
  pk_precompute_windows(ctx, *d);
  pk_witness_ranges(*d, q, own, st);
  pk_part_cuts(*d, st);
  *pk_dev = d.release();
  return ZK_OK;
}

// ---------------------------------------------------- QAP::evaluate_at ---
// A(t) = sum_i z_i A_i(t) = sum_j (Az)_j L_j(t) (A_i interpolates column i of
// the constraint matrix over the domain, qap:143-170; columns >= V dropped,
// qap:122-124), likewise B, C; Z(t) = t^n - 1 (qap:173-176, 211).
__global__ void __launch_bounds__(256) k_eval_rows(CsrArgs m, const Fr* __restrict__ zc, uint64_t nc, uint64_t V,
                                                   const Fr* __restrict__ L, Fr* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nc) return;
  const Fr l = ld_vec(&L[j]);
#pragma unroll
  for (int k = 0; k < 3; k++) st_vec(&out[k * nc + j], fp_mul(row_dot(m.rp[k], m.col[k], m.val[k], j, zc, V), l));
}
// out[b] = sum of in[i] over i = b, b + stride, ... (per block b: one LDS tree)
__global__ void __launch_bounds__(256) k_fr_sum(const Fr* __restrict__ in, uint64_t n, Fr* __restrict__ out) {
  __shared__ Fr part[256];
  Fr acc = fp_zero<FrParams>();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc = fp_add(acc, ld_vec(&in[i]));
  part[threadIdx.x] = acc;
  __syncthreads();
  for (unsigned h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) part[threadIdx.x] = fp_add(part[threadIdx.x], part[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) st_vec(&out[blockIdx.x], part[0]);
}

// sum of n device Fr (Montgomery) -> host canonical
static void fr_sum_to_host(const Fr* d_in, uint64_t n, zk_fr* out, hipStream_t st) {
  DevBuf part;
  const uint32_t nb = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ceil_div(n, 256), 1), 1024);
  part.ensure(sizeof(Fr) * (nb + 1));
  k_fr_sum<<<nb, 256, 0, st>>>(d_in, n, part.as<Fr>());
  ZK_LAUNCH_CHECK();
  k_fr_sum<<<1, 256, 0, st>>>(part.as<Fr>(), nb, part.as<Fr>() + nb);
  ZK_LAUNCH_CHECK();
  fr_from_mont(part.as<Fr>() + nb, reinterpret_cast<uint64_t*>(part.as<Fr>() + nb), 1, st);
  ZK_HIP(hipMemcpyAsync(out, part.as<Fr>() + nb, sizeof(zk_fr), hipMemcpyDeviceToHost, st));
  ZK_HIP(hipStreamSynchronize(st));
}

int qap_evaluate_impl(zk_ctx* ctx, const zk_r1cs_csr* q, const zk_fr* point, const zk_fr* z, size_t zlen,
                      zk_fr out[4]) {
  hipStream_t st = ctx->stream;
  const uint64_t V = q->num_variables, nc = q->num_constraints;
  if (zlen != V) return ZK_ERR_DIMENSION;   // qap:191-198
  if (!fr_canonical(*point)) return ZK_ERR_ARG;
  for (size_t i = 0; i < zlen; i++)
    if (!fr_canonical(z[i])) return ZK_ERR_ARG;
  if (nc > (1ull << 32)) return ZK_ERR_DOMAIN;   // Fr 2-adicity 32 (qap:101-105); also keeps the loop finite
  uint64_t n = 1;
  while (n < nc) n <<= 1;
  const uint32_t log_n = (uint32_t)__builtin_ctzll(n);
  auto to_dev = [](const host::Fr& h) { Fr d; const host::Fr v = host::fr_to_dev(h); std::memcpy(d.v, v.l, 32); return d; };
  const host::Fr t = host::fr_to_mont(point->l);
  host::Fr tn = t;
  for (uint32_t i = 0; i < log_n; i++) tn = host::fr_mul(tn, tn);
  const host::Fr zt = host::fr_sub(tn, host::fr_one());
  host::fr_from_mont(zt, out[3].l);
  for (int k = 0; k < 3; k++) std::memset(out[k].l, 0, 32);
  if (nc == 0) return ZK_OK;
  DevBuf wpow, L, dz, rows;
  CsrDev csr;
  csr_upload(csr, q, st);
  wpow.ensure(sizeof(Fr) * n);
  L.ensure(sizeof(Fr) * n);
  Fr one_d, w_d;
  for (int i = 0; i < 8; i++) one_d.v[i] = FrParams::ONE[i];
  for (int i = 0; i < 8; i++) w_d.v[i] = FR_ROOTS[log_n][i];
  fr_powers(wpow.as<Fr>(), w_d, one_d, n, st);
  if (host::fr_is_zero(zt)) {
    k_lagrange_point<<<ceil_div(n, 256), 256, 0, st>>>(wpow.as<Fr>(), to_dev(t), n, L.as<Fr>());
  } else {
    const host::Fr kk = host::fr_mul(zt, host::fr_inv(host::fr_from_u64(n)));
    k_lagrange<<<ceil_div(ceil_div(n, LAG_CHUNK), 256), 256, 0, st>>>(wpow.as<Fr>(), to_dev(t), to_dev(kk), n,
                                                                      L.as<Fr>());
  }
  ZK_LAUNCH_CHECK();
  dz.ensure(sizeof(zk_fr) * std::max<size_t>(zlen, 1));
  if (zlen) ZK_HIP(hipMemcpyAsync(dz.p, z, sizeof(zk_fr) * zlen, hipMemcpyHostToDevice, st));
  rows.ensure(sizeof(Fr) * 3 * nc);
  k_eval_rows<<<ceil_div(nc, 256), 256, 0, st>>>(csr_args(csr), dz.as<Fr>(), nc, V, L.as<Fr>(), rows.as<Fr>());
  ZK_LAUNCH_CHECK();
  for (int k = 0; k < 3; k++) fr_sum_to_host(rows.as<Fr>() + k * nc, nc, &out[k], st);
  return ZK_OK;
}

// ------------------------------------------------------- serialization ---
// ark-serialize 0.4 / zcash compressed encoding (ark-bls12-381 0.4): big-endian
// x with flags in byte 0: 0x80 compressed, 0x40 infinity, 0x20 y > (p-1)/2
// (Fq2: compare c1, or c0 when c1 == 0).
static void be48(const uint64_t* l, uint8_t* o) {
  for (int i = 0; i < 48; i++) o[i] = (uint8_t)(l[(47 - i) / 8] >> (8 * ((47 - i) % 8)));
}
bool fq_canonical_largest(const uint64_t* c) {
  const uint64_t* m = host::FQ().m;
  uint64_t half[6];
  for (int i = 0; i < 6; i++) half[i] = (m[i] >> 1) | (i < 5 ? (m[i + 1] << 63) : 0);
  for (int i = 5; i >= 0; i--) {
    if (c[i] > half[i]) return true;
    if (c[i] < half[i]) return false;
  }
  return false;
}
static bool is_zero6(const uint64_t* c) {
  uint64_t x = 0;
  for (int i = 0; i < 6; i++) x |= c[i];
  return x == 0;
}
void serialize_g1_compressed(const zk_g1_affine& p, uint8_t* out) {
  std::memset(out, 0, 48);
  if (p.infinity) { out[0] = 0xc0; return; }
  be48(p.x, out);
  out[0] |= 0x80;
  if (fq_canonical_largest(p.y)) out[0] |= 0x20;
}
void serialize_g2_compressed(const zk_g2_affine& p, uint8_t* out) {
  std::memset(out, 0, 96);
  if (p.infinity) { out[0] = 0xc0; return; }
  be48(p.x + 6, out);
  be48(p.x, out + 48);
  out[0] |= 0x80;
  const bool big = is_zero6(p.y + 6) ? fq_canonical_largest(p.y) : fq_canonical_largest(p.y + 6);
  if (big) out[0] |= 0x20;
}

}  // namespace zk
