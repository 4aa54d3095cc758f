// dist.hip -- the quotient distributed over the ranks of a sharded prover
// (see dist.hpp for the four-step decomposition).
//
// Rank r of N, n = N m, q = m / N:
//   A  evaluate (Az, Bz, Cz) at rows a m + b for its columns b = r q + b'
//      (every a < N), size-N inverse DFT down each column, twiddle
//      omega_n^(-b k1)                          -> exchange 1 (3q per rank)
//   B  row k1 = r: size-m inverse DFT (A/B/C coefficients i = r + N k2),
//      scale n^-1 g^i, size-m forward DFT, twiddle omega_n^(r e)
//                                               -> exchange 2 (3q per rank)
//   C  columns e = r q + e': size-N forward DFT (coset evaluations at
//      k = e + m f), (A B - C) / Z, size-N inverse DFT, twiddle
//      omega_n^(-c e)                           -> exchange 3 (q per rank)
//   D  row c = r: size-m inverse DFT, n^-1 g^-i, lo64 -> H_(r + N d)
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "dist.hpp"
#include "quotient.hpp"

#include <rccl/rccl.h>

namespace zk {

bool dist_quotient_ok(uint64_t n, int world) {
  if (world != 2 && world != 4 && world != 8) return false;
  return n % ((uint64_t)world * world) == 0;
}

constexpr int brev_c(int k, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((k >> i) & 1) << (bits - 1 - i);
  return r;
}

// In-register radix-2 DIF DFT of 2^LOGN elements, twiddles omega_2048^j
// (sm: forward or inverse table).  Output X[k] sits at x[brev(k)].
template <int LOGN>
ZK_DI void small_dft(Fr (&x)[1 << LOGN], const Fr* __restrict__ sm) {
  constexpr int N = 1 << LOGN;
#pragma unroll
  for (int hl = LOGN - 1; hl >= 0; hl--) {
    const int h = 1 << hl;
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
      const int j = i & (h - 1), lo = ((i >> hl) << (hl + 1)) | j;
      const Fr u = x[lo], v = x[lo + h];
      x[lo] = fp_add(u, v);
      x[lo + h] = j ? fp_mul(fp_sub(u, v), ld_vec(&sm[j << (10 - hl)])) : fp_sub(u, v);
    }
  }
}

// ------------------------------------------------------------ stage A ---
template <int LOGN>
__global__ void __launch_bounds__(128) k_dq_eval(CsrArgs mm, const Fr* __restrict__ zc, uint64_t nc, uint64_t V,
                                                 uint64_t vrow, int rank, uint64_t m, uint64_t q, NttTabs itab,
                                                 uint32_t log_n, uint32_t* __restrict__ flags,
                                                 Fr* __restrict__ s1) {
  constexpr int N = 1 << LOGN;
  const uint64_t bp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (rank == 0 && bp == 0) {
    const Fr z0 = ld_vec(&zc[0]);
    bool one = z0.v[0] == 1;
#pragma unroll
    for (int i = 1; i < 8; i++) one = one && z0.v[i] == 0;
    if (!one) atomicOr(flags, 4u);   // core:89-93
  }
  if (bp >= q) return;
  const uint64_t b = (uint64_t)rank * q + bp;
  Fr xa[N], xb[N], xc[N];
#pragma unroll
  for (int a = 0; a < N; a++) {
    const uint64_t j = (uint64_t)a * m + b;
    xa[a] = fp_zero<FrParams>();
    xb[a] = xa[a];
    xc[a] = xa[a];
    if (j < nc) {   // rows >= nc are zero padding (qap:155-164)
      xa[a] = row_dot(mm.rp[0], mm.col[0], mm.val[0], j, zc, V);
      xb[a] = row_dot(mm.rp[1], mm.col[1], mm.val[1], j, zc, V);
      xc[a] = row_dot(mm.rp[2], mm.col[2], mm.val[2], j, zc, V);
      if (!fp_eq(fp_mul(xa[a], xb[a]), xc[a])) atomicOr(flags, j == vrow ? 3u : 2u);
    }
  }
  small_dft<LOGN>(xa, itab.sm);
  small_dft<LOGN>(xb, itab.sm);
  small_dft<LOGN>(xc, itab.sm);
#pragma unroll
  for (int k1 = 0; k1 < N; k1++) {
    const int p = brev_c(k1, LOGN);
    Fr ya = xa[p], yb = xb[p], yc = xc[p];
    if (k1) {
      const Fr w = tw_full(itab, (uint32_t)(b * k1), log_n);   // omega_n^(-b k1)
      ya = fp_mul(ya, w);
      yb = fp_mul(yb, w);
      yc = fp_mul(yc, w);
    }
    Fr* dst = s1 + (size_t)k1 * 3 * q + bp;
    st_vec(&dst[0], ya);
    st_vec(&dst[q], yb);
    st_vec(&dst[2 * q], yc);
  }
}

// ------------------------------------------------------------ stage B ---
// r1 [s][vec][b'] -> rows [vec][s q + b']
__global__ void __launch_bounds__(256) k_dq_rows(const Fr* __restrict__ r1, uint64_t m, uint64_t q,
                                                 Fr* __restrict__ rows) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 3 * m) return;
  const uint64_t vec = idx / m, b = idx % m, s = b / q, bp = b % q;
  st_vec(&rows[idx], ld_vec(&r1[(s * 3 + vec) * q + bp]));
}

// bit-reversed coefficients: position p holds k2 = brev(p) -> times n^-1 g^(r + N k2)
__global__ void __launch_bounds__(256) k_dq_coset(Fr* __restrict__ rows, const Fr* __restrict__ gpow, int rank,
                                                  int world, uint64_t m, uint32_t log_m) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 3 * m) return;
  const uint64_t p = idx % m;
  const uint64_t k2 = log_m ? (__builtin_bitreverse32((uint32_t)p) >> (32 - log_m)) : 0;
  st_vec(&rows[idx], fp_mul(ld_vec(&rows[idx]), ld_vec(&gpow[rank + (uint64_t)world * k2])));
}

// rows [vec][e] * omega_n^(r e) -> s2 [s][vec][e'] (e = s q + e')
__global__ void __launch_bounds__(256) k_dq_send2(const Fr* __restrict__ rows, int rank, uint64_t m, uint64_t q,
                                                  NttTabs ftab, uint32_t log_n, Fr* __restrict__ s2) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 3 * m) return;
  const uint64_t vec = idx / m, e = idx % m, s = e / q, ep = e % q;
  Fr v = ld_vec(&rows[idx]);
  if (rank) v = fp_mul(v, tw_full(ftab, (uint32_t)(rank * e), log_n));
  st_vec(&s2[(s * 3 + vec) * q + ep], v);
}

// ------------------------------------------------------------ stage C ---
template <int LOGN>
__global__ void __launch_bounds__(128) k_dq_pointwise(const Fr* __restrict__ r2, int rank, uint64_t q,
                                                      const Fr* __restrict__ zinv, NttTabs ftab, NttTabs itab,
                                                      uint32_t log_n, Fr* __restrict__ s3) {
  constexpr int N = 1 << LOGN;
  const uint64_t ep = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ep >= q) return;
  const uint64_t e = (uint64_t)rank * q + ep;
  Fr u[N], Q[N];
  // coset evaluations Y[e + m f] = sum_c omega_N^(c f) u_c[e]
#pragma unroll
  for (int c = 0; c < N; c++) u[c] = ld_vec(&r2[((size_t)c * 3 + 0) * q + ep]);
  small_dft<LOGN>(u, ftab.sm);
#pragma unroll
  for (int f = 0; f < N; f++) Q[f] = u[brev_c(f, LOGN)];
#pragma unroll
  for (int c = 0; c < N; c++) u[c] = ld_vec(&r2[((size_t)c * 3 + 1) * q + ep]);
  small_dft<LOGN>(u, ftab.sm);
#pragma unroll
  for (int f = 0; f < N; f++) Q[f] = fp_mul(Q[f], u[brev_c(f, LOGN)]);
#pragma unroll
  for (int c = 0; c < N; c++) u[c] = ld_vec(&r2[((size_t)c * 3 + 2) * q + ep]);
  small_dft<LOGN>(u, ftab.sm);
  const Fr zi = ld_vec(zinv);
#pragma unroll
  for (int f = 0; f < N; f++) Q[f] = fp_mul(fp_sub(Q[f], u[brev_c(f, LOGN)]), zi);   // (A B - C) / Z
  // v[c] = sum_f Q[e + m f] omega_N^(-c f), then omega_n^(-c e)
  small_dft<LOGN>(Q, itab.sm);
#pragma unroll
  for (int c = 0; c < N; c++) {
    Fr v = Q[brev_c(c, LOGN)];
    if (c) v = fp_mul(v, tw_full(itab, (uint32_t)(c * e), log_n));
    st_vec(&s3[(size_t)c * q + ep], v);
  }
}

// ------------------------------------------------------------ stage D ---
__global__ void __launch_bounds__(256) k_dq_h(const Fr* __restrict__ hb, const Fr* __restrict__ gipow, int rank,
                                              int world, uint64_t m, uint32_t log_m, uint64_t* __restrict__ hlo) {
  const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= m) return;
  const uint64_t p = log_m ? (__builtin_bitreverse32((uint32_t)d) >> (32 - log_m)) : 0;
  const Fr h = fp_from_mont(fp_mul(ld_vec(&hb[p]), ld_vec(&gipow[rank + (uint64_t)world * d])));
  hlo[d] = (uint64_t)h.v[0] | ((uint64_t)h.v[1] << 32);   // core:203-208
}

// ------------------------------------------------------------- driver ---
static int log2i(uint64_t v) { return 63 - __builtin_clzll(v); }

size_t dq_chunk_bytes(const zk_pk_dev* pk, int world, int which) {
  const uint64_t q = pk->n / world / world;
  return sizeof(Fr) * q * (which == 3 ? 1 : 3);
}

static void ensure_bufs(const zk_pk_dev* pk, int world, DistQ& dq) {
  const uint64_t m = pk->n / world;
  dq.s1.ensure(sizeof(Fr) * 3 * m);
  dq.r1.ensure(sizeof(Fr) * 3 * m);
  dq.s2.ensure(sizeof(Fr) * 3 * m);
  dq.r2.ensure(sizeof(Fr) * 3 * m);
  dq.s3.ensure(sizeof(Fr) * m);
  dq.r3.ensure(sizeof(Fr) * m);
}

void dq_stage_a(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, int rank, int world, DistQ& dq,
                uint32_t* d_flags, hipStream_t st) {
  ensure_bufs(pk, world, dq);
  const uint64_t n = pk->n, m = n / world, q = m / world;
  NttDomain& dn = ctx->domain(pk->log_n);
  const NttTabs itab = tabs_of(dn, true);
  const CsrArgs mm = csr_args(pk->csr);
  const uint64_t vrow = n > 1 ? 1 : 0;
  const Fr* zc = reinterpret_cast<const Fr*>(d_z);
  const uint32_t nb = ceil_div(q, 128);
  switch (world) {
    case 2: k_dq_eval<1><<<nb, 128, 0, st>>>(mm, zc, pk->nc, pk->V, vrow, rank, m, q, itab, pk->log_n, d_flags, dq.s1.as<Fr>()); break;
    case 4: k_dq_eval<2><<<nb, 128, 0, st>>>(mm, zc, pk->nc, pk->V, vrow, rank, m, q, itab, pk->log_n, d_flags, dq.s1.as<Fr>()); break;
    case 8: k_dq_eval<3><<<nb, 128, 0, st>>>(mm, zc, pk->nc, pk->V, vrow, rank, m, q, itab, pk->log_n, d_flags, dq.s1.as<Fr>()); break;
    default: throw Error(ZK_ERR_ARG, "distributed quotient: world must be 2, 4 or 8");
  }
  ZK_LAUNCH_CHECK();
}

void dq_stage_b(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& dq, hipStream_t st) {
  const uint64_t n = pk->n, m = n / world, q = m / world;
  const uint32_t log_m = (uint32_t)log2i(m);
  NttDomain& dn = ctx->domain(pk->log_n);
  NttDomain& dm = ctx->domain(log_m);
  Fr* rows = dq.s1.as<Fr>();   // stage A's send buffer is free again
  k_dq_rows<<<ceil_div(3 * m, 256), 256, 0, st>>>(dq.r1.as<Fr>(), m, q, rows);
  ZK_LAUNCH_CHECK();
  for (int v = 0; v < 3; v++) ntt_dif(rows + v * m, dm, /*inverse*/ true, st, &ctx->prof);   // n A_i, bit-reversed
  k_dq_coset<<<ceil_div(3 * m, 256), 256, 0, st>>>(rows, domain_gpow(dn, st), rank, world, m, log_m);
  ZK_LAUNCH_CHECK();
  for (int v = 0; v < 3; v++) ntt_dit(rows + v * m, dm, /*inverse*/ false, st, &ctx->prof);  // natural e
  k_dq_send2<<<ceil_div(3 * m, 256), 256, 0, st>>>(rows, rank, m, q, tabs_of(dn, false), pk->log_n,
                                                   dq.s2.as<Fr>());
  ZK_LAUNCH_CHECK();
}

void dq_stage_c(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& dq, hipStream_t st) {
  const uint64_t n = pk->n, m = n / world, q = m / world;
  NttDomain& dn = ctx->domain(pk->log_n);
  const NttTabs ftab = tabs_of(dn, false), itab = tabs_of(dn, true);
  const uint32_t nb = ceil_div(q, 128);
  const Fr* r2 = dq.r2.as<Fr>();
  Fr* s3 = dq.s3.as<Fr>();
  const Fr* zinv = dn.zinv.as<Fr>();
  switch (world) {
    case 2: k_dq_pointwise<1><<<nb, 128, 0, st>>>(r2, rank, q, zinv, ftab, itab, pk->log_n, s3); break;
    case 4: k_dq_pointwise<2><<<nb, 128, 0, st>>>(r2, rank, q, zinv, ftab, itab, pk->log_n, s3); break;
    case 8: k_dq_pointwise<3><<<nb, 128, 0, st>>>(r2, rank, q, zinv, ftab, itab, pk->log_n, s3); break;
    default: throw Error(ZK_ERR_ARG, "distributed quotient: world must be 2, 4 or 8");
  }
  ZK_LAUNCH_CHECK();
}

void dq_stage_d(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& dq, uint64_t* h_out,
                hipStream_t st) {
  const uint64_t n = pk->n, m = n / world;
  const uint32_t log_m = (uint32_t)log2i(m);
  NttDomain& dn = ctx->domain(pk->log_n);
  NttDomain& dm = ctx->domain(log_m);
  ntt_dif(dq.r3.as<Fr>(), dm, /*inverse*/ true, st, &ctx->prof);
  k_dq_h<<<ceil_div(m, 256), 256, 0, st>>>(dq.r3.as<Fr>(), domain_gipow(dn, st), rank, world, m, log_m, h_out);
  ZK_LAUNCH_CHECK();
}

void dq_prepare(zk_ctx* ctx, const zk_pk_dev* pk, int world, DistQ& dq, hipStream_t st) {
  ensure_bufs(pk, world, dq);
  NttDomain& dn = ctx->domain(pk->log_n);
  (void)ctx->domain((uint32_t)log2i(pk->n / world));
  domain_gpow(dn, st);
  domain_gipow(dn, st);
  ZK_HIP(hipStreamSynchronize(st));
}

void dist_quotient(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, Exchange& ex, DistQ& dq,
                   uint32_t* d_flags, uint64_t* h_out, hipStream_t st) {
  const int r = ex.rank, N = ex.world;
  const int fault = ex.fault_after;
  ex.fault_after = 0;   // one proof
  auto exchange = [&](int k, const DevBuf& s, DevBuf& rv) {
    ex.all_to_all(s.p, rv.p, dq_chunk_bytes(pk, N, k), st);
    if (fault == k) throw Error(ZK_ERR_DEVICE, "injected fault after exchange " + std::to_string(k));
  };
  dq_stage_a(ctx, pk, d_z, r, N, dq, d_flags, st);
  exchange(1, dq.s1, dq.r1);
  dq_stage_b(ctx, pk, r, N, dq, st);
  exchange(2, dq.s2, dq.r2);
  dq_stage_c(ctx, pk, r, N, dq, st);
  exchange(3, dq.s3, dq.r3);
  dq_stage_d(ctx, pk, r, N, dq, h_out, st);
}

void sync_watchdog(hipStream_t st, Exchange& ex) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) ZK_HIP(q);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ex.async_error()) throw Error(ZK_ERR_RCCL, "exchange: asynchronous transport error");
    if (ms > ex.timeout_ms) throw Error(ZK_ERR_RCCL, "exchange: a peer did not answer within the timeout");
    std::this_thread::yield();
  }
}

// --------------------------------------------------------------- RCCL ---
// The communicator is created non-blocking (ncclConfig_t::blocking = 0):
// ncclCommInitRankConfig and the collectives may return ncclInProgress, and
// the operation then completes in the background; nccl_wait polls
// ncclCommGetAsyncError until it has, under the exchange's watchdog.  A
// blocking ncclCommInitRank waits forever for a peer that never calls it
// (a rank that failed before the attach), which no caller can recover from.
static void nccl_wait(ncclComm_t comm, double timeout_ms, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError(comm, &st);
    if (q != ncclSuccess) throw Error(ZK_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(q));
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) throw Error(ZK_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(st));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > timeout_ms)
      throw Error(ZK_ERR_RCCL, std::string(what) + ": not complete within the exchange timeout (a peer missing?)");
    std::this_thread::yield();
  }
}

#define ZK_NCCL(comm, timeout_ms, call)                                                        \
  do {                                                                                         \
    const ncclResult_t r_ = (call);                                                            \
    if (r_ == ncclInProgress)                                                                  \
      nccl_wait((comm), (timeout_ms), #call);                                                  \
    else if (r_ != ncclSuccess)                                                                \
      throw ::zk::Error(ZK_ERR_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_));     \
  } while (0)

struct RcclExchange : Exchange {
  ncclComm_t comm = nullptr;
  DevBuf stat;
  PinnedBuf stat_host;
  void all_to_all(const void* send, void* recv, size_t chunk_bytes, hipStream_t st) override {
    ZK_NCCL(comm, timeout_ms, ncclAllToAll(send, recv, chunk_bytes, ncclUint8, comm, st));
  }
  int agree_max(int status, hipStream_t st) override {
    int32_t v[2] = {status, 0};
    agree_max2(v, st);
    return v[0];
  }
  void agree_max2(int32_t v[2], hipStream_t st) override {
    stat.ensure(16);
    stat_host.ensure(16);
    std::memcpy(stat_host.p, v, 8);
    ZK_HIP(hipMemcpyAsync(stat.p, stat_host.p, 8, hipMemcpyHostToDevice, st));
    ZK_NCCL(comm, timeout_ms, ncclAllReduce(stat.p, stat.p, 2, ncclInt32, ncclMax, comm, st));
    ZK_HIP(hipMemcpyAsync(stat_host.p, stat.p, 8, hipMemcpyDeviceToHost, st));
    sync_watchdog(st, *this);
    std::memcpy(v, stat_host.p, 8);
  }
  bool agree_max_dev(uint32_t* d_val, hipStream_t st) override {
    ZK_NCCL(comm, timeout_ms, ncclAllReduce(d_val, d_val, 1, ncclUint32, ncclMax, comm, st));
    return true;
  }
  // ncclCommAbort sets the communicator's abort flag, which its in-flight
  // kernels poll: this rank's collectives end, and so do the peers' once
  // their own watchdog (prove.hip) aborts them.
  void abort() override {
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
  }
  bool async_error() override {
    if (!comm) return true;
    ncclResult_t r = ncclSuccess;
    return ncclCommGetAsyncError(comm, &r) != ncclSuccess || (r != ncclSuccess && r != ncclInProgress);
  }
  ~RcclExchange() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
};

// ---------------------------------------------------------- host-staged ---
// Each all-to-all: the send chunks come back to pinned host memory (after the
// stream's preceding kernels), the caller's callback moves them between the
// ranks, and the received chunks go back to the device ahead of the next
// stage.  Synchronous on the calling thread; the other streams (the MSMs)
// keep running meanwhile.  A callback error or a non-zero status becomes
// ZK_ERR_RCCL.
struct HostExchange : Exchange {
  zk_exchange_ops ops{};
  PinnedBuf send_h, recv_h;
  void all_to_all(const void* send, void* recv, size_t chunk_bytes, hipStream_t st) override {
    const size_t bytes = chunk_bytes * (size_t)world;
    send_h.ensure(bytes);
    recv_h.ensure(bytes);
    ZK_HIP(hipMemcpyAsync(send_h.p, send, bytes, hipMemcpyDeviceToHost, st));
    ZK_HIP(hipStreamSynchronize(st));
    if (ops.all_to_all(ops.user, send_h.p, recv_h.p, chunk_bytes) != 0)
      throw Error(ZK_ERR_RCCL, "host exchange: all_to_all callback failed");
    ZK_HIP(hipMemcpyAsync(recv, recv_h.p, bytes, hipMemcpyHostToDevice, st));
  }
  int agree_max(int status, hipStream_t st) override {
    (void)st;
    int32_t v = status;
    if (ops.all_reduce_max(ops.user, &v) != 0) throw Error(ZK_ERR_RCCL, "host exchange: all_reduce_max callback failed");
    return v;
  }
  void abort() override {
    if (ops.abort) ops.abort(ops.user);
  }
  void detach() override {}
};

std::unique_ptr<Exchange> make_host_exchange(const zk_exchange_ops& ops, int rank, int world) {
  if (!ops.all_to_all || !ops.all_reduce_max) throw Error(ZK_ERR_ARG, "host exchange: missing callbacks");
  std::unique_ptr<HostExchange> ex(new HostExchange());
  ex->ops = ops;
  ex->rank = rank;
  ex->world = world;
  return ex;
}

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");

void rccl_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw Error(ZK_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, 128);
}

std::unique_ptr<Exchange> make_rccl_exchange(const uint8_t unique_id[128], int rank, int world, double timeout_ms) {
  std::unique_ptr<RcclExchange> ex(new RcclExchange());
  ex->rank = rank;
  ex->world = world;
  ex->timeout_ms = timeout_ms;
  ncclUniqueId id;
  std::memcpy(&id, unique_id, 128);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = ncclCommInitRankConfig(&ex->comm, world, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (ex->comm) (void)ncclCommAbort(ex->comm);
    ex->comm = nullptr;
    throw Error(ZK_ERR_RCCL, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  try {
    nccl_wait(ex->comm, timeout_ms, "ncclCommInitRankConfig");
  } catch (...) {
    ex->abort();   // a half-made communicator: abort is local, destroy would wait for the peers
    throw;
  }
  return ex;
}

}  // namespace zk
