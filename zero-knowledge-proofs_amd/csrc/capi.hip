// capi.hip -- extern "C" boundary (include/zkp.h).  Every entry point catches
// zk::Error / std::exception and returns a zk_status; nothing throws across.
#include <cstring>
#include <vector>

#include "ctx.hpp"

namespace zk {
zk_pk_dev* pk_upload(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* q, uint32_t shard, uint32_t nshards);
int prove_impl(zk_ctx*, const zk_pk_dev*, const void*, size_t, size_t, const zk_fr*, const zk_fr*, zk_proof*,
               const zk_fr* z_host = nullptr);
int prove_partial_impl(zk_ctx*, const zk_pk_dev*, const void*, size_t, size_t, const zk_fr*, const zk_fr*,
                       zk_prove_partial*);
int prove_partial_host_impl(zk_ctx*, const zk_pk_dev*, const zk_fr*, size_t, size_t, size_t, const zk_fr*,
                            const zk_fr*, zk_prove_partial*);
std::vector<uint64_t> witness_ranges(const zk_ctx*, const zk_pk_dev*);
int combine_impl(const zk_prove_partial*, size_t, const zk_fr*, const zk_fr*, zk_proof*);
int setup_impl(zk_ctx*, const zk_r1cs_csr*, const zk_setup_params*, uint64_t, uint32_t, uint32_t, zk_pk*,
               zk_pk_dev**, zk_vk*);
void serialize_g1_compressed(const zk_g1_affine& p, uint8_t* out);
void serialize_g2_compressed(const zk_g2_affine& p, uint8_t* out);
}  // namespace zk

using namespace zk;

NttDomain& zk_ctx::domain(uint32_t log_n) {
  auto it = domains.find(log_n);
  if (it != domains.end()) return *it->second;
  std::unique_ptr<NttDomain> d(new NttDomain());
  ntt_domain_init(*d, log_n, stream);
  NttDomain& ref = *d;
  domains[log_n] = std::move(d);
  return ref;
}

#define ZK_GUARD(ctx, ...)                                    \
  try {                                                       \
    if (ctx) ZK_HIP(hipSetDevice((ctx)->device));             \
    __VA_ARGS__                                               \
  } catch (const zk::Error& e) {                              \
    if (ctx) (ctx)->err = e.what();                           \
    return e.code;                                            \
  } catch (const std::exception& e) {                         \
    if (ctx) (ctx)->err = e.what();                           \
    return ZK_ERR_DEVICE;                                     \
  }

// Definitions below inherit C linkage from their declarations in include/zkp.h.

zk_ctx* zk_ctx_create(int device) {
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    ZK_HIP(hipSetDevice(device));
    std::unique_ptr<zk_ctx> c(new zk_ctx());
    c->device = device;
    for (int i = 0; i < NUM_MSM; i++) c->msm[i].prof = &c->prof;
    for (int k = 0; k < HOST_PARTS - 1; k++) c->part_g2[k].prof = c->part_abi[k].prof = &c->prof;
    int lo_prio = 0, hi_prio = 0;
    ZK_HIP(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
    ZK_HIP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_prio));   // quotient + H
    // side[0]: G2 MSM (high), side[1..]: the G1 batches (low); other
    // priority assignments measured within noise
    // (ZK_SIDE_PRIO_MASK: A/B builds, bit i = side[i] at high priority)
#ifndef ZK_SIDE_PRIO_MASK
#define ZK_SIDE_PRIO_MASK 1
#endif
    for (int i = 0; i < NUM_SIDE; i++)
      ZK_HIP(hipStreamCreateWithPriority(&c->side[i], hipStreamNonBlocking,
                                         (ZK_SIDE_PRIO_MASK >> i) & 1 ? hi_prio : lo_prio));
    ZK_HIP(hipEventCreateWithFlags(&c->ev_scal, hipEventDisableTiming));
    ZK_HIP(hipEventCreateWithFlags(&c->ev_quot, hipEventDisableTiming));
    for (auto& e : c->ev_done) ZK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ZK_HIP(hipEventCreateWithFlags(&c->ev_ic, hipEventDisableTiming));
    return c.release();
  } catch (...) {
    return nullptr;
  }
}

void zk_ctx_destroy(zk_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (int i = 0; i < NUM_SIDE; i++) (void)hipStreamSynchronize(ctx->side[i]);
  ctx->domains.clear();
  for (int i = 0; i < NUM_SIDE; i++) (void)hipStreamDestroy(ctx->side[i]);
  (void)hipStreamDestroy(ctx->stream);
  (void)hipEventDestroy(ctx->ev_scal);
  (void)hipEventDestroy(ctx->ev_quot);
  for (auto& e : ctx->ev_done) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ctx->ev_ic);
  delete ctx;
}

const char* zk_last_error(const zk_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int zk_ctx_profile(zk_ctx* ctx, int enable) {
  if (!ctx) return ZK_ERR_ARG;
  if (enable < 0 || enable > 2) return ZK_ERR_ARG;
  ctx->prof.on = enable != 0;
  ctx->prof.timeline = enable == 2;
  if (!enable) {
    ctx->prof.stats.clear();
    ctx->prof.tl.clear();
  }
  return ZK_OK;
}

int zk_ctx_timeline_read(zk_ctx* ctx, char* buf, size_t cap, size_t* len) {
  if (!ctx || !len) return ZK_ERR_ARG;
  const std::string& t = ctx->prof.tl;
  *len = t.size();
  if (buf && cap) {
    const size_t k = std::min(cap - 1, t.size());
    std::memcpy(buf, t.data(), k);
    buf[k] = 0;
    if (k == t.size()) ctx->prof.tl.clear();
  }
  return ZK_OK;
}

int zk_ctx_profile_read(zk_ctx* ctx, char* names, size_t names_cap, double* ms, uint64_t* launches,
                        uint64_t* units, size_t max_phases, size_t* nphases) {
  if (!ctx || !nphases) return ZK_ERR_ARG;
  size_t k = 0, off = 0;
  for (const auto& kv : ctx->prof.stats) {
    if (k < max_phases) {
      if (ms) ms[k] = kv.second.ms;
      if (launches) launches[k] = kv.second.launches;
      if (units) units[k] = kv.second.units;
      if (names && off + kv.first.size() + 1 < names_cap) {
        std::memcpy(names + off, kv.first.c_str(), kv.first.size() + 1);
        off += kv.first.size() + 1;
      }
    }
    k++;
  }
  if (names && off < names_cap) names[off] = 0;
  *nphases = k;
  return ZK_OK;
}

int zk_ctx_synchronize(zk_ctx* ctx) {
  if (!ctx) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { ZK_HIP(hipStreamSynchronize(ctx->stream)); return ZK_OK; })
}

// ------------------------------------------------------------------ MSM ---
// Scalars must be canonical Fr (< r, as ark's Fr always is) of at most
// scalar_bits bits; anything else is ZK_ERR_ARG rather than a silently
// different sum.
static bool scalar_ok(const zk_fr& a, uint32_t bits) {
  if (!fr_canonical(a)) return false;
  for (uint32_t w = 0; w < 4; w++) {
    const uint32_t lo = 64 * w;
    if (bits >= lo + 64) continue;
    const uint64_t allowed = bits <= lo ? 0 : (~0ull >> (64 - (bits - lo)));
    if (a.l[w] & ~allowed) return false;
  }
  return true;
}
// flags |= 1 when a device scalar is >= r or wider than bits
__global__ void __launch_bounds__(256) k_check_scalars(const uint64_t* __restrict__ sc, size_t n, uint32_t bits,
                                                       uint32_t* __restrict__ flags) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t l[4];
#pragma unroll
  for (int w = 0; w < 4; w++) l[w] = sc[4 * i + w];
  const uint64_t R[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                        0x73eda753299d7d48ull};
  bool lt = false, decided = false;
#pragma unroll
  for (int w = 3; w >= 0; w--) {
    if (!decided && l[w] != R[w]) { lt = l[w] < R[w]; decided = true; }
  }
  bool ok = lt;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t lo = 64 * w;
    if (bits >= lo + 64) continue;
    const uint64_t allowed = bits <= lo ? 0 : (~0ull >> (64 - (bits - lo)));
    ok = ok && !(l[w] & ~allowed);
  }
  if (!ok) atomicOr(flags, 1u);
}

template <class C, class ABI>
static int msm_host(zk_ctx* ctx, const ABI* bases, size_t nb, const zk_fr* sc, size_t ns, uint32_t bits,
                    ABI* out) {
  if (!ctx || !out) return ZK_ERR_ARG;
  if (nb != ns) return ZK_ERR_MSM_LEN;  // ark VariableBaseMSM::msm -> Err(min_len)
  if (bits == 0 || bits > 256 || nb > 0x7fffffffull) return ZK_ERR_ARG;
  for (size_t i = 0; i < ns; i++)
    if (!scalar_ok(sc[i], bits)) {
      ctx->err = "scalar " + std::to_string(i) + " is not a canonical Fr of at most scalar_bits bits";
      return ZK_ERR_ARG;
    }
  ZK_GUARD(ctx, {
    hipStream_t st = ctx->stream;
    const int sw = bits <= 64 ? 1 : 4;
    DevBuf raw, dev, scal;
    raw.ensure(sizeof(ABI) * std::max<size_t>(nb, 1));
    dev.ensure(sizeof(typename C::A) * std::max<size_t>(nb, 1));
    scal.ensure(sizeof(uint64_t) * sw * std::max<size_t>(nb, 1));
    if (nb) {
      ZK_HIP(hipMemcpyAsync(raw.p, bases, sizeof(ABI) * nb, hipMemcpyHostToDevice, st));
      if (sw == 4) {
        ZK_HIP(hipMemcpyAsync(scal.p, sc, sizeof(zk_fr) * nb, hipMemcpyHostToDevice, st));
      } else {
        ZK_HIP(hipMemcpy2DAsync(scal.p, 8, sc, sizeof(zk_fr), 8, nb, hipMemcpyHostToDevice, st));
      }
      convert_bases<C>(raw.as<uint64_t>(), dev.as<typename C::A>(), nb, st);
    }
    MsmWork& w = ctx->msm[0];
    msm_launch<C>(w, dev.as<typename C::A>(), scal.as<uint64_t>(), sw, (uint32_t)nb, sw == 1 ? 64 : 255, st);
    msm_download<C>(w, st);
    ZK_HIP(hipStreamSynchronize(st));
    ctx->prof.collect();
    host_to_abi<C>(msm_finish<C>(w), reinterpret_cast<uint64_t*>(out));
    return ZK_OK;
  })
}

int zk_msm_g1(zk_ctx* ctx, const zk_g1_affine* bases, size_t nb, const zk_fr* sc, size_t ns, uint32_t bits,
              zk_g1_affine* out) {
  return msm_host<G1>(ctx, bases, nb, sc, ns, bits, out);
}
int zk_msm_g2(zk_ctx* ctx, const zk_g2_affine* bases, size_t nb, const zk_fr* sc, size_t ns, uint32_t bits,
              zk_g2_affine* out) {
  return msm_host<G2>(ctx, bases, nb, sc, ns, bits, out);
}

// Window-shifted uploads (zk_msm_*_upload_windows): c = 16-bit digit windows,
// W = ceil(scalar_bits / c) copies 2^(c w) P of every base, so every
// later MSM of <= scalar_bits-bit scalars sums all its windows into ONE
// bucket set (msm_launch_shared; the prove path's trick, prove.hip).
// Window width c: 16 up to 64-bit scalars (4 windows, 2^15 buckets), 20 for
// wider ones -- 13 windows over 2^19 buckets instead of 16 over 2^15: the
// 2^20 full-width MSM 3.79-3.87 vs 3.92-4.01 ms; c = 18, 19, 22 lose
// (4.5-5.0 ms; profiles/r02_upload_win_sweep.txt).
// ZK_UPLOAD_WIN_C: A/B variant builds only (tools/build_variant.sh)
#ifndef ZK_UPLOAD_WIN_C
#define ZK_UPLOAD_WIN_C 20
#endif
static int upload_win_c(uint32_t win_bits) { return win_bits > 64 ? ZK_UPLOAD_WIN_C : 16; }

template <class C, class ABI>
static int msm_upload(zk_ctx* ctx, const ABI* bases, size_t n, int group, uint32_t win_bits, zk_msm_bases** out) {
  if (!ctx || !out) return ZK_ERR_ARG;
  if (win_bits > 256) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    std::unique_ptr<zk_msm_bases> b(new zk_msm_bases());
    b->device = ctx->device;
    b->group = group;
    b->n = n;
    const int MSM_UPLOAD_WIN_C = upload_win_c(win_bits);
    const int W = win_bits ? (int)((win_bits + MSM_UPLOAD_WIN_C - 1) / MSM_UPLOAD_WIN_C) : 1;
    if ((uint64_t)n * W >= 0x7fffffffull) throw Error(ZK_ERR_ARG, "msm: too many window bases");
    b->bases.ensure(sizeof(typename C::A) * std::max<size_t>(n * W, 1));
    DevBuf raw;
    raw.ensure(sizeof(ABI) * std::max<size_t>(n, 1));
    if (n) {
      ZK_HIP(hipMemcpyAsync(raw.p, bases, sizeof(ABI) * n, hipMemcpyHostToDevice, ctx->stream));
      convert_bases<C>(raw.as<uint64_t>(), b->bases.as<typename C::A>(), n, ctx->stream);
      if (W > 1) msm_precompute_windows<C>(b->bases.as<typename C::A>(), n, W, MSM_UPLOAD_WIN_C, ctx->stream);
      b->stride = msm_pad_bases<C>(b->bases, n * W, ctx->stream);
    }
    if (W > 1) {
      b->win = W;
      b->win_c = MSM_UPLOAD_WIN_C;
      b->win_bits = win_bits;
    }
    ZK_HIP(hipStreamSynchronize(ctx->stream));
    *out = b.release();
    return ZK_OK;
  })
}
int zk_msm_g1_upload(zk_ctx* ctx, const zk_g1_affine* bases, size_t n, zk_msm_bases** out) {
  return msm_upload<G1>(ctx, bases, n, 1, 0, out);
}
int zk_msm_g2_upload(zk_ctx* ctx, const zk_g2_affine* bases, size_t n, zk_msm_bases** out) {
  return msm_upload<G2>(ctx, bases, n, 2, 0, out);
}
int zk_msm_g1_upload_windows(zk_ctx* ctx, const zk_g1_affine* bases, size_t n, uint32_t scalar_bits,
                             zk_msm_bases** out) {
  return msm_upload<G1>(ctx, bases, n, 1, scalar_bits ? scalar_bits : 255, out);
}
int zk_msm_g2_upload_windows(zk_ctx* ctx, const zk_g2_affine* bases, size_t n, uint32_t scalar_bits,
                             zk_msm_bases** out) {
  return msm_upload<G2>(ctx, bases, n, 2, scalar_bits ? scalar_bits : 255, out);
}
void zk_msm_bases_free(zk_msm_bases* b) {
  if (!b) return;
  (void)hipSetDevice(b->device);
  delete b;
}

// Device scalars are canonical zk_fr (4 words).  64-bit mode reads the low
// word of each (stride 4) through a compaction into the ctx scratch.
__global__ void k_low_words(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[4 * i];
}

template <class C, class ABI>
static int msm_dev(zk_ctx* ctx, const zk_msm_bases* b, const void* d_sc, size_t n, uint32_t bits, ABI* out,
                   int group) {
  if (!ctx || !b || !out || b->group != group) return ZK_ERR_ARG;
  if (n != b->n) return ZK_ERR_MSM_LEN;
  if (bits == 0 || bits > 256) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    Range range("zk_msm_dev");
    hipStream_t st = ctx->stream;
    const uint64_t* sc = reinterpret_cast<const uint64_t*>(d_sc);
    ctx->flags.ensure(16);
    ctx->flags_host.ensure(16);
    ZK_HIP(hipMemsetAsync(ctx->flags.p, 0, 4, st));
    if (n) {
      k_check_scalars<<<ceil_div(n, 256), 256, 0, st>>>(sc, n, bits, ctx->flags.as<uint32_t>());
      ZK_LAUNCH_CHECK();
    }
    ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
    int sw = 4;
    if (bits <= 64) {
      ctx->tmp_scal.ensure(sizeof(uint64_t) * std::max<size_t>(n, 1));
      if (n) {
        k_low_words<<<ceil_div(n, 256), 256, 0, st>>>(sc, ctx->tmp_scal.as<uint64_t>(), n);
        ZK_LAUNCH_CHECK();
      }
      sc = ctx->tmp_scal.as<uint64_t>();
      sw = 1;
    }
    MsmWork& w = ctx->msm[0];
    const int mbits = sw == 1 ? 64 : 255;
    if (b->win > 1 && (uint32_t)mbits <= b->win_bits)   // one bucket set over the shifted copies
      msm_launch_shared<C>(w, b->bases.as<typename C::A>(), sc, sw, (uint32_t)n, mbits, b->win_c, st, b->stride);
    else
      msm_launch<C>(w, b->bases.as<typename C::A>(), sc, sw, (uint32_t)n, mbits, st, b->stride);
    msm_download<C>(w, st);
    ZK_HIP(hipStreamSynchronize(st));
    ctx->prof.collect();
    if (*ctx->flags_host.as<uint32_t>()) {
      ctx->err = "a device scalar is not a canonical Fr of at most scalar_bits bits";
      return ZK_ERR_ARG;
    }
    host_to_abi<C>(msm_finish<C>(w), reinterpret_cast<uint64_t*>(out));
    return ZK_OK;
  })
}
int zk_msm_g1_dev(zk_ctx* ctx, const zk_msm_bases* b, const void* d_sc, size_t n, uint32_t bits,
                  zk_g1_affine* out) {
  return msm_dev<G1>(ctx, b, d_sc, n, bits, out, 1);
}
int zk_msm_g2_dev(zk_ctx* ctx, const zk_msm_bases* b, const void* d_sc, size_t n, uint32_t bits,
                  zk_g2_affine* out) {
  return msm_dev<G2>(ctx, b, d_sc, n, bits, out, 2);
}

// ------------------------------------------------------------------ NTT ---
// The transform runs on the canonical values as they are: with twiddles in
// Montgomery form w R, a butterfly's fp_mul(v, w R) = v w, so canonical data
// stay canonical through every pass and no to/from-Montgomery pass is needed.
// Natural order in and out (ntt_natural: DIT passes, the first gathering its
// tile from the bit-reversed positions).  Every input element is checked to
// be a canonical Fr (ark's Fr is always reduced) in that first pass's load:
// a flag, read after the transform, turns into ZK_ERR_ARG (the data are then
// unspecified).  The caller synchronises.
static int ntt_device(zk_ctx* ctx, void* d_data, uint32_t log_n, int dir, const zk_fr* coset) {
  Range range("zk_ntt");
  hipStream_t st = ctx->stream;
  const size_t n = (size_t)1 << log_n;
  if (coset && !fr_canonical(*coset)) return ZK_ERR_ARG;
  ctx->flags.ensure(16);
  ctx->flags_host.ensure(16);
  ZK_HIP(hipMemsetAsync(ctx->flags.p, 0, 4, st));
  uint32_t* chk = ctx->flags.as<uint32_t>();
  auto flag_result = [&]() {
    ZK_HIP(hipMemcpyAsync(ctx->flags_host.p, ctx->flags.p, 4, hipMemcpyDeviceToHost, st));
    ZK_HIP(hipStreamSynchronize(st));
    if (*ctx->flags_host.as<uint32_t>()) {
      ctx->err = "an NTT input element is not a canonical Fr (>= r)";
      return (int)ZK_ERR_ARG;
    }
    return (int)ZK_OK;
  };
  if (log_n == 0) {   // a size-1 DFT (and its coset / inverse) is the identity
    check_canonical(d_data, 1, chk, st);
    return flag_result() == ZK_OK ? ZK_OK : ZK_ERR_ARG;
  }
  NttDomain& dom = ctx->domain(log_n);
  ctx->tmp_fr.ensure(sizeof(Fr) * 2 * n);
  Fr* a = ctx->tmp_fr.as<Fr>();
  Fr* b = a + n;
  Fr* d = reinterpret_cast<Fr*>(d_data);
  auto to_dev = [](const host::Fr& h) { Fr x; const host::Fr v = host::fr_to_dev(h); std::memcpy(x.v, v.l, 32); return x; };
  const host::Fr one = host::fr_one();
  const host::Fr ninv = host::fr_inv(host::fr_from_u64(n));
  // natural -> natural (ntt_natural: the bit reversal is the first pass's gather)
  if (dir > 0) {
    const Fr* ltab = nullptr;
    if (coset) {                                   // a_i *= g^i, fused into the first pass's load
      fr_powers(b, to_dev(host::fr_to_mont(coset->l)), to_dev(one), n, st);
      ltab = b;
    }
    ntt_natural(d, d, a, dom, false, st, &ctx->prof, ltab, nullptr, nullptr, chk);
  } else if (coset) {                              // out_i *= n^-1 g^-i, fused into the last pass's store
    host::Fr g = host::fr_to_mont(coset->l);
    if (host::fr_is_zero(g)) return ZK_ERR_ARG;
    fr_powers(b, to_dev(host::fr_inv(g)), to_dev(ninv), n, st);
    ntt_natural(d, d, a, dom, true, st, &ctx->prof, nullptr, b, nullptr, chk);
  } else {
    const Fr c = to_dev(ninv);
    ntt_natural(d, d, a, dom, true, st, &ctx->prof, nullptr, nullptr, &c, chk);
  }
  return flag_result();
}

int zk_ntt_fr_dev(zk_ctx* ctx, void* d_data, uint32_t log_n, int dir, const zk_fr* coset) {
  if (!ctx || (dir != 1 && dir != -1)) return ZK_ERR_ARG;
  if (log_n > 32) return ZK_ERR_DOMAIN;
  ZK_GUARD(ctx, {
    int rc = ntt_device(ctx, d_data, log_n, dir, coset);
    ZK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->prof.collect();
    return rc;
  })
}

int zk_ntt_fr(zk_ctx* ctx, zk_fr* data, uint32_t log_n, int dir, const zk_fr* coset) {
  if (!ctx || !data || (dir != 1 && dir != -1)) return ZK_ERR_ARG;
  if (log_n > 32) return ZK_ERR_DOMAIN;
  ZK_GUARD(ctx, {
    const size_t n = (size_t)1 << log_n;
    DevBuf d;
    d.ensure(sizeof(zk_fr) * n);
    ZK_HIP(hipMemcpyAsync(d.p, data, sizeof(zk_fr) * n, hipMemcpyHostToDevice, ctx->stream));
    int rc = ntt_device(ctx, d.p, log_n, dir, coset);
    ZK_HIP(hipMemcpyAsync(data, d.p, sizeof(zk_fr) * n, hipMemcpyDeviceToHost, ctx->stream));
    ZK_HIP(hipStreamSynchronize(ctx->stream));
    return rc;
  })
}

// ---------------------------------------------------------------- setup ---
int zk_groth16_setup(zk_ctx* ctx, const zk_r1cs_csr* qap, const zk_setup_params* params, uint64_t num_public,
                     zk_pk* pk, zk_vk* vk) {
  if (!ctx || !qap || !params || !pk || !vk) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return setup_impl(ctx, qap, params, num_public, 0, 1, pk, nullptr, vk); })
}
int zk_groth16_setup_dev(zk_ctx* ctx, const zk_r1cs_csr* qap, const zk_setup_params* params, uint64_t num_public,
                         zk_pk_dev** out, zk_vk* vk) {
  if (!ctx || !qap || !params || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return setup_impl(ctx, qap, params, num_public, 0, 1, nullptr, out, vk); })
}
int zk_groth16_setup_dev_shard(zk_ctx* ctx, const zk_r1cs_csr* qap, const zk_setup_params* params,
                               uint64_t num_public, uint32_t shard, uint32_t nshards, zk_pk_dev** out) {
  if (!ctx || !qap || !params || !out || nshards == 0 || shard >= nshards) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return setup_impl(ctx, qap, params, num_public, shard, nshards, nullptr, out, nullptr); })
}

// ---------------------------------------------------------------- prove ---
int zk_pk_upload(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* qap, zk_pk_dev** out) {
  if (!ctx || !pk || !qap || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    *out = pk_upload(ctx, pk, qap, 0, 1);
    return ZK_OK;
  })
}
int zk_pk_upload_shard(zk_ctx* ctx, const zk_pk* pk, const zk_r1cs_csr* qap, uint32_t shard, uint32_t nshards,
                       zk_pk_dev** out) {
  if (!ctx || !pk || !qap || !out || nshards == 0 || shard >= nshards) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    *out = pk_upload(ctx, pk, qap, shard, nshards);
    return ZK_OK;
  })
}
void zk_pk_free(zk_pk_dev* pk) {
  if (!pk) return;
  (void)hipSetDevice(pk->device);
  delete pk;
}

int zk_groth16_prove_dev(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, size_t zlen, size_t num_public,
                         const zk_fr* r, const zk_fr* s, zk_proof* out) {
  if (!ctx || !pk || !d_z || !r || !s || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return prove_impl(ctx, pk, d_z, zlen, num_public, r, s, out); })
}

int zk_groth16_prove(zk_ctx* ctx, const zk_pk_dev* pk, const zk_fr* z, size_t zlen, size_t num_public,
                     const zk_fr* r, const zk_fr* s, zk_proof* out) {
  if (!ctx || !pk || !z || !r || !s || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    // the witness crosses PCIe in two parts inside the prove, the first
    // part's MSMs overlapping the second part's copy (prove.hip)
    ctx->z_canon.ensure(sizeof(zk_fr) * std::max<size_t>(zlen, 1));
    if (zlen != pk->V) return prove_impl(ctx, pk, ctx->z_canon.p, zlen, num_public, r, s, out);   // the length error
    return prove_impl(ctx, pk, ctx->z_canon.p, zlen, num_public, r, s, out, z);
  })
}

int zk_groth16_prove_partial(zk_ctx* ctx, const zk_pk_dev* pk, const void* d_z, size_t zlen, size_t num_public,
                             const zk_fr* r, const zk_fr* s, zk_prove_partial* out) {
  if (!ctx || !pk || !d_z || !r || !s || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return prove_partial_impl(ctx, pk, d_z, zlen, num_public, r, s, out); })
}

int zk_groth16_prove_combine(const zk_prove_partial* parts, size_t nparts, const zk_fr* r, const zk_fr* s,
                             zk_proof* out) {
  if (!parts || !nparts || !r || !s || !out) return ZK_ERR_ARG;
  try {
    return combine_impl(parts, nparts, r, s, out);
  } catch (...) {
    return ZK_ERR_DEVICE;
  }
}

int zk_rccl_unique_id(uint8_t out[128]) {
  if (!out) return ZK_ERR_ARG;
  try {
    rccl_unique_id(out);
    return ZK_OK;
  } catch (const Error& e) {
    return e.code;
  } catch (...) {
    return ZK_ERR_RCCL;
  }
}

int zk_ctx_attach_rccl(zk_ctx* ctx, const uint8_t unique_id[128], int rank, int world) {
  if (!ctx || !unique_id || world < 1 || rank < 0 || rank >= world) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    ctx->exch.reset();
    ctx->exch = make_rccl_exchange(unique_id, rank, world, ctx->exch_timeout_ms);
    return ZK_OK;
  })
}

int zk_ctx_detach_exchange(zk_ctx* ctx) {
  if (!ctx) return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    if (ctx->exch) {
      // the exchange is dropped whatever the stream's state: after a GPU
      // fault (a likely reason to detach) the wait fails, and keeping the
      // exchange would leave this rank's peers to meet it in a collective
      const hipError_t e = hipStreamSynchronize(ctx->stream);
      ctx->exch->detach();
      ctx->exch.reset();
      if (e != hipSuccess) throw Error(ZK_ERR_DEVICE, std::string("detach: stream wait: ") + hipGetErrorString(e));
    }
    return ZK_OK;
  })
}

int zk_ctx_attach_exchange(zk_ctx* ctx, const zk_exchange_ops* ops, int rank, int world) {
  if (!ctx || !ops || !ops->all_to_all || !ops->all_reduce_max || world < 1 || rank < 0 || rank >= world)
    return ZK_ERR_ARG;
  ZK_GUARD(ctx, {
    ctx->exch.reset();
    ctx->exch = make_host_exchange(*ops, rank, world);
    ctx->exch->timeout_ms = ctx->exch_timeout_ms;
    return ZK_OK;
  })
}

int zk_groth16_witness_ranges(zk_ctx* ctx, const zk_pk_dev* pk, uint64_t* ranges, size_t cap, size_t* nranges) {
  if (!ctx || !pk || !nranges || (cap && !ranges)) return ZK_ERR_ARG;
  const std::vector<uint64_t> w = witness_ranges(ctx, pk);
  *nranges = w.size() / 2;
  for (size_t k = 0; k < std::min(cap, w.size() / 2); k++) {
    ranges[2 * k] = w[2 * k];
    ranges[2 * k + 1] = w[2 * k + 1];
  }
  return ZK_OK;
}

int zk_groth16_prove_partial_host(zk_ctx* ctx, const zk_pk_dev* pk, const zk_fr* z_slice, size_t slice_len,
                                  size_t zlen, size_t num_public, const zk_fr* r, const zk_fr* s,
                                  zk_prove_partial* out) {
  if (!ctx || !pk || !r || !s || !out) return ZK_ERR_ARG;
  ZK_GUARD(ctx, { return prove_partial_host_impl(ctx, pk, z_slice, slice_len, zlen, num_public, r, s, out); })
}

int zk_proof_serialize_compressed(const zk_proof* proof, uint8_t out[192]) {
  if (!proof || !out) return ZK_ERR_ARG;
  serialize_g1_compressed(proof->a, out);
  serialize_g2_compressed(proof->b, out + 48);
  serialize_g1_compressed(proof->c, out + 144);
  return ZK_OK;
}

