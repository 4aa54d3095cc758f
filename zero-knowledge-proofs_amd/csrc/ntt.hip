// ntt.hip -- LDS-tiled radix-2 NTT passes over Fr (see ntt.hpp).
#include <algorithm>

#include "ntt.hpp"

namespace zk {

constexpr int NTT_TILE_LOG = 11;  // 2048 elements x 32 B = 64 KiB of LDS per workgroup
constexpr int NTT_THREADS = 256;

__device__ __forceinline__ uint32_t bitrev32(uint32_t x, uint32_t log_n) {
  return log_n ? (__builtin_bitreverse32(x) >> (32 - log_n)) : 0;
}

// One pass: stages s_lo .. s_lo+ns-1 on tiles of 2^ns rows x C columns.
// Element (tile hi, row r, column lo) lives at i = hi*2^(s_lo+ns) + r*2^s_lo + lo.
template <bool DIT>
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_pass(Fr* __restrict__ data, const Fr* __restrict__ tw,
                                                          uint32_t log_n, uint32_t s_lo, uint32_t ns,
                                                          uint32_t logC) {
  extern __shared__ Fr sh[];
  const uint32_t C = 1u << logC;
  const uint32_t rows = 1u << ns;
  const uint32_t tile_elems = rows << logC;
  const uint32_t lo_blocks = (1u << s_lo) >> logC;      // column blocks per hi
  const uint32_t tile = blockIdx.x;
  const uint32_t hi = tile / lo_blocks;
  const uint32_t lo0 = (tile % lo_blocks) << logC;
  const size_t base = ((size_t)hi << (s_lo + ns)) + lo0;

  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) {
    const uint32_t r = k >> logC, c = k & (C - 1);
    sh[k] = ld_vec(&data[base + ((size_t)r << s_lo) + c]);
  }
  __syncthreads();

  const uint32_t nbf = tile_elems >> 1;
  for (uint32_t st = 0; st < ns; st++) {
    const uint32_t ls = DIT ? st : ns - 1 - st;    // local stage
    const uint32_t s = s_lo + ls;                   // global stage: pairs (i, i + 2^s)
    const uint32_t tw_shift = log_n - 1 - s;
    for (uint32_t b = threadIdx.x; b < nbf; b += NTT_THREADS) {
      const uint32_t c = b & (C - 1), rb = b >> logC;
      const uint32_t r = ((rb >> ls) << (ls + 1)) | (rb & ((1u << ls) - 1));
      const uint32_t k0 = (r << logC) | c, k1 = k0 + (1u << (ls + logC));
      // exponent: (i mod 2^s) * n / 2^(s+1)
      const uint32_t im = ((r & ((1u << ls) - 1)) << s_lo) | (lo0 + c);
      const Fr w = ld_vec(&tw[(size_t)im << tw_shift]);
      Fr u = sh[k0], v = sh[k1];
      if (DIT) {
        v = fp_mul(v, w);
        sh[k0] = fp_add(u, v);
        sh[k1] = fp_sub(u, v);
      } else {
        sh[k0] = fp_add(u, v);
        sh[k1] = fp_mul(fp_sub(u, v), w);
      }
    }
    __syncthreads();
  }
  for (uint32_t k = threadIdx.x; k < tile_elems; k += NTT_THREADS) {
    const uint32_t r = k >> logC, c = k & (C - 1);
    st_vec(&data[base + ((size_t)r << s_lo) + c], sh[k]);
  }
}

static void run_pass(bool dit, Fr* d, const Fr* tw, uint32_t log_n, uint32_t s_lo, uint32_t ns,
                     hipStream_t st) {
  const uint32_t logC = std::min<uint32_t>(s_lo, std::min<uint32_t>(2, NTT_TILE_LOG - ns));
  const uint32_t tiles = (uint32_t)((1ull << log_n) >> (ns + logC));
  const size_t lds = sizeof(Fr) << (ns + logC);
  if (dit)
    k_ntt_pass<true><<<tiles, NTT_THREADS, lds, st>>>(d, tw, log_n, s_lo, ns, logC);
  else
    k_ntt_pass<false><<<tiles, NTT_THREADS, lds, st>>>(d, tw, log_n, s_lo, ns, logC);
  ZK_LAUNCH_CHECK();
}

// Stage grouping: up to 9 stages per pass while columns can be batched 4-wide
// (coalesced 128 B rows), up to 11 in the final stride-1 pass.
static uint32_t pass_stages(uint32_t s_lo, uint32_t remaining) {
  uint32_t cap = s_lo >= 2 ? NTT_TILE_LOG - 2 : NTT_TILE_LOG - s_lo;
  return std::min(cap, remaining);
}

void ntt_dif(Fr* d, const NttDomain& dom, bool inv, hipStream_t st, Prof* pf) {
  const uint32_t L = dom.log_n;
  if (L == 0) return;
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)1 << L) : -1;
  const Fr* tw = (inv ? dom.itw : dom.tw).as<Fr>();
  // stages L-1 .. 0, top-down: choose pass sizes so that the last pass (s_lo = 0) is widest
  uint32_t s_hi = L;  // exclusive
  while (s_hi > 0) {
    uint32_t ns = std::min<uint32_t>(s_hi, NTT_TILE_LOG);
    uint32_t s_lo = s_hi - ns;
    if (s_lo > 0) {               // a strided pass: at most 9 stages, and leave >= 0
      ns = std::min<uint32_t>(ns, NTT_TILE_LOG - 2);
      s_lo = s_hi - ns;
    }
    run_pass(false, d, tw, L, s_lo, ns, st);
    s_hi = s_lo;
  }
  if (pf) pf->end(st, ph);
}

void ntt_dit(Fr* d, const NttDomain& dom, bool inv, hipStream_t st, Prof* pf) {
  const uint32_t L = dom.log_n;
  if (L == 0) return;
  const int ph = pf ? pf->begin(st, "ntt", (uint64_t)1 << L) : -1;
  const Fr* tw = (inv ? dom.itw : dom.tw).as<Fr>();
  uint32_t s_lo = 0;
  while (s_lo < L) {
    uint32_t ns = pass_stages(s_lo, L - s_lo);
    run_pass(true, d, tw, L, s_lo, ns, st);
    s_lo += ns;
  }
  if (pf) pf->end(st, ph);
}

// ------------------------------------------------------------ tables -----
__device__ __forceinline__ Fr fr_pow_u64(Fr b, uint64_t e) {
  Fr acc = fp_one<FrParams>();
  while (e) {
    if (e & 1) acc = fp_mul(acc, b);
    b = fp_mul(b, b);
    e >>= 1;
  }
  return acc;
}

constexpr int POW_CHUNK = 64;
__global__ void __launch_bounds__(256) k_powers(Fr* __restrict__ out, Fr base, Fr scale, size_t n) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i0 = t * POW_CHUNK;
  if (i0 >= n) return;
  Fr x = fp_mul(scale, fr_pow_u64(base, i0));
  const size_t e = min(i0 + POW_CHUNK, n);
  for (size_t i = i0; i < e; i++) {
    st_vec(&out[i], x);
    x = fp_mul(x, base);
  }
}

void fr_powers(Fr* d_out, const Fr& base, const Fr& scale, size_t n, hipStream_t st) {
  if (!n) return;
  const size_t thr = (n + POW_CHUNK - 1) / POW_CHUNK;
  k_powers<<<ceil_div(thr, 256), 256, 0, st>>>(d_out, base, scale, n);
  ZK_LAUNCH_CHECK();
}

static Fr fr_const(const uint32_t (&c)[8]) {
  Fr r;
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
  return r;
}

// Z(g w^i) = g^n - 1 on the whole coset; Fermat inverse, one thread, once per domain.
__global__ void k_coset_zinv(Fr* out, uint32_t log_n) {
  Fr g;
#pragma unroll
  for (int i = 0; i < 8; i++) g.v[i] = FR_GEN[i];
  for (uint32_t k = 0; k < log_n; k++) g = fp_mul(g, g);
  g = fp_sub(g, fp_one<FrParams>());
  uint32_t e[8];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = __builtin_subc(FrParams::MOD[i], i == 0 ? 2u : 0u, br, &br);
  Fr acc = fp_one<FrParams>();
#pragma unroll
  for (int i = 7; i >= 0; i--)
    for (int k = 31; k >= 0; k--) {
      acc = fp_mul(acc, acc);
      if ((e[i] >> k) & 1) acc = fp_mul(acc, g);
    }
  *out = acc;
}

void ntt_domain_init(NttDomain& d, uint32_t log_n, hipStream_t st) {
  d.log_n = log_n;
  const size_t n = (size_t)1 << log_n;
  const size_t half = std::max<size_t>(n / 2, 1);
  d.tw.ensure(sizeof(Fr) * half);
  d.itw.ensure(sizeof(Fr) * half);
  d.gpow.ensure(sizeof(Fr) * n);
  d.gipow.ensure(sizeof(Fr) * n);
  Fr one = fr_const(FrParams::ONE);
  Fr ninv = fr_const(FR_INV_2K[log_n]);
  fr_powers(d.tw.as<Fr>(), fr_const(FR_ROOTS[log_n]), one, half, st);
  fr_powers(d.itw.as<Fr>(), fr_const(FR_ROOTS_INV[log_n]), one, half, st);
  fr_powers(d.gpow.as<Fr>(), fr_const(FR_GEN), ninv, n, st);
  fr_powers(d.gipow.as<Fr>(), fr_const(FR_GEN_INV), ninv, n, st);
  d.zinv.ensure(sizeof(Fr));
  k_coset_zinv<<<1, 1, 0, st>>>(d.zinv.as<Fr>(), log_n);
  ZK_LAUNCH_CHECK();
}

// -------------------------------------------------------- elementwise ---
__global__ void __launch_bounds__(256) k_to_mont(const uint64_t* __restrict__ in, Fr* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr a = ld_vec(reinterpret_cast<const Fr*>(in) + i);
  st_vec(&out[i], fp_to_mont(a));
}
__global__ void __launch_bounds__(256) k_from_mont(const Fr* __restrict__ in, uint64_t* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_vec(reinterpret_cast<Fr*>(out) + i, fp_from_mont(ld_vec(&in[i])));
}
__global__ void __launch_bounds__(256) k_scale_table(Fr* __restrict__ d, const Fr* __restrict__ tab,
                                                     uint32_t log_n, bool bitrev) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >> log_n) return;
  const size_t j = bitrev ? bitrev32((uint32_t)p, log_n) : p;
  st_vec(&d[p], fp_mul(ld_vec(&d[p]), ld_vec(&tab[j])));
}
__global__ void __launch_bounds__(256) k_bitrev_copy(const Fr* __restrict__ in, Fr* __restrict__ out, uint32_t log_n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >> log_n) return;
  st_vec(&out[i], ld_vec(&in[bitrev32((uint32_t)i, log_n)]));
}
__global__ void __launch_bounds__(256) k_scale_const(Fr* __restrict__ d, Fr c, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_vec(&d[i], fp_mul(ld_vec(&d[i]), c));
}

void fr_to_mont(const uint64_t* d_canon, Fr* d_out, size_t n, hipStream_t st) {
  if (!n) return;
  k_to_mont<<<ceil_div(n, 256), 256, 0, st>>>(d_canon, d_out, n);
  ZK_LAUNCH_CHECK();
}
void fr_from_mont(const Fr* d_in, uint64_t* d_canon, size_t n, hipStream_t st) {
  if (!n) return;
  k_from_mont<<<ceil_div(n, 256), 256, 0, st>>>(d_in, d_canon, n);
  ZK_LAUNCH_CHECK();
}
void fr_scale_table(Fr* d, const Fr* tab, uint32_t log_n, bool bitrev, hipStream_t st) {
  k_scale_table<<<ceil_div((size_t)1 << log_n, 256), 256, 0, st>>>(d, tab, log_n, bitrev);
  ZK_LAUNCH_CHECK();
}
void fr_bitrev_copy(const Fr* in, Fr* out, uint32_t log_n, hipStream_t st) {
  k_bitrev_copy<<<ceil_div((size_t)1 << log_n, 256), 256, 0, st>>>(in, out, log_n);
  ZK_LAUNCH_CHECK();
}
void fr_scale_const(Fr* d, const Fr& c, size_t n, hipStream_t st) {
  if (!n) return;
  k_scale_const<<<ceil_div(n, 256), 256, 0, st>>>(d, c, n);
  ZK_LAUNCH_CHECK();
}

}  // namespace zk
