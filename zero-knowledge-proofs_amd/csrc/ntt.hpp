// ntt.hpp -- radix-2 NTT over BLS12-381 Fr on gfx950.
//
// Replaces ark-poly 0.4.2 Radix2EvaluationDomain::{fft, ifft} and the coset
// variants as used by QAP::from_r1cs (crates/groth16-qap/src/lib.rs:101,
// 167-169) and by DensePolynomial mul / divide_by_vanishing_poly inside
// compute_quotient_polynomial (qap:260-263).  Same domain generator as ark:
// omega_n = (7^((r-1)/2^32))^(2^(32 - log n)).
//
// Layout: Fr elements are 32 B (8 x u32 Montgomery limbs), contiguous.
// Four-step (recursive) structure: a pass loads a tile of 2^ns rows x C
// consecutive columns into LDS (<= 1024 elements = 32 KiB), runs the
// 2^ns-point sub-transform down its columns with twiddles from a small
// cached table, and applies the inter-level twiddles once per element, so
// log n stages cost ~log n / 10 HBM round trips and no per-butterfly
// gathers from an n/2-entry table.  DIF passes take natural order to
// bit-reversed order, DIT passes the reverse, so the quotient pipeline
// (iNTT -> coset NTT -> divide -> coset iNTT) never needs a standalone
// permutation except once, fused into its final gather.
#pragma once
#include "common.hpp"
#include "ff.hpp"

namespace zk {

// Per-domain constant tables, built on device once and cached by the ctx.
// A sub-transform twiddle pre-cut into the product's 9 x 29-bit limbs (the
// multiply then unpacks only the data operand); 48 B = three 16-B loads.
struct FrU {
  uint32_t l[FrParams::NL];
  uint32_t pad[12 - FrParams::NL];
};

struct NttDomain {
  uint32_t log_n = 0;
  DevBuf sm, ism;   // omega_2048^j, j < 1024 (and inverse): sub-transform twiddles
  DevBuf smu, ismu; // the same as FrU (pre-cut limbs)
  DevBuf tl, itl;   // omega_n^x, x < min(n, 4096)
  DevBuf th, ith;   // omega_n^(4096 y), y < n / 4096
  DevBuf ts, its;   // omega_S^e, e < S = 2^min(16, log n) (log n > 12): cache-resident direct twiddles
  uint32_t ts_log = 0;
  DevBuf zinv;    // (g^n - 1)^-1: 1/Z on the coset g<w>
  // n-entry coset tables, built on first use only (n x 32 B each: 512 MB at
  // 2^24), so API-only transforms build none and each quotient path builds
  // the ones it reads -- single GPU: gpow_br + gipow, distributed: gpow + gipow
  DevBuf gpow;    // n^-1 * g^i, i < n   (coset shift g = 7)
  DevBuf gpow_br; // gpow in bit-reversed order: read contiguously by the quotient's coset shift
  DevBuf gipow;   // n^-1 * g^-i, i < n
};

void ntt_domain_init(NttDomain& d, uint32_t log_n, hipStream_t st);
const Fr* domain_gpow(NttDomain& d, hipStream_t st);
const Fr* domain_gpow_br(NttDomain& d, hipStream_t st);
const Fr* domain_gipow(NttDomain& d, hipStream_t st);

constexpr int NTT_SM_LOG = 11;    // sub-transform twiddles: powers of omega_2048 (domain-independent)
constexpr int NTT_TL_LOG = 12;    // omega_n^x = TL[x mod 4096] * TH[x / 4096]
#ifndef ZK_NTT_TS_LOG
#define ZK_NTT_TS_LOG 16
#endif
constexpr uint32_t NTT_TS_LOG = ZK_NTT_TS_LOG;   // direct pass-twiddle table: 2^16 x 32 B = 2 MB (A/B: 0 = none)

// a (8 little-endian u32 limbs, as stored) < r: a canonical Fr
ZK_DI bool fr_lt_r(const Fr& a) {
  uint32_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) (void)__builtin_subc(a.v[k], FrParams::MOD[k], br, &br);
  return br != 0;   // a - r borrowed
}

ZK_DI uint32_t bitrev32(uint32_t x, uint32_t log_n) {
  return log_n ? (__builtin_bitreverse32(x) >> (32 - log_n)) : 0;
}

struct NttTabs {
  const Fr* sm;   // omega_2048^j, j < 1024 (or the inverse root)
  const FrU* smu; // sm pre-cut into limbs
  const Fr* tl;   // omega_n^x, x < min(n, 4096)
  const Fr* th;   // omega_n^(4096 y), y < n / 4096
  const Fr* ts;   // omega_S^e, e < S = 2^ts_log (nullptr: none)
  uint32_t ts_log;
};

// The inter-level twiddle of a pass over blocks of N = 2^logN elements:
// omega_N^x, x < N.  With N <= S it is ONE load from the direct table
// (omega_S^(x 2^(ts_log - logN)): 2 MB at S = 2^16, L2-resident), else
// TL x TH below (RED = false: < 2r, not canonical).
template <bool RED = true>
ZK_DI Fr tw_pass(const NttTabs& t, uint32_t x, uint32_t logN, uint32_t log_n);
// omega_n^x, x < n (RED = false: < 2r, not canonical)
template <bool RED = true>
ZK_DI Fr tw_full(const NttTabs& t, uint32_t x, uint32_t log_n) {
  Fr w = ld_vec(&t.tl[x & ((1u << NTT_TL_LOG) - 1)]);
  if (log_n > NTT_TL_LOG) w = fp_mul<FrParams, RED>(w, ld_vec(&t.th[x >> NTT_TL_LOG]));
  return w;
}

template <bool RED>
ZK_DI Fr tw_pass(const NttTabs& t, uint32_t x, uint32_t logN, uint32_t log_n) {
  if (t.ts && logN <= t.ts_log) return ld_vec(&t.ts[x << (t.ts_log - logN)]);
  return tw_full<RED>(t, x << (log_n - logN), log_n);
}

inline NttTabs tabs_of(const NttDomain& dom, bool inv) {
  return inv ? NttTabs{dom.ism.as<Fr>(), dom.ismu.as<FrU>(), dom.itl.as<Fr>(), dom.ith.as<Fr>(), dom.its.as<Fr>(),
                       dom.ts_log}
             : NttTabs{dom.sm.as<Fr>(), dom.smu.as<FrU>(), dom.tl.as<Fr>(), dom.th.as<Fr>(), dom.ts.as<Fr>(),
                       dom.ts_log};
}


// In-place passes over n Montgomery Fr; nb > 1: nb transforms back to back
// in d_data (n apart), every pass one launch for all of them.
// ntt_dif's first pass may read `src` instead of d_data (out of place) and
// multiply each loaded element by ltab[i] (natural index), e.g. a coset's g^i.
void ntt_dif(Fr* d_data, const NttDomain& dom, bool inverse_twiddles, hipStream_t st, Prof* pf = nullptr,
             const Fr* src = nullptr, const Fr* ltab = nullptr, uint32_t nb = 1);
void ntt_dit(Fr* d_data, const NttDomain& dom, bool inverse_twiddles, hipStream_t st, Prof* pf = nullptr,
             uint32_t nb = 1);
// Natural order in (src) and out (dst), the API transform: DIT passes whose
// first pass gathers from bit-reversed positions; ltab: factor on the input
// (natural index), stab / scale: factor on the output.  tmp: n elements of
// scratch (src may equal dst).  chk: when given, *chk |= 1 if some input
// element is not a canonical Fr (checked in the first pass's load).
void ntt_natural(Fr* dst, const Fr* src, Fr* tmp, const NttDomain& dom, bool inverse_twiddles, hipStream_t st,
                 Prof* pf, const Fr* ltab, const Fr* stab, const Fr* scale, uint32_t* chk = nullptr);

// d <- NTT(tab_br[p] * iNTT(d)) with the inverse DIF's last pass, the
// scale and the forward DIT's first pass fused into one tile kernel (the
// quotient's coefficients -> coset evaluations step).  tab_br is the factor
// table in bit-reversed order (NttDomain::gpow_br: n^-1 g^bitrev(p)), so the
// tile reads it contiguously instead of gathering 32-B words across n.
void ntt_coset_shift(Fr* d_data, const NttDomain& dom, const Fr* d_tab_br, hipStream_t st, Prof* pf = nullptr,
                     uint32_t nb = 1);
// Elementwise helpers
void fr_to_mont(const uint64_t* d_canon, Fr* d_out, size_t n, hipStream_t st);
void fr_from_mont(const Fr* d_in, uint64_t* d_canon, size_t n, hipStream_t st);
// data[p] *= tab[bitrev(p)] (bitrev over log_n bits)  or  tab[p] when !bitrev;
// nb transforms of 2^log_n back to back, the same table for each
void fr_scale_table(Fr* d_data, const Fr* d_tab, uint32_t log_n, bool bitrev, hipStream_t st, uint32_t nb = 1);
// out[i] = in[bitrev(i)] (out-of-place)
void fr_bitrev_copy(const Fr* d_in, Fr* d_out, uint32_t log_n, hipStream_t st);
// out[bitrev(i)] = in[i] * f, f = tab[bitrev(i)] (tab != nullptr), else c
// (use_c), else 1: the natural-order permutation after a DIF transform,
// tiled through LDS so reads and writes stay coalesced (log_n >= 10)
void fr_bitrev_scale(const Fr* d_in, Fr* d_out, uint32_t log_n, const Fr* tab, const Fr* c, hipStream_t st);
// data[i] *= c (Montgomery constant)
void fr_scale_const(Fr* d_data, const Fr& c_host, size_t n, hipStream_t st);
// out[i] = base^i * scale (Montgomery), i < n
void fr_powers(Fr* d_out, const Fr& base, const Fr& scale, size_t n, hipStream_t st);

}  // namespace zk
