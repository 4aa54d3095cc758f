// msm.hpp -- Pippenger bucket MSM over BLS12-381 G1 / G2 on gfx950.
//
// Replaces G1Projective::msm / G2Projective::msm (ark-ec 0.4.2
// VariableBaseMSM) as called by Prover::multi_scalar_mult_g1/g2,
// crates/groth16-core/src/lib.rs:275-300.  The result is the unique group
// element sum_i k_i P_i, so the algorithm may differ from ark's while the
// normalised affine output is bit-identical.
//
// Pipeline per MSM (one HIP stream; workspace reused across calls):
//   1 keys     signed c-bit window digits -> one (bucket, point | sign) pair
//              per (point, window), computed inside step 2's first pass
//   2 group    stable LSD counting sort of the pairs by bucket (group.hip),
//              then bucket offsets
//   4 accum    the M non-zero digits split evenly over one full-occupancy
//              round of threads, XYZZ += affine with run-length flush:
//              load-balanced whatever the digit distribution
//   5 merge    buckets split across chunks: log-depth segmented merge of
//              the per-chunk open pieces (k_msm_merge)
//   6 rowcol   window w's nb = 2^(kr+kc) buckets seen as a 2^kr x 2^kc grid,
//              bucket m = hi*2^kc + lo has weight m+1 = hi*2^kc + lo + 1, so
//              sum_m (m+1) B_m = 2^kc sum_hi hi C_hi + sum_lo (lo+1) D_lo with
//              C = row sums, D = column sums: 2 nb plain adds, tree depth 8
//   7 quant    U^C_b = sum_{hi: bit b} C_hi, U^D_b = sum_{lo: bit b} D_lo,
//              P = sum_lo D_lo: one masked tree (depth <= 8) per quantity
//   host tail  sum_w 2^(c w) (2^kc sum_b 2^b U^C_b + sum_b 2^b U^D_b + P):
//              one Horner pass over ~16 nwin partials (latency-bound; see
//              host_ec.hpp for why this tail runs on the host)
#pragma once
#include <string>
#include <vector>

#include "common.hpp"
#include "curve.hpp"
#include "host_ec.hpp"

namespace zk {

// Bits [off, off + width) of a little-endian scalar of SW u64 words.
template <int SW>
__device__ __forceinline__ uint32_t scal_window(const uint64_t (&s)[SW], int off, int width) {
  int wd = off >> 6, sh = off & 63;
  uint64_t lo = 0;
#pragma unroll
  for (int k = 0; k < SW; k++)
    if (k == wd) lo = s[k] >> sh;
  if (sh + width > 64) {
#pragma unroll
    for (int k = 0; k < SW; k++)
      if (k == wd + 1) lo |= s[k] << (64 - sh);
  }
  return (uint32_t)(lo & ((1ull << width) - 1));
}

struct G1 {
  using F = Fq;
  using A = G1A;
  using X = G1X;
  using HF = host::Fq;
  static constexpr int ABI_WORDS = 13;  // zk_g1_affine
};
struct G2 {
  using F = Fq2;
  using A = G2A;
  using X = G2X;
  using HF = host::Fq2;
  static constexpr int ABI_WORDS = 25;  // zk_g2_affine
};

constexpr int MSM_MAXWIN = 64;
constexpr uint32_t MSM_DUMMY = 0x7fffffffu;   // entry that contributes nothing (a zero digit)

struct MsmPlan {
  int c, nwin, bits, sw;            // window bits, #windows, scalar bits, u64 words/scalar
  uint32_t T;                       // accumulate threads (chunk = ceil(M / T) on device)
  uint32_t fix_max;                 // buckets over <= fix_max chunks: serial fixup, else merge
  uint32_t n;                       // points
  uint32_t G;                       // total buckets
  uint32_t nrc, nq;                 // total row/col sums, total quantities
  uint32_t nb[MSM_MAXWIN];          // buckets in window w (digits 1..nb), a power of two
  uint32_t boff[MSM_MAXWIN + 1];    // first global bucket id of window w
  uint8_t kr[MSM_MAXWIN], kc[MSM_MAXWIN];   // nb = 2^(kr + kc): rows x columns
  // each row sum is 2^lsr partial sums over consecutive column ranges, each
  // column sum 2^lsc over consecutive row ranges (msm_split_sums): rc holds
  // row i's partial s at i 2^lsr + s, then the columns likewise
  uint8_t lsr[MSM_MAXWIN], lsc[MSM_MAXWIN];
  uint32_t rcoff[MSM_MAXWIN + 1];   // first row/col partial sum of window w (rows, then columns)
  uint32_t qoff[MSM_MAXWIN + 1];    // first quantity of window w (U^C, U^D, P)
  uint32_t nred;                    // reduction windows (nwin, or 1 when shared, or nseg)
  int shared;                       // windows share one bucket set (precomputed 2^(c w) P bases)
  int nseg;                         // batch: independent MSMs, reduction window k = MSM k
  uint32_t segshift;                // batch: bucket g belongs to MSM g >> segshift
  int all_valid;                    // every bucket holds a value (msm_batch_back COMBINE wrote them all)
};

// One MSM of a batch (msm_launch_batch): n points, window-shifted bases
// (nwin x n, window-major) and n one-word scalars.
constexpr int MSM_MAXSEG = 4;
struct MsmSeg {
  const void* bases;
  const uint64_t* scalars;
  uint32_t n;
  uint32_t stride = 0;   // bytes between bases (0 = sizeof the affine point)
  // a sub-range of a window-shifted base vector: point i of the segment is
  // base ioff + i, and window w of it sits at w wstride + ioff + i (wstride
  // 0 = n: the segment is the whole vector)
  uint32_t wstride = 0, ioff = 0;
};

MsmPlan msm_make_plan(uint32_t n, int bits, int sw, int force_c = 0);
// Bucket grouping (group.hip): the (point, window) entries of the segments'
// scalars (sw u64 words each), sorted stably by bucket into w.key / w.ent,
// w.off[g] = first entry of bucket g (g <= G), and the merge's control
// words w.nbig zeroed.  Deterministic: the same inputs give the same bytes.
struct MsmWork;
struct MsmSeg;
void msm_group(MsmWork& w, const MsmSeg* segs, int nseg, int sw, hipStream_t st);
// w.off[] from the sorted w.key[0, M) (and w.nbig zeroed)
void msm_offsets(MsmWork& w, uint32_t M, hipStream_t st);
// Window-shared plan: digit window w of point i uses the precomputed base
// 2^(c w) P_i (msm_precompute_windows), so every window accumulates into
// ONE set of 2^max(c-1, top) buckets -- the bucket reduction shrinks by the
// window count and the per-window Horner disappears.
MsmPlan msm_make_plan_shared(uint32_t n, int bits, int sw, int c);

// Device workspace of one in-flight MSM.
struct MsmWork {
  DevBuf off, ent, key, buckets, partials, partials2, rc, res;
  DevBuf key_in, ent_in;             // grouping: the other half of its ping-pong
  DevBuf nbig;                       // control words: merge count, its grid barrier
  DevBuf gcnt, gcnt_sums;            // grouping (group.hip): per-tile digit counts / their scan, chunk sums
  PinnedBuf host_res;
  MsmPlan plan{};
  Prof* prof = nullptr;  // optional live kernel timing
  std::string tag;      // phase-name prefix (per-MSM profiling)
};

// Launch the device part of an MSM over n Montgomery-affine device bases and
// n scalars of `sw` u64 words each (canonical little-endian, < 2^bits).
template <class C>
void msm_launch(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw,
                uint32_t n, int bits, hipStream_t st, uint32_t stride = 0);
// Same over window-shifted bases: d_bases holds nwin x n points, window-major.
template <class C>
void msm_launch_shared(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw,
                       uint32_t n, int bits, int c, hipStream_t st, uint32_t stride = 0);
// Up to MSM_MAXSEG independent MSMs over window-shifted bases with 64-bit
// scalars, run as ONE key pass / sort / accumulate / merge / bucket
// reduction: MSM k owns buckets [k 2^s, (k+1) 2^s).  The latency-bound
// phases (merge, row/column sums, quantities) then cost one tree depth for
// the whole batch instead of one per MSM.  msm_finish_seg(w, k) gives MSM k.
template <class C>
void msm_launch_batch(MsmWork& w, const MsmSeg* segs, int nseg, int bits, int c, hipStream_t st);
// The same in two halves, for an MSM whose points arrive in parts: the
// front (keys, sort, accumulate) and the back (bucket fixup / merge, then
// the bucket reduction).  back modes: MSM_BACK_FULL (msm_launch_batch),
// MSM_BACK_FIXUP (complete the buckets only: the first part of a split MSM),
// MSM_BACK_ACCUM (complete the buckets and add the completed buckets of
// `prev` -- an earlier part over the same plan, already past its own back on
// this stream -- into every bucket: a middle part) and MSM_BACK_COMBINE (the
// same, then reduce: the last part, the sum of all parts).
enum { MSM_BACK_FULL = 0, MSM_BACK_FIXUP = 1, MSM_BACK_COMBINE = 2, MSM_BACK_ACCUM = 3 };
template <class C>
void msm_batch_front(MsmWork& w, const MsmSeg* segs, int nseg, int bits, int c, hipStream_t st);
template <class C>
void msm_batch_back(MsmWork& w, hipStream_t st, int mode, const MsmWork* prev);
// d_bases[w n + i] = 2^(c w) d_bases[i] for 0 < w < W (the first n are given;
// capacity W n).  One-time, at proving-key upload.
template <class C>
void msm_precompute_windows(typename C::A* d_bases, size_t n, int W, int c, hipStream_t st);
// Base gathers by the accumulate are random: a packed 96-B G1 point straddles
// two 128-B lines half the time (192-B G2: always 2-3 lines).  Padding each
// point to whole lines (G1 128 B, G2 256 B) makes every gather exactly one
// (two) line(s).  Returns the new stride in bytes; `d` is replaced by the
// padded copy of its n points.
template <class C>
uint32_t msm_pad_bases(DevBuf& d, size_t n, hipStream_t st);
// XYZZ -> affine for n points with one Fermat inversion per 16-point chunk
// (pre: n field elements of scratch).
template <class C>
void batch_normalize(const typename C::X* d_in, size_t n, typename C::F* d_pre, typename C::A* d_out,
                     hipStream_t st);
// Copy the per-window partials back (async) -- call msm_finish after a sync.
template <class C>
void msm_download(MsmWork& w, hipStream_t st);
// Host tail: combine the window partials into sum k_i P_i (host XYZZ).
template <class C>
host::X<typename C::HF> msm_finish(const MsmWork& w);
// Host tail of MSM `seg` of a batch.
template <class C>
host::X<typename C::HF> msm_finish_seg(const MsmWork& w, int seg);

// canonical ABI points -> device Montgomery affine ((0,0) = infinity)
template <class C>
void convert_bases(const uint64_t* d_abi_words, typename C::A* d_out, size_t n, hipStream_t st);
// gather variant: d_out[k] = convert(abi[idx[k]])
template <class C>
void convert_bases_gather(const uint64_t* d_abi_words, const uint32_t* d_idx, typename C::A* d_out,
                          size_t n, hipStream_t st);

// host XYZZ -> canonical ABI words
template <class C>
void host_to_abi(const host::X<typename C::HF>& p, uint64_t* words);

}  // namespace zk
