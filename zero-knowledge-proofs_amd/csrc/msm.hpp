// msm.hpp -- Pippenger bucket MSM over BLS12-381 G1 / G2 on gfx950.
//
// Replaces G1Projective::msm / G2Projective::msm (ark-ec 0.4.2
// VariableBaseMSM) as called by Prover::multi_scalar_mult_g1/g2,
// crates/groth16-core/src/lib.rs:275-300.  The result is the unique group
// element sum_i k_i P_i, so the algorithm may differ from ark's while the
// normalised affine output is bit-identical.
//
// Pipeline per MSM (all on one HIP stream, workspace reused):
//   1 count    signed c-bit window digits, bucket histogram (global atomics)
//   2 scan     exclusive scan of bucket counts -> bucket offsets
//   3 scatter  (point index | sign) entries grouped by bucket (counting sort)
//   4 accum    fixed K entries per thread, XYZZ += affine, run-length flush:
//              load-balanced whatever the digit distribution
//   5 fixup    buckets split across threads: sum the <= 2 partials per thread
//   6 reduce1  per (window, L-bucket segment) running sums -> S_j, W_j
//   7 reduce2  per window: sum_j W_j and U_b = sum_{j: bit b of j} S_j
//   host tail  sum_w 2^(c w) (sum W + L sum_b 2^b U_b): one Horner pass over
//              the ~nwin*(Q) partials (latency-bound; see host_ec.hpp)
#pragma once
#include "common.hpp"
#include "curve.hpp"
#include "host_ec.hpp"

#include <vector>

namespace zk {

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

struct MsmPlan {
  int c, nwin, bits, sw;           // window bits, #windows, scalar bits, u64 words/scalar
  int L, K, Q;                     // reduce segment, accumulate chunk, reduce2 quantities
  uint32_t n;                      // points
  uint32_t G;                      // total buckets
  uint32_t T;                      // total reduce segments
  uint32_t nb[MSM_MAXWIN];         // buckets in window w (digits 1..nb)
  uint32_t boff[MSM_MAXWIN + 1];   // first global bucket id of window w
  uint32_t segoff[MSM_MAXWIN + 1]; // first reduce segment of window w
};

MsmPlan msm_make_plan(uint32_t n, int bits, int sw, int force_c = 0);

// Device workspace of one in-flight MSM.
struct MsmWork {
  DevBuf counts, off, cursor, ent, key, buckets, partials, segS, segW, res;
  std::vector<uint8_t> host_res;
  MsmPlan plan{};
};

// Launch the device part of an MSM over n Montgomery-affine device bases and
// n scalars of `sw` u64 words each (canonical little-endian, < 2^bits).
template <class C>
void msm_launch(MsmWork& w, const typename C::A* d_bases, const uint64_t* d_scalars, int sw,
                uint32_t n, int bits, hipStream_t st);
// Copy the per-window partials back (async) -- call msm_finish after a sync.
template <class C>
void msm_download(MsmWork& w, hipStream_t st);
// Host tail: combine the window partials into sum k_i P_i (host XYZZ).
template <class C>
host::X<typename C::HF> msm_finish(const MsmWork& w);

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
