// group.hip -- bucket grouping of the prove path's MSM entries without a
// general radix sort (msm.hpp step 2, shared / batch plans with <= 16-bit
// bucket ids and <= 4 windows: every prove MSM at c = 16).
//
// The accumulate needs the (point, window) entries grouped by bucket and
// the first entry of every bucket (off[]); the order inside a bucket does
// not matter (its entries are summed, and the group element is unique), so
// this is a two-level counting sort keyed on the 16-bit bucket id (+ the
// batch segment):
//   count    per tile of 2048 points: the digits computed from the scalars,
//            an LDS histogram of the coarse bin (bucket >> FINE_BITS), one
//            column per tile (segment-major, then coarse bin, then tile);
//   scan     one exclusive scan of those columns (rocPRIM): the first global
//            position of every (coarse bin, tile);
//   scatter  the same tiles again: entries ranked by coarse bin in LDS,
//            staged there, then written out as contiguous runs per bin;
//   fine     one workgroup per coarse bin (~8 K entries at 2^20): an LDS
//            histogram of the fine bits, the bucket offsets written
//            directly, then each entry moved to its bucket's range inside
//            the bin (a 64-KB window of L2).
// The keys are never materialised before grouping and nothing re-reads them
// globally: against rocPRIM's onesweep (keys pass + histogram + two 9-bit
// passes + offsets pass), ~32 instead of ~50 bytes per entry.
#include <rocprim/device/device_scan.hpp>

#include "msm.hpp"

namespace zk {

constexpr uint32_t GRP_TP = 2048;              // points per tile
constexpr uint32_t GRP_THREADS = 256;
constexpr uint32_t GRP_FB = 7;                 // fine bits
constexpr uint32_t GRP_NF = 1u << GRP_FB;      // fine bins per coarse bin
constexpr uint32_t GRP_KB = 16;                // bucket bits of the plans this path takes
constexpr uint32_t GRP_NC = 1u << (GRP_KB - GRP_FB);   // coarse bins per segment (512)
constexpr uint32_t GRP_U = 8;                  // entries per thread per batch (fine pass)

struct GrpArgs {
  const uint64_t* sc[MSM_MAXSEG];
  uint32_t n[MSM_MAXSEG], wstride[MSM_MAXSEG], ioff[MSM_MAXSEG];
  uint32_t blk0[MSM_MAXSEG + 1];    // first tile of segment k
  uint32_t ebase[MSM_MAXSEG + 1];   // first entry of segment k
  uint32_t nseg, nwin, c, bits, kb;
};

ZK_DI uint32_t grp_seg(const GrpArgs& a, uint32_t blk) {
  uint32_t k = 0;
#pragma unroll
  for (uint32_t j = 1; j < MSM_MAXSEG; j++)
    if (j < a.nseg && blk >= a.blk0[j]) k = j;
  return k;
}

// Entry (point i of segment k, window w): its local bucket id (0 for a zero
// digit, whose entry is the dummy) and its entry word, as k_msm_keys makes them
// for shared plans.
template <class F>
ZK_DI void grp_entries(const GrpArgs& a, uint32_t k, uint32_t i, uint64_t s, F&& f) {
  uint32_t carry = 0;
  const uint32_t half = 1u << (a.c - 1);
  for (uint32_t w = 0; w < a.nwin; w++) {
    const bool top = w == a.nwin - 1;
    const uint32_t off = a.c * w, width = top ? a.bits - off : a.c;
    const uint32_t v = (uint32_t)((s >> off) & ((1ull << width) - 1)) + carry;
    uint32_t mag;
    bool neg = false;
    if (!top && v > half) {
      mag = (1u << a.c) - v;
      neg = true;
      carry = 1;
    } else {
      mag = v;
      carry = 0;
    }
    const uint32_t b = w * a.wstride[k] + a.ioff[k] + i;
    f(mag ? mag - 1 : 0u, mag ? (b | (neg ? 0x80000000u : 0u)) : MSM_DUMMY, w);
  }
}
// The tile's points i0 + threadIdx.x + GRP_THREADS j (GRP_TP / GRP_THREADS of
// them per thread): every scalar load is issued before the first digit is
// used, so the loads overlap instead of each waiting out its own latency.
constexpr uint32_t GRP_PPT = GRP_TP / GRP_THREADS;
template <class F>
ZK_DI void grp_tile(const GrpArgs& a, uint32_t k, uint32_t i0, uint32_t i1, F&& f) {
  uint64_t s[GRP_PPT];
#pragma unroll
  for (uint32_t j = 0; j < GRP_PPT; j++) {
    const uint32_t i = i0 + threadIdx.x + GRP_THREADS * j;
    s[j] = i < i1 ? a.sc[k][i] : 0ull;
  }
#pragma unroll
  for (uint32_t j = 0; j < GRP_PPT; j++) {
    const uint32_t i = i0 + threadIdx.x + GRP_THREADS * j;
    if (i < i1) grp_entries(a, k, i, s[j], f);
  }
}

__global__ void __launch_bounds__(GRP_THREADS) k_grp_count(GrpArgs a, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t hist[GRP_NC];
  const uint32_t blk = blockIdx.x, k = grp_seg(a, blk), lb = blk - a.blk0[k];
  const uint32_t nb = a.blk0[k + 1] - a.blk0[k];
  for (uint32_t t = threadIdx.x; t < GRP_NC; t += GRP_THREADS) hist[t] = 0;
  __syncthreads();
  const uint32_t i0 = lb * GRP_TP, i1 = min(i0 + GRP_TP, a.n[k]);
  grp_tile(a, k, i0, i1, [&](uint32_t key, uint32_t, uint32_t) { atomicAdd(&hist[key >> GRP_FB], 1u); });
  __syncthreads();
  const uint32_t base = GRP_NC * a.blk0[k];   // segment k's columns start here
  for (uint32_t t = threadIdx.x; t < GRP_NC; t += GRP_THREADS) cnt[base + t * nb + lb] = hist[t];
}

// Exclusive scan of GRP_NC values in LDS (GRP_THREADS threads, 2 each).
ZK_DI void grp_scan_nc(uint32_t* v, uint32_t* tmp) {
  static_assert(GRP_NC == 2 * GRP_THREADS, "two bins per thread");
  const uint32_t t = threadIdx.x;
  const uint32_t a0 = v[2 * t], a1 = v[2 * t + 1];
  tmp[t] = a0 + a1;
  __syncthreads();
  for (uint32_t d = 1; d < GRP_THREADS; d <<= 1) {   // inclusive Hillis-Steele over the pair sums
    const uint32_t x = t >= d ? tmp[t - d] : 0u;
    __syncthreads();
    tmp[t] += x;
    __syncthreads();
  }
  const uint32_t ex = tmp[t] - (a0 + a1);
  v[2 * t] = ex;
  v[2 * t + 1] = ex + a0;
  __syncthreads();
}

__global__ void __launch_bounds__(GRP_THREADS) k_grp_scatter(GrpArgs a, const uint32_t* __restrict__ cnt,
                                                             const uint32_t* __restrict__ cnt_off,
                                                             uint32_t* __restrict__ tkey, uint32_t* __restrict__ tent) {
  __shared__ uint32_t lbase[GRP_NC], lcur[GRP_NC], gbase[GRP_NC], stmp[GRP_THREADS];
  __shared__ uint32_t skey[GRP_TP * 4], sent[GRP_TP * 4];   // nwin <= 4: 64 KB staging
  const uint32_t blk = blockIdx.x, k = grp_seg(a, blk), lb = blk - a.blk0[k];
  const uint32_t nb = a.blk0[k + 1] - a.blk0[k];
  const uint32_t base = GRP_NC * a.blk0[k];
  for (uint32_t t = threadIdx.x; t < GRP_NC; t += GRP_THREADS) lbase[t] = cnt[base + t * nb + lb];
  __syncthreads();
  grp_scan_nc(lbase, stmp);
  for (uint32_t t = threadIdx.x; t < GRP_NC; t += GRP_THREADS) {
    lcur[t] = lbase[t];
    gbase[t] = cnt_off[base + t * nb + lb] - lbase[t];   // global position of local slot 0 of bin t
  }
  __syncthreads();
  // rank by coarse bin (LDS atomics: order inside a bin is arbitrary) and stage
  const uint32_t i0 = lb * GRP_TP, i1 = min(i0 + GRP_TP, a.n[k]);
  const uint32_t kbase = k << a.kb;
  grp_tile(a, k, i0, i1, [&](uint32_t key, uint32_t e, uint32_t) {
    const uint32_t s = atomicAdd(&lcur[key >> GRP_FB], 1u);
    skey[s] = kbase | key;
    sent[s] = e;
  });
  __syncthreads();
  // contiguous runs per bin: local slot j of bin t lands at gbase[t] + j
  const uint32_t ne = (i1 > i0 ? i1 - i0 : 0) * a.nwin;
  const uint32_t kmask = (1u << a.kb) - 1;
  for (uint32_t j = threadIdx.x; j < ne; j += GRP_THREADS) {
    const uint32_t key = skey[j];
    const uint32_t g = gbase[(key & kmask) >> GRP_FB] + j;
    tkey[g] = key;
    tent[g] = sent[j];
  }
}

__global__ void __launch_bounds__(GRP_THREADS) k_grp_fine(GrpArgs a, const uint32_t* __restrict__ cnt_off,
                                                          const uint32_t* __restrict__ tkey,
                                                          const uint32_t* __restrict__ tent, uint32_t* __restrict__ key,
                                                          uint32_t* __restrict__ ent, uint32_t* __restrict__ off,
                                                          uint32_t G) {
  __shared__ uint32_t fcur[GRP_NF];
  const uint32_t h = blockIdx.x, k = h / GRP_NC, cb = h % GRP_NC;
  const uint32_t nb = a.blk0[k + 1] - a.blk0[k];
  const uint32_t base = GRP_NC * a.blk0[k];
  uint32_t S, E;
  if (nb == 0) {
    S = E = a.ebase[k];
  } else {
    S = cnt_off[base + cb * nb];
    E = cb + 1 < GRP_NC ? cnt_off[base + (cb + 1) * nb] : a.ebase[k + 1];
  }
  for (uint32_t t = threadIdx.x; t < GRP_NF; t += GRP_THREADS) fcur[t] = 0;
  __syncthreads();
  // batches of GRP_U entries per thread: their loads in flight together
  constexpr uint32_t U = GRP_U;
  for (uint32_t e0 = S; e0 < E; e0 += U * GRP_THREADS) {
    uint32_t kk[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t e = e0 + threadIdx.x + GRP_THREADS * u;
      kk[u] = e < E ? tkey[e] : 0xffffffffu;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (kk[u] != 0xffffffffu) atomicAdd(&fcur[kk[u] & (GRP_NF - 1)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 64) {   // exclusive scan of the 128 fine counts: one wave, 2 each
    const uint32_t t = threadIdx.x, c0 = fcur[2 * t], c1 = fcur[2 * t + 1];
    uint32_t incl = c0 + c1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(incl, d);
      if (t >= (uint32_t)d) incl += x;
    }
    const uint32_t ex = S + incl - (c0 + c1);
    fcur[2 * t] = ex;
    fcur[2 * t + 1] = ex + c0;
    const uint32_t g0 = (k << a.kb) | (cb << GRP_FB) | (2 * t);
    off[g0] = ex;
    off[g0 + 1] = ex + c0;
  }
  if (h == 0 && threadIdx.x == 0) off[G] = a.ebase[a.nseg];
  __syncthreads();
  for (uint32_t e0 = S; e0 < E; e0 += U * GRP_THREADS) {
    uint32_t kk[U], ee[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t e = e0 + threadIdx.x + GRP_THREADS * u;
      kk[u] = e < E ? tkey[e] : 0xffffffffu;
      ee[u] = e < E ? tent[e] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      if (kk[u] == 0xffffffffu) continue;
      const uint32_t pos = atomicAdd(&fcur[kk[u] & (GRP_NF - 1)], 1u);
      key[pos] = kk[u];
      ent[pos] = ee[u];
    }
  }
}

bool msm_group_ok(const MsmPlan& p, int sw) {
  return p.shared && sw == 1 && p.nwin <= 4 && (uint32_t)(p.kr[0] + p.kc[0]) == GRP_KB && p.nseg >= 1 &&
         p.nseg <= MSM_MAXSEG;
}

void msm_group(MsmWork& w, const MsmSeg* segs, int nseg, hipStream_t st) {
  const MsmPlan& p = w.plan;
  GrpArgs a{};
  a.nseg = (uint32_t)nseg;
  a.nwin = (uint32_t)p.nwin;
  a.c = (uint32_t)p.c;
  a.bits = (uint32_t)p.bits;
  a.kb = GRP_KB;
  uint32_t blk = 0, e = 0;
  for (int k = 0; k < nseg; k++) {
    a.sc[k] = segs[k].scalars;
    a.n[k] = segs[k].n;
    a.wstride[k] = segs[k].wstride ? segs[k].wstride : segs[k].n;
    a.ioff[k] = segs[k].ioff;
    a.blk0[k] = blk;
    a.ebase[k] = e;
    blk += ceil_div(segs[k].n, GRP_TP);
    e += segs[k].n * (uint32_t)p.nwin;
  }
  for (int k = nseg; k <= MSM_MAXSEG; k++) {
    a.blk0[k] = blk;
    a.ebase[k] = e;
  }
  const size_t ncnt = (size_t)GRP_NC * blk;
  w.gcnt.ensure(sizeof(uint32_t) * std::max<size_t>(ncnt, 1));
  w.gcnt_off.ensure(sizeof(uint32_t) * std::max<size_t>(ncnt, 1));
  if (blk) {
    k_grp_count<<<blk, GRP_THREADS, 0, st>>>(a, w.gcnt.as<uint32_t>());
    ZK_LAUNCH_CHECK();
    size_t tmp_bytes = 0;
    ZK_HIP(rocprim::exclusive_scan(nullptr, tmp_bytes, w.gcnt.as<uint32_t>(), w.gcnt_off.as<uint32_t>(), 0u, ncnt,
                                   rocprim::plus<uint32_t>(), st));
    w.sort_tmp.ensure(std::max<size_t>(tmp_bytes, 1));
    ZK_HIP(rocprim::exclusive_scan(w.sort_tmp.p, tmp_bytes, w.gcnt.as<uint32_t>(), w.gcnt_off.as<uint32_t>(), 0u,
                                   ncnt, rocprim::plus<uint32_t>(), st));
    k_grp_scatter<<<blk, GRP_THREADS, 0, st>>>(a, w.gcnt.as<uint32_t>(), w.gcnt_off.as<uint32_t>(),
                                                w.key_in.as<uint32_t>(), w.ent_in.as<uint32_t>());
    ZK_LAUNCH_CHECK();
  }
  k_grp_fine<<<(uint32_t)nseg * GRP_NC, GRP_THREADS, 0, st>>>(a, w.gcnt_off.as<uint32_t>(), w.key_in.as<uint32_t>(),
                                                               w.ent_in.as<uint32_t>(), w.key.as<uint32_t>(),
                                                               w.ent.as<uint32_t>(), w.off.as<uint32_t>(), p.G);
  ZK_LAUNCH_CHECK();
}

}  // namespace zk
