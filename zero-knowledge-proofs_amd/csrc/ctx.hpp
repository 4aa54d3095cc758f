// ctx.hpp -- zk_ctx (one GPU: streams, cached NTT domains, MSM workspaces)
// and zk_pk_dev (a proving key resident in HBM).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "dist.hpp"
#include "msm.hpp"
#include "ntt.hpp"

namespace zk {

constexpr int NUM_MSM = 5;  // pi_A (G1), pi_B (G2), B1 (G1), IC (G1), H (G1)
constexpr int NUM_SIDE = 3; // side streams (+ main = 4 = GPU_MAX_HW_QUEUES)
// Parts of a host witness upload (zk_groth16_prove): part k's MSMs run while
// part k+1 is still crossing PCIe (pk_part_cuts).
#ifndef ZK_HOST_PARTS
#define ZK_HOST_PARTS 2
#endif
constexpr int HOST_PARTS = ZK_HOST_PARTS;
static_assert(HOST_PARTS >= 2 && HOST_PARTS <= 6, "host witness parts");
enum MsmSlot { MSM_A = 0, MSM_B2 = 1, MSM_B1 = 2, MSM_IC = 3, MSM_H = 4 };

// Device copy of the constraint matrices (the QAP in sparse form).
struct CsrDev {
  uint64_t nc = 0, V = 0;
  DevBuf rp[3], col[3], val[3];
  bool unit[3] = {false, false, false};
};

}  // namespace zk

struct zk_ctx {
  int device = 0;
  hipStream_t stream = nullptr;                 // main stream
  hipStream_t side[zk::NUM_SIDE] = {};          // G2 / IC / A+B1 MSM streams
  hipEvent_t ev_scal = nullptr;                 // witness checked (flags reset)
  hipEvent_t ev_quot = nullptr;                 // quotient done (ZK_OPT_EXCHANGE_FIRST)
  hipEvent_t ev_done[zk::NUM_MSM] = {};         // per-MSM completion (results downloaded)
  hipEvent_t ev_ic = nullptr;                   // IC's scalars gathered (side stream)
  std::string err;
  zk::MsmWork msm[zk::NUM_MSM];
  // the G2 and A+B1+IC MSMs' workspaces for every part of a host witness
  // upload but the last (which uses msm[]): buckets, keys and sort scratch
  // of each part stay allocated, ~60 MB per part at 2^20 constraints (c = 16)
  // and ~2 GB at 2^24 (c = 22: 2^21 buckets per MSM)
  zk::MsmWork part_g2[zk::HOST_PARTS - 1], part_abi[zk::HOST_PARTS - 1];
  std::map<uint32_t, std::unique_ptr<zk::NttDomain>> domains;
  // prove scratch
  zk::DevBuf z_canon, qabc, flags;   // qabc: the quotient's A, B, C vectors back to back (3n)
  zk::PinnedBuf flags_host;
  zk::DevBuf scal[zk::NUM_MSM];
  zk::DevBuf tmp_scal, tmp_fr;
  zk::Prof prof;
  std::unique_ptr<zk::Exchange> exch;          // RCCL communicator (sharded prover), if attached
  zk::DistQ dq;                                // distributed-quotient buffers
  // Explicit choices (zk_ctx_set_schedule / zk_ctx_set_option); never read
  // from the environment, and no proof depends on them.
  int sched = 0;                               // 0 overlapped streams, 3 serial (per-kernel timing)
  int quot_path = -1;                          // -1 by domain size, 0 small-domain, 1 large-domain
  int prove_win_c = 0;                         // 0 by size, else 16 or 22 (keys made after the call)
  double exch_timeout_ms = 60000;              // watchdog of an attached exchange
  int dist_quotient = -1;                      // -1 distributed when an exchange of the key's shape
                                               // is attached, 0 never (each rank the whole quotient)
  int exchange_first = 0;                      // 1: distributed proofs run the quotient before the MSMs

  zk::NttDomain& domain(uint32_t log_n);
};

struct zk_pk_dev {
  int device = 0;
  uint64_t V = 0, n = 0, nc = 0, num_public = 0;
  uint32_t log_n = 0;
  uint32_t shard = 0, nshards = 1;
  zk::CsrDev csr;
  // Compacted non-identity bases (device Montgomery affine) followed by the
  // shard-0 extras, and the variable index feeding each base's scalar.
  zk::DevBuf bases[zk::NUM_MSM];
  zk::DevBuf idx[zk::NUM_MSM];      // u32 variable index per compacted base (H: coefficient index)
  uint32_t count[zk::NUM_MSM] = {};  // compacted bases (without extras)
  uint32_t extras[zk::NUM_MSM] = {}; // extra bases appended (shard 0 only)
  // Window-shifted base copies (msm_precompute_windows): bases[slot] holds
  // win x (count + extras) points, window w = 2^(win_c w) x the base.
  // The IC and H vectors are ONE MSM of the prove (both terms of pi_C):
  // bases[MSM_H] holds win x (count[IC] + count[H]) points, each window the
  // IC bases then the H bases (ich_tot() per window), and bases[MSM_IC] is
  // empty once the windows are built.
  int win = 1, win_c = 0;
  uint32_t ich_tot() const { return count[zk::MSM_IC] + extras[zk::MSM_IC] + count[zk::MSM_H] + extras[zk::MSM_H]; }
  // idx[MSM_H][k] == k for every compacted H base (an unsharded key without
  // identity H bases): the local quotient then writes lo64(H_i) straight
  // into the IC+H scalar vector and no gather follows it
  bool h_ident = false;
  // Bytes between consecutive bases of bases[slot]: 0 = packed (sizeof the
  // affine point), else padded to whole 128-B lines (msm_pad_bases).
  uint32_t stride[zk::NUM_MSM] = {};
  // [lo, hi) pairs: the z entries this shard reads with a distributed
  // quotient (zk_groth16_witness_ranges); without one it reads all of z
  std::vector<uint64_t> wr_dist;
  // Host-witness prove (zk_groth16_prove): z crosses PCIe in HOST_PARTS
  // parts, variables [vcut[k], vcut[k+1]); pcut[k][slot] = compacted bases
  // whose variable is < vcut[k], so part k's MSMs run while part k+1 is still
  // in flight (pk_part_cuts).
  uint64_t vcut[zk::HOST_PARTS + 1] = {};
  uint32_t pcut[zk::HOST_PARTS + 1][zk::NUM_MSM] = {};
};

namespace zk {
// Expand every slot's bases into the window-shifted copies the shared-bucket
// MSM reads.
void pk_precompute_windows(zk_ctx* ctx, zk_pk_dev& pk);
// canonical-input checks (prove.hip): a < r on the host; on the device,
// flags |= 8 when some of the n canonical Fr at d_z is >= r
bool fr_canonical(const zk_fr& a);
void check_canonical(const void* d_z, uint64_t n, uint32_t* d_flags, hipStream_t st);
// vcut and pcut of a finished key (device binary search over its idx vectors)
void pk_part_cuts(zk_pk_dev& pk, hipStream_t st);
// the witness ranges of a finished key (its idx vectors and shard) from the
// host constraint matrices: fills pk.wr_dist
// (own: var_owner of the key's shape; its variables owned by this shard
// are added, so every z entry is read -- and checked canonical -- by some rank)
void pk_witness_ranges(zk_pk_dev& pk, const zk_r1cs_csr* q, const std::vector<uint8_t>& own, hipStream_t st);
// Which shard holds variable v's A / B1 / B2 / IC bases: with a distributed
// quotient possible (nshards 2, 4 or 8, n % nshards^2 == 0) the shard whose
// quotient rows first reference v, so a rank's MSM variables are the ones
// its quotient rows read anyway and its witness slice is ~1/nshards of z;
// unreferenced variables by contiguous range.  Empty: contiguous ranges of
// every base vector.
std::vector<uint8_t> var_owner(const zk_r1cs_csr* q, uint64_t n, uint32_t nshards);
}

struct zk_msm_bases {
  int device = 0;
  int group = 1;  // 1 = G1, 2 = G2
  size_t n = 0;
  zk::DevBuf bases;   // n points, or win x n window-shifted copies (window-major)
  int win = 1, win_c = 0;
  uint32_t win_bits = 0;   // scalars up to this width use the shared bucket set
  uint32_t stride = 0;     // bytes between bases (0 = packed), see msm_pad_bases
};
