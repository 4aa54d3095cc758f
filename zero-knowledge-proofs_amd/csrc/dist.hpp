// dist.hpp -- the QAP quotient distributed over the ranks of a sharded
// prover, with RCCL all-to-all over xGMI as its exchange.
//
// With N ranks and domain n = N m, every transform of the quotient
// (3 iNTT + 3 coset NTT + 1 coset iNTT, qap:225-271) is a four-step
// n = N x m transform: size-N DFTs down the columns of an N x m matrix,
// a twiddle omega_n^(b k1), then size-m DFTs along its rows.  Rank r owns
// one column slice for the first half and row r for the second, so each
// transform needs ONE all-to-all, the three A/B/C pipelines share theirs,
// and the whole quotient costs three exchanges of m elements per rank
// instead of every rank recomputing the size-n quotient.  The witness and
// the constraint matrices are replicated, so every rank evaluates the
// rows of its column slice directly (no initial scatter), and rank r ends
// with the H coefficients i = r mod N -- exactly the H bases its proving-key
// shard holds (zk_pk_upload_shard / zk_groth16_setup_dev_shard).
#pragma once
#include <memory>

#include "common.hpp"

struct zk_ctx;
struct zk_pk_dev;

namespace zk {

// All-to-all of equal chunks: chunk k of `send` goes to rank k, chunk s of
// `recv` comes from rank s.
struct Exchange {
  int rank = 0, world = 1;
  virtual void all_to_all(const void* send, void* recv, size_t chunk_bytes, hipStream_t st) = 0;
  // max over ranks of a host status code (synchronous)
  virtual int agree_max(int status, hipStream_t st) = 0;
  virtual ~Exchange() = default;
};

// Per-rank buffers of the distributed quotient (grow-only).
struct DistQ {
  DevBuf s1, r1, s2, r2, s3, r3;
};

// Whether the distributed quotient applies: N a power of two <= 16 and
// n >= N^2 (every rank owns >= 1 column of the N x m matrix).
bool dist_quotient_ok(uint64_t n, int world);

// The four rank-local stages between the three exchanges.  h_out gets
// lo64(H_(rank + N d)), d < m.
void dq_stage_a(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, int rank, int world, DistQ& q,
                uint32_t* d_flags, hipStream_t st);
void dq_stage_b(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& q, hipStream_t st);
void dq_stage_c(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& q, hipStream_t st);
void dq_stage_d(zk_ctx* ctx, const zk_pk_dev* pk, int rank, int world, DistQ& q, uint64_t* h_out,
                hipStream_t st);
// chunk bytes of the three exchanges
size_t dq_chunk_bytes(const zk_pk_dev* pk, int world, int which);

// The whole pipeline with a live exchange (RCCL): stage, all-to-all, ...
void dist_quotient(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, Exchange& ex, DistQ& q,
                   uint32_t* d_flags, uint64_t* h_out, hipStream_t st);

// RCCL communicator wrapper (ncclAllToAll, bytes as ncclUint8).
std::unique_ptr<Exchange> make_rccl_exchange(const uint8_t unique_id[128], int rank, int world);
void rccl_unique_id(uint8_t out[128]);

}  // namespace zk
