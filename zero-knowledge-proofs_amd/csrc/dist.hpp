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
// `recv` comes from rank s.  Two transports: RCCL (ncclAllToAll over xGMI,
// enqueued on the stream) and host-staged callbacks (zk_exchange_ops: the
// chunks cross through pinned host memory and the caller's transport, e.g.
// torch.distributed over gloo).
struct Exchange {
  int rank = 0, world = 1;
  // set once a proof failed after the ranks agreed to start: the peers may
  // be blocked in (or have abandoned) a collective, so the exchange is dead
  bool broken = false;
  virtual void all_to_all(const void* send, void* recv, size_t chunk_bytes, hipStream_t st) = 0;
  // max over ranks of a host status code (synchronous)
  virtual int agree_max(int status, hipStream_t st) = 0;
  // max over ranks of two host values at once (RCCL: one all-reduce of 2)
  virtual void agree_max2(int32_t v[2], hipStream_t st) {
    v[0] = agree_max(v[0], st);
    v[1] = agree_max(v[1], st);
  }
  // max over ranks of the device word *d_val, enqueued on st without a host
  // round trip; false when the transport cannot (the caller then agrees the
  // value with agree_max once st is done)
  virtual bool agree_max_dev(uint32_t* d_val, hipStream_t st) { (void)d_val; (void)st; return false; }
  // make the peers' pending collectives with this rank fail instead of
  // waiting forever (RCCL: ncclCommAbort; host: the caller's abort callback)
  virtual void abort() = 0;
  // zk_ctx_detach_exchange: what dropping this exchange must do first.  RCCL
  // aborts its communicator (local, so no rank waits in a collective for a
  // rank that left); a host-staged exchange does nothing -- its abort hook
  // belongs to the caller's transport (TorchExchange destroys a process
  // group), and a broken one has had its abort already
  virtual void detach() { abort(); }
  // an asynchronous transport error is pending (RCCL: ncclCommGetAsyncError)
  virtual bool async_error() { return false; }
  // watchdog for waits on work that depends on the peers: give up (throw
  // ZK_ERR_RCCL) after this long or on an asynchronous transport error
  double timeout_ms = 60000;
  // test hook (zk_ctx_set_option ZK_OPT_FAULT_AFTER_EXCHANGE): throw after
  // the k-th all-to-all of the next proof, as a rank-local failure would
  int fault_after = 0;
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

// The whole pipeline with a live exchange: stage, all-to-all, ...
void dist_quotient(zk_ctx* ctx, const zk_pk_dev* pk, const uint64_t* d_z, Exchange& ex, DistQ& q,
                   uint32_t* d_flags, uint64_t* h_out, hipStream_t st);
// Every allocation and table the pipeline will need, made BEFORE the ranks
// agree to start (an allocation failure then becomes the agreed status, not
// a rank leaving its peers inside a collective).
void dq_prepare(zk_ctx* ctx, const zk_pk_dev* pk, int world, DistQ& q, hipStream_t st);

// RCCL communicator wrapper (ncclAllToAll, bytes as ncclUint8).  The
// communicator is non-blocking: its creation and every call on it are polled
// with the watchdog, so a peer that never joins (or a transport that stalls)
// ends in ZK_ERR_RCCL after timeout_ms instead of a hang.
std::unique_ptr<Exchange> make_rccl_exchange(const uint8_t unique_id[128], int rank, int world, double timeout_ms);
void rccl_unique_id(uint8_t out[128]);
// Wait for stream st, polling: throws ZK_ERR_RCCL once ex's watchdog fires.
void sync_watchdog(hipStream_t st, Exchange& ex);
// Host-staged exchange over the caller's callbacks.
std::unique_ptr<Exchange> make_host_exchange(const zk_exchange_ops& ops, int rank, int world);

}  // namespace zk
