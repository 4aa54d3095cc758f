// testhooks.hip -- libzkp_amd_test.so: the diagnostic entry points of
// include/zkp_test.h, built as a separate library on top of libzkp_amd.so so
// that the shipped ABI (include/zkp.h) holds no way to inject a failure or to
// drive the virtual-rank path.  Only the GPU tests load it.
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "../../include/zkp_test.h"

namespace zk {
void bases_to_abi_host(bool g2, const void* d_in, uint32_t stride, size_t n, uint64_t* host_out, hipStream_t st);
int prove_virtual_shards_impl(zk_ctx*, const zk_pk_dev* const*, uint32_t, const void*, size_t, size_t,
                              const zk_fr*, const zk_fr*, zk_proof*);
}  // namespace zk

using namespace zk;

#define ZK_TGUARD(ctx, ...)                                   \
  try {                                                       \
    ZK_HIP(hipSetDevice((ctx)->device));                      \
    __VA_ARGS__                                               \
  } catch (const zk::Error& e) {                              \
    (ctx)->err = e.what();                                    \
    return e.code;                                            \
  } catch (const std::exception& e) {                         \
    (ctx)->err = e.what();                                    \
    return ZK_ERR_DEVICE;                                     \
  }

int zk_test_prove_virtual_shards(zk_ctx* ctx, const zk_pk_dev* const* shards, uint32_t nshards, const void* d_z,
                                 size_t zlen, size_t num_public, const zk_fr* r, const zk_fr* s, zk_proof* out) {
  if (!ctx || !shards || !d_z || !r || !s || !out) return ZK_ERR_ARG;
  ZK_TGUARD(ctx, { return prove_virtual_shards_impl(ctx, shards, nshards, d_z, zlen, num_public, r, s, out); })
}

int zk_test_exchange(zk_ctx* ctx, size_t chunk_bytes, int32_t status, int32_t* out_max) {
  if (!ctx || !out_max || !chunk_bytes || chunk_bytes > ((size_t)1 << 30)) return ZK_ERR_ARG;
  ZK_TGUARD(ctx, {
    if (!ctx->exch) throw Error(ZK_ERR_ARG, "test_exchange: no exchange attached");
    Exchange& ex = *ctx->exch;
    const size_t W = (size_t)ex.world, bytes = chunk_bytes * W;
    std::vector<uint8_t> h(bytes);
    for (size_t k = 0; k < W; k++)
      for (size_t i = 0; i < chunk_bytes; i++) h[k * chunk_bytes + i] = (uint8_t)((ex.rank * 31 + k * 7 + i) & 0xff);
    DevBuf send, recv;
    send.ensure(bytes);
    recv.ensure(bytes);
    ZK_HIP(hipMemcpyAsync(send.p, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
    ZK_HIP(hipMemsetAsync(recv.p, 0, bytes, ctx->stream));
    ex.all_to_all(send.p, recv.p, chunk_bytes, ctx->stream);
    *out_max = ex.agree_max(status, ctx->stream);
    ZK_HIP(hipMemcpyAsync(h.data(), recv.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
    ZK_HIP(hipStreamSynchronize(ctx->stream));
    for (size_t s = 0; s < W; s++)   // chunk s came from rank s, which filled its chunk `rank` for us
      for (size_t i = 0; i < chunk_bytes; i++)
        if (h[s * chunk_bytes + i] != (uint8_t)((s * 31 + (size_t)ex.rank * 7 + i) & 0xff)) return ZK_ERR_RCCL;
    return ZK_OK;
  })
}

int zk_test_fault_after_exchange(zk_ctx* ctx, int k) {
  if (!ctx || k < 0 || k > 3 || !ctx->exch) return ZK_ERR_ARG;
  ctx->exch->fault_after = k;
  return ZK_OK;
}

int zk_test_pk_bases(zk_ctx* ctx, const zk_pk_dev* pk, int slot, int window, uint32_t* idx_out, uint64_t* words_out,
                     size_t cap, size_t* count, size_t* nextras) {
  if (!ctx || !pk || !count || !nextras || slot < 0 || slot >= NUM_MSM || window < 0 || window >= pk->win)
    return ZK_ERR_ARG;
  const size_t cnt = pk->count[slot], nex = pk->extras[slot], tot = cnt + nex;
  *count = cnt;
  *nextras = nex;
  if (!cap) return ZK_OK;
  if (cap < tot || !idx_out || !words_out) return ZK_ERR_ARG;
  ZK_TGUARD(ctx, {
    const bool g2 = slot == MSM_B2;
    const size_t asz = g2 ? sizeof(G2A) : sizeof(G1A);
    // IC and H share one window buffer (bases[MSM_H]: each window [IC | H])
    const bool ich = slot == MSM_IC || slot == MSM_H;
    const int bslot = ich ? MSM_H : slot;
    const size_t step = pk->stride[bslot] ? pk->stride[bslot] : asz;
    const size_t wtot = ich ? pk->ich_tot() : tot;
    const size_t skip = slot == MSM_H ? (size_t)pk->count[MSM_IC] + pk->extras[MSM_IC] : 0;
    const char* base = static_cast<const char*>(pk->bases[bslot].p) + ((size_t)window * wtot + skip) * step;
    if (cnt) ZK_HIP(hipMemcpyAsync(idx_out, pk->idx[slot].p, sizeof(uint32_t) * cnt, hipMemcpyDeviceToHost, ctx->stream));
    bases_to_abi_host(g2, base, pk->stride[bslot], tot, words_out, ctx->stream);
    ZK_HIP(hipStreamSynchronize(ctx->stream));
    return ZK_OK;
  })
}

int zk_test_pk_info(const zk_pk_dev* pk, uint32_t* win, uint32_t* win_c, uint32_t* shard, uint32_t* nshards) {
  if (!pk || !win || !win_c || !shard || !nshards) return ZK_ERR_ARG;
  *win = (uint32_t)pk->win;
  *win_c = (uint32_t)pk->win_c;
  *shard = pk->shard;
  *nshards = pk->nshards;
  return ZK_OK;
}
