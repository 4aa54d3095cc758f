/*
 * zkp_test.h -- diagnostic entry points of libzkp_amd_test.so, a separate
 * library built on top of libzkp_amd.so for the GPU tests.  None of these is
 * part of the drop-in ABI (include/zkp.h) and none has a reference
 * counterpart: they reach paths a one-GPU box cannot reach through the
 * product ABI (N ranks on one device) and inject failures.
 */
#ifndef ZKP_TEST_H
#define ZKP_TEST_H
#include "zkp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* nshards virtual ranks of one key on this ctx's single device (the
 * distributed quotient's all-to-alls become device copies) -- checks the
 * distributed path's arithmetic and index maps without N devices. */
int zk_test_prove_virtual_shards(zk_ctx *ctx, const zk_pk_dev *const *shards, uint32_t nshards,
                                 const void *d_z, size_t zlen, size_t num_public, const zk_fr *r,
                                 const zk_fr *s, zk_proof *out);
/* The attached exchange's two operations on their own, on the ctx's stream
 * -- one all-to-all of chunk_bytes per rank over a device buffer whose chunk
 * k holds bytes (rank * 31 + k * 7 + i) & 0xff, then the status agreement of
 * `status`.  *out_max = the agreed maximum; ZK_OK when every received chunk
 * s equals what rank s sent, ZK_ERR_RCCL otherwise (or on a transport
 * error).  Runs ncclAllToAll / ncclAllReduce themselves on a world-1 RCCL
 * communicator, where a one-GPU box can reach them. */
int zk_test_exchange(zk_ctx *ctx, size_t chunk_bytes, int32_t status, int32_t *out_max);
/* k = 1..3: the next distributed-quotient proof on this ctx fails right
 * after its k-th all-to-all, as a rank-local error would (tests of the abort
 * path); 0 clears it.  ZK_ERR_ARG without an attached exchange. */
int zk_test_fault_after_exchange(zk_ctx *ctx, int k);
/* Readback of a device proving key (setup parity at size): slot 0 pi_A
 * (a_g1), 1 pi_B (b_g2), 2 B_1 (b_g1), 3 IC (ic_g1), 4 H (h_g1); window w
 * of the window-shifted copies (w = 0: the bases themselves, w: 2^(win_c w)
 * times them).  *count = compacted non-identity bases of this shard,
 * *nextras = extra bases appended after them (shard 0: alpha_1 and
 * 2^(64k) delta_1 / beta_2 and 2^(64k) delta_2 / beta_1).  With cap >=
 * count + nextras: idx_out[k] = the variable (H: coefficient) index of base
 * k < count, words_out = all count + nextras bases as canonical ABI words
 * (13 per G1, 25 per G2 point).  cap = 0 only queries the counts. */
int zk_test_pk_bases(zk_ctx *ctx, const zk_pk_dev *pk, int slot, int window, uint32_t *idx_out,
                     uint64_t *words_out, size_t cap, size_t *count, size_t *nextras);
/* The key's window plan and shard: win copies of c = win_c bits. */
int zk_test_pk_info(const zk_pk_dev *pk, uint32_t *win, uint32_t *win_c, uint32_t *shard, uint32_t *nshards);

#ifdef __cplusplus
}
#endif
#endif /* ZKP_TEST_H */
