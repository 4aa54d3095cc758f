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

#ifdef __cplusplus
}
#endif
#endif /* ZKP_TEST_H */
