// quotient.hpp -- pieces of the QAP quotient shared by the single-GPU path
// (prove.hip) and the distributed one (dist.hip).
#pragma once
#include "ctx.hpp"

namespace zk {

// The constraint matrices as CSR device pointers (val == nullptr: unit).
struct CsrArgs {
  const uint64_t* rp[3];
  const uint32_t* col[3];
  const Fr* val[3];
};

__device__ __forceinline__ Fr row_dot(const uint64_t* __restrict__ rp, const uint32_t* __restrict__ col,
                                      const Fr* __restrict__ val, uint64_t row, const Fr* __restrict__ zc,
                                      uint64_t V) {
  Fr acc = fp_zero<FrParams>();
  const uint64_t e = rp[row + 1];
  for (uint64_t k = rp[row]; k < e; k++) {
    const uint32_t c = col[k];
    if (c >= V) continue;                   // qap:122-124
    Fr zv = fp_to_mont(ld_vec(&zc[c]));
    if (val) zv = fp_mul(zv, ld_vec(&val[k]));
    acc = fp_add(acc, zv);
  }
  return acc;
}

// Device-side view of a pk's CSR.
inline CsrArgs csr_args(const CsrDev& c) {
  CsrArgs m;
  for (int k = 0; k < 3; k++) {
    m.rp[k] = c.rp[k].as<uint64_t>();
    m.col[k] = c.col[k].as<uint32_t>();
    m.val[k] = c.unit[k] ? nullptr : c.val[k].as<Fr>();
  }
  return m;
}

}  // namespace zk
