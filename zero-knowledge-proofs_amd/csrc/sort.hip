// sort.hip -- device radix sort of (bucket, entry) pairs for the MSM's
// bucket grouping, on rocPRIM (AMD's native device-primitive library),
// kept in its own translation unit: its templates dominate compile time.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace zk {

// Onesweep passes of up to ZK_SORT_MAX_BITS key bits: a key of end_bit bits
// takes ceil(end_bit / ZK_SORT_MAX_BITS) passes of equal width (rocPRIM's
// gfx950 default for u32 pairs, 8-bit digits and 1024 x 16 items per block,
// otherwise).  Round 3, same box: the prove's 18-bit A+B1+IC keys in 2 x 9
// instead of 3 x 8 bits, 10.14 -> 9.88 ms; the configs[1] MSM's 19-bit keys
// in 2 x 10, 3.63 -> 3.56 ms (profiles/r03_ab_sort_bits.txt).  16-bit keys
// (H, G2) keep 2 x 8.  ZK_SORT_MAX_BITS: A/B builds only.
#ifndef ZK_SORT_MAX_BITS
#define ZK_SORT_MAX_BITS 10
#endif
// Onesweep block shape (ZK_SORT_BLOCK threads x ZK_SORT_ITEMS items; A/B
// builds only).
#ifndef ZK_SORT_BLOCK
#define ZK_SORT_BLOCK 1024
#endif
#ifndef ZK_SORT_ITEMS
#define ZK_SORT_ITEMS 16
#endif
template <unsigned R>
using OnesweepCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<ZK_SORT_BLOCK, ZK_SORT_ITEMS>,
                                        rocprim::kernel_config<ZK_SORT_BLOCK, ZK_SORT_ITEMS>, R,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <unsigned R>
static hipError_t sort_r(void* tmp, size_t& tmp_bytes, const uint32_t* ki, uint32_t* ko, const uint32_t* vi,
                         uint32_t* vo, size_t n, unsigned end_bit, hipStream_t st) {
  return rocprim::radix_sort_pairs<OnesweepCfg<R>>(tmp, tmp_bytes, ki, ko, vi, vo, n, 0u, end_bit, st);
}

// Stable ascending sort of n (key, value) pairs on bits [0, end_bit) of the
// key.  With tmp == nullptr only sets tmp_bytes.
void sort_pairs_u32(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                    const uint32_t* vals_in, uint32_t* vals_out, size_t n, unsigned end_bit, hipStream_t st) {
  const unsigned passes = (end_bit + ZK_SORT_MAX_BITS - 1) / ZK_SORT_MAX_BITS;
  const unsigned r = passes ? (end_bit + passes - 1) / passes : 8;
  if (ZK_SORT_MAX_BITS <= 8 || r <= 8) {
    ZK_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0u, end_bit, st));
    return;
  }
  hipError_t e;
  if (r == 9) e = sort_r<9>(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, end_bit, st);
  else if (r == 10) e = sort_r<10>(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, end_bit, st);
  else e = sort_r<11>(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, end_bit, st);
  ZK_HIP(e);
}

}  // namespace zk
