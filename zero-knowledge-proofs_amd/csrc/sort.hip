// sort.hip -- device radix sort of (bucket, entry) pairs for the MSM's
// bucket grouping, on rocPRIM (AMD's native device-primitive library),
// kept in its own translation unit: its templates dominate compile time.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace zk {

// Stable ascending sort of n (key, value) pairs on bits [0, end_bit) of the
// key.  With tmp == nullptr only sets tmp_bytes.
void sort_pairs_u32(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                    const uint32_t* vals_in, uint32_t* vals_out, size_t n, unsigned end_bit, hipStream_t st) {
  ZK_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0u, end_bit, st));
}

}  // namespace zk
