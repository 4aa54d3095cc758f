// sort.hip -- device radix sort of (bucket, entry) pairs for the MSM's
// bucket grouping, on rocPRIM (AMD's native device-primitive library),
// kept in its own translation unit: its templates dominate compile time.
#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace zk {

// rocPRIM's gfx950 onesweep default for 32-bit keys and values sorts 8 bits
// per pass; batched MSM keys have 17-18 bits (MSM k << 16 | bucket), which
// take 3 passes at 8 bits and 2 at 9 (same kernel shapes, 512 bins).
using Onesweep9 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, 9,
                                        rocprim::block_radix_rank_algorithm::match>>;

static bool sort9_enabled() {
  static const bool on = [] {
    const char* e = getenv("ZK_SORT9");   // opt-in: -0.15 ms serial, not better overlapped
    return e && atoi(e) != 0;
  }();
  return on;
}

// Stable ascending sort of n (key, value) pairs on bits [0, end_bit) of the
// key.  With tmp == nullptr only sets tmp_bytes.
void sort_pairs_u32(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                    const uint32_t* vals_in, uint32_t* vals_out, size_t n, unsigned end_bit, hipStream_t st) {
  if (end_bit > 16 && end_bit <= 18 && sort9_enabled())
    ZK_HIP(rocprim::radix_sort_pairs<Onesweep9>(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0u,
                                                end_bit, st));
  else
    ZK_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0u, end_bit, st));
}

}  // namespace zk
