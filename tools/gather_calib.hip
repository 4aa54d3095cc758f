// FETCH_SIZE calibration for the MSM accumulate's access shape (tools only).
//
// MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the bytes of a wide
// coalesced streaming read on gfx950, and other access widths are
// uncalibrated.  The G1 accumulate gathers random 96-byte affine points
// (6 x 16-byte loads per lane, records straddling 128-byte lines); this
// program runs that shape, a 128-byte-aligned variant and a streaming read,
// each over a known byte count, so
//   rocprofv3 --pmc FETCH_SIZE -- tools/gather_calib
// gives the counter's bytes per algorithmic byte for each.  One line per
// kernel on stdout: name, records, algorithmic bytes, distinct 128-B lines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
#include <set>
#include <vector>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

// gather `per` 16-byte words of record idx[i] (record stride `stride` bytes)
template <int PER, int S16>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ base, const uint32_t* __restrict__ idx,
                                                uint32_t n, uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* p = base + (size_t)idx[i] * S16;
  uint4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint4 v = p[k];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  out[i] = acc;
}

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ in, size_t n16, uint4* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n16) return;
  const uint4 v = in[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = v;   // keeps the load, ~never stores
}

int main() {
  const uint32_t N = 1u << 22;           // gathered records per launch
  const uint32_t POOL = 1u << 24;        // 24M records: 1.5-2 GB, far beyond the 256 MiB L3
  std::vector<uint32_t> idx(N);
  std::mt19937 rng(7);
  for (auto& v : idx) v = rng() % POOL;
  std::set<uint64_t> lines96, lines128;
  for (uint32_t v : idx) {
    const uint64_t a = (uint64_t)v * 96;
    for (uint64_t l = a / 128; l <= (a + 95) / 128; l++) lines96.insert(l);
    lines128.insert((uint64_t)v);
  }
  uint4 *pool, *out;
  uint32_t* didx;
  CHK(hipMalloc(&pool, (size_t)POOL * 128));
  CHK(hipMemset(pool, 1, (size_t)POOL * 128));
  CHK(hipMalloc(&out, (size_t)N * 16));
  CHK(hipMalloc(&didx, (size_t)N * 4));
  CHK(hipMemcpy(didx, idx.data(), (size_t)N * 4, hipMemcpyHostToDevice));
  const size_t stream_bytes = (size_t)1 << 30;
  for (int rep = 0; rep < 2; rep++) {
    k_gather<6, 6><<<(N + 255) / 256, 256>>>(pool, didx, N, out);            // 96-B records, 96-B stride
    CHK(hipGetLastError());
    k_gather<6, 8><<<(N + 255) / 256, 256>>>(pool, didx, N, out);            // 96 B read from 128-B slots
    CHK(hipGetLastError());
    k_gather<8, 8><<<(N + 255) / 256, 256>>>(pool, didx, N, out);            // whole 128-B records
    CHK(hipGetLastError());
    k_stream<<<(uint32_t)((stream_bytes / 16 + 255) / 256), 256>>>(pool, stream_bytes / 16, out);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
  }
  printf("k_gather<6,6>:  records %u algorithmic_bytes %llu distinct_128B_lines %zu (x128 = %llu B)\n", N,
         (unsigned long long)N * 96, lines96.size(), (unsigned long long)lines96.size() * 128);
  printf("k_gather<6,8>: records %u algorithmic_bytes %llu distinct_128B_lines %zu (x128 = %llu B)\n", N,
         (unsigned long long)N * 96, lines128.size(), (unsigned long long)lines128.size() * 128);
  printf("k_gather<8,8>: records %u algorithmic_bytes %llu distinct_128B_lines %zu (x128 = %llu B)\n", N,
         (unsigned long long)N * 128, lines128.size(), (unsigned long long)lines128.size() * 128);
  printf("k_stream: algorithmic_bytes %zu\n", stream_bytes);
  CHK(hipFree(pool));
  CHK(hipFree(out));
  CHK(hipFree(didx));
  return 0;
}
