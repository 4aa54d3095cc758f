// addlat.hip -- latency of one dependent full XYZZ add (the bucket
// reductions' unit of work) for a wave alone on its SIMD and for 2 / 4
// waves per SIMD, in each form the reductions use:
//   g1_ilp    G1, one lane per add, no scheduling barriers (xyzz_add_ilp)
//   g1_quad   G1, one add per lane quad (xyzz_add_quad)
//   g2_pair   G2, one add per lane pair (Fq2h, xyzz_add_ilp)
//   g2_duo    G2, one add per two lane pairs (xyzz_add_duo)
// Each lane (quad, pair) runs a chain acc <- acc + T[(i + s) & 255] of
// STEPS adds, the addend loaded from a 256-point L2-resident table as the
// row/column sums load buckets.  Values are random field elements (the
// chord formulas do not use the curve equation).  Timing: best of 3.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/addlat.hip -o tools/addlat
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "../zero-knowledge-proofs_amd/csrc/curve.hpp"



#define CHK(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

enum { G1_ILP = 0, G1_QUAD = 1, G2_PAIR = 2, G2_DUO = 3 };

template <int MODE>
__global__ void __launch_bounds__(256) k_lat(const G1A* __restrict__ pts, uint32_t steps, uint32_t* __restrict__ out) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (MODE == G2_PAIR || MODE == G2_DUO) {
    const uint32_t i = MODE == G2_DUO ? tid >> 2 : tid >> 1;
    auto ld = [&](uint32_t k) {
      const G1A a = ld_vec(&pts[k & 255]);
      XYZZ<Fq2h> r;
      r.X.v = pair_half() ? a.y : a.x;
      r.Y.v = pair_half() ? a.x : a.y;
      f_set_one(r.ZZ);
      f_set_one(r.ZZZ);
      return r;
    };
    XYZZ<Fq2h> acc = ld(i);
#pragma unroll 1
    for (uint32_t s = 1; s <= steps; s++) {
      if constexpr (MODE == G2_DUO) acc = xyzz_add_duo(acc, ld(i + s));
      else acc = xyzz_add_ilp(acc, ld(i + s));
    }
    out[tid] = acc.X.v.v[0];
  } else {
    const uint32_t i = MODE == G1_QUAD ? tid >> 2 : tid;
    XYZZ<Fq> acc = xyzz_from_aff(ld_vec(&pts[i & 255]));
#pragma unroll 1
    for (uint32_t s = 1; s <= steps; s++) {
      const XYZZ<Fq> q = xyzz_from_aff(ld_vec(&pts[(i + s) & 255]));
      if constexpr (MODE == G1_QUAD) acc = xyzz_add_quad(acc, q);
      else acc = xyzz_add_ilp(acc, q);
    }
    out[tid] = acc.X.v[0];
  }
}

template <class K>
static double best_ms(K k) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  double best = 1e30;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(a));
    k();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  std::vector<uint32_t> h(256 * 24);
  uint64_t s = 0x5eedull;
  for (size_t i = 0; i < h.size(); i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)(s >> 11);
    if (i % 12 == 11) h[i] &= 0x0fffffffu;
  }
  G1A* pts;
  uint32_t* out;
  CHK(hipMalloc(&pts, 256 * sizeof(G1A)));
  CHK(hipMalloc(&out, (size_t)cus * 4 * 256 * sizeof(uint32_t)));
  CHK(hipMemcpy(pts, h.data(), 256 * sizeof(G1A), hipMemcpyHostToDevice));
  const uint32_t STEPS = 64;
  const char* names[4] = {"g1_ilp", "g1_quad", "g2_pair", "g2_duo"};
  for (int mode = 0; mode < 4; mode++) {
    for (int wps : {1, 2, 4}) {
      const int blocks = cus * wps;   // 4 waves per block: one per SIMD of a CU
      auto run = [&] {
        if (mode == 0) k_lat<G1_ILP><<<blocks, 256>>>(pts, STEPS, out);
        else if (mode == 1) k_lat<G1_QUAD><<<blocks, 256>>>(pts, STEPS, out);
        else if (mode == 2) k_lat<G2_PAIR><<<blocks, 256>>>(pts, STEPS, out);
        else k_lat<G2_DUO><<<blocks, 256>>>(pts, STEPS, out);
      };
      run();
      CHK(hipDeviceSynchronize());
      const double ms = best_ms(run);
      const double per_add_us = ms * 1000.0 / STEPS;
      const double lanes_per_add = mode == 0 ? 1 : mode == 1 ? 4 : mode == 2 ? 2 : 4;
      const double adds = (double)blocks * 256 / lanes_per_add * STEPS;
      printf("%-8s waves/SIMD %d  %7.2f us per dependent add  %6.3f G adds/s\n", names[mode], wps, per_add_us,
             adds / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
