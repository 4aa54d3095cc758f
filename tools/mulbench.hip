// Microbenchmark of 381-bit Montgomery multiplication variants on gfx950.
// v1: current CIOS (rolled rows, 32-bit limbs)   v2: CIOS with addc carry chain
// r28: radix-2^28 product scanning (14 limbs, one v_mad_u64_u32 per product)
// Each thread runs ITER dependent multiplies; reports Gmul/s.  Correctness:
// all variants must agree after conversion to canonical form.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../zero-knowledge-proofs_amd/csrc/ff.hpp"

typedef unsigned __int128 u128;
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// ---------------- v2: CIOS, carries via addc ----------------
__device__ __forceinline__ Fq mul_v2(const Fq& a, const Fq& b) {
  constexpr int N = 12;
  uint64_t T[N];
  uint32_t bb[N];
#pragma unroll
  for (int j = 0; j < N; j++) { T[j] = 0; bb[j] = b.v[j]; }
#pragma unroll 1
  for (int i = 0; i < N; i++) {
    const uint32_t bi = bb[0];
#pragma unroll
    for (int j = 0; j < N - 1; j++) bb[j] = bb[j + 1];
    uint32_t cc = 0, hprev = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
      uint64_t Pj = (uint64_t)a.v[j] * bi + T[j];
      T[j] = __builtin_addc((uint32_t)Pj, hprev, cc, &cc);
      hprev = (uint32_t)(Pj >> 32);
    }
    uint32_t top = hprev + cc;
    const uint32_t m = (uint32_t)T[0] * 0xfffcfffdu;  // -p^-1 mod 2^32
    uint64_t Q = (uint64_t)m * FqParams::MOD[0] + T[0];
    hprev = (uint32_t)(Q >> 32);
    cc = 0;
#pragma unroll
    for (int j = 1; j < N; j++) {
      Q = (uint64_t)m * FqParams::MOD[j] + T[j];
      T[j - 1] = __builtin_addc((uint32_t)Q, hprev, cc, &cc);
      hprev = (uint32_t)(Q >> 32);
    }
    T[N - 1] = top + hprev + cc;
  }
  Fq r;
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = (uint32_t)T[j];
  return fp_reduce_once(r);
}

// ---------------- r28: radix 2^28, 14 limbs ----------------
struct F28 { uint32_t v[14]; };
__constant__ uint32_t P28[14];
__constant__ uint32_t INV28;
template <int NACC>
__device__ __forceinline__ F28 mul_r28(const F28& a, const F28& b) {
  constexpr int N = 14;
  constexpr uint32_t MASK = (1u << 28) - 1;
  uint32_t m[N], r[N];
  uint64_t acc[NACC];
#pragma unroll
  for (int q = 0; q < NACC; q++) acc[q] = 0;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    int t = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N) { acc[t % NACC] += (uint64_t)a.v[i] * b.v[j]; t++; }
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N) { acc[t % NACC] += (uint64_t)m[i] * P28[j]; t++; }
    }
    uint64_t s = carry;
#pragma unroll
    for (int q = 0; q < NACC; q++) { s += acc[q]; acc[q] = 0; }
    if (k < N) {
      m[k] = ((uint32_t)s * INV28) & MASK;
      s += (uint64_t)m[k] * P28[0];
    } else {
      r[k - N] = (uint32_t)s & MASK;
    }
    carry = s >> 28;
  }
  r[N - 1] = (uint32_t)carry;
  F28 o;
#pragma unroll
  for (int j = 0; j < N; j++) o.v[j] = r[j];
  return o;
}

template <int V>
__global__ void __launch_bounds__(256) kbench(const uint32_t* in, uint32_t* out, int iters) {
  extern __shared__ uint32_t pad[];   // latency mode: a large dynamic LDS request caps one block per CU
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (iters < 0) pad[threadIdx.x] = 0;
  if (V <= 2) {
    Fq x, y;
    for (int i = 0; i < 12; i++) { x.v[i] = in[(t % 1024) * 24 + i]; y.v[i] = in[(t % 1024) * 24 + 12 + i]; }
    for (int k = 0; k < iters; k++) x = V == 1 ? fp_mul(x, y) : mul_v2(x, y);
    for (int i = 0; i < 12; i++) out[t * 14 + i] = x.v[i];
  } else {
    F28 x, y;
    for (int i = 0; i < 14; i++) { x.v[i] = in[(t % 1024) * 28 + i]; y.v[i] = in[(t % 1024) * 28 + 14 + i]; }
    for (int k = 0; k < iters; k++) x = V == 3 ? mul_r28<1>(x, y) : mul_r28<2>(x, y);
    for (int i = 0; i < 14; i++) out[t * 14 + i] = x.v[i];
  }
}

// host big-int helpers (Python-free): p, conversions
static void to_r28(u128 dummy, const uint32_t* w32, uint32_t* w28) {
  (void)dummy;
  // w32: 12 words little endian -> 14 x 28-bit
  for (int i = 0; i < 14; i++) {
    int bit = 28 * i, wd = bit / 32, sh = bit % 32;
    uint64_t lo = w32[wd] >> sh;
    if (wd + 1 < 12) lo |= (uint64_t)w32[wd + 1] << (32 - sh);
    w28[i] = (uint32_t)(lo & ((1u << 28) - 1));
  }
}

int main() {
  const int threads = 256 * 256 * 4, iters = 2000;
  // operands: random values < p (top word masked)
  std::vector<uint32_t> in32(1024 * 24), in28(1024 * 28);
  uint64_t s = 12345;
  for (auto& x : in32) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; x = (uint32_t)(s >> 32); }
  for (int i = 0; i < 1024 * 2; i++) in32[i * 12 + 11] &= 0x0fffffff;
  for (int i = 0; i < 1024 * 2; i++) to_r28(0, &in32[i * 12], &in28[i * 14]);
  uint32_t p28[14];
  to_r28(0, FqParams::MOD, p28);
  // -p^-1 mod 2^28
  uint32_t x = 1;
  for (int k = 0; k < 6; k++) x *= 2 - p28[0] * x;
  uint32_t inv28 = (0u - x) & ((1u << 28) - 1);
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(P28), p28, sizeof p28));
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(INV28), &inv28, 4));
  uint32_t *d32, *d28, *dout;
  CHK(hipMalloc(&d32, in32.size() * 4));
  CHK(hipMalloc(&d28, in28.size() * 4));
  CHK(hipMalloc(&dout, (size_t)threads * 14 * 4));
  CHK(hipMemcpy(d32, in32.data(), in32.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(d28, in28.data(), in28.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const char* names[4] = {"fp_mul (ff.hpp)", "v2 CIOS addc", "r28 comba 1acc", "r28 comba 2acc"};
  // mode 0: full occupancy; mode 1: one 256-thread block per CU (1 wave/SIMD), latency-bound
  for (int mode = 0; mode < 2; mode++) {
    const int nthr = mode ? 256 * 256 : threads;
    const size_t lds = mode ? 96 * 1024 : 0;
    const int it = mode ? iters / 4 : iters;
    for (int v = 1; v <= 4; v++) {
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(a));
        switch (v) {
          case 1: kbench<1><<<nthr / 256, 256, lds>>>(d32, dout, it); break;
          case 2: kbench<2><<<nthr / 256, 256, lds>>>(d32, dout, it); break;
          case 3: kbench<3><<<nthr / 256, 256, lds>>>(d28, dout, it); break;
          case 4: kbench<4><<<nthr / 256, 256, lds>>>(d28, dout, it); break;
        }
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (rep)
          printf("%s %-18s %8.2f ms  %8.2f Gmul/s  %6.0f ns/mul/thread\n", mode ? "1wave/SIMD" : "full      ",
                 names[v - 1], ms, (double)nthr * it / ms / 1e6, ms * 1e6 / it);
      }
    }
  }
  return 0;
}
