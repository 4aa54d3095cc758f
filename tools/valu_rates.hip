// valu_rates.hip -- measured issue rate of the VALU instructions a field
// multiply can be built from (v_mad_u64_u32, v_mul_lo/hi_u32, 24-bit muls,
// v_fma_f64, 64-bit adds) on one gfx950: 8 independent chains per lane,
// 16 waves per CU, so the rate is throughput, not latency.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) (void)(x)

constexpr int CH = 8, IT = 2048;

template <int OP>
__global__ void __launch_bounds__(256) k_rate(const uint32_t* __restrict__ in, uint64_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t y = in[t & 1023] | 1u;
  uint64_t acc[CH];
  uint32_t x[CH];
  double d[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) {
    x[i] = in[(t + 7 * i) & 1023];
    acc[i] = x[i];
    d[i] = (double)x[i];
  }
  const double e = 1.0000001 + (double)(y & 7) * 1e-9, f = (double)(y >> 20);
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      // inline asm: the compiler would fold plain C chains (x += y ... -> x + IT y)
      if constexpr (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(x[i]), "v"(y) : "vcc");
      if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if constexpr (OP == 3) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x[i]) : "v"(y));
      if constexpr (OP == 4) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(e), "v"(f));
      if constexpr (OP == 5) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(acc[(i + 1) % CH]));
      if constexpr (OP == 6) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if constexpr (OP == 7) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[i]) : "v"(y) : "vcc");
      if constexpr (OP == 8) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(x[i]), "v"(y) : "vcc");
      if constexpr (OP == 9) asm volatile("v_ashrrev_i64 %0, 28, %0" : "+v"(acc[i]));
      if constexpr (OP == 10) asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(acc[i]));
      if constexpr (OP == 11) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if constexpr (OP == 12) asm volatile("v_alignbit_b32 %0, %0, %1, 28" : "+v"(x[i]) : "v"(y));
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) r += acc[i] + x[i] + (uint64_t)d[i];
  out[t] = r;
}

template <int OP>
float run(const uint32_t* in, uint64_t* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_rate<OP><<<blocks, 256>>>(in, out);
  hipEventRecord(a);
  k_rate<OP><<<blocks, 256>>>(in, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const int blocks = cus * 4 * 4;   // 16 waves per CU (4 per SIMD)
  uint32_t* in;
  uint64_t* out;
  hipMalloc(&in, 4096);
  hipMalloc(&out, sizeof(uint64_t) * blocks * 256);
  uint32_t h[1024];
  for (int i = 0; i < 1024; i++) h[i] = 0x9e3779b9u * (i + 1);
  hipMemcpy(in, h, 4096, hipMemcpyHostToDevice);
  const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32+xor", "v_mad_u32_u24", "v_fma_f64",
                         "v_lshl_add_u64", "v_add_u32", "v_add_co_u32", "v_mad_i64_i32", "v_ashrrev_i64", "v_lshrrev_b64", "v_and_b32", "v_alignbit_b32"};
  float ms[13] = {run<0>(in, out, blocks), run<1>(in, out, blocks), run<2>(in, out, blocks), run<3>(in, out, blocks),
                  run<4>(in, out, blocks), run<5>(in, out, blocks), run<6>(in, out, blocks), run<7>(in, out, blocks),
                  run<8>(in, out, blocks), run<9>(in, out, blocks), run<10>(in, out, blocks), run<11>(in, out, blocks),
                  run<12>(in, out, blocks)};
  const double ops = (double)blocks * 256 * IT * CH;
  printf("cus %d clock %d MHz\n", cus, clk / 1000);
  for (int k = 0; k < 13; k++) {
    const double rate = ops / (ms[k] * 1e-3);   // lane-ops/s
    const double per_simd_cycle = rate / (cus * 4.0 * clk * 1e3);   // lane-ops per SIMD per cycle
    printf("%-20s %8.3f ms  %7.2f Tlane-op/s  %6.2f lane-op/SIMD/clk  (%.2f cycles per wave64 op)\n", names[k], ms[k],
           rate * 1e-12, per_simd_cycle, 64.0 / per_simd_cycle);
  }
  return 0;
}
