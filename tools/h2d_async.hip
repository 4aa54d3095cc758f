// How hipMemcpyAsync from PAGEABLE host memory behaves on this runtime
// (informs the drop-in host-witness prove): time until the call returns vs
// until the stream has the data, whole buffer vs two halves, and with a
// long kernel running on another stream meanwhile.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin(unsigned long long cycles, int* out) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0 && blockIdx.x == 0) *out = 1;
}

static double ms(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

int main() {
  const size_t bytes = (3ull * (1 << 20) + 1) * 32;
  char* h = (char*)malloc(bytes);
  memset(h, 1, bytes);
  void* d;
  CK(hipMalloc(&d, bytes));
  int* flag;
  CK(hipMalloc(&flag, 4));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = clk::now();
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s0));
    auto t1 = clk::now();
    CK(hipStreamSynchronize(s0));
    auto t2 = clk::now();
    printf("whole: call returns %.3f ms, data in %.3f ms\n", ms(t0, t1), ms(t0, t2));
    t0 = clk::now();
    CK(hipMemcpyAsync(d, h, bytes / 2, hipMemcpyHostToDevice, s0));
    t1 = clk::now();
    CK(hipMemcpyAsync((char*)d + bytes / 2, h + bytes / 2, bytes - bytes / 2, hipMemcpyHostToDevice, s0));
    auto t1b = clk::now();
    CK(hipStreamSynchronize(s0));
    t2 = clk::now();
    printf("halves: first returns %.3f, second returns %.3f, data in %.3f ms\n", ms(t0, t1), ms(t0, t1b), ms(t0, t2));
    // with a ~5 ms kernel on another stream
    spin<<<1024, 256, 0, s1>>>(12000000ull, flag);
    t0 = clk::now();
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s0));
    t1 = clk::now();
    CK(hipStreamSynchronize(s0));
    t2 = clk::now();
    CK(hipStreamSynchronize(s1));
    auto t3 = clk::now();
    printf("beside a kernel: call returns %.3f, data in %.3f, kernel done %.3f ms\n", ms(t0, t1), ms(t0, t2), ms(t0, t3));
  }
  return 0;
}
