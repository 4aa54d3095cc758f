// common.hpp -- status codes, HIP error plumbing, device buffers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/zkp.h"

namespace zk {

// A failed HIP call becomes a C++ exception carrying ZK_ERR_DEVICE; the C ABI
// boundary (capi.cpp) turns it back into a status code.  Nothing else throws.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define ZK_HIP(call)                                                              \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess)                                                         \
      throw ::zk::Error(ZK_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_) + \
                                           " @" __FILE__ ":" + std::to_string(__LINE__)); \
  } while (0)

#define ZK_LAUNCH_CHECK() ZK_HIP(hipGetLastError())

// Owning device allocation (grow-only, reused across calls).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void ensure(size_t b) {
    if (b <= bytes) return;
    release();
    ZK_HIP(hipMalloc(&p, b ? b : 16));
    bytes = b;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

inline uint32_t ceil_div(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace zk
