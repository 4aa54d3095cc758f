// common.hpp -- status codes, HIP error plumbing, device buffers.
#pragma once
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdint.h>

#include <cstdio>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

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

// Pinned host allocation (grow-only).  Device->host copies into pageable
// memory block the calling thread, which would serialise the per-MSM
// streams; results therefore land in pinned buffers.
struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  void ensure(size_t b) {
    if (b <= bytes) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    ZK_HIP(hipHostMalloc(&p, b ? b : 16, hipHostMallocDefault));
    bytes = b;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

inline uint32_t ceil_div(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// roctx range on the host timeline around a phase's launches (rocprofv3
// --marker-trace shows them beside the kernels; a no-op without a tracer).
struct Range {
  explicit Range(const char* what) { roctxRangePushA(what); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// Live kernel timing with HIP events on the launching stream (enabled by
// zk_ctx_profile).  Each phase accumulates device time, launches and work
// units (e.g. scalar-point pairs) so bench.py can price the dominant kernel
// against its algorithmic bytes.
struct PhaseStat {
  double ms = 0;
  uint64_t launches = 0, units = 0;
};
struct Prof {
  bool on = false;
  struct Rec {
    std::string phase;
    hipEvent_t a, b;
    uint64_t units;
    hipStream_t st;
  };
  // Timeline (zk_ctx_profile(ctx, 2), read by zk_ctx_timeline_read):
  // collect() appends one line per phase -- name, stream, start and end in
  // ms after the last mark_origin() -- and "--" per collection, so a run
  // shows how the streams overlap.
  bool timeline = false;
  std::string tl;
  hipEvent_t origin = nullptr;
  bool origin_set = false;
  void mark_origin(hipStream_t st) {
    if (!on || !timeline) return;
    if (!origin) ZK_HIP(hipEventCreate(&origin));
    ZK_HIP(hipEventRecord(origin, st));
    origin_set = true;
  }
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  std::map<std::string, PhaseStat> stats;

  hipEvent_t ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    ZK_HIP(hipEventCreate(&e));
    return e;
  }
  // returns an index to close with end(); -1 when disabled
  int begin(hipStream_t st, const char* phase, uint64_t units) {
    if (!on) return -1;
    Rec r{phase, ev(), ev(), units, st};
    ZK_HIP(hipEventRecord(r.a, st));
    pending.push_back(r);
    return (int)pending.size() - 1;
  }
  void end(hipStream_t st, int i) {
    if (i < 0) return;
    ZK_HIP(hipEventRecord(pending[i].b, st));
  }
  // host-side wall time of a phase (measured by the caller)
  void add_host(const char* phase, double ms) {
    if (!on) return;
    PhaseStat& s = stats[phase];
    s.ms += ms;
    s.launches += 1;
  }
  // after the stream has been synchronised
  void collect() {
    const bool rec_tl = origin_set && timeline;
    for (Rec& r : pending) {
      float ms = 0;
      ZK_HIP(hipEventSynchronize(r.b));
      ZK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
      if (rec_tl) {
        float t0 = 0, t1 = 0;
        ZK_HIP(hipEventElapsedTime(&t0, origin, r.a));
        ZK_HIP(hipEventElapsedTime(&t1, origin, r.b));
        char line[256];
        snprintf(line, sizeof line, "%s %p %.4f %.4f\n", r.phase.c_str(), (void*)r.st, t0, t1);
        tl += line;
      }
      PhaseStat& s = stats[r.phase];
      s.ms += ms;
      s.launches += 1;
      s.units += r.units;
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
    if (rec_tl) tl += "--\n";
    origin_set = false;
  }
  ~Prof() {
    if (origin) (void)hipEventDestroy(origin);
    for (Rec& r : pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace zk
