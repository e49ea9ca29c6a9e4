// hk_common.hpp — shared definitions for the hkcsa HIP library (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace hk {

constexpr int kWave = 64;  // CDNA wavefront width (hard-coded, see cdna_hip_programming.md §1)

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);

struct HipError {
  hipError_t code;
  std::string where;
};

#define HK_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) throw ::hk::HipError{e_, std::string(#call) + " @" __FILE__ ":" + \
                                                      std::to_string(__LINE__)};            \
  } while (0)

struct ApiError {
  int code;
  std::string msg;
};

// ------------------------------------------------------- device helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// popcount of `m` restricted to lanes below the calling lane
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T t = __shfl_up(v, o, kWave);
    if (l >= (uint32_t)o) v += t;
  }
  return v;
}

// DPP forms (gfx9 row_shr / row_bcast, no LDS traffic): the inclusive wave64 prefix sum of u32, and
// u32 all-lane reductions (the result read from lane 63, wave-uniform).  The shuffles above go through
// ds_bpermute and queue behind the LDS traffic of a co-resident workgroup.
template <typename Op>
__device__ __forceinline__ uint32_t dpp_scan_u32(uint32_t v, uint32_t id, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t dpp_incl_sum(uint32_t v) {
  return dpp_scan_u32(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
template <typename Op>
__device__ __forceinline__ uint32_t dpp_reduce_u32(uint32_t v, uint32_t id, Op op) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dpp_scan_u32(v, id, op), 63);
}
// Every u32 wave scan takes the DPP form.  Precondition: the whole wave is active (EXEC = ~0): row_shr
// with bound_ctrl = 0 reads an inactive source lane as the identity, which breaks the prefix chain, and
// dpp_reduce_u32 reads lane 63.  Every call site is full-wave (the WT partition, occ lines, slice
// pre-pass, bucket sort, cursor passes); a divergent caller needs the generic shuffle form instead.
template <>
__device__ __forceinline__ uint32_t wave_incl_sum<uint32_t>(uint32_t v) {
  return dpp_incl_sum(v);
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T t = __shfl_up(v, o, kWave);
    if (l >= (uint32_t)o) v = v > t ? v : t;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Relaxed agent-scope 8-byte accesses (sc1; L1 bypass) for lookback granules.
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------ device buffers
// A DevBuf either owns its allocation or is a view into another buffer (owned = false: release() and
// the destructor leave the memory alone, and an ensure() past the view's size drops the view for an
// allocation of its own) - the multi-slice build points the slice's SA / BWT at the full arrays.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  bool owned = true;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes), owned(o.owned) { o.p = nullptr; o.bytes = 0; o.owned = true; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      owned = o.owned;
      o.p = nullptr;
      o.bytes = 0;
      o.owned = true;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p && owned) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    owned = true;
  }
  void view(void* ptr, size_t nbytes) {   // non-owning window [ptr, ptr + nbytes)
    release();
    p = ptr;
    bytes = nbytes;
    owned = false;
  }
  // grow-only allocation (contents not preserved)
  void ensure(size_t nbytes) {
    if (nbytes <= bytes && p) return;
    release();
    size_t b = nbytes ? nbytes : 16;
    hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      throw ApiError{-5, "hipMalloc of " + std::to_string(b) + " bytes failed"};
    }
    bytes = b;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// grow-only pinned host buffer (asynchronous copies in both directions)
// an event owned by a scope: no leak when a HIP call between its creation and its last use throws
struct ScopedEvent {
  hipEvent_t e = nullptr;
  ScopedEvent() { HK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
  ~ScopedEvent() {
    if (e) (void)hipEventDestroy(e);
  }
  ScopedEvent(const ScopedEvent&) = delete;
  ScopedEvent& operator=(const ScopedEvent&) = delete;
  operator hipEvent_t() const { return e; }
};

struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  void ensure(size_t nbytes) {
    if (nbytes <= bytes && p) return;
    release();
    size_t b = nbytes ? nbytes : 16;
    if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      throw ApiError{-5, "hipHostMalloc of " + std::to_string(b) + " bytes failed"};
    }
    bytes = b;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// ----------------------------------------------------- timing registry
struct KernelTimer {
  struct Pending { std::string name; hipEvent_t a, b; double bytes; };
  struct Stat { uint64_t launches = 0; double ms = 0, bytes = 0; };
  bool enabled = false;
  std::vector<Pending> pending;
  std::vector<std::pair<std::string, Stat>> stats;
  std::vector<hipEvent_t> pool;   // resolved events, reused: no event creation on the launch path
  hipStream_t stream = nullptr;

  Stat& stat(const std::string& n) {
    for (auto& s : stats) if (s.first == n) return s.second;
    stats.emplace_back(n, Stat{});
    return stats.back().second;
  }
  // timing events need no system-scope release (the host reads only their timestamps)
  hipEvent_t get() {
    hipEvent_t e = nullptr;
    if (!pool.empty()) {
      e = pool.back();
      pool.pop_back();
    } else {
      HK_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    }
    return e;
  }
  // returns the event to record after the launch (or nullptr when disabled)
  hipEvent_t begin(const std::string& name, double bytes) {
    if (!enabled) return nullptr;
    Pending pd{name, get(), get(), bytes};
    HK_HIP(hipEventRecord(pd.a, stream));
    pending.push_back(pd);
    return pd.b;
  }
  void end(hipEvent_t ev) {
    if (ev) HK_HIP(hipEventRecord(ev, stream));
  }
  void resolve() {
    for (auto& pd : pending) {
      HK_HIP(hipEventSynchronize(pd.b));
      float ms = 0;
      HK_HIP(hipEventElapsedTime(&ms, pd.a, pd.b));
      Stat& s = stat(pd.name);
      s.launches++;
      s.ms += ms;
      s.bytes += pd.bytes;
      pool.push_back(pd.a);
      pool.push_back(pd.b);
    }
    pending.clear();
  }
  void reset() { resolve(); stats.clear(); }
  ~KernelTimer() {
    for (auto& pd : pending) { (void)hipEventDestroy(pd.a); (void)hipEventDestroy(pd.b); }
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};

// RAII scope that brackets one launch with timing events
struct TimedLaunch {
  KernelTimer& t;
  hipEvent_t ev;
  TimedLaunch(KernelTimer& tm, const char* name, double bytes) : t(tm), ev(tm.begin(name, bytes)) {}
  ~TimedLaunch() { if (ev) (void)hipEventRecord(ev, t.stream); }
};

}  // namespace hk
