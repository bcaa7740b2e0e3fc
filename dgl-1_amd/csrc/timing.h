// Bench support shared by the kernels' launchers: hipEvent pairs around each
// launch, on the launch stream, while timing is enabled (dglhip_timing_*).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "common.h"

#ifndef HIP_CALL
#define HIP_CALL(expr)                                                      \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    DGLHIP_CHECK(_e == hipSuccess, #expr << " -> " << hipGetErrorString(_e)); \
  } while (0)
#endif

namespace dglhip {

struct Timing {
  std::mutex mu;
  bool enabled = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  double total_ms = 0.0;
  int64_t launches = 0;
};
extern Timing g_timing;


static inline std::pair<hipEvent_t, hipEvent_t> take_events() {
  if (!g_timing.pool.empty()) {
    auto p = g_timing.pool.back();
    g_timing.pool.pop_back();
    return p;
  }
  std::pair<hipEvent_t, hipEvent_t> p;
  HIP_CALL(hipEventCreate(&p.first));
  HIP_CALL(hipEventCreate(&p.second));
  return p;
}

template <typename LaunchFn>
static inline void timed_launch(hipStream_t stream, LaunchFn&& fn) {
  std::unique_lock<std::mutex> lk(g_timing.mu);
  if (!g_timing.enabled) {
    lk.unlock();
    fn();
    HIP_CALL(hipGetLastError());
    return;
  }
  auto ev = take_events();
  HIP_CALL(hipEventRecord(ev.first, stream));
  fn();
  HIP_CALL(hipGetLastError());
  HIP_CALL(hipEventRecord(ev.second, stream));
  g_timing.pending.push_back(ev);
}

}  // namespace dglhip
