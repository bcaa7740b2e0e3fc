// Shared helpers for libdgl_hip: error state, argument checks, host threads.
//
// The error convention restates the reference runtime's: a C entry point runs
// its body inside API_BEGIN/API_END; any exception becomes a thread-local
// message plus a -1 return (src/runtime/runtime_base.h:13-32,
// src/runtime/c_runtime_api.cc:130-145).
#pragma once

#include <algorithm>
#include <cstdint>
#include <functional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace dglhip {

void set_last_error(const std::string& msg);

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

#define DGLHIP_CHECK(cond, msg_expr)                                  \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::ostringstream _os;                                         \
      _os << "[dgl_hip] check failed: " #cond ": " << msg_expr;       \
      throw ::dglhip::Error(_os.str());                               \
    }                                                                 \
  } while (0)

#define API_BEGIN() try {
#define API_END()                                          \
  }                                                        \
  catch (const std::exception& _e) {                       \
    ::dglhip::set_last_error(_e.what());                   \
    return -1;                                             \
  }                                                        \
  return 0;

// Number of host worker threads: DGL_NUM_THREADS / OMP_NUM_THREADS (the
// reference's knobs, src/runtime/threading_backend.cc:200-202), else the
// hardware concurrency, capped at 64.
int default_num_threads();

// Persistent worker pool (threadpool.cc). pool_run executes task(tid) for tid
// in [0, min(nparts, pool size)) and returns the number of parts it used; the
// first exception from any part is rethrown here.
bool in_parallel_region();
int pool_run(int nparts, const std::function<void(int)>& task);

// Static partition of [0, n) over up to `nthreads` pool workers; fn(begin, end,
// tid). Ranges shorter than `min_n` items (each item being cheap), single-thread
// requests and calls made from inside a running parallel_for execute inline;
// pass min_n = 2 when every item is a large task.
template <typename Fn>
void parallel_for(int64_t n, int nthreads, Fn&& fn, int64_t min_n = 256) {
  if (nthreads <= 1 || n < min_n || in_parallel_region()) {
    fn(int64_t(0), n, 0);
    return;
  }
  if (nthreads > n) nthreads = static_cast<int>(n);
  const int64_t chunk = (n + nthreads - 1) / nthreads;
  const std::function<void(int)> task = [&](int t) {
    const int64_t b = t * chunk, e = std::min<int64_t>(n, b + chunk);
    if (b < e) fn(b, e, t);
  };
  const int used = pool_run(nthreads, task);
  if (used < nthreads) {  // pool smaller than asked: finish the remaining chunks here
    for (int t = used; t < nthreads; ++t) task(t);
  }
}

}  // namespace dglhip
