// Shared helpers for libdgl_hip: error state, argument checks, host threads.
//
// The error convention restates the reference runtime's: a C entry point runs
// its body inside API_BEGIN/API_END; any exception becomes a thread-local
// message plus a -1 return (src/runtime/runtime_base.h:13-32,
// src/runtime/c_runtime_api.cc:130-145).
#pragma once

#include <cstdint>
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

// Static partition of [0, n) over `nthreads` std::threads; fn(begin, end, tid).
template <typename Fn>
void parallel_for(int64_t n, int nthreads, Fn&& fn) {
  if (nthreads <= 1 || n < 4096) {
    fn(int64_t(0), n, 0);
    return;
  }
  if (nthreads > n) nthreads = static_cast<int>(n);
  std::vector<std::thread> pool;
  pool.reserve(nthreads - 1);
  const int64_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 1; t < nthreads; ++t) {
    const int64_t b = t * chunk, e = std::min<int64_t>(n, b + chunk);
    if (b >= e) break;
    pool.emplace_back([&fn, b, e, t] { fn(b, e, t); });
  }
  fn(int64_t(0), std::min<int64_t>(n, chunk), 0);
  for (auto& th : pool) th.join();
}

}  // namespace dglhip
