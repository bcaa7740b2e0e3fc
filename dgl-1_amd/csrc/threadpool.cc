// Persistent host worker pool behind parallel_for (common.h).
//
// The host kernels (CSR builders, host g-SpMM / g-SDDMM, degree bucketing)
// used to start fresh std::threads on every call, which cost more than the
// work on small graphs (a Cora-sized g-SpMM took 0.28 ms single-threaded
// because spawning was not worth it below 4096 rows). The pool keeps
// default_num_threads() - 1 workers parked on a condition variable:
//  * one job at a time (submissions from several host threads serialise);
//  * a parallel_for issued from inside a job runs inline on that thread;
//  * the first exception thrown by any part of a job is rethrown on the
//    submitting thread after the whole job has finished, so the C-ABI's
//    last-error convention still applies;
//  * after fork() the child builds a fresh pool on first use (the parent's
//    workers do not exist there); the old object is leaked on purpose, as is
//    the process-lifetime pool itself (no joins at interpreter exit).
#include <pthread.h>

#include <algorithm>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace dglhip {
namespace {

thread_local bool tls_in_pool_job = false;

class ThreadPool {
 public:
  explicit ThreadPool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this, i] { loop(i + 1); });
    for (auto& t : threads_) t.detach();
  }

  int size() const { return static_cast<int>(threads_.size()) + 1; }

  // task(tid) for tid in [0, nparts); the caller runs tid 0.
  void run(int nparts, const std::function<void(int)>& task) {
    std::lock_guard<std::mutex> submit(submit_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      task_ = &task;
      nparts_ = nparts;
      pending_ = nparts - 1;
      error_ = nullptr;
      ++generation_;
    }
    cv_start_.notify_all();
    run_part(0);
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [this] { return pending_ == 0; });
    task_ = nullptr;
    if (error_) std::rethrow_exception(error_);
  }

 private:
  void run_part(int tid) {
    tls_in_pool_job = true;
    try {
      (*task_)(tid);
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!error_) error_ = std::current_exception();
    }
    tls_in_pool_job = false;
  }

  void loop(int tid) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_start_.wait(lk, [&] { return generation_ != seen; });
        seen = generation_;
        if (tid >= nparts_) continue;  // not needed for this job
      }
      run_part(tid);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) cv_done_.notify_one();
    }
  }

  std::vector<std::thread> threads_;
  std::mutex submit_mu_, mu_;
  std::condition_variable cv_start_, cv_done_;
  const std::function<void(int)>* task_ = nullptr;
  int nparts_ = 0, pending_ = 0;
  uint64_t generation_ = 0;
  std::exception_ptr error_;
};

ThreadPool* g_pool = nullptr;
std::mutex g_pool_mu;

void reset_after_fork() { g_pool = nullptr; }  // the child's first job builds a new pool

ThreadPool& pool() {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (!g_pool) {
    static bool registered = false;
    if (!registered) {
      pthread_atfork(nullptr, nullptr, reset_after_fork);
      registered = true;
    }
    g_pool = new ThreadPool(std::max(0, default_num_threads() - 1));
  }
  return *g_pool;
}

}  // namespace

bool in_parallel_region() { return tls_in_pool_job; }

int pool_run(int nparts, const std::function<void(int)>& task) {
  ThreadPool& p = pool();
  const int parts = std::min(nparts, p.size());
  p.run(parts, task);
  return parts;
}

}  // namespace dglhip
