// A small persistent host thread pool for the per-window host folds (point
// operations on the host: each window's sum is ~30 independent point ops).
// Spawning a std::thread per window per MSM cost ~20 us a thread -- as much as
// the work -- so the workers are created once and reused; parallel_for blocks
// until every index ran.  Calls from several host threads (one per context)
// are serialised on the pool.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ecg {

class HostPool {
 public:
  static HostPool& get() {
    static HostPool pool;
    return pool;
  }

  // fn(i) for i < n, on the workers and the calling thread
  void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    if (n == 1 || workers_.empty()) {
      for (size_t i = 0; i < n; i++) fn(i);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_ = workers_.size();
      gen_++;
    }
    cv_.notify_all();
    run();  // the caller takes indices too
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  HostPool() {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned nw = std::min(15u, hw > 1 ? hw - 1 : 0u);
    for (unsigned i = 0; i < nw; i++) workers_.emplace_back([this] { loop(); });
  }

  void run() {
    for (size_t i = next_.fetch_add(1); i < n_; i = next_.fetch_add(1)) (*fn_)(i);
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      run();
      std::lock_guard<std::mutex> g(mu_);
      if (--busy_ == 0) done_cv_.notify_one();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  size_t busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace ecg
