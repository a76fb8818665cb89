// host_pool.h -- the context's host worker threads (pipeline.cpp): the
// per-commit plan, pinned-staging pack and verdict replay of a large
// cmtv_verify_commits call are split over them. One parallel_for at a time
// (the pipeline's bulk lock serialises its users); the calling thread works
// too, so a pool of n threads has n - 1 workers.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace cmtv {

class HostPool {
 public:
  explicit HostPool(unsigned threads) {
    // a thread that cannot be created (container thread limits) leaves the
    // pool smaller, never a half-built one: the calling thread always works
    for (unsigned i = 1; i < threads; i++) {
      try {
        workers_.emplace_back([this] { run(); });
      } catch (...) {
        break;
      }
    }
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;

  unsigned threads() const { return (unsigned)workers_.size() + 1; }

  // fn(begin, end) over [0, n) in blocks of `grain` items, on every thread;
  // returns once all blocks are done.
  void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
    if (n == 0) return;
    if (grain == 0) grain = 1;
    if (workers_.empty() || n <= grain) {
      fn(0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      grain_ = grain;
      next_.store(0, std::memory_order_relaxed);
      busy_ = (unsigned)workers_.size();
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const size_t b = next_.fetch_add(grain_, std::memory_order_relaxed);
      if (b >= n_) return;
      (*fn_)(b, b + grain_ < n_ ? b + grain_ : n_);
    }
  }
  void run() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_one();
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  uint64_t gen_ = 0;
  unsigned busy_ = 0;
  const std::function<void(size_t, size_t)>* fn_ = nullptr;
  size_t n_ = 0, grain_ = 1;
  std::atomic<size_t> next_{0};
};

}  // namespace cmtv
