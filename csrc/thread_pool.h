// mxstream — a small persistent worker pool (host side): run(n, f) calls f(0..n-1) on the
// workers and the calling thread and returns when every task is done. Used where a call is
// split into pieces every step or chunk (the sharded session store, the text file reader):
// starting threads per call cost more than the pieces themselves on the GPU box.
#pragma once
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mxs {

// Fixed workers; run(n, f) calls f(0..n-1) across them and the calling thread, returns when all
// tasks are done. One run at a time (the store's callers are serialised by the operator).
class WorkerPool {
 public:
  explicit WorkerPool(int workers) {
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      ntask_ = n;
      next_.store(0);
      left_ = n;
      err_ = nullptr;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return left_ == 0; });
    job_ = nullptr;
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void work() {
    for (;;) {
      const int i = next_.fetch_add(1);
      if (i >= ntask_) return;
      try {
        (*job_)(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(mu_);
        if (!err_) err_ = std::current_exception();
      }
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        if (!job_) continue;
      }
      work();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  std::atomic<int> next_{0};
  int ntask_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};


}  // namespace mxs
