// mxstream — a small persistent worker pool (host side): run(n, f) calls f(0..n-1) on the
// workers and the calling thread and returns when every task is done. Used where a call is
// split into pieces every step or chunk (the sharded session store, the text file reader):
// starting threads per call cost more than the pieces themselves on the GPU box.
#pragma once
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
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
  int workers() const { return (int)th_.size(); }
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    // Each run gets its own task counter: a worker still inside work() from an earlier run
    // holds that run's Job, whose counter is exhausted, so it can never take (or double-count)
    // a task index of this one.
    auto job = std::make_shared<Job>();
    job->f = &f;
    job->n = n;
    job->left = n;
    {
      std::lock_guard<std::mutex> g(mu_);
      cur_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return job->left == 0; });
    cur_.reset();
    if (job->err) std::rethrow_exception(job->err);
  }

 private:
  struct Job {
    const std::function<void(int)>* f = nullptr;
    int n = 0;
    std::atomic<int> next{0};
    int left = 0;  // guarded by mu_
    std::exception_ptr err;
  };
  void work(Job& j) {
    for (;;) {
      const int i = j.next.fetch_add(1);
      if (i >= j.n) return;
      try {
        (*j.f)(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(mu_);
        if (!j.err) j.err = std::current_exception();
      }
      std::lock_guard<std::mutex> g(mu_);
      if (--j.left == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        j = cur_;
      }
      if (j) work(*j);
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Job> cur_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};


}  // namespace mxs
