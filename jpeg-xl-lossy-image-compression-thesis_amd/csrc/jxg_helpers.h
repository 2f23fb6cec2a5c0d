// jxg_helpers.h -- the streaming pipeline's helper threads (jxg_host.cpp):
// a fixed pool that runs the per-frame code builds (clustering, ANS tables,
// headers, LF-group codes) off the submitting thread.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/jxg.h"

namespace jxg {

// Helper threads of a pipeline: persistent (a std::async thread per frame cost
// its creation on the submitting thread every frame), HIP device set once.
class Helpers {
 public:
  Helpers(int dev, int n) {
    try {
      for (int i = 0; i < n; i++) start(dev);
    } catch (...) {  // no thread: stop the ones started, the caller builds inline
      stop_all();
      throw;
    }
  }
  ~Helpers() { stop_all(); }
  std::future<jxg_status> run(std::function<jxg_status()> f) {
    std::packaged_task<jxg_status()> job(std::move(f));
    std::future<jxg_status> fut = job.get_future();
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(job));
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void start(int dev) {
    t_.emplace_back([this, dev]() {
      (void)hipSetDevice(dev);
      for (;;) {
        std::packaged_task<jxg_status()> job;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [this]() { return stop_ || !q_.empty(); });
          if (q_.empty()) return;  // stop_, nothing left
          job = std::move(q_.front());
          q_.pop_front();
        }
        job();
      }
    });
  }
  void stop_all() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : t_) t.join();
    t_.clear();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::packaged_task<jxg_status()>> q_;
  std::vector<std::thread> t_;
  bool stop_ = false;
};

}  // namespace jxg
