// A small process-wide thread pool for request continuations that have no
// front-end thread of their own: graphs evaluated through the Python API
// (Deployment.predict / predict_pb / feedback).  Without it such a request
// continues on whichever thread completed its last unit -- a GPU pump -- and a
// later node that waits synchronously on a GPU unit of the same pump (a
// Python transformer calling a device detector) would wait for itself.
#pragma once

#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "engine.h"

namespace sca {

class PoolExecutor : public Executor {
 public:
  explicit PoolExecutor(int threads) {
    for (int i = 0; i < threads; ++i) ths_.emplace_back([this] { loop(); });
  }
  ~PoolExecutor() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : ths_)
      if (t.joinable()) t.join();
  }
  void post(std::function<void()> fn) override {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(fn));
    }
    cv_.notify_one();
  }
  // Process lifetime (never destroyed: continuations may be posted while
  // static destructors run at interpreter exit).
  static const std::shared_ptr<PoolExecutor>& shared() {
    static auto* p = new std::shared_ptr<PoolExecutor>(std::make_shared<PoolExecutor>(2));
    return *p;
  }

 private:
  void loop() {
    while (true) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        fn = std::move(q_.front());
        q_.pop_front();
      }
      fn();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::vector<std::thread> ths_;
};

}  // namespace sca
