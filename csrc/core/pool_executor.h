// A small process-wide thread pool for request continuations that have no
// front-end thread of their own: graphs evaluated through the Python API
// (Deployment.predict / predict_pb).  Without it such a request continues on
// whichever thread completed its last unit -- a GPU pump -- so the graph walk,
// meta merge and serialisation of Python-API requests would delay the pump's
// next launch.  (Python nodes never run on these threads either way: a PyUnit
// has its own work-queue threads, csrc/bindings/py_unit.h.)
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

// Elastic: a post that finds no idle thread starts another (up to kMax), so
// a slow continuation never holds up unrelated ones.
class PoolExecutor : public Executor {
 public:
  static constexpr int kMax = 64;
  explicit PoolExecutor(int threads) {
    std::lock_guard<std::mutex> g(mu_);
    for (int i = 0; i < threads; ++i) spawn();
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
      if (idle_ < int(q_.size()) && int(ths_.size()) < kMax) spawn();
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
  void spawn() { ths_.emplace_back([this] { loop(); }); }  // caller holds mu_
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      ++idle_;
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      --idle_;
      if (q_.empty()) return;
      std::function<void()> fn = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      fn();
      lk.lock();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  int idle_ = 0;  // threads waiting for work (guarded by mu_)
  std::vector<std::thread> ths_;
};

}  // namespace sca
