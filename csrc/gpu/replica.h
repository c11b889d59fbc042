// Data-parallel GPU replicas of one graph node.
//
// The reference scales a predictor by running `replicas` identical pods behind
// a Kubernetes Service (seldon_deployment.proto:57, seldondeployment_controller.go:296-302)
// with kube-proxy picking a pod per connection.  In-process, a node bound to N
// GPUs holds one micro-batching BatchedUnit per GPU (each with its own copy of
// the parameters in that GPU's HBM) and sends every request to the replica
// with the fewest rows in flight -- join-shortest-queue, which keeps every
// GPU's batches similarly sized instead of hashing connections.
//
// Failure handling ("drop a failed replica from the scheduler and
// re-route"): replicas whose circuit is open (BatchedUnit::healthy) get no new
// requests while a healthy one exists, and a request that fails with a device
// fault (launch/execution error, hang watchdog) is re-run on another healthy
// replica, up to `max_retries` times -- the in-process counterpart of the
// engine's REST retries (InternalPredictionService.java:388-452) and
// Ambassador's connect-failure retry (ambassador.go:84-87).
#pragma once

#include <atomic>
#include <memory>
#include <vector>

#include "batcher.h"

namespace sca::gpu {

class ReplicaUnit : public Unit {
 public:
  explicit ReplicaUnit(std::vector<std::shared_ptr<BatchedUnit>> replicas, int max_retries = 1);

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override { submit(c, std::move(in), std::move(k), 0, -1); }
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { submit(c, std::move(in), std::move(k), 0, -1); }
  std::string kind() const override;
  // Degraded but serving while any replica is healthy.
  bool ready() const override;

  const std::vector<std::shared_ptr<BatchedUnit>>& replicas() const { return reps_; }
  std::vector<uint64_t> requests_per_replica() const;
  uint64_t retries() const { return retries_.load(); }
  void stop();
  void collect_metrics(MetricsRegistry& m, const Labels& labels) const override {
    for (size_t i = 0; i < reps_.size(); ++i) {
      Labels l = labels;
      l.emplace_back("replica", std::to_string(i));
      reps_[i]->collect_metrics(m, l);
    }
    m.counter("seldon_replica_retries", labels)->set(double(retries()));
  }

 private:
  int pick(int exclude);
  void submit(const CallCtx& c, MsgPtr in, Done k, int attempt, int exclude);
  std::vector<std::shared_ptr<BatchedUnit>> reps_;
  int max_retries_;
  std::atomic<uint32_t> rr_{0};
  std::atomic<uint64_t> retries_{0};
  std::unique_ptr<std::atomic<uint64_t>[]> picked_;
};

}  // namespace sca::gpu
