// Data-parallel GPU replicas of one graph node.
//
// The reference scales a predictor by running `replicas` identical pods behind
// a Kubernetes Service (seldon_deployment.proto:57, seldondeployment_controller.go:296-302)
// with kube-proxy picking a pod per connection.  In-process, a node bound to N
// GPUs holds one micro-batching BatchedUnit per GPU (each with its own copy of
// the parameters in that GPU's HBM) and sends every request to the replica
// with the fewest rows in flight -- join-shortest-queue, which keeps every
// GPU's batches similarly sized instead of hashing connections.
#pragma once

#include <atomic>
#include <memory>
#include <vector>

#include "batcher.h"

namespace sca::gpu {

class ReplicaUnit : public Unit {
 public:
  explicit ReplicaUnit(std::vector<std::shared_ptr<BatchedUnit>> replicas);

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override { pick()->transform_input(c, std::move(in), std::move(k)); }
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { pick()->transform_output(c, std::move(in), std::move(k)); }
  std::string kind() const override;
  bool ready() const override;

  const std::vector<std::shared_ptr<BatchedUnit>>& replicas() const { return reps_; }
  std::vector<uint64_t> requests_per_replica() const;
  void stop();
  void collect_metrics(MetricsRegistry& m, const Labels& labels) const override {
    for (size_t i = 0; i < reps_.size(); ++i) {
      Labels l = labels;
      l.emplace_back("replica", std::to_string(i));
      reps_[i]->collect_metrics(m, l);
    }
  }

 private:
  BatchedUnit* pick();
  std::vector<std::shared_ptr<BatchedUnit>> reps_;
  std::atomic<uint32_t> rr_{0};
  std::unique_ptr<std::atomic<uint64_t>[]> picked_;
};

}  // namespace sca::gpu
