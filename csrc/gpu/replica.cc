#include "replica.h"

#include <stdexcept>

namespace sca::gpu {

ReplicaUnit::ReplicaUnit(std::vector<std::shared_ptr<BatchedUnit>> replicas) : reps_(std::move(replicas)) {
  if (reps_.empty()) throw std::runtime_error("ReplicaUnit: no replicas");
  picked_.reset(new std::atomic<uint64_t>[reps_.size()]);
  for (size_t i = 0; i < reps_.size(); ++i) picked_[i].store(0);
}

BatchedUnit* ReplicaUnit::pick() {
  const size_t n = reps_.size();
  // Rotate the starting point so ties (idle GPUs) spread round-robin.
  size_t best = rr_.fetch_add(1, std::memory_order_relaxed) % n;
  int64_t best_load = reps_[best]->inflight_rows();
  for (size_t i = 1; i < n && best_load > 0; ++i) {
    const size_t j = (best + i) % n;
    const int64_t l = reps_[j]->inflight_rows();
    if (l < best_load) { best = j; best_load = l; }
  }
  picked_[best].fetch_add(1, std::memory_order_relaxed);
  return reps_[best].get();
}

std::string ReplicaUnit::kind() const { return "replicas" + std::to_string(reps_.size()) + ":" + reps_[0]->kind(); }

bool ReplicaUnit::ready() const {
  for (const auto& r : reps_)
    if (!r->ready()) return false;
  return true;
}

std::vector<uint64_t> ReplicaUnit::requests_per_replica() const {
  std::vector<uint64_t> v(reps_.size());
  for (size_t i = 0; i < reps_.size(); ++i) v[i] = picked_[i].load();
  return v;
}

void ReplicaUnit::stop() {
  for (auto& r : reps_) r->stop();
}

}  // namespace sca::gpu
