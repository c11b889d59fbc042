#include "replica.h"

#include <stdexcept>

namespace sca::gpu {

ReplicaUnit::ReplicaUnit(std::vector<std::shared_ptr<BatchedUnit>> replicas, int max_retries)
    : reps_(std::move(replicas)), max_retries_(max_retries < 0 ? 0 : max_retries) {
  if (reps_.empty()) throw std::runtime_error("ReplicaUnit: no replicas");
  picked_.reset(new std::atomic<uint64_t>[reps_.size()]);
  for (size_t i = 0; i < reps_.size(); ++i) picked_[i].store(0);
}

int ReplicaUnit::pick(int exclude) {
  const int n = int(reps_.size());
  if (n == 1) {
    picked_[0].fetch_add(1, std::memory_order_relaxed);
    return 0;
  }
  // Rotate the starting point so ties (idle GPUs) spread round-robin; healthy
  // replicas first, then (all tripped) the least loaded one anyway -- its
  // cooldown may be over by the time the batch launches.
  const int start = int(rr_.fetch_add(1, std::memory_order_relaxed) % uint32_t(n));
  int best = -1, fallback = -1;
  int64_t best_load = 0, fallback_load = 0;
  for (int d = 0; d < n; ++d) {
    const int j = (start + d) % n;
    if (j == exclude) continue;
    const int64_t l = reps_[j]->inflight_rows();
    if (reps_[j]->healthy()) {
      if (best < 0 || l < best_load) { best = j; best_load = l; }
      if (best_load == 0) break;
    } else if (fallback < 0 || l < fallback_load) {
      fallback = j;
      fallback_load = l;
    }
  }
  if (best < 0) best = fallback >= 0 ? fallback : (exclude >= 0 ? exclude : 0);
  picked_[best].fetch_add(1, std::memory_order_relaxed);
  return best;
}

void ReplicaUnit::submit(const CallCtx& c, MsgPtr in, Done k, int attempt, int exclude) {
  const int i = pick(exclude);
  BatchedUnit* r = reps_[size_t(i)].get();
  if (attempt >= max_retries_ || reps_.size() < 2) {
    r->transform_input(c, std::move(in), std::move(k));
    return;
  }
  // Keep the request so a device fault can re-run it elsewhere (the batcher
  // never mutates its input message).
  r->transform_input(c, in, [this, cc = c, in, k = std::move(k), attempt, i](Outcome o) mutable {
    if (o.err && o.err->device_fault) {
      bool other = false;
      for (size_t j = 0; j < reps_.size() && !other; ++j) other = int(j) != i && reps_[j]->healthy();
      if (other) {
        retries_.fetch_add(1, std::memory_order_relaxed);
        submit(cc, std::move(in), std::move(k), attempt + 1, i);
        return;
      }
    }
    k(std::move(o));
  });
}

std::string ReplicaUnit::kind() const { return "replicas" + std::to_string(reps_.size()) + ":" + reps_[0]->kind(); }

bool ReplicaUnit::ready() const {
  for (const auto& r : reps_)
    if (r->ready()) return true;
  return false;
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
