// Multi-armed-bandit router units (reference components/routers/
// epsilon-greedy/EpsilonGreedy.py and thompson-sampling/ThompsonSampling.py).
//
// Routing decisions for concurrent requests are micro-batched through the
// same GPU batcher as models: one bandit kernel launch decides every queued
// request (csrc/kernels/bandit.hip).  Feedback updates the host-authoritative
// state under a mutex; the state lives in fine-grained pinned memory that the
// kernel reads directly, so an update is visible to the next launch without a
// copy.
#pragma once

#include <atomic>
#include <mutex>
#include <random>

#include "batcher.h"
#include "models.h"

namespace sca::gpu {

class BanditModel : public RowModel {
 public:
  enum Kind { kEpsilonGreedy = 0, kThompson = 1 };
  static constexpr int kMaxBranches = 256;
  BanditModel(Kind kind, int n_branches, float epsilon, int64_t seed, int best_branch);
  std::string name() const override { return kind_ == kEpsilonGreedy ? "epsilon_greedy" : "thompson_sampling"; }
  int in_cols() const override { return 0; }
  int out_cols(int) const override { return 1; }
  void to_device(int device) override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;

  // Reward update (EpsilonGreedy.send_feedback / ThompsonSampling.send_feedback).
  void feedback(int routing, int n_success, int n_failures);
  int n_branches() const { return nb_; }
  std::string snapshot() const;
  void restore(const std::string& s);
  std::vector<double> values() const;
  int best_branch() const;
  // Epsilon-greedy decision for the next request on the host: the same
  // Philox stream (seed, request counter) and rule as eg_route_kernel, so
  // the decision sequence is identical to the batched device path's.
  bool host_routable() const { return kind_ == kEpsilonGreedy; }
  int route_host();

  // Cross-process state (serve --gpus N runs one engine process per GPU and
  // the reference keeps ONE router object per deployment,
  // EpsilonGreedy.py:87-130): the counters and the best branch live in the
  // shared mapping `name` (POSIX shm, created by the first attacher, which
  // seeds it with its own state), so every worker learns from every
  // worker's feedback and routes by the same best branch.  `worker` mixes
  // into the Philox seed so workers draw different random streams.
  void attach_shared(const std::string& name, int worker);
  bool shared() const { return shm_ != nullptr; }
  ~BanditModel() override;

 private:
  struct Shared;
  void pull_shared();         // shared -> local + pinned (mu_ held)
  void maybe_pull() const;    // pull if another worker updated the shared state
  void update_locked(int routing, int n_success, int n_failures);  // the reference's update rule (mu_ held)
  struct State {
    int32_t best;
    int32_t pad[3];
    float alpha[kMaxBranches];
    float beta[kMaxBranches];
  };
  void publish();  // host state -> pinned state (mutex held)
  Kind kind_;
  int nb_;
  float eps_;
  uint64_t seed_;
  mutable std::mutex mu_;
  mutable std::mt19937_64 rng_;
  std::vector<int64_t> success_, tries_;
  std::vector<double> values_;
  int best_ = 0;
  std::vector<double> a_, b_;
  PinnedBuffer state_;
  State host_state_{};
  std::atomic<int> best_pub_{0};  // published best branch (host route)
  std::atomic<uint64_t> offset_{0};
  Shared* shm_ = nullptr;
  mutable std::atomic<uint64_t> seen_version_{0};
};

class BanditRouterUnit : public Unit {
 public:
  // device_route: decide through the micro-batched bandit kernel (one GPU
  // round trip per routed request).  Otherwise an epsilon-greedy router
  // decides on the caller's thread with the kernel's Philox stream: a
  // routed request then costs one GPU round trip (its branch) instead of two
  // (profiles/r03j_router).  Thompson sampling always uses the kernel.
  BanditRouterUnit(std::shared_ptr<BanditModel> model, BatcherOptions opts, bool device_route = false);
  std::string kind() const override {
    if (host_route_) return "host:" + model_->name();
    return (opts_.device >= 0 ? "gpu:" : "cpu:") + model_->name();
  }
  void route(const CallCtx& c, MsgPtr in, Done k) override;
  void send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) override;
  std::string snapshot() const override { return model_->snapshot(); }
  void restore(const std::string& s) override { model_->restore(s); }
  std::shared_ptr<BanditModel> model() const { return model_; }
  std::shared_ptr<BatchedUnit> batcher() const { return batched_; }

 private:
  std::shared_ptr<BanditModel> model_;
  BatcherOptions opts_;
  std::shared_ptr<BatchedUnit> batched_;
  bool host_route_ = false;
};

}  // namespace sca::gpu
