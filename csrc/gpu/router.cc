#include "router.h"

#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <sstream>
#include <thread>

#include "../kernels/philox.h"

namespace sca::gpu {

// One bandit's state shared by the engine processes of a host.  Updates take
// a robust process-shared mutex in the mapping (feedback is rare next to
// routing, and the critical section is a few hundred nanoseconds); readers
// compare `version` with the last one they pulled.  A lock whose owner
// process died inside the critical section passes to the next waiter
// (ShmLock, EOWNERDEAD).
struct BanditModel::Shared {
  std::atomic<uint32_t> init;  // 0 fresh, 1 being seeded, 2 ready
  pthread_mutex_t mu;          // process-shared, robust (initialised by the seeding worker)
  std::atomic<uint64_t> version;
  std::atomic<int32_t> best;
  int32_t kind, nb;
  int64_t success[kMaxBranches], tries[kMaxBranches];
  double values[kMaxBranches], alpha[kMaxBranches], beta[kMaxBranches];
};

namespace {
// A robust process-shared mutex in the mapping: the kernel hands a lock
// whose owner died inside the critical section to the next waiter with
// EOWNERDEAD (no PID liveness guess, which fails across PID namespaces and
// on PID reuse).  The dead owner's partial update is at most one feedback's
// counters; the state is marked consistent and used as is.
struct ShmLock {
  pthread_mutex_t* m;
  explicit ShmLock(pthread_mutex_t& mu) : m(&mu) {
    const int r = pthread_mutex_lock(m);
    if (r == EOWNERDEAD) pthread_mutex_consistent(m);
    else if (r != 0) throw std::runtime_error(std::string("bandit: shared lock failed: ") + std::strerror(r));
  }
  ~ShmLock() { pthread_mutex_unlock(m); }
};

void init_shared_mutex(pthread_mutex_t* m) {
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  const int r = pthread_mutex_init(m, &a);
  pthread_mutexattr_destroy(&a);
  if (r != 0) throw std::runtime_error(std::string("bandit: shared mutex init failed: ") + std::strerror(r));
}
}  // namespace

BanditModel::~BanditModel() {
  if (shm_) munmap(shm_, sizeof(Shared));
}

void BanditModel::attach_shared(const std::string& name, int worker) {
  if (shm_) return;
  const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("bandit: shm_open(" + name + ") failed: " + std::strerror(errno));
  if (ftruncate(fd, off_t(sizeof(Shared))) != 0) {
    ::close(fd);
    throw std::runtime_error(std::string("bandit: ftruncate failed: ") + std::strerror(errno));
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) throw std::runtime_error(std::string("bandit: mmap failed: ") + std::strerror(errno));
  auto* sh = static_cast<Shared*>(p);
  uint32_t fresh = 0;
  std::lock_guard<std::mutex> g(mu_);
  if (sh->init.compare_exchange_strong(fresh, 1)) {  // first worker seeds the shared state with its own
    init_shared_mutex(&sh->mu);
    sh->kind = int32_t(kind_);
    sh->nb = nb_;
    for (int i = 0; i < nb_; ++i) {
      sh->success[i] = success_[size_t(i)];
      sh->tries[i] = tries_[size_t(i)];
      sh->values[i] = values_[size_t(i)];
      sh->alpha[i] = a_[size_t(i)];
      sh->beta[i] = b_[size_t(i)];
    }
    sh->best.store(best_);
    sh->version.store(1);
    sh->init.store(2, std::memory_order_release);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (sh->init.load(std::memory_order_acquire) != 2) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        munmap(p, sizeof(Shared));
        throw std::runtime_error("bandit: shared state " + name + " never became ready");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    if (sh->kind != int32_t(kind_) || sh->nb != nb_) {
      munmap(p, sizeof(Shared));
      throw std::runtime_error("bandit: shared state " + name + " belongs to a different router");
    }
  }
  shm_ = sh;
  seed_ ^= 0x9E3779B97F4A7C15ull * uint64_t(worker + 1);
  rng_.seed(seed_);
  pull_shared();
}

void BanditModel::pull_shared() {
  ShmLock l(shm_->mu);
  for (int i = 0; i < nb_; ++i) {
    success_[size_t(i)] = shm_->success[i];
    tries_[size_t(i)] = shm_->tries[i];
    values_[size_t(i)] = shm_->values[i];
    a_[size_t(i)] = shm_->alpha[i];
    b_[size_t(i)] = shm_->beta[i];
  }
  best_ = shm_->best.load(std::memory_order_relaxed);
  seen_version_.store(shm_->version.load(std::memory_order_relaxed), std::memory_order_relaxed);
  publish();
}

void BanditModel::maybe_pull() const {
  if (!shm_ || shm_->version.load(std::memory_order_acquire) == seen_version_.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> g(mu_);
  const_cast<BanditModel*>(this)->pull_shared();
}

BanditModel::BanditModel(Kind kind, int n_branches, float epsilon, int64_t seed, int best_branch)
    : kind_(kind), nb_(n_branches), eps_(epsilon) {
  if (n_branches < 1 || n_branches > kMaxBranches)
    throw std::runtime_error("bandit router: n_branches must be in [1, " + std::to_string(kMaxBranches) + "]");
  seed_ = seed >= 0 ? uint64_t(seed) : std::random_device()() ^ (uint64_t(std::random_device()()) << 32);
  rng_.seed(seed_);
  success_.assign(size_t(nb_), 0);
  tries_.assign(size_t(nb_), 0);
  values_.assign(size_t(nb_), 0.0);
  a_.assign(size_t(nb_), 1.0);
  b_.assign(size_t(nb_), 1.0);
  if (best_branch >= 0 && best_branch < nb_) best_ = best_branch;
  else best_ = int(rng_() % uint64_t(nb_));  // EpsilonGreedy: random starting branch
  std::lock_guard<std::mutex> g(mu_);
  publish();
}

void BanditModel::publish() {
  host_state_.best = best_;
  best_pub_.store(best_, std::memory_order_release);
  for (int i = 0; i < nb_; ++i) {
    host_state_.alpha[i] = float(a_[size_t(i)]);
    host_state_.beta[i] = float(b_[size_t(i)]);
  }
  if (state_.bytes()) memcpy(state_.host<State>(), &host_state_, sizeof(State));
}

void BanditModel::to_device(int) {
  std::lock_guard<std::mutex> g(mu_);
  state_.alloc(sizeof(State));
  publish();
}

void BanditModel::launch(const double*, int rows, int, double* out, void*, hipStream_t s) {
  maybe_pull();
  const uint64_t off = offset_.fetch_add(uint64_t(rows));
  State* st = state_.dev<State>();
  if (kind_ == kEpsilonGreedy)
    kern::eg_route(&st->best, nb_, eps_, seed_, off, rows, out, s);
  else
    kern::ts_route(st->alpha, st->beta, nb_, seed_, off, rows, out, s);
}

int BanditModel::route_host() {
  const uint64_t off = offset_.fetch_add(1, std::memory_order_relaxed);
  kern::Philox rng(seed_, off);
  const int b = shm_ ? shm_->best.load(std::memory_order_acquire) : best_pub_.load(std::memory_order_acquire);
  int pick = b;
  if (nb_ > 1 && rng.uniform() <= eps_) {
    int other = int(rng.next() % uint32_t(nb_ - 1));
    if (other >= b) ++other;
    pick = other;
  }
  return pick;
}

void BanditModel::run_cpu(const double*, int rows, int, double* out) const {
  maybe_pull();
  std::lock_guard<std::mutex> g(mu_);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int r = 0; r < rows; ++r) {
    if (kind_ == kEpsilonGreedy) {
      int pick = best_;
      if (nb_ > 1 && !(U(rng_) > eps_)) {
        int other = int(rng_() % uint64_t(nb_ - 1));
        if (other >= best_) ++other;
        pick = other;
      }
      out[r] = pick;
    } else {
      double best = -1;
      int pick = 0;
      for (int i = 0; i < nb_; ++i) {
        std::gamma_distribution<double> ga(a_[size_t(i)], 1.0), gb(b_[size_t(i)], 1.0);
        const double x = ga(rng_), y = gb(rng_);
        const double v = x / (x + y);
        if (v > best) { best = v; pick = i; }
      }
      out[r] = pick;
    }
  }
}

void BanditModel::feedback(int routing, int n_success, int n_failures) {
  if (routing < 0 || routing >= nb_) throw std::runtime_error("bandit feedback: invalid routing " + std::to_string(routing));
  std::lock_guard<std::mutex> g(mu_);
  if (shm_) {  // the update happens on the shared counters, under their lock
    ShmLock l(shm_->mu);
    for (int i = 0; i < nb_; ++i) {
      success_[size_t(i)] = shm_->success[i];
      tries_[size_t(i)] = shm_->tries[i];
      a_[size_t(i)] = shm_->alpha[i];
      b_[size_t(i)] = shm_->beta[i];
      values_[size_t(i)] = shm_->values[i];
    }
    update_locked(routing, n_success, n_failures);
    shm_->success[routing] = success_[size_t(routing)];
    shm_->tries[routing] = tries_[size_t(routing)];
    shm_->values[routing] = values_[size_t(routing)];
    shm_->alpha[routing] = a_[size_t(routing)];
    shm_->beta[routing] = b_[size_t(routing)];
    shm_->best.store(best_, std::memory_order_release);
    seen_version_.store(shm_->version.fetch_add(1, std::memory_order_acq_rel) + 1, std::memory_order_relaxed);
  } else {
    update_locked(routing, n_success, n_failures);
  }
  publish();
}

void BanditModel::update_locked(int routing, int n_success, int n_failures) {
  success_[size_t(routing)] += n_success;
  tries_[size_t(routing)] += n_success + n_failures;
  if (kind_ == kEpsilonGreedy) {
    if (tries_[size_t(routing)] > 0)
      values_[size_t(routing)] = double(success_[size_t(routing)]) / double(tries_[size_t(routing)]);
    double mx = values_[0];
    for (double v : values_) mx = std::max(mx, v);
    std::vector<int> ties;
    for (int i = 0; i < nb_; ++i)
      if (values_[size_t(i)] == mx) ties.push_back(i);
    best_ = ties[size_t(rng_() % ties.size())];  // break ties randomly
  } else {
    a_[size_t(routing)] += n_success;
    b_[size_t(routing)] += n_failures;
  }
}

std::vector<double> BanditModel::values() const {
  maybe_pull();
  std::lock_guard<std::mutex> g(mu_);
  return values_;
}

int BanditModel::best_branch() const {
  maybe_pull();
  std::lock_guard<std::mutex> g(mu_);
  return best_;
}

std::string BanditModel::snapshot() const {
  maybe_pull();
  std::lock_guard<std::mutex> g(mu_);
  std::ostringstream o;
  o.precision(17);
  // version: the shared state's version this snapshot reflects (restore)
  const uint64_t ver = shm_ ? shm_->version.load(std::memory_order_acquire) : seen_version_.load();
  o << "{\"kind\":" << int(kind_) << ",\"best\":" << best_ << ",\"offset\":" << offset_.load()
    << ",\"version\":" << ver << ",\"success\":[";
  for (int i = 0; i < nb_; ++i) o << (i ? "," : "") << success_[size_t(i)];
  o << "],\"tries\":[";
  for (int i = 0; i < nb_; ++i) o << (i ? "," : "") << tries_[size_t(i)];
  o << "],\"values\":[";
  for (int i = 0; i < nb_; ++i) o << (i ? "," : "") << values_[size_t(i)];
  o << "],\"alpha\":[";
  for (int i = 0; i < nb_; ++i) o << (i ? "," : "") << a_[size_t(i)];
  o << "],\"beta\":[";
  for (int i = 0; i < nb_; ++i) o << (i ? "," : "") << b_[size_t(i)];
  o << "]}";
  return o.str();
}

void BanditModel::restore(const std::string& s) {
  Json j = parse_json(s);
  auto arr = [&](const char* k, auto& dst) {
    const Json* a = j.find(k);
    if (!a || !a->is_array() || int(a->items().size()) != nb_) throw std::runtime_error(std::string("bad router snapshot field ") + k);
    using T = std::remove_reference_t<decltype(dst[0])>;
    for (int i = 0; i < nb_; ++i) dst[size_t(i)] = T(a->items()[size_t(i)].as_number());
  };
  std::lock_guard<std::mutex> g(mu_);
  arr("success", success_);
  arr("tries", tries_);
  arr("values", values_);
  arr("alpha", a_);
  arr("beta", b_);
  if (const Json* b = j.find("best")) best_ = int(b->as_number());
  if (const Json* o = j.find("offset")) offset_.store(uint64_t(o->as_number()));
  if (shm_) {
    // Workers share one state: a snapshot replaces it only if it is newer
    // than the shared state (its version is the shared version it was taken
    // at).  The first worker restoring after a fresh start installs it; the
    // others -- and a worker restarted while the rest kept serving -- find the
    // live state at least as new and pull it instead, so feedback applied
    // since the checkpoint is kept.
    const Json* v = j.find("version");
    const uint64_t snap_v = v ? uint64_t(v->as_number()) : 0;
    ShmLock l(shm_->mu);
    const uint64_t live_v = shm_->version.load(std::memory_order_acquire);
    // version 1: seeded by the first worker, no feedback, nothing restored yet
    if (live_v <= 1 || snap_v > live_v) {
      for (int i = 0; i < nb_; ++i) {
        shm_->success[i] = success_[size_t(i)];
        shm_->tries[i] = tries_[size_t(i)];
        shm_->values[i] = values_[size_t(i)];
        shm_->alpha[i] = a_[size_t(i)];
        shm_->beta[i] = b_[size_t(i)];
      }
      shm_->best.store(best_, std::memory_order_release);
      const uint64_t nv = std::max(snap_v, live_v) + 1;
      shm_->version.store(nv, std::memory_order_release);
      seen_version_.store(nv, std::memory_order_relaxed);
    } else {
      for (int i = 0; i < nb_; ++i) {
        success_[size_t(i)] = shm_->success[i];
        tries_[size_t(i)] = shm_->tries[i];
        values_[size_t(i)] = shm_->values[i];
        a_[size_t(i)] = shm_->alpha[i];
        b_[size_t(i)] = shm_->beta[i];
      }
      best_ = shm_->best.load(std::memory_order_relaxed);
      seen_version_.store(live_v, std::memory_order_relaxed);
    }
  }
  publish();
}

// ------------------------------------------------------------------ unit
BanditRouterUnit::BanditRouterUnit(std::shared_ptr<BanditModel> model, BatcherOptions opts, bool device_route)
    : model_(std::move(model)), opts_(opts) {
  batched_ = std::make_shared<BatchedUnit>(model_, opts_);
  host_route_ = opts_.device >= 0 && !device_route && model_->host_routable();
}

void BanditRouterUnit::route(const CallCtx& c, MsgPtr, Done k) {
  if (host_route_) {
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    m->data.kind = DataKind::Tensor;
    m->data.shape = {1, 1};
    m->data.values = {double(model_->route_host())};
    k(Outcome::ok(std::move(m)));
    return;
  }
  static thread_local MsgPtr probe = [] {
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    m->data.kind = DataKind::Tensor;
    m->data.shape = {1, 1};
    m->data.values = {0.0};
    return m;
  }();
  batched_->transform_input(c, probe, [k](Outcome o) {
    if (o.err) { k(std::move(o)); return; }
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    m->data.kind = DataKind::Tensor;
    m->data.shape = {1, 1};
    m->data.values = {o.msg->data.values.empty() ? 0.0 : o.msg->data.values[0]};
    k(Outcome::ok(std::move(m)));
  });
}

void BanditRouterUnit::send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) {
  int32_t routing = -1;
  if (!c.node || !fb->response.meta.routing_of(c.node->name, routing) || routing < 0) {
    k(nullptr);  // not routed through this router (or routing unknown): nothing to learn
    return;
  }
  int64_t n = 0;
  if (fb->request.payload == Payload::Data) n = fb->request.data.rows();
  const int n_success = int(double(fb->reward) * double(n));
  try {
    model_->feedback(routing, n_success, int(n) - n_success);
  } catch (const std::exception& e) {
    k(make_error(ApiError::INVALID_ROUTING, e.what()));
    return;
  }
  k(nullptr);
}

}  // namespace sca::gpu
