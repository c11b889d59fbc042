#include "fabric.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace sca::par {

#define SCA_NCCL_CHECK(expr)                                                                               \
  do {                                                                                                     \
    ncclResult_t _r = (expr);                                                                              \
    if (_r != ncclSuccess)                                                                                 \
      throw std::runtime_error(std::string("RCCL error: ") + #expr + " -> " + ncclGetErrorString(_r) + " @ " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                                 \
  } while (0)

namespace {
void write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) throw std::runtime_error(std::string("fabric socket send failed: ") + std::strerror(errno));
    c += w;
    n -= size_t(w);
  }
}
void read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    const ssize_t r = ::read(fd, c, n);
    if (r < 0 && errno == EINTR) continue;
    if (r == 0) throw std::runtime_error("fabric peer closed the connection");
    if (r < 0) throw std::runtime_error(std::string("fabric socket read failed: ") + std::strerror(errno));
    c += r;
    n -= size_t(r);
  }
}

// Wait policy of the header ring: spin through the usual few-microsecond
// hand-off, then yield, then sleep (a worker idle between graphs must not burn
// a core); `slow` runs in the sleeping phase (liveness checks).
template <class Ready, class Slow>
void backoff_until(Ready ready, Slow slow) {
  using clk = std::chrono::steady_clock;
  int spins = 0;
  clk::time_point t0{};
  while (!ready()) {
    if (spins < 2048) {
      ++spins;
      _mm_pause();
      continue;
    }
    if (spins == 2048) {
      ++spins;
      t0 = clk::now();
    }
    if (clk::now() - t0 < std::chrono::microseconds(200)) {
      std::this_thread::yield();
    } else {
      slow();
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
}
}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId ids[2];
  SCA_NCCL_CHECK(ncclGetUniqueId(&ids[0]));
  SCA_NCCL_CHECK(ncclGetUniqueId(&ids[1]));
  return std::string(reinterpret_cast<const char*>(ids), sizeof ids);
}

// ------------------------------------------------------------------ fabric
Fabric::Fabric(int rank, int world, const std::string& unique_id, int device, std::vector<int> ctrl_fds)
    : rank_(rank), world_(world), device_(device), fds_(std::move(ctrl_fds)) {
  if (rank < 0 || rank >= world) throw std::runtime_error("Fabric: rank out of range");
  if (int(fds_.size()) != world) throw std::runtime_error("Fabric: need one control socket slot per rank");
  map_rings();
  if (device_ < 0) return;
  if (unique_id.size() != 2 * sizeof(ncclUniqueId)) throw std::runtime_error("Fabric: bad RCCL unique id size");
  ncclUniqueId ids[2];
  std::memcpy(ids, unique_id.data(), sizeof ids);
  gpu::DeviceGuard g(device);
  sx_.create(device);
  sy_.create(device);
  SCA_NCCL_CHECK(ncclCommInitRank(&comm_x_, world, ids[0], rank));
  SCA_NCCL_CHECK(ncclCommInitRank(&comm_y_, world, ids[1], rank));
}

Fabric::~Fabric() {
  close();
  for (auto*& r : rings_)
    if (r) {
      munmap(r, sizeof(HeaderRing));
      r = nullptr;
    }
}

// Rank 0 creates one shared header ring per worker and sends its name over
// the control socket; the worker maps it and acknowledges; rank 0 then
// unlinks the name, so nothing is left in /dev/shm whatever happens later.
void Fabric::map_rings() {
  static std::atomic<int> counter{0};
  const size_t bytes = sizeof(HeaderRing);
  auto map = [&](int shm) {
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, shm, 0);
    ::close(shm);
    if (p == MAP_FAILED) throw std::runtime_error(std::string("fabric: mmap failed: ") + std::strerror(errno));
    return static_cast<HeaderRing*>(p);
  };
  if (rank_ == 0) {
    rings_.assign(size_t(world_), nullptr);
    next_.assign(size_t(world_), 0);
    for (int r = 1; r < world_; ++r) {
      const std::string name = "/sca_fab_" + std::to_string(getpid()) + "_" + std::to_string(counter++) + "_" +
                               std::to_string(r);
      const int shm = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (shm < 0) throw std::runtime_error("fabric: shm_open(" + name + ") failed: " + std::strerror(errno));
      if (ftruncate(shm, off_t(bytes)) != 0) {
        ::close(shm);
        shm_unlink(name.c_str());
        throw std::runtime_error(std::string("fabric: ftruncate failed: ") + std::strerror(errno));
      }
      rings_[size_t(r)] = map(shm);  // fresh pages are zero: every seq 0, consumed 0
      const uint32_t n = uint32_t(name.size());
      try {
        write_all(fd(r), &n, sizeof n);
        write_all(fd(r), name.data(), n);
        char ack = 0;
        read_all(fd(r), &ack, 1);
      } catch (...) {
        shm_unlink(name.c_str());
        throw;
      }
      shm_unlink(name.c_str());
    }
  } else {
    uint32_t n = 0;
    read_all(fd(0), &n, sizeof n);
    if (n == 0 || n > 255) throw std::runtime_error("fabric: bad ring name");
    std::string name(n, '\0');
    read_all(fd(0), &name[0], n);
    const int shm = shm_open(name.c_str(), O_RDWR, 0600);
    if (shm < 0) throw std::runtime_error("fabric: shm_open(" + name + ") failed: " + std::strerror(errno));
    rings_.assign(1, map(shm));
    next_.assign(1, 0);
    const char ack = 1;
    write_all(fd(0), &ack, 1);
  }
}

void Fabric::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (!open_.exchange(false)) return;
  if (comm_x_ || comm_y_) {
    gpu::DeviceGuard d(device_);
    // A peer that died leaves posted operations that never finish: wait a
    // bounded time, then abort the communicators instead of hanging.
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(5);
    bool idle = false;
    while (std::chrono::steady_clock::now() < until) {
      if (hipStreamQuery(sx_.get()) == hipSuccess && hipStreamQuery(sy_.get()) == hipSuccess) {
        idle = true;
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    for (ncclComm_t* c : {&comm_x_, &comm_y_}) {
      if (*c) (void)(idle ? ncclCommDestroy(*c) : ncclCommAbort(*c));
      *c = nullptr;
    }
  }
  for (auto& q : rq_)
    if (q) {
      std::lock_guard<std::mutex> qg(q->mu);
      q->cv.notify_all();
    }
  for (int& fd : fds_)
    if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  for (auto& q : rq_)
    if (q && q->th.joinable()) q->th.join();
  for (int& fd : fds_)
    if (fd >= 0) {
      ::close(fd);
      fd = -1;
    }
  // The rings stay mapped until the destructor: a worker thread may still be
  // polling one (its take() sees open_ == false and leaves).
}

int Fabric::fd(int peer) const {
  if (peer < 0 || peer >= world_ || fds_[size_t(peer)] < 0)
    throw std::runtime_error("Fabric: no control link to rank " + std::to_string(peer));
  return fds_[size_t(peer)];
}

bool Fabric::peer_gone(int peer) const {
  const int f = fds_[size_t(peer)];
  if (f < 0) return true;
  char c;
  const ssize_t r = ::recv(f, &c, 1, MSG_PEEK | MSG_DONTWAIT);
  return r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
}

void Fabric::publish(int peer, const PeerHeader& h) {
  if (rank_ != 0) throw std::runtime_error("Fabric::publish: only rank 0 issues batches");
  HeaderRing* R = rings_.at(size_t(peer));
  if (!R) throw std::runtime_error("Fabric: no header ring to rank " + std::to_string(peer));
  const uint64_t seq = next_[size_t(peer)];
  // credit: the worker must have taken the header kSlots back
  backoff_until([&] { return seq - R->consumed.load(std::memory_order_acquire) < HeaderRing::kSlots; },
                [&] {
                  if (peer_gone(peer)) throw std::runtime_error("fabric: rank " + std::to_string(peer) + " is gone");
                });
  auto& s = R->slots[seq % HeaderRing::kSlots];
  s.h = h;
  s.seq.store(seq + 1, std::memory_order_release);  // the doorbell
  next_[size_t(peer)] = seq + 1;
}

PeerHeader Fabric::take() {
  HeaderRing* R = rings_.empty() ? nullptr : rings_[0];
  if (!R || !open_.load()) throw std::runtime_error("fabric closed");
  const uint64_t seq = next_[0];
  auto& s = R->slots[seq % HeaderRing::kSlots];
  backoff_until([&] { return s.seq.load(std::memory_order_acquire) == seq + 1; },
                [&] {
                  if (!open_.load()) throw std::runtime_error("fabric closed");
                  if (s.seq.load(std::memory_order_acquire) != seq + 1 && peer_gone(0))
                    throw std::runtime_error("fabric: rank 0 is gone");
                });
  const PeerHeader h = s.h;
  R->consumed.store(seq + 1, std::memory_order_release);
  next_[0] = seq + 1;
  return h;
}

void Fabric::send_x(const void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclSend(p, bytes, ncclChar, peer, comm_x_, sx_.get()));
  else write_all(fd(peer), p, bytes);
}
void Fabric::recv_x(void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclRecv(p, bytes, ncclChar, peer, comm_x_, sx_.get()));
  else read_all(fd(peer), p, bytes);
}
void Fabric::send_y(const void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclSend(p, bytes, ncclChar, peer, comm_y_, sy_.get()));
  else write_all(fd(peer), p, bytes);
}
void Fabric::recv_y(void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclRecv(p, bytes, ncclChar, peer, comm_y_, sy_.get()));
  else read_all(fd(peer), p, bytes);
}
void Fabric::group_start() {
  if (gpu()) SCA_NCCL_CHECK(ncclGroupStart());
}
void Fabric::group_end() {
  if (gpu()) SCA_NCCL_CHECK(ncclGroupEnd());
}

void Fabric::expect_reply(int peer, void* dst, size_t bytes, std::shared_ptr<Waiter> w) {
  if (rq_.empty()) rq_.resize(size_t(world_));
  auto& q = rq_[size_t(peer)];
  if (!q) {
    q = std::make_unique<RecvQ>();
    q->th = std::thread([this, peer] { receiver(peer); });
  }
  std::lock_guard<std::mutex> g(q->mu);
  q->q.push_back({dst, bytes, std::move(w)});
  q->cv.notify_one();
}

// Rank 0, CPU fabrics: replies of one worker arrive in issue order; hand each
// to the caller that queued it.
void Fabric::receiver(int peer) {
  RecvQ& q = *rq_[size_t(peer)];
  auto finish = [](Pending& p, const std::string& err) {
    std::lock_guard<std::mutex> g(p.w->mu);
    if (!err.empty() && p.w->error.empty()) p.w->error = err;
    if (--p.w->pending == 0) p.w->cv.notify_all();
  };
  while (true) {
    Pending p;
    {
      std::unique_lock<std::mutex> lk(q.mu);
      q.cv.wait(lk, [&] { return !q.q.empty() || !open_.load(); });
      if (q.q.empty()) return;
      p = q.q.front();
      q.q.pop_front();
    }
    try {
      read_all(fds_[size_t(peer)], p.dst, p.bytes);
      finish(p, "");
    } catch (const std::exception& e) {
      finish(p, e.what());
      std::lock_guard<std::mutex> lk(q.mu);
      for (auto& r : q.q) finish(r, e.what());
      q.q.clear();
      return;
    }
  }
}

void stop_peers(Fabric& f) {
  std::lock_guard<std::mutex> g(f.issue_mutex());
  if (!f.open()) return;
  PeerHeader h;
  h.op = kPeerStop;
  for (int r = 0; r < f.world(); ++r)
    if (r != f.rank()) f.publish(r, h);
  if (f.gpu()) {
    SCA_HIP_CHECK(hipStreamSynchronize(f.stream_x()));
    SCA_HIP_CHECK(hipStreamSynchronize(f.stream_y()));
  }
}

// ----------------------------------------------------------- front end side
PeerRowModel::PeerRowModel(FabricPtr fabric, std::vector<int> peers, int model_id, int in_cols, int out_cols)
    : f_(std::move(fabric)), peers_(std::move(peers)), model_id_(model_id), in_cols_(in_cols), out_cols_(out_cols) {
  if (peers_.empty()) throw std::runtime_error("PeerRowModel: no peer ranks");
  for (int p : peers_)
    if (p < 0 || p >= f_->world() || p == f_->rank()) throw std::runtime_error("PeerRowModel: invalid peer rank");
  if (in_cols_ <= 0 || out_cols_ <= 0) throw std::runtime_error("PeerRowModel: widths must be known");
}

PeerRowModel::~PeerRowModel() = default;

void PeerRowModel::to_device(int device) {
  if (device != f_->device()) throw std::runtime_error("PeerRowModel: must run on the fabric's GPU");
  ev_in_.create(device);
  ev_done_.create(device);
}

size_t PeerRowModel::workspace_bytes(int max_rows, int) const {
  // one gathered output slab per peer (fan-out combine)
  return peers_.size() > 1 ? peers_.size() * size_t(max_rows) * out_cols_ * sizeof(double) : 0;
}

void PeerRowModel::headers(int rows, int cols) const {
  PeerHeader h;
  h.op = kPeerRun;
  h.model = model_id_;
  h.rows = rows;
  h.cols = cols;
  for (int p : peers_) f_->publish(p, h);
}

// GPU: everything is stream-ordered and returns at once.  X leaves on the
// fabric's X stream once the batcher has staged it; the reply lands on the Y
// stream (gather + combine for fan-outs), and the batcher's stream waits for
// that -- so the next batch's send is never queued behind this reply.
void PeerRowModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  std::lock_guard<std::mutex> g(f_->issue_mutex());
  if (!f_->open()) throw std::runtime_error("RCCL fabric closed");
  hipStream_t sx = f_->stream_x(), sy = f_->stream_y();
  SCA_HIP_CHECK(hipEventRecord(ev_in_.get(), s));  // X staged on the batcher's stream
  SCA_HIP_CHECK(hipStreamWaitEvent(sx, ev_in_.get(), 0));
  headers(rows, cols);  // doorbells: the workers post their receives now
  const size_t bx = size_t(rows) * cols * sizeof(double), by = size_t(rows) * out_cols_ * sizeof(double);
  if (peers_.size() == 1) {
    f_->send_x(X, bx, peers_[0]);
    f_->recv_y(out, by, peers_[0]);
  } else {
    // broadcast the batch, gather every replica's output, average on this GPU
    auto* slabs = static_cast<double*>(ws);
    f_->group_start();
    for (int p : peers_) f_->send_x(X, bx, p);
    f_->group_end();
    f_->group_start();
    for (size_t i = 0; i < peers_.size(); ++i) f_->recv_y(slabs + i * size_t(rows) * out_cols_, by, peers_[i]);
    f_->group_end();
    kern::combine_mean_strided_f64(slabs, int(peers_.size()), int64_t(rows) * out_cols_, out, sy);
  }
  SCA_HIP_CHECK(hipEventRecord(ev_done_.get(), sy));
  SCA_HIP_CHECK(hipStreamWaitEvent(s, ev_done_.get(), 0));
  batches_++;
}

// CPU fabric: issue under the fabric's mutex (header + payload), then wait
// for the reply outside it, so concurrent callers keep several batches in
// flight per worker.
void PeerRowModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  if (f_->gpu()) throw std::runtime_error("rccl_peer: GPU fabric models run on their GPU");
  const size_t bx = size_t(rows) * cols * sizeof(double), ny = size_t(rows) * out_cols_;
  std::vector<std::vector<double>> slabs(peers_.size() > 1 ? peers_.size() : 0, std::vector<double>(ny));
  auto w = std::make_shared<Fabric::Waiter>();
  w->pending = int(peers_.size());
  {
    std::lock_guard<std::mutex> g(f_->issue_mutex());
    if (!f_->open()) throw std::runtime_error("fabric closed");
    headers(rows, cols);
    for (size_t i = 0; i < peers_.size(); ++i) {
      f_->send_x(X, bx, peers_[i]);
      f_->expect_reply(peers_[i], peers_.size() == 1 ? static_cast<void*>(out) : slabs[i].data(),
                       ny * sizeof(double), w);
    }
  }
  {
    std::unique_lock<std::mutex> lk(w->mu);
    w->cv.wait(lk, [&] { return w->pending == 0; });
    if (!w->error.empty()) throw std::runtime_error(w->error);
  }
  if (peers_.size() > 1) {
    std::fill(out, out + ny, 0.0);
    for (const auto& sl : slabs)
      for (size_t i = 0; i < ny; ++i) out[i] += sl[i];
    for (size_t i = 0; i < ny; ++i) out[i] /= double(peers_.size());
  }
  batches_++;
}

// ---------------------------------------------------------------- worker side
PeerServer::PeerServer(FabricPtr fabric) : f_(std::move(fabric)) {
  if (const char* e = std::getenv("SCA_FABRIC_SLOTS")) slots_ = std::max(1, std::min(64, std::atoi(e)));
}

PeerServer::~PeerServer() { join(); }

int PeerServer::add_model(gpu::RowModelPtr m) {
  if (th_.joinable()) throw std::runtime_error("PeerServer: add models before start()");
  if (f_->gpu()) m->to_device(f_->device());
  models_.push_back(std::move(m));
  return int(models_.size()) - 1;
}

void PeerServer::start() {
  if (th_.joinable()) return;
  th_ = std::thread([this] {
    try {
      if (f_->gpu()) loop();
      else loop_cpu();
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(err_mu_);
      err_ = e.what();
    }
  });
}

void PeerServer::join() {
  if (th_.joinable()) th_.join();
}

std::string PeerServer::error() const {
  std::lock_guard<std::mutex> g(err_mu_);
  return err_;
}

void PeerServer::note_inflight(uint64_t n) {
  uint64_t m = max_inflight_.load(std::memory_order_relaxed);
  while (n > m && !max_inflight_.compare_exchange_weak(m, n)) {
  }
}

// GPU worker: K slots; slot k's receive (X stream), kernel (compute stream)
// and reply (Y stream) are chained with events, and a slot is reused only
// after its previous kernel has read X and its previous reply has left.  The
// thread takes the next header as soon as this batch is enqueued.
void PeerServer::loop() {
  gpu::DeviceGuard g(f_->device());
  const int dev = f_->device();
  hipStream_t sx = f_->stream_x(), sy = f_->stream_y();
  gpu::Stream sc(dev);
  struct Slot {
    gpu::DeviceBuffer x, y;
    gpu::Event ev_recv, ev_done, ev_sent;
    bool used = false;
  };
  std::vector<Slot> slots(static_cast<size_t>(slots_));
  for (auto& s : slots) {
    s.ev_recv.create(dev);
    s.ev_done.create(dev);
    s.ev_sent.create(dev);
  }
  gpu::DeviceBuffer ws;  // kernels are serialised on the compute stream: one workspace
  std::deque<size_t> inflight;  // slots of batches whose reply may still be in flight, oldest first
  uint64_t seq = 0;
  while (true) {
    const PeerHeader h = f_->take();
    if (h.op == kPeerStop) break;
    if (h.model < 0 || h.model >= int(models_.size()) || h.rows <= 0 || h.cols <= 0)
      throw std::runtime_error("PeerServer: bad header (model " + std::to_string(h.model) + ")");
    auto& m = models_[size_t(h.model)];
    const int oc = m->out_cols(h.cols);
    const size_t bx = size_t(h.rows) * h.cols * sizeof(double), by = size_t(h.rows) * oc * sizeof(double);
    const size_t bw = m->workspace_bytes(h.rows, h.cols);
    const size_t k = size_t(seq++ % uint64_t(slots_));
    Slot& s = slots[k];
    if (bx > s.x.bytes() || by > s.y.bytes()) {
      if (s.used) SCA_HIP_CHECK(hipEventSynchronize(s.ev_sent.get()));  // previous use fully done
      host_syncs_++;
      if (bx > s.x.bytes()) s.x.alloc(std::max(bx, 2 * s.x.bytes()), dev);
      if (by > s.y.bytes()) s.y.alloc(std::max(by, 2 * s.y.bytes()), dev);
    }
    if (bw > ws.bytes()) {
      SCA_HIP_CHECK(hipStreamSynchronize(sc.get()));
      host_syncs_++;
      ws.alloc(std::max(bw, 2 * ws.bytes()), dev);
    }
    if (s.used) SCA_HIP_CHECK(hipStreamWaitEvent(sx, s.ev_done.get(), 0));  // previous kernel read x
    f_->recv_x(s.x.get(), bx, 0);
    SCA_HIP_CHECK(hipEventRecord(s.ev_recv.get(), sx));
    SCA_HIP_CHECK(hipStreamWaitEvent(sc.get(), s.ev_recv.get(), 0));
    if (s.used) SCA_HIP_CHECK(hipStreamWaitEvent(sc.get(), s.ev_sent.get(), 0));  // previous y has left
    m->launch(s.x.as<double>(), h.rows, h.cols, s.y.as<double>(), ws.get(), sc.get());
    SCA_HIP_CHECK(hipEventRecord(s.ev_done.get(), sc.get()));
    SCA_HIP_CHECK(hipStreamWaitEvent(sy, s.ev_done.get(), 0));
    f_->send_y(s.y.get(), by, 0);
    SCA_HIP_CHECK(hipEventRecord(s.ev_sent.get(), sy));
    s.used = true;
    batches_++;
    rows_ += uint64_t(h.rows);
    // in flight = enqueued batches whose reply has not left (a slot's event
    // completing implies every older use of the stream completed)
    inflight.push_back(k);
    while (!inflight.empty() && hipEventQuery(slots[inflight.front()].ev_sent.get()) == hipSuccess)
      inflight.pop_front();
    note_inflight(inflight.size());
  }
  SCA_HIP_CHECK(hipStreamSynchronize(sx));
  SCA_HIP_CHECK(hipStreamSynchronize(sc.get()));
  SCA_HIP_CHECK(hipStreamSynchronize(sy));
}

// CPU worker (device -1 fabrics): a reader thread takes headers and payloads
// into up to K buffered batches while this thread computes and replies.
void PeerServer::loop_cpu() {
  struct Batch {
    PeerHeader h;
    std::vector<double> x;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Batch> q;
  bool done = false, computing = false;
  std::string rerr;
  int delay_us = 0;  // test knob: slow model
  if (const char* e = std::getenv("SCA_FABRIC_WORKER_DELAY_US")) delay_us = std::max(0, std::atoi(e));
  std::thread reader([&] {
    try {
      while (true) {
        Batch b;
        b.h = f_->take();
        if (b.h.op != kPeerStop) {
          if (b.h.model < 0 || b.h.model >= int(models_.size()) || b.h.rows <= 0 || b.h.cols <= 0)
            throw std::runtime_error("PeerServer: bad header (model " + std::to_string(b.h.model) + ")");
          b.x.resize(size_t(b.h.rows) * b.h.cols);
          f_->recv_x(b.x.data(), b.x.size() * sizeof(double), 0);
        }
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return q.size() + (computing ? 1 : 0) < size_t(slots_) || done; });  // K slots incl. the one computing
        if (done) return;  // the compute side failed
        const bool stop = b.h.op == kPeerStop;
        q.push_back(std::move(b));
        note_inflight(q.size() + (computing ? 1 : 0) - (stop ? 1 : 0));
        cv.notify_all();
        if (stop) return;
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu);
      rerr = e.what();
      done = true;
      cv.notify_all();
    }
  });
  std::vector<double> y;
  std::string err;
  while (true) {
    Batch b;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return !q.empty() || done; });
      if (q.empty()) break;
      b = std::move(q.front());
      q.pop_front();
      computing = b.h.op != kPeerStop;
      cv.notify_all();
    }
    if (b.h.op == kPeerStop) break;
    try {
      auto& m = models_[size_t(b.h.model)];
      y.resize(size_t(b.h.rows) * m->out_cols(b.h.cols));
      if (delay_us) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
      m->run_cpu(b.x.data(), b.h.rows, b.h.cols, y.data());
      f_->send_y(y.data(), y.size() * sizeof(double), 0);
    } catch (const std::exception& e) {
      err = e.what();
      break;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      computing = false;
      cv.notify_all();
    }
    batches_++;
    rows_ += uint64_t(b.h.rows);
  }
  if (!err.empty()) {  // unblock the reader: it cannot make progress without us
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
      cv.notify_all();
    }
    f_->close();
  }
  reader.join();
  if (!err.empty()) throw std::runtime_error(err);
  if (!rerr.empty()) throw std::runtime_error(rerr);
}

}  // namespace sca::par
