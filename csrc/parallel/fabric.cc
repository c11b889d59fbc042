#include "fabric.h"

#include <poll.h>

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

constexpr int kChanX = 0, kChanY = 1;
}  // namespace

std::string rccl_unique_ids(int world) {
  if (world < 2) return std::string();
  std::vector<ncclUniqueId> ids(size_t(2 * (world - 1)));
  for (auto& id : ids) SCA_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(ids.data()), ids.size() * sizeof(ncclUniqueId));
}

// ------------------------------------------------------------ loopback hub
LoopbackHub::LoopbackHub(int device) : device_(device) {
  if (device < 0) throw std::runtime_error("LoopbackHub: needs a GPU");
  if (const char* e = std::getenv("SCA_LOOPBACK_TIMEOUT_MS")) recv_timeout_ms_ = std::max(100, std::atoi(e));
}

LoopbackHub::~LoopbackHub() {
  // Stages may still be read by copies in flight on streams that are gone by
  // now; the device drains before the buffers go.
  gpu::DeviceGuard g(device_);
  (void)hipDeviceSynchronize();
}

LoopbackHub::Stage* LoopbackHub::acquire(size_t bytes) {
  // caller holds mu_
  for (auto& st : pool_)
    if (!st->busy && st->buf.bytes() >= bytes && hipEventQuery(st->freed.get()) == hipSuccess) {
      st->busy = true;
      return st.get();
    }
  auto st = std::make_unique<Stage>();
  st->buf.alloc(std::max<size_t>(bytes, 4096), device_);
  st->ready.create(device_);
  st->freed.create(device_);
  st->busy = true;
  pool_.push_back(std::move(st));
  return pool_.back().get();
}

uint64_t LoopbackHub::staging_buffers() const {
  std::lock_guard<std::mutex> g(mu_);
  return pool_.size();
}

void LoopbackHub::send(int src, int dst, int chan, const void* p, size_t bytes, hipStream_t s) {
  gpu::DeviceGuard g(device_);
  std::lock_guard<std::mutex> lk(mu_);
  if (std::find(closed_.begin(), closed_.end(), src) != closed_.end())
    throw std::runtime_error("loopback fabric closed");
  Stage* st = acquire(bytes);
  SCA_HIP_CHECK(hipMemcpyAsync(st->buf.get(), p, bytes, hipMemcpyDeviceToDevice, s));
  SCA_HIP_CHECK(hipEventRecord(st->ready.get(), s));
  chans_[std::make_tuple(src, dst, chan)].q.push_back({st, bytes});
  messages_++;
  cv_.notify_all();
}

void LoopbackHub::recv(int src, int dst, int chan, void* p, size_t bytes, hipStream_t s) {
  gpu::DeviceGuard g(device_);
  std::unique_lock<std::mutex> lk(mu_);
  Chan& c = chans_[std::make_tuple(src, dst, chan)];
  auto closed = [&] { return std::find(closed_.begin(), closed_.end(), dst) != closed_.end(); };
  if (!c.q.empty()) immediate_++;
  if (!cv_.wait_for(lk, std::chrono::milliseconds(recv_timeout_ms_), [&] { return !c.q.empty() || closed(); }))
    throw std::runtime_error("loopback fabric: no send from rank " + std::to_string(src) + " within " +
                             std::to_string(recv_timeout_ms_) + " ms");
  if (c.q.empty()) throw std::runtime_error("loopback fabric closed");
  const Msg m = c.q.front();
  c.q.pop_front();
  if (m.bytes != bytes) {
    m.st->busy = false;
    throw std::runtime_error("loopback fabric: rank " + std::to_string(src) + " sent " + std::to_string(m.bytes) +
                             " bytes, rank " + std::to_string(dst) + " expects " + std::to_string(bytes));
  }
  SCA_HIP_CHECK(hipStreamWaitEvent(s, m.st->ready.get(), 0));
  SCA_HIP_CHECK(hipMemcpyAsync(p, m.st->buf.get(), bytes, hipMemcpyDeviceToDevice, s));
  SCA_HIP_CHECK(hipEventRecord(m.st->freed.get(), s));
  m.st->busy = false;  // reusable once `freed` has fired
}

void LoopbackHub::close_rank(int rank) {
  std::lock_guard<std::mutex> lk(mu_);
  if (std::find(closed_.begin(), closed_.end(), rank) == closed_.end()) closed_.push_back(rank);
  cv_.notify_all();
}

// ------------------------------------------------------------------ fabric
Fabric::Fabric(int rank, int world, const std::string& unique_ids, int device, std::vector<int> ctrl_fds,
               LoopbackHubPtr hub)
    : rank_(rank), world_(world), device_(device), hub_(std::move(hub)), fds_(std::move(ctrl_fds)) {
  if (rank < 0 || rank >= world) throw std::runtime_error("Fabric: rank out of range");
  if (int(fds_.size()) != world) throw std::runtime_error("Fabric: need one control socket slot per rank");
  if (hub_ && hub_->device() != device) throw std::runtime_error("Fabric: loopback hub lives on another GPU");
  links_.resize(size_t(world));
  for (int r = 0; r < world; ++r)
    if ((rank == 0) != (r == 0)) links_[size_t(r)] = std::make_unique<Link>();
  map_rings();
  if (device_ < 0) {
    rq_.resize(size_t(world_));
    if (rank_ == 0)
      for (int r = 1; r < world_; ++r) rq_[size_t(r)] = std::make_unique<RecvQ>();
    return;
  }
  gpu::DeviceGuard g(device);
  for (auto& l : links_)
    if (l) {
      l->sx.create(device);
      l->sy.create(device);
    }
  if (hub_) return;
  if (unique_ids.size() != size_t(2 * (world - 1)) * sizeof(ncclUniqueId))
    throw std::runtime_error("Fabric: bad RCCL unique id blob size");
  auto id_of = [&](int link, int chan) {
    ncclUniqueId id;
    std::memcpy(&id, unique_ids.data() + size_t(2 * (link - 1) + chan) * sizeof(ncclUniqueId), sizeof id);
    return id;
  };
  // One 2-rank communicator pair per rank-0 <-> worker link: rank 0 is rank 0
  // of each, the worker rank 1.  Rank 0 joins its links in worker order; a
  // worker waits in its init until rank 0 reaches its link.
  for (int r = 1; r < world; ++r) {
    if (rank != 0 && rank != r) continue;
    Link& l = *links_[size_t(rank == 0 ? r : 0)];
    SCA_NCCL_CHECK(ncclCommInitRank(&l.cx, 2, id_of(r, kChanX), rank == 0 ? 0 : 1));
    SCA_NCCL_CHECK(ncclCommInitRank(&l.cy, 2, id_of(r, kChanY), rank == 0 ? 0 : 1));
  }
}

Fabric::~Fabric() {
  close();
  for (auto*& r : rings_)
    if (r) {
      munmap(r, sizeof(HeaderRing));
      r = nullptr;
    }
}

Fabric::Link& Fabric::link(int peer) const {
  if (peer < 0 || peer >= world_ || !links_[size_t(peer)])
    throw std::runtime_error("Fabric: no link from rank " + std::to_string(rank_) + " to rank " + std::to_string(peer));
  return *links_[size_t(peer)];
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
  std::lock_guard<std::mutex> g(close_mu_);
  if (!open_.exchange(false)) return;
  if (hub_) hub_->close_rank(rank_);
  if (gpu()) {
    gpu::DeviceGuard d(device_);
    // A peer that died leaves posted operations that never finish: wait a
    // bounded time, then abort the communicators instead of hanging.
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(5);
    bool idle = false;
    while (std::chrono::steady_clock::now() < until) {
      idle = true;
      for (auto& l : links_)
        if (l && (hipStreamQuery(l->sx.get()) != hipSuccess || hipStreamQuery(l->sy.get()) != hipSuccess))
          idle = false;
      if (idle) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    for (auto& l : links_) {
      if (!l) continue;
      for (ncclComm_t* c : {&l->cx, &l->cy}) {
        if (*c) (void)(idle ? ncclCommDestroy(*c) : ncclCommAbort(*c));
        *c = nullptr;
      }
    }
  }
  for (int& fd : fds_)
    if (fd >= 0) ::shutdown(fd, SHUT_RDWR);  // a reader blocked in recv() returns
  for (size_t r = 0; r < fds_.size(); ++r) {
    std::unique_lock<std::mutex> rd;
    if (r < rq_.size() && rq_[r]) rd = std::unique_lock<std::mutex>(rq_[r]->rd);
    if (fds_[r] >= 0) {
      ::close(fds_[r]);
      fds_[r] = -1;
    }
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

// Callers hold the link's mutex (one publisher per ring).
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

void Fabric::wait_readable(const std::vector<int>& peers, int us) const {
  pollfd pf[16];
  int n = 0;
  for (int p : peers) {
    if (n == 16 || p <= 0 || p >= world_) continue;
    const int f = fds_[size_t(p)];
    if (f >= 0) pf[n++] = pollfd{f, POLLIN, 0};
  }
  if (n == 0) return;
  const timespec ts{0, long(std::max(1, us)) * 1000L};
  (void)::ppoll(pf, nfds_t(n), &ts, nullptr);
}

int Fabric::backlog() const {
  if (rank_ == 0 || rings_.empty() || !rings_[0]) return 0;
  const HeaderRing* R = rings_[0];
  const uint64_t seq = next_[0];
  int n = 0;
  while (n < 64 && R->slots[(seq + uint64_t(n)) % HeaderRing::kSlots].seq.load(std::memory_order_acquire) ==
                       seq + uint64_t(n) + 1)
    ++n;
  return n;
}

void Fabric::xfer(bool send, int chan, void* p, size_t bytes, int peer) {
  if (!gpu()) {
    if (send) write_all(fd(peer), p, bytes);
    else read_all(fd(peer), p, bytes);
    return;
  }
  Link& l = link(peer);
  hipStream_t s = chan == kChanX ? l.sx.get() : l.sy.get();
  if (hub_) {
    if (send) hub_->send(rank_, peer, chan, p, bytes, s);
    else hub_->recv(peer, rank_, chan, p, bytes, s);
    return;
  }
  ncclComm_t c = chan == kChanX ? l.cx : l.cy;
  const int to = rank_ == 0 ? 1 : 0;  // the other end, as a rank of the link's 2-rank communicator
  if (send) SCA_NCCL_CHECK(ncclSend(p, bytes, ncclChar, to, c, s));
  else SCA_NCCL_CHECK(ncclRecv(p, bytes, ncclChar, to, c, s));
}

void Fabric::send_x(const void* p, size_t bytes, int peer) { xfer(true, kChanX, const_cast<void*>(p), bytes, peer); }
void Fabric::recv_x(void* p, size_t bytes, int peer) { xfer(false, kChanX, p, bytes, peer); }
void Fabric::send_y(const void* p, size_t bytes, int peer) { xfer(true, kChanY, const_cast<void*>(p), bytes, peer); }
void Fabric::recv_y(void* p, size_t bytes, int peer) { xfer(false, kChanY, p, bytes, peer); }

void Fabric::expect_reply(int peer, void* dst, size_t bytes, std::shared_ptr<Waiter> w) {
  RecvQ& q = recvq(peer);
  std::lock_guard<std::mutex> g(q.mu);
  q.q.push_back({dst, bytes, std::move(w)});
}

Fabric::RecvQ& Fabric::recvq(int peer) {
  if (gpu() || rank_ != 0 || peer <= 0 || peer >= world_ || !rq_[size_t(peer)])
    throw std::runtime_error("Fabric: no reply queue for rank " + std::to_string(peer));
  return *rq_[size_t(peer)];
}

// Rank 0, CPU fabrics.  Replies of one worker arrive on its socket in issue
// order; whichever caller polls reads them into the buffers queued by
// expect_reply and finishes their waiters (no receiver thread: the batcher's
// pump polls between launches, so a reply costs no extra thread wake-up).
// One reader per link at a time (q.rd); the queue lock only guards push/pop,
// and a deque's elements stay put under push_back.
bool Fabric::poll_replies(int peer, bool block) {
  RecvQ& q = recvq(peer);
  std::unique_lock<std::mutex> rd(q.rd, std::defer_lock);
  if (block) rd.lock();
  else if (!rd.try_lock()) return false;
  auto finish = [](Pending& p, const std::string& err) {
    std::lock_guard<std::mutex> g(p.w->mu);
    if (!err.empty() && p.w->error.empty()) p.w->error = err;
    if (--p.w->pending == 0) p.w->cv.notify_all();
  };
  auto fail_all = [&](const std::string& err) {
    std::lock_guard<std::mutex> g(q.mu);
    for (auto& r : q.q) finish(r, err);
    q.q.clear();
    q.off = 0;
  };
  bool progress = false;
  while (true) {
    Pending* p;
    {
      std::lock_guard<std::mutex> g(q.mu);
      if (q.q.empty()) return progress;
      p = &q.q.front();
    }
    const int fd = fds_[size_t(peer)];
    if (fd < 0) {
      fail_all("fabric closed");
      return true;
    }
    char* dst = static_cast<char*>(p->dst);
    while (q.off < p->bytes) {
      const ssize_t r = ::recv(fd, dst + q.off, p->bytes - q.off, block ? 0 : MSG_DONTWAIT);
      if (r > 0) {
        q.off += size_t(r);
        continue;
      }
      if (r < 0 && errno == EINTR) continue;
      if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return progress;
      fail_all(r == 0 ? std::string("fabric peer closed the connection")
                      : std::string("fabric socket read failed: ") + std::strerror(errno));
      return true;
    }
    Pending done;
    {
      std::lock_guard<std::mutex> g(q.mu);
      done = std::move(q.q.front());
      q.q.pop_front();
      q.off = 0;
    }
    finish(done, "");
    progress = true;
    if (block) return true;  // the caller re-checks its own waiter
  }
}

void stop_peers(Fabric& f) {
  if (!f.open()) return;
  PeerHeader h;
  h.op = kPeerStop;
  for (int r = 0; r < f.world(); ++r) {
    if (r == f.rank()) continue;
    std::lock_guard<std::mutex> g(f.link_mutex(r));
    f.publish(r, h);
  }
  if (f.gpu())
    for (int r = 1; r < f.world(); ++r) {
      SCA_HIP_CHECK(hipStreamSynchronize(f.stream_x(r)));
      SCA_HIP_CHECK(hipStreamSynchronize(f.stream_y(r)));
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
  ev_y_ = std::vector<gpu::Event>(peers_.size());
  for (auto& e : ev_y_) e.create(device);
}

size_t PeerRowModel::workspace_bytes(int max_rows, int) const {
  // one gathered output slab per peer (fan-out combine)
  return peers_.size() > 1 ? peers_.size() * size_t(max_rows) * out_cols_ * sizeof(double) : 0;
}

void PeerRowModel::header(int peer, int rows, int cols) const {
  PeerHeader h;
  h.op = kPeerRun;
  h.model = model_id_;
  h.rows = rows;
  h.cols = cols;
  f_->publish(peer, h);
}

// GPU: everything is stream-ordered and returns at once.  Each peer's link
// waits for the batcher's staged X, sends it on the link's X stream and
// receives the reply on the link's Y stream; only that link's mutex is held,
// so batches for other peers (other units' device threads) go out in
// parallel.  The batcher's stream waits for every link's reply, then (fan-out)
// averages the gathered slabs.
void PeerRowModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  std::lock_guard<std::mutex> g(mu_);
  if (!f_->open()) throw std::runtime_error("RCCL fabric closed");
  SCA_HIP_CHECK(hipEventRecord(ev_in_.get(), s));  // X staged on the batcher's stream
  const size_t bx = size_t(rows) * cols * sizeof(double), by = size_t(rows) * out_cols_ * sizeof(double);
  const bool fan = peers_.size() > 1;
  auto* slabs = static_cast<double*>(ws);
  for (size_t i = 0; i < peers_.size(); ++i) {
    const int p = peers_[i];
    std::lock_guard<std::mutex> lg(f_->link_mutex(p));
    SCA_HIP_CHECK(hipStreamWaitEvent(f_->stream_x(p), ev_in_.get(), 0));
    header(p, rows, cols);  // doorbell: the worker posts its receive now
    f_->send_x(X, bx, p);
    f_->recv_y(fan ? slabs + i * size_t(rows) * out_cols_ : out, by, p);
    SCA_HIP_CHECK(hipEventRecord(ev_y_[i].get(), f_->stream_y(p)));
  }
  for (auto& e : ev_y_) SCA_HIP_CHECK(hipStreamWaitEvent(s, e.get(), 0));
  if (fan) kern::combine_mean_strided_f64(slabs, int(peers_.size()), int64_t(rows) * out_cols_, out, s);
  batches_++;
}

// CPU fabric: header + payload go out under each link's mutex; the replies
// land in call-owned buffers when a caller polls the link (poll_replies).
std::shared_ptr<Fabric::Waiter> PeerRowModel::issue_cpu(const double* X, int rows, int cols) const {
  if (f_->gpu()) throw std::runtime_error("rccl_peer: GPU fabric models run on their GPU");
  if (!f_->open()) throw std::runtime_error("fabric closed");
  const size_t bx = size_t(rows) * cols * sizeof(double), ny = size_t(rows) * out_cols_;
  auto w = std::make_shared<Fabric::Waiter>();
  w->pending = int(peers_.size());
  w->bufs.assign(peers_.size(), std::vector<double>(ny));
  for (size_t i = 0; i < peers_.size(); ++i) {
    const int p = peers_[i];
    std::lock_guard<std::mutex> g(f_->link_mutex(p));
    // payload first: the worker, spinning on its ring, then finds the bytes
    // already in its socket buffer instead of sleeping in read()
    f_->expect_reply(p, w->bufs[i].data(), ny * sizeof(double), w);
    f_->send_x(X, bx, p);
    header(p, rows, cols);
  }
  batches_++;
  return w;
}

namespace {
// The reply (mean of the gathered replies for a fan-out) goes into `out` once.
struct PeerCall : gpu::CpuCall {
  FabricPtr f;             // held: an abandoned call may outlive its model
  std::vector<int> peers;
  std::shared_ptr<Fabric::Waiter> w;
  double* out;
  bool finished = false;
  std::string err;
  bool pending() {
    std::lock_guard<std::mutex> g(w->mu);
    return w->pending > 0;
  }
  bool done() override {
    if (finished) return true;
    if (pending())
      for (int p : peers) f->poll_replies(p, false);
    {
      std::lock_guard<std::mutex> g(w->mu);
      if (w->pending > 0) return false;
      err = w->error;
    }
    if (err.empty()) {
      const auto& b = w->bufs;
      const size_t n = b[0].size();
      if (b.size() == 1) {
        std::copy(b[0].begin(), b[0].end(), out);
      } else {
        for (size_t i = 0; i < n; ++i) {
          double acc = 0.0;
          for (const auto& sl : b) acc += sl[i];
          out[i] = acc / double(b.size());
        }
      }
    }
    finished = true;
    return true;
  }
  std::string error() const override { return err; }
  bool wait_us(int us) override {
    if (finished || !pending()) return true;
    f->wait_readable(peers, us);
    return true;
  }
};
}  // namespace

gpu::CpuCallPtr PeerRowModel::start_cpu(const double* X, int rows, int cols, double* out) {
  auto c = std::make_shared<PeerCall>();
  c->f = f_;
  c->peers = peers_;
  c->w = issue_cpu(X, rows, cols);
  c->out = out;
  return c;
}

void PeerRowModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  PeerCall c;
  c.f = f_;
  c.peers = peers_;
  c.w = issue_cpu(X, rows, cols);
  c.out = out;
  // Read replies (ours and older callers') until ours are in: a blocking
  // read of a peer returns after one reply, so no peer is waited on for
  // longer than its oldest outstanding batch.
  // Spin briefly first: a worker's reply usually lands within tens of
  // microseconds, and waking from a blocking read costs about as much again.
  const auto spin_until = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
  unsigned polls = 0;
  while (c.pending()) {
    bool got = false;
    for (int p : peers_)
      if (c.pending()) got |= f_->poll_replies(p, false);
    if (!got && c.pending() && ((++polls & 7) != 0 || std::chrono::steady_clock::now() < spin_until)) {
      _mm_pause();
      continue;
    }
    if (!got && c.pending()) {
      for (int p : peers_)
        if (c.pending() && f_->poll_replies(p, true)) break;
    }
  }
  c.done();
  if (!c.err.empty()) throw std::runtime_error(c.err);
}

// ---------------------------------------------------------------- worker side
PeerServer::PeerServer(FabricPtr fabric) : f_(std::move(fabric)) {
  if (const char* e = std::getenv("SCA_FABRIC_SLOTS")) slots_ = std::max(1, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("SCA_FABRIC_WORKER_DELAY_US")) delay_us_ = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("SCA_FABRIC_WORKER_HOST_DELAY_US")) host_delay_us_ = std::max(0, std::atoi(e));
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
  hipStream_t sx = f_->stream_x(0), sy = f_->stream_y(0);
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
    if (delay_us_) kern::device_delay_us(delay_us_, sc.get());
    m->launch(s.x.as<double>(), h.rows, h.cols, s.y.as<double>(), ws.get(), sc.get());
    SCA_HIP_CHECK(hipEventRecord(s.ev_done.get(), sc.get()));
    SCA_HIP_CHECK(hipStreamWaitEvent(sy, s.ev_done.get(), 0));
    if (host_delay_us_) std::this_thread::sleep_for(std::chrono::microseconds(host_delay_us_));
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

// CPU worker (device -1 fabrics): one thread takes a header, reads its
// payload, computes and replies, back to back.  Rank 0 keeps up to K calls
// outstanding; their headers wait in the ring and their payloads in the
// socket buffer, so a hand-off to a second thread would only add a wake-up
// per batch (profiles/r04d_fabric_cpu).
void PeerServer::loop_cpu() {
  std::vector<double> x, y;
  while (true) {
    const PeerHeader h = f_->take();
    if (h.op == kPeerStop) break;
    if (h.model < 0 || h.model >= int(models_.size()) || h.rows <= 0 || h.cols <= 0)
      throw std::runtime_error("PeerServer: bad header (model " + std::to_string(h.model) + ")");
    note_inflight(uint64_t(1 + f_->backlog()));
    x.resize(size_t(h.rows) * h.cols);
    f_->recv_x(x.data(), x.size() * sizeof(double), 0);
    try {
      auto& m = models_[size_t(h.model)];
      y.resize(size_t(h.rows) * m->out_cols(h.cols));
      if (delay_us_) std::this_thread::sleep_for(std::chrono::microseconds(delay_us_));
      m->run_cpu(x.data(), h.rows, h.cols, y.data());
    } catch (...) {
      f_->close();  // rank 0's outstanding calls fail instead of waiting for replies
      throw;
    }
    f_->send_y(y.data(), y.size() * sizeof(double), 0);
    batches_++;
    rows_ += uint64_t(h.rows);
  }
}

}  // namespace sca::par
