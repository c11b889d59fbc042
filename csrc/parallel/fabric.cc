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

std::string rccl_unique_ids(int world, int per_link) {
  if (world < 2) return std::string();
  if (per_link != 1 && per_link != 2) throw std::runtime_error("rccl_unique_ids: 1 or 2 communicators per link");
  std::vector<ncclUniqueId> ids(size_t(per_link * (world - 1)));
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
               LoopbackHubPtr hub, int comms_per_link)
    : rank_(rank), world_(world), device_(device), hub_(std::move(hub)), fds_(std::move(ctrl_fds)),
      per_link_(comms_per_link) {
  if (rank < 0 || rank >= world) throw std::runtime_error("Fabric: rank out of range");
  if (device < 0) throw std::runtime_error("Fabric: the RCCL / loopback fabric needs a GPU (CPU gangs use the shm mesh)");
  if (per_link_ != 1 && per_link_ != 2) throw std::runtime_error("Fabric: 1 or 2 communicators per link");
  if (int(fds_.size()) != world) throw std::runtime_error("Fabric: need one control socket slot per rank");
  if (hub_ && hub_->device() != device) throw std::runtime_error("Fabric: loopback hub lives on another GPU");
  links_.resize(size_t(world));
  for (int r = 0; r < world; ++r)
    if ((rank == 0) != (r == 0)) links_[size_t(r)] = std::make_unique<Link>();
  map_rings();
  gpu::DeviceGuard g(device);
  for (auto& l : links_)
    if (l) {
      l->sx.create(device);
      if (per_link_ == 2) l->sy.create(device);
    }
  if (hub_) return;
  if (unique_ids.size() != size_t(per_link_ * (world - 1)) * sizeof(ncclUniqueId))
    throw std::runtime_error("Fabric: bad RCCL unique id blob size");
  auto id_of = [&](int link, int chan) {
    ncclUniqueId id;
    std::memcpy(&id, unique_ids.data() + size_t(per_link_ * (link - 1) + chan) * sizeof(ncclUniqueId), sizeof id);
    return id;
  };
  // One 2-rank communicator (pair) per rank-0 <-> worker link: rank 0 is rank
  // 0 of each, the worker rank 1.  Rank 0 joins its links in worker order; a
  // worker waits in its init until rank 0 reaches its link.  With one
  // communicator per link, X and Y share it and one stream, so every
  // operation of a communicator is issued from a single stream.
  for (int r = 1; r < world; ++r) {
    if (rank != 0 && rank != r) continue;
    Link& l = *links_[size_t(rank == 0 ? r : 0)];
    SCA_NCCL_CHECK(ncclCommInitRank(&l.cx, 2, id_of(r, kChanX), rank == 0 ? 0 : 1));
    if (per_link_ == 2) SCA_NCCL_CHECK(ncclCommInitRank(&l.cy, 2, id_of(r, kChanY), rank == 0 ? 0 : 1));
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
        if (l && (hipStreamQuery(l->sx.get()) != hipSuccess || (l->sy.get() && hipStreamQuery(l->sy.get()) != hipSuccess)))
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
    if (fd >= 0) {
      ::shutdown(fd, SHUT_RDWR);
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

void Fabric::xfer(bool send, int chan, void* p, size_t bytes, int peer) {
  Link& l = link(peer);
  hipStream_t s = chan == kChanX || per_link_ == 1 ? l.sx.get() : l.sy.get();
  if (hub_) {
    if (send) hub_->send(rank_, peer, chan, p, bytes, s);
    else hub_->recv(peer, rank_, chan, p, bytes, s);
    return;
  }
  ncclComm_t c = chan == kChanX || per_link_ == 1 ? l.cx : l.cy;
  const int to = rank_ == 0 ? 1 : 0;  // the other end, as a rank of the link's 2-rank communicator
  if (send) SCA_NCCL_CHECK(ncclSend(p, bytes, ncclChar, to, c, s));
  else SCA_NCCL_CHECK(ncclRecv(p, bytes, ncclChar, to, c, s));
}

void Fabric::send_x(const void* p, size_t bytes, int peer) { xfer(true, kChanX, const_cast<void*>(p), bytes, peer); }
void Fabric::recv_x(void* p, size_t bytes, int peer) { xfer(false, kChanX, p, bytes, peer); }
void Fabric::send_y(const void* p, size_t bytes, int peer) { xfer(true, kChanY, const_cast<void*>(p), bytes, peer); }
void Fabric::recv_y(void* p, size_t bytes, int peer) { xfer(false, kChanY, p, bytes, peer); }

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

void PeerRowModel::run_cpu(const double*, int, int, double*) const {
  throw std::runtime_error("rccl_peer: GPU fabric models run on their GPU (CPU gangs use the shm mesh)");
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
  m->to_device(f_->device());
  models_.push_back(std::move(m));
  return int(models_.size()) - 1;
}

void PeerServer::start() {
  if (th_.joinable()) return;
  th_ = std::thread([this] {
    try {
      loop();
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

}  // namespace sca::par
