#include "fabric.h"

#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
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
}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  SCA_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof id);
}

// ------------------------------------------------------------------ fabric
Fabric::Fabric(int rank, int world, const std::string& unique_id, int device, std::vector<int> ctrl_fds)
    : rank_(rank), world_(world), device_(device), fds_(std::move(ctrl_fds)) {
  if (rank < 0 || rank >= world) throw std::runtime_error("Fabric: rank out of range");
  if (int(fds_.size()) != world) throw std::runtime_error("Fabric: need one control socket slot per rank");
  if (device_ < 0) return;
  if (unique_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("Fabric: bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof id);
  gpu::DeviceGuard g(device);
  stream_.create(device);
  SCA_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

Fabric::~Fabric() { close(); }

void Fabric::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (!open_) return;
  open_ = false;
  if (comm_) {
    gpu::DeviceGuard d(device_);
    (void)hipStreamSynchronize(stream_.get());
    (void)ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  for (int& fd : fds_)
    if (fd >= 0) {
      ::shutdown(fd, SHUT_RDWR);
      ::close(fd);
      fd = -1;
    }
}

int Fabric::fd(int peer) const {
  if (peer < 0 || peer >= world_ || fds_[size_t(peer)] < 0)
    throw std::runtime_error("Fabric: no control link to rank " + std::to_string(peer));
  return fds_[size_t(peer)];
}

void Fabric::send_header(int peer, const PeerHeader& h) { write_all(fd(peer), &h, sizeof h); }

PeerHeader Fabric::recv_header(int peer) {
  PeerHeader h;
  read_all(fd(peer), &h, sizeof h);
  return h;
}

void Fabric::send(const void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclSend(p, bytes, ncclChar, peer, comm_, stream_.get()));
  else write_all(fd(peer), p, bytes);
}

void Fabric::recv(void* p, size_t bytes, int peer) {
  if (gpu()) SCA_NCCL_CHECK(ncclRecv(p, bytes, ncclChar, peer, comm_, stream_.get()));
  else read_all(fd(peer), p, bytes);
}

void Fabric::group_start() {
  if (gpu()) SCA_NCCL_CHECK(ncclGroupStart());
}

void Fabric::group_end() {
  if (gpu()) SCA_NCCL_CHECK(ncclGroupEnd());
}

void stop_peers(Fabric& f) {
  std::lock_guard<std::mutex> g(f.issue_mutex());
  if (!f.open()) return;
  PeerHeader h;
  h.op = kPeerStop;
  for (int r = 0; r < f.world(); ++r)
    if (r != f.rank()) f.send_header(r, h);
  if (f.gpu()) SCA_HIP_CHECK(hipStreamSynchronize(f.stream()));
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
  for (int p : peers_) f_->send_header(p, h);
}

void PeerRowModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  std::lock_guard<std::mutex> g(f_->issue_mutex());
  if (!f_->open()) throw std::runtime_error("RCCL fabric closed");
  hipStream_t fs = f_->stream();
  SCA_HIP_CHECK(hipEventRecord(ev_in_.get(), s));  // X staged on the batcher's stream
  SCA_HIP_CHECK(hipStreamWaitEvent(fs, ev_in_.get(), 0));
  headers(rows, cols);  // host -> worker hosts, immediately; the payloads follow stream-ordered
  const size_t bx = size_t(rows) * cols * sizeof(double), by = size_t(rows) * out_cols_ * sizeof(double);
  if (peers_.size() == 1) {
    f_->send(X, bx, peers_[0]);
    f_->recv(out, by, peers_[0]);
  } else {
    // broadcast the batch, gather every replica's output, average on this GPU
    auto* slabs = static_cast<double*>(ws);
    f_->group_start();
    for (size_t i = 0; i < peers_.size(); ++i) {
      f_->send(X, bx, peers_[i]);
      f_->recv(slabs + i * size_t(rows) * out_cols_, by, peers_[i]);
    }
    f_->group_end();
    kern::combine_mean_strided_f64(slabs, int(peers_.size()), int64_t(rows) * out_cols_, out, fs);
  }
  SCA_HIP_CHECK(hipEventRecord(ev_done_.get(), fs));
  SCA_HIP_CHECK(hipStreamWaitEvent(s, ev_done_.get(), 0));
  batches_++;
}

void PeerRowModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  if (f_->gpu()) throw std::runtime_error("rccl_peer: GPU fabric models run on their GPU");
  std::lock_guard<std::mutex> g(f_->issue_mutex());
  if (!f_->open()) throw std::runtime_error("fabric closed");
  headers(rows, cols);
  const size_t bx = size_t(rows) * cols * sizeof(double), ny = size_t(rows) * out_cols_;
  for (int p : peers_) f_->send(X, bx, p);
  if (peers_.size() == 1) {
    f_->recv(out, ny * sizeof(double), peers_[0]);
  } else {
    std::vector<double> slab(ny);
    std::fill(out, out + ny, 0.0);
    for (int p : peers_) {
      f_->recv(slab.data(), ny * sizeof(double), p);
      for (size_t i = 0; i < ny; ++i) out[i] += slab[i];
    }
    for (size_t i = 0; i < ny; ++i) out[i] /= double(peers_.size());
  }
  batches_++;
}

// ---------------------------------------------------------------- worker side
PeerServer::PeerServer(FabricPtr fabric) : f_(std::move(fabric)) {}

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

// GPU worker: the header arrives on the host socket, so receive, kernel and
// reply are posted back to back on the fabric stream -- the thread never
// waits on the device except to grow its buffers.
void PeerServer::loop() {
  gpu::DeviceGuard g(f_->device());
  const int dev = f_->device();
  hipStream_t fs = f_->stream();
  gpu::DeviceBuffer x, y, ws;
  while (true) {
    const PeerHeader h = f_->recv_header(0);
    if (h.op == kPeerStop) break;
    if (h.model < 0 || h.model >= int(models_.size()) || h.rows <= 0 || h.cols <= 0)
      throw std::runtime_error("PeerServer: bad header (model " + std::to_string(h.model) + ")");
    auto& m = models_[size_t(h.model)];
    const int oc = m->out_cols(h.cols);
    const size_t bx = size_t(h.rows) * h.cols * sizeof(double), by = size_t(h.rows) * oc * sizeof(double);
    const size_t bw = m->workspace_bytes(h.rows, h.cols);
    if (bx > x.bytes() || by > y.bytes() || bw > ws.bytes()) {
      SCA_HIP_CHECK(hipStreamSynchronize(fs));  // earlier batches may still use the buffers
      host_syncs_++;
      if (bx > x.bytes()) x.alloc(std::max(bx, 2 * x.bytes()), dev);
      if (by > y.bytes()) y.alloc(std::max(by, 2 * y.bytes()), dev);
      if (bw > ws.bytes()) ws.alloc(std::max(bw, 2 * ws.bytes()), dev);
    }
    f_->recv(x.get(), bx, 0);
    m->launch(x.as<double>(), h.rows, h.cols, y.as<double>(), ws.get(), fs);
    f_->send(y.get(), by, 0);
    batches_++;
    rows_ += uint64_t(h.rows);
  }
  SCA_HIP_CHECK(hipStreamSynchronize(fs));
}

// CPU worker (device -1 fabrics): the same protocol with the payloads on the
// sockets and the model's CPU path.
void PeerServer::loop_cpu() {
  std::vector<double> x, y;
  while (true) {
    const PeerHeader h = f_->recv_header(0);
    if (h.op == kPeerStop) break;
    if (h.model < 0 || h.model >= int(models_.size()) || h.rows <= 0 || h.cols <= 0)
      throw std::runtime_error("PeerServer: bad header (model " + std::to_string(h.model) + ")");
    auto& m = models_[size_t(h.model)];
    const int oc = m->out_cols(h.cols);
    x.resize(size_t(h.rows) * h.cols);
    y.resize(size_t(h.rows) * oc);
    f_->recv(x.data(), x.size() * sizeof(double), 0);
    m->run_cpu(x.data(), h.rows, h.cols, y.data());
    f_->send(y.data(), y.size() * sizeof(double), 0);
    batches_++;
    rows_ += uint64_t(h.rows);
  }
}

}  // namespace sca::par
