#include "fabric.h"

#include <immintrin.h>

#include <algorithm>
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
constexpr size_t kHeaderBytes = 256;  // 4 x int32 header, padded so payload stays 256-B aligned

void wait_event(hipEvent_t e) {
  int spins = 0;
  hipError_t st;
  while ((st = hipEventQuery(e)) == hipErrorNotReady) {
    if (++spins < 4000) _mm_pause();
    else std::this_thread::yield();
  }
  SCA_HIP_CHECK(st);
}
}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  SCA_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof id);
}

// ------------------------------------------------------------------ fabric
Fabric::Fabric(int rank, int world, const std::string& unique_id, int device)
    : rank_(rank), world_(world), device_(device) {
  if (unique_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("Fabric: bad RCCL unique id size");
  if (rank < 0 || rank >= world) throw std::runtime_error("Fabric: rank out of range");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof id);
  gpu::DeviceGuard g(device);
  stream_.create(device);
  SCA_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

Fabric::~Fabric() { close(); }

void Fabric::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (!comm_) return;
  gpu::DeviceGuard d(device_);
  (void)hipStreamSynchronize(stream_.get());
  (void)ncclCommDestroy(comm_);
  comm_ = nullptr;
}

void stop_peers(Fabric& f) {
  std::lock_guard<std::mutex> g(f.issue_mutex());
  if (!f.comm()) return;
  gpu::DeviceGuard d(f.device());
  gpu::DeviceBuffer hdr(kHeaderBytes, f.device());
  kern::fill_i32x4(hdr.as<int32_t>(), kPeerStop, 0, 0, 0, f.stream());
  SCA_NCCL_CHECK(ncclGroupStart());
  for (int r = 0; r < f.world(); ++r)
    if (r != f.rank()) SCA_NCCL_CHECK(ncclSend(hdr.get(), 4, ncclInt32, r, f.comm(), f.stream()));
  SCA_NCCL_CHECK(ncclGroupEnd());
  SCA_HIP_CHECK(hipStreamSynchronize(f.stream()));
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
  // header + one gathered output slab per peer (fan-out combine)
  return kHeaderBytes + (peers_.size() > 1 ? peers_.size() * size_t(max_rows) * out_cols_ * sizeof(double) : 0);
}

void PeerRowModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  std::lock_guard<std::mutex> g(f_->issue_mutex());
  if (!f_->comm()) throw std::runtime_error("RCCL fabric closed");
  hipStream_t fs = f_->stream();
  auto* hdr = static_cast<int32_t*>(ws);
  SCA_HIP_CHECK(hipEventRecord(ev_in_.get(), s));  // X staged on the batcher's stream
  SCA_HIP_CHECK(hipStreamWaitEvent(fs, ev_in_.get(), 0));
  kern::fill_i32x4(hdr, kPeerRun, model_id_, rows, cols, fs);
  const size_t nx = size_t(rows) * cols, ny = size_t(rows) * out_cols_;
  ncclComm_t c = f_->comm();
  if (peers_.size() == 1) {
    const int p = peers_[0];
    SCA_NCCL_CHECK(ncclSend(hdr, 4, ncclInt32, p, c, fs));
    SCA_NCCL_CHECK(ncclSend(X, nx, ncclFloat64, p, c, fs));
    SCA_NCCL_CHECK(ncclRecv(out, ny, ncclFloat64, p, c, fs));
  } else {
    // scatter the header + broadcast the batch, then gather every replica's output
    auto* slabs = reinterpret_cast<double*>(static_cast<char*>(ws) + kHeaderBytes);
    SCA_NCCL_CHECK(ncclGroupStart());
    for (int p : peers_) SCA_NCCL_CHECK(ncclSend(hdr, 4, ncclInt32, p, c, fs));
    SCA_NCCL_CHECK(ncclGroupEnd());
    SCA_NCCL_CHECK(ncclGroupStart());
    for (size_t i = 0; i < peers_.size(); ++i) {
      SCA_NCCL_CHECK(ncclSend(X, nx, ncclFloat64, peers_[i], c, fs));
      SCA_NCCL_CHECK(ncclRecv(slabs + i * ny, ny, ncclFloat64, peers_[i], c, fs));
    }
    SCA_NCCL_CHECK(ncclGroupEnd());
    kern::combine_mean_strided_f64(slabs, int(peers_.size()), int64_t(ny), out, fs);
  }
  SCA_HIP_CHECK(hipEventRecord(ev_done_.get(), fs));
  SCA_HIP_CHECK(hipStreamWaitEvent(s, ev_done_.get(), 0));
}

void PeerRowModel::run_cpu(const double*, int, int, double*) const {
  throw std::runtime_error("rccl_peer models run on GPUs only");
}

// ---------------------------------------------------------------- worker side
PeerServer::PeerServer(FabricPtr fabric) : f_(std::move(fabric)) {}

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

void PeerServer::loop() {
  gpu::DeviceGuard g(f_->device());
  const int dev = f_->device();
  hipStream_t fs = f_->stream();
  ncclComm_t c = f_->comm();
  gpu::DeviceBuffer hdr(kHeaderBytes, dev);
  gpu::PinnedBuffer hh(kHeaderBytes);
  gpu::Event ev;
  ev.create(dev);
  gpu::DeviceBuffer x, y, ws;
  while (true) {
    SCA_NCCL_CHECK(ncclRecv(hdr.get(), 4, ncclInt32, 0, c, fs));
    SCA_HIP_CHECK(hipMemcpyAsync(hh.host<int32_t>(), hdr.get(), 4 * sizeof(int32_t), hipMemcpyDeviceToHost, fs));
    SCA_HIP_CHECK(hipEventRecord(ev.get(), fs));
    wait_event(ev.get());
    const int32_t* h = hh.host<int32_t>();
    const int op = h[0], mid = h[1], rows = h[2], cols = h[3];
    if (op == kPeerStop) break;
    if (mid < 0 || mid >= int(models_.size()) || rows <= 0 || cols <= 0)
      throw std::runtime_error("PeerServer: bad header (model " + std::to_string(mid) + ")");
    auto& m = models_[size_t(mid)];
    const int oc = m->out_cols(cols);
    const size_t bx = size_t(rows) * cols * sizeof(double), by = size_t(rows) * oc * sizeof(double);
    const size_t bw = m->workspace_bytes(rows, cols);
    if (bx > x.bytes() || by > y.bytes() || bw > ws.bytes()) {
      SCA_HIP_CHECK(hipStreamSynchronize(fs));  // previous batch may still use the buffers
      if (bx > x.bytes()) x.alloc(std::max(bx, 2 * x.bytes()), dev);
      if (by > y.bytes()) y.alloc(std::max(by, 2 * y.bytes()), dev);
      if (bw > ws.bytes()) ws.alloc(std::max(bw, 2 * ws.bytes()), dev);
    }
    SCA_NCCL_CHECK(ncclRecv(x.get(), size_t(rows) * cols, ncclFloat64, 0, c, fs));
    m->launch(x.as<double>(), rows, cols, y.as<double>(), ws.get(), fs);
    SCA_NCCL_CHECK(ncclSend(y.get(), size_t(rows) * oc, ncclFloat64, 0, c, fs));
    batches_++;
    rows_ += uint64_t(rows);
  }
  SCA_HIP_CHECK(hipStreamSynchronize(fs));
}

}  // namespace sca::par
