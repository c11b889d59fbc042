#include "mesh.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <linux/futex.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <climits>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <set>
#include <stdexcept>

#include "../kernels/kernels.h"

namespace sca::par {

namespace {
using clk = std::chrono::steady_clock;
constexpr size_t kLine = 64;
constexpr size_t kErrText = 256;
constexpr size_t kPage = 4096;
constexpr size_t kZeroCopyMax = 256 << 10;  // larger batches go through HBM (batcher.h)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
uint64_t load_acq(const char* p) { return __atomic_load_n(reinterpret_cast<const uint64_t*>(p), __ATOMIC_ACQUIRE); }
void store_rel(char* p, uint64_t v) { __atomic_store_n(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELEASE); }

bool fd_gone(int f) {
  if (f < 0) return true;
  char c;
  const ssize_t r = ::recv(f, &c, 1, MSG_PEEK | MSG_DONTWAIT);
  return r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
}

int env_int(const char* k, int dflt) {
  const char* e = std::getenv(k);
  return e ? std::atoi(e) : dflt;
}
}  // namespace

// ------------------------------------------------------------------ layout
// Where rank c keeps its part of a program (identical arithmetic on every rank).
struct Layout {
  std::vector<int> src;       // incoming sources: stage ids, -1 = program input; ascending
  std::vector<int> width;     // per source: columns
  std::vector<char> on_dev;   // per source: in the device slab allocation (GPU gangs, worker -> worker)
  std::vector<size_t> off;    // per source: slot 0's offset (region or device allocation)
  std::vector<size_t> slab;   // per source: bytes per slot
  size_t ring_off = 0, bell_off = 0, flags_off = 0, err_off = 0, bytes = 0, dev_bytes = 0;
  int index_of(int s) const {
    for (size_t i = 0; i < src.size(); ++i)
      if (src[i] == s) return int(i);
    return -1;
  }
};

// A region's futex doorbell: every host store into the region (a ready or
// freed flag, a ring header) bumps `seq` and wakes the sleepers, so host
// waiters on host-written flags sleep in the kernel instead of spinning.
// Flags written by a GPU (stream write-value) cannot ring it: their waiters
// poll.
struct Bell {
  std::atomic<uint32_t> seq;
  std::atomic<uint32_t> sleepers;
};

void bell_ring(Bell* b) {
  b->seq.fetch_add(1, std::memory_order_seq_cst);  // (full barrier: the flag store is visible first)
  if (b->sleepers.load(std::memory_order_seq_cst) != 0)
    syscall(SYS_futex, reinterpret_cast<uint32_t*>(&b->seq), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

struct Region {
  char* host = nullptr;  // the mapping
  char* hdev = nullptr;  // its device address (GPU workers; registered)
  char* dev = nullptr;   // device slabs (own allocation, or IPC-opened by a producer)
  size_t bytes = 0;
  bool registered = false, ipc = false;
  std::string name;
};

// Rank 0: one issued batch (a chunk of a call) waiting for its output.
struct CallState {
  double* out = nullptr;  // the batcher's buffer: written only while the call is live
  int out_cols = 0;
  bool abandoned = false;  // (guarded by the program's reap_mu) the caller gave up: never write `out` again
  std::atomic<int> remaining{0};
  std::mutex mu;
  std::string error;
};
using CallStatePtr = std::shared_ptr<CallState>;

struct Exec;  // a worker's per-program execution state

struct Prog {
  int id = 0;
  MeshProgram d;
  std::vector<char> part;                 // per rank
  std::vector<Layout> lay;                // per rank
  std::vector<Region> reg;                // per rank
  gpu::DeviceBuffer own_dev;              // this rank's device slabs
  std::vector<int> local;                 // stages on this rank, topological
  std::vector<std::vector<int>> consumers;  // per stage: remote consumer ranks
  std::vector<char> local_consumer;       // per stage: consumed by a stage on its own rank
  std::vector<std::pair<int, int>> alias;  // per rank: (consumer rank, stage) whose ready flag doubles as freed
  std::vector<gpu::RowModelPtr> model;    // per stage (own stages)
  std::vector<HostFn> fn;                 // per stage (own host stages)
  // rank 0
  std::mutex issue_mu;
  uint64_t next = 0;                      // last issued seq
  std::mutex reap_mu;
  struct Pend {
    uint64_t seq = 0;
    CallStatePtr call;
    int row0 = 0, rows = 0;
  };
  std::vector<Pend> pend;                 // per slot of rank 0's region
  uint64_t reaped = 0;                    // every seq <= reaped has been copied out
  // worker
  std::thread th;
  std::unique_ptr<Exec> ex;
  uint64_t taken = 0;                     // headers taken from the ring

  HeaderRing* ring(int r) const { return reinterpret_cast<HeaderRing*>(reg[size_t(r)].host + lay[size_t(r)].ring_off); }
  Bell* bell(int r) const { return reinterpret_cast<Bell*>(reg[size_t(r)].host + lay[size_t(r)].bell_off); }
  char* flag(int r, int k, int e) const {
    const Layout& L = lay[size_t(r)];
    return reg[size_t(r)].host + L.flags_off + (size_t(k) * (L.src.size() + 2) + size_t(e)) * kLine;
  }
  char* flag_dev(int r, int k, int e) const {
    const Layout& L = lay[size_t(r)];
    return reg[size_t(r)].hdev + L.flags_off + (size_t(k) * (L.src.size() + 2) + size_t(e)) * kLine;
  }
  char* ready(int r, int k, int src) const { return flag(r, k, lay[size_t(r)].index_of(src)); }
  char* freed(int r, int k) const { return flag(r, k, int(lay[size_t(r)].src.size())); }
  char* errf(int r, int k) const { return flag(r, k, int(lay[size_t(r)].src.size()) + 1); }
  char* err_text(int r, int k) const { return reg[size_t(r)].host + lay[size_t(r)].err_off + size_t(k) * kErrText; }
  // rank r's slab of `src` at slot k: host address, device address
  char* slab_host(int r, int src, int k) const {
    const Layout& L = lay[size_t(r)];
    const int e = L.index_of(src);
    return reg[size_t(r)].host + L.off[size_t(e)] + size_t(k) * L.slab[size_t(e)];
  }
  char* slab_dev(int r, int src, int k) const {
    const Layout& L = lay[size_t(r)];
    const int e = L.index_of(src);
    const size_t o = L.off[size_t(e)] + size_t(k) * L.slab[size_t(e)];
    return L.on_dev[size_t(e)] ? reg[size_t(r)].dev + o : reg[size_t(r)].hdev + o;
  }
  bool slab_on_dev(int r, int src) const {
    const Layout& L = lay[size_t(r)];
    return L.on_dev[size_t(L.index_of(src))] != 0;
  }
  int width_of(int src) const { return src < 0 ? d.in_cols : d.stages[size_t(src)].out_cols; }
};

struct Exec {
  gpu::Stream st;
  std::vector<gpu::DeviceBuffer> out;   // per stage id (own stages): K slots
  std::vector<size_t> out_slab;         // per stage id
  std::vector<gpu::DeviceBuffer> ws;    // per stage id
  std::vector<gpu::DeviceBuffer> tab;   // per stage id (mean): K x n_inputs device pointers
  gpu::DeviceBuffer xdev;               // staged program input, K slots
  size_t x_slab = 0;
  std::vector<std::vector<double>> hout;  // CPU gangs: per stage id, K slots
  std::vector<double> hx, hy;           // host-stage scratch (GPU gangs)
  std::vector<const double*> ptrs;      // CPU mean inputs
};

struct Mesh::Impl {
  std::vector<std::unique_ptr<Prog>> progs;
  // peer readiness (probe_*): [producer][consumer] 1 = device slabs over IPC
  std::vector<std::vector<int>> peer_ok;
  gpu::DeviceBuffer probe_buf;                 // this worker's probe buffer
  std::vector<void*> probe_opened;             // other workers' buffers, IPC-opened
  std::string probe_err;
  bool prepared = false, connected = false, started = false;
  int timeout_ms = 60000;
  int delay_us = 0;
  int spin_us = 100;
  mutable std::mutex err_mu;
  std::string err;
  std::atomic<uint64_t> batches{0}, rows{0}, max_inflight{0}, host_waits{0}, stage_errors{0};
  void note_inflight(uint64_t n) {
    uint64_t m = max_inflight.load(std::memory_order_relaxed);
    while (n > m && !max_inflight.compare_exchange_weak(m, n)) {
    }
  }
  void set_error(const std::string& e) {
    std::lock_guard<std::mutex> g(err_mu);
    if (err.empty()) err = e;
  }
};

// ------------------------------------------------------------------ waiting
namespace {
// Wait for ready(): spin for `spin_us` (the usual back-to-back hand-off),
// then -- when the flag's writer is a host thread that rings `bell` -- sleep
// on the region's futex in 1 ms slices, else (a GPU writes the flag) yield
// for 200 us and then sleep 20 us at a time.  `check(elapsed)` runs between
// slices and throws when the wait is hopeless (peer gone, mesh closed,
// timeout).  Returns whether it had to wait at all.
template <class Ready, class Check>
bool wait_ready(Ready ready, Check check, Bell* bell, int spin_us) {
  if (ready()) return false;
  const auto t0 = clk::now();
  const auto spin = std::chrono::microseconds(spin_us);
  do {
    for (int i = 0; i < 32; ++i) _mm_pause();
    if (ready()) return true;
  } while (clk::now() - t0 < spin);
  if (bell) {
    while (true) {
      const uint32_t s = bell->seq.load(std::memory_order_seq_cst);
      bell->sleepers.fetch_add(1, std::memory_order_seq_cst);
      if (ready()) {
        bell->sleepers.fetch_sub(1, std::memory_order_seq_cst);
        return true;
      }
      const timespec ts{0, 1000000};
      syscall(SYS_futex, reinterpret_cast<uint32_t*>(&bell->seq), FUTEX_WAIT, s, &ts, nullptr, 0);
      bell->sleepers.fetch_sub(1, std::memory_order_seq_cst);
      if (ready()) return true;
      check(clk::now() - t0);
    }
  }
  while (!ready()) {
    const auto dt = clk::now() - t0;
    if (dt < spin + std::chrono::microseconds(200)) {
      std::this_thread::yield();
    } else {
      check(dt);
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  return true;
}

template <class Ready, class Check>
bool wait_until(Ready ready, Check check) {
  return wait_ready(ready, check, nullptr, 20);
}
}  // namespace

// ------------------------------------------------------------------ mesh
Mesh::Mesh(int rank, int world, int device, std::vector<int> ctrl_fds, int slots)
    : rank_(rank), world_(world), device_(device), K_(std::max(1, std::min(64, slots))), fds_(std::move(ctrl_fds)),
      im_(std::make_unique<Impl>()) {
  if (rank < 0 || rank >= world) throw std::runtime_error("Mesh: rank out of range");
  if (int(fds_.size()) != world) throw std::runtime_error("Mesh: need one control socket slot per rank");
  im_->timeout_ms = std::max(100, env_int("SCA_MESH_TIMEOUT_MS", 60000));
  im_->delay_us = std::max(0, env_int("SCA_FABRIC_WORKER_DELAY_US", 0));
  im_->spin_us = std::max(0, env_int("SCA_MESH_SPIN_US", 100));
}

Mesh::~Mesh() {
  close();
  join();
  std::unique_ptr<gpu::DeviceGuard> g;
  if (gpu() && rank_ != 0) g = std::make_unique<gpu::DeviceGuard>(device_);
  for (auto& P : im_->progs) {
    P->ex.reset();
    for (size_t r = 0; r < P->reg.size(); ++r) {
      Region& R = P->reg[r];
      if (R.ipc && R.dev) (void)hipIpcCloseMemHandle(R.dev);
      if (R.registered) (void)hipHostUnregister(R.host);
      if (R.host) munmap(R.host, R.bytes);
      R = Region{};
    }
    P->own_dev.reset();
  }
  g.reset();
  for (int& f : fds_)
    if (f >= 0) {
      ::close(f);
      f = -1;
    }
}

int Mesh::add_program(MeshProgram d) {
  if (im_->prepared) throw std::runtime_error("Mesh: add programs before prepare()");
  auto P = std::make_unique<Prog>();
  P->id = int(im_->progs.size());
  const int n = int(d.stages.size());
  if (n == 0) throw std::runtime_error("Mesh: empty program");
  if (d.max_rows <= 0 || d.in_cols <= 0) throw std::runtime_error("Mesh: program needs max_rows and in_cols");
  for (int i = 0; i < n; ++i) {
    const MeshStage& s = d.stages[size_t(i)];
    const std::string where = "Mesh: stage " + std::to_string(i) + " (" + s.node + ")";
    if (s.rank < 0 || s.rank >= world_) throw std::runtime_error(where + ": rank out of range");
    if (s.out_cols <= 0) throw std::runtime_error(where + ": output width unknown");
    if (s.inputs.empty()) throw std::runtime_error(where + ": no inputs");
    for (int j : s.inputs) {
      if (j >= i || j < -1) throw std::runtime_error(where + ": inputs must come earlier");
      if (j == -1 && s.rank == 0) throw std::runtime_error(where + ": rank 0 cannot take the program input");
      if (j >= 0 && s.rank == 0 && d.stages[size_t(j)].rank == 0)
        throw std::runtime_error(where + ": rank-0 stages must read remote outputs");
    }
    if (s.kind != kMeshMean && s.inputs.size() != 1) throw std::runtime_error(where + ": one input per model stage");
    if (s.rank == 0 && (i != n - 1 || s.kind != kMeshMean))
      throw std::runtime_error(where + ": only the final mean may run on rank 0");
    if (s.kind == kMeshMean)
      for (int j : s.inputs)
        if ((j >= 0 ? d.stages[size_t(j)].out_cols : d.in_cols) != s.out_cols)
          throw std::runtime_error(where + ": mean over inputs of different widths");
  }
  P->d = std::move(d);
  const auto& st = P->d.stages;
  P->part.assign(size_t(world_), 0);
  P->part[0] = 1;
  for (auto& s : st) P->part[size_t(s.rank)] = 1;
  P->consumers.assign(size_t(n), {});
  P->local_consumer.assign(size_t(n), 0);
  P->lay.assign(size_t(world_), Layout{});
  for (int c = 0; c < world_; ++c) {
    if (!P->part[size_t(c)]) continue;
    std::set<int> S;
    for (int i = 0; i < n; ++i) {
      if (st[size_t(i)].rank != c) continue;
      for (int j : st[size_t(i)].inputs) {
        if (j == -1) S.insert(-1);
        else if (st[size_t(j)].rank != c) S.insert(j);
        else P->local_consumer[size_t(j)] = 1;
      }
    }
    if (c == 0 && st.back().rank != 0) S.insert(n - 1);
    Layout& L = P->lay[size_t(c)];
    L.src.assign(S.begin(), S.end());
    size_t cur = 0;
    if (c != 0) {
      L.ring_off = 0;
      cur = align_up(sizeof(HeaderRing), kLine);
    }
    L.bell_off = cur;
    cur += kLine;
    L.flags_off = cur;
    cur += size_t(K_) * (L.src.size() + 2) * kLine;
    L.err_off = cur;
    cur += size_t(K_) * kErrText;
    cur = align_up(cur, kPage);
    size_t dcur = 0;
    for (int s : L.src) {
      const int w = P->width_of(s);
      const size_t slab = align_up(size_t(P->d.max_rows) * size_t(w) * sizeof(double), 256);
      // worker -> worker edges land in the consumer's HBM unless the peer
      // probe failed for the producing rank (then: host-staged, "ipc-host")
      bool dev = gpu() && c != 0 && s != -1;
      if (dev && !im_->peer_ok.empty()) {
        const int prod = P->d.stages[size_t(s)].rank;
        dev = im_->peer_ok[size_t(prod)][size_t(c)] != 0;
      }
      L.width.push_back(w);
      L.on_dev.push_back(dev ? 1 : 0);
      L.slab.push_back(slab);
      if (dev) {
        L.off.push_back(dcur);
        dcur += size_t(K_) * slab;
      } else {
        L.off.push_back(cur);
        cur += size_t(K_) * slab;
      }
    }
    L.bytes = align_up(cur, kPage);
    L.dev_bytes = dcur;
    for (int s : L.src)
      if (s >= 0) P->consumers[size_t(s)].push_back(c);
  }
  P->alias.assign(size_t(world_), {-1, -1});
  for (int c = 1; c < world_; ++c) {
    if (!P->part[size_t(c)]) continue;
    std::vector<std::pair<int, int>> outs;
    for (int i = 0; i < n; ++i)
      if (st[size_t(i)].rank == c)
        for (int d2 : P->consumers[size_t(i)]) outs.push_back({d2, i});
    if (outs.size() == 1) P->alias[size_t(c)] = outs[0];
  }
  for (int i = 0; i < n; ++i)
    if (st[size_t(i)].rank == rank_ && rank_ != 0) P->local.push_back(i);
  P->model.assign(size_t(n), nullptr);
  P->fn.assign(size_t(n), nullptr);
  P->reg.assign(size_t(world_), Region{});
  P->pend.assign(size_t(K_), Prog::Pend{});
  im_->progs.push_back(std::move(P));
  return int(im_->progs.size()) - 1;
}

void Mesh::set_model(int prog, int stage, gpu::RowModelPtr m) {
  Prog& P = *im_->progs.at(size_t(prog));
  const MeshStage& s = P.d.stages.at(size_t(stage));
  if (s.rank != rank_ || s.kind != kMeshModel) throw std::runtime_error("Mesh::set_model: not a model stage of this rank");
  P.model[size_t(stage)] = std::move(m);
}

void Mesh::set_host_fn(int prog, int stage, HostFn f) {
  Prog& P = *im_->progs.at(size_t(prog));
  const MeshStage& s = P.d.stages.at(size_t(stage));
  if (s.rank != rank_ || s.kind != kMeshHost) throw std::runtime_error("Mesh::set_host_fn: not a host stage of this rank");
  P.fn[size_t(stage)] = std::move(f);
}

int Mesh::messages_per_batch(int prog) const {
  const Prog& P = *im_->progs.at(size_t(prog));
  int m = 0;
  for (int c = 1; c < world_; ++c)
    if (P.part[size_t(c)] && P.lay[size_t(c)].index_of(-1) >= 0) ++m;
  for (auto& cs : P.consumers) m += int(cs.size());
  return m;
}

// ------------------------------------------------------------------ probe
namespace {
constexpr int kProbeLane = 32;  // doubles per rank lane of a probe buffer
double probe_value(int owner, int writer, int i) { return 1e6 * (owner + 1) + 1e3 * (writer + 1) + i + 0.25; }
}  // namespace

std::string Mesh::probe_prepare() {
  std::string blob(1 + sizeof(hipIpcMemHandle_t), '\0');
  if (!gpu() || rank_ == 0) return blob;
  gpu::DeviceGuard g(device_);
  const size_t bytes = size_t(world_) * kProbeLane * sizeof(double);
  im_->probe_buf.alloc(bytes, device_, true);  // fine-grained, like the program slabs
  std::vector<double> pat(size_t(world_) * kProbeLane, 0.0);
  for (int i = 0; i < kProbeLane; ++i) pat[size_t(rank_) * kProbeLane + size_t(i)] = probe_value(rank_, rank_, i);
  SCA_HIP_CHECK(hipMemcpy(im_->probe_buf.get(), pat.data(), bytes, hipMemcpyHostToDevice));
  hipIpcMemHandle_t h{};
  SCA_HIP_CHECK(hipIpcGetMemHandle(&h, im_->probe_buf.get()));
  blob[0] = 1;
  std::memcpy(&blob[1], &h, sizeof h);
  return blob;
}

std::vector<int> Mesh::probe_connect(const std::vector<std::string>& blobs) {
  if (int(blobs.size()) != world_) throw std::runtime_error("Mesh::probe_connect: one blob per rank");
  std::vector<int> res(size_t(world_), -1);
  im_->probe_opened.assign(size_t(world_), nullptr);
  if (!gpu() || rank_ == 0) return res;
  const char* fe = std::getenv("SCA_MESH_FAULT");
  const std::string fault = fe ? fe : "";
  gpu::DeviceGuard g(device_);
  gpu::DeviceBuffer mine(kProbeLane * sizeof(double), device_);
  std::vector<double> pat(kProbeLane), back(kProbeLane);
  auto note = [&](int r, const std::string& why) {
    res[size_t(r)] = 0;
    if (im_->probe_err.empty()) im_->probe_err = "rank " + std::to_string(rank_) + " -> " + std::to_string(r) + ": " + why;
  };
  for (int r = 1; r < world_; ++r) {
    if (r == rank_) {
      res[size_t(r)] = 1;
      continue;
    }
    const std::string& b = blobs[size_t(r)];
    if (b.size() < 1 + sizeof(hipIpcMemHandle_t) || b[0] == 0) {
      note(r, "no probe buffer exported");
      continue;
    }
    if (fault == "peer") {
      note(r, "injected hipIpcOpenMemHandle failure (SCA_MESH_FAULT=peer)");
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, b.data() + 1, sizeof h);
    void* dv = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&dv, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess || !dv) {
      (void)hipGetLastError();
      note(r, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
      continue;
    }
    im_->probe_opened[size_t(r)] = dv;
    // the programs' write path: a device-to-device copy into the peer's HBM
    for (int i = 0; i < kProbeLane; ++i) pat[size_t(i)] = probe_value(r, rank_, i);
    double* lane = static_cast<double*>(dv) + size_t(rank_) * kProbeLane;
    double* owner = static_cast<double*>(dv) + size_t(r) * kProbeLane;
    bool ok = hipMemcpy(mine.get(), pat.data(), kProbeLane * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(lane, mine.get(), kProbeLane * sizeof(double), hipMemcpyDeviceToDevice) == hipSuccess &&
              hipDeviceSynchronize() == hipSuccess &&
              hipMemcpy(back.data(), lane, kProbeLane * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
    if (!ok) {
      (void)hipGetLastError();
      note(r, "canary copy failed");
      continue;
    }
    for (int i = 0; i < kProbeLane && ok; ++i) ok = back[size_t(i)] == pat[size_t(i)];
    if (ok && hipMemcpy(back.data(), owner, kProbeLane * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess) {
      for (int i = 0; i < kProbeLane && ok; ++i) ok = back[size_t(i)] == probe_value(r, r, i);
    } else {
      ok = false;
    }
    if (fault == "canary") ok = false;
    if (!ok) note(r, fault == "canary" ? "injected canary mismatch (SCA_MESH_FAULT=canary)" : "canary mismatch");
    else res[size_t(r)] = 1;
  }
  return res;
}

std::string Mesh::probe_error() const { return im_->probe_err; }

void Mesh::probe_finish() {
  std::unique_ptr<gpu::DeviceGuard> g;
  if (gpu() && rank_ != 0) g = std::make_unique<gpu::DeviceGuard>(device_);
  for (void*& p : im_->probe_opened)
    if (p) {
      (void)hipIpcCloseMemHandle(p);
      p = nullptr;
    }
  im_->probe_buf.reset();
}

void Mesh::set_peer_ok(const std::vector<std::vector<int>>& ok) {
  if (!im_->progs.empty()) throw std::runtime_error("Mesh::set_peer_ok: before add_program");
  if (int(ok.size()) != world_) throw std::runtime_error("Mesh::set_peer_ok: world x world matrix");
  for (auto& row : ok)
    if (int(row.size()) != world_) throw std::runtime_error("Mesh::set_peer_ok: world x world matrix");
  im_->peer_ok = ok;
}

std::vector<std::tuple<int, int, std::string>> Mesh::edge_transports(int prog) const {
  const Prog& P = *im_->progs.at(size_t(prog));
  std::vector<std::tuple<int, int, std::string>> out;
  for (size_t i = 0; i < P.consumers.size(); ++i)
    for (int c : P.consumers[i]) {
      std::string t;
      if (!gpu()) t = "shm";
      else if (c == 0) t = "host";
      else t = P.slab_on_dev(c, int(i)) ? "ipc" : "ipc-host";
      out.emplace_back(int(i), c, t);
    }
  return out;
}

// Blob: per program [u8 part][u32 len][name][u8 has_dev][hipIpcMemHandle_t]
std::string Mesh::prepare() {
  if (im_->prepared) throw std::runtime_error("Mesh::prepare: called twice");
  static std::atomic<int> counter{0};
  std::string blob;
  auto put = [&](const void* p, size_t n) { blob.append(static_cast<const char*>(p), n); };
  for (auto& Pp : im_->progs) {
    Prog& P = *Pp;
    const uint8_t part = P.part[size_t(rank_)];
    put(&part, 1);
    std::string name;
    uint8_t has_dev = 0;
    hipIpcMemHandle_t h{};
    if (part) {
      const Layout& L = P.lay[size_t(rank_)];
      for (int s : P.local)
        if (s >= 0 && P.d.stages[size_t(s)].kind == kMeshModel && !P.model[size_t(s)])
          throw std::runtime_error("Mesh: stage '" + P.d.stages[size_t(s)].node + "' has no model on rank " +
                                   std::to_string(rank_));
      for (int s : P.local)
        if (P.d.stages[size_t(s)].kind == kMeshHost && !P.fn[size_t(s)])
          throw std::runtime_error("Mesh: host stage '" + P.d.stages[size_t(s)].node + "' has no function");
      name = "/sca_mesh_" + std::to_string(getpid()) + "_" + std::to_string(counter++) + "_p" + std::to_string(P.id);
      const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("Mesh: shm_open(" + name + ") failed: " + std::strerror(errno));
      if (ftruncate(fd, off_t(L.bytes)) != 0) {
        ::close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error(std::string("Mesh: ftruncate failed: ") + std::strerror(errno));
      }
      void* p = mmap(nullptr, L.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      ::close(fd);
      if (p == MAP_FAILED) {
        shm_unlink(name.c_str());
        throw std::runtime_error(std::string("Mesh: mmap failed: ") + std::strerror(errno));
      }
      Region& R = P.reg[size_t(rank_)];
      R.host = static_cast<char*>(p);  // fresh pages: every flag 0
      R.bytes = L.bytes;
      R.name = name;
      if (gpu() && rank_ != 0 && L.dev_bytes > 0) {
        // Producers on other GPUs write these slabs over xGMI and this GPU's
        // kernels then read them: fine-grained (coherent) memory keeps a line
        // of an earlier use of the slot from being served out of this GPU's
        // L2.  SCA_MESH_SLAB=coarse selects plain hipMalloc memory.
        static const bool coarse = [] {
          const char* e = std::getenv("SCA_MESH_SLAB");
          return e && std::string(e) == "coarse";
        }();
        P.own_dev.alloc(L.dev_bytes, device_, !coarse);
        gpu::DeviceGuard g(device_);
        SCA_HIP_CHECK(hipIpcGetMemHandle(&h, P.own_dev.get()));
        R.dev = static_cast<char*>(P.own_dev.get());
        has_dev = 1;
      }
    }
    const uint32_t n = uint32_t(name.size());
    put(&n, 4);
    put(name.data(), n);
    put(&has_dev, 1);
    put(&h, sizeof h);
  }
  im_->prepared = true;
  return blob;
}

void Mesh::connect(const std::vector<std::string>& blobs) {
  if (!im_->prepared || im_->connected) throw std::runtime_error("Mesh::connect: prepare() first, once");
  if (int(blobs.size()) != world_) throw std::runtime_error("Mesh::connect: one blob per rank");
  struct Entry {
    bool part;
    std::string name;
    bool has_dev;
    hipIpcMemHandle_t h;
  };
  std::vector<std::vector<Entry>> ent(static_cast<size_t>(world_));
  for (int r = 0; r < world_; ++r) {
    const std::string& b = blobs[size_t(r)];
    size_t o = 0;
    auto get = [&](void* p, size_t n) {
      if (o + n > b.size()) throw std::runtime_error("Mesh::connect: truncated blob from rank " + std::to_string(r));
      std::memcpy(p, b.data() + o, n);
      o += n;
    };
    for (size_t i = 0; i < im_->progs.size(); ++i) {
      Entry e{};
      uint8_t part = 0, hd = 0;
      uint32_t n = 0;
      get(&part, 1);
      get(&n, 4);
      e.name.resize(n);
      if (n) get(&e.name[0], n);
      get(&hd, 1);
      get(&e.h, sizeof e.h);
      e.part = part != 0;
      e.has_dev = hd != 0;
      ent[size_t(r)].push_back(std::move(e));
    }
  }
  const bool gpu_worker = gpu() && rank_ != 0;
  std::unique_ptr<gpu::DeviceGuard> g;
  if (gpu_worker) g = std::make_unique<gpu::DeviceGuard>(device_);
  for (auto& Pp : im_->progs) {
    Prog& P = *Pp;
    if (!P.part[size_t(rank_)]) continue;
    for (int r = 0; r < world_; ++r) {
      if (!P.part[size_t(r)]) continue;
      const Entry& e = ent[size_t(r)][size_t(P.id)];
      if (!e.part) throw std::runtime_error("Mesh::connect: rank " + std::to_string(r) + " disagrees on program " +
                                            std::to_string(P.id));
      Region& R = P.reg[size_t(r)];
      if (r != rank_) {
        const int fd = shm_open(e.name.c_str(), O_RDWR, 0600);
        if (fd < 0) throw std::runtime_error("Mesh: shm_open(" + e.name + ") failed: " + std::strerror(errno));
        void* p = mmap(nullptr, P.lay[size_t(r)].bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (p == MAP_FAILED) throw std::runtime_error(std::string("Mesh: mmap failed: ") + std::strerror(errno));
        R.host = static_cast<char*>(p);
        R.bytes = P.lay[size_t(r)].bytes;
        R.name = e.name;
      }
      if (gpu_worker) {
        SCA_HIP_CHECK(hipHostRegister(R.host, R.bytes, hipHostRegisterMapped | hipHostRegisterPortable));
        R.registered = true;
        void* dp = nullptr;
        SCA_HIP_CHECK(hipHostGetDevicePointer(&dp, R.host, 0));
        R.hdev = static_cast<char*>(dp);
        // open r's device slabs if a stage here produces into them
        bool produce = false;
        for (int s : P.local)
          for (int c : P.consumers[size_t(s)])
            if (c == r && P.slab_on_dev(r, s)) produce = true;
        if (r != rank_ && produce) {
          if (!e.has_dev) throw std::runtime_error("Mesh::connect: rank " + std::to_string(r) + " exported no slabs");
          void* dv = nullptr;
          SCA_HIP_CHECK(hipIpcOpenMemHandle(&dv, e.h, hipIpcMemLazyEnablePeerAccess));
          R.dev = static_cast<char*>(dv);
          R.ipc = true;
        }
      }
    }
  }
  im_->connected = true;
}

void Mesh::unlink() {
  for (auto& P : im_->progs) {
    Region& R = P->reg[size_t(rank_)];
    if (!R.name.empty() && R.host) shm_unlink(R.name.c_str());
  }
}

void Mesh::close() {
  open_.store(false);
}

void Mesh::join() {
  for (auto& P : im_->progs)
    if (P->th.joinable()) P->th.join();
}

std::string Mesh::error() const {
  std::lock_guard<std::mutex> g(im_->err_mu);
  return im_->err;
}

MeshStats Mesh::stats() const {
  MeshStats s;
  s.batches = im_->batches.load();
  s.rows = im_->rows.load();
  s.max_inflight = im_->max_inflight.load();
  s.host_waits = im_->host_waits.load();
  s.stage_errors = im_->stage_errors.load();
  return s;
}

// ------------------------------------------------------------- the workers
namespace {

struct WorkerCtx {
  Mesh* m;
  Mesh::Impl* im;
  Prog* P;
  int me, K;
  const std::vector<int>* fds;
  // Bounded host wait for a flag of another process; `bell`: the region's
  // doorbell when a host thread writes the flag (else polled).
  void wait_flag(const char* f, uint64_t v, const char* what, Bell* bell) {
    const bool waited = wait_ready([&] { return load_acq(f) >= v; },
                                   [&](clk::duration dt) {
                                     if (!m->open()) throw std::runtime_error("mesh closed");
                                     if (fd_gone((*fds)[0])) throw std::runtime_error("mesh: rank 0 is gone");
                                     if (dt > std::chrono::milliseconds(im->timeout_ms))
                                       throw std::runtime_error(std::string("mesh: no ") + what + " within " +
                                                                std::to_string(im->timeout_ms) + " ms");
                                   },
                                   bell, im->spin_us);
    if (waited) im->host_waits.fetch_add(1, std::memory_order_relaxed);
  }
  // A remote stage's output for this rank (written by the producer's host
  // on CPU gangs, by its GPU on GPU gangs).
  void wait_input(int k, int j, uint64_t seq) {
    wait_flag(P->ready(me, k, j), seq, "stage input", m->gpu() ? nullptr : P->bell(me));
  }
  uint64_t credit(int c, int k) const {
    const auto a = P->alias[size_t(c)];
    return a.first >= 0 ? load_acq(P->ready(a.first, k, a.second)) : load_acq(P->freed(c, k));
  }
  void wait_credit(int c, int k, uint64_t seq) {
    if (seq <= uint64_t(K)) return;
    const auto a = P->alias[size_t(c)];
    const int region = a.first >= 0 ? a.first : c;
    const char* f = a.first >= 0 ? P->ready(a.first, k, a.second) : P->freed(c, k);
    // rank 0 frees its own slots from the host; workers of a GPU gang from their streams
    Bell* b = (!m->gpu() || (a.first < 0 && c == 0)) ? P->bell(region) : nullptr;
    wait_flag(f, seq - uint64_t(K), "slot credit", b);
  }
  uint64_t completed() const {
    uint64_t mx = 0;
    for (int k = 0; k < K; ++k) mx = std::max(mx, credit(me, k));
    return mx;
  }
  // Host store of a flag in rank r's region, then its doorbell.
  void host_flag(int r, char* f, uint64_t v) {
    store_rel(f, v);
    bell_ring(P->bell(r));
  }
  // Take the next header of this program (rank 0's doorbell in our ring).
  bool take(PeerHeader& h) {
    HeaderRing* R = P->ring(me);
    const uint64_t pos = P->taken;
    auto& s = R->slots[pos % HeaderRing::kSlots];
    wait_ready([&] { return s.seq.load(std::memory_order_acquire) == pos + 1; },
               [&](clk::duration) {
                 if (!m->open()) throw std::runtime_error("mesh closed");
                 if (s.seq.load(std::memory_order_acquire) != pos + 1 && fd_gone((*fds)[0]))
                   throw std::runtime_error("mesh: rank 0 is gone");
               },
               P->bell(me), im->spin_us);
    h = s.h;
    R->consumed.store(pos + 1, std::memory_order_release);
    P->taken = pos + 1;
    return h.op != kPeerStop;
  }
  int backlog() const {
    const HeaderRing* R = P->ring(me);
    int n = 0;
    while (n < 64 && R->slots[(P->taken + uint64_t(n)) % HeaderRing::kSlots].seq.load(std::memory_order_acquire) ==
                         P->taken + uint64_t(n) + 1)
      ++n;
    return n;
  }
  // First failure of batch `seq` wins the text slot of rank 0's region; the
  // batch still completes everywhere (outputs and flags), rank 0 fails it.
  void report_error(int k, uint64_t seq, const std::string& what) {
    char* f = P->errf(0, k);
    if (load_acq(f) == seq) return;
    im->stage_errors.fetch_add(1, std::memory_order_relaxed);
    std::string t = "rank " + std::to_string(me) + ": " + what;
    t.resize(std::min(t.size(), kErrText - 1));
    std::memcpy(P->err_text(0, k), t.c_str(), t.size() + 1);
    store_rel(f, seq);
  }
};

// CPU gang: every slab is host memory; stages compute with run_cpu.
void run_cpu_loop(WorkerCtx& W) {
  Prog& P = *W.P;
  Exec& E = *P.ex;
  const int K = W.K;
  const auto& st = P.d.stages;
  uint64_t seq = 0;
  PeerHeader h;
  while (W.take(h)) {
    ++seq;
    const int k = int((seq - 1) % uint64_t(K));
    const int rows = h.rows;
    W.im->note_inflight(uint64_t(1 + W.backlog()));
    std::string fail;
    if (rows <= 0 || rows > P.d.max_rows || h.cols != P.d.in_cols)
      fail = "bad header: " + std::to_string(rows) + " rows x " + std::to_string(h.cols) + " cols";
    for (int i : P.local) {
      const MeshStage& s = st[size_t(i)];
      auto in_ptr = [&](int j) -> const double* {
        if (j == -1) return reinterpret_cast<const double*>(P.slab_host(W.me, -1, k));
        if (st[size_t(j)].rank == W.me) return E.hout[size_t(j)].data() + size_t(k) * P.d.max_rows * st[size_t(j)].out_cols;
        W.wait_input(k, j, seq);
        return reinterpret_cast<const double*>(P.slab_host(W.me, j, k));
      };
      std::vector<const double*> ins;
      for (int j : s.inputs) ins.push_back(in_ptr(j));
      // write straight into the one consumer's slab when nothing local reads it
      const auto& cons = P.consumers[size_t(i)];
      const bool direct = cons.size() == 1 && !P.local_consumer[size_t(i)];
      double* out;
      if (direct) {
        W.wait_credit(cons[0], k, seq);
        out = reinterpret_cast<double*>(P.slab_host(cons[0], i, k));
      } else {
        out = E.hout[size_t(i)].data() + size_t(k) * P.d.max_rows * s.out_cols;
      }
      const size_t n = size_t(rows) * size_t(s.out_cols);
      if (fail.empty()) {
        try {
          if (W.im->delay_us) std::this_thread::sleep_for(std::chrono::microseconds(W.im->delay_us));
          if (s.kind == kMeshModel) {
            P.model[size_t(i)]->run_cpu(ins[0], rows, s.in_cols, out);
          } else if (s.kind == kMeshMean) {
            for (size_t e = 0; e < n; ++e) {
              double acc = 0.0;
              for (const double* p : ins) acc += p[e];
              out[e] = acc / double(ins.size());
            }
          } else {
            P.fn[size_t(i)](ins[0], rows, s.in_cols, out, s.out_cols);
          }
        } catch (const std::exception& e) {
          fail = "stage '" + s.node + "': " + e.what();
        }
      }
      if (!fail.empty()) {
        std::fill(out, out + n, 0.0);
        W.report_error(k, seq, fail);
      }
      for (int c : cons) {
        if (!direct) {
          W.wait_credit(c, k, seq);
          std::memcpy(P.slab_host(c, i, k), out, n * sizeof(double));
        }
        W.host_flag(c, P.ready(c, k, i), seq);
      }
    }
    if (P.alias[size_t(W.me)].first < 0) W.host_flag(W.me, P.freed(W.me, k), seq);
    W.im->batches.fetch_add(1, std::memory_order_relaxed);
    W.im->rows.fetch_add(uint64_t(rows > 0 ? rows : 0), std::memory_order_relaxed);
  }
}

// GPU gang: one stream per program; the host waits for every cross-process
// condition before it enqueues (mesh.h), so no enqueued op ever waits on
// another process.
void run_gpu_loop(WorkerCtx& W) {
  Prog& P = *W.P;
  Exec& E = *P.ex;
  const int K = W.K;
  const auto& st = P.d.stages;
  hipStream_t s = E.st.get();
  uint64_t seq = 0;
  PeerHeader h;
  while (W.take(h)) {
    ++seq;
    const int k = int((seq - 1) % uint64_t(K));
    const int rows = h.rows;
    std::string fail;
    if (rows <= 0 || rows > P.d.max_rows || h.cols != P.d.in_cols)
      fail = "bad header: " + std::to_string(rows) + " rows x " + std::to_string(h.cols) + " cols";
    const int rws = fail.empty() ? rows : 0;
    const size_t xbytes = size_t(rws) * size_t(P.d.in_cols) * sizeof(double);
    // the program input: read in place over PCIe (zero-copy) or staged into HBM
    bool x_staged = false;
    const char* x_dev = P.lay[size_t(W.me)].index_of(-1) >= 0 ? P.slab_dev(W.me, -1, k) : nullptr;
    auto stage_x = [&]() -> const double* {
      if (!x_staged && xbytes) {
        SCA_HIP_CHECK(hipMemcpyAsync(E.xdev.as<char>() + size_t(k) * E.x_slab, P.slab_host(W.me, -1, k), xbytes,
                                     hipMemcpyHostToDevice, s));
        x_staged = true;
      }
      return reinterpret_cast<const double*>(E.xdev.as<char>() + size_t(k) * E.x_slab);
    };
    for (int i : P.local) {
      const MeshStage& sg = st[size_t(i)];
      const auto& cons = P.consumers[size_t(i)];
      const size_t obytes = size_t(rws) * size_t(sg.out_cols) * sizeof(double);
      char* own_out = E.out[size_t(i)].as<char>() + size_t(k) * E.out_slab[size_t(i)];
      // remote inputs must be in place before anything that reads them is enqueued
      for (int j : sg.inputs)
        if (j >= 0 && st[size_t(j)].rank != W.me) W.wait_input(k, j, seq);
      const bool zc_in = sg.kind == kMeshModel && !P.model[size_t(i)]->device_io_only() &&
                         P.model[size_t(i)]->zero_copy_input_for(rws, sg.in_cols) && xbytes <= kZeroCopyMax;
      auto dev_in = [&](int j) -> const double* {
        if (j == -1) return zc_in ? reinterpret_cast<const double*>(x_dev) : stage_x();
        if (st[size_t(j)].rank == W.me)
          return reinterpret_cast<const double*>(E.out[size_t(j)].as<char>() + size_t(k) * E.out_slab[size_t(j)]);
        return reinterpret_cast<const double*>(P.slab_dev(W.me, j, k));
      };
      // a model whose only reader is rank 0 writes its rows straight into rank 0's pinned slab
      const bool direct0 = sg.kind == kMeshModel && cons.size() == 1 && cons[0] == 0 && !P.local_consumer[size_t(i)] &&
                           !P.model[size_t(i)]->device_io_only() && obytes <= kZeroCopyMax && fail.empty();
      double* out = reinterpret_cast<double*>(own_out);
      if (direct0) {
        W.wait_credit(0, k, seq);
        out = reinterpret_cast<double*>(P.slab_dev(0, i, k));
      }
      if (fail.empty()) {
        try {
          if (W.im->delay_us) kern::device_delay_us(W.im->delay_us, s);
          if (sg.kind == kMeshModel) {
            if (sg.inputs[0] == -1 && !zc_in) stage_x();
            P.model[size_t(i)]->launch(dev_in(sg.inputs[0]), rws, sg.in_cols, out, E.ws[size_t(i)].get(), s);
          } else if (sg.kind == kMeshMean) {
            for (int j : sg.inputs)
              if (j == -1) stage_x();
            kern::combine_mean_f64(reinterpret_cast<const double* const*>(E.tab[size_t(i)].as<char>() +
                                                                          size_t(k) * sg.inputs.size() * sizeof(void*)),
                                   int(sg.inputs.size()), int64_t(rws) * sg.out_cols, out, s);
          } else {
            // a Python component: bring its input to the host, call it, put the rows back in HBM
            const int j = sg.inputs[0];
            const size_t ib = size_t(rws) * size_t(sg.in_cols) * sizeof(double);
            E.hx.resize(size_t(rws) * size_t(sg.in_cols));
            E.hy.resize(size_t(rws) * size_t(sg.out_cols));
            const double* hin;
            if (j == -1) {
              hin = reinterpret_cast<const double*>(P.slab_host(W.me, -1, k));
            } else {
              const double* di = dev_in(j);
              SCA_HIP_CHECK(hipMemcpyAsync(E.hx.data(), di, ib, hipMemcpyDeviceToHost, s));
              SCA_HIP_CHECK(hipStreamSynchronize(s));
              hin = E.hx.data();
            }
            P.fn[size_t(i)](hin, rws, sg.in_cols, E.hy.data(), sg.out_cols);
            SCA_HIP_CHECK(hipMemcpyAsync(own_out, E.hy.data(), obytes, hipMemcpyHostToDevice, s));
            SCA_HIP_CHECK(hipStreamSynchronize(s));
          }
        } catch (const std::exception& e) {
          fail = "stage '" + sg.node + "': " + e.what();
        }
      }
      if (!fail.empty()) W.report_error(k, seq, fail);
      for (int c : cons) {
        if (!(direct0 && c == 0)) {
          W.wait_credit(c, k, seq);
          if (obytes) {
            const bool to_dev = P.slab_on_dev(c, i);
            void* dst = to_dev ? static_cast<void*>(P.slab_dev(c, i, k)) : static_cast<void*>(P.slab_host(c, i, k));
            SCA_HIP_CHECK(hipMemcpyAsync(dst, own_out, obytes, to_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
          }
        }
        SCA_HIP_CHECK(hipStreamWriteValue64(s, P.flag_dev(c, k, P.lay[size_t(c)].index_of(i)), seq, 0));
      }
    }
    if (P.alias[size_t(W.me)].first < 0)
      SCA_HIP_CHECK(hipStreamWriteValue64(s, P.flag_dev(W.me, k, int(P.lay[size_t(W.me)].src.size())), seq, 0));
    W.im->batches.fetch_add(1, std::memory_order_relaxed);
    W.im->rows.fetch_add(uint64_t(rws), std::memory_order_relaxed);
    W.im->note_inflight(seq - std::min(seq, W.completed()));
  }
  SCA_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

void Mesh::start() {
  if (!im_->connected) throw std::runtime_error("Mesh::start: connect() first");
  if (im_->started || rank_ == 0) {
    im_->started = true;
    return;
  }
  im_->started = true;
  for (auto& Pp : im_->progs) {
    Prog* P = Pp.get();
    if (P->local.empty()) continue;
    auto E = std::make_unique<Exec>();
    const size_t n = P->d.stages.size();
    const auto& st = P->d.stages;
    const size_t mr = size_t(P->d.max_rows);
    if (gpu()) {
      gpu::DeviceGuard g(device_);
      E->st.create(device_);
      E->out.resize(n);
      E->out_slab.assign(n, 0);
      E->ws.resize(n);
      E->tab.resize(n);
      bool need_x = false;
      for (int i : P->local) {
        const MeshStage& s = st[size_t(i)];
        E->out_slab[size_t(i)] = align_up(mr * size_t(s.out_cols) * sizeof(double), 256);
        E->out[size_t(i)].alloc(size_t(K_) * E->out_slab[size_t(i)], device_);
        if (s.kind == kMeshModel) {
          P->model[size_t(i)]->to_device(device_);
          const size_t wb = P->model[size_t(i)]->workspace_bytes(int(mr), s.in_cols);
          if (wb) E->ws[size_t(i)].alloc(wb, device_);
        }
        for (int j : s.inputs) need_x |= j == -1;
      }
      if (need_x) {
        E->x_slab = align_up(mr * size_t(P->d.in_cols) * sizeof(double), 256);
        E->xdev.alloc(size_t(K_) * E->x_slab, device_);
      }
      for (int i : P->local) {
        const MeshStage& s = st[size_t(i)];
        if (s.kind != kMeshMean) continue;
        std::vector<const void*> tab;
        for (int k = 0; k < K_; ++k)
          for (int j : s.inputs) {
            const void* p;
            if (j == -1) p = E->xdev.as<char>() + size_t(k) * E->x_slab;
            else if (st[size_t(j)].rank == rank_) p = E->out[size_t(j)].as<char>() + size_t(k) * E->out_slab[size_t(j)];
            else p = P->slab_dev(rank_, j, k);
            tab.push_back(p);
          }
        E->tab[size_t(i)].alloc(tab.size() * sizeof(void*), device_);
        E->tab[size_t(i)].upload(tab.data(), tab.size() * sizeof(void*));
      }
    } else {
      E->hout.resize(n);
      for (int i : P->local) E->hout[size_t(i)].assign(size_t(K_) * mr * size_t(st[size_t(i)].out_cols), 0.0);
    }
    P->ex = std::move(E);
    P->th = std::thread([this, P] {
      WorkerCtx W{this, im_.get(), P, rank_, K_, &fds_};
      try {
        std::unique_ptr<gpu::DeviceGuard> g;
        if (gpu()) {
          g = std::make_unique<gpu::DeviceGuard>(device_);
          run_gpu_loop(W);
        } else {
          run_cpu_loop(W);
        }
      } catch (const std::exception& e) {
        im_->set_error("program " + std::to_string(P->id) + ": " + e.what());
        open_.store(false);  // the other programs of this rank leave too; the supervisor restarts the gang
      }
    });
  }
}

void Mesh::stop_peers() {
  if (rank_ != 0) return;
  for (auto& Pp : im_->progs) {
    Prog& P = *Pp;
    if (!P.reg[0].host) continue;
    std::lock_guard<std::mutex> g(P.issue_mu);
    for (int c = 1; c < world_; ++c) {
      if (!P.part[size_t(c)] || !P.reg[size_t(c)].host) continue;
      HeaderRing* R = P.ring(c);
      const uint64_t wpos = P.next;  // every worker of the program gets every header: same position
      const auto t0 = clk::now();
      while (wpos - R->consumed.load(std::memory_order_acquire) >= HeaderRing::kSlots) {
        if (fd_gone(fds_[size_t(c)]) || clk::now() - t0 > std::chrono::seconds(5)) break;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      auto& s = R->slots[wpos % HeaderRing::kSlots];
      s.h = PeerHeader{};
      s.h.op = kPeerStop;
      s.seq.store(wpos + 1, std::memory_order_release);
      bell_ring(P.bell(c));
    }
    P.next += 1;  // the stop occupies one ring position everywhere; no batch may follow
  }
  open_.store(false);
}

// ------------------------------------------------------------ the front end
class ProgramModel : public gpu::RowModel {
 public:
  ProgramModel(MeshPtr m, Mesh::Impl* im, Prog* P) : m_(std::move(m)), im_(im), P_(P) {}
  std::string name() const override { return "mesh_program"; }
  int in_cols() const override { return P_->d.in_cols; }
  int out_cols(int) const override { return P_->d.stages.back().out_cols; }
  void to_device(int) override {}
  bool exclusive_driver() const override { return false; }
  bool async_cpu() const override { return true; }
  void launch(const double*, int, int, double*, void*, hipStream_t) override {
    throw std::runtime_error("mesh program: serve it from a CPU-batching unit (device -1)");
  }
  gpu::CpuCallPtr start_cpu(const double* X, int rows, int cols, double* out) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;

  // Copy out every finished batch in seq order (any thread).  True if any.
  bool reap();
  // The caller gave up on a call (error, watchdog, shutdown): its batches
  // still complete and free their slots, but nothing is written to `out`.
  void abandon(const CallStatePtr& cs) {
    std::lock_guard<std::mutex> g(P_->reap_mu);
    cs->abandoned = true;
  }
  void check_alive(const char* what, clk::time_point since);

 private:
  MeshPtr m_;
  Mesh::Impl* im_;
  Prog* P_;
  std::weak_ptr<ProgramModel> self_;
  friend class Mesh;

 public:
  std::atomic<uint32_t> polls{0};  // liveness checks every 1024th poll
  // Rank 0's doorbell when CPU workers write its flags (GPU gangs: none, the
  // flags are written by streams).
  Bell* reply_bell() const { return m_->gpu() ? nullptr : P_->bell(0); }
};

namespace {
struct MeshCall : gpu::CpuCall {
  std::shared_ptr<ProgramModel> pm;
  CallStatePtr cs;
  clk::time_point t0;
  bool finished = false;
  std::string err;
  ~MeshCall() override {
    if (pm && cs && cs->remaining.load(std::memory_order_acquire) > 0) pm->abandon(cs);
  }
  bool done() override {
    if (finished) return true;
    if (cs->remaining.load(std::memory_order_acquire) > 0) {
      pm->reap();
      if (cs->remaining.load(std::memory_order_acquire) > 0) {
        if ((pm->polls.fetch_add(1, std::memory_order_relaxed) & 1023) == 0) {
          try {
            pm->check_alive("reply", t0);
          } catch (const std::exception& e) {
            pm->abandon(cs);  // late replies must not land in the batcher's reused buffer
            err = e.what();
            finished = true;
            return true;
          }
        }
        return false;
      }
    }
    std::lock_guard<std::mutex> g(cs->mu);
    err = cs->error;
    finished = true;
    return true;
  }
  std::string error() const override { return err; }
  // The batcher's low-CPU mode: block up to `us` for this call's replies
  // (CPU gangs: on rank 0's futex doorbell, woken by the worker's store;
  // GPU gangs: yielding polls, since streams write the flags).
  bool wait_us(int us) override {
    if (done()) return true;
    const auto lim = std::chrono::microseconds(std::max(1, us));
    if (Bell* b = pm->reply_bell()) {
      const uint32_t s = b->seq.load(std::memory_order_seq_cst);
      b->sleepers.fetch_add(1, std::memory_order_seq_cst);
      if (!done()) {
        const timespec ts{0, long(lim.count()) * 1000L};
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&b->seq), FUTEX_WAIT, s, &ts, nullptr, 0);
      }
      b->sleepers.fetch_sub(1, std::memory_order_seq_cst);
      return true;
    }
    const auto t0 = clk::now();
    while (!done() && clk::now() - t0 < lim) std::this_thread::yield();
    return true;
  }
};
}  // namespace

void ProgramModel::check_alive(const char* what, clk::time_point since) {
  if (!m_->open()) throw std::runtime_error("mesh closed");
  for (int c = 1; c < m_->world(); ++c)
    if (P_->part[size_t(c)] && fd_gone(m_->fds_[size_t(c)]))
      throw std::runtime_error("mesh: rank " + std::to_string(c) + " is gone");
  if (clk::now() - since > std::chrono::milliseconds(im_->timeout_ms))
    throw std::runtime_error(std::string("mesh: no ") + what + " within " + std::to_string(im_->timeout_ms) + " ms");
}

bool ProgramModel::reap() {
  Prog& P = *P_;
  std::unique_lock<std::mutex> g(P.reap_mu, std::try_to_lock);
  if (!g.owns_lock()) return false;
  const int K = m_->slots();
  const Layout& L = P.lay[0];
  bool any = false;
  while (true) {
    const uint64_t seq = P.reaped + 1;
    const int k = int((seq - 1) % uint64_t(K));
    Prog::Pend& pd = P.pend[size_t(k)];
    if (pd.seq != seq) break;  // not issued yet
    bool ready = true;
    for (size_t e = 0; e < L.src.size() && ready; ++e) ready = load_acq(P.flag(0, k, int(e))) >= seq;
    if (!ready) break;
    CallState& cs = *pd.call;
    const int oc = cs.out_cols;
    const size_t n = size_t(pd.rows) * size_t(oc);
    double* out = cs.out + size_t(pd.row0) * size_t(oc);
    if (cs.abandoned) {
      // the caller is gone: free the slot, write nothing
    } else if (load_acq(P.errf(0, k)) == seq) {
      std::lock_guard<std::mutex> lk(cs.mu);
      if (cs.error.empty()) cs.error = std::string(P.err_text(0, k));
    } else if (L.src.size() == 1) {
      std::memcpy(out, P.slab_host(0, L.src[0], k), n * sizeof(double));
    } else {  // the final mean on rank 0 (a COMBINER over remote branches)
      std::fill(out, out + n, 0.0);
      for (int s : L.src) {
        const double* p = reinterpret_cast<const double*>(P.slab_host(0, s, k));
        for (size_t i = 0; i < n; ++i) out[i] += p[i];
      }
      const double inv = 1.0 / double(L.src.size());
      for (size_t i = 0; i < n; ++i) out[i] *= inv;
    }
    store_rel(P.freed(0, k), seq);
    bell_ring(P.bell(0));  // a producer may wait for this slot
    auto call = std::move(pd.call);
    pd = Prog::Pend{};
    P.reaped = seq;
    call->remaining.fetch_sub(1, std::memory_order_acq_rel);
    any = true;
  }
  return any;
}

gpu::CpuCallPtr ProgramModel::start_cpu(const double* X, int rows, int cols, double* out) {
  if (!m_->open()) throw std::runtime_error("mesh closed");
  Prog& P = *P_;
  if (cols != P.d.in_cols)
    throw std::runtime_error("mesh program expects " + std::to_string(P.d.in_cols) + " columns, got " +
                             std::to_string(cols));
  const int K = m_->slots();
  auto cs = std::make_shared<CallState>();
  cs->out = out;
  cs->out_cols = out_cols(cols);
  const int mr = P.d.max_rows;
  const int chunks = std::max(1, (rows + mr - 1) / mr);
  cs->remaining.store(rows > 0 ? chunks : 0);
  const auto t0 = clk::now();
  try {
    std::lock_guard<std::mutex> g(P.issue_mu);
    for (int ch = 0; ch < chunks && rows > 0; ++ch) {
      const int row0 = ch * mr, nr = std::min(mr, rows - row0);
      const uint64_t seq = P.next + 1;
      const int k = int((seq - 1) % uint64_t(K));
      // slot k must be free everywhere this batch writes: rank 0's own slab
      // (reaped) and every X consumer's input slab (credited)
      auto credit_ok = [&] {
        if (P.pend[size_t(k)].seq != 0) return false;
        if (seq <= uint64_t(K)) return true;
        const uint64_t need = seq - uint64_t(K);
        for (int c = 1; c < m_->world(); ++c) {
          if (!P.part[size_t(c)] || P.lay[size_t(c)].index_of(-1) < 0) continue;
          const auto a = P.alias[size_t(c)];
          const uint64_t v = a.first >= 0 ? load_acq(P.ready(a.first, k, a.second)) : load_acq(P.freed(c, k));
          if (v < need) return false;
        }
        return true;
      };
      wait_until(
          [&] {
            reap();
            std::lock_guard<std::mutex> rl(P.reap_mu);  // guards pend
            return credit_ok();
          },
          [&](clk::duration) { check_alive("slot credit", t0); });
      for (int c = 1; c < m_->world(); ++c)
        if (P.part[size_t(c)] && P.lay[size_t(c)].index_of(-1) >= 0)
          std::memcpy(P.slab_host(c, -1, k), X + size_t(row0) * size_t(cols), size_t(nr) * size_t(cols) * sizeof(double));
      {
        std::lock_guard<std::mutex> rl(P.reap_mu);
        P.pend[size_t(k)] = Prog::Pend{seq, cs, row0, nr};
      }
      for (int c = 1; c < m_->world(); ++c) {
        if (!P.part[size_t(c)]) continue;
        HeaderRing* R = P.ring(c);
        const uint64_t pos = seq - 1;
        wait_until([&] { return pos - R->consumed.load(std::memory_order_acquire) < HeaderRing::kSlots; },
                   [&](clk::duration) { check_alive("ring credit", t0); });
        auto& s = R->slots[pos % HeaderRing::kSlots];
        s.h.op = kPeerRun;
        s.h.model = P.id;
        s.h.rows = nr;
        s.h.cols = cols;
        s.seq.store(pos + 1, std::memory_order_release);  // the doorbell
        bell_ring(P.bell(c));
      }
      P.next = seq;
    }
  } catch (...) {
    // a peer is gone or stuck past the timeout: the program's ranks can no
    // longer be kept in step, so the mesh closes (the supervisor restarts the
    // gang); chunks already issued never touch `out`
    abandon(cs);
    m_->close();
    throw;
  }
  auto c = std::make_shared<MeshCall>();
  c->pm = self_.lock();
  if (!c->pm) throw std::runtime_error("mesh program model is not owned by a shared_ptr");
  c->cs = std::move(cs);
  c->t0 = t0;
  return c;
}

void ProgramModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  auto* self = const_cast<ProgramModel*>(this);
  auto c = self->start_cpu(X, rows, cols, out);
  while (!c->done()) c->wait_us(100);
  if (!c->error().empty()) throw std::runtime_error(c->error());
}

gpu::RowModelPtr Mesh::program_model(int prog, std::vector<std::string> class_names, bool flat) {
  if (rank_ != 0) throw std::runtime_error("Mesh::program_model: rank 0 only");
  if (!im_->connected) throw std::runtime_error("Mesh::program_model: connect() first");
  Prog* P = im_->progs.at(size_t(prog)).get();
  auto m = std::make_shared<ProgramModel>(shared_from_this(), im_.get(), P);
  m->self_ = m;
  m->set_class_names(std::move(class_names));
  m->set_flat_output(flat);
  return m;
}

}  // namespace sca::par
