#include "batcher.h"

#include "../core/roctx.h"
#include "driver.h"

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstring>

namespace sca::gpu {

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

bool available() { return device_count() > 0; }

bool large_bar(int device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeIsLargeBar, device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return v != 0;
}

namespace {
// SCA_BATCH_INPUT=bar|host: where a zero-copy batch's rows are staged.
// "bar" writes them into fine-grained HBM through the PCIe BAR (large-BAR
// devices only), so the kernel's row read stays on the device (2.3 vs 4.1 us,
// profiles/r05n_launch_floor); "host" leaves them in pinned host memory, read
// over PCIe.  Unset: each model's preference (tree ensembles: bar -- xgb1000
// 7.04 -> 5.96 us per small batch; the rest host: the pump's write-combined
// stores cost the iris headline ~2%, profiles/r05sl_tree_split).
bool bar_input_wanted(int device, bool model_prefers) {
  const char* e = std::getenv("SCA_BATCH_INPUT");
  const bool want = e ? std::string(e) == "bar" : model_prefers;
  return want && large_bar(device);
}

// Write-combined stores into BAR-mapped memory (the caller drains them with
// sfence before the launch: the kernel must see every byte).
inline void bar_store(double* dst, const double* src, size_t n) {
  std::memcpy(dst, src, n * sizeof(double));
}
}  // namespace

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t pos = 0;
  while (true) {
    const size_t end = s.find(sep, pos);
    out.push_back(s.substr(pos, end == std::string::npos ? std::string::npos : end - pos));
    if (end == std::string::npos) return out;
    pos = end + 1;
  }
}

}  // namespace

FaultSpec fault_from_env(int device) {
  FaultSpec f;
  const char* env = std::getenv("SCA_FAULT");
  if (!env || !*env) return f;
  for (const auto& entry : split(env, ';')) {
    const size_t c1 = entry.find(':');
    const size_t c2 = c1 == std::string::npos ? c1 : entry.find(':', c1 + 1);
    if (c2 == std::string::npos) continue;
    const std::string kind = entry.substr(0, c1), dev = entry.substr(c1 + 1, c2 - c1 - 1);
    if ((kind == "gpu") != (device >= 0) || (kind != "gpu" && kind != "cpu")) continue;
    if (dev != "*" && (kind == "cpu" || std::atoi(dev.c_str()) != device)) continue;
    for (const auto& kv : split(entry.substr(c2 + 1), ',')) {
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) continue;
      const std::string k = kv.substr(0, eq);
      const long long v = std::atoll(kv.c_str() + eq + 1);
      if (k == "fail_after") f.fail_after = v;
      else if (k == "fail_count") f.fail_count = v;
      else if (k == "hang_ms") f.hang_ms = int(v);
    }
  }
  return f;
}

BatchedUnit::BatchedUnit(RowModelPtr model, BatcherOptions opts) : model_(std::move(model)), opts_(opts) {
  if (opts_.max_batch < 1) opts_.max_batch = 1;
  if (opts_.slots < 1) opts_.slots = 1;
  if (opts_.fail_threshold < 1) opts_.fail_threshold = 1;
  inject_fault(fault_from_env(opts_.device));
  device_io_ = model_->device_io_only();
  zc_input_ = model_->zero_copy_input();
  bar_input_ = opts_.device >= 0 && opts_.device < device_count() &&
               bar_input_wanted(opts_.device, model_->prefers_bar_input());
  segmented_ = model_->segmented();
  if (bar_input_) {
    const char* f = std::getenv("SCA_HDP_FLUSH");
    if (!f || std::atoi(f) != 0) {
      hipDeviceProp_t prop{};
      if (hipGetDeviceProperties(&prop, opts_.device) == hipSuccess && prop.hdpMemFlushCntl)
        hdp_flush_ = prop.hdpMemFlushCntl;
    }
  }
  {
    auto info = std::make_shared<RespInfo>();
    info->model = model_;
    const int oc = model_->out_cols(model_->in_cols() > 0 ? model_->in_cols() : 1);
    info->names = model_->class_names();
    if (info->names.empty())
      for (int c = 0; c < oc; ++c) info->names.push_back("t:" + std::to_string(c));
    resp_ = std::move(info);
  }
  if (opts_.device < 0) {
    running_.store(true);
    if (opts_.cpu_batching) {
      cpu_ = true;
      for (int i = 0; i < opts_.slots; ++i) slots_.push_back(std::make_unique<Slot>());
      for (auto& s : slots_) ps_.free_list.push_back(s.get());
      // launch() may compute inline: a pump of its own -- unless the model only
      // issues work to other ranks (mesh programs), whose units share one pump
      driver_ = model_->async_cpu() ? DeviceDriver::acquire(kAsyncCpuDriver, true) : DeviceDriver::acquire(-1, false);
      driver_->add(this);
    }
    return;
  }
  if (opts_.device >= device_count())
    throw std::runtime_error("BatchedUnit: GPU " + std::to_string(opts_.device) + " not available (" +
                             std::to_string(device_count()) + " visible)");
  DeviceGuard g(opts_.device);
  model_->to_device(opts_.device);
  const int cols = model_->in_cols() > 0 ? model_->in_cols() : 16;
  for (int i = 0; i < opts_.slots; ++i) {
    auto s = std::make_unique<Slot>();
    s->stream.create(opts_.device);
    s->ev.create(opts_.device);
    ensure_capacity(*s, opts_.max_batch, cols);
    slots_.push_back(std::move(s));
  }
  for (auto& s : slots_) ps_.free_list.push_back(s.get());
  running_.store(true);
  // one pump + hand-off thread pair per GPU, unless launch() may block on the host
  driver_ = DeviceDriver::acquire(opts_.device, !model_->exclusive_driver());
  driver_->add(this);
}

BatchedUnit::~BatchedUnit() { stop(); }

void BatchedUnit::stop() {
  if (!running_.exchange(false)) return;
  if (driver_) {
    driver_->remove(this);  // completes everything taken or in flight, posts every response
    driver_.reset();
  }
  std::deque<Item> rest;
  drain_shards(rest);
  for (auto& it : rest) it.k(Outcome::fail(make_error(ApiError::UNAVAILABLE, "GPU unit stopped")));
}

namespace {
std::atomic<int> g_next_shard{0};
int shard_of_this_thread(int shards) {
  thread_local const int idx = g_next_shard.fetch_add(1, std::memory_order_relaxed);
  return idx % shards;
}
}  // namespace

void BatchedUnit::drain_shards(std::deque<Item>& into) {
  for (auto& sh : shards_) {
    if (sh.n.load(std::memory_order_acquire) == 0) continue;
    std::deque<Item> got;
    {
      std::lock_guard<std::mutex> g(sh.mu);
      got.swap(sh.q);
      sh.n.fetch_sub(int(got.size()), std::memory_order_relaxed);
      queued_n_.fetch_sub(int(got.size()), std::memory_order_relaxed);
    }
    for (auto& it : got) {
      queued_rows_.fetch_sub(it.rows, std::memory_order_relaxed);
      into.push_back(std::move(it));
    }
  }
}

constexpr size_t kDirectH2DBytes = size_t(1) << 20;

thread_local const RowModel* g_raw_output_model = nullptr;

void BatchedUnit::ensure_capacity(Slot& s, int rows, int cols) {
  const int oc = std::max(model_->out_cols(cols), model_->raw_out_cols(rows, cols));
  const size_t need_in = size_t(rows) * cols * sizeof(double);
  const size_t need_out = size_t(rows) * oc * sizeof(double);
  // Geometric growth: pinned/device allocations are slow, batches vary.
  auto grow = [](size_t have, size_t need) { return std::max(need, 2 * have); };
  if (s.h_in.bytes() < need_in) {
    const size_t b = grow(s.h_in.bytes(), need_in);
    s.h_in.alloc(b);
    s.d_in.alloc(b, opts_.device);
  }
  if (s.h_out.bytes() < need_out) {
    const size_t b = grow(s.h_out.bytes(), need_out);
    s.h_out.alloc(b);
    s.d_out.alloc(b, opts_.device);
  }
  if (bar_input_ && need_in <= opts_.zero_copy_max_bytes && s.v_in.bytes() < need_in)
    s.v_in.alloc(std::min(grow(s.v_in.bytes(), need_in), std::max(need_in, opts_.zero_copy_max_bytes)), opts_.device);
  const size_t ws = model_->workspace_bytes(rows, cols);
  if (s.ws.bytes() < ws) s.ws.alloc(grow(s.ws.bytes(), ws), opts_.device);
  s.cap_rows = std::max(s.cap_rows, size_t(rows));
}

MsgPtr BatchedUnit::make_response(const RespInfo& info, const Item& it, const double* out, int out_cols) {
  auto m = std::make_shared<SeldonMessage>();
  m->payload = Payload::Data;
  const bool flat = info.model->flat_output() && out_cols == 1;
  if (!flat) {
    if (int(info.names.size()) == out_cols) {
      m->data.names = info.names;
    } else {
      m->data.names = info.model->class_names();
      if (m->data.names.empty())
        for (int c = 0; c < out_cols; ++c) m->data.names.push_back("t:" + std::to_string(c));
    }
  }
  DataKind kind = it.req->payload == Payload::Data ? it.req->data.kind : DataKind::Tensor;
  std::vector<double> vals(out, out + size_t(it.rows) * out_cols);
  std::vector<int64_t> shape = flat ? std::vector<int64_t>{int64_t(it.rows)} : std::vector<int64_t>{int64_t(it.rows), int64_t(out_cols)};
  m->data.set_dense(kind, std::move(shape), std::move(vals));
  m->has_meta = true;
  m->meta.puid = it.req->meta.puid;
  return m;
}

void BatchedUnit::transform_input(const CallCtx& c, MsgPtr in, Done k) {
  if (in->payload != Payload::Data) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, model_->name() + " expects numeric 'data' payload")));
    return;
  }
  Item it;
  std::vector<int64_t> shape;
  std::string err;
  size_t nvals = 0;
  const DefaultData& dd = in->data;
  bool flat = (dd.kind == DataKind::Tensor || (dd.kind == DataKind::NdArray && dd.nd_dense)) && !dd.shape.empty();
  if (flat) {  // rows read in place from the message (it stays alive in it.req)
    int64_t n = 1;
    for (auto d : dd.shape) {
      if (d < 0) flat = false;
      n *= d;
    }
    flat = flat && n == int64_t(dd.values.size());
  }
  if (flat) {
    shape = dd.shape;
    it.xp = dd.values.data();
    nvals = dd.values.size();
  } else {
    if (!dd.dense(shape, it.x, &err)) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, err)));
      return;
    }
    it.xp = it.x.data();
    nvals = it.x.size();
  }
  if (shape.empty()) {
    it.rows = nvals == 0 ? 0 : 1;
    it.cols = int(nvals);
  } else if (shape.size() == 1) {
    it.rows = 1;
    it.cols = int(shape[0]);
  } else {
    it.rows = int(shape[0]);
    int64_t cc = 1;
    for (size_t i = 1; i < shape.size(); ++i) cc *= shape[i];
    it.cols = int(cc);
  }
  const auto& cols_want = model_->input_names();
  if (!cols_want.empty() && !dd.names.empty() && int(dd.names.size()) == it.cols && dd.names != cols_want) {
    // the request names its columns in another order than the model's
    // signature: gather them into signature order (MLflow schema enforcement)
    std::vector<int> src(cols_want.size());
    std::string missing;
    for (size_t c = 0; c < cols_want.size(); ++c) {
      const auto f = std::find(dd.names.begin(), dd.names.end(), cols_want[c]);
      if (f == dd.names.end()) missing += (missing.empty() ? "'" : ", '") + cols_want[c] + "'";
      src[c] = int(f - dd.names.begin());
    }
    if (!missing.empty()) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "request is missing signature column(s) [" + missing + "]")));
      return;
    }
    std::vector<double> perm(size_t(it.rows) * cols_want.size());
    for (int r = 0; r < it.rows; ++r)
      for (size_t c = 0; c < cols_want.size(); ++c)
        perm[size_t(r) * cols_want.size() + c] = it.xp[size_t(r) * it.cols + size_t(src[c])];
    it.x = std::move(perm);
    it.xp = it.x.data();
    it.cols = int(cols_want.size());
  }
  const int want = model_->in_cols();
  if (it.rows <= 0 || it.cols <= 0) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, model_->name() + " expects a non-empty 2-D numeric payload")));
    return;
  }
  if (want > 0 && it.cols != want) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR,
                               "X has " + std::to_string(it.cols) + " features, but " + model_->name() +
                                   " is expecting " + std::to_string(want) + " features as input.")));
    return;
  }
  it.req = std::move(in);
  it.k = std::move(k);
  if (c.exec) it.exec = *c.exec;
  submit_item(std::move(it));
}

void BatchedUnit::submit_item(Item it) {
  if (opts_.device < 0 && !cpu_) {
    if (fault_armed_.load(std::memory_order_relaxed) && take_injected_failure()) {
      note_failure();
      it.k(Outcome::fail(device_error(ApiError::EXECUTION_FAILURE, "injected device fault (SCA_FAULT)")));
      return;
    }
    note_success();
    const int oc = model_->out_cols(it.cols);
    std::vector<double> out(size_t(it.rows) * oc);
    model_->run_cpu(it.xp, it.rows, it.cols, out.data());
    MsgPtr r = make_response(*resp_, it, out.data(), oc);
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.batches++;
      stats_.rows += uint64_t(it.rows);
      stats_.requests++;
    }
    it.k(Outcome::ok(std::move(r)));
    return;
  }
  if (!running_.load()) {
    it.k(Outcome::fail(make_error(ApiError::UNAVAILABLE, "GPU unit stopped")));
    return;
  }
  if (abandoned_slots_.load(std::memory_order_relaxed) >= int(slots_.size())) {
    it.k(Outcome::fail(device_error(ApiError::UNAVAILABLE, "every batch slot of this GPU is wedged")));
    return;
  }
  const int rows = it.rows;
  inflight_rows_.fetch_add(rows, std::memory_order_relaxed);
  queued_rows_.fetch_add(rows, std::memory_order_relaxed);
  Shard& sh = shards_[shard_of_this_thread(kShards)];
  {
    std::lock_guard<std::mutex> g(sh.mu);
    sh.q.push_back(std::move(it));
    sh.n.fetch_add(1, std::memory_order_release);
    queued_n_.fetch_add(1, std::memory_order_seq_cst);
  }
  // Pairs with the driver's sleeping_ store + queued re-check under its
  // mutex: either it sees this item or we see it asleep and wake it.
  if (driver_) driver_->notify();
}

bool BatchedUnit::launch(Slot* s) {
  const int rows = s->rows, cols = s->cols;
  s->out_cols = model_->out_cols(cols);
  if (fault_armed_.load(std::memory_order_relaxed) && take_injected_failure()) {
    auto e = device_error(ApiError::EXECUTION_FAILURE, "injected device fault (SCA_FAULT)");
    note_failure();
    inflight_rows_.fetch_sub(rows, std::memory_order_relaxed);
    for (auto& it : s->items) it.k(Outcome::fail(e));
    s->items.clear();
    return false;
  }
  if (cpu_) {  // reference path, one call per request (segment semantics for per-request models)
    s->t_launch = std::chrono::steady_clock::now();
    try {
      s->cpu_out.assign(size_t(rows) * s->out_cols, 0.0);
      if (!segmented_) {
        // Models that compute elsewhere (a peer rank) take the whole batch as
        // one asynchronous call: up to `slots` batches stay outstanding and the
        // reap loop below polls them like GPU events.
        const double* x = s->items.front().xp;
        if (s->items.size() > 1) {
          s->cpu_in.resize(size_t(rows) * cols);
          size_t off = 0;
          for (const auto& it : s->items) {
            std::memcpy(s->cpu_in.data() + off, it.xp, size_t(it.rows) * cols * sizeof(double));
            off += size_t(it.rows) * cols;
          }
          x = s->cpu_in.data();
        }
        s->call = model_->start_cpu(x, rows, cols, s->cpu_out.data());
        if (s->call) return true;
      }
      size_t row = 0;
      for (const auto& it : s->items) {
        model_->run_cpu(it.xp, it.rows, cols, s->cpu_out.data() + row * s->out_cols);
        if (it.seq_out) *it.seq_out = model_->last_sequence_base();
        row += size_t(it.rows);
      }
      return true;
    } catch (const std::exception& ex) {
      auto e = make_error(ApiError::EXECUTION_FAILURE, std::string("CPU model failed: ") + ex.what());
      inflight_rows_.fetch_sub(rows, std::memory_order_relaxed);
      for (auto& it : s->items) it.k(Outcome::fail(e));
      s->items.clear();
      return false;
    }
  }
  hipError_t err = hipSuccess;
  std::string launch_error;
  try {
    ensure_capacity(*s, rows, cols);
    s->raw_cols = model_->raw_out_cols(rows, cols);
    struct RawScope {  // this model (not a graph's stage models) may write raw output
      const RowModel* prev;
      explicit RawScope(const RowModel* m) : prev(g_raw_output_model) { g_raw_output_model = m; }
      ~RawScope() { g_raw_output_model = prev; }
    } raw_scope(model_.get());
    const int dev_cols = s->raw_cols > 0 ? s->raw_cols : s->out_cols;  // what the kernel writes per row
    double* hin = s->h_in.host<double>();
    const size_t bin = size_t(rows) * cols * sizeof(double), bout = size_t(rows) * dev_cols * sizeof(double);
    // A lone large request is DMA'd straight from its message's memory: no
    // host copy into the pinned slot first (8192 x 784 fp64: 51 MB).  Not a
    // run_ptr caller's buffer: the watchdog must be able to answer that
    // caller (who then frees the buffer) while the device may still read.
    const bool direct = s->items.size() == 1 && bin >= kDirectH2DBytes && !s->items[0].caller_mem;
    s->direct = direct;
    const bool zc = !direct && opts_.zero_copy && !device_io_ && bin + bout <= opts_.zero_copy_max_bytes;
    // zero-copy batches on a large-BAR device: rows straight into HBM -- for
    // kernels that read each row once (fine-grained HBM is not L2-cached, so
    // models that re-read X from many workgroups keep their DMA into d_in)
    const bool bar = zc && bar_input_ && s->v_in.bytes() >= bin &&
                     (zc_input_ || model_->zero_copy_input_for(rows, cols) || model_->bar_input_for(rows, cols));
    if (!direct) {
      double* dst = bar ? s->v_in.as<double>() : hin;
      size_t off = 0;
      for (const auto& it : s->items) {
        const size_t n = size_t(it.rows) * it.cols;
        if (bar) bar_store(dst + off, it.xp, n);
        else memcpy(dst + off, it.xp, n * sizeof(double));
        off += n;
      }
      if (bar) {
        _mm_sfence();  // the write-combined stores are out of the CPU ...
        if (hdp_flush_) {  // ... and out of the HDP write buffer before the launch (as the HIP runtime does)
          *hdp_flush_ = 1u;
          (void)*hdp_flush_;
        }
      }
    }
    hipStream_t st = s->stream.get();
    const int32_t* seg = nullptr;
    const int nseg = int(s->items.size());
    if (segmented_) {  // request boundaries for per-request models
      if (s->h_seg.bytes() < (s->items.size() + 1) * sizeof(int32_t))
        s->h_seg.alloc(std::max<size_t>(1024, 2 * (s->items.size() + 1)) * sizeof(int32_t));
      int32_t* o = s->h_seg.host<int32_t>();
      o[0] = 0;
      for (size_t i = 0; i < s->items.size(); ++i) o[i + 1] = o[i] + s->items[i].rows;
      seg = s->h_seg.dev<int32_t>();
    }
    bool signalled = false;  // the model's last kernel completes s->ev itself
    auto run = [&](const double* x, double* y) {
      if (seg) {
        model_->launch_segments(x, rows, cols, y, s->ws.get(), seg, nseg, st);
        const int64_t base = model_->last_sequence_base();
        int64_t off = 0;
        for (auto& it : s->items) {
          if (it.seq_out) *it.seq_out = base < 0 ? -1 : base + off;
          off += it.rows;
        }
      } else {
        model_->launch(x, rows, cols, y, s->ws.get(), st);
      }
    };
    if (zc) {
      // Output always zero-copy (written once); input zero-copy only if the
      // kernel reads each element once -- models that re-read X from many
      // workgroups (tree chunks) get one DMA into HBM first.  Rows already
      // written into HBM through the BAR need neither.
      const double* xin = bar ? s->v_in.as<double>() : s->h_in.dev<double>();
      if (!bar && !zc_input_ && !model_->zero_copy_input_for(rows, cols)) {
        err = hipMemcpyAsync(s->d_in.get(), hin, bin, hipMemcpyHostToDevice, st);
        xin = s->d_in.as<double>();
      }
      if (err == hipSuccess) {
        // zero-copy output: nothing follows the kernel on the stream, so a
        // model that can lets its kernel's own dispatch complete the event
        signalled = !seg && model_->launch_signal(xin, rows, cols, s->h_out.dev<double>(), s->ws.get(), st,
                                                  s->ev.get());
        if (!signalled) run(xin, s->h_out.dev<double>());
      }
    } else {
      err = hipMemcpyAsync(s->d_in.get(), direct ? static_cast<const void*>(s->items[0].xp) : hin, bin,
                           hipMemcpyHostToDevice, st);
      if (err == hipSuccess) {
        run(s->d_in.as<double>(), s->d_out.as<double>());
        err = hipMemcpyAsync(s->h_out.host<double>(), s->d_out.get(), bout, hipMemcpyDeviceToHost, st);
      }
    }
    if (err == hipSuccess) err = hipGetLastError();
    if (err == hipSuccess && !signalled) err = hipEventRecord(s->ev.get(), st);
  } catch (const std::exception& ex) {
    err = hipErrorUnknown;
    launch_error = ex.what();
  }
  s->t_launch = std::chrono::steady_clock::now();
  if (err == hipSuccess) {
    if (trace::roctx_on())
      s->roctx = trace::range_start((model_->name() + " batch rows=" + std::to_string(rows)).c_str());
    return true;
  }
  auto e = device_error(ApiError::EXECUTION_FAILURE,
                        "GPU launch failed: " + (launch_error.empty() ? std::string(hipGetErrorString(err)) : launch_error));
  note_failure();
  inflight_rows_.fetch_sub(rows, std::memory_order_relaxed);
  for (auto& it : s->items) it.k(Outcome::fail(e));
  s->items.clear();
  return false;
}

BatchedUnit::ParcelPool::~ParcelPool() {
  for (Parcel* p = head.load(); p;) {
    Parcel* n = p->next;
    delete p;
    p = n;
  }
}

void BatchedUnit::ParcelPool::put(Parcel* p) {
  Parcel* h = head.load(std::memory_order_relaxed);
  do {
    p->next = h;
  } while (!head.compare_exchange_weak(h, p, std::memory_order_release, std::memory_order_relaxed));
}

void BatchedUnit::Parcel::run() {
  size_t off = 0;
  for (auto& it : items) {
    Done k = std::move(it.k);
    k(Outcome::ok(make_response(*info, it, y.data() + off, oc)));
    off += size_t(it.rows) * size_t(oc);
  }
  items.clear();  // destroys the Items on the thread that created them
  y.clear();
  std::shared_ptr<ParcelPool> keep = std::move(pool);  // the pool may go with the last reference
  keep->put(this);
}

// One parcel per front-end executor: its task builds the responses and runs
// the continuations on that thread.
void BatchedUnit::post_responses(Handoff& h, std::vector<Parcel*>& spare) {
  Parcel* groups[32];
  int ng = 0;
  auto fresh = [&]() -> Parcel* {
    if (spare.empty())
      for (Parcel* p = parcels_->take_all(); p; p = p->next) spare.push_back(p);
    Parcel* p;
    if (spare.empty()) {
      p = new Parcel();
    } else {
      p = spare.back();
      spare.pop_back();
    }
    p->pool = parcels_;
    p->info = resp_;
    p->oc = h.out_cols;
    return p;
  };
  auto flush = [&](Parcel* p) {
    ExecPtr ex = p->items.front().exec;
    ex->post([p] { p->run(); });
  };
  const int oc = h.out_cols;
  for (size_t i = 0; i < h.items.size(); ++i) {
    Item& it = h.items[i];
    Parcel* g = nullptr;
    for (int j = 0; j < ng; ++j)
      if (groups[j]->items.front().exec.get() == it.exec.get()) { g = groups[j]; break; }
    if (!g) {
      if (ng == 32) {  // more executors than the table holds: ship what we have
        for (int j = 0; j < ng; ++j) flush(groups[j]);
        ng = 0;
      }
      g = groups[ng++] = fresh();
    }
    const double* src = h.out.data() + h.offs[i];
    g->y.insert(g->y.end(), src, src + size_t(it.rows) * oc);
    g->items.push_back(std::move(it));
  }
  for (int j = 0; j < ng; ++j) flush(groups[j]);
  h.items.clear();
  h.offs.clear();
  h.out.clear();
}

void BatchedUnit::complete(Slot* s, hipError_t st) {
  const double busy = std::chrono::duration<double>(std::chrono::steady_clock::now() - s->t_launch).count();
  if (s->roctx) {
    trace::range_stop(s->roctx);
    s->roctx = 0;
  }
  batch_hist_.observe(busy);
  rows_hist_.observe(double(s->rows) * 1e-6);
  std::string call_err;
  if (s->call) {
    call_err = s->call->error();
    s->call.reset();
    if (!call_err.empty() && st == hipSuccess) st = hipErrorUnknown;
  }
  if (s->abandoned) {  // the watchdog already answered these requests
    s->abandoned = false;
    abandoned_slots_.fetch_sub(1, std::memory_order_relaxed);
    if (st != hipSuccess) note_failure();
    // the device is done with the direct-path source: release it now
    s->parked.clear();
    return;
  }
  inflight_rows_.fetch_sub(s->rows, std::memory_order_relaxed);
  std::vector<Item>& items = s->items;  // cleared below; the slot keeps the capacity
  const size_t n_items = items.size();
  if (st != hipSuccess) {
    auto e = call_err.empty()
                 ? device_error(ApiError::EXECUTION_FAILURE, std::string("GPU execution failed: ") + hipGetErrorString(st))
                 : make_error(ApiError::EXECUTION_FAILURE, "CPU model failed: " + call_err);
    note_failure();
    for (auto& it : items) it.k(Outcome::fail(e));
  } else {
    note_success();
    // Requests with a front-end executor go to the hand-off thread with one
    // copy of the output block; synchronous callers (no executor) are
    // answered here, before the slot is reused.
    const int oc = s->out_cols;
    const double* out = cpu_ ? s->cpu_out.data() : s->h_out.host<double>();
    if (!cpu_ && s->raw_cols > 0) {  // fold the kernel's raw values (RowModel::finish_host)
      s->fin.resize(size_t(s->rows) * size_t(oc));
      model_->finish_host(out, s->rows, s->raw_cols, s->fin.data());
      out = s->fin.data();
    }
    Handoff h = driver_->take_free_handoff();  // reuse a drained hand-off's buffers
    h.unit = this;
    h.out_cols = oc;
    size_t row = 0;
    for (auto& it : items) {
      const size_t r = size_t(it.rows);
      if (!it.exec) {
        Done k = std::move(it.k);
        k(Outcome::ok(make_response(*resp_, it, out + row * oc, oc)));
      } else {
        h.offs.push_back(row * oc);
        h.items.push_back(std::move(it));
      }
      row += r;
    }
    if (!h.items.empty()) {
      h.out.assign(out, out + size_t(s->rows) * oc);
      driver_->push_handoff(std::move(h));
    }
  }
  items.clear();
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_.batches++;
  stats_.rows += uint64_t(s->rows);
  stats_.requests += n_items;
  stats_.max_rows = std::max<uint64_t>(stats_.max_rows, uint64_t(s->rows));
  stats_.gpu_busy_s += busy;
}

// One round for this unit on its driver's pump thread (see driver.h).
bool BatchedUnit::pump(bool watch, bool& busy) {
  using clk = std::chrono::steady_clock;
  PumpState& P = ps_;
  bool progress = false;
  // ---- take what the front ends queued (O(1) under each shard's lock:
  // producers never wait behind batch formation), then launch everything
  // that fits into the free slots
  if (!P.free_list.empty() && queued_n_.load(std::memory_order_acquire) > 0) drain_shards(P.pending);
  bool hold = false;
  if (opts_.max_wait_us > 0 && P.inflight.empty() && !P.pending.empty()) {
    // idle device: give a lone request up to max_wait_us to gather company
    int64_t rows = queued_rows_.load(std::memory_order_relaxed);
    for (const auto& it : P.pending) rows += it.rows;
    if (rows < opts_.max_batch) {
      const auto now = clk::now();
      if (!P.holding) {
        P.holding = true;
        P.hold_start = now;
      }
      hold = now - P.hold_start < std::chrono::microseconds(opts_.max_wait_us) && running_.load();
    }
  }
  if (!hold) P.holding = false;
  while (!hold && !P.pending.empty() && !P.free_list.empty()) {
    Slot* s = P.free_list.back();
    P.free_list.pop_back();
    int rows = 0;
    const int cols = P.pending.front().cols;
    while (!P.pending.empty()) {
      Item& it = P.pending.front();
      if (!s->items.empty() && (it.cols != cols || rows + it.rows > opts_.max_batch)) break;
      rows += it.rows;
      s->items.push_back(std::move(it));
      P.pending.pop_front();
    }
    s->rows = rows;
    s->cols = cols;
    const auto t0 = clk::now();
    const bool ok = launch(s);
    launch_cpu_s_.store(launch_cpu_s_.load(std::memory_order_relaxed) +
                            std::chrono::duration<double>(clk::now() - t0).count(),
                        std::memory_order_relaxed);
    (ok ? P.inflight : P.free_list).push_back(s);
    progress = true;
  }
  // ---- reap finished batches
  if (!P.inflight.empty()) {
    const int hang_ms = hang_ms_.load(std::memory_order_relaxed);
    // The clock is read only when a check needs it: the injected-hang test
    // on completion, and the watchdog when the driver asks (`watch`).
    clk::time_point now{};
    bool have_now = false;
    auto now_ = [&] {
      if (!have_now) {
        now = clk::now();
        have_now = true;
      }
      return now;
    };
    const bool wd = opts_.hang_timeout_ms > 0 && watch;
    for (size_t i = 0; i < P.inflight.size();) {
      Slot* s = P.inflight[i];
      hipError_t st =
          cpu_ ? (!s->call || s->call->done() ? hipSuccess : hipErrorNotReady) : hipEventQuery(s->ev.get());
      if (st == hipSuccess && hang_ms > 0 && now_() - s->t_launch < std::chrono::milliseconds(hang_ms))
        st = hipErrorNotReady;  // injected slow / hung device
      if (st == hipErrorNotReady) {
        if (wd && !s->abandoned && now_() - s->t_launch > std::chrono::milliseconds(opts_.hang_timeout_ms))
          abandon(s);
        // Slots are polled in launch order and the poll stops at the first
        // busy one (an hipEventQuery per slot per spin was ~3% of serving
        // CPU): batches of one unit finish in order in practice, and an
        // abandoned slot does not hold back the younger ones.
        if (!s->abandoned) break;
        ++i;
        continue;
      }
      const auto t0 = clk::now();
      complete(s, st);
      complete_cpu_s_.store(complete_cpu_s_.load(std::memory_order_relaxed) +
                                std::chrono::duration<double>(clk::now() - t0).count(),
                            std::memory_order_relaxed);
      P.inflight.erase(P.inflight.begin() + long(i));
      P.free_list.push_back(s);
      progress = true;
    }
  }
  if (!progress && abandoned_slots_.load(std::memory_order_relaxed) >= int(slots_.size())) {
    // Wedged device: answer what is still queued instead of letting it wait.
    std::deque<Item> rest;
    drain_shards(rest);
    for (auto& it : P.pending) rest.push_back(std::move(it));
    P.pending.clear();
    if (!rest.empty()) {
      auto e = device_error(ApiError::UNAVAILABLE, "every batch slot of this GPU is wedged");
      for (auto& it : rest) {
        inflight_rows_.fetch_sub(it.rows, std::memory_order_relaxed);
        it.k(Outcome::fail(e));
      }
    }
  }
  busy = !P.inflight.empty() || !P.pending.empty();
  return progress;
}

// Shutdown (pump thread, from DeviceDriver::retire): launch what was taken,
// then finish and answer everything in flight.  An asynchronous CPU call gets
// a bounded wait (it owns its buffers, so one that never finishes is dropped
// safely and its requests fail).
void BatchedUnit::finish_all() {
  using clk = std::chrono::steady_clock;
  PumpState& P = ps_;
  const auto until = clk::now() + std::chrono::seconds(10);
  while (!P.pending.empty() && clk::now() < until) {
    bool busy = false;
    if (!pump(true, busy)) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  for (Slot* s : P.inflight) {
    hipError_t st = hipSuccess;
    if (!cpu_) {
      st = hipEventSynchronize(s->ev.get());
    } else if (s->call) {
      while (!s->call->done() && clk::now() < until) std::this_thread::sleep_for(std::chrono::microseconds(50));
      if (!s->call->done()) {
        s->call.reset();
        st = hipErrorNotReady;
      }
    }
    complete(s, st);
    P.free_list.push_back(s);
  }
  P.inflight.clear();
  for (auto& it : P.pending) {
    inflight_rows_.fetch_sub(it.rows, std::memory_order_relaxed);
    it.k(Outcome::fail(make_error(ApiError::UNAVAILABLE, "GPU unit stopped")));
  }
  P.pending.clear();
}

// Low-CPU mode (spin_wait off), the only busy unit of its driver: block on
// its oldest batch -- unless the hang watchdog or an injected hang needs the
// pump to keep polling.
bool BatchedUnit::block_on_oldest() {
  if (ps_.inflight.empty()) return false;
  if (cpu_) {  // an asynchronous CPU call (a peer rank): a bounded wait on its replies
    auto& c = ps_.inflight.front()->call;
    return c && c->wait_us(200);
  }
  if (opts_.hang_timeout_ms > 0 || hang_ms_.load(std::memory_order_relaxed) > 0) return false;
  (void)hipEventSynchronize(ps_.inflight.front()->ev.get());
  return true;
}

ErrPtr BatchedUnit::device_error(ApiError kind, std::string info) {
  auto e = std::make_shared<EngineError>(*make_error(kind, std::move(info)));
  e->device_fault = true;
  return e;
}

void BatchedUnit::note_failure() {
  failed_batches_.fetch_add(1, std::memory_order_relaxed);
  if (consec_fail_.fetch_add(1, std::memory_order_relaxed) + 1 >= opts_.fail_threshold) {
    open_until_ns_.store(now_ns() + int64_t(opts_.cooldown_ms) * 1000000, std::memory_order_release);
    trips_.fetch_add(1, std::memory_order_relaxed);
  }
}

void BatchedUnit::note_success() {
  if (consec_fail_.load(std::memory_order_relaxed) != 0) consec_fail_.store(0, std::memory_order_relaxed);
}

bool BatchedUnit::healthy() const {
  const int64_t until = open_until_ns_.load(std::memory_order_acquire);
  return until == 0 || now_ns() >= until;
}

void BatchedUnit::abandon(Slot* s) {
  std::vector<Item> items;
  items.swap(s->items);
  inflight_rows_.fetch_sub(s->rows, std::memory_order_relaxed);
  s->rows = 0;
  s->abandoned = true;
  abandoned_slots_.fetch_add(1, std::memory_order_relaxed);
  hangs_.fetch_add(1, std::memory_order_relaxed);
  // A hang trips the unit at once; the next failure after the cooldown re-trips it.
  consec_fail_.store(std::max(consec_fail_.load(), opts_.fail_threshold - 1));
  note_failure();
  auto e = device_error(ApiError::DEADLINE_EXCEEDED, "GPU batch exceeded the hang watchdog (" +
                                                         std::to_string(opts_.hang_timeout_ms) + " ms)");
  for (auto& it : items) {
    it.k(Outcome::fail(e));  // run_ptr callers too: their buffers are never a DMA source
    if (s->direct) s->parked.push_back(std::move(it));  // keep the request (DMA source) alive
  }
}

bool BatchedUnit::take_injected_failure() {
  std::lock_guard<std::mutex> g(fault_mu_);
  if (fault_.fail_after < 0) return false;
  ++fault_launches_;
  if (fault_launches_ <= fault_.fail_after) return false;
  if (fault_.fail_count >= 0 && fault_injected_ >= fault_.fail_count) return false;
  ++fault_injected_;
  return true;
}

void BatchedUnit::inject_fault(const FaultSpec& f) {
  std::lock_guard<std::mutex> g(fault_mu_);
  fault_ = f;
  fault_launches_ = 0;
  fault_injected_ = 0;
  fault_armed_.store(f.fail_after >= 0, std::memory_order_relaxed);
  hang_ms_.store(std::max(0, f.hang_ms), std::memory_order_relaxed);
}

UnitHealth BatchedUnit::health() const {
  UnitHealth h;
  h.healthy = healthy();
  h.consecutive_failures = consec_fail_.load();
  h.failed_batches = failed_batches_.load();
  h.hangs = hangs_.load();
  h.trips = trips_.load();
  std::lock_guard<std::mutex> g(fault_mu_);
  h.injected = uint64_t(fault_injected_);
  return h;
}

BatcherStats BatchedUnit::stats() const {
  std::lock_guard<std::mutex> g(stats_mu_);
  BatcherStats s = stats_;
  s.launch_cpu_s = launch_cpu_s_.load(std::memory_order_relaxed);
  s.complete_cpu_s = complete_cpu_s_.load(std::memory_order_relaxed);
  return s;
}

void BatchedUnit::collect_metrics(MetricsRegistry& m, const Labels& labels) const {
  const BatcherStats st = stats();
  Labels l = labels;
  l.emplace_back("device", std::to_string(opts_.device));
  m.counter("seldon_gpu_batches", l)->set(double(st.batches));
  m.counter("seldon_gpu_rows", l)->set(double(st.rows));
  m.counter("seldon_gpu_requests", l)->set(double(st.requests));
  m.counter("seldon_gpu_busy_seconds", l)->set(st.gpu_busy_s);
  m.gauge("seldon_gpu_max_batch_rows", l)->set(double(st.max_rows));
  m.gauge("seldon_gpu_inflight_rows", l)->set(double(inflight_rows()));
  m.gauge("seldon_gpu_slots", l)->set(double(opts_.slots));
  const UnitHealth h = health();
  m.gauge("seldon_gpu_healthy", l)->set(h.healthy ? 1.0 : 0.0);
  m.counter("seldon_gpu_failed_batches", l)->set(double(h.failed_batches));
  m.counter("seldon_gpu_hangs", l)->set(double(h.hangs));
  m.counter("seldon_gpu_unhealthy_trips", l)->set(double(h.trips));
  // per-unit kernel-time histogram (launch -> completion event of each batch)
  // and batch-size distribution
  m.timer("seldon_gpu_batch_device", l, true)->hist.copy_from(batch_hist_);
  Series* rows = m.gauge("seldon_gpu_batch_rows_p50", l);
  rows->set(rows_hist_.quantile(0.5) * 1e6);
  m.gauge("seldon_gpu_batch_rows_p99", l)->set(rows_hist_.quantile(0.99) * 1e6);
}

void BatchedUnit::reset_stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_ = BatcherStats();
  launch_cpu_s_.store(0.0, std::memory_order_relaxed);
  complete_cpu_s_.store(0.0, std::memory_order_relaxed);
}

namespace {
// A synchronous caller's wait for its continuation (run_ptr / run_dense:
// Python ops, the device Mahalanobis step, tests).  The pump thread answers
// within tens of microseconds, so the caller spins that long before it
// sleeps: a futex wake-up of a blocked waiter costs about as much again as
// the whole GPU round trip (std::promise always took that path).
struct SyncWait {
  std::atomic<int> state{0};  // 0 waiting, 1 done
  std::atomic<bool> sleeping{false};
  std::mutex mu;
  std::condition_variable cv;
  Outcome out;
  void set(Outcome o) {
    out = std::move(o);
    // seq_cst on both sides of the state / sleeping handshake: a release
    // store here could still sit in the store buffer while the load of
    // `sleeping` below reads false and the waiter, about to sleep, reads
    // state == 0 -- both would miss each other
    state.store(1, std::memory_order_seq_cst);
    if (sleeping.load(std::memory_order_seq_cst)) {
      std::lock_guard<std::mutex> g(mu);
      cv.notify_all();
    }
  }
  Outcome wait() {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(200);
    for (unsigned n = 1; state.load(std::memory_order_acquire) == 0; ++n) {
      _mm_pause();
      if ((n & 63) == 0 && std::chrono::steady_clock::now() >= until) {
        std::unique_lock<std::mutex> lk(mu);
        sleeping.store(true, std::memory_order_seq_cst);
        cv.wait(lk, [&] { return state.load(std::memory_order_seq_cst) != 0; });
        break;
      }
    }
    return std::move(out);
  }
};
}  // namespace

std::vector<double> BatchedUnit::run_ptr(const double* X, int rows, int cols, int64_t* seq) {
  if (rows <= 0 || cols <= 0) throw std::runtime_error("run_ptr: empty input");
  const int want = model_->in_cols();
  if (want > 0 && cols != want)
    throw std::runtime_error("X has " + std::to_string(cols) + " features, but " + model_->name() + " is expecting " +
                             std::to_string(want) + " features as input.");
  auto msg = std::make_shared<SeldonMessage>();
  msg->payload = Payload::Data;
  msg->data.kind = DataKind::Tensor;
  msg->data.shape = {rows, cols};
  auto w = std::make_shared<SyncWait>();
  Item it;
  it.req = std::move(msg);
  it.xp = X;
  it.caller_mem = true;
  it.rows = rows;
  it.cols = cols;
  if (seq) {  // written by the pump thread before the continuation; read after wait()
    *seq = -1;
    it.seq_out = seq;
  }
  it.k = [w](Outcome o) { w->set(std::move(o)); };
  submit_item(std::move(it));
  Outcome o = w->wait();
  if (o.err) throw std::runtime_error(o.err->info);
  return std::move(o.msg->data.values);
}

std::vector<double> BatchedUnit::run_dense(const std::vector<double>& X, int rows, int cols) {
  auto msg = std::make_shared<SeldonMessage>();
  msg->payload = Payload::Data;
  msg->data.kind = DataKind::Tensor;
  msg->data.shape = {rows, cols};
  msg->data.values = X;
  auto w = std::make_shared<SyncWait>();
  CallCtx c{nullptr, nullptr};
  transform_input(c, msg, [w](Outcome o) { w->set(std::move(o)); });
  Outcome o = w->wait();
  if (o.err) throw std::runtime_error(o.err->info);
  return std::move(o.msg->data.values);
}

}  // namespace sca::gpu
