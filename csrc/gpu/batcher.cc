#include "batcher.h"

#include <immintrin.h>

#include <chrono>
#include <cstring>
#include <future>

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

BatchedUnit::BatchedUnit(RowModelPtr model, BatcherOptions opts) : model_(std::move(model)), opts_(opts) {
  if (opts_.max_batch < 1) opts_.max_batch = 1;
  if (opts_.slots < 1) opts_.slots = 1;
  device_io_ = model_->device_io_only();
  zc_input_ = model_->zero_copy_input();
  segmented_ = model_->segmented();
  {
    const int oc = model_->out_cols(model_->in_cols() > 0 ? model_->in_cols() : 1);
    default_names_ = model_->class_names();
    if (default_names_.empty())
      for (int c = 0; c < oc; ++c) default_names_.push_back("t:" + std::to_string(c));
  }
  if (opts_.device < 0) {
    running_.store(true);
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
  running_.store(true);
  submit_th_ = std::thread([this] { submit_loop(); });
  // One completion thread per slot: responses of concurrent batches are
  // scattered (and their graph continuations run) in parallel.
  for (auto& s : slots_) {
    Slot* raw = s.get();
    s->th = std::thread([this, raw] { complete_loop(raw); });
  }
}

BatchedUnit::~BatchedUnit() { stop(); }

void BatchedUnit::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(mu_);
  }
  cv_submit_.notify_all();
  for (auto& s : slots_) s->cv.notify_all();
  if (submit_th_.joinable()) submit_th_.join();
  for (auto& s : slots_)
    if (s->th.joinable()) s->th.join();
  // Fail anything still queued.
  std::deque<Item> rest;
  {
    std::lock_guard<std::mutex> g(mu_);
    rest.swap(queue_);
  }
  for (auto& it : rest) it.k(Outcome::fail(make_error(ApiError::UNAVAILABLE, "GPU unit stopped")));
}

void BatchedUnit::ensure_capacity(Slot& s, int rows, int cols) {
  const int oc = model_->out_cols(cols);
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
  const size_t ws = model_->workspace_bytes(rows, cols);
  if (s.ws.bytes() < ws) s.ws.alloc(grow(s.ws.bytes(), ws), opts_.device);
  s.cap_rows = std::max(s.cap_rows, size_t(rows));
}

MsgPtr BatchedUnit::make_response(const Item& it, const double* out, int out_cols) const {
  auto m = std::make_shared<SeldonMessage>();
  m->payload = Payload::Data;
  const bool flat = model_->flat_output() && out_cols == 1;
  if (!flat) {  // client_class_names: explicit names, else t:0..t:C-1
    if (int(default_names_.size()) == out_cols) {
      m->data.names = default_names_;
    } else {
      m->data.names = model_->class_names();
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

void BatchedUnit::transform_input(const CallCtx&, MsgPtr in, Done k) {
  if (in->payload != Payload::Data) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, model_->name() + " expects numeric 'data' payload")));
    return;
  }
  Item it;
  std::vector<int64_t> shape;
  std::string err;
  if (!in->data.dense(shape, it.x, &err)) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, err)));
    return;
  }
  if (shape.empty()) {
    it.rows = it.x.empty() ? 0 : 1;
    it.cols = int(it.x.size());
  } else if (shape.size() == 1) {
    it.rows = 1;
    it.cols = int(shape[0]);
  } else {
    it.rows = int(shape[0]);
    int64_t c = 1;
    for (size_t i = 1; i < shape.size(); ++i) c *= shape[i];
    it.cols = int(c);
  }
  const int want = model_->in_cols();
  if (it.rows == 0 || (want > 0 && it.cols != want)) {
    k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR,
                               "X has " + std::to_string(it.cols) + " features, but " + model_->name() +
                                   " is expecting " + std::to_string(want) + " features as input.")));
    return;
  }
  it.req = std::move(in);
  it.k = std::move(k);
  if (opts_.device < 0) {
    const int oc = model_->out_cols(it.cols);
    std::vector<double> out(size_t(it.rows) * oc);
    model_->run_cpu(it.x.data(), it.rows, it.cols, out.data());
    MsgPtr r = make_response(it, out.data(), oc);
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
  inflight_rows_.fetch_add(it.rows, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> g(mu_);
    queued_rows_ += size_t(it.rows);
    queue_.push_back(std::move(it));
  }
  cv_submit_.notify_one();
}

void BatchedUnit::submit_loop() {
  (void)hipSetDevice(opts_.device);
  std::unique_lock<std::mutex> lk(mu_);
  auto free_slot = [&]() -> Slot* {
    for (auto& s : slots_)
      if (!s->busy) return s.get();
    return nullptr;
  };
  while (true) {
    cv_submit_.wait(lk, [&] { return !running_.load() || (!queue_.empty() && free_slot()); });
    if (!running_.load()) break;
    if (opts_.max_wait_us > 0 && queued_rows_ < size_t(opts_.max_batch)) {
      auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(opts_.max_wait_us);
      cv_submit_.wait_until(lk, deadline, [&] { return !running_.load() || queued_rows_ >= size_t(opts_.max_batch); });
      if (!running_.load()) break;
    }
    Slot* s = free_slot();
    s->busy = true;
    s->items.clear();
    int rows = 0;
    const int cols = queue_.front().cols;
    while (!queue_.empty()) {
      Item& it = queue_.front();
      if (!s->items.empty() && (it.cols != cols || rows + it.rows > opts_.max_batch)) break;
      rows += it.rows;
      queued_rows_ -= size_t(it.rows);
      s->items.push_back(std::move(it));
      queue_.pop_front();
    }
    lk.unlock();

    s->rows = rows;
    s->cols = cols;
    s->out_cols = model_->out_cols(cols);
    hipError_t err = hipSuccess;
    std::string launch_error;
    try {
      ensure_capacity(*s, rows, cols);
      double* hin = s->h_in.host<double>();
      size_t off = 0;
      for (const auto& it : s->items) {
        memcpy(hin + off, it.x.data(), it.x.size() * sizeof(double));
        off += it.x.size();
      }
      const size_t bin = size_t(rows) * cols * sizeof(double), bout = size_t(rows) * s->out_cols * sizeof(double);
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
      auto run = [&](const double* x, double* y) {
        if (seg) model_->launch_segments(x, rows, cols, y, s->ws.get(), seg, nseg, st);
        else model_->launch(x, rows, cols, y, s->ws.get(), st);
      };
      if (opts_.zero_copy && !device_io_ && bin + bout <= opts_.zero_copy_max_bytes) {
        // Output always zero-copy (written once); input zero-copy only if the
        // kernel reads each element once -- models that re-read X from many
        // workgroups (tree chunks) get one DMA into HBM first.
        const double* xin = s->h_in.dev<double>();
        if (!zc_input_) {
          err = hipMemcpyAsync(s->d_in.get(), hin, bin, hipMemcpyHostToDevice, st);
          xin = s->d_in.as<double>();
        }
        if (err == hipSuccess) run(xin, s->h_out.dev<double>());
      } else {
        err = hipMemcpyAsync(s->d_in.get(), hin, bin, hipMemcpyHostToDevice, st);
        if (err == hipSuccess) {
          run(s->d_in.as<double>(), s->d_out.as<double>());
          err = hipMemcpyAsync(s->h_out.host<double>(), s->d_out.get(), bout, hipMemcpyDeviceToHost, st);
        }
      }
      if (err == hipSuccess) err = hipGetLastError();
      if (err == hipSuccess) err = hipEventRecord(s->ev.get(), st);
    } catch (const std::exception& ex) {
      err = hipErrorUnknown;
      launch_error = ex.what();
    }
    if (err != hipSuccess) {
      auto e = make_error(ApiError::EXECUTION_FAILURE,
                          "GPU launch failed: " + (launch_error.empty() ? std::string(hipGetErrorString(err)) : launch_error));
      inflight_rows_.fetch_sub(rows, std::memory_order_relaxed);
      for (auto& it : s->items) it.k(Outcome::fail(e));
      s->items.clear();
      lk.lock();
      s->busy = false;
      continue;
    }
    lk.lock();
    s->launched = true;
    s->cv.notify_one();
  }
}

void BatchedUnit::complete_loop(Slot* s) {
  (void)hipSetDevice(opts_.device);
  while (true) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      s->cv.wait(lk, [&] { return s->launched || !running_.load(); });
      if (!s->launched) break;
      s->launched = false;
    }
    auto t0 = std::chrono::steady_clock::now();
    hipError_t st;
    if (opts_.spin_wait) {
      // A batch round trip is ~10-30 us: spin briefly, then back off.
      int spins = 0;
      while ((st = hipEventQuery(s->ev.get())) == hipErrorNotReady) {
        if (++spins < 2000) _mm_pause();
        else std::this_thread::yield();
      }
    } else {
      st = hipEventSynchronize(s->ev.get());
    }
    const double busy = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    inflight_rows_.fetch_sub(s->rows, std::memory_order_relaxed);
    if (st != hipSuccess) {
      auto e = make_error(ApiError::EXECUTION_FAILURE, std::string("GPU execution failed: ") + hipGetErrorString(st));
      for (auto& it : s->items) it.k(Outcome::fail(e));
    } else {
      finish_items(s->items, s->h_out.host<double>(), s->out_cols);
    }
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.batches++;
      stats_.rows += uint64_t(s->rows);
      stats_.requests += s->items.size();
      stats_.max_rows = std::max<uint64_t>(stats_.max_rows, uint64_t(s->rows));
      stats_.gpu_busy_s += busy;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      s->items.clear();
      s->busy = false;
    }
    cv_submit_.notify_one();
  }
}

void BatchedUnit::finish_items(std::vector<Item>& items, const double* out, int out_cols) {
  size_t row = 0;
  for (auto& it : items) {
    MsgPtr r = make_response(it, out + row * out_cols, out_cols);
    row += size_t(it.rows);
    it.k(Outcome::ok(std::move(r)));
  }
}

BatcherStats BatchedUnit::stats() const {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

void BatchedUnit::reset_stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_ = BatcherStats();
}

std::vector<double> BatchedUnit::run_dense(const std::vector<double>& X, int rows, int cols) {
  auto msg = std::make_shared<SeldonMessage>();
  msg->payload = Payload::Data;
  msg->data.kind = DataKind::Tensor;
  msg->data.shape = {rows, cols};
  msg->data.values = X;
  std::promise<Outcome> p;
  auto f = p.get_future();
  CallCtx c{nullptr, nullptr};
  transform_input(c, msg, [&p](Outcome o) { p.set_value(std::move(o)); });
  Outcome o = f.get();
  if (o.err) throw std::runtime_error(o.err->info);
  return o.msg->data.values;
}

}  // namespace sca::gpu
