// Python-implemented predictive unit.
//
// Wraps a Python adapter (seldon_core_amd.serving.adapter.PythonUnit) that
// applies the reference wrapper's dispatch precedence
// (python/seldon_core/seldon_methods.py:17-302: *_rest / *_grpc hooks ->
// *_raw -> high-level predict(X, names, meta)) to a user component.
//
// The reference runs each component as a Flask/gunicorn microservice: every
// graph hop serialises the SeldonMessage to JSON, POSTs it, and gunicorn hands
// it to one of N worker processes (python/seldon_core/microservice.py:153-174,
// 250-261).  Here the component lives next to the engine and is fed three ways:
//
// * Dense hand-off.  For a numeric DefaultData payload (tensor / ndarray /
//   tftensor) and a method without low-level hooks, the user's high-level
//   method gets a numpy view over the message's fp64 values (no JSON, no
//   copy) and its numeric result is written straight back into a dense
//   message that keeps the request's data kind -- the same response rules as
//   the reference (utils.py:306-407).  Everything else (raw hooks, strData,
//   jsonData, aggregate, feedback) takes the JSON-text path, exactly the
//   payload the reference microservice would have seen.
// * Work queue.  Engine threads only enqueue; Python runs on the unit's own
//   thread(s), so front-end threads never block on the GIL.  With
//   `batch_rows > 0` (opt-in: the component must be row-wise), concurrent
//   dense requests of one method and width are stacked into one call and the
//   result rows are split back -- micro-batching for Python models.
// * Process pool (`workers > 0`, the analogue of gunicorn --workers): N fresh
//   Python processes, each with its own copy of the component and its own
//   GIL, fed binary frames (header + raw fp64 rows + small JSON text) over a
//   Unix socketpair by one dispatcher thread each.  The parent takes no GIL
//   for a dense call at all.
#pragma once

#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../core/engine.h"

namespace sca {

namespace py = pybind11;

struct PyUnitOptions {
  int batch_rows = 0;           // > 0: stack concurrent dense requests (row-wise components only)
  std::vector<int> worker_fds;  // process pool sockets (owned); empty = in-process
};

// Binary frame of the process-pool protocol (little-endian, both directions):
// header, then x_bytes of fp64 values, then text_bytes of UTF-8 text.
struct PoolFrame {
  static constexpr uint32_t kMagic = 0x57414353;  // "SCAW"
  uint32_t magic = kMagic;
  uint32_t op = 0;     // request: PyUnit::Op; response: 0 dense, 1 json, 3 error, 4 component error reply
  uint32_t ndim = 0;
  uint32_t flags = 0;  // request: 1 = dense payload
  int64_t shape[8] = {};
  uint64_t x_bytes = 0;
  uint64_t text_bytes = 0;
};
static_assert(sizeof(PoolFrame) == 96, "pool frame header layout");

class PyUnit : public Unit {
 public:
  enum Op : uint32_t { kPredict = 1, kTransformInput = 2, kTransformOutput = 3, kRoute = 4, kAggregate = 5,
                       kFeedback = 6 };

  struct Stats {
    uint64_t jobs = 0, calls = 0, rows = 0, batched_calls = 0, pool_calls = 0;
  };

  PyUnit(py::object adapter, uint32_t builtin_mask, PyUnitOptions opts = {})
      : adapter_(std::move(adapter)), builtin_(builtin_mask), opts_(std::move(opts)) {
    if (py::hasattr(adapter_, "dense_methods")) {
      for (auto& m : adapter_.attr("dense_methods")().cast<std::vector<std::string>>()) {
        const int op = op_of(m);
        if (op) dense_mask_ |= 1u << op;
      }
    }
    has_call_json_ = py::hasattr(adapter_, "call_json");
    dead_.reset(new std::atomic<bool>[std::max<size_t>(1, opts_.worker_fds.size())]());
    running_ = true;
    if (opts_.worker_fds.empty()) {
      threads_.emplace_back([this] { loop(-1); });
    } else {
      for (size_t i = 0; i < opts_.worker_fds.size(); ++i) threads_.emplace_back([this, i] { loop(int(i)); });
    }
  }

  ~PyUnit() override {
    stop();
    py::gil_scoped_acquire g;
    adapter_ = py::object();
  }

  // Drain: queued work is failed, worker sockets are closed (each worker
  // process sees EOF and exits).  Idempotent.
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stopped_) return;
      stopped_ = true;
      running_ = false;
    }
    cv_.notify_all();
    for (int fd : opts_.worker_fds) ::shutdown(fd, SHUT_RDWR);
    {
      // The in-process thread may be waiting for the GIL this thread holds.
      std::unique_ptr<py::gil_scoped_release> rel;
      if (PyGILState_Check()) rel = std::make_unique<py::gil_scoped_release>();
      for (auto& t : threads_)
        if (t.joinable()) t.join();
    }
    for (int fd : opts_.worker_fds) ::close(fd);
    fail_all("python unit stopped");
  }

  uint32_t builtin_methods() const override { return builtin_; }
  std::string kind() const override { return opts_.worker_fds.empty() ? "python" : "python-pool"; }

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override { submit(kTransformInput, c, std::move(in), std::move(k)); }
  void predict(const CallCtx& c, MsgPtr in, Done k) override { submit(kPredict, c, std::move(in), std::move(k)); }
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { submit(kTransformOutput, c, std::move(in), std::move(k)); }
  void route(const CallCtx& c, MsgPtr in, Done k) override { submit(kRoute, c, std::move(in), std::move(k)); }
  void aggregate(const CallCtx& c, std::vector<MsgPtr> in, Done k) override {
    Job j = make_job(kAggregate, c);
    j.ins = std::move(in);
    j.k = std::move(k);
    enqueue(std::move(j));
  }
  void send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) override {
    Job j = make_job(kFeedback, c);
    j.fb = std::move(fb);
    j.fk = std::move(k);
    enqueue(std::move(j));
  }
  bool ready() const override {
    if (!opts_.worker_fds.empty() && alive_workers() == 0) return false;
    py::gil_scoped_acquire g;
    if (!py::hasattr(adapter_, "ready")) return true;
    try {
      return adapter_.attr("ready")().cast<bool>();
    } catch (...) {
      return false;
    }
  }
  std::string snapshot() const override {
    py::gil_scoped_acquire g;
    if (!py::hasattr(adapter_, "snapshot")) return "";
    return adapter_.attr("snapshot")().cast<std::string>();
  }
  void restore(const std::string& s) override {
    py::gil_scoped_acquire g;
    if (py::hasattr(adapter_, "restore")) adapter_.attr("restore")(py::bytes(s));
  }

  Stats stats() const {
    std::lock_guard<std::mutex> g(stats_mu_);
    return stats_;
  }
  int alive_workers() const {
    int n = 0;
    for (size_t i = 0; i < opts_.worker_fds.size(); ++i) n += dead_[i].load() ? 0 : 1;
    return n;
  }
  const PyUnitOptions& options() const { return opts_; }

 private:
  struct Job {
    Op op = kPredict;
    MsgPtr in;
    std::vector<MsgPtr> ins;
    std::shared_ptr<const Feedback> fb;
    Done k;
    FbDone fk;
    ExecPtr exec;
    std::string node;
    bool dense = false;
    std::vector<int64_t> shape;
    std::vector<double> own;  // decoded values when the message holds no flat fp64 array
    const double* x = nullptr;
    int64_t rows = 0, cols = 0;
  };

  static int op_of(const std::string& m) {
    if (m == "predict") return kPredict;
    if (m == "transform_input") return kTransformInput;
    if (m == "transform_output") return kTransformOutput;
    if (m == "route") return kRoute;
    return 0;
  }
  static const char* kind_name(DataKind k) {
    return k == DataKind::NdArray ? "ndarray" : k == DataKind::TfTensor ? "tftensor" : "tensor";
  }
  static const char* op_name(Op op) {
    switch (op) {
      case kPredict: return "predict";
      case kTransformInput: return "transform_input";
      case kTransformOutput: return "transform_output";
      case kRoute: return "route";
      case kAggregate: return "aggregate";
      case kFeedback: return "send_feedback";
    }
    return "?";
  }

  Job make_job(Op op, const CallCtx& c) {
    Job j;
    j.op = op;
    if (c.exec) j.exec = *c.exec;
    if (c.node) j.node = c.node->name;
    return j;
  }

  void submit(Op op, const CallCtx& c, MsgPtr in, Done k) {
    Job j = make_job(op, c);
    j.k = std::move(k);
    if ((dense_mask_ >> op) & 1u) prepare_dense(j, in);
    j.in = std::move(in);
    enqueue(std::move(j));
  }

  // Dense view of a numeric DefaultData payload (no copy for tensor / numeric
  // ndarray messages: the view points into the message, which the job owns).
  static void prepare_dense(Job& j, const MsgPtr& in) {
    if (!in || in->payload != Payload::Data || in->data.kind == DataKind::None) return;
    const DefaultData& d = in->data;
    if (d.kind == DataKind::Tensor || (d.kind == DataKind::NdArray && d.nd_dense)) {
      int64_t n = 1;
      for (auto s : d.shape) {
        if (s < 0) return;
        n *= s;
      }
      if (d.shape.empty() || n != int64_t(d.values.size())) return;
      j.shape = d.shape;
      j.x = d.values.data();
    } else {
      std::vector<int64_t> shp;
      if (!d.dense(shp, j.own, nullptr) || shp.empty()) return;
      j.shape = std::move(shp);
      j.x = j.own.data();
    }
    if (j.shape.size() > 8) return;
    j.rows = j.shape[0];
    j.cols = 1;
    for (size_t i = 1; i < j.shape.size(); ++i) j.cols *= j.shape[i];
    j.dense = true;
  }

  void enqueue(Job j) {
    bool stopped = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      stopped = !running_;
      if (!stopped) queue_.push_back(std::move(j));
    }
    if (stopped) lk_fail(j, "python unit stopped");
    else cv_.notify_one();
  }

  static void lk_fail(Job& j, const std::string& why) {
    auto e = make_error(ApiError::MICROSERVICE_ERROR, why);
    if (j.fk) j.fk(e);
    else if (j.k) j.k(Outcome::fail(e));
  }

  void fail_all(const std::string& why) {
    std::deque<Job> q;
    {
      std::lock_guard<std::mutex> g(mu_);
      q.swap(queue_);
    }
    for (auto& j : q) lk_fail(j, why);
  }

  // Two dense jobs can share one stacked call: same method, same trailing
  // dimensions (2-D rows of one width, or e.g. [n, 3, 224, 224] images), same
  // feature names; they stack along the first axis.
  static bool stackable(const Job& a, const Job& b) {
    return a.dense && b.dense && a.op == b.op && a.shape.size() >= 2 && a.shape.size() == b.shape.size() &&
           std::equal(a.shape.begin() + 1, a.shape.end(), b.shape.begin() + 1) && a.in->data.names == b.in->data.names;
  }

  bool take(std::vector<Job>& out) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !running_ || !queue_.empty(); });
    if (!running_ && queue_.empty()) return false;
    out.push_back(std::move(queue_.front()));
    queue_.pop_front();
    if (opts_.batch_rows > 0 && out[0].dense && out[0].op != kRoute && out[0].shape.size() >= 2) {
      int64_t rows = out[0].rows;
      for (auto it = queue_.begin(); it != queue_.end() && rows < opts_.batch_rows;) {
        if (stackable(out[0], *it) && rows + it->rows <= opts_.batch_rows) {
          rows += it->rows;
          out.push_back(std::move(*it));
          it = queue_.erase(it);
        } else {
          ++it;
        }
      }
    }
    return true;
  }

  void loop(int worker) {
    std::vector<Job> jobs;
    while (true) {
      jobs.clear();
      if (!take(jobs)) return;
      if (worker >= 0 && dead_[size_t(worker)].load()) {
        // this worker process is gone: hand the work back to the others
        if (alive_workers() > 0) {
          std::lock_guard<std::mutex> g(mu_);
          for (auto& j : jobs) queue_.push_front(std::move(j));
          cv_.notify_all();
          return;
        }
        for (auto& j : jobs) lk_fail(j, "all python worker processes have exited");
        continue;
      }
      std::vector<Outcome> res;
      std::vector<ErrPtr> fb_res;
      try {
        if (worker < 0) run_inproc(jobs, res, fb_res);
        else run_pool(worker, jobs, res, fb_res);
      } catch (const std::exception& e) {  // backstop: a request error must never end the serving thread
        auto err = make_error(ApiError::MICROSERVICE_ERROR, e.what());
        res.assign(jobs.size(), Outcome::fail(err));
        fb_res.assign(1, err);
      }
      if (res.size() != jobs.size()) res.resize(jobs.size(), Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "no result")));
      complete(jobs, res, fb_res);
    }
  }

  // Continuations run on the request's executor when it has one (as the GPU
  // batcher does), else on this thread.
  void complete(std::vector<Job>& jobs, std::vector<Outcome>& res, std::vector<ErrPtr>& fb_res) {
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.jobs += jobs.size();
    }
    for (size_t i = 0; i < jobs.size(); ++i) {
      Job& j = jobs[i];
      if (j.op == kFeedback) {
        FbDone k = std::move(j.fk);
        ErrPtr e = fb_res.empty() ? nullptr : fb_res[0];
        if (j.exec) j.exec->post([k = std::move(k), e]() { k(e); });
        else k(e);
      } else {
        Done k = std::move(j.k);
        Outcome o = std::move(res[i]);
        if (j.exec) j.exec->post([k = std::move(k), o = std::move(o)]() mutable { k(std::move(o)); });
        else k(std::move(o));
      }
    }
  }

  // ------------------------------------------------------------ response
  static MsgPtr dense_response(const Job& j, const double* y, const std::vector<int64_t>& shape,
                               std::vector<std::string> names, const std::string& meta_text,
                               const DataKind* kind = nullptr) {
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    int64_t n = 1;
    for (auto s : shape) n *= s;
    m->data.set_dense(kind ? *kind : j.in->data.kind, shape, std::vector<double>(y, y + n));
    m->data.names = std::move(names);
    m->has_meta = true;
    if (!meta_text.empty()) {
      SeldonMessage tmp;
      message_from_json(parse_json("{\"meta\":" + meta_text + "}"), tmp);
      m->meta = std::move(tmp.meta);
    }
    m->meta.puid = j.in->meta.puid;
    return m;
  }

  // (float64 array, names, kind, meta json | None) from PythonUnit.call_json;
  // called with the GIL held.
  static Outcome dense_reply(const Job& j, const py::tuple& t) {
    py::array_t<double, py::array::c_style | py::array::forcecast> Y(t[0]);
    std::vector<int64_t> shape(Y.shape(), Y.shape() + Y.ndim());
    const std::string kind = t[2].cast<std::string>();
    const DataKind k = kind == "tftensor" ? DataKind::TfTensor : kind == "ndarray" ? DataKind::NdArray : DataKind::Tensor;
    auto m = std::make_shared<SeldonMessage>();
    m->payload = Payload::Data;
    m->data.set_dense(k, shape, std::vector<double>(Y.data(), Y.data() + Y.size()));
    m->data.names = t[1].cast<std::vector<std::string>>();
    m->has_meta = true;
    if (!t[3].is_none()) {
      try {
        SeldonMessage tmp;
        message_from_json(parse_json("{\"meta\":" + t[3].cast<std::string>() + "}"), tmp);
        m->meta = std::move(tmp.meta);
      } catch (const std::exception& e) {
        return Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, std::string("bad meta from python unit: ") + e.what()));
      }
    }
    if (j.in) m->meta.puid = j.in->meta.puid;
    return Outcome::ok(std::move(m));
  }

  static Outcome json_response(const std::string& text) {
    if (text.empty() || text == "null") return Outcome::ok(nullptr);
    auto m = std::make_shared<SeldonMessage>();
    try {
      message_from_json(parse_json(text), *m);
    } catch (const std::exception& e) {
      return Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, std::string("bad response from python unit: ") + e.what()));
    }
    return Outcome::ok(std::move(m));
  }

  static std::string meta_json(const SeldonMessage& in) {
    if (!in.has_meta) return "null";
    SeldonMessage tmp;
    tmp.has_meta = true;
    tmp.meta = in.meta;
    std::string s;
    message_to_json(tmp, s);  // {"meta":{...}}
    // strip the wrapper object
    const size_t b = s.find(':');
    return s.substr(b + 1, s.size() - b - 2);
  }

  std::string request_text(const Job& j) const {
    std::string text;
    if (j.op == kAggregate) {
      std::vector<const SeldonMessage*> v;
      for (auto& m : j.ins) v.push_back(m.get());
      message_list_to_json(v, text);
    } else if (j.op == kFeedback) {
      feedback_to_json(*j.fb, text);
    } else {
      text.reserve(256);
      message_to_json(*j.in, text);
    }
    return text;
  }

  // ------------------------------------------------------------ in-process
  void run_inproc(std::vector<Job>& jobs, std::vector<Outcome>& res, std::vector<ErrPtr>& fb_res) {
    res.assign(jobs.size(), Outcome::fail(nullptr));
    Job& j0 = jobs[0];
    std::vector<std::string> texts;
    if (!j0.dense) texts.push_back(request_text(j0));  // serialise outside the GIL
    py::gil_scoped_acquire g;
    try {
      if (j0.dense) {
        call_dense_inproc(jobs, res);
      } else {
        py::object r = has_call_json_ ? adapter_.attr("call_json")(op_name(j0.op), texts[0], j0.node)
                                      : adapter_.attr(op_name(j0.op))(texts[0], j0.node);
        if (j0.op == kFeedback) fb_res.push_back(nullptr);
        else if (py::isinstance<py::tuple>(r)) {
          res[0] = dense_reply(j0, r.cast<py::tuple>());  // a raw hook's numeric array: no JSON
        } else {
          std::string out = r.is_none() ? std::string() : r.cast<std::string>();
          py::gil_scoped_release nogil;
          res[0] = json_response(out);
        }
      }
      std::lock_guard<std::mutex> sg(stats_mu_);
      stats_.calls++;
    } catch (py::error_already_set& e) {
      auto err = user_error(e);
      for (auto& r : res) r = Outcome::fail(err);
      fb_res.assign(1, err);
    } catch (const std::exception& e) {
      auto err = make_error(ApiError::MICROSERVICE_ERROR, e.what());
      for (auto& r : res) r = Outcome::fail(err);
      fb_res.assign(1, err);
    }
  }

  // A Python exception -> engine error.  The adapter's error_reply() applies
  // the reference wrapper's rules (wrapper.py:22-31, flask_utils.py:67-81):
  // the component's model_error_handler, else SeldonMicroserviceException's
  // own status / reason / to_dict(); anything else stays a plain 203.
  // Called with the GIL held.
  ErrPtr user_error(py::error_already_set& e) {
    std::string what = e.what();
    try {
      if (py::hasattr(adapter_, "error_reply")) {
        py::object r = adapter_.attr("error_reply")(e.value());
        if (!r.is_none()) {
          auto t = r.cast<py::tuple>();
          return make_user_error(t[0].cast<int>(), t[1].cast<std::string>(), t[2].cast<std::string>());
        }
      }
    } catch (py::error_already_set& inner) {
      what += std::string(" (error handler failed: ") + inner.what() + ")";
    } catch (const std::exception& inner) {
      what += std::string(" (error handler failed: ") + inner.what() + ")";
    }
    return make_error(ApiError::MICROSERVICE_ERROR, what);
  }

  // Pool reply op 4: {"status": int, "body": "<json>", "info": "..."}.
  static ErrPtr pool_user_error(const std::string& text) {
    try {
      Json j = parse_json(text);
      const Json* st = j.find("status");
      const Json* body = j.find("body");
      const Json* info = j.find("info");
      if (st && body) return make_user_error(int(st->as_number()), body->as_string(), info ? info->as_string() : "");
    } catch (const std::exception&) {
    }
    return make_error(ApiError::MICROSERVICE_ERROR, text);
  }

  void call_dense_inproc(std::vector<Job>& jobs, std::vector<Outcome>& res) {
    Job& j0 = jobs[0];
    py::array X;
    int64_t total = 0;
    for (auto& j : jobs) total += j.rows;
    if (jobs.size() == 1) {
      // zero-copy view; the capsule keeps the message (and decoded copy) alive
      auto* keep = new std::pair<MsgPtr, std::vector<double>>(j0.in, std::move(j0.own));
      const double* ptr = keep->second.empty() ? j0.x : keep->second.data();
      py::capsule base(keep, [](void* p) { delete static_cast<std::pair<MsgPtr, std::vector<double>>*>(p); });
      std::vector<py::ssize_t> shp(j0.shape.begin(), j0.shape.end());
      X = py::array_t<double>(shp, ptr, base);
      j0.x = ptr;
    } else {
      std::vector<py::ssize_t> shp(j0.shape.begin(), j0.shape.end());
      shp[0] = py::ssize_t(total);
      py::array_t<double> a(shp);
      double* dst = a.mutable_data();
      for (auto& j : jobs) {
        std::memcpy(dst, j.x, size_t(j.rows * j.cols) * sizeof(double));
        dst += j.rows * j.cols;
      }
      X = std::move(a);
    }
    py::object meta = jobs.size() == 1 ? py::object(py::str(meta_json(*j0.in))) : py::object(py::none());
    py::tuple t = adapter_.attr("call_dense")(op_name(j0.op), X, j0.in->data.names, meta, kind_name(j0.in->data.kind))
                      .cast<py::tuple>();
    const int code = t[0].cast<int>();
    {
      std::lock_guard<std::mutex> sg(stats_mu_);
      stats_.rows += uint64_t(total);
      if (jobs.size() > 1) stats_.batched_calls++;
    }
    if (code == 1) {  // anything but a numeric array: the full JSON response
      std::string text = t[1].cast<std::string>();
      py::gil_scoped_release nogil;
      if (jobs.size() == 1) res[0] = json_response(text);
      else
        for (auto& r : res)
          r = Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR,
                                       "batched python unit must return a numeric array with one row per input row"));
      return;
    }
    py::array_t<double, py::array::c_style | py::array::forcecast> Y(t[1]);
    std::vector<int64_t> yshape(Y.shape(), Y.shape() + Y.ndim());
    std::vector<std::string> names = t[2].cast<std::vector<std::string>>();
    std::string meta_text = t[3].is_none() ? std::string() : t[3].cast<std::string>();
    std::string meta_first = t[4].is_none() ? std::string() : t[4].cast<std::string>();
    const double* y = Y.data();
    py::gil_scoped_release nogil;
    split_dense(jobs, res, y, yshape, names, meta_text, meta_first, total);
  }

  // One result array -> one response per job (rows in job order).
  static void split_dense(std::vector<Job>& jobs, std::vector<Outcome>& res, const double* y,
                          const std::vector<int64_t>& yshape, const std::vector<std::string>& names,
                          const std::string& meta_all, const std::string& meta_first, int64_t total,
                          const DataKind* kind = nullptr) {
    if (jobs.size() == 1) {
      const std::string& mt = meta_first.empty() ? meta_all : meta_first;
      res[0] = Outcome::ok(dense_response(jobs[0], y, yshape, names, mt, kind));
      return;
    }
    if (yshape.empty() || yshape[0] != total) {
      for (auto& r : res)
        r = Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR,
                                     "batched python unit returned " + std::to_string(yshape.empty() ? 0 : yshape[0]) +
                                         " rows for " + std::to_string(total) + " input rows"));
      return;
    }
    int64_t per_row = 1;
    for (size_t i = 1; i < yshape.size(); ++i) per_row *= yshape[i];
    int64_t row = 0;
    for (size_t i = 0; i < jobs.size(); ++i) {
      std::vector<int64_t> shp = yshape;
      shp[0] = jobs[i].rows;
      // custom metrics describe one call: attach them to the first request only
      const std::string& mt = i == 0 && !meta_first.empty() ? meta_first : meta_all;
      res[i] = Outcome::ok(dense_response(jobs[i], y + row * per_row, shp, names, mt));
      row += jobs[i].rows;
    }
  }

  // ------------------------------------------------------------ process pool
  static bool write_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
      ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      c += w;
      n -= size_t(w);
    }
    return true;
  }
  static bool read_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n > 0) {
      ssize_t r = ::read(fd, c, n);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return false;
      c += r;
      n -= size_t(r);
    }
    return true;
  }

  void run_pool(int w, std::vector<Job>& jobs, std::vector<Outcome>& res, std::vector<ErrPtr>& fb_res) {
    const int fd = opts_.worker_fds[size_t(w)];
    res.assign(jobs.size(), Outcome::fail(nullptr));
    Job& j0 = jobs[0];
    PoolFrame h;
    h.op = j0.op;
    std::string text;
    std::vector<double> stacked;
    const double* x = nullptr;
    int64_t total = 0;
    for (auto& j : jobs) total += j.rows;
    if (j0.dense) {
      h.flags = 1;
      h.ndim = uint32_t(j0.shape.size());
      for (size_t i = 0; i < j0.shape.size(); ++i) h.shape[i] = j0.shape[i];
      h.shape[0] = total;
      if (jobs.size() == 1) {
        x = j0.x;
      } else {
        stacked.reserve(size_t(total * j0.cols));
        for (auto& j : jobs) stacked.insert(stacked.end(), j.x, j.x + j.rows * j.cols);
        x = stacked.data();
      }
      h.x_bytes = uint64_t(total * j0.cols) * sizeof(double);
      Json names = Json::array();
      for (auto& n : j0.in->data.names) names.push_back(Json(n));
      text = "{\"names\":" + names.dump() + ",\"meta\":" + (jobs.size() == 1 ? meta_json(*j0.in) : "null") +
             ",\"kind\":\"" + kind_name(j0.in->data.kind) + "\",\"node\":" + Json(j0.node).dump() + "}";
    } else {
      text = request_text(j0);
      text = Json(j0.node).dump() + "\n" + text;
    }
    h.text_bytes = text.size();
    PoolFrame r;
    std::vector<double> y;
    std::string rtext;
    bool ok = write_all(fd, &h, sizeof h) && (h.x_bytes == 0 || write_all(fd, x, h.x_bytes)) &&
              write_all(fd, text.data(), text.size()) && read_all(fd, &r, sizeof r) && r.magic == PoolFrame::kMagic;
    // a reply frame must describe whole doubles and sane sizes (1 GiB each)
    ok = ok && r.x_bytes % sizeof(double) == 0 && r.x_bytes <= (1ull << 30) && r.text_bytes <= (1ull << 30);
    if (ok) {
      y.resize(r.x_bytes / sizeof(double));
      rtext.resize(r.text_bytes);
      ok = (r.x_bytes == 0 || read_all(fd, y.data(), r.x_bytes)) && (r.text_bytes == 0 || read_all(fd, &rtext[0], r.text_bytes));
    }
    if (!ok) {
      dead_[size_t(w)].store(true);
      auto err = make_error(ApiError::MICROSERVICE_ERROR, "python worker process " + std::to_string(w) + " exited");
      for (auto& o : res) o = Outcome::fail(err);
      fb_res.assign(1, err);
      return;
    }
    {
      std::lock_guard<std::mutex> sg(stats_mu_);
      stats_.calls++;
      stats_.pool_calls++;
      stats_.rows += uint64_t(total);
      if (jobs.size() > 1) stats_.batched_calls++;
    }
    if (r.op == 3 || r.op == 4) {
      auto err = r.op == 4 ? pool_user_error(rtext) : make_error(ApiError::MICROSERVICE_ERROR, rtext);
      for (auto& o : res) o = Outcome::fail(err);
      fb_res.assign(1, err);
      return;
    }
    if (j0.op == kFeedback) {
      fb_res.push_back(nullptr);
      return;
    }
    if (r.op == 1) {
      if (jobs.size() == 1) res[0] = json_response(rtext);
      else
        for (auto& o : res)
          o = Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR,
                                       "batched python unit must return a numeric array with one row per input row"));
      return;
    }
    // dense: text = {"names":[...],"meta":{...}|null,"meta_first":{...}|null}
    // A worker's reply is untrusted input: its shape must fit the frame and
    // describe exactly the doubles sent, and a malformed names/meta document
    // (e.g. a metric with an unknown key) fails these jobs, not the server.
    try {
      constexpr uint32_t kMaxDims = sizeof(r.shape) / sizeof(r.shape[0]);
      if (r.ndim == 0 || r.ndim > kMaxDims) throw std::runtime_error("reply has " + std::to_string(r.ndim) + " dims");
      uint64_t n = 1;
      for (uint32_t i = 0; i < r.ndim; ++i) {
        if (r.shape[i] < 0) throw std::runtime_error("reply has a negative dimension");
        n *= uint64_t(r.shape[i]);
      }
      if (n * sizeof(double) != r.x_bytes)
        throw std::runtime_error("reply shape holds " + std::to_string(n) + " values but " +
                                 std::to_string(r.x_bytes / sizeof(double)) + " were sent");
      Json info = parse_json(rtext);
      std::vector<std::string> names;
      if (const Json* nm = info.find("names"))
        for (const auto& s : nm->items()) names.push_back(s.as_string());
      auto meta_of = [&](const char* key) {
        const Json* m = info.find(key);
        return m && !m->is_null() ? m->dump() : std::string();
      };
      std::vector<int64_t> yshape(r.shape, r.shape + r.ndim);
      // a raw hook's numeric reply (worker-side PythonUnit.call_json) names
      // its own data kind; a dense call keeps the request's
      DataKind k = DataKind::None;
      const Json* kj = info.find("kind");
      if (kj && kj->is_string() && jobs.size() == 1) {
        const std::string ks = kj->as_string();
        k = ks == "tftensor" ? DataKind::TfTensor : ks == "ndarray" ? DataKind::NdArray : DataKind::Tensor;
      }
      split_dense(jobs, res, y.data(), yshape, names, meta_of("meta"), meta_of("meta_first"), total,
                  k == DataKind::None ? nullptr : &k);
    } catch (const std::exception& e) {
      auto err = make_error(ApiError::MICROSERVICE_ERROR, std::string("bad reply from python worker: ") + e.what());
      for (auto& o : res) o = Outcome::fail(err);
    }
  }

  py::object adapter_;
  uint32_t builtin_;
  PyUnitOptions opts_;
  uint32_t dense_mask_ = 0;
  bool has_call_json_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> queue_;
  bool running_ = false, stopped_ = false;
  std::vector<std::thread> threads_;
  std::unique_ptr<std::atomic<bool>[]> dead_;
  mutable std::mutex stats_mu_;
  Stats stats_;
};

}  // namespace sca
