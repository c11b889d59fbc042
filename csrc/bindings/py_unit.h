// Python-implemented predictive unit.
//
// Wraps a Python adapter object (seldon_core_amd.serving.adapter.PythonUnit)
// that applies the reference wrapper's dispatch precedence
// (python/seldon_core/seldon_methods.py:17-302: *_rest / *_grpc hooks ->
// *_raw -> high level predict(X, names, meta)) to a user component.  Messages
// cross the boundary as SeldonMessage JSON text so the user sees exactly the
// REST payloads the reference wrapper would have given it.
#pragma once

#include <pybind11/pybind11.h>

#include "../core/engine.h"

namespace sca {

namespace py = pybind11;

class PyUnit : public Unit {
 public:
  PyUnit(py::object adapter, uint32_t builtin_mask) : adapter_(std::move(adapter)), builtin_(builtin_mask) {}
  ~PyUnit() override {
    py::gil_scoped_acquire g;
    adapter_ = py::object();
  }
  uint32_t builtin_methods() const override { return builtin_; }
  std::string kind() const override { return "python"; }

  void transform_input(const CallCtx& c, MsgPtr in, Done k) override { call1("transform_input", c, in, std::move(k)); }
  void predict(const CallCtx& c, MsgPtr in, Done k) override { call1("predict", c, in, std::move(k)); }
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override { call1("transform_output", c, in, std::move(k)); }
  void route(const CallCtx& c, MsgPtr in, Done k) override { call1("route", c, in, std::move(k)); }
  void aggregate(const CallCtx& c, std::vector<MsgPtr> in, Done k) override {
    std::vector<const SeldonMessage*> v;
    for (auto& m : in) v.push_back(m.get());
    std::string text;
    message_list_to_json(v, text);
    invoke("aggregate", c, text, std::move(k));
  }
  void send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) override {
    std::string text;
    feedback_to_json(*fb, text);
    invoke("send_feedback", c, text, [k](Outcome o) { k(o.err); });
  }
  bool ready() const override {
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

 private:
  void call1(const char* method, const CallCtx& c, const MsgPtr& in, Done k) {
    std::string text;
    text.reserve(256);
    message_to_json(*in, text);
    invoke(method, c, text, std::move(k));
  }
  void invoke(const char* method, const CallCtx& c, const std::string& text, Done k) {
    std::string out;
    std::string err;
    bool failed = false;
    int code = 0;
    {
      py::gil_scoped_acquire g;
      try {
        py::object r = adapter_.attr(method)(text, c.node ? c.node->name : std::string());
        if (r.is_none()) out.clear();
        else out = r.cast<std::string>();
      } catch (py::error_already_set& e) {
        failed = true;
        err = e.what();
        if (e.value() && py::hasattr(e.value(), "status_code")) {
          try { code = e.value().attr("status_code").cast<int>(); } catch (...) {}
        }
        e.restore();
        PyErr_Clear();
      }
    }
    (void)code;
    if (failed) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, err)));
      return;
    }
    if (out.empty()) {
      k(Outcome::ok(nullptr));
      return;
    }
    auto m = std::make_shared<SeldonMessage>();
    try {
      message_from_json(parse_json(out), *m);
    } catch (const std::exception& e) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, std::string("bad response from python unit: ") + e.what())));
      return;
    }
    k(Outcome::ok(std::move(m)));
  }

  py::object adapter_;
  uint32_t builtin_;
};

}  // namespace sca
