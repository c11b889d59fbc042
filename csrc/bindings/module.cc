// pybind11 module `seldon_core_amd._C`: the native engine, front ends, GPU
// units and raw kernel launchers.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <future>

#include "../core/cpuprof.h"
#include "../core/engine.h"
#include "../core/pool_executor.h"
#include "../core/json.h"
#include "../core/message.h"
#include "../core/msglog.h"
#include "../gpu/batcher.h"
#include "../gpu/graph.h"
#include "../gpu/lstm_model.h"
#include "../gpu/maha_device.h"
#include "../gpu/mlp_model.h"
#include "../gpu/replica.h"
#include "../gpu/models.h"
#include "../gpu/router.h"
#include "../kernels/kernels.h"
#include "../parallel/fabric.h"
#include "../parallel/mesh.h"
#include "../server/grpc_server.h"
#include "../server/http_server.h"
#include "../server/remote_unit.h"
#include "py_unit.h"

namespace py = pybind11;
using namespace sca;

namespace {

template <class T>
std::vector<T> to_vec(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
  return std::vector<T>(a.data(), a.data() + a.size());
}

std::pair<int, std::string> render(const Outcome& o) {
  if (o.err) return {o.err->http_status, error_to_json(*o.err)};
  std::string out;
  if (o.msg) message_to_json(*o.msg, out);
  else out = "{}";
  return {200, out};
}

Outcome wait_outcome(const std::function<void(Done)>& start) {
  std::promise<Outcome> p;
  auto f = p.get_future();
  {
    py::gil_scoped_release nogil;
    start([&p](Outcome o) { p.set_value(std::move(o)); });
    return f.get();
  }
}

gpu::BatcherOptions batcher_opts(int device, int max_batch, int max_wait_us, int slots, bool zero_copy,
                                 size_t zero_copy_max_bytes, bool spin, bool cpu_batching = false,
                                 int fail_threshold = 3, int cooldown_ms = 2000, int hang_timeout_ms = 10000) {
  gpu::BatcherOptions o;
  o.fail_threshold = fail_threshold;
  o.cooldown_ms = cooldown_ms;
  o.hang_timeout_ms = hang_timeout_ms;
  o.device = device;
  o.max_batch = max_batch;
  o.max_wait_us = max_wait_us;
  o.slots = slots;
  o.zero_copy = zero_copy;
  o.zero_copy_max_bytes = zero_copy_max_bytes;
  o.spin_wait = spin;
  o.cpu_batching = cpu_batching;
  return o;
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T> T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native Seldon-compatible inference graph engine (native core)";
  m.def("version", [] { return std::string("0.1.0"); });
  m.def("gpu_device_count", [] { return gpu::device_count(); });
  m.def("can_access_peer", [](int dev, int peer) {
    // hipDeviceCanAccessPeer: whether `dev` can map `peer`'s HBM over xGMI
    // (recorded per graph placement by bench.py).
    if (dev == peer) return true;
    int ok = 0;
    if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess) return false;
    return ok != 0;
  });

  // ------------------------------------------------------------- codecs
  m.def("cpu_profile_start", [](int hz, int depth) { return prof::start(hz, size_t(1) << 20, depth); },
        py::arg("hz") = 997, py::arg("depth") = 1,
        "Start sampling this process's CPU time (SIGPROF per thread at `hz` per CPU-second).");
  m.def("cpu_profile_stop", [] {
    py::list out;
    for (const auto& s : prof::stop().samples) {
      py::list frames;
      for (const auto& f : s.frames) frames.append(py::make_tuple(f.module, f.offset));
      out.append(py::make_tuple(frames, s.count));
    }
    return out;
  }, "Stop sampling: [([(module, offset), ...], samples)], most frequent first.");
  m.def("json_roundtrip", [](const std::string& text) {
    SeldonMessage msg;
    message_from_json(parse_json(text), msg);
    std::string out;
    message_to_json(msg, out);
    return out;
  });
  m.def("json_fast_roundtrip", [](const std::string& text) -> py::object {
    SeldonMessage msg;
    if (!fast_dense_message(text, msg)) return py::none();
    std::string js, pb;
    message_to_json(msg, js);
    message_to_pb(msg, pb);
    return py::make_tuple(js, py::bytes(pb));
  }, "The REST fast path (dense ndarray requests): (json, protobuf) re-encodings, or None when it declines.");
  m.def("json_to_pb", [](const std::string& text) {
    SeldonMessage msg;
    message_from_json(parse_json(text), msg);
    std::string out;
    message_to_pb(msg, out);
    return py::bytes(out);
  });
  m.def("pb_to_json", [](const py::bytes& b) {
    SeldonMessage msg;
    if (!message_from_pb(std::string(b), msg)) throw std::runtime_error("invalid SeldonMessage protobuf");
    std::string out;
    message_to_json(msg, out);
    return out;
  });
  m.def("feedback_json_to_pb", [](const std::string& text) {
    Feedback f;
    feedback_from_json(parse_json(text), f);
    std::string out;
    feedback_to_pb(f, out);
    return py::bytes(out);
  });
  m.def("feedback_pb_to_json", [](const py::bytes& b) {
    Feedback f;
    if (!feedback_from_pb(std::string(b), f)) throw std::runtime_error("invalid Feedback protobuf");
    std::string out;
    feedback_to_json(f, out);
    return out;
  });
  m.def("list_json_to_pb", [](const std::string& text) {
    std::vector<SeldonMessage> v;
    message_list_from_json(parse_json(text), v);
    std::vector<const SeldonMessage*> p;
    for (auto& x : v) p.push_back(&x);
    std::string out;
    message_list_to_pb(p, out);
    return py::bytes(out);
  });
  m.def("list_pb_to_json", [](const py::bytes& b) {
    std::vector<SeldonMessage> v;
    if (!message_list_from_pb(std::string(b), v)) throw std::runtime_error("invalid SeldonMessageList protobuf");
    std::vector<const SeldonMessage*> p;
    for (auto& x : v) p.push_back(&x);
    std::string out;
    message_list_to_json(p, out);
    return out;
  });
  m.def("dense_of", [](const std::string& text) {
    SeldonMessage msg;
    message_from_json(parse_json(text), msg);
    std::vector<int64_t> shape;
    std::vector<double> vals;
    std::string err;
    if (!msg.data.dense(shape, vals, &err)) throw std::runtime_error(err);
    return py::make_tuple(shape, vals);
  });
  m.def("new_puid", [] {
    Engine e(default_predictor_spec(), EngineOptions());
    return e.new_puid();
  });
  m.def("parse_spec", [](const std::string& text, const std::string& predictor) {
    PredictorSpecC s = parse_predictor_spec(parse_json(text), predictor);
    py::dict d;
    d["name"] = s.name;
    d["graph"] = s.graph.name;
    d["replicas"] = s.replicas;
    return d;
  }, py::arg("text"), py::arg("predictor") = "");

  // ------------------------------------------------------------- models
  py::class_<gpu::RowModel, std::shared_ptr<gpu::RowModel>>(m, "RowModel")
      .def_property_readonly("name", &gpu::RowModel::name)
      .def_property_readonly("in_cols", &gpu::RowModel::in_cols)
      .def("out_cols", &gpu::RowModel::out_cols)
      .def("set_class_names", &gpu::RowModel::set_class_names)
      .def("class_names", &gpu::RowModel::class_names)
      .def_property("flat_output", &gpu::RowModel::flat_output, &gpu::RowModel::set_flat_output)
      .def_property("input_names", &gpu::RowModel::input_names, &gpu::RowModel::set_input_names)
      .def("clone", &gpu::RowModel::clone)
      .def("clone_on", [](const gpu::RowModel& mdl, int device) {
        auto* g = dynamic_cast<const gpu::GraphModel*>(&mdl);
        return g ? g->clone_on(device) : mdl.clone();
      })
      .def("run_cpu", [](const gpu::RowModel& mdl, py::array_t<double, py::array::c_style | py::array::forcecast> X) {
        if (X.ndim() != 2) throw std::runtime_error("X must be 2-D");
        const int rows = int(X.shape(0)), cols = int(X.shape(1));
        const int oc = mdl.out_cols(cols);
        py::array_t<double> out({rows, oc});
        const double* x = X.data();
        double* y = out.mutable_data();
        {
          py::gil_scoped_release nogil;  // concurrent callers (e.g. several batches over one fabric)
          mdl.run_cpu(x, rows, cols, y);
        }
        return out;
      });
  m.def("linear_model",
        [](py::array_t<double, py::array::c_style | py::array::forcecast> W,
           py::array_t<double, py::array::c_style | py::array::forcecast> b, int act) {
          if (W.ndim() != 2) throw std::runtime_error("W must be [C, K]");
          return std::static_pointer_cast<gpu::RowModel>(std::make_shared<gpu::LinearModel>(
              to_vec(W), to_vec(b), int(W.shape(0)), int(W.shape(1)), act));
        },
        py::arg("W"), py::arg("b"), py::arg("act"));
  // stages: list of dicts {kind: "model"|"mean", model?, device, inputs: [int], node}
  m.def("graph_model", [](py::list stages, int in_cols, int split_streams) {
    std::vector<gpu::GraphStage> st;
    for (auto h : stages) {
      py::dict d = h.cast<py::dict>();
      gpu::GraphStage s;
      const std::string kind = d["kind"].cast<std::string>();
      s.kind = kind == "mean" ? gpu::GraphStage::kMean : gpu::GraphStage::kModel;
      if (s.kind == gpu::GraphStage::kModel) s.model = d["model"].cast<std::shared_ptr<gpu::RowModel>>();
      s.device = d.contains("device") ? d["device"].cast<int>() : 0;
      s.inputs = d["inputs"].cast<std::vector<int>>();
      s.node = d.contains("node") ? d["node"].cast<std::string>() : std::string();
      st.push_back(std::move(s));
    }
    auto g = std::make_shared<gpu::GraphModel>(std::move(st), in_cols);
    if (split_streams) g->set_split(split_streams);
    return std::static_pointer_cast<gpu::RowModel>(g);
  }, py::arg("stages"), py::arg("in_cols") = 0, py::arg("split_streams") = 0);
  m.def("graph_devices", [](std::shared_ptr<gpu::RowModel> m) {
    auto g = std::dynamic_pointer_cast<gpu::GraphModel>(m);
    if (!g) throw std::runtime_error("not a graph model");
    return g->devices();
  });
  m.def("graph_info", [](std::shared_ptr<gpu::RowModel> m) {
    auto g = std::dynamic_pointer_cast<gpu::GraphModel>(m);
    if (!g) throw std::runtime_error("not a graph model");
    py::dict d;
    d["devices"] = g->devices();
    d["split"] = g->split();
    d["split_mode"] = g->split_mode();
    d["peer_direct"] = g->peer_direct();
    d["stages"] = int(g->stages().size());
    d["fused"] = g->fused();  // one linear_graph kernel per batch
    py::dict pc;
    for (const auto& c : g->peer_canary_results())
      pc[py::str(std::to_string(c.producer) + "->" + std::to_string(c.consumer))] = c.ok;
    d["peer_canary"] = pc;  // producer -> consumer: a consumer kernel read the producer's HBM correctly
    return d;
  });
  auto to_layers = [](py::list ls) {
    std::vector<gpu::DenseLayer> out;
    for (auto h : ls) {
      py::dict d = h.cast<py::dict>();
      auto W = d["W"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      auto b = d["b"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      if (W.ndim() != 2) throw std::runtime_error("layer W must be [out, in]");
      gpu::DenseLayer L;
      L.N = int(W.shape(0));
      L.K = int(W.shape(1));
      L.W = to_vec(W);
      L.b = to_vec(b);
      L.act = d.contains("act") ? d["act"].cast<int>() : 0;
      out.push_back(std::move(L));
    }
    return out;
  };
  auto prec = [](const std::string& p) {
    if (p == "fp32" || p == "float32") return 0;
    if (p == "bf16" || p == "bfloat16") return 1;
    throw std::runtime_error("precision must be 'fp32' or 'bf16'");
  };
  m.def("mlp_model", [to_layers, prec](py::list layers, int out_mode, const std::string& precision) {
    auto mm = std::make_shared<gpu::MlpModel>(to_layers(layers), out_mode);
    if (prec(precision)) mm->set_precision(prec(precision));
    return std::static_pointer_cast<gpu::RowModel>(mm);
  }, py::arg("layers"), py::arg("out_mode") = 0, py::arg("precision") = "fp32");
  m.def("mlp_precision", [](std::shared_ptr<gpu::RowModel> m) {
    auto p = std::dynamic_pointer_cast<gpu::MlpModel>(m);
    if (!p) throw std::runtime_error("not an MLP model");
    return std::string(p->precision() ? "bf16" : "fp32");
  });
  m.def("mlp_layerwise", [](std::shared_ptr<gpu::RowModel> m, int rows) {
    auto p = std::dynamic_pointer_cast<gpu::MlpModel>(m);
    if (!p) throw std::runtime_error("not an MLP model");
    return p->layerwise(rows);
  });
  m.def("mlp_workspace_bytes", [](std::shared_ptr<gpu::RowModel> m, int rows) {
    return m->workspace_bytes(rows, m->in_cols());
  });
  m.def("vae_model", [to_layers, prec](py::list encoder, int latent, py::list decoder, int samples, uint64_t seed,
                                       const std::string& precision) {
    auto mm = gpu::MlpModel::vae(to_layers(encoder), latent, to_layers(decoder), samples, seed);
    if (prec(precision)) mm->set_precision(prec(precision));
    return std::static_pointer_cast<gpu::RowModel>(mm);
  }, py::arg("encoder"), py::arg("latent"), py::arg("decoder"), py::arg("samples") = 10, py::arg("seed") = 0,
     py::arg("precision") = "fp32");
  auto to_lstm = [](py::handle h) {
    py::dict d = h.cast<py::dict>();
    auto Wi = d["W_ih"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
    auto Wh = d["W_hh"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
    auto b = d["b"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
    if (Wi.ndim() != 2 || Wh.ndim() != 2) throw std::runtime_error("LSTM W_ih / W_hh must be 2-D [4H, in] / [4H, H]");
    gpu::LstmWeights w;
    w.H = int(Wh.shape(1));
    w.in = int(Wi.shape(1));
    w.W_ih = to_vec(Wi);
    w.W_hh = to_vec(Wh);
    w.b = to_vec(b);
    return w;
  };
  m.def("lstm_seq2seq_model",
        [to_lstm](int T, int F, py::list enc, py::list dec, py::array_t<float, py::array::c_style | py::array::forcecast> W,
                  py::array_t<float, py::array::c_style | py::array::forcecast> b, int out_act) {
          std::vector<std::pair<gpu::LstmWeights, gpu::LstmWeights>> e;
          for (auto h : enc) {
            py::sequence pair = h.cast<py::sequence>();
            if (pair.size() != 2) throw std::runtime_error("encoder layer = (forward, backward)");
            e.emplace_back(to_lstm(pair[0]), to_lstm(pair[1]));
          }
          std::vector<gpu::LstmWeights> d;
          for (auto h : dec) d.push_back(to_lstm(h));
          return std::static_pointer_cast<gpu::RowModel>(
              std::make_shared<gpu::LstmSeqModel>(T, F, std::move(e), std::move(d), to_vec(W), to_vec(b), out_act));
        },
        py::arg("T"), py::arg("F"), py::arg("encoder"), py::arg("decoder"), py::arg("dense_W"), py::arg("dense_b"),
        py::arg("out_act") = 1);
  m.def("lstm_program", [](std::shared_ptr<gpu::RowModel> m) {
    auto p = std::dynamic_pointer_cast<gpu::LstmSeqModel>(m);
    if (!p) throw std::runtime_error("not an LSTM model");
    const auto& g = p->program();
    py::dict d;
    d["w_lds"] = g.w_lds;
    d["lds_bytes"] = g.lds_floats * 4;
    d["workspace_floats_per_wg"] = g.seq_ws_floats;
    const auto& v = p->valu_program(1);
    d["valu_ok"] = v.ok;
    d["valu_kpl"] = v.KPL;
    d["valu_threads"] = v.threads;
    d["valu_lds_bytes_r1"] = v.lds_floats * 4;
    d["valu_lds_bytes_r4"] = p->valu_program(4).lds_floats * 4;
    return d;
  });
  m.def("lstm_path", [](std::shared_ptr<gpu::RowModel> m, int rows) {
    auto p = std::dynamic_pointer_cast<gpu::LstmSeqModel>(m);
    if (!p) throw std::runtime_error("not an LSTM model");
    return p->path_for(rows);
  }, "Kernel a batch of `rows` sequences runs: 'valu' (small batches) or 'mfma'");
  py::class_<gpu::MahalanobisDevice, std::shared_ptr<gpu::MahalanobisDevice>>(m, "MahalanobisDevice")
      .def(py::init<int, int, double, double, double, double, int>(), py::arg("p"), py::arg("k"),
           py::arg("n_stdev") = 3.0, py::arg("start_clip") = 50.0, py::arg("max_n") = -1.0, py::arg("eps") = 1e-8,
           py::arg("device") = 0)
      .def("step", [](gpu::MahalanobisDevice& d, py::array_t<double, py::array::c_style | py::array::forcecast> X) {
        if (X.ndim() != 2 || X.shape(1) != d.p()) throw std::runtime_error("X must be [rows, p]");
        std::vector<double> s;
        {
          py::gil_scoped_release nogil;
          s = d.step(X.data(), int(X.shape(0)));
        }
        return py::array_t<double>(py::ssize_t(s.size()), s.data());
      })
      .def("step_seq", [](gpu::MahalanobisDevice& d, py::array_t<double, py::array::c_style | py::array::forcecast> X) {
        if (X.ndim() != 2 || X.shape(1) != d.p()) throw std::runtime_error("X must be [rows, p]");
        std::vector<double> s;
        int64_t seq = -1;
        {
          py::gil_scoped_release nogil;
          s = d.step(X.data(), int(X.shape(0)), &seq);
        }
        return py::make_tuple(py::array_t<double>(py::ssize_t(s.size()), s.data()), seq);
      }, "step() that also returns where the state applied this request's first row (launch order over every "
         "view of the state): concurrent callers can be replayed in the device's order")
      .def("state", [](const gpu::MahalanobisDevice& d) {
        auto s = d.state();
        return py::array_t<double>(py::ssize_t(s.size()), s.data());
      })
      .def("set_state", [](gpu::MahalanobisDevice& d, std::vector<double> s) { d.set_state(s); })
      .def("lock_state", [](gpu::MahalanobisDevice& d) {
        py::gil_scoped_release nogil;  // a native step may hold it briefly
        d.lock_state();
      })
      .def("unlock_state", &gpu::MahalanobisDevice::unlock_state)
      .def("solver_stats", [](const gpu::MahalanobisDevice& d) {
        const auto t = d.solver_stats();
        py::dict r;
        if (t.size() == 17) {
          r["steps"] = t[1];
          r["rank1_steps"] = t[13];     // eigen-tracking (secular-equation) steps
          r["rank1_fallbacks"] = t[14];  // of which re-solved by Jacobi (cache or residual check failed)
          r["jacobi_solves"] = t[16];
          r["jacobi_sweeps_per_solve"] = t[16] > 0 ? t[15] / t[16] : 0.0;
          // s_memtime cycles / s_memrealtime (100 MHz) ticks over the eigen phase
          r["eigen_clock_mhz"] = t[2] > 0 ? t[0] / (t[2] * 0.01) : 0.0;
          static const char* names[10] = {"clip", "cov", "eigen.vectors", "eigen", "proj", "sm", "update",
                                          "eigen.tridiag", "eigen.eigenvalues", "eigen.back_transform"};
          py::dict ph;
          for (int i = 0; i < 10; ++i) ph[names[i]] = t[1] > 0 ? t[3 + i] / t[1] : 0.0;
          r["phase_us_per_step"] = ph;
        }
        return r;
      })
      .def("predict_view", [](const gpu::MahalanobisDevice& d, double threshold) {
        return std::static_pointer_cast<gpu::RowModel>(d.predict_view(threshold));
      }, py::arg("threshold"), "RowModel of predictions (score > threshold) over this detector's state")
      .def("batches", [](const gpu::MahalanobisDevice& d) {
        const auto st = d.stats();
        py::dict r;
        r["batches"] = st.batches;
        r["requests"] = st.requests;
        r["rows"] = st.rows;
        return r;
      })
      .def_property_readonly("p", &gpu::MahalanobisDevice::p)
      .def_property_readonly("k", &gpu::MahalanobisDevice::k);
  m.def("mahalanobis_model", [](int p, int k, double n_stdev, double start_clip, double max_n, double eps, int out_mode,
                                double threshold) {
    return std::static_pointer_cast<gpu::RowModel>(
        std::make_shared<gpu::MahalanobisModel>(p, k, n_stdev, start_clip, max_n, eps, out_mode, threshold));
  }, py::arg("p"), py::arg("k"), py::arg("n_stdev") = 3.0, py::arg("start_clip") = 50.0, py::arg("max_n") = -1.0,
        py::arg("eps") = 1e-8, py::arg("out_mode") = 1, py::arg("threshold") = 25.0,
        "Segmented, state-chained Mahalanobis detector RowModel (out_mode 0 scores, 1 predictions)");
  m.def("mahalanobis_state", [](std::shared_ptr<gpu::RowModel> rm) {
    auto mm = std::dynamic_pointer_cast<gpu::MahalanobisModel>(rm);
    if (!mm) throw std::runtime_error("not a Mahalanobis model");
    auto s = mm->state();
    return py::array_t<double>(py::ssize_t(s.size()), s.data());
  });
  m.def("minmax_model", [] { return std::static_pointer_cast<gpu::RowModel>(std::make_shared<gpu::MinMaxModel>()); });
  m.def("mean_sigmoid_model", [](double thr) {
    return std::static_pointer_cast<gpu::RowModel>(std::make_shared<gpu::MeanSigmoidModel>(thr));
  });
  m.def("tree_model",
        [](py::dict d) {
          gpu::TreeEnsembleSpec s;
          s.n_trees = d["n_trees"].cast<int>();
          s.n_features = d["n_features"].cast<int>();
          s.groups = d.contains("groups") ? d["groups"].cast<int>() : 1;
          s.out_cols = d.contains("out_cols") ? d["out_cols"].cast<int>() : s.groups;
          s.transform = d.contains("transform") ? d["transform"].cast<int>() : 0;
          s.cmp_le = d.contains("cmp_le") ? d["cmp_le"].cast<int>() : 0;
          s.scale = d.contains("scale") ? d["scale"].cast<float>() : 1.f;
          if (d.contains("base_margin")) s.base_margin = d["base_margin"].cast<std::vector<float>>();
          if (d.contains("tree_group")) s.tree_group = d["tree_group"].cast<std::vector<int>>();
          s.depth = d.contains("depth") ? d["depth"].cast<int>() : 0;
          if (s.depth > 0) {
            s.thr = to_vec(d["thr"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>());
            s.feat = to_vec(d["feat"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>());
            s.leaves = to_vec(d["leaves"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>());
          } else {
            auto thr = to_vec(d["thr"].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>());
            auto feat = to_vec(d["feat"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>());
            auto left = to_vec(d["left"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>());
            auto right = to_vec(d["right"].cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>());
            if (thr.size() != feat.size() || thr.size() != left.size() || thr.size() != right.size())
              throw std::runtime_error("sparse tree arrays must have equal length");
            s.nodes.resize(thr.size());
            for (size_t i = 0; i < thr.size(); ++i) s.nodes[i] = kern::SparseNode{thr[i], feat[i], left[i], right[i]};
            s.tree_root = d["tree_root"].cast<std::vector<int>>();
          }
          auto tm = std::make_shared<gpu::TreeEnsembleModel>(std::move(s));
          if (d.contains("fused_reduce")) tm->set_fused_reduce(d["fused_reduce"].cast<bool>());
          if (d.contains("whole_max_rows")) tm->set_whole_max_rows(d["whole_max_rows"].cast<int>());
          return std::static_pointer_cast<gpu::RowModel>(tm);
        });

  py::class_<Unit, std::shared_ptr<Unit>>(m, "Unit")
      .def_property_readonly("kind", &Unit::kind)
      .def("snapshot", [](const Unit& u) { return py::bytes(u.snapshot()); })
      .def("restore", [](Unit& u, const py::bytes& b) { u.restore(std::string(b)); });

  py::class_<PyUnit, Unit, std::shared_ptr<PyUnit>>(m, "PyUnit")
      .def("stop", &PyUnit::stop)
      .def("stats", [](const PyUnit& u) {
        auto s = u.stats();
        py::dict d;
        d["jobs"] = s.jobs;
        d["calls"] = s.calls;
        d["rows"] = s.rows;
        d["batched_calls"] = s.batched_calls;
        d["pool_calls"] = s.pool_calls;
        d["workers"] = u.options().worker_fds.size();
        d["alive_workers"] = u.alive_workers();
        d["batch_rows"] = u.options().batch_rows;
        return d;
      });

  py::class_<gpu::BatchedUnit, Unit, std::shared_ptr<gpu::BatchedUnit>>(m, "BatchedUnit")
      .def(py::init([](std::shared_ptr<gpu::RowModel> model, int device, int max_batch, int max_wait_us, int slots,
                       bool zero_copy, size_t zc_bytes, bool spin, bool cpu_batching, int fail_threshold,
                       int cooldown_ms, int hang_timeout_ms) {
             return std::make_shared<gpu::BatchedUnit>(
                 model, batcher_opts(device, max_batch, max_wait_us, slots, zero_copy, zc_bytes, spin, cpu_batching,
                                     fail_threshold, cooldown_ms, hang_timeout_ms));
           }),
           py::arg("model"), py::arg("device") = 0, py::arg("max_batch") = 1024, py::arg("max_wait_us") = 0,
           py::arg("slots") = 4, py::arg("zero_copy") = true, py::arg("zero_copy_max_bytes") = 256 << 10,
           py::arg("spin_wait") = true, py::arg("cpu_batching") = false, py::arg("fail_threshold") = 3,
           py::arg("cooldown_ms") = 2000, py::arg("hang_timeout_ms") = 10000)
      .def("health", [](const gpu::BatchedUnit& u) {
        const auto h = u.health();
        py::dict d;
        d["healthy"] = h.healthy;
        d["consecutive_failures"] = h.consecutive_failures;
        d["failed_batches"] = h.failed_batches;
        d["hangs"] = h.hangs;
        d["trips"] = h.trips;
        d["injected"] = h.injected;
        return d;
      })
      .def("inject_fault", [](gpu::BatchedUnit& u, int64_t fail_after, int64_t fail_count, int hang_ms) {
             gpu::FaultSpec f;
             f.fail_after = fail_after;
             f.fail_count = fail_count;
             f.hang_ms = hang_ms;
             u.inject_fault(f);
           },
           py::arg("fail_after") = -1, py::arg("fail_count") = -1, py::arg("hang_ms") = 0)
      .def_property_readonly("ready", &gpu::BatchedUnit::ready)
      .def_property_readonly("model", &gpu::BatchedUnit::model)
      .def("run", [](gpu::BatchedUnit& u, py::array_t<double, py::array::c_style | py::array::forcecast> X) {
        if (X.ndim() != 2) throw std::runtime_error("X must be 2-D");
        const int rows = int(X.shape(0)), cols = int(X.shape(1));
        std::vector<double> out;
        {
          py::gil_scoped_release nogil;  // X (held by this frame) is read in place: no host copy
          out = u.run_ptr(X.data(), rows, cols);
        }
        const int oc = int(out.size() / size_t(rows));
        py::array_t<double> r({rows, oc});
        std::copy(out.begin(), out.end(), r.mutable_data());
        return r;
      })
      .def("stats", [](const gpu::BatchedUnit& u) {
        auto s = u.stats();
        py::dict d;
        d["batches"] = s.batches;
        d["rows"] = s.rows;
        d["requests"] = s.requests;
        d["max_rows"] = s.max_rows;
        d["gpu_busy_s"] = s.gpu_busy_s;
        d["launch_cpu_s"] = s.launch_cpu_s;
        d["complete_cpu_s"] = s.complete_cpu_s;
        d["device"] = u.options().device;
        return d;
      })
      .def("reset_stats", &gpu::BatchedUnit::reset_stats)
      .def("stop", [](gpu::BatchedUnit& u) {
        py::gil_scoped_release nogil;
        u.stop();
      });

  py::class_<gpu::ReplicaUnit, Unit, std::shared_ptr<gpu::ReplicaUnit>>(m, "ReplicaUnit")
      .def(py::init([](std::vector<std::shared_ptr<gpu::BatchedUnit>> reps, int max_retries) {
             return std::make_shared<gpu::ReplicaUnit>(std::move(reps), max_retries);
           }),
           py::arg("replicas"), py::arg("max_retries") = 1)
      .def_property_readonly("replicas", &gpu::ReplicaUnit::replicas)
      .def_property_readonly("ready", &gpu::ReplicaUnit::ready)
      .def_property_readonly("retries", &gpu::ReplicaUnit::retries)
      .def("requests_per_replica", &gpu::ReplicaUnit::requests_per_replica)
      .def("stats", [](const gpu::ReplicaUnit& u) {
        py::dict d;
        uint64_t b = 0, r = 0, q = 0, mx = 0;
        double busy = 0;
        for (const auto& rep : u.replicas()) {
          auto s = rep->stats();
          b += s.batches; r += s.rows; q += s.requests; busy += s.gpu_busy_s;
          mx = std::max<uint64_t>(mx, s.max_rows);
        }
        d["batches"] = b;
        d["rows"] = r;
        d["requests"] = q;
        d["max_rows"] = mx;
        d["gpu_busy_s"] = busy;
        d["per_replica"] = u.requests_per_replica();
        py::list per_dev;
        for (const auto& rep : u.replicas()) {
          auto s = rep->stats();
          py::dict e;
          e["device"] = rep->options().device;
          e["batches"] = s.batches;
          e["rows"] = s.rows;
          per_dev.append(e);
        }
        d["per_device"] = per_dev;
        return d;
      })
      .def("reset_stats", [](gpu::ReplicaUnit& u) {
        for (auto& rep : u.replicas()) rep->reset_stats();
      })
      .def("stop", [](gpu::ReplicaUnit& u) {
        py::gil_scoped_release nogil;
        u.stop();
      });

  // ------------------------------------------------------- RCCL fabric
  m.def("rccl_unique_ids", [](int world, int per_link) { return py::bytes(par::rccl_unique_ids(world, per_link)); },
        py::arg("world"), py::arg("per_link") = 2);
  py::class_<par::LoopbackHub, std::shared_ptr<par::LoopbackHub>>(m, "LoopbackHub")
      .def(py::init<int>(), py::arg("device"))
      .def_property_readonly("device", &par::LoopbackHub::device)
      .def_property_readonly("messages", &par::LoopbackHub::messages)
      .def_property_readonly("staging_buffers", &par::LoopbackHub::staging_buffers)
      .def_property_readonly("matched_immediately", &par::LoopbackHub::matched_immediately);
  py::class_<par::Fabric, std::shared_ptr<par::Fabric>>(m, "Fabric")
      .def(py::init([](int rank, int world, const py::bytes& uid, int device, std::vector<int> ctrl_fds,
                       std::shared_ptr<par::LoopbackHub> hub, int comms_per_link) {
             std::string id(uid);
             py::gil_scoped_release nogil;  // collective: blocks until every rank joins
             return std::make_shared<par::Fabric>(rank, world, id, device, std::move(ctrl_fds), std::move(hub),
                                                  comms_per_link);
           }),
           py::arg("rank"), py::arg("world"), py::arg("unique_id"), py::arg("device"), py::arg("ctrl_fds"),
           py::arg("hub") = nullptr, py::arg("comms_per_link") = 2)
      .def_property_readonly("gpu", &par::Fabric::gpu)
      .def_property_readonly("transport", &par::Fabric::transport)
      .def_property_readonly("rank", &par::Fabric::rank)
      .def_property_readonly("world", &par::Fabric::world)
      .def_property_readonly("device", &par::Fabric::device)
      .def("stop_peers", [](par::Fabric& f) {
        py::gil_scoped_release nogil;
        par::stop_peers(f);
      })
      .def("close", [](par::Fabric& f) {
        py::gil_scoped_release nogil;
        f.close();
      });
  m.def("peer_row_model",
        [](std::shared_ptr<par::Fabric> f, std::vector<int> peers, int model_id, int in_cols, int out_cols,
           std::vector<std::string> names, bool flat) {
          auto mdl = std::make_shared<par::PeerRowModel>(std::move(f), std::move(peers), model_id, in_cols, out_cols);
          mdl->set_class_names(std::move(names));
          mdl->set_flat_output(flat);
          return std::static_pointer_cast<gpu::RowModel>(mdl);
        },
        py::arg("fabric"), py::arg("peers"), py::arg("model_id"), py::arg("in_cols"), py::arg("out_cols"),
        py::arg("class_names") = std::vector<std::string>(), py::arg("flat_output") = false);
  py::class_<par::PeerServer, std::shared_ptr<par::PeerServer>>(m, "PeerServer")
      .def(py::init<std::shared_ptr<par::Fabric>>())
      .def("add_model", &par::PeerServer::add_model)
      .def("start", &par::PeerServer::start)
      .def("join", [](par::PeerServer& s) {
        py::gil_scoped_release nogil;
        s.join();
      })
      .def_property_readonly("batches", &par::PeerServer::batches)
      .def_property_readonly("rows", &par::PeerServer::rows)
      .def_property_readonly("host_syncs", &par::PeerServer::host_syncs)
      .def_property_readonly("max_inflight", &par::PeerServer::max_inflight)
      .def_property_readonly("slots", &par::PeerServer::slots)
      .def("error", &par::PeerServer::error);

  // ------------------------------------------------- mesh (ipc / shm)
  py::class_<par::Mesh, std::shared_ptr<par::Mesh>>(m, "Mesh")
      .def(py::init<int, int, int, std::vector<int>, int>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("ctrl_fds"), py::arg("slots") = 4)
      .def_property_readonly("rank", &par::Mesh::rank)
      .def_property_readonly("world", &par::Mesh::world)
      .def_property_readonly("device", &par::Mesh::device)
      .def_property_readonly("gpu", &par::Mesh::gpu)
      .def_property_readonly("slots", &par::Mesh::slots)
      .def_property_readonly("transport", &par::Mesh::transport)
      .def("add_program",
           [](par::Mesh& me, const py::dict& d) {
             par::MeshProgram p;
             p.max_rows = d["max_rows"].cast<int>();
             p.in_cols = d["in_cols"].cast<int>();
             for (auto item : d["stages"].cast<py::list>()) {
               auto s = item.cast<py::dict>();
               par::MeshStage st;
               st.rank = s["rank"].cast<int>();
               st.kind = s["kind"].cast<int>();
               st.inputs = s["inputs"].cast<std::vector<int>>();
               st.in_cols = s["in_cols"].cast<int>();
               st.out_cols = s["out_cols"].cast<int>();
               st.node = s.contains("node") ? s["node"].cast<std::string>() : std::string();
               p.stages.push_back(std::move(st));
             }
             return me.add_program(std::move(p));
           })
      .def("probe_prepare", [](par::Mesh& me) { return py::bytes(me.probe_prepare()); })
      .def("probe_connect",
           [](par::Mesh& me, const std::vector<py::bytes>& blobs) {
             std::vector<std::string> b;
             for (auto& x : blobs) b.push_back(std::string(x));
             py::gil_scoped_release nogil;
             return me.probe_connect(b);
           })
      .def("probe_error", &par::Mesh::probe_error)
      .def("probe_finish", &par::Mesh::probe_finish)
      .def("set_peer_ok", &par::Mesh::set_peer_ok)
      .def("edge_transports", &par::Mesh::edge_transports)
      .def("set_model", &par::Mesh::set_model)
      .def("set_host_fn",
           [](par::Mesh& me, int prog, int stage, py::object fn) {
             // A Python component on this rank: called with the GIL from the
             // program's thread, on a copy of the rows.
             auto f = std::make_shared<py::object>(std::move(fn));
             me.set_host_fn(prog, stage, [f](const double* x, int rows, int cols, double* y, int oc) {
               py::gil_scoped_acquire gil;
               py::array_t<double> X({rows, cols});
               std::memcpy(X.mutable_data(), x, size_t(rows) * size_t(cols) * sizeof(double));
               py::object r = (*f)(X);
               auto Y = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(r);
               if (!Y) throw std::runtime_error("component returned a non-numeric payload");
               const size_t want = size_t(rows) * size_t(oc);
               if (size_t(Y.size()) != want)
                 throw std::runtime_error("component returned " + std::to_string(Y.size()) + " values, expected " +
                                          std::to_string(rows) + " x " + std::to_string(oc));
               std::memcpy(y, Y.data(), want * sizeof(double));
             });
           })
      .def("prepare", [](par::Mesh& me) { return py::bytes(me.prepare()); })
      .def("connect",
           [](par::Mesh& me, const std::vector<py::bytes>& blobs) {
             std::vector<std::string> b;
             for (auto& x : blobs) b.emplace_back(std::string(x));
             py::gil_scoped_release nogil;
             me.connect(b);
           })
      .def("unlink", &par::Mesh::unlink)
      .def("start", [](par::Mesh& me) {
        py::gil_scoped_release nogil;
        me.start();
      })
      .def("join", [](par::Mesh& me) {
        py::gil_scoped_release nogil;
        me.join();
      })
      .def("stop_peers", [](par::Mesh& me) {
        py::gil_scoped_release nogil;
        me.stop_peers();
      })
      .def("close", [](par::Mesh& me) {
        py::gil_scoped_release nogil;
        me.close();
      })
      .def_property_readonly("open", &par::Mesh::open)
      .def("error", &par::Mesh::error)
      .def("messages_per_batch", &par::Mesh::messages_per_batch)
      .def("stats", [](const par::Mesh& me) {
        const auto s = me.stats();
        py::dict d;
        d["batches"] = s.batches;
        d["rows"] = s.rows;
        d["max_inflight"] = s.max_inflight;
        d["host_waits"] = s.host_waits;
        d["stage_errors"] = s.stage_errors;
        return d;
      })
      .def("program_model", &par::Mesh::program_model, py::arg("prog"),
           py::arg("class_names") = std::vector<std::string>(), py::arg("flat_output") = false);

  // ------------------------------------------------------------- engine
  py::class_<Engine, std::shared_ptr<Engine>>(m, "Engine")
      .def(py::init([](const std::string& spec_json, const std::string& deployment_name, const std::string& predictor,
                       bool log_requests, bool log_responses, bool log_feedback,
                       std::shared_ptr<Engine> share_metrics_with, const std::string& logging_service,
                       bool log_externally, const std::string& message_type, const std::string& dep_name_env,
                       const std::string& dep_namespace) {
             PredictorSpecC spec = spec_json.empty() ? default_predictor_spec()
                                                     : parse_predictor_spec(parse_json(spec_json), predictor);
             EngineOptions o;
             o.deployment_name = deployment_name;
             o.log_requests = log_requests;
             o.log_responses = log_responses;
             o.log_feedback = log_feedback;
             o.message_logging_service = logging_service;
             o.log_messages_externally = log_externally;
             o.message_type = message_type;
             o.deployment_name_env = dep_name_env;
             o.deployment_namespace = dep_namespace;
             return std::make_shared<Engine>(std::move(spec), o,
                                             share_metrics_with ? share_metrics_with->metrics_ptr() : nullptr);
           }),
           py::arg("spec_json") = "", py::arg("deployment_name") = "None", py::arg("predictor") = "",
           py::arg("log_requests") = false, py::arg("log_responses") = false, py::arg("log_feedback") = false,
           py::arg("share_metrics_with") = nullptr, py::arg("message_logging_service") = "",
           py::arg("log_messages_externally") = false, py::arg("message_type") = "seldon.message.pair",
           py::arg("deployment_name_env") = "", py::arg("deployment_namespace") = "")
      .def("flush_message_log", [](Engine& e) {
        py::gil_scoped_release nogil;
        if (auto* l = e.message_logger()) l->flush();
      })
      .def("message_log_stats", [](Engine& e) {
        py::dict d;
        auto* l = e.message_logger();
        d["sent"] = l ? l->sent() : 0;
        d["failed"] = l ? l->failed() : 0;
        d["dropped"] = l ? l->dropped() : 0;
        return d;
      })
      .def("set_traffic", &Engine::set_traffic, py::arg("self_weight"), py::arg("peers"), py::arg("shadows"))
      .def("add_header_route", &Engine::add_header_route, py::arg("name"), py::arg("value"), py::arg("regex"),
           py::arg("target"))
      .def("bind_python",
           [](Engine& e, const std::string& node, py::object adapter, uint32_t builtin_methods, int batch_rows,
              std::vector<int> worker_fds) {
             PyUnitOptions o;
             o.batch_rows = batch_rows;
             o.worker_fds = std::move(worker_fds);
             auto u = std::make_shared<PyUnit>(std::move(adapter), builtin_methods, std::move(o));
             e.bind(node, u);
             return u;
           },
           py::arg("node"), py::arg("adapter"), py::arg("builtin_methods") = 0, py::arg("batch_rows") = 0,
           py::arg("worker_fds") = std::vector<int>{})
      .def("bind_batched", [](Engine& e, const std::string& node,
                              std::shared_ptr<gpu::BatchedUnit> u) { e.bind(node, u); })
      .def("bind_unit", [](Engine& e, const std::string& node, std::shared_ptr<Unit> u) { e.bind(node, u); })
      .def("bind_fused", [](Engine& e, const std::string& root, std::shared_ptr<Unit> u,
                            const std::vector<std::string>& absorbed) { e.bind_fused(root, u, absorbed); })
      .def("fused_nodes", [](const Engine& e, const std::string& n) {
        std::vector<std::string> v;
        if (const Node* nd = e.node(n))
          for (const Node* f : nd->fused) v.push_back(f->name);
        return v;
      })
      .def("finalize", &Engine::finalize)
      .def("inflight", &Engine::inflight)
      .def("enable_tracing", &Engine::enable_tracing, py::arg("rate") = 1.0)
      .def("drain_spans", [](Engine& e) {
        py::list out;
        for (auto& s : e.drain_spans()) {
          py::dict d;
          d["traceId"] = s.trace_id;
          d["id"] = s.span_id;
          if (!s.parent_id.empty()) d["parentId"] = s.parent_id;
          d["name"] = s.name;
          d["timestamp"] = s.start_us;
          d["duration"] = std::max<int64_t>(1, s.dur_us);
          py::dict tags;
          tags["seldon.puid"] = s.puid;
          if (s.error) tags["error"] = "true";
          d["tags"] = tags;
          out.append(d);
        }
        return out;
      })
      .def("ready", &Engine::ready)
      .def("node_names", &Engine::node_names)
      .def("unit_kind", [](const Engine& e, const std::string& n) {
        auto u = e.unit_of(n);
        return u ? u->kind() : std::string();
      })
      .def("node_methods", [](const Engine& e, const std::string& n) {
        const Node* nd = e.node(n);
        return nd ? nd->methods : 0u;
      })
      .def("snapshot", [](const Engine& e, const std::string& n) {
        auto u = e.unit_of(n);
        return py::bytes(u ? u->snapshot() : std::string());
      })
      .def("restore", [](const Engine& e, const std::string& n, const py::bytes& b) {
        auto u = e.unit_of(n);
        if (u) u->restore(std::string(b));
      })
      .def("predict_json",
           [](Engine& e, const std::string& text, const std::map<std::string, std::string>& headers) {
             auto msg = std::make_shared<SeldonMessage>();
             try {
               message_from_json(parse_json(text), *msg);
             } catch (const std::exception&) {
               auto err = make_error(ApiError::INVALID_JSON, text);
               return std::make_pair(err->http_status, error_to_json(*err));
             }
             std::vector<std::pair<std::string, std::string>> hv;
             for (const auto& kv : headers)
               if (e.is_route_header(kv.first)) hv.emplace_back(kv.first, kv.second);
             // continuations on the shared pool, off the GPU pumps (pool_executor.h)
             Outcome o = wait_outcome([&](Done k) {
               if (hv.empty()) e.predict(msg, std::move(k), PoolExecutor::shared());
               else e.predict_with_headers(msg, std::move(k), PoolExecutor::shared(), hv);
             });
             return render(o);
           },
           py::arg("text"), py::arg("headers") = std::map<std::string, std::string>())
      .def("predict_pb",
           [](Engine& e, const py::bytes& b) -> py::tuple {
             auto msg = std::make_shared<SeldonMessage>();
             if (!message_from_pb(std::string(b), *msg)) {
               auto err = make_error(ApiError::INVALID_JSON, "invalid protobuf");
               return py::make_tuple(err->http_status, py::bytes(error_to_json(*err)));
             }
             Outcome o = wait_outcome([&](Done k) { e.predict(msg, std::move(k), PoolExecutor::shared()); });
             if (o.err) return py::make_tuple(o.err->http_status, py::bytes(error_to_json(*o.err)));
             std::string out;
             message_to_pb(*o.msg, out);
             return py::make_tuple(200, py::bytes(out));
           })
      .def("feedback_json",
           [](Engine& e, const std::string& text) {
             auto fb = std::make_shared<Feedback>();
             try {
               feedback_from_json(parse_json(text), *fb);
             } catch (const std::exception&) {
               auto err = make_error(ApiError::INVALID_JSON, text);
               return std::make_pair(err->http_status, error_to_json(*err));
             }
             std::promise<ErrPtr> p;
             auto f = p.get_future();
             ErrPtr err;
             {
               py::gil_scoped_release nogil;
               e.send_feedback(fb, [&p](ErrPtr x) { p.set_value(std::move(x)); });
               err = f.get();
             }
             if (err) return std::make_pair(err->http_status, error_to_json(*err));
             return std::make_pair(200, std::string("{}"));
           })
      .def("call_node_json",
           [](Engine& e, const std::string& node, int method, const std::string& text) {
             std::vector<MsgPtr> in;
             Json j = parse_json(text);
             if (Method(method) == Method::AGGREGATE) {
               std::vector<SeldonMessage> list;
               message_list_from_json(j, list);
               for (auto& x : list) in.push_back(std::make_shared<SeldonMessage>(std::move(x)));
             } else {
               auto msg = std::make_shared<SeldonMessage>();
               message_from_json(j, *msg);
               in.push_back(msg);
             }
             Outcome o = wait_outcome([&](Done k) { e.call_node(node, method, std::move(in), std::move(k)); });
             return render(o);
           })
      .def("metrics_text", [](Engine& e) { py::gil_scoped_release r; return e.render_metrics(); })
      .def("new_puid", &Engine::new_puid);

  py::class_<HttpServer, std::shared_ptr<HttpServer>>(m, "HttpServer")
      .def(py::init([](std::shared_ptr<Engine> e, const std::string& host, std::vector<int> ports, int threads,
                       const std::string& microservice_node, bool internal_api, const std::string& openapi) {
             HttpOptions o;
             o.host = host;
             o.ports = std::move(ports);
             o.threads = threads;
             o.microservice_node = microservice_node;
             o.internal_api = internal_api;
             o.openapi_json = openapi;
             return std::make_shared<HttpServer>(std::move(e), o);
           }),
           py::arg("engine"), py::arg("host") = "0.0.0.0", py::arg("ports") = std::vector<int>{8000},
           py::arg("threads") = 4, py::arg("microservice_node") = "", py::arg("internal_api") = true,
           py::arg("openapi") = "")
      .def("start", &HttpServer::start)
      .def("stop", [](HttpServer& s) {
        py::gil_scoped_release nogil;
        s.stop();
      })
      .def_property_readonly("ports", &HttpServer::bound_ports)
      .def_property("paused", &HttpServer::paused, &HttpServer::set_paused)
      .def_property_readonly("requests_served", &HttpServer::requests_served);

  py::class_<GrpcServer, std::shared_ptr<GrpcServer>>(m, "GrpcServer")
      .def(py::init([](std::shared_ptr<Engine> e, const std::string& host, int port, int threads,
                       const std::string& microservice_node, size_t max_message) {
             GrpcOptions o;
             o.host = host;
             o.port = port;
             o.threads = threads;
             o.microservice_node = microservice_node;
             o.max_message = max_message;
             return std::make_shared<GrpcServer>(std::move(e), o);
           }),
           py::arg("engine"), py::arg("host") = "0.0.0.0", py::arg("port") = 5001, py::arg("threads") = 4,
           py::arg("microservice_node") = "", py::arg("max_message") = size_t(64) << 20)
      .def("start", &GrpcServer::start)
      .def("stop", [](GrpcServer& s) {
        py::gil_scoped_release nogil;
        s.stop();
      })
      .def_property_readonly("port", &GrpcServer::bound_port)
      .def_property_readonly("requests_served", &GrpcServer::requests_served);

  // ------------------------------------------------------------- raw kernels
  // Pointers are device (or mapped) addresses as Python ints (tensor.data_ptr()),
  // stream is torch.cuda.current_stream().cuda_stream.
  py::module_ k = m.def_submodule("kernels", "raw gfx950 kernel launchers");
  k.def("linear_f64", [](uintptr_t X, int rows, int K, uintptr_t W, uintptr_t b, int C, int act, uintptr_t out,
                         uintptr_t s) {
    kern::linear_f64(P<const double>(X), rows, K, P<const double>(W), P<const double>(b), C, act, P<double>(out),
                     as_stream(s));
  });
  k.def("linear_uses_mfma", &kern::linear_uses_mfma, py::arg("rows"), py::arg("K"), py::arg("C"),
        "Does linear_f64 run this shape on the f64 matrix cores (SCA_LINEAR_MFMA=0 off, =2 forced)?");
  k.def("tree_perfect_partial", [](uintptr_t X, int rows, int F, uintptr_t nodes, uintptr_t leaves, int depth,
                                   int cmp_le, uintptr_t chunk_begin, int n_chunks, int rb, uintptr_t partial,
                                   uintptr_t s, int lds_trees) {
    kern::tree_perfect_partial(P<const double>(X), rows, F, P<const kern::TreeNode>(nodes), P<const float>(leaves),
                               depth, cmp_le, P<const int>(chunk_begin), n_chunks, rb, P<double>(partial),
                               as_stream(s), lds_trees);
  }, py::arg("X"), py::arg("rows"), py::arg("F"), py::arg("nodes"), py::arg("leaves"), py::arg("depth"),
     py::arg("cmp_le"), py::arg("chunk_begin"), py::arg("n_chunks"), py::arg("rb"), py::arg("partial"), py::arg("s"),
     py::arg("lds_trees") = 0);
  k.def("tree_perfect_fused", [](uintptr_t X, int rows, int F, uintptr_t nodes, uintptr_t leaves, int depth,
                                 int cmp_le, uintptr_t chunk_begin, int n_chunks, int rb, uintptr_t partial,
                                 uintptr_t counter, uintptr_t chunk_group, int groups, uintptr_t base, float scale,
                                 int transform, uintptr_t out, int out_cols, uintptr_t s, int lds_trees) {
    const kern::TreeReduceArgs red{P<int>(counter), P<const int>(chunk_group), groups, P<const float>(base), scale,
                                   transform, P<double>(out), out_cols};
    kern::tree_perfect_fused(P<const double>(X), rows, F, P<const kern::TreeNode>(nodes), P<const float>(leaves),
                             depth, cmp_le, P<const int>(chunk_begin), n_chunks, rb, P<double>(partial), red,
                             as_stream(s), lds_trees);
  });
  k.def("tree_lds_max_trees", &kern::tree_lds_max_trees);
  k.def("tree_whole_rows_per_block", &kern::tree_whole_rows_per_block);
  k.def("tree_perfect_whole", [](uintptr_t X, int rows, int F, uintptr_t nodes, uintptr_t leaves, int depth,
                                 int cmp_le, int n_trees, int rb, uintptr_t base, float scale, int transform,
                                 uintptr_t out, int out_cols, uintptr_t s, int lookahead) {
    kern::tree_perfect_whole(P<const double>(X), rows, F, P<const kern::TreeNode>(nodes), P<const float>(leaves),
                             depth, cmp_le, n_trees, rb, P<const float>(base), scale, transform, P<double>(out),
                             out_cols, as_stream(s), nullptr, lookahead);
  }, py::arg("X"), py::arg("rows"), py::arg("F"), py::arg("nodes"), py::arg("leaves"), py::arg("depth"),
     py::arg("cmp_le"), py::arg("n_trees"), py::arg("rb"), py::arg("base"), py::arg("scale"), py::arg("transform"),
     py::arg("out"), py::arg("out_cols"), py::arg("s"), py::arg("lookahead") = -1);
  k.def("tree_perfect_split", [](uintptr_t X, int rows, int F, uintptr_t nodes, uintptr_t leaves, int depth,
                                 int cmp_le, int n_trees, int parts, uintptr_t base, float scale, int transform,
                                 uintptr_t out, int out_cols, uintptr_t acc, uintptr_t counter, uintptr_t s) {
    kern::tree_perfect_split(P<const double>(X), rows, F, P<const kern::TreeNode>(nodes), P<const float>(leaves),
                             depth, cmp_le, n_trees, parts, P<const float>(base), scale, transform, P<double>(out),
                             out_cols, P<double>(acc), P<int>(counter), as_stream(s));
  });
  k.def("tree_perfect_tile", [](uintptr_t X, int rows, int F, uintptr_t nodes, uintptr_t leaves, int depth,
                                int cmp_le, int n_trees, uintptr_t base, float scale, int transform, uintptr_t out,
                                int out_cols, uintptr_t acc, uintptr_t counter, uintptr_t s) {
    return kern::tree_perfect_tile(P<const double>(X), rows, F, P<const kern::TreeNode>(nodes), P<const float>(leaves),
                                   depth, cmp_le, n_trees, P<const float>(base), scale, transform, P<double>(out),
                                   out_cols, P<double>(acc), P<int>(counter), as_stream(s));
  });
  k.def("tree_reduce", [](uintptr_t partial, int rows, int n_chunks, uintptr_t chunk_group, int groups,
                          uintptr_t base, float scale, int transform, uintptr_t out, int out_cols, uintptr_t s) {
    kern::tree_reduce(P<const double>(partial), rows, n_chunks, P<const int>(chunk_group), groups, P<const float>(base),
                      scale, transform, P<double>(out), out_cols, as_stream(s));
  });
  k.def("combine_mean_f64", [](uintptr_t inputs, int n_in, int64_t n, uintptr_t out, uintptr_t s) {
    kern::combine_mean_f64(P<const double* const>(inputs), n_in, n, P<double>(out), as_stream(s));
  });
  k.def("softmax_rows_f64", [](uintptr_t in, int rows, int C, uintptr_t out, uintptr_t s) {
    kern::softmax_rows_f64(P<const double>(in), rows, C, P<double>(out), as_stream(s));
  });
  k.def("argmax_rows_f64", [](uintptr_t in, int rows, int C, uintptr_t out, uintptr_t s) {
    kern::argmax_rows_f64(P<const double>(in), rows, C, P<int32_t>(out), as_stream(s));
  });
  k.def("minmax_normalize_f64", [](uintptr_t in, int64_t n, uintptr_t out, uintptr_t scratch, uintptr_t s) {
    kern::minmax_normalize_f64(P<const double>(in), n, P<double>(out), P<double>(scratch), as_stream(s));
  });
  k.def("segment_minmax_f64", [](uintptr_t in, uintptr_t seg, int nseg, int cols, uintptr_t out, uintptr_t s) {
    kern::segment_minmax_f64(P<const double>(in), P<const int32_t>(seg), nseg, cols, P<double>(out), as_stream(s));
  });
  k.def("add_relu_bf16", [](uintptr_t a, uintptr_t b, size_t n, uintptr_t out, uintptr_t s) {
    if (n % 8) throw std::invalid_argument("add_relu_bf16: element count not a multiple of 8");
    kern::add_relu_bf16(P<const void>(a), P<const void>(b), n, P<void>(out), as_stream(s));
  });
  k.def("scale_shift_relu_bf16_ok", &kern::scale_shift_relu_bf16_ok);
  k.def("scale_shift_relu_bf16", [](uintptr_t x, uintptr_t scale, uintptr_t shift, int N, int C, int HW, int cl,
                                    uintptr_t out, uintptr_t s) {
    if (!kern::scale_shift_relu_bf16_ok(C, HW, cl)) throw std::invalid_argument("scale_shift_relu_bf16: shape not 8-aligned");
    kern::scale_shift_relu_bf16(P<const void>(x), P<const float>(scale), P<const float>(shift), N, C, HW, cl,
                                P<void>(out), as_stream(s));
  });
  k.def("crop_resize_chw_u8", [](uintptr_t img, int H, int W, int C, int crop, uintptr_t out, uintptr_t s) {
    kern::crop_resize_chw_u8(P<const uint8_t>(img), H, W, C, crop, P<float>(out), as_stream(s));
  });
  k.def("combine_mean_strided_f64", [](uintptr_t base, int k_, int64_t n, uintptr_t out, uintptr_t s) {
    kern::combine_mean_strided_f64(P<const double>(base), k_, n, P<double>(out), as_stream(s));
  });
  k.def("mahalanobis_sm_scores", [](uintptr_t B, uintptr_t cov0, uintptr_t xd, int nb, int k_, double n, uintptr_t out,
                                     uintptr_t s) {
    return kern::mahalanobis_sm_scores(P<const double>(B), P<const double>(cov0), P<const double>(xd), nb, k_, n,
                                       P<double>(out), as_stream(s));
  });
  k.def("maha_step_segments", [](uintptr_t X, uintptr_t seg, int nseg, int p, int k_, double n_stdev, double start_clip,
                                  double max_n, double eps, int out_mode, double threshold, uintptr_t state,
                                  uintptr_t eig, uintptr_t ws, uintptr_t out, uintptr_t s) {
    if (p < 1 || p > kern::kMahaMaxP || k_ < 1 || k_ > std::min(p, kern::kMahaMaxK))
      throw std::runtime_error("maha_step_segments: 1 <= k <= min(p, 16), p <= 64");
    kern::MahaParams prm;
    prm.p = p;
    prm.k = k_;
    prm.n_stdev = n_stdev;
    prm.start_clip = start_clip;
    prm.max_n = max_n;
    prm.eps = eps;
    prm.out_mode = out_mode;
    prm.threshold = threshold;
    kern::maha_step_segments(P<const double>(X), P<const int32_t>(seg), nseg, prm, P<double>(state), P<double>(eig),
                             P<double>(ws), P<double>(out), as_stream(s));
  });
  k.def("gemm_bf16", [](uintptr_t A, int lda, int rows, uintptr_t W, int Kp, int Np, int N, uintptr_t bias, int act,
                        uintptr_t O, int ldo, int o_f32, int path, uintptr_t s) {
    // O[rows][N] = act(A[rows][Kp] . W[Np][Kp]^T + bias): bf16 operands, fp32 accumulate
    if (Kp % 64 || Np % 64 || N > Np || lda < Kp || ldo < N || rows <= 0)
      throw std::runtime_error("gemm_bf16: Kp, Np multiples of 64, N <= Np, lda >= Kp, ldo >= N");
    kern::DenseGemmArgs a;
    a.bf16 = 1;
    a.W = P<const void>(W);
    a.bias = P<const float>(bias);
    a.K = Kp;
    a.Kp = Kp;
    a.N = N;
    a.Np = Np;
    a.act = act;
    a.A = P<const void>(A);
    a.lda = lda;
    a.rows = rows;
    a.rows_eff = rows;
    a.O = P<void>(O);
    a.ldo = ldo;
    a.o_f32 = o_f32;
    a.n_store = N;
    a.path = path;
    kern::dense_gemm(a, as_stream(s));
  }, py::arg("A"), py::arg("lda"), py::arg("rows"), py::arg("W"), py::arg("Kp"), py::arg("Np"), py::arg("N"),
        py::arg("bias"), py::arg("act"), py::arg("O"), py::arg("ldo"), py::arg("o_f32"), py::arg("path"),
        py::arg("stream") = 0);
  k.def("mean_sigmoid_rows_f64", [](uintptr_t in, int rows, int F, double thr, uintptr_t out, uintptr_t s) {
    kern::mean_sigmoid_rows_f64(P<const double>(in), rows, F, thr, P<double>(out), as_stream(s));
  });
  k.def("eg_route", [](uintptr_t best, int nb, float eps, uint64_t seed, uint64_t offset, int n, uintptr_t out,
                       uintptr_t s) {
    kern::eg_route(P<const int32_t>(best), nb, eps, seed, offset, n, P<double>(out), as_stream(s));
  });
  k.def("ts_route", [](uintptr_t alpha, uintptr_t beta, int nb, uint64_t seed, uint64_t offset, int n, uintptr_t out,
                       uintptr_t s) {
    kern::ts_route(P<const float>(alpha), P<const float>(beta), nb, seed, offset, n, P<double>(out), as_stream(s));
  });

  // ------------------------------------------------------------- remote nodes
  py::class_<RemoteUnit, Unit, std::shared_ptr<RemoteUnit>>(m, "RemoteUnit")
      .def(py::init([](const std::string& host, int port, bool grpc, const std::string& node_type,
                       const std::string& model_name, const std::string& model_image, const std::string& model_version,
                       int connect_timeout_ms, int read_timeout_ms, int retries, int threads) {
             RemoteOptions o;
             o.host = host;
             o.port = port;
             o.grpc = grpc;
             o.node_type = node_type;
             o.model_name = model_name;
             o.model_image = model_image;
             o.model_version = model_version;
             o.connect_timeout_ms = connect_timeout_ms;
             o.read_timeout_ms = read_timeout_ms;
             o.retries = retries;
             o.threads = threads;
             return std::make_shared<RemoteUnit>(o);
           }),
           py::arg("host"), py::arg("port"), py::arg("grpc") = false, py::arg("node_type") = "MODEL",
           py::arg("model_name") = "", py::arg("model_image") = "", py::arg("model_version") = "",
           py::arg("connect_timeout_ms") = 200, py::arg("read_timeout_ms") = 5000, py::arg("retries") = 3,
           py::arg("threads") = 8)
      .def("ready", &RemoteUnit::ready)
      .def("call_rest", [](RemoteUnit& u, const std::string& path, const std::string& body) {
        py::gil_scoped_release nogil;
        return u.call_rest(path, body);
      })
      .def("stop", [](RemoteUnit&) {});

  // ------------------------------------------------------------- routers
  py::class_<gpu::BanditModel, gpu::RowModel, std::shared_ptr<gpu::BanditModel>>(m, "BanditModel")
      .def(py::init([](int kind, int n_branches, float epsilon, int64_t seed, int best_branch) {
             return std::make_shared<gpu::BanditModel>(gpu::BanditModel::Kind(kind), n_branches, epsilon, seed,
                                                       best_branch);
           }),
           py::arg("kind"), py::arg("n_branches"), py::arg("epsilon") = 0.1f, py::arg("seed") = -1,
           py::arg("best_branch") = -1)
      .def("feedback", &gpu::BanditModel::feedback)
      .def("values", &gpu::BanditModel::values)
      .def_property_readonly("best_branch", &gpu::BanditModel::best_branch)
      .def_property_readonly("n_branches", &gpu::BanditModel::n_branches)
      .def("snapshot", &gpu::BanditModel::snapshot)
      .def("restore", &gpu::BanditModel::restore)
      .def("route_host", &gpu::BanditModel::route_host, "epsilon-greedy decision on the host (kernel's Philox stream)")
      .def("attach_shared", &gpu::BanditModel::attach_shared, py::arg("name"), py::arg("worker") = 0,
           "keep the counters in the host-wide shared mapping `name` (one router state across engine processes)")
      .def_property_readonly("shared", &gpu::BanditModel::shared);
  py::class_<gpu::BanditRouterUnit, Unit, std::shared_ptr<gpu::BanditRouterUnit>>(m, "BanditRouterUnit")
      .def(py::init([](std::shared_ptr<gpu::BanditModel> model, int device, int max_batch, int slots, bool device_route) {
             gpu::BatcherOptions o;
             o.device = device;
             o.max_batch = max_batch;
             o.slots = slots;
             return std::make_shared<gpu::BanditRouterUnit>(model, o, device_route);
           }),
           py::arg("model"), py::arg("device") = 0, py::arg("max_batch") = 4096, py::arg("slots") = 2,
           py::arg("device_route") = false)
      .def_property_readonly("batcher", &gpu::BanditRouterUnit::batcher)
      .def_property_readonly("model", &gpu::BanditRouterUnit::model)
      .def("stats", [](const gpu::BanditRouterUnit& u) {
        auto s = u.batcher()->stats();
        py::dict d;
        d["batches"] = s.batches;
        d["rows"] = s.rows;
        d["requests"] = s.requests;
        return d;
      })
      .def("stop", [](gpu::BanditRouterUnit& u) {
        py::gil_scoped_release nogil;
        u.batcher()->stop();
      });
}
