#include "graph.h"

#include <algorithm>
#include <cstdlib>
#include <set>
#include <stdexcept>

namespace sca::gpu {

struct GraphModel::Aux {
  size_t cap_rows = 0;
  int cap_cols = -1;
  std::vector<int> cols;                          // output cols per stage (for cap_cols)
  std::vector<DeviceBuffer> out;                  // per stage output, on the stage's GPU
  std::vector<DeviceBuffer> ws;                   // per stage model workspace
  std::vector<std::vector<DeviceBuffer>> staged;  // non-peer mode: consumer-local copies of inputs
  std::vector<PinnedBuffer> ptrs;                 // mean stages: device-visible input pointer arrays
  std::map<int, Stream> streams;                  // per non-root lane (GPU, or stage in split mode)
  std::vector<Event> ev;                          // per stage, recorded on the stage's stream
  Event ev_start;                                 // root stream: inputs staged
};

GraphModel::~GraphModel() = default;

GraphModel::GraphModel(std::vector<GraphStage> stages, int in_cols) : st_(std::move(stages)), in_cols_(in_cols) {
  if (st_.empty()) throw std::runtime_error("GraphModel: no stages");
  if (const char* e = std::getenv("SCA_GRAPH_SPLIT")) split_ = std::atoi(e) != 0;
  std::map<const RowModel*, int> placed;
  for (size_t i = 0; i < st_.size(); ++i) {
    const auto& s = st_[i];
    for (int j : s.inputs)
      if (j < -1 || j >= int(i)) throw std::runtime_error("GraphModel: stage inputs must precede the stage (" + s.node + ")");
    if (s.kind == GraphStage::kModel) {
      if (!s.model || s.inputs.size() != 1) throw std::runtime_error("GraphModel: model stage needs a model and one input (" + s.node + ")");
      auto it = placed.find(s.model.get());
      if (it != placed.end() && it->second != s.device)
        throw std::runtime_error("GraphModel: one model object placed on two GPUs (" + s.node + ")");
      placed[s.model.get()] = s.device;
    } else if (s.kind == GraphStage::kMean) {
      if (s.inputs.empty()) throw std::runtime_error("GraphModel: combiner stage without inputs (" + s.node + ")");
    } else {
      throw std::runtime_error("GraphModel: unknown stage kind");
    }
  }
  if (in_cols_ <= 0)
    for (const auto& s : st_)
      if (s.kind == GraphStage::kModel && s.inputs[0] == -1 && s.model->in_cols() > 0) { in_cols_ = s.model->in_cols(); break; }
  std::vector<int> cols;
  stage_cols(in_cols_ > 0 ? in_cols_ : 1, cols);  // validates combiner widths
  const auto& last = st_.back();
  if (last.kind == GraphStage::kModel) set_flat_output(last.model->flat_output());
}

void GraphModel::stage_cols(int in_cols, std::vector<int>& cols) const {
  cols.resize(st_.size());
  auto col_of = [&](int j) { return j < 0 ? in_cols : cols[size_t(j)]; };
  for (size_t i = 0; i < st_.size(); ++i) {
    const auto& s = st_[i];
    if (s.kind == GraphStage::kModel) {
      const int c = col_of(s.inputs[0]);
      if (s.model->in_cols() > 0 && c != s.model->in_cols())
        throw std::runtime_error("GraphModel: stage " + s.node + " expects " + std::to_string(s.model->in_cols()) +
                                 " columns but receives " + std::to_string(c));
      cols[i] = s.model->out_cols(c);
    } else {
      const int c = col_of(s.inputs[0]);
      for (int j : s.inputs)
        if (col_of(j) != c)
          throw std::runtime_error("Expected batch length " + std::to_string(c) + " but found " + std::to_string(col_of(j)));
      cols[i] = c;
    }
  }
}

std::shared_ptr<RowModel> GraphModel::clone_on(int device) const {
  std::vector<GraphStage> st = st_;
  std::map<const RowModel*, std::shared_ptr<RowModel>> copies;  // keep shared models shared
  for (auto& s : st) {
    if (device != -2) s.device = device;
    if (s.kind != GraphStage::kModel) continue;
    auto& c = copies[s.model.get()];
    if (!c) c = s.model->clone();
    s.model = c;
  }
  auto g = std::make_shared<GraphModel>(std::move(st), in_cols_);
  g->set_split(split_);
  return with_meta(g);
}

int GraphModel::out_cols(int in_cols) const {
  std::vector<int> cols;
  stage_cols(in_cols, cols);
  return cols.back();
}

std::vector<std::string> GraphModel::names_of(int stage) const {
  if (stage < 0) return {};
  const auto& s = st_[size_t(stage)];
  if (s.kind == GraphStage::kModel) return s.model->class_names();
  return names_of(s.inputs[0]);  // AverageCombinerUnit keeps the first child's names
}

std::vector<std::string> GraphModel::class_names() const {
  if (!names_.empty()) return names_;
  return names_of(int(st_.size()) - 1);
}

std::vector<int> GraphModel::devices() const {
  std::set<int> d;
  for (const auto& s : st_) d.insert(s.device);
  return {d.begin(), d.end()};
}

void GraphModel::to_device(int device) {
  root_device_ = device;
  std::set<int> devs;
  devs.insert(device);
  for (auto& s : st_) {
    devs.insert(s.device);
    if (s.kind == GraphStage::kModel) s.model->to_device(s.device);
  }
  // Every GPU pair of the graph talks over xGMI: enable direct peer access so a
  // consumer kernel loads the producer's HBM without a copy.
  peer_direct_ = true;
  for (int a : devs)
    for (int b : devs) {
      if (a == b) continue;
      int can = 0;
      SCA_HIP_CHECK(hipDeviceCanAccessPeer(&can, a, b));
      if (!can) { peer_direct_ = false; continue; }
      DeviceGuard g(a);
      hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      else if (e != hipSuccess) { (void)hipGetLastError(); peer_direct_ = false; }
    }
  if (split_ == 1) peer_direct_ = false;
  // Verify every cross-GPU edge before serving: a kernel
  // on the consumer GPU reads a pattern out of the producer's HBM through the
  // peer pointer -- exactly what a stage kernel does -- and the result is
  // compared on the host.  Any failure drops the graph to staged copies.
  // Split mode 2 (lanes on one GPU reading each other's buffers) checks the
  // device against itself.  SCA_GRAPH_PEER_FAULT=1 injects a failure.
  peer_canary_.clear();
  if (peer_direct_) {
    std::vector<std::pair<int, int>> pairs;
    for (int a : devs)
      for (int b : devs)
        if (a != b) pairs.push_back({a, b});
    if (split_ == 2 && devs.size() == 1) pairs.push_back({device, device});
    for (auto& pr : pairs) {
      const bool ok = peer_canary(pr.first, pr.second);
      peer_canary_.push_back({pr.first, pr.second, ok});
      if (!ok) peer_direct_ = false;
    }
  }
  build_fused();
}

bool GraphModel::peer_canary(int consumer, int producer) {
  if (const char* e = std::getenv("SCA_GRAPH_PEER_FAULT"))
    if (std::atoi(e) != 0) return false;
  constexpr int n = 256;
  std::vector<double> pat(n), back(n, 0.0);
  for (int i = 0; i < n; ++i) pat[size_t(i)] = 1e3 * (producer + 1) + 7.0 * (consumer + 1) + i + 0.125;
  try {
    DeviceBuffer src(n * sizeof(double), producer);
    src.upload(pat.data(), n * sizeof(double));
    DeviceBuffer dst(n * sizeof(double), consumer), tab(sizeof(double*), consumer);
    const double* p = src.as<double>();
    tab.upload(&p, sizeof p);
    DeviceGuard g(consumer);
    kern::combine_mean_f64(tab.as<const double* const>(), 1, n, dst.as<double>(), nullptr);  // mean of one = copy
    if (hipDeviceSynchronize() != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (hipMemcpy(back.data(), dst.get(), n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
  } catch (const std::exception&) {
    (void)hipGetLastError();
    return false;
  }
  return back == pat;
}

void GraphModel::build_fused() {
  fused_ = false;
  if (const char* e = std::getenv("SCA_GRAPH_FUSE"))
    if (std::atoi(e) == 0) return;
  if (split_ || st_.empty() || int(st_.size()) > kern::kLinearGraphMaxStages || in_cols_ <= 0 ||
      in_cols_ > kern::kLinearGraphMaxWidth)
    return;
  for (const auto& s : st_)
    if (s.device != root_device_) return;
  std::vector<int> oc;
  try {
    stage_cols(in_cols_, oc);
  } catch (const std::exception&) {
    return;
  }
  std::vector<kern::LinearGraphStage> fs(st_.size());
  std::vector<double> params;
  int slots = 0;
  for (size_t i = 0; i < st_.size(); ++i) {
    const auto& s = st_[i];
    kern::LinearGraphStage& f = fs[i];
    if (s.inputs.empty() || int(s.inputs.size()) > kern::kLinearGraphMaxInputs) return;
    f.n_in = int(s.inputs.size());
    for (size_t q = 0; q < s.inputs.size(); ++q) f.in[q] = s.inputs[q];
    f.out_cols = oc[i];
    if (oc[i] > kern::kLinearGraphMaxWidth) return;
    if (s.kind == GraphStage::kMean) {
      f.kind = 1;
      f.C = oc[i];
    } else {
      const auto* lm = dynamic_cast<const LinearModel*>(s.model.get());
      if (!lm || lm->features() > kern::kLinearGraphMaxWidth || lm->classes() > kern::kLinearGraphMaxWidth) return;
      f.kind = 0;
      f.K = lm->features();
      f.C = lm->classes();
      f.act = lm->activation();
      f.w_off = int(params.size());
      params.insert(params.end(), lm->weights().begin(), lm->weights().end());
      if (!lm->bias().empty()) {
        f.b_off = int(params.size());
        params.insert(params.end(), lm->bias().begin(), lm->bias().end());
      }
    }
    f.out_off = slots;
    slots += oc[i];
  }
  if (slots > kern::kLinearGraphMaxSlots || int(params.size()) > kern::kLinearGraphMaxParams) return;
  d_fstages_.alloc(fs.size() * sizeof(kern::LinearGraphStage), root_device_);
  d_fstages_.upload(fs.data(), fs.size() * sizeof(kern::LinearGraphStage));
  d_fparams_.alloc(std::max<size_t>(1, params.size()) * sizeof(double), root_device_);
  if (!params.empty()) d_fparams_.upload(params.data(), params.size() * sizeof(double));
  fused_stages_ = int(fs.size());
  fused_params_ = int(params.size());
  fused_slots_ = slots;
  fused_ = true;
}

bool GraphModel::launch_signal(const double* X, int rows, int cols, double* out, void*, hipStream_t s,
                               hipEvent_t done) {
  if (!fused_ || cols != in_cols_) return false;
  DeviceGuard g(root_device_);
  kern::linear_graph_f64(X, rows, cols, d_fstages_.as<kern::LinearGraphStage>(), fused_stages_,
                         d_fparams_.as<double>(), fused_params_, fused_slots_, out, s, done);
  return true;
}

int GraphModel::lane_of(int stage) const {
  if (stage < 0) return kRootLane;
  if (split_) return 1 << 20 | stage;
  const int d = st_[size_t(stage)].device;
  return d == root_device_ ? kRootLane : d;
}

bool GraphModel::multi_lane() const {
  for (size_t i = 0; i < st_.size(); ++i)
    if (lane_of(int(i)) != kRootLane) return true;
  return false;
}

GraphModel::Aux& GraphModel::aux_for(hipStream_t s, int rows, int cols) {
  std::lock_guard<std::mutex> g(mu_);
  auto& slot = aux_[s];
  if (!slot) {
    slot = std::make_unique<Aux>();
    Aux& a = *slot;
    a.out.resize(st_.size());
    a.ws.resize(st_.size());
    a.staged.resize(st_.size());
    a.ptrs = std::vector<PinnedBuffer>(st_.size());
    a.ev = std::vector<Event>(st_.size());
    const bool multi = multi_lane();
    for (size_t i = 0; i < st_.size(); ++i) {
      const int lane = lane_of(int(i));
      if (lane != kRootLane && !a.streams.count(lane)) a.streams[lane].create(st_[i].device);
      if (multi) a.ev[i].create(st_[i].device);
      if (st_[i].kind == GraphStage::kMean) a.ptrs[i].alloc(st_[i].inputs.size() * sizeof(double*));
    }
    if (multi) a.ev_start.create(root_device_);
  }
  Aux& a = *slot;
  if (size_t(rows) > a.cap_rows || cols != a.cap_cols) {
    // Growth (rare: geometric) frees buffers that earlier batches of this
    // slot used on every stage device: drain the slot's streams first rather
    // than rely on hipFree's implicit synchronisation, which covers only the
    // current device.
    if (a.cap_rows > 0) {
      SCA_HIP_CHECK(hipStreamSynchronize(s));
      for (auto& kv : a.streams) SCA_HIP_CHECK(hipStreamSynchronize(kv.second.get()));
    }
    size_t cap = std::max<size_t>(64, a.cap_rows);
    while (cap < size_t(rows)) cap <<= 1;
    stage_cols(cols, a.cols);
    for (size_t i = 0; i < st_.size(); ++i) {
      const auto& st = st_[i];
      a.out[i].alloc(cap * size_t(a.cols[i]) * sizeof(double), st.device);
      if (st.kind == GraphStage::kModel) {
        const int ic = st.inputs[0] < 0 ? cols : a.cols[size_t(st.inputs[0])];
        a.ws[i].alloc(st.model->workspace_bytes(int(cap), ic), st.device);
      }
      a.staged[i].clear();
      if (!peer_direct_) {
        a.staged[i].resize(st.inputs.size());
        for (size_t k = 0; k < st.inputs.size(); ++k) {
          const int j = st.inputs[k];
          if (lane_of(j) != lane_of(int(i))) {
            const int c = j < 0 ? cols : a.cols[size_t(j)];
            a.staged[i][k].alloc(cap * size_t(c) * sizeof(double), st.device);
          }
        }
      }
    }
    a.cap_rows = cap;
    a.cap_cols = cols;
  }
  return a;
}

void GraphModel::launch_segments(const double* X, int rows, int cols, double* out, void*, const int32_t* seg,
                                 int nseg, hipStream_t s) {
  if (root_device_ < 0) throw std::runtime_error("GraphModel: to_device() not called");
  if (fused_ && cols == in_cols_) {
    DeviceGuard g(root_device_);
    kern::linear_graph_f64(X, rows, cols, d_fstages_.as<kern::LinearGraphStage>(), fused_stages_,
                           d_fparams_.as<double>(), fused_params_, fused_slots_, out, s);
    return;
  }
  Aux& a = aux_for(s, rows, cols);
  const bool multi = a.ev_start.get() != nullptr;
  const size_t last = st_.size() - 1;
  auto stream_of = [&](int lane) { return lane == kRootLane ? s : a.streams[lane].get(); };
  if (multi) SCA_HIP_CHECK(hipEventRecord(a.ev_start.get(), s));
  for (size_t i = 0; i < st_.size(); ++i) {
    const auto& st = st_[i];
    DeviceGuard g(st.device);
    const int lane = lane_of(int(i));
    hipStream_t ss = stream_of(lane);
    const double* in_ptr[64];
    const size_t n_in = std::min<size_t>(st.inputs.size(), 64);
    for (size_t k = 0; k < n_in; ++k) {
      const int j = st.inputs[k];
      const double* p = j < 0 ? X : a.out[size_t(j)].as<double>();
      if (multi && lane_of(j) != lane)
        SCA_HIP_CHECK(hipStreamWaitEvent(ss, j < 0 ? a.ev_start.get() : a.ev[size_t(j)].get(), 0));
      if (!peer_direct_ && lane_of(j) != lane) {
        const int c = j < 0 ? cols : a.cols[size_t(j)];
        double* dst = a.staged[i][k].as<double>();
        SCA_HIP_CHECK(hipMemcpyAsync(dst, p, size_t(rows) * c * sizeof(double), hipMemcpyDefault, ss));
        p = dst;
      }
      in_ptr[k] = p;
    }
    // The output stage writes straight into the caller's buffer when it can
    // address it (same GPU, pinned host, or xGMI peer).
    const bool direct_out = i == last && (lane == kRootLane || peer_direct_);
    double* o = direct_out ? out : a.out[i].as<double>();
    if (st.kind == GraphStage::kModel) {
      const int ic = st.inputs[0] < 0 ? cols : a.cols[size_t(st.inputs[0])];
      if (seg && st.model->segmented()) st.model->launch_segments(in_ptr[0], rows, ic, o, a.ws[i].get(), seg, nseg, ss);
      else st.model->launch(in_ptr[0], rows, ic, o, a.ws[i].get(), ss);
    } else {
      const double** arr = a.ptrs[i].host<const double*>();
      for (size_t k = 0; k < n_in; ++k) arr[k] = in_ptr[k];
      kern::combine_mean_f64(a.ptrs[i].dev<const double* const>(), int(n_in), int64_t(rows) * a.cols[i], o, ss);
    }
    if (i == last && !direct_out)
      SCA_HIP_CHECK(hipMemcpyAsync(out, o, size_t(rows) * a.cols[i] * sizeof(double), hipMemcpyDefault, ss));
    if (multi) SCA_HIP_CHECK(hipEventRecord(a.ev[i].get(), ss));
  }
  if (multi && lane_of(int(last)) != kRootLane) SCA_HIP_CHECK(hipStreamWaitEvent(s, a.ev[last].get(), 0));
}

void GraphModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  std::vector<int> oc;
  stage_cols(cols, oc);
  std::vector<std::vector<double>> buf(st_.size());
  auto ptr = [&](int j) { return j < 0 ? X : buf[size_t(j)].data(); };
  for (size_t i = 0; i < st_.size(); ++i) {
    const auto& st = st_[i];
    buf[i].assign(size_t(rows) * oc[i], 0.0);
    if (st.kind == GraphStage::kModel) {
      const int ic = st.inputs[0] < 0 ? cols : oc[size_t(st.inputs[0])];
      st.model->run_cpu(ptr(st.inputs[0]), rows, ic, buf[i].data());
    } else {
      for (int j : st.inputs) {
        const double* p = ptr(j);
        for (size_t e = 0; e < buf[i].size(); ++e) buf[i][e] += p[e];
      }
      const double inv = 1.0 / double(st.inputs.size());
      for (auto& v : buf[i]) v *= inv;
    }
  }
  std::copy(buf.back().begin(), buf.back().end(), out);
}

}  // namespace sca::gpu
