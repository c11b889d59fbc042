// Device graph: a fused, device-resident sub-graph of row models.
//
// The reference evaluates every node of an inference graph as a separate
// microservice hop (PredictiveUnitBean.java:112-197 -> InternalPredictionService
// HTTP/gRPC call per node), serialising the SeldonMessage to JSON at every edge.
// On MI355X a chain (TRANSFORMER -> MODEL -> OUTPUT_TRANSFORMER) or an ensemble
// (COMBINER over N MODELs, possibly placed on different GPUs) whose nodes are all
// row models runs as ONE micro-batched unit:
//
//   request rows -> [pinned host] -> stage 0 on GPU a -> stage 1 on GPU b ... ->
//   mean-combine on GPU c -> [pinned host] -> responses
//
// Activations never leave HBM between stages.  Cross-GPU edges are direct xGMI
// peer accesses (the consumer kernel reads the producer's HBM; peer access is
// enabled between every pair of participating GPUs at to_device()), ordered by
// cross-device events on per-slot streams, so a fan-out to K GPUs is K
// concurrent kernels and a fan-in is one combine kernel gathering over xGMI.
// Stages that do not feed the graph output (non-first children of a MODEL,
// whose outputs the default aggregate discards) are pruned at build time.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "models.h"

namespace sca::gpu {

struct GraphStage {
  enum Kind { kModel = 0, kMean = 1 };
  int kind = kModel;
  RowModelPtr model;        // kModel
  int device = 0;           // GPU the stage runs on
  std::vector<int> inputs;  // producer stage indices; -1 = graph input
  std::string node;         // graph node name (diagnostics)
};

class GraphModel : public RowModel {
 public:
  // `stages` in topological order; the last stage is the graph output.
  GraphModel(std::vector<GraphStage> stages, int in_cols);
  ~GraphModel() override;
  std::string name() const override { return "graph" + std::to_string(st_.size()); }
  int in_cols() const override { return in_cols_; }
  int out_cols(int in_cols) const override;
  std::vector<std::string> class_names() const override;
  void to_device(int device) override;
  bool zero_copy_input() const override {
    for (const auto& s : st_)
      for (int j : s.inputs)
        if (j < 0 && s.model && !s.model->zero_copy_input()) return false;
    return true;
  }
  bool device_io_only() const override {
    for (const auto& s : st_)
      if (s.model && s.model->device_io_only()) return true;
    return false;
  }
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override {
    launch_segments(X, rows, cols, out, ws, nullptr, 0, s);
  }
  bool exclusive_driver() const override {
    for (const auto& s : st_)
      if (s.model && s.model->exclusive_driver()) return true;
    return false;
  }
  bool segmented() const override {
    for (const auto& s : st_)
      if (s.model && s.model->segmented()) return true;
    return false;
  }
  void launch_segments(const double* X, int rows, int cols, double* out, void* ws, const int32_t* seg, int nseg,
                       hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  // Fused graphs (every stage a small linear model or a mean, one GPU): the
  // whole graph is one kernel, which completes `done` itself.
  bool launch_signal(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                     hipEvent_t done) override;
  bool fused() const { return fused_; }
  struct PeerCheck {
    int consumer, producer;
    bool ok;
  };
  // start-up canaries of the cross-GPU edges (to_device)
  const std::vector<PeerCheck>& peer_canary_results() const { return peer_canary_; }

  std::shared_ptr<RowModel> clone() const override { return clone_on(-2); }
  // Copy with every stage placed on `device` (-2: keep stage placement): one
  // whole-graph replica per GPU for data-parallel serving.
  std::shared_ptr<RowModel> clone_on(int device) const;
  const std::vector<GraphStage>& stages() const { return st_; }
  std::vector<int> devices() const;
  bool peer_direct() const { return peer_direct_; }
  // Split mode (tests / rehearsal on one GPU): every stage gets its own
  // stream and event chain even when stages share a GPU.  Mode 1: cross-stage
  // inputs go through the staged-copy branch (peer_direct_ = false) -- the
  // code a graph spread over GPUs WITHOUT peer access runs.  Mode 2: the
  // lanes read each other's HBM directly and the last lane writes the
  // caller's buffer (peer_direct_ as probed) -- the code an xGMI-connected
  // multi-GPU graph runs.  Set before to_device(); clone_on() keeps it.
  void set_split(int mode) { split_ = mode; }
  bool split() const { return split_ != 0; }
  int split_mode() const { return split_; }

 private:
  struct Aux;  // per-caller-stream resources (one per batcher slot)
  void stage_cols(int in_cols, std::vector<int>& cols) const;
  std::vector<std::string> names_of(int stage) const;
  Aux& aux_for(hipStream_t s, int rows, int cols);
  // Stream lane of a stage (-1 = graph input): stages on one lane share a
  // stream; kRootLane is the caller's stream.
  static constexpr int kRootLane = -1;
  int lane_of(int stage) const;
  bool multi_lane() const;

  std::vector<GraphStage> st_;
  int in_cols_ = 0;
  int root_device_ = -1;
  bool peer_direct_ = true;
  int split_ = 0;
  bool peer_canary(int consumer, int producer);
  std::vector<PeerCheck> peer_canary_;
  // one-kernel form (kern::linear_graph_f64), built at to_device()
  void build_fused();
  bool fused_ = false;
  int fused_stages_ = 0, fused_params_ = 0, fused_slots_ = 0;
  DeviceBuffer d_fstages_, d_fparams_;
  std::mutex mu_;
  std::unordered_map<hipStream_t, std::unique_ptr<Aux>> aux_;
};

}  // namespace sca::gpu
