// Row-wise models served by the GPU micro-batcher.
//
// Each model owns its parameters in HBM (uploaded once, resident for the
// life of the deployment) and exposes an async launch over a micro-batch of
// request rows plus a CPU reference path (used for `device: -1` placement and
// as the test oracle on machines without a GPU).
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.h"
#include "hip_util.h"

namespace sca::gpu {

// A CPU-path call still in flight (models whose work happens elsewhere, e.g.
// on another rank): the batcher polls done() and keeps up to `slots` of them
// outstanding instead of blocking its device thread on each.
struct CpuCall {
  virtual ~CpuCall() = default;
  virtual bool done() = 0;            // non-blocking; true once `out` holds the result (or it failed)
  virtual std::string error() const = 0;
  // Block up to `us` for progress (the batcher's low-CPU mode, instead of a
  // sleep-and-poll whose timer slack costs ~50 us); false = not supported.
  virtual bool wait_us(int) { return false; }
};
using CpuCallPtr = std::shared_ptr<CpuCall>;

class RowModel;
// The row model a BatchedUnit is launching directly, set by the batcher around
// its launch call: only that model may write host-finished raw output.
extern thread_local const RowModel* g_raw_output_model;

class RowModel {
 public:
  virtual ~RowModel() = default;
  virtual std::string name() const = 0;
  virtual int in_cols() const = 0;  // 0 = any width
  virtual int out_cols(int in_cols) const = 0;
  virtual std::vector<std::string> class_names() const { return names_; }
  void set_class_names(std::vector<std::string> n) { names_ = std::move(n); }
  // Single-output models whose reference server returns a 1-D array
  // (e.g. xgboost Booster.predict): response shape [rows], no class names.
  bool flat_output() const { return flat_; }
  void set_flat_output(bool f) { flat_ = f; }
  // Named input columns (an MLflow signature): a request whose
  // `data.names` lists the same columns in another order is permuted into
  // this order before batching; one missing a column is rejected.
  const std::vector<std::string>& input_names() const { return in_names_; }
  void set_input_names(std::vector<std::string> n) { in_names_ = std::move(n); }
  virtual void to_device(int device) = 0;
  // True if launch() needs X/out in device memory (no zero-copy host I/O).
  virtual bool device_io_only() const { return false; }
  // False if many workgroups re-read X (stage it in HBM instead of reading
  // pinned host memory over PCIe from every workgroup).
  virtual bool zero_copy_input() const { return true; }
  // Stage zero-copy batches in HBM through the BAR by default
  // (SCA_BATCH_INPUT unset; batcher.cc): for kernels whose time the row read
  // dominates and whose workgroups read the rows more than once.
  virtual bool prefers_bar_input() const { return false; }
  // Per-batch refinement: a model whose re-read factor depends on the batch
  // geometry may still read small batches straight from pinned host memory
  // (saves the H2D blit launch).
  virtual bool zero_copy_input_for(int rows, int cols) const { (void)rows; (void)cols; return zero_copy_input(); }
  // Rows many workgroups re-read (not zero-copy from pinned host), but which
  // may be written straight into HBM through the BAR (SCA_BATCH_INPUT=bar)
  // instead of DMA'd there.
  virtual bool bar_input_for(int rows, int cols) const { (void)rows; (void)cols; return false; }
  // Segment-aware models compute per request (not per row): the batcher passes
  // the request boundaries (nseg + 1 row offsets, device-visible).
  // Host-finished outputs (only when the batcher launches this model itself,
  // raw_output_allowed(); a model launched as a stage of a device graph or a
  // mesh program always writes final output): for a batch of `rows` the kernel writes
  // raw_out_cols(rows, cols) values per row (e.g. one partial sum per tree
  // part) and finish_host() folds them into the out_cols() values of the
  // response on the pump thread once the batch completed -- for folds whose
  // cross-workgroup form (atomics + an arrival counter + a last workgroup)
  // costs more device time than the host spends adding a few doubles per
  // row.  0 = the kernel writes the final output.
  virtual int raw_out_cols(int rows, int cols) const { (void)rows; (void)cols; return 0; }
  bool raw_output_allowed() const { return g_raw_output_model == this; }
  virtual void finish_host(const double* raw, int rows, int raw_cols, double* out) const {
    (void)raw; (void)rows; (void)raw_cols; (void)out;
  }
  virtual bool segmented() const { return false; }
  // Stateful segmented models: the position in the state's application order
  // of the first row of the last launch_segments() / run_cpu() call made on
  // this view (-1: not tracked).  Read by the batcher right after the call,
  // on the same thread, to tell each request where its rows were applied.
  virtual int64_t last_sequence_base() const { return -1; }
  virtual void launch_segments(const double* X, int rows, int cols, double* out, void* ws, const int32_t* seg, int nseg,
                               hipStream_t s) {
    (void)seg;
    (void)nseg;
    launch(X, rows, cols, out, ws, s);
  }
  virtual size_t workspace_bytes(int max_rows, int cols) const { (void)max_rows; (void)cols; return 0; }
  virtual void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) = 0;
  // launch() whose last kernel completes `done` from its own dispatch
  // (hipExtLaunchKernelGGL) -- the batcher then skips its hipEventRecord.
  // Returns false (nothing launched) if the model cannot.
  virtual bool launch_signal(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                             hipEvent_t done) {
    (void)X; (void)rows; (void)cols; (void)out; (void)ws; (void)s; (void)done;
    return false;
  }
  virtual void run_cpu(const double* X, int rows, int cols, double* out) const = 0;
  // True if launch() can wait on the host (a peer model taking a link lock /
  // the loopback transport's rendezvous): its unit gets a pump thread of its
  // own instead of sharing the GPU's, so it never stalls the other units.
  virtual bool exclusive_driver() const { return false; }
  // True if start_cpu() never blocks for long (it only issues work to other
  // processes): CPU-batching units of such models share one pump thread.
  virtual bool async_cpu() const { return false; }
  // Asynchronous run_cpu: returns a call to poll, or nullptr if the model has
  // none (X must stay valid and `out` untouched until done()).
  virtual CpuCallPtr start_cpu(const double* X, int rows, int cols, double* out) {
    (void)X; (void)rows; (void)cols; (void)out;
    return nullptr;
  }
  // Independent copy (host parameters only; call to_device on it) -- one per
  // GPU replica.
  virtual std::shared_ptr<RowModel> clone() const { throw std::runtime_error(name() + " cannot be replicated"); }

 protected:
  template <class T> std::shared_ptr<RowModel> with_meta(std::shared_ptr<T> m) const {
    m->names_ = names_;
    m->flat_ = flat_;
    m->in_names_ = in_names_;
    return m;
  }
  std::vector<std::string> names_;
  std::vector<std::string> in_names_;
  bool flat_ = false;
};
using RowModelPtr = std::shared_ptr<RowModel>;

// ---------------------------------------------------------------- linear
class LinearModel : public RowModel {
 public:
  LinearModel(std::vector<double> W, std::vector<double> b, int C, int K, int act);
  std::string name() const override { return "linear"; }
  int in_cols() const override { return K_; }
  int out_cols(int) const override { return act_ == kern::kActBinaryLogistic ? 2 : C_; }
  void to_device(int device) override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  bool launch_signal(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                     hipEvent_t done) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  std::shared_ptr<RowModel> clone() const override {
    return with_meta(std::make_shared<LinearModel>(W_, b_, C_, K_, act_));
  }
  // parameters, for graph fusion (csrc/kernels/linear_graph.hip)
  const std::vector<double>& weights() const { return W_; }
  const std::vector<double>& bias() const { return b_; }
  int classes() const { return C_; }
  int features() const { return K_; }
  int activation() const { return act_; }

 private:
  std::vector<double> W_, b_;
  int C_, K_, act_;
  DeviceBuffer dW_, db_;
};

// ---------------------------------------------------------- tree ensemble
struct TreeEnsembleSpec {
  // Common
  int n_trees = 0;
  int n_features = 0;
  int groups = 1;          // output margins (classes for multi:softprob)
  int out_cols = 1;
  int transform = 0;       // kern::TreeTransform
  int cmp_le = 0;          // 1: x <= thr (sklearn), 0: x < thr (xgboost)
  float scale = 1.f;       // margin multiplier (1/n_trees for averaging)
  std::vector<float> base_margin;  // [groups]
  std::vector<int> tree_group;     // [n_trees], must be non-decreasing
  // Perfect layout (depth > 0)
  int depth = 0;
  std::vector<float> thr;          // [n_trees * (2^D - 1)]
  std::vector<int32_t> feat;       // same, bit31 = default-left
  std::vector<float> leaves;       // [n_trees * 2^D]
  // Sparse layout (depth == 0)
  std::vector<kern::SparseNode> nodes;
  std::vector<int> tree_root;      // [n_trees]
};

class TreeEnsembleModel : public RowModel {
 public:
  // xgb1000 serving kernel 8.04 -> 7.17 us (whole) / 7.04 -> 5.96 us (split)
  // with BAR rows (profiles/r05sl_tree_split)
  bool prefers_bar_input() const override { return true; }
  explicit TreeEnsembleModel(TreeEnsembleSpec spec);
  std::string name() const override { return spec_.depth > 0 ? "tree_perfect" : "tree_sparse"; }
  int in_cols() const override { return spec_.n_features; }
  int out_cols(int) const override { return spec_.out_cols; }
  void to_device(int device) override;
  size_t workspace_bytes(int max_rows, int cols) const override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  bool launch_signal(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                     hipEvent_t done) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  const TreeEnsembleSpec& spec() const { return spec_; }
  bool zero_copy_input() const override { return false; }  // every tree-chunk block stages the X tile
  // Host reads = rows x cols x 8 B x chunks: zero-copy while that stays small.
  bool zero_copy_input_for(int rows, int cols) const override;
  bool bar_input_for(int rows, int cols) const override { (void)cols; return uses_tile(rows); }
  // split batches fold their per-part sums on the host (SCA_TREE_HOST_FOLD=0:
  // in-kernel atomic fold instead): 3.8-4.5 vs 5.0-7.2 us per batch at 4-96
  // rows (profiles/r06i_host_fold)
  int raw_out_cols(int rows, int cols) const override;
  void finish_host(const double* raw, int rows, int raw_cols, double* out) const override;
  bool uses_split(int rows) const;
  // mid-size batches of single-output perfect ensembles: kern::tree_perfect_tile
  bool uses_tile(int rows) const;
  std::shared_ptr<RowModel> clone() const override {
    auto m = std::make_shared<TreeEnsembleModel>(spec_);
    m->fused_reduce_ = fused_reduce_;
    m->whole_max_rows_ = whole_max_rows_;
    return with_meta(m);
  }
  // Launch geometry chosen for a batch (exposed for tests/benchmarks).
  void plan_for(int rows, int* rows_per_block, int* plan_index, int* lds_trees = nullptr) const;
  // In-kernel last-workgroup slab fold for small batches (default off: slower
  // than the two-pass reduce on MI355X, see plan_for).
  void set_fused_reduce(bool on) { fused_reduce_ = on; }
  // Batches up to this many rows of a single-output perfect ensemble run as
  // one whole-ensemble launch (kern::tree_perfect_whole); 0 = never.
  void set_whole_max_rows(int n) { whole_max_rows_ = n; }
  bool uses_whole(int rows) const;

 private:
  bool launch_impl(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s, hipEvent_t done);
  bool uses_fused(int rows) const;
  struct Plan {
    int chunk_trees;
    int n_chunks;
    DeviceBuffer begin, group;
    std::vector<int> h_begin, h_group;
  };
  float tree_value_cpu(int t, const float* x) const;
  TreeEnsembleSpec spec_;
  std::vector<std::unique_ptr<Plan>> plans_;
  DeviceBuffer d_nodes_, d_leaves_, d_sparse_, d_roots_, d_base_;
  int max_chunks_ = 1;
  int device_ = -1;
  bool fused_reduce_ = false;
  int whole_max_rows_ = 256;
};

// ------------------------------------------------------------- elementwise
// sigmoid(mean(row) - threshold): examples/models/mean_classifier.
class MeanSigmoidModel : public RowModel {
 public:
  explicit MeanSigmoidModel(double threshold) : thr_(threshold) {}
  std::string name() const override { return "mean_sigmoid"; }
  int in_cols() const override { return 0; }
  int out_cols(int) const override { return 1; }
  void to_device(int) override {}
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  std::shared_ptr<RowModel> clone() const override { return with_meta(std::make_shared<MeanSigmoidModel>(thr_)); }

 private:
  double thr_;
};

// ------------------------------------------------------- min-max transform
// (X - min) / (max - min) over each request's whole X (0 if constant):
// examples/transformers/mean_transformer/MeanTransformer.py:8-12.
class MinMaxModel : public RowModel {
 public:
  std::string name() const override { return "minmax"; }
  int in_cols() const override { return 0; }
  int out_cols(int c) const override { return c; }
  void to_device(int) override {}
  bool segmented() const override { return true; }
  size_t workspace_bytes(int, int) const override { return 2 * sizeof(double); }
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void launch_segments(const double* X, int rows, int cols, double* out, void* ws, const int32_t* seg, int nseg,
                       hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  std::shared_ptr<RowModel> clone() const override { return with_meta(std::make_shared<MinMaxModel>()); }
};

}  // namespace sca::gpu
