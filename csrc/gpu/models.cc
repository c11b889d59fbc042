#include "models.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace sca::gpu {

// ------------------------------------------------------------------ linear
LinearModel::LinearModel(std::vector<double> W, std::vector<double> b, int C, int K, int act)
    : W_(std::move(W)), b_(std::move(b)), C_(C), K_(K), act_(act) {
  if (int64_t(W_.size()) != int64_t(C) * K) throw std::runtime_error("LinearModel: W size mismatch");
  if (!b_.empty() && int(b_.size()) != C) throw std::runtime_error("LinearModel: b size mismatch");
  if (b_.empty()) b_.assign(size_t(C), 0.0);
  if (act == kern::kActBinaryLogistic && C != 1) throw std::runtime_error("LinearModel: binary logistic needs C == 1");
}

void LinearModel::to_device(int device) {
  dW_.alloc(W_.size() * sizeof(double), device);
  dW_.upload(W_.data(), W_.size() * sizeof(double));
  db_.alloc(b_.size() * sizeof(double), device);
  db_.upload(b_.data(), b_.size() * sizeof(double));
}

void LinearModel::launch(const double* X, int rows, int cols, double* out, void*, hipStream_t s) {
  (void)cols;
  kern::linear_f64(X, rows, K_, dW_.as<double>(), db_.as<double>(), C_, act_, out, s);
}

bool LinearModel::launch_signal(const double* X, int rows, int, double* out, void*, hipStream_t s, hipEvent_t done) {
  if (rows <= 0) return false;  // nothing would be launched to complete `done`
  kern::linear_f64(X, rows, K_, dW_.as<double>(), db_.as<double>(), C_, act_, out, s, done);
  return true;
}

void LinearModel::run_cpu(const double* X, int rows, int, double* out) const {
  std::vector<double> z(static_cast<size_t>(C_));
  const int oc = out_cols(K_);
  for (int r = 0; r < rows; ++r) {
    for (int c = 0; c < C_; ++c) {
      double acc = b_[size_t(c)];
      for (int k = 0; k < K_; ++k) acc = std::fma(X[size_t(r) * K_ + k], W_[size_t(c) * K_ + k], acc);
      z[size_t(c)] = acc;
    }
    double* o = out + size_t(r) * oc;
    switch (act_) {
      case kern::kActIdentity: for (int c = 0; c < C_; ++c) o[c] = z[size_t(c)]; break;
      case kern::kActSoftmax: {
        double m = *std::max_element(z.begin(), z.end()), s = 0;
        for (auto& v : z) { v = std::exp(v - m); s += v; }
        for (int c = 0; c < C_; ++c) o[c] = z[size_t(c)] / s;
        break;
      }
      case kern::kActBinaryLogistic: {
        double p = 1.0 / (1.0 + std::exp(-z[0]));
        o[0] = 1.0 - p;
        o[1] = p;
        break;
      }
      case kern::kActOvr: {
        double s = 0;
        for (auto& v : z) { v = 1.0 / (1.0 + std::exp(-v)); s += v; }
        for (int c = 0; c < C_; ++c) o[c] = z[size_t(c)] / s;
        break;
      }
      default: for (int c = 0; c < C_; ++c) o[c] = 1.0 / (1.0 + std::exp(-z[size_t(c)]));
    }
  }
}

// ------------------------------------------------------------ tree ensemble
static const int kPlanSizes[] = {4, 8, 16, 32, 64, 128, 256, 512};

TreeEnsembleModel::TreeEnsembleModel(TreeEnsembleSpec spec) : spec_(std::move(spec)) {
  // SCA_TREE_FUSED=0/1 forces the single-launch fused-fold plan off / on (A/B runs)
  if (const char* f = std::getenv("SCA_TREE_FUSED")) fused_reduce_ = f[0] == '1';
  // SCA_TREE_WHOLE_ROWS: largest batch served by the single-launch
  // whole-ensemble kernel (0 = off)
  if (const char* f = std::getenv("SCA_TREE_WHOLE_ROWS")) whole_max_rows_ = std::max(0, std::atoi(f));
  const int T = spec_.n_trees;
  if (T <= 0) throw std::runtime_error("TreeEnsembleModel: no trees");
  if (int(spec_.tree_group.size()) != T) spec_.tree_group.assign(size_t(T), 0);
  for (int t = 1; t < T; ++t)
    if (spec_.tree_group[size_t(t)] < spec_.tree_group[size_t(t - 1)])
      throw std::runtime_error("TreeEnsembleModel: trees must be sorted by group");
  if (int(spec_.base_margin.size()) != spec_.groups) spec_.base_margin.resize(size_t(spec_.groups), 0.f);
  if (spec_.depth > 0) {
    const size_t ni = (size_t(1) << spec_.depth) - 1;
    if (spec_.thr.size() != ni * T || spec_.feat.size() != ni * T || spec_.leaves.size() != (ni + 1) * T)
      throw std::runtime_error("TreeEnsembleModel: perfect-tree arrays have wrong size");
  } else {
    if (int(spec_.tree_root.size()) != T) throw std::runtime_error("TreeEnsembleModel: tree_root size mismatch");
  }
  for (int f : spec_.feat)
    if ((f & 0x7fffffff) >= spec_.n_features) throw std::runtime_error("TreeEnsembleModel: feature index out of range");
  for (const auto& n : spec_.nodes) {
    if (n.left >= 0 && ((n.feat & 0x7fffffff) >= spec_.n_features || n.left >= int(spec_.nodes.size()) ||
                        n.right < 0 || n.right >= int(spec_.nodes.size())))
      throw std::runtime_error("TreeEnsembleModel: bad sparse node");
  }
  // Chunk plans: split each group's tree range into chunks of <= S trees.
  for (int S : kPlanSizes) {
    auto p = std::make_unique<Plan>();
    p->chunk_trees = S;
    int t = 0;
    while (t < T) {
      int g = spec_.tree_group[size_t(t)];
      int e = t;
      while (e < T && spec_.tree_group[size_t(e)] == g && e - t < S) ++e;
      p->h_begin.push_back(t);
      p->h_group.push_back(g);
      t = e;
    }
    p->h_begin.push_back(T);
    p->n_chunks = int(p->h_group.size());
    max_chunks_ = std::max(max_chunks_, p->n_chunks);
    plans_.push_back(std::move(p));
  }
}

void TreeEnsembleModel::to_device(int device) {
  device_ = device;
  if (spec_.depth > 0) {
    const size_t n = spec_.thr.size();
    std::vector<kern::TreeNode> packed(n);
    for (size_t i = 0; i < n; ++i) packed[i] = kern::TreeNode{spec_.thr[i], spec_.feat[i]};
    d_nodes_.alloc(n * sizeof(kern::TreeNode), device);
    d_nodes_.upload(packed.data(), n * sizeof(kern::TreeNode));
    d_leaves_.alloc(spec_.leaves.size() * sizeof(float), device);
    d_leaves_.upload(spec_.leaves.data(), spec_.leaves.size() * sizeof(float));
  } else {
    d_sparse_.alloc(spec_.nodes.size() * sizeof(kern::SparseNode), device);
    d_sparse_.upload(spec_.nodes.data(), spec_.nodes.size() * sizeof(kern::SparseNode));
    d_roots_.alloc(spec_.tree_root.size() * sizeof(int), device);
    d_roots_.upload(spec_.tree_root.data(), spec_.tree_root.size() * sizeof(int));
  }
  d_base_.alloc(spec_.base_margin.size() * sizeof(float), device);
  d_base_.upload(spec_.base_margin.data(), spec_.base_margin.size() * sizeof(float));
  for (auto& p : plans_) {
    p->begin.alloc(p->h_begin.size() * sizeof(int), device);
    p->begin.upload(p->h_begin.data(), p->h_begin.size() * sizeof(int));
    p->group.alloc(p->h_group.size() * sizeof(int), device);
    p->group.upload(p->h_group.data(), p->h_group.size() * sizeof(int));
  }
}

// Workspace: [fused-reduce counter | tile-kernel counter at byte 128 |
// split / tile row accumulators from byte 256, up to kSplitMaxRows |
// split-kernel per-row-tile arrival counters from byte 4096 (1024)]
// [chunk partial slab].  The header starts zeroed (DeviceBuffer::alloc) and
// every kernel that uses a counter or accumulator re-zeroes it.
static constexpr size_t kTreeWsHeader = 8192;
static constexpr size_t kSplitCounters = 4096;
static constexpr int kSplitMaxRows = int((kSplitCounters - 256) / sizeof(double));

size_t TreeEnsembleModel::workspace_bytes(int max_rows, int) const {
  // Largest slab any batch size up to max_rows plans for (chunks shrink as
  // batches grow, so this is far below max_chunks x max_rows).
  size_t slab = 0;
  for (int r = 1; r <= std::max(1, max_rows); ++r) {
    int rb, pi;
    plan_for(r, &rb, &pi);
    slab = std::max(slab, size_t(plans_[size_t(pi)]->n_chunks) * size_t(r));
  }
  return kTreeWsHeader + slab * sizeof(double);
}

void TreeEnsembleModel::plan_for(int rows, int* rows_per_block, int* plan_index, int* lds_trees) const {
  // Measured on MI355X (profiles/r01g_tree_variants): a descent costs ~2 us of
  // dependent L2 loads per tree a lane walks, and every extra tree chunk adds
  // slab to fold.  So: few rows per block (more lanes per row = one tree per
  // lane with few chunks), growing with the batch (rows / 16, 2..64), and
  // trees per lane raised only once the grid passes ~2048 workgroups.
  int rb = 1;
  if (rows > 1) {
    rb = 2;
    while (rb * 2 <= rows / 16 && rb < 64) rb <<= 1;
  }
  const int tpr = 256 / rb;
  const int row_tiles = (rows + rb - 1) / rb;
  *rows_per_block = rb;
  // Trees are traversed from global memory (L2-resident across batches).
  // Staging a chunk's trees in LDS (lds_trees) and folding the slab in the
  // partial kernel's last workgroup (fused reduce) are kept as options but
  // measured slower: per-batch time is dominated by per-kernel dispatch +
  // completion and the descent chain, not by where the nodes are read from,
  // and the in-kernel fold's cross-XCD write-through / atomic / reload chain
  // costs more than a second launch.
  if (lds_trees) *lds_trees = 0;
  const long long want = (static_cast<long long>(spec_.n_trees) * row_tiles + 2047) / 2048;
  const int chunk = static_cast<int>(std::max<long long>(tpr, want));
  int idx = int(plans_.size()) - 1;
  for (int i = 0; i < int(plans_.size()); ++i)
    if (plans_[size_t(i)]->chunk_trees >= chunk) { idx = i; break; }
  *plan_index = idx;
}

bool TreeEnsembleModel::uses_whole(int rows) const {
  return spec_.depth > 0 && spec_.groups == 1 && rows <= whole_max_rows_;
}

bool TreeEnsembleModel::uses_split(int rows) const {
  return uses_whole(rows) && kern::tree_split_parts() > 0 &&
         rows <= std::min(kSplitMaxRows, kern::tree_split_max_rows()) && spec_.depth >= 4 && spec_.depth <= 10;
}

static bool tree_host_fold() {
  static const bool v = [] {
    const char* e = std::getenv("SCA_TREE_HOST_FOLD");
    return !e || std::atoi(e) != 0;
  }();
  return v;
}

int TreeEnsembleModel::raw_out_cols(int rows, int) const {
  return tree_host_fold() && uses_split(rows) ? kern::tree_split_parts_for(rows) : 0;
}

// The split kernel's per-part row sums -> the objective transform, exactly as
// the kernels' apply_transform (and run_cpu) state it; parts are added in
// part order, so the result does not depend on which workgroup finished first.
void TreeEnsembleModel::finish_host(const double* raw, int rows, int parts, double* out) const {
  const double base = spec_.base_margin.empty() ? 0.0 : double(spec_.base_margin[0]);
  for (int r = 0; r < rows; ++r) {
    double m = 0.0;
    const double* p = raw + size_t(r) * size_t(parts);
    for (int i = 0; i < parts; ++i) m += p[i];
    m = m * double(spec_.scale) + base;
    double* o = out + size_t(r) * spec_.out_cols;
    switch (spec_.transform) {
      case kern::kTreeSigmoid: o[0] = 1.0 / (1.0 + std::exp(-m)); break;
      case kern::kTreeBinaryProba: {
        const double pr = 1.0 / (1.0 + std::exp(-m));
        o[0] = 1.0 - pr;
        o[1] = pr;
        break;
      }
      case kern::kTreeIsolation: o[0] = -std::exp2(-(m - base)) - base; break;
      default: o[0] = m;  // identity / mean (single group)
    }
  }
}

bool TreeEnsembleModel::uses_tile(int rows) const {
  return uses_whole(rows) && spec_.depth >= 4 && spec_.depth <= 10 && rows <= kSplitMaxRows &&
         rows <= kern::tree_tile_max_rows() && !uses_split(rows);
}

bool TreeEnsembleModel::zero_copy_input_for(int rows, int cols) const {
  // tree tiles: every tree chunk's workgroups re-read the rows -- HBM only
  // (BAR-written, bar_input_for, or DMA'd), never pinned host memory
  if (uses_tile(rows)) return false;
  // whole-ensemble kernel: each workgroup reads its rows once
  if (uses_whole(rows)) return size_t(rows) * size_t(cols) * sizeof(double) <= (256u << 10);
  int rb, pi;
  plan_for(rows, &rb, &pi);
  // Every chunk's workgroups re-read their rows' tile: keep the host traffic of
  // one batch within ~64 KB (one PCIe/IF round trip per workgroup is cheaper
  // than a separate H2D blit launch below that).
  return size_t(rows) * size_t(cols) * sizeof(double) * size_t(plans_[size_t(pi)]->n_chunks) <= (64u << 10);
}

void TreeEnsembleModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  launch_impl(X, rows, cols, out, ws, s, nullptr);
}

bool TreeEnsembleModel::launch_signal(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                                      hipEvent_t done) {
  if (rows <= 0) return false;  // contract: false = nothing launched
  return launch_impl(X, rows, cols, out, ws, s, done);
}

bool TreeEnsembleModel::uses_fused(int rows) const {
  int rb, pi, lt;
  plan_for(rows, &rb, &pi, &lt);
  const Plan& p = *plans_[size_t(pi)];
  return fused_reduce_ && spec_.groups <= kern::kTreeFusedMaxGroups && size_t(rows) * p.n_chunks <= 4096;
}

// `done` (optional): completed by the batch's last kernel; returns whether it was
bool TreeEnsembleModel::launch_impl(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s,
                                    hipEvent_t done) {
  (void)cols;
  if (uses_split(rows)) {
    char* hdr = static_cast<char*>(ws);
    // out holds [rows][parts] part sums (finish_host) when the batcher launches this model itself
    const bool host = raw_output_allowed() && raw_out_cols(rows, cols) > 0;
    kern::tree_perfect_split(X, rows, spec_.n_features, d_nodes_.as<kern::TreeNode>(), d_leaves_.as<float>(),
                             spec_.depth, spec_.cmp_le, spec_.n_trees, kern::tree_split_parts_for(rows),
                             d_base_.as<float>(), spec_.scale, spec_.transform, out, spec_.out_cols,
                             host ? nullptr : reinterpret_cast<double*>(hdr + 256),
                             host ? nullptr : reinterpret_cast<int*>(hdr + kSplitCounters), s, done);
    return done != nullptr;
  }
  if (uses_tile(rows)) {
    char* hdr = static_cast<char*>(ws);
    if (kern::tree_perfect_tile(X, rows, spec_.n_features, d_nodes_.as<kern::TreeNode>(), d_leaves_.as<float>(),
                                spec_.depth, spec_.cmp_le, spec_.n_trees, d_base_.as<float>(), spec_.scale,
                                spec_.transform, out, spec_.out_cols, reinterpret_cast<double*>(hdr + 256),
                                reinterpret_cast<int*>(hdr + 128), s, done))
      return done != nullptr;
  }
  if (uses_whole(rows)) {
    kern::tree_perfect_whole(X, rows, spec_.n_features, d_nodes_.as<kern::TreeNode>(), d_leaves_.as<float>(),
                             spec_.depth, spec_.cmp_le, spec_.n_trees,
                             kern::tree_whole_rows_per_block(spec_.n_trees, rows), d_base_.as<float>(), spec_.scale,
                             spec_.transform, out, spec_.out_cols, s, done);
    return done != nullptr;
  }
  int rb, pi, lt;
  plan_for(rows, &rb, &pi, &lt);
  const Plan& p = *plans_[size_t(pi)];
  int* counter = static_cast<int*>(ws);
  double* partial = reinterpret_cast<double*>(static_cast<char*>(ws) + kTreeWsHeader);
  // Small slabs may fold in the partial kernel's last workgroup (one launch
  // per batch; the tail does <= 16 slab loads per thread) -- off by default,
  // see plan_for.
  if (uses_fused(rows)) {
    const kern::TreeReduceArgs red{counter, p.group.as<int>(), spec_.groups, d_base_.as<float>(), spec_.scale,
                                   spec_.transform, out, spec_.out_cols};
    if (spec_.depth > 0)
      kern::tree_perfect_fused(X, rows, spec_.n_features, d_nodes_.as<kern::TreeNode>(), d_leaves_.as<float>(),
                               spec_.depth, spec_.cmp_le, p.begin.as<int>(), p.n_chunks, rb, partial, red, s, lt,
                               done);
    else
      kern::tree_sparse_fused(X, rows, spec_.n_features, d_sparse_.as<kern::SparseNode>(), d_roots_.as<int>(),
                              spec_.cmp_le, p.begin.as<int>(), p.n_chunks, rb, partial, red, s, done);
    return done != nullptr;
  }
  if (spec_.depth > 0)
    kern::tree_perfect_partial(X, rows, spec_.n_features, d_nodes_.as<kern::TreeNode>(), d_leaves_.as<float>(),
                               spec_.depth, spec_.cmp_le, p.begin.as<int>(), p.n_chunks, rb, partial, s, lt);
  else
    kern::tree_sparse_partial(X, rows, spec_.n_features, d_sparse_.as<kern::SparseNode>(), d_roots_.as<int>(),
                              spec_.cmp_le, p.begin.as<int>(), p.n_chunks, rb, partial, s);
  kern::tree_reduce(partial, rows, p.n_chunks, p.group.as<int>(), spec_.groups, d_base_.as<float>(), spec_.scale,
                    spec_.transform, out, spec_.out_cols, s, done);
  return done != nullptr;
}

float TreeEnsembleModel::tree_value_cpu(int t, const float* x) const {
  auto left = [&](float xv, float thr, int32_t f) {
    if (xv != xv) return f < 0;
    return spec_.cmp_le ? xv <= thr : xv < thr;
  };
  if (spec_.depth > 0) {
    const int ni = (1 << spec_.depth) - 1;
    int idx = 0;
    for (int d = 0; d < spec_.depth; ++d) {
      const size_t o = size_t(t) * ni + idx;
      const int32_t f = spec_.feat[o];
      idx = 2 * idx + (left(x[f & 0x7fffffff], spec_.thr[o], f) ? 1 : 2);
    }
    return spec_.leaves[size_t(t) * (ni + 1) + (idx - ni)];
  }
  int i = spec_.tree_root[size_t(t)];
  while (spec_.nodes[size_t(i)].left >= 0) {
    const auto& n = spec_.nodes[size_t(i)];
    i = left(x[n.feat & 0x7fffffff], n.thr, n.feat) ? n.left : n.right;
  }
  return spec_.nodes[size_t(i)].thr;
}

void TreeEnsembleModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  std::vector<float> x(static_cast<size_t>(cols));
  std::vector<double> m(static_cast<size_t>(spec_.groups));
  for (int r = 0; r < rows; ++r) {
    for (int f = 0; f < cols; ++f) x[size_t(f)] = float(X[size_t(r) * cols + f]);
    std::fill(m.begin(), m.end(), 0.0);
    for (int t = 0; t < spec_.n_trees; ++t) m[size_t(spec_.tree_group[size_t(t)])] += tree_value_cpu(t, x.data());
    for (int g = 0; g < spec_.groups; ++g) m[size_t(g)] = m[size_t(g)] * spec_.scale + spec_.base_margin[size_t(g)];
    double* o = out + size_t(r) * spec_.out_cols;
    switch (spec_.transform) {
      case kern::kTreeSigmoid: o[0] = 1.0 / (1.0 + std::exp(-m[0])); break;
      case kern::kTreeBinaryProba: { double p = 1.0 / (1.0 + std::exp(-m[0])); o[0] = 1 - p; o[1] = p; break; }
      case kern::kTreeSoftmax: {
        double mx = *std::max_element(m.begin(), m.end()), s = 0;
        for (auto& v : m) { v = std::exp(v - mx); s += v; }
        for (int g = 0; g < spec_.groups; ++g) o[g] = m[size_t(g)] / s;
        break;
      }
      case kern::kTreeIsolation: {
        double raw = m[0] - spec_.base_margin[0];
        o[0] = -std::exp2(-raw) - spec_.base_margin[0];
        break;
      }
      default: for (int g = 0; g < spec_.groups; ++g) o[g] = m[size_t(g)];
    }
  }
}

// -------------------------------------------------------------- elementwise
void MeanSigmoidModel::launch(const double* X, int rows, int cols, double* out, void*, hipStream_t s) {
  kern::mean_sigmoid_rows_f64(X, rows, cols, thr_, out, s);
}

void MeanSigmoidModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  for (int r = 0; r < rows; ++r) {
    double s = 0;
    for (int f = 0; f < cols; ++f) s += X[size_t(r) * cols + f];
    out[r] = 1.0 / (1.0 + std::exp(-(s / cols - thr_)));
  }
}

// ------------------------------------------------------------------ minmax
void MinMaxModel::launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) {
  kern::minmax_normalize_f64(X, int64_t(rows) * cols, out, static_cast<double*>(ws), s);
}

void MinMaxModel::launch_segments(const double* X, int, int cols, double* out, void*, const int32_t* seg, int nseg,
                                  hipStream_t s) {
  kern::segment_minmax_f64(X, seg, nseg, cols, out, s);
}

void MinMaxModel::run_cpu(const double* X, int rows, int cols, double* out) const {
  const size_t n = size_t(rows) * cols;
  if (!n) return;
  const auto mm = std::minmax_element(X, X + n);
  const double lo = *mm.first, range = *mm.second - *mm.first;
  for (size_t i = 0; i < n; ++i) out[i] = range == 0.0 ? 0.0 : (X[i] - lo) / range;
}

}  // namespace sca::gpu
