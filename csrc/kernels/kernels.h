// Host-side launch API for the engine's hand-written CDNA4 (gfx950) kernels.
//
// Every launcher is asynchronous on `stream`, allocates nothing, and never
// synchronises (so a caller may capture it into a hipGraph).  Pointers may be
// device memory or host memory mapped into the device address space
// (zero-copy pinned buffers used by the micro-batcher for tiny payloads).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace sca::kern {

// ---------------------------------------------------------------- linear
// out[r, :] = act(X[r, :] . W^T + b), W is [C, K] row-major.
// Reference: servers/sklearnserver/.../SKLearnServer.py:32-42 (predict_proba of
// LogisticRegression / LinearRegression); SURVEY K3.
enum LinearAct : int {
  kActIdentity = 0,      // regression: out [R, C]
  kActSoftmax = 1,       // multinomial logistic regression: out [R, C]
  kActBinaryLogistic = 2,// binary LR (C == 1): out [R, 2] = [1-p, p]
  kActOvr = 3,           // one-vs-rest LR: sigmoid per class, row-normalised
  kActSigmoid = 4,       // independent sigmoid per column
};
// fp64 I/O, fp64 accumulate (parity with sklearn to ~1e-15).
// `stop` (optional): completed by the kernel's own dispatch, replacing a
// hipEventRecord after it.
// Fused device graph of small linear stages (linear_graph.hip): one thread
// per row runs every stage in LDS.  kind 0 = linear (K, C <= 16), 1 = mean
// over n_in inputs; in[] = producer stages (-1 = the request row); out_off =
// the stage's first activation slot; out_cols = its output width (2 for a
// binary logistic stage).
constexpr int kLinearGraphMaxStages = 16;
constexpr int kLinearGraphMaxWidth = 16;
constexpr int kLinearGraphMaxInputs = 8;
constexpr int kLinearGraphMaxSlots = 96;    // activation doubles per row
constexpr int kLinearGraphMaxParams = 4096; // W + b doubles of every stage
struct LinearGraphStage {
  int kind = 0;
  int n_in = 1;
  int in[kLinearGraphMaxInputs] = {};
  int K = 0, C = 0, act = 0;
  int w_off = 0, b_off = -1;
  int out_off = 0, out_cols = 0;
};
size_t linear_graph_lds_bytes(int n_params, int act_slots);
void linear_graph_f64(const double* X, int rows, int cols, const LinearGraphStage* stages, int n_stages,
                      const double* params, int n_params, int act_slots, double* out, hipStream_t stream,
                      hipEvent_t stop = nullptr);

// True when linear_f64 runs this shape on the f64 matrix cores (SCA_LINEAR_MFMA=0 off, =2 forced).
bool linear_uses_mfma(int rows, int K, int C);
void linear_f64(const double* X, int rows, int K, const double* W, const double* b, int C, int act,
                double* out, hipStream_t stream, hipEvent_t stop = nullptr);

// ------------------------------------------------------------ tree ensemble
// Perfect (complete) binary trees of fixed depth D, breadth-first.  Node i of
// tree t: nodes[t * (2^D - 1) + i] = {threshold, feature | (default_left << 31)}.
// Decision (XGBoost semantics): go left iff x[f] < thr, NaN -> default dir.
struct TreeNode {
  float thr;
  int32_t feat;  // bit 31: default-left for missing values
};
// Partial sums per tree chunk: partial[chunk, r] = sum_{t in chunk} leaf.
// chunk_begin has n_chunks + 1 entries (tree index ranges).
// X is the fp64 request matrix [rows, F] (converted to fp32 on load, as
// XGBoost's DMatrix does).  cmp_le: 1 = sklearn `x <= thr`, 0 = XGBoost `x < thr`.
// rows_per_block (1..64, power of two) trades row- vs tree-parallelism.
// lds_trees > 0: chunks hold at most that many trees and are staged in LDS
// (perfect trees of depth <= 10; see tree_lds_max_trees).
void tree_perfect_partial(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves,
                          int depth, int cmp_le, const int* chunk_begin, int n_chunks, int rows_per_block,
                          double* partial, hipStream_t stream, int lds_trees = 0);
// Largest chunk (in trees) whose nodes + leaves fit in LDS next to the
// feature tile for this geometry (0: depth too large for LDS staging).
int tree_lds_max_trees(int depth, int rows_per_block, int F);
// General trees (arbitrary depth): node {thr, feat|flags, left, right}.
struct SparseNode {
  float thr;
  int32_t feat;
  int32_t left;
  int32_t right;
};
// feat bit 31 = default-left; left < 0 marks a leaf (value in thr).
void tree_sparse_partial(const double* X, int rows, int F, const SparseNode* nodes, const int* tree_root,
                         int cmp_le, const int* chunk_begin, int n_chunks, int rows_per_block, double* partial,
                         hipStream_t stream);
// Reduce chunk partials to per-group margins and apply the objective transform.
// chunk_group[c] = output column of chunk c; out [rows, out_cols] fp64.
enum TreeTransform : int {
  kTreeIdentity = 0,      // reg:squarederror
  kTreeSigmoid = 1,       // binary:logistic -> [p]
  kTreeSoftmax = 2,       // multi:softprob
  kTreeBinaryProba = 3,   // binary:logistic as predict_proba -> [1-p, p]
  kTreeMean = 4,          // random forest regression average
  kTreeIsolation = 5,     // isolation forest: 2^(-mean_path / c(n)) score
};
void tree_reduce(const double* partial, int rows, int n_chunks, const int* chunk_group, int groups,
                 const float* base_margin, float scale, int transform, double* out, int out_cols,
                 hipStream_t stream, hipEvent_t stop = nullptr);
// Fused variant: the partial kernel's last workgroup to finish (device-scope
// counter, reset by that workgroup) folds the slab and writes `out` -- one
// launch per batch instead of two.  Used for small slabs (rows x chunks) and
// <= kTreeFusedMaxGroups output groups.  `counter` must start at 0 (it is
// returned to 0 by every launch).
constexpr int kTreeFusedMaxGroups = 16;
struct TreeReduceArgs {
  int* counter;
  const int* chunk_group;
  int groups;
  const float* base_margin;
  float scale;
  int transform;
  double* out;
  int out_cols;
};
void tree_perfect_fused(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, const int* chunk_begin, int n_chunks, int rows_per_block, double* partial,
                        const TreeReduceArgs& red, hipStream_t stream, int lds_trees = 0,
                        hipEvent_t stop = nullptr);
void tree_sparse_fused(const double* X, int rows, int F, const SparseNode* nodes, const int* tree_root, int cmp_le,
                       const int* chunk_begin, int n_chunks, int rows_per_block, double* partial,
                       const TreeReduceArgs& red, hipStream_t stream, hipEvent_t stop = nullptr);
// Single-output perfect-tree ensembles, small batches: one 1024-thread
// workgroup per tile of rows_per_block rows walks every tree, folds in LDS and
// writes the transformed output -- one launch, no slab.  rows_per_block from
// tree_whole_rows_per_block (power of two <= 16, <= 4 trees per thread).
int tree_whole_rows_per_block(int n_trees, int rows);
// lookahead (depth 8): 10 x levels per round + trees per iteration of the
// lookahead descent (21 .. 42), 0 = the level-by-level descent, -1 =
// SCA_TREE_LOOKAHEAD (default 0).
// The whole-ensemble small-batch kernel with each row tile's trees split
// over `parts` workgroups (one fp64 atomic per row and part into acc, the
// last workgroup transforms and writes the rows and re-zeroes acc[0..rows)
// and *counter).  acc and counter must be zero before the first launch.
// SCA_TREE_SPLIT / SCA_TREE_SPLIT_ROWS set the serving default (8 parts for
// batches of up to 32 rows); depths 4..10.
int tree_split_parts();
int tree_split_parts_for(int rows);  // workgroups per row tile for a batch (0 = no split)
int tree_split_max_rows();
// Tree-major tiles for mid-size batches (single output, depth 4..10): one
// launch, trees staged in LDS per row tile, atomic row fold (acc / counter as
// tree_perfect_split).  Returns false when the shape does not apply.
bool tree_perfect_tile(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                       int cmp_le, int n_trees, const float* base_margin, float scale, int transform, double* out,
                       int out_cols, double* acc, int* counter, hipStream_t stream, hipEvent_t stop = nullptr);
int tree_tile_max_rows();  // SCA_TREE_TILE_ROWS (default 0 = off)
void tree_perfect_split(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, int n_trees, int parts, const float* base_margin, float scale, int transform,
                        double* out, int out_cols, double* acc, int* counter, hipStream_t s,
                        hipEvent_t stop = nullptr);
void tree_perfect_whole(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, int n_trees, int rows_per_block, const float* base_margin, float scale,
                        int transform, double* out, int out_cols, hipStream_t stream, hipEvent_t stop = nullptr,
                        int lookahead = -1);

// ------------------------------------------------------------ combiners
// out = mean over N inputs (each [n] fp64). inputs: device array of pointers.
void combine_mean_f64(const double* const* inputs, int n_inputs, int64_t n, double* out, hipStream_t stream);
// out = mean over k slabs base[j*n : (j+1)*n] (gathered replica outputs).
void combine_mean_strided_f64(const double* base, int k, int64_t n, double* out, hipStream_t stream);
// One wave idling `us` microseconds (capped at 100 ms) on `stream`: test knob for a slow model.
void device_delay_us(int us, hipStream_t stream);
// Per-segment (request) global min-max normalisation; seg = nseg+1 row offsets.
void segment_minmax_f64(const double* in, const int32_t* seg, int nseg, int cols, double* out, hipStream_t stream);
// Decoded HWC uint8 image -> centre crop (bilinear up-size of short axes) -> CHW fp32.
void crop_resize_chw_u8(const uint8_t* img, int H, int W, int C, int crop, float* out, hipStream_t stream);
// relu(x * scale[c] + shift[c]) over a bf16 [N, C, H, W] activation stored
// NCHW or (channels_last) NHWC; needs C % 8 == 0 (NHWC) or H*W % 8 == 0 (NCHW).
bool scale_shift_relu_bf16_ok(int C, int HW, int channels_last);
// relu(a + b) over n bf16 elements (n % 8 == 0, 16-byte aligned buffers).
void add_relu_bf16(const void* a, const void* b, size_t n, void* out, hipStream_t stream);
void scale_shift_relu_bf16(const void* x, const float* scale, const float* shift, int N, int C, int HW,
                           int channels_last, void* out, hipStream_t stream);
// ------------------------------------------------------------ fused MLP
// A whole dense network (and the VAE outlier detector's encoder -> MC
// reparameterised decoder -> reconstruction-MSE loop) in one launch: a
// A workgroup of 4 or 8 waves owns a 16-row tile, keeps every activation in
// LDS and runs each Dense layer on f32-input MFMA (v_mfma_f32_16x16x4_f32:
// exact fp32 products, i.e. Keras/torch float32 numerics) with bias +
// activation fused into the epilogue.  Weights are transposed, zero-padded to
// Kp % 16 == 0, Np % 16 == 0 and packed fragment-major
// ([Np/16][Kp/16][64][4] floats: one 16-byte load per lane feeds four MFMAs),
// so the K loop has no bounds checks and every B load is a coalesced 1 KiB.
enum MlpOpType : int { kMlpDense = 0, kMlpDenseMse = 1, kMlpReparam = 2 };
enum MlpAct : int { kMlpIdentity = 0, kMlpRelu = 1, kMlpSigmoid = 2, kMlpTanh = 3 };
struct MlpOp {
  int type, act;
  int in_buf, out_buf;
  int K, Kp, N, Np;        // Reparam: N = latent dim (input holds [mean | log_var])
  long long w_off, b_off;  // float offsets into the parameter blob
  long long wb_off;        // bf16 precision: offset (elements) into the bf16 weight blob
  int Kpb, Npb;            //   its K / N padded to 32
};
constexpr int kMlpMaxOps = 24;
constexpr int kMlpMaxBufs = 6;
constexpr int kMlpRows = 16;  // rows per workgroup (one MFMA tile)
struct MlpProgram {
  int n_pre = 0, n_loop = 0, loops = 0;  // ops[0, n_pre) once; ops[n_pre, n_pre + n_loop) `loops` times
  int F = 0, Fp = 0;                     // input width (buffer 0 keeps the input tile)
  int buf_off[kMlpMaxBufs] = {}, buf_ld[kMlpMaxBufs] = {};
  int out_buf = 0, out_dim = 0, out_softmax = 0;
  int mse_mode = 0, mse_dim = 0;         // 1: out[r] = mean over loops of mean_c (recon - x)^2
  int lds_floats = 0;
  int waves = 4;                         // workgroup = 64 * waves threads
  MlpOp ops[kMlpMaxOps];
};
void mlp_forward(const double* X, int rows, const MlpProgram& prog, const float* params, uint64_t seed,
                 uint64_t offset, double* out, hipStream_t stream);

// Layer-wise path for batches too small to fill the chip with one workgroup
// per 16-row tile: one launch per Dense layer, one wave per 16x16 output tile
// (grid = row tiles x column tiles), activations round-trip through an
// L2-resident fp32 workspace (the fp64 request rows are converted once).  Same packed weights and k permutation as the
// fused kernel.  A VAE's MC decodes run as one batch of rows x samples rows
// (sample-major): the first decoder layer draws z = mu + exp(lv / 2) eps on
// the fly from the same Philox streams as the fused kernel, the last one
// reduces (act(y) - x)^2 into per-row sums.
struct MlpLayerArgs {
  const float* W = nullptr;  // packed fragment-major [Np/16][Kp/16][64][4]
  const float* bias = nullptr;
  int K = 0, Kp = 0, N = 0, Np = 0, act = 0;
  const float* A = nullptr;  // A = fp32 activations [rows_eff][lda] ...
  int lda = 0;
  const float* H = nullptr;  // ... or a VAE head [rows][ldh] = [mu | log_var] (reparameterised A)
  int ldh = 0, latent = 0;
  uint64_t key = 0;
  int rows = 0;      // request rows (X, H)
  int rows_eff = 0;  // rows x samples on decoder layers, else rows
  float* O = nullptr;    // fp32 out [rows_eff][ldo], columns >= N zeroed
  int ldo = 0;
  float* mse = nullptr;  // if set: MSE epilogue against xref [rows][ldx], sums into mse[row % rows]
  const float* xref = nullptr;
  int ldx = 0;
};
void mlp_layer(const MlpLayerArgs& a, hipStream_t stream);

// Large-batch layer GEMM (csrc/kernels/gemm.hip): one wave per 64 x (16 TN)
// output tile straight from L2 -- no LDS -- so each 16-B B fragment feeds 4
// MFMAs (4 row tiles) and each A fragment TN: 4x the operand reuse of the
// 16x16-per-wave layer kernel.  Two operand types:
//   fp32: A fp32 [rows][lda], W packed as for mlp_layer (v_mfma_f32_16x16x4_f32)
//   bf16: A bf16 [rows][lda], W bf16 row-major [Np][Kp], Kp % 64 == 0 and
//         Np % 64 == 0 (zero padded); LDS-tiled 128 x 128 workgroup tiles on
//         v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
// Epilogue: + bias, activation, store fp32 or bf16 (columns >= N zeroed), or
// the VAE's MSE reduction.  AMODE 2 = VAE reparameterised A (as mlp_layer).
struct DenseGemmArgs {
  int bf16 = 0;
  const void* W = nullptr;
  const float* bias = nullptr;
  int K = 0, Kp = 0, N = 0, Np = 0, act = 0;
  const void* A = nullptr;
  int lda = 0;
  int a_f64 = 0;
  int xcd_remap = 1;  // bf16 path: XCD-aware tile order (set by dense_gemm)
  // bf16 path, N <= 16: write the model output (fp64) straight from the
  // epilogue -- mode 0 plain [rows][N], 1 row softmax, 2 binary [1 - p, p] --
  // instead of fp32 logits + mlp_finish (one launch and a round trip less)
  double* out64 = nullptr;
  int out_mode = 0;
  // fp32: W is row-major [Np][Kp] (Kp % 32 == 0, Np % 64 == 0, zero padded) and A rows hold Kp
  // readable floats -- the LDS-tiled exact-fp32 MFMA kernel instead of the fragment-packed one
  int lds_f32 = 0;
  int n_store = 0;  // LDS-tiled paths: output columns to store (0 = Np); the rest of the padded tile is dropped  // bf16 path: A is the fp64 request batch [rows][lda], K = lda (converted while staging)
  const float* H = nullptr;
  int ldh = 0, latent = 0;
  uint64_t key = 0;
  int rows = 0, rows_eff = 0;
  void* O = nullptr;
  int ldo = 0, o_f32 = 1;
  float* mse = nullptr;
  const float* xref = nullptr;
  int ldx = 0;
  int group_m = 0;  // glds-family bf16 GEMMs: tile rows per L2 group (0: SCA_GEMM_GROUP_M, default 4; 1 = row-major)
  int path = 0;  // bf16 plain A: 0 auto, 1 register-staged LDS kernel, 2 glds ring 128^2, 3 glds 256^2, 4 8-phase, 5 4-wave, 6 8-phase spread reads, 7 / 8 ablations, 9 8-phase spread + 10-half-tile ring (tests / benches)
};
void dense_gemm(const DenseGemmArgs& a, hipStream_t stream);
// fp64 rows [rows][F] -> bf16 [rows][ld], zero-padded columns
void convert_bf16(const double* X, int rows, int F, int ld, void* out, hipStream_t stream);
// fp64 rows [rows][F] -> fp32 [rows][ld], zero-padded columns
void mlp_convert(const double* X, int rows, int F, int ld, float* out, hipStream_t stream);
// logits [rows][ld] -> out: mode 0 plain [rows][n], 1 row softmax, 2 binary [1 - p, p]
void mlp_finish(const float* logits, int ld, int rows, int n, int mode, double* out, hipStream_t stream);
// out[r] = mse[r] * scale
void mlp_mse_finish(const float* mse, int rows, double scale, double* out, hipStream_t stream);

// Mahalanobis detector: Sherman-Morrison recurrence + scores over a batch
// (B [nb][k][k], cov0 [k][k], xd [nb][k]); false if k > 16.
// Whole Mahalanobis detector step on the device (CoreMahalanobis.py:68-151):
// clip, running mean / covariance update, top-k eigenvectors (one-wave
// Householder tridiagonalisation + Sturm multisection + inverse iteration in
// LDS), projections, Sherman-Morrison scores, state update -- one
// single-workgroup launch per request batch, state resident in HBM.
constexpr int kMahaMaxP = 64;
constexpr int kMahaMaxK = 16;
struct MahaParams {
  int p = 0, k = 0;
  double n_stdev = 3.0, start_clip = 50.0, max_n = -1.0, eps = 1e-8;
  int out_mode = 0;        // 0: scores, 1: predictions (score > threshold ? 1 : 0)
  double threshold = 25.0;
  // the 256-thread kernel splits the tridiagonalisation's per-column sweep
  // over its 4 waves from this p on (SCA_MAHA_MW_MIN_P; > 64 = never).
  // Measured: p = 64 87.0 -> 74.9 us, p = 32 30.5 -> 32.3 us, p = 20 16.1 ->
  // 19.8 us (the two barriers per column cost more than a short sweep saves)
  int mw_min_p = 48;
  // p <= jacobi_max_p: warm-started cyclic Jacobi (one wave) instead of the
  // Householder / Sturm / inverse-iteration path (SCA_MAHA_JACOBI_MAX_P,
  // 0 = never)
  int jacobi_max_p = 32;
  // p <= rank1_max_p: eigen-tracking -- a one-row step updates the cached
  // full eigendecomposition by the rank-1 secular equation (O(p^2) roots +
  // one p^3 basis product) with a residual check; Jacobi re-seeds it when
  // the check or the cache fails (SCA_MAHA_RANK1_MAX_P, 0 = never)
  int rank1_max_p = 64;
};
// state layout (doubles): mean[p] | C[p*p] | clip_lo[p] | clip_hi[p] | n | c_zero | has_clip
inline size_t maha_state_doubles(int p) { return size_t(p) * (p + 3) + 3; }
// workspace doubles for a batch of nb rows
inline size_t maha_ws_doubles(int nb, int p, int k) { return size_t(nb) * (4 * size_t(p) + 2 * size_t(k)); }
// eig: kMahaEigDoubles doubles, zero-initialised: the first kMahaMaxP^2 hold
// the last step's eigenvectors, sorted by descending eigenvalue (the Jacobi
// path's warm start and the eigen-tracking basis; a cache, not part of the
// checkpointed state), then the tail, the eigenvalues (kMahaEigLam) and the
// meta block (kMahaEigMeta: [state n the cache describes, eigen-tracking
// steps, eigen-tracking fallbacks, Jacobi sweeps, Jacobi solves]).
// Tail: [p of the cached eigenvectors, warm steps since the last cold start,
// eigen-phase shader cycles, steps, eigen-phase 100 MHz ticks,
// phase us x 10]: clip, cov, eigen.eigenvectors (twisted factorisation),
// eigen (total), projections, Sherman-Morrison, state update,
// eigen.tridiagonalise, eigen.eigenvalues (multisection),
// eigen.back-transformation.
constexpr int kMahaEigTail = kMahaMaxP * kMahaMaxP;
constexpr int kMahaEigLam = kMahaEigTail + 16;
constexpr int kMahaEigMeta = kMahaEigLam + kMahaMaxP;
constexpr int kMahaEigDoubles = kMahaEigMeta + 8;
void maha_step(const double* X, int nb, const MahaParams& prm, double* state, double* eig, double* ws, double* scores,
               hipStream_t stream);
// Several request batches in order (seg: nseg + 1 row offsets, device-visible):
// one launch steps the state through each request exactly as nseg maha_step
// calls would; ws is sized for the largest segment.
void maha_step_segments(const double* X, const int32_t* seg, int nseg, const MahaParams& prm, double* state,
                        double* eig, double* ws, double* out, hipStream_t stream);
bool mahalanobis_sm_scores(const double* B, const double* cov0, const double* xd, int nb, int k, double n, double* out,
                           hipStream_t stream);

// dst[0..3] = {a, b, c, d} (device-side header for fabric transfers).
void fill_i32x4(int32_t* dst, int a, int b, int c, int d, hipStream_t stream);
// Row softmax / argmax over [rows, C].
void softmax_rows_f64(const double* in, int rows, int C, double* out, hipStream_t stream);
void argmax_rows_f64(const double* in, int rows, int C, int32_t* out, hipStream_t stream);
// Global min-max normalisation (examples/transformers/mean_transformer).
void minmax_normalize_f64(const double* in, int64_t n, double* out, double* scratch2, hipStream_t stream);
// sigmoid(mean(row) - threshold)  (examples/models/mean_classifier).
void mean_sigmoid_rows_f64(const double* in, int rows, int F, double threshold, double* out, hipStream_t stream);

// ------------------------------------------------------------ bandits
// Epsilon-greedy route for `n` requests given the current best branch
// (components/routers/epsilon-greedy/EpsilonGreedy.py:87-106).
void eg_route(const int32_t* best_branch, int n_branches, float epsilon, uint64_t seed, uint64_t offset, int n,
              double* branch_out, hipStream_t stream);
// Thompson sampling: sample Beta(a_i, b_i), argmax (ThompsonSampling.py:78-91).
void ts_route(const float* alpha, const float* beta, int n_branches, uint64_t seed, uint64_t offset, int n,
              double* branch_out, hipStream_t stream);

// ------------------------------------------------------------------ LSTM
// Seq2seq LSTM reconstruction error (seq2seq outlier detector, reference
// components/outlier-detection/seq2seq-lstm/model.py:6-92 and
// CoreSeq2SeqLSTM.py:107-174): bidirectional LSTM encoder stack, LSTM decoder
// stack initialised with the concatenated final encoder states, Dense output,
// T-1 step greedy decode, per-sequence MSE.  One persistent kernel per batch
// (csrc/kernels/lstm.hip).
constexpr int kLstmMaxLayers = 4;
constexpr int kLstmRows = 16;  // sequences per workgroup (one MFMA tile)
struct LstmCell {              // one direction of one layer
  int w_off = 0, b_off = 0;    // floats, relative to the phase blob: B fragments [Np/16][Kp/4][64], bias [Np]
  int in = 0, H = 0, Kp = 0, Np = 0;
  int lda = 0, ldg = 0;        // LDS strides of its A [16][lda] and gate [16][ldg] buffers
  int a_off = 0, g_off = 0, c_off = 0;  // LDS offsets (floats) of A, gates, cell state [16][H]
};
struct LstmProgram {
  int T = 0, F = 0, n_enc = 0, n_dec = 0;
  LstmCell enc[kLstmMaxLayers][2];
  LstmCell dec[kLstmMaxLayers];
  long long enc_phase[kLstmMaxLayers] = {};  // global offsets (floats) of each encoder layer's blob
  int enc_phase_floats[kLstmMaxLayers] = {};
  long long dec_phase = 0;
  int dec_phase_floats = 0;
  int dense_w = 0, dense_b = 0;  // relative to the decoder blob: W fragments [Np/16][Kp/4][64], b [F]
  int dense_kp = 0, dense_np = 0;
  int D = 0, out_act = 0;        // decoder top units; 0 linear, 1 sigmoid, 2 tanh, 3 relu
  int w_lds = 0;                 // stage each phase's weights in LDS
  int w_region = 0;              // LDS floats reserved for weights (0 when !w_lds)
  int y_off = 0, mse_off = 0;    // LDS offsets: dense inputs staged, mse [16]
  int x_lds = 0, x_off = 0;      // input tile [16][T][F] (fp32) staged in LDS when it fits
  int lds_floats = 0;
  long long seq_ws_floats = 0;   // per-workgroup global workspace (encoder sequences, ping-pong)
  int Hmax2 = 0;                 // 2 x widest encoder layer
};
void lstm_seq2seq_mse(const double* X, int rows, const LstmProgram& prog, const float* params, float* ws,
                      double* out, hipStream_t stream);

// Small-batch form of the same model (csrc/kernels/lstm_valu.hip): one
// workgroup per 1..4 sequences, every gate row's weights resident in VGPRs
// (4 gates x KPL per lane, Q lanes per unit, DPP group sums), the step's
// [x | h] vector double-buffered in LDS -- one barrier per encoder step, one
// per decoder layer + one for the Dense feedback per decoder step.  Used when
// rows / CUs <= 4 (a 1-sequence request no longer pays the 16-row MFMA tile's
// dependent MFMA chains).
constexpr int kLstmvMaxRows = 4;
struct LstmvCell {
  int in = 0, H = 0, Q = 0, Kv = 0;  // Kv = Q * KPL (the v row, zero padded past in + H)
  int lane0 = 0;                     // first thread of the cell (multiple of 64)
  long long w_off = 0;               // global floats: [H][Q][4][KPL]
  long long b_off = 0;               // global floats: [4][H] (i, f, g, o)
  int v_off = 0;                     // LDS floats: v[2][R][Kv]
};
struct LstmvProgram {
  int ok = 0;
  int T = 0, F = 0, n_enc = 0, n_dec = 0, R = 0, KPL = 0, threads = 0;
  LstmvCell enc[kLstmMaxLayers][2];
  LstmvCell dec[kLstmMaxLayers];
  int D = 0, Qy = 0, y_lane0 = 0, out_act = 0;  // Dense: F outputs x Qy lanes, KPL weights each
  long long yw_off = 0, yb_off = 0;            // global floats: [F][Qy][KPL], [F]
  int x_off = 0;                               // LDS: input rows [R][T][F] fp32
  int seq_off[2] = {0, 0}, seq_ld = 0;         // LDS: encoder output sequences [R][T][seq_ld] (n_enc > 1)
  int hfin_off = 0, cfin_off = 0;              // LDS: final encoder h / c [R][2 He]
  int mse_off = 0;                             // LDS: [R]
  int lds_floats = 0;
};
void lstm_valu_mse(const double* X, int rows, const LstmvProgram& prog, const float* params, double* out,
                   hipStream_t stream);

}  // namespace sca::kern
