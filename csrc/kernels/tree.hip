// Tree-ensemble inference (reference
// servers/xgboostserver/xgboostserver/XGBoostServer.py:10-26 — xgboost
// Booster.predict on the CPU — and sklearn IsolationForest / RandomForest).
//
// CDNA4 mapping.  A 256-thread workgroup owns a tile of RB request rows and a
// contiguous chunk of trees (grid = row tiles x tree chunks, so even a batch of
// one row fills the chip with tree-parallel work):
//   thread i -> row (i % RB), tree slot (i / RB), stride 256 / RB
// The RB x F feature tile is staged once in LDS as fp32 (XGBoost's DMatrix
// precision), so the per-level `x[feature]` gather is an LDS read; node records
// are 8 bytes ({thr, feat|default_left}) laid out breadth-first per tree so a
// perfect tree of depth D needs no child pointers (child = 2i + 1 + right) and
// the whole 1000 x depth-8 model (2 MiB nodes + 1 MiB leaves) stays resident in
// each XCD's 4 MiB L2 across batches.  Per-row partial sums over the thread's
// trees are reduced through LDS and written to a [chunk, row] slab that
// tree_reduce folds (deterministic, no float atomics).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>

#include "kernels.h"

#include <type_traits>

namespace sca::kern {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxLdsFloats = 12288;  // 48 KiB feature tile

__device__ __forceinline__ bool go_left(float x, float thr, int32_t feat, int cmp_le) {
  if (x != x) return feat < 0;  // missing value -> default direction (bit 31)
  return cmp_le ? (x <= thr) : (x < thr);
}

// Feature-major LDS tile: feature f of tile row r lives at tile[f * RB + r]
// (RB = rows per block, a power of two; lrb = log2 RB).  A ds_read_b32 banks
// on (addr / 4) % 32 per 32-lane half, and the lanes of a half read 32
// different rows, so a level's reads hit 32 distinct banks whatever feature
// each lane's node tests.  (A row-major tile with F = 32 folded every lane
// onto one bank at the root and stayed 2..32-way below it: 92.9% of LDS
// cycles were bank conflicts, profiles/r01l_pmc.)
__device__ __forceinline__ float tile_x(const float* xs, int32_t feat, int lrb) {
  return xs[(feat & 0x7fffffff) << lrb];
}

// Stage the RB x F feature tile (fp64 -> fp32) into LDS, feature-major.
// Consecutive threads take consecutive rows of one feature, so the LDS
// writes are consecutive addresses (conflict-free); rows past `rows` are
// zero-filled so every thread can traverse unconditionally.  Loads are issued
// kU at a time into registers before any LDS write (one round trip).
template <int BS = kBlock>
__device__ __forceinline__ void stage_tile(float* tile, const double* __restrict__ X, int row0, int rows, int RB,
                                           int lrb, int F) {
  constexpr int kU = 8;
  const int n = RB * F, nrow = min(RB, rows - row0);
  for (int i0 = threadIdx.x; i0 < n; i0 += BS * kU) {
    double v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // branch-free: clamped address, select after the load
      const int i = min(i0 + u * BS, n - 1);
      const int r = i & (RB - 1), f = i >> lrb;
      const double x = X[size_t(row0 + min(r, nrow - 1)) * F + f];
      v[u] = r < nrow ? x : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * BS;
      if (i < n) tile[i] = float(v[u]);
    }
  }
}

// U perfect-tree descents interleaved: the U node loads of a level are
// independent, so a lane keeps U L2 (or LDS) round trips in flight instead of
// one.  The descent is a chain of D dependent loads per tree -- at 4096 rows x
// 1000 trees x depth 8 a lane walking its 8 trees one after the other spent
// 85% of its cycles waiting on that chain (profiles/r02a_tree).  Invalid
// slots (past the chunk end) walk tree t0 and contribute 0.
template <int D, int U, bool STAGED>
__device__ __forceinline__ double descend_perfect(const TreeNode* __restrict__ nodes, const float* __restrict__ leaves,
                                                 int n_internal, int depth, int t, int t1, int tstride, int tfirst,
                                                 const float* xs, int lrb, const double* __restrict__ xg, int cmp_le) {
  const TreeNode* tn[U];
  const float* lf[U];
  bool ok[U];
  int idx[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int tu = t + u * tstride;
    ok[u] = tu < t1;
    const int tt = ok[u] ? tu : tfirst;
    tn[u] = nodes + size_t(tt) * n_internal;
    lf[u] = leaves + size_t(tt) * (n_internal + 1);
    idx[u] = 0;
  }
  auto level = [&]() {
    TreeNode nd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) nd[u] = tn[u][idx[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float x = STAGED ? tile_x(xs, nd[u].feat, lrb) : float(xg[nd[u].feat & 0x7fffffff]);
      idx[u] = 2 * idx[u] + (go_left(x, nd[u].thr, nd[u].feat, cmp_le) ? 1 : 2);
    }
  };
  if constexpr (D > 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) level();
  } else {
    for (int d = 0; d < depth; ++d) level();
  }
  double acc = 0.0;  // fp64 sums of fp32 leaves: nearly order-free (see reduce_write)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float v = lf[u][idx[u] - n_internal];
    acc += ok[u] ? double(v) : 0.0;
  }
  return acc;
}

// Contiguous global -> LDS copy with gfx950 direct-to-LDS loads
// (global_load_lds_dwordx4: each lane's 16 B land at M0 + lane * 16, no VGPR
// round trip, all loads in flight at once).  Falls back to dword granules when
// the source or size is not 16 B aligned.  Caller waits (vmcnt) + barriers.
__device__ __forceinline__ void copy_to_lds(void* lds_dst, const void* gsrc, int bytes) {
  typedef __attribute__((address_space(1))) const void* gptr;
  typedef __attribute__((address_space(3))) void* lptr;
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63, stride = kBlock;
  char* dst = static_cast<char*>(lds_dst);
  const char* src = static_cast<const char*>(gsrc);
  if (((reinterpret_cast<uintptr_t>(gsrc) | uintptr_t(bytes)) & 15) == 0) {
    const int n = bytes >> 4;
    for (int base = wave * 64; base < n; base += stride)
      if (base + lane < n)
        __builtin_amdgcn_global_load_lds((gptr)(src + size_t(base + lane) * 16), (lptr)(dst + size_t(base) * 16), 16,
                                         0, 0);
  } else {
    const int n = bytes >> 2;
    for (int base = wave * 64; base < n; base += stride)
      if (base + lane < n)
        __builtin_amdgcn_global_load_lds((gptr)(src + size_t(base + lane) * 4), (lptr)(dst + size_t(base) * 4), 4, 0,
                                         0);
  }
}

// Reduce per-thread accumulators of the same row and write the slab row.
// Lanes of one row sit RB apart inside a wave: a butterfly (shfl_xor over
// offsets 32..RB) leaves each wave's per-row sums in lanes 0..RB-1, and the
// four waves' sums are added from LDS -- O(log) steps instead of a serial
// 256 / RB-long LDS walk by one lane (6 us at RB = 1).
// COHERENT: the slab is read back inside the same launch by the fused tail on
// another XCD, so rows are written with agent-scope (sc1, write-through past
// this XCD's L2) stores -- no whole-L2 writeback/invalidate fences needed.
// Accumulators and the slab are fp64: while the fp32 leaves of a row's trees
// span at most ~29 binades (53 - 24 bits, less log2(trees) of headroom) their
// fp64 sums carry no rounding, so the result does not depend on how trees
// were chunked or rows grouped and a row scores the same in a batch of 1 or
// 4096.  Models whose late trees have leaves far below the early ones can
// exceed that span; their scores are then nearly, not exactly, order-free
// across batch sizes (the chunk plan follows the batch size).
template <bool COHERENT>
__device__ __forceinline__ void reduce_write(double* red, double acc, int RB, int row0, int rows, int chunk,
                                             double* __restrict__ partial) {
  for (int off = 32; off >= RB; off >>= 1) acc += __shfl_xor(acc, off, 64);
  const int lane = int(threadIdx.x) & 63, wave = int(threadIdx.x) >> 6;
  if (lane < RB) red[wave * RB + lane] = acc;
  __syncthreads();
  if (int(threadIdx.x) < RB) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += red[w * RB + threadIdx.x];
    const int r = row0 + threadIdx.x;
    if (r < rows) {
      if constexpr (COHERENT)
        __hip_atomic_store(partial + size_t(chunk) * rows + r, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        partial[size_t(chunk) * rows + r] = s;
    }
  }
}

// Objective transform of one row's margins m[0..groups) (scale and base
// margin applied here) -> o.  G > 0: loops are unrolled to G with a guard so
// a caller's register array m[G] stays in VGPRs (no scratch); G == 0: generic.
#define SCA_FOR_G(g) _Pragma("unroll") for (int g = 0; g < (G ? G : groups); ++g) if (G == 0 || g < groups)
template <int G>
__device__ __forceinline__ void apply_transform(double* m, int groups, int transform, float scale,
                                                const float* base_margin, double* o) {
  SCA_FOR_G(g) m[g] = m[g] * double(scale) + (base_margin ? double(base_margin[g]) : 0.0);
  switch (transform) {
    case kTreeSigmoid: o[0] = 1.0 / (1.0 + exp(-m[0])); break;
    case kTreeBinaryProba: {
      const double p = 1.0 / (1.0 + exp(-m[0]));
      o[0] = 1.0 - p;
      o[1] = p;
      break;
    }
    case kTreeSoftmax: {
      double mx = m[0];
      SCA_FOR_G(g) mx = fmax(mx, m[g]);
      double s = 0.0;
      SCA_FOR_G(g) { m[g] = exp(m[g] - mx); s += m[g]; }
      SCA_FOR_G(g) o[g] = m[g] / s;
      break;
    }
    case kTreeIsolation: {
      // m = mean path length / c(max_samples) (scale folds both); base = offset
      const double raw = m[0] - (base_margin ? double(base_margin[0]) : 0.0);
      o[0] = -exp2(-raw) - (base_margin ? double(base_margin[0]) : 0.0);
      break;
    }
    default:
      SCA_FOR_G(g) o[g] = m[g];
  }
}
#undef SCA_FOR_G

// Last-workgroup-reduces tail of the fused kernels.  Every workgroup has
// written its slab rows with write-through agent-scope stores; it waits for
// them to complete (s_waitcnt), then one lane bumps the device-scope counter.
// The workgroup that brings it to the grid size folds the slab -- read with
// agent-scope loads that bypass stale L2 lines -- in fixed chunk order
// (deterministic, no float atomics) and rearms the counter.  A __threadfence()
// here would instead emit buffer_wbl2 + buffer_inv on every workgroup, which
// flushes each XCD's L2 and evicts the resident tree model (measured 15 us vs
// ~6 us per launch).  The fold uses the whole workgroup: RB rows x (256 / RB)
// chunk lanes, lanes combined through LDS per group.
__device__ __forceinline__ double coherent_load(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void fused_tail(const double* partial, int rows, int n_chunks, const TreeReduceArgs& red) {
  __shared__ int s_last;
  __shared__ double s_fold[kBlock];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slab stores acknowledged at the coherence point
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(red.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             int(gridDim.x * gridDim.y) - 1;
  __syncthreads();
  if (!s_last) return;
  int RB = 1;
  while (RB < rows && RB < kBlock) RB <<= 1;
  const int r_local = int(threadIdx.x) & (RB - 1), slot = int(threadIdx.x) / RB, tpr = kBlock / RB;
  // Per-group margins are folded into the output row itself (out_cols >=
  // groups for every objective) and transformed in place, so the tail adds no
  // register pressure to the traversal part of the kernel.
  for (int row0 = 0; row0 < rows; row0 += RB) {
    const int r = row0 + r_local;
    double* o = red.out + size_t(r) * red.out_cols;
    for (int g = 0; g < red.groups; ++g) {
      double acc = 0.0;
      if (r < rows) {
        if (red.groups == 1) {  // common case: unconditional, unrolled loads (ILP across the slab)
#pragma unroll 4
          for (int c = slot; c < n_chunks; c += tpr) acc += double(coherent_load(partial + size_t(c) * rows + r));
        } else {
          for (int c = slot; c < n_chunks; c += tpr)
            if (red.chunk_group[c] == g) acc += double(coherent_load(partial + size_t(c) * rows + r));
        }
      }
      if (tpr > 1) {
        s_fold[threadIdx.x] = acc;
        __syncthreads();
        if (slot == 0)
          for (int j = 1; j < tpr; ++j) acc += s_fold[j * RB + r_local];
        __syncthreads();
      }
      if (slot == 0 && r < rows) o[g] = acc;
    }
    if (slot == 0 && r < rows) apply_transform<0>(o, red.groups, red.transform, red.scale, red.base_margin, o);
  }
  if (threadIdx.x == 0) __hip_atomic_store(red.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// TREES_LDS: the chunk's trees (nodes + leaves, contiguous in HBM) are copied
// into LDS with wide coalesced loads before traversal, so each of the D + 1
// dependent loads of a descent is a ds_read (~100 cycles) instead of an L2/MALL
// round trip (~1 us): one memory round trip per workgroup instead of D + 1 per
// tree.  The host caps the chunk at what fits (lds_trees trees).
template <int D, bool FUSED, bool TREES_LDS>
__global__ __launch_bounds__(kBlock) void perfect_partial(const double* __restrict__ X, int rows, int F,
                                                          const TreeNode* __restrict__ nodes,
                                                          const float* __restrict__ leaves, int depth, int cmp_le,
                                                          const int* __restrict__ chunk_begin, int RB,
                                                          int stage_lds, double* __restrict__ partial, int n_chunks,
                                                          int lds_trees, TreeReduceArgs red) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  double* red_lds = reinterpret_cast<double*>(lds);  // [kBlock] doubles
  float* tile = lds + 2 * kBlock;                     // [F][RB] when staged
  const int tile_floats = stage_lds ? ((RB * F + 3) & ~3) : 0;
  const int n_internal = (1 << depth) - 1;
  TreeNode* s_nodes = reinterpret_cast<TreeNode*>(lds + 2 * kBlock + tile_floats);  // [lds_trees][n_internal]
  float* s_leaves = reinterpret_cast<float*>(reinterpret_cast<char*>(s_nodes) +
                                            ((size_t(lds_trees) * n_internal * sizeof(TreeNode) + 15) & ~size_t(15)));
  const int lrb = __builtin_ctz(unsigned(RB));
  const int row0 = blockIdx.x * RB;
  const int chunk = blockIdx.y;
  const int r_local = threadIdx.x & (RB - 1);
  const int slot = threadIdx.x >> lrb;
  const int tpr = kBlock >> lrb;
  const int t0 = chunk_begin[chunk], t1 = chunk_begin[chunk + 1];
  if constexpr (TREES_LDS) {  // issued first: in flight while the feature tile loads
    copy_to_lds(s_nodes, nodes + size_t(t0) * n_internal, (t1 - t0) * n_internal * int(sizeof(TreeNode)));
    copy_to_lds(s_leaves, leaves + size_t(t0) * (n_internal + 1), (t1 - t0) * (n_internal + 1) * int(sizeof(float)));
  }
  if (stage_lds) stage_tile(tile, X, row0, rows, RB, lrb, F);
  if constexpr (TREES_LDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (stage_lds || TREES_LDS) __syncthreads();
  const float* xs = tile + r_local;
  const bool row_ok = row0 + r_local < rows;
  const double* xg = X + size_t(min(row0 + r_local, rows - 1)) * F;
  const TreeNode* nbase = TREES_LDS ? s_nodes - size_t(t0) * n_internal : nodes;
  const float* lbase = TREES_LDS ? s_leaves - size_t(t0) * (n_internal + 1) : leaves;
  constexpr int U = 4;
  double acc = 0.0;
  if (stage_lds) {
    for (int t = t0 + slot; t < t1; t += tpr * U)
      acc += descend_perfect<D, U, true>(nbase, lbase, n_internal, depth, t, t1, tpr, t0, xs, lrb, xg, cmp_le);
  } else if (row_ok) {  // wide feature vectors: fp64 features straight from global
    for (int t = t0 + slot; t < t1; t += tpr * U)
      acc += descend_perfect<D, U, false>(nbase, lbase, n_internal, depth, t, t1, tpr, t0, xs, lrb, xg, cmp_le);
  }
  if (!row_ok) acc = 0.0;
  if (stage_lds) __syncthreads();  // tile no longer needed; `red` is disjoint anyway
  reduce_write<FUSED>(red_lds, acc, RB, row0, rows, chunk, partial);
  if constexpr (FUSED) fused_tail(partial, rows, n_chunks, red);
}

// Sparse (pointer) trees: U descents interleaved as above; each runs until it
// reaches a leaf (left < 0), the others idle through the remaining trips.
template <bool FUSED>
__global__ __launch_bounds__(kBlock) void sparse_partial(const double* __restrict__ X, int rows, int F,
                                                         const SparseNode* __restrict__ nodes,
                                                         const int* __restrict__ tree_root, int cmp_le,
                                                         const int* __restrict__ chunk_begin, int RB, int stage_lds,
                                                         double* __restrict__ partial, int n_chunks,
                                                         TreeReduceArgs red) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  double* red_lds = reinterpret_cast<double*>(lds);
  float* tile = lds + 2 * kBlock;
  const int lrb = __builtin_ctz(unsigned(RB));
  const int row0 = blockIdx.x * RB;
  const int chunk = blockIdx.y;
  const int r_local = threadIdx.x & (RB - 1);
  const int slot = threadIdx.x >> lrb;
  const int tpr = kBlock >> lrb;
  if (stage_lds) {
    stage_tile(tile, X, row0, rows, RB, lrb, F);
    __syncthreads();
  }
  const bool row_ok = row0 + r_local < rows;
  const int t0 = chunk_begin[chunk], t1 = chunk_begin[chunk + 1];
  constexpr int U = 4;
  double acc = 0.0;
  if (row_ok) {
    const float* xs = tile + r_local;
    const double* xg = X + size_t(row0 + r_local) * F;
    for (int t = t0 + slot; t < t1; t += tpr * U) {
      SparseNode nd[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = t + u * tpr < t1;
        nd[u] = nodes[tree_root[ok[u] ? t + u * tpr : t0]];
      }
      for (int guard = 0; guard < 4096; ++guard) {
        bool any = false;
        int nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool inner = nd[u].left >= 0;
          any |= inner;
          const float x = stage_lds ? tile_x(xs, nd[u].feat, lrb) : float(xg[nd[u].feat & 0x7fffffff]);
          nxt[u] = inner ? (go_left(x, nd[u].thr, nd[u].feat, cmp_le) ? nd[u].left : nd[u].right) : -1;
        }
        if (!any) break;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (nxt[u] >= 0) nd[u] = nodes[nxt[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += ok[u] ? double(nd[u].thr) : 0.0;
    }
  }
  if (stage_lds) __syncthreads();
  reduce_write<FUSED>(red_lds, acc, RB, row0, rows, chunk, partial);
  if constexpr (FUSED) fused_tail(partial, rows, n_chunks, red);
}

// Lookahead descent of ONE perfect tree: each round loads the whole 4-level
// subtree below the current node (1 + 2 + 4 + 8 nodes; each level's nodes are
// contiguous in the breadth-first layout) with independent loads, then
// resolves its 4 levels from registers (select chains on the path bits).  The
// last round also loads its subtree's 2^levels leaves.  Depth 8 is TWO
// dependent memory round trips instead of nine.  Why it matters: every
// launch starts with the ensemble outside this XCD's L2 (PMC at 9 rows: L2
// hit rate 6-8%, ~1 MB fetched per dispatch, profiles/r05i_tree_small), so
// each dependent level costs an Infinity-Cache / HBM round trip, and the
// latency of the chain -- not the number of workgroups -- set the ~11 us of
// the whole-ensemble kernel at any batch size.
template <int NL, bool LAST, bool STAGED>
__device__ __forceinline__ void lookahead_round(const TreeNode* __restrict__ tn, const float* __restrict__ lf,
                                                int n_internal, int& idx, float& leaf, const float* xs, int lrb,
                                                const double* __restrict__ xg, int cmp_le) {
  TreeNode sub[(1 << NL) - 1];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int first = ((idx + 1) << k) - 1;
#pragma unroll
    for (int m = 0; m < (1 << k); ++m) sub[(1 << k) - 1 + m] = tn[first + m];
  }
  float lv[1 << NL];
  if constexpr (LAST) {
    const int lfirst = ((idx + 1) << NL) - 1 - n_internal;
#pragma unroll
    for (int m = 0; m < (1 << NL); ++m) lv[m] = lf[lfirst + m];
  }
  int path = 0;  // decisions so far, MSB first (0 = left, 1 = right)
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    TreeNode nd = sub[(1 << k) - 1];
#pragma unroll
    for (int m = 1; m < (1 << k); ++m)
      if (path == m) nd = sub[(1 << k) - 1 + m];
    const float x = STAGED ? tile_x(xs, nd.feat, lrb) : float(xg[nd.feat & 0x7fffffff]);
    path = 2 * path + (go_left(x, nd.thr, nd.feat, cmp_le) ? 0 : 1);
  }
  idx = ((idx + 1) << NL) - 1 + path;
  if constexpr (LAST) {
    float v = lv[0];
#pragma unroll
    for (int m = 1; m < (1 << NL); ++m)
      if (path == m) v = lv[m];
    leaf = v;
  }
}

template <int REM, int L, bool STAGED>
__device__ __forceinline__ void lookahead_rounds(const TreeNode* __restrict__ tn, const float* __restrict__ lf,
                                                 int n_internal, int& idx, float& leaf, const float* xs, int lrb,
                                                 const double* __restrict__ xg, int cmp_le) {
  constexpr int NL = REM < L ? REM : L;
  lookahead_round<NL, REM == NL, STAGED>(tn, lf, n_internal, idx, leaf, xs, lrb, xg, cmp_le);
  if constexpr (REM > NL) lookahead_rounds<REM - NL, L, STAGED>(tn, lf, n_internal, idx, leaf, xs, lrb, xg, cmp_le);
}

// L levels per round (2..4): depth D costs ceil(D / L) dependent round trips
// and (2^L - 1) / L node loads per level instead of one.
template <int D, int L, bool STAGED>
__device__ __forceinline__ float descend_lookahead(const TreeNode* __restrict__ tn, const float* __restrict__ lf,
                                                   int n_internal, const float* xs, int lrb,
                                                   const double* __restrict__ xg, int cmp_le) {
  static_assert(D >= 1 && D <= 12 && L >= 1 && L <= 4, "lookahead descent: depth 1..12, 1..4 levels per round");
  int idx = 0;
  float leaf = 0.f;
  lookahead_rounds<D, L, STAGED>(tn, lf, n_internal, idx, leaf, xs, lrb, xg, cmp_le);
  return leaf;
}

// Small batches, single-output models: ONE workgroup of 1024 threads owns a
// tile of RB rows and the WHOLE ensemble (thread i -> row i % RB, trees
// i / RB, i / RB + 1024 / RB, ...; RB is sized so a thread walks <= 4 trees,
// one interleaved U = 4 round), folds its rows' sums in-workgroup (butterfly
// + LDS across the 16 waves) and applies the objective transform -- one
// launch per batch, no slab, no second kernel, no cross-workgroup
// signalling.  The batch rows are read once per workgroup, so they come
// straight from the batcher's pinned buffer (no H2D copy).
constexpr int kWholeBlock = 1024;

template <int D, int LA, int TU>
__global__ __launch_bounds__(kWholeBlock) void perfect_whole(const double* __restrict__ X, int rows, int F,
                                                             const TreeNode* __restrict__ nodes,
                                                             const float* __restrict__ leaves, int depth, int cmp_le,
                                                             int n_trees, int RB, int stage_lds,
                                                             const float* __restrict__ base_margin, float scale,
                                                             int transform, double* __restrict__ out, int out_cols) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  double* red = reinterpret_cast<double*>(lds);  // [16 waves][RB <= 16]
  float* tile = lds + 2 * 256;                   // [F][RB] when staged
  const int n_internal = (1 << depth) - 1;
  const int lrb = __builtin_ctz(unsigned(RB));
  const int row0 = int(blockIdx.x) * RB;
  const int r_local = int(threadIdx.x) & (RB - 1);
  const int slot = int(threadIdx.x) >> lrb;
  const int tpr = kWholeBlock >> lrb;
  if (stage_lds) {
    stage_tile<kWholeBlock>(tile, X, row0, rows, RB, lrb, F);
    __syncthreads();
  }
  const float* xs = tile + r_local;
  const bool row_ok = row0 + r_local < rows;
  const double* xg = X + size_t(min(row0 + r_local, rows - 1)) * F;
  constexpr int U = 4;
  double acc = 0.0;
  if constexpr (LA > 0 && D > 0) {
    // TU trees per iteration, all walked unconditionally (a clamped index
    // contributes 0): one basic block, so their loads are in flight together
    auto walk = [&](auto staged) {
      constexpr bool S = decltype(staged)::value;
      for (int t = slot; t < n_trees; t += TU * tpr) {
        float v[TU];
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const int tu = t + u * tpr < n_trees ? t + u * tpr : t;
          v[u] = descend_lookahead<D, LA, S>(nodes + size_t(tu) * n_internal, leaves + size_t(tu) * (n_internal + 1),
                                             n_internal, xs, lrb, xg, cmp_le);
        }
#pragma unroll
        for (int u = 0; u < TU; ++u) acc += t + u * tpr < n_trees ? double(v[u]) : 0.0;
      }
    };
    if (stage_lds) walk(std::true_type{});
    else if (row_ok) walk(std::false_type{});
  } else if (stage_lds) {
    for (int t = slot; t < n_trees; t += tpr * U)
      acc += descend_perfect<D, U, true>(nodes, leaves, n_internal, depth, t, n_trees, tpr, 0, xs, lrb, xg, cmp_le);
  } else if (row_ok) {
    for (int t = slot; t < n_trees; t += tpr * U)
      acc += descend_perfect<D, U, false>(nodes, leaves, n_internal, depth, t, n_trees, tpr, 0, xs, lrb, xg, cmp_le);
  }
  if (!row_ok) acc = 0.0;
  for (int off = 32; off >= RB; off >>= 1) acc += __shfl_xor(acc, off, 64);
  const int lane = int(threadIdx.x) & 63, wave = int(threadIdx.x) >> 6;
  if (lane < RB) red[wave * RB + lane] = acc;
  __syncthreads();
  if (int(threadIdx.x) < RB) {
    const int r = row0 + int(threadIdx.x);
    if (r < rows) {
      double m[1] = {0.0};
#pragma unroll
      for (int w = 0; w < kWholeBlock / 64; ++w) m[0] += red[w * RB + threadIdx.x];
      apply_transform<1>(m, 1, transform, scale, base_margin, out + size_t(r) * out_cols);
    }
  }
}

// Small batches, single-output models, the ensemble SPLIT over S workgroups
// per row tile (blockIdx.y = part): with the whole ensemble on one CU per
// row, the descent is bound by that CU's load issue (profiles/r05xl_l2_levels:
// the ensemble stays L2-resident between batches, a dependent hop costs
// ~70 ns), so S CUs walk S shares of the trees.  Each workgroup folds its
// rows in-workgroup and adds them into acc[row] with one agent-scope fp64
// atomic per row (exact under the same span condition as reduce_write, so
// the order of the S adds does not matter); the workgroup that brings the
// counter to the grid size applies the objective transform, writes the rows
// and re-zeroes acc and the counter for the next batch on this slot.
template <int D>
__global__ __launch_bounds__(kBlock) void perfect_split(const double* __restrict__ X, int rows, int F,
                                                        const TreeNode* __restrict__ nodes,
                                                        const float* __restrict__ leaves, int cmp_le, int n_trees,
                                                        int RB, int stage_lds, const float* __restrict__ base_margin,
                                                        float scale, int transform, double* __restrict__ out,
                                                        int out_cols, double* __restrict__ acc,
                                                        int* __restrict__ counter) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  double* red = reinterpret_cast<double*>(lds);  // [4 waves][RB]
  float* tile = lds + 2 * kBlock;                // [F][RB] when staged
  __shared__ int s_last;
  constexpr int n_internal = (1 << D) - 1;
  const int lrb = __builtin_ctz(unsigned(RB));
  const int row0 = int(blockIdx.x) * RB;
  const int r_local = int(threadIdx.x) & (RB - 1);
  const int slot = int(threadIdx.x) >> lrb;
  const int tpr = kBlock >> lrb;
  const int parts = int(gridDim.y), part = int(blockIdx.y);
  const int t_begin = int((long long)n_trees * part / parts), t_end = int((long long)n_trees * (part + 1) / parts);
  if (stage_lds) {
    stage_tile<kBlock>(tile, X, row0, rows, RB, lrb, F);
    __syncthreads();
  }
  const float* xs = tile + r_local;
  const bool row_ok = row0 + r_local < rows;
  const double* xg = X + size_t(min(row0 + r_local, rows - 1)) * F;
  double a = 0.0;
  if (stage_lds) {
    for (int t = t_begin + slot; t < t_end; t += tpr)
      a += double(descend_lookahead<D, 2, true>(nodes + size_t(t) * n_internal, leaves + size_t(t) * (n_internal + 1),
                                                n_internal, xs, lrb, xg, cmp_le));
  } else if (row_ok) {
    for (int t = t_begin + slot; t < t_end; t += tpr)
      a += double(descend_lookahead<D, 2, false>(nodes + size_t(t) * n_internal, leaves + size_t(t) * (n_internal + 1),
                                                 n_internal, xs, lrb, xg, cmp_le));
  }
  if (!row_ok) a = 0.0;
  for (int off = 32; off >= RB; off >>= 1) a += __shfl_xor(a, off, 64);
  const int lane = int(threadIdx.x) & 63, wave = int(threadIdx.x) >> 6;
  if (lane < RB) red[wave * RB + lane] = a;
  __syncthreads();
  if (int(threadIdx.x) < RB) {
    const int r = row0 + int(threadIdx.x);
    if (r < rows) {
      double m = 0.0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) m += red[w * RB + threadIdx.x];
      if (!acc) {  // host fold: part sums out[r][part]; the host adds them in part order and transforms
        out[size_t(r) * parts + part] = m;
        return;
      }
      __hip_atomic_fetch_add(acc + r, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (!acc) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's adds performed at the coherence point
  __syncthreads();
  // one arrival counter per row tile: the `parts` workgroups of a tile
  // serialise on it, not every workgroup of the grid on one word (that single
  // counter grew the kernel 5.5 -> 8.0 us from 16 to 64 rows, r06e)
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(counter + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == parts - 1;
  __syncthreads();
  if (!s_last) return;
  if (int(threadIdx.x) < RB && row0 + int(threadIdx.x) < rows) {
    const int r = row0 + int(threadIdx.x);
    double m[1] = {__hip_atomic_load(acc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
    __hip_atomic_store(acc + r, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    apply_transform<1>(m, 1, transform, scale, base_margin, out + size_t(r) * out_cols);
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Mid-size batches (33..256 rows), single-output models: tree-major tiles.
// A workgroup is RB rows x TPW trees (thread i -> tree i >> lrb, row i & (RB-1));
// the chunk's TPW trees -- contiguous in the perfect layout -- are staged into
// LDS once and every row of the tile descends them there: D dependent LDS
// reads (~100 cycles each) instead of ceil(D/2) L2 round trips, and each
// node line leaves L2 once per row tile instead of once per row, which is what
// bounded the one-row-per-workgroup whole-ensemble kernel at these sizes
// (xgb1000: 6.7 us at 64 rows, 9.5-10.7 us at 256, profiles/r06d_micro).
// Rows fold as in perfect_split: in-workgroup sum over the TPW trees, one
// agent-scope fp64 atomic per row and tree chunk, the last workgroup applies
// the transform and re-zeroes the accumulators.  Consecutive lanes are
// consecutive rows of ONE tree, so a wave starts its descent on one node
// (an LDS broadcast) and the X tile reads hit 32 distinct banks (tile_x).
constexpr int kTileMaxBlock = 1024;

template <int D>
__global__ __launch_bounds__(kTileMaxBlock) void perfect_tile(const double* __restrict__ X, int rows, int F,
                                                              const TreeNode* __restrict__ nodes,
                                                              const float* __restrict__ leaves, int cmp_le,
                                                              int n_trees, int RB, int TPW, int stage_x,
                                                              const float* __restrict__ base_margin, float scale,
                                                              int transform, double* __restrict__ out, int out_cols,
                                                              double* __restrict__ acc, int* __restrict__ counter) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NI = (1 << D) - 1;
  const int nthr = int(blockDim.x);
  uint2* sN = reinterpret_cast<uint2*>(lds);                                      // [TPW][NI] TreeNode bits
  float* sL = reinterpret_cast<float*>(sN + size_t(TPW) * NI);                    // [TPW][NI + 1]
  float* tile = sL + size_t(TPW) * (NI + 1);                                      // [F][RB] when staged
  __shared__ int s_last;
  const int lrb = __builtin_ctz(unsigned(RB));
  const int row0 = int(blockIdx.x) * RB;
  const int t0 = int(blockIdx.y) * TPW;
  const int nt = min(TPW, n_trees - t0);
  {  // the chunk's nodes and leaves: two contiguous runs
    const uint2* gn = reinterpret_cast<const uint2*>(nodes) + size_t(t0) * NI;
    for (int i = int(threadIdx.x); i < nt * NI; i += nthr) sN[i] = gn[i];
    const float* gl = leaves + size_t(t0) * (NI + 1);
    for (int i = int(threadIdx.x); i < nt * (NI + 1); i += nthr) sL[i] = gl[i];
  }
  if (stage_x) {  // RB x F rows -> fp32 feature-major tile (tile_x), zero past the batch
    const int n = RB * F, nrow = min(RB, rows - row0);
    for (int i = int(threadIdx.x); i < n; i += nthr) {
      const int r = i & (RB - 1), f = i >> lrb;
      tile[i] = r < nrow ? float(X[size_t(row0 + r) * F + f]) : 0.f;
    }
  }
  __syncthreads();
  const int r_local = int(threadIdx.x) & (RB - 1);
  const int tl = int(threadIdx.x) >> lrb;
  const bool row_ok = row0 + r_local < rows;
  double a = 0.0;
  if (tl < nt && row_ok) {
    const uint2* tn = sN + size_t(tl) * NI;
    const float* xs = tile + r_local;
    const double* xg = X + size_t(row0 + r_local) * F;
    int idx = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint2 nb = tn[idx];
      const float thr = __uint_as_float(nb.x);
      const int32_t feat = int32_t(nb.y);
      const float x = stage_x ? tile_x(xs, feat, lrb) : float(xg[feat & 0x7fffffff]);
      idx = 2 * idx + (go_left(x, thr, feat, cmp_le) ? 1 : 2);
    }
    a = double(sL[size_t(tl) * (NI + 1) + (idx - NI)]);
  }
  for (int off = 32; off >= RB; off >>= 1) a += __shfl_xor(a, off, 64);
  const int lane = int(threadIdx.x) & 63, wave = int(threadIdx.x) >> 6;
  __syncthreads();  // every descent is done with the staged trees: their LDS becomes the fold area
  double* red = reinterpret_cast<double*>(lds);  // [waves][RB]
  // (RB <= 64: after the fold lanes 0..RB-1 of every wave hold its rows' sums)
  if (lane < RB) red[wave * RB + lane] = a;
  __syncthreads();
  if (int(threadIdx.x) < RB) {
    const int r = row0 + int(threadIdx.x);
    if (r < rows) {
      double m = 0.0;
      for (int w = 0; w < nthr / 64; ++w) m += red[w * RB + int(threadIdx.x)];
      __hip_atomic_fetch_add(acc + r, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's adds performed at the coherence point
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             int(gridDim.x * gridDim.y) - 1;
  __syncthreads();
  if (!s_last) return;
  for (int r = int(threadIdx.x); r < rows; r += nthr) {
    double m[1] = {__hip_atomic_load(acc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
    __hip_atomic_store(acc + r, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    apply_transform<1>(m, 1, transform, scale, base_margin, out + size_t(r) * out_cols);
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kMaxGroups = 64;

// Block = RB rows x (blockDim / RB) chunk-lanes: the lanes of a row sum a
// strided subset of the tree chunks (independent, coalesced slab loads), fold
// through LDS, and lane 0 applies the objective transform.
__global__ __launch_bounds__(kBlock) void reduce_transform(const double* __restrict__ partial, int rows, int n_chunks,
                                                           const int* __restrict__ chunk_group, int groups,
                                                           const float* __restrict__ base_margin, float scale,
                                                           int transform, double* __restrict__ out, int out_cols,
                                                           int RB) {
  extern __shared__ __attribute__((aligned(16))) double m_lds[];  // [blockDim][groups]
  const int nthr = int(blockDim.x);
  const int r_local = int(threadIdx.x) % RB, slot = int(threadIdx.x) / RB, tpr = nthr / RB;
  const int r = int(blockIdx.x) * RB + r_local;
  double* acc = m_lds + size_t(threadIdx.x) * groups;
  for (int g = 0; g < groups; ++g) acc[g] = 0.0;
  if (r < rows)
    for (int c = slot; c < n_chunks; c += tpr) acc[chunk_group[c]] += double(partial[size_t(c) * rows + r]);
  __syncthreads();
  if (slot != 0 || r >= rows) return;
  double* m = acc;
  for (int s = 1; s < tpr; ++s) {
    const double* o2 = m_lds + size_t(s * RB + r_local) * groups;
    for (int g = 0; g < groups; ++g) m[g] += o2[g];
  }
  apply_transform<0>(m, groups, transform, scale, base_margin, out + size_t(r) * out_cols);
}

int lds_bytes_for(int RB, int F, bool* stage) {
  *stage = RB * F <= kMaxLdsFloats;
  return int((2 * kBlock + (*stage ? RB * F : 0)) * sizeof(float));  // fp64 reduce area + fp32 tile
}

constexpr int kMaxTreeLdsDepth = 10;
constexpr int kMaxLdsBytes = 64 * 1024;

int tree_bytes(int depth) { return ((1 << depth) - 1) * int(sizeof(TreeNode)) + (1 << depth) * int(sizeof(float)); }
constexpr int kTreeLdsPad = 16;  // leaves slab rounded up to 16 B

template <bool FUSED>
void launch_perfect(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                    int cmp_le, const int* chunk_begin, int n_chunks, int RB, double* partial, const TreeReduceArgs& red,
                    int lds_trees, hipStream_t s, hipEvent_t stop = nullptr) {
  bool stage;
  int lds = lds_bytes_for(RB, F, &stage);
  if (stage) lds = int((2 * kBlock + ((RB * F + 3) & ~3)) * sizeof(float));
  if (depth > kMaxTreeLdsDepth || lds + lds_trees * tree_bytes(depth) + kTreeLdsPad > kMaxLdsBytes) lds_trees = 0;
  if (lds_trees) lds += lds_trees * tree_bytes(depth) + kTreeLdsPad;
  dim3 grid((rows + RB - 1) / RB, n_chunks);
#define SCA_TREE_LAUNCH(DD, TL)                                                                                    \
  do {                                                                                                            \
    if (stop)                                                                                                     \
      hipExtLaunchKernelGGL((perfect_partial<DD, FUSED, TL>), grid, dim3(kBlock), uint32_t(lds), s, nullptr, stop, \
                            0, X, rows, F, nodes, leaves, depth, cmp_le, chunk_begin, RB, int(stage), partial,    \
                            n_chunks, lds_trees, red);                                                            \
    else                                                                                                          \
      hipLaunchKernelGGL((perfect_partial<DD, FUSED, TL>), grid, dim3(kBlock), lds, s, X, rows, F, nodes, leaves, \
                         depth, cmp_le, chunk_begin, RB, int(stage), partial, n_chunks, lds_trees, red);          \
  } while (0)
#define SCA_TREE_CASE(DD)                                  \
  case DD:                                                 \
    if (lds_trees) SCA_TREE_LAUNCH(DD, true);              \
    else SCA_TREE_LAUNCH(DD, false);                       \
    break;
  switch (depth) {
    SCA_TREE_CASE(1) SCA_TREE_CASE(2) SCA_TREE_CASE(3) SCA_TREE_CASE(4) SCA_TREE_CASE(5) SCA_TREE_CASE(6)
    SCA_TREE_CASE(7) SCA_TREE_CASE(8) SCA_TREE_CASE(9) SCA_TREE_CASE(10)
    case 11: SCA_TREE_LAUNCH(11, false); break;
    case 12: SCA_TREE_LAUNCH(12, false); break;
    default: SCA_TREE_LAUNCH(0, false);
  }
#undef SCA_TREE_CASE
#undef SCA_TREE_LAUNCH
}

template <bool FUSED>
void launch_sparse(const double* X, int rows, int F, const SparseNode* nodes, const int* tree_root, int cmp_le,
                   const int* chunk_begin, int n_chunks, int RB, double* partial, const TreeReduceArgs& red,
                   hipStream_t s, hipEvent_t stop = nullptr) {
  bool stage;
  const int lds = lds_bytes_for(RB, F, &stage);
  dim3 grid((rows + RB - 1) / RB, n_chunks);
  if (stop)
    hipExtLaunchKernelGGL((sparse_partial<FUSED>), grid, dim3(kBlock), uint32_t(lds), s, nullptr, stop, 0, X, rows, F,
                          nodes, tree_root, cmp_le, chunk_begin, RB, int(stage), partial, n_chunks, red);
  else
    hipLaunchKernelGGL((sparse_partial<FUSED>), grid, dim3(kBlock), lds, s, X, rows, F, nodes, tree_root, cmp_le,
                       chunk_begin, RB, int(stage), partial, n_chunks, red);
}

}  // namespace

void tree_perfect_partial(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                          int cmp_le, const int* chunk_begin, int n_chunks, int RB, double* partial,
                          hipStream_t s, int lds_trees) {
  if (rows <= 0 || n_chunks <= 0) return;
  launch_perfect<false>(X, rows, F, nodes, leaves, depth, cmp_le, chunk_begin, n_chunks, RB, partial,
                        TreeReduceArgs{}, lds_trees, s);
}

int tree_lds_max_trees(int depth, int rows_per_block, int F) {
  if (depth <= 0 || depth > kMaxTreeLdsDepth) return 0;
  bool stage;
  int lds = lds_bytes_for(rows_per_block, F, &stage);
  if (stage) lds = int((2 * kBlock + ((rows_per_block * F + 3) & ~3)) * sizeof(float));
  return std::max(0, (kMaxLdsBytes - lds - kTreeLdsPad) / tree_bytes(depth));
}

void tree_sparse_partial(const double* X, int rows, int F, const SparseNode* nodes, const int* tree_root, int cmp_le,
                         const int* chunk_begin, int n_chunks, int RB, double* partial, hipStream_t s) {
  if (rows <= 0 || n_chunks <= 0) return;
  launch_sparse<false>(X, rows, F, nodes, tree_root, cmp_le, chunk_begin, n_chunks, RB, partial, TreeReduceArgs{}, s);
}

void tree_perfect_fused(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, const int* chunk_begin, int n_chunks, int RB, double* partial,
                        const TreeReduceArgs& red, hipStream_t s, int lds_trees, hipEvent_t stop) {
  if (rows <= 0 || n_chunks <= 0) return;
  launch_perfect<true>(X, rows, F, nodes, leaves, depth, cmp_le, chunk_begin, n_chunks, RB, partial, red, lds_trees,
                       s, stop);
}

void tree_sparse_fused(const double* X, int rows, int F, const SparseNode* nodes, const int* tree_root, int cmp_le,
                       const int* chunk_begin, int n_chunks, int RB, double* partial, const TreeReduceArgs& red,
                       hipStream_t s, hipEvent_t stop) {
  if (rows <= 0 || n_chunks <= 0) return;
  launch_sparse<true>(X, rows, F, nodes, tree_root, cmp_le, chunk_begin, n_chunks, RB, partial, red, s, stop);
}

int tree_whole_lookahead_default();

int tree_whole_rows_per_block(int n_trees, int rows) {
  // trees one thread walks (SCA_TREE_WHOLE_TPT): 1 with the lookahead descent
  // (one tree per lane, more workgroups per batch), 4 for the level-by-level
  // descent (one interleaved U = 4 round)
  static const int tpt = [] {
    const char* e = std::getenv("SCA_TREE_WHOLE_TPT");
    const int v = e ? std::atoi(e) : (tree_whole_lookahead_default() > 0 ? 1 : 4);
    return v < 1 ? 1 : v;
  }();
  int rb = 1;
  while (rb < 16 && rb < rows && (long long)n_trees * (rb * 2) <= (long long)tpt * kWholeBlock) rb <<= 1;
  return rb;
}

int tree_whole_lookahead_default() {
  static const int v = [] {
    const char* e = std::getenv("SCA_TREE_LOOKAHEAD");
    return e ? std::atoi(e) : 21;
  }();
  return v;
}

void tree_perfect_whole(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, int n_trees, int RB, const float* base_margin, float scale, int transform,
                        double* out, int out_cols, hipStream_t s, hipEvent_t stop, int lookahead) {
  if (rows <= 0 || n_trees <= 0) return;
  // lookahead = 10 * levels per round + trees per iteration; 21 (default,
  // depths 4..10): two levels per dependent round trip, one tree at a time
  // (9 rows x 1000 trees x depth 8: 6.2 us vs 11.2 us level by level,
  // profiles/r05i_tree_small); 22 .. 42 at depth 8 for A/B; 0 = the
  // level-by-level descent
  const int la = lookahead < 0 ? tree_whole_lookahead_default() : lookahead;
  const bool stage = RB * F <= kMaxLdsFloats;
  const uint32_t lds = uint32_t((2 * 256 + (stage ? ((RB * F + 3) & ~3) : 0)) * sizeof(float));
  const dim3 grid((rows + RB - 1) / RB);
#define SCA_WHOLE_LAUNCH1(DD, LA, TU)                                                                              \
  do {                                                                                                            \
    if (stop)                                                                                                     \
      hipExtLaunchKernelGGL((perfect_whole<DD, LA, TU>), grid, dim3(kWholeBlock), lds, s, nullptr, stop, 0, X,     \
                            rows, F, nodes, leaves, depth, cmp_le, n_trees, RB, int(stage), base_margin, scale,    \
                            transform, out, out_cols);                                                            \
    else                                                                                                          \
      hipLaunchKernelGGL((perfect_whole<DD, LA, TU>), grid, dim3(kWholeBlock), lds, s, X, rows, F, nodes, leaves,  \
                         depth, cmp_le, n_trees, RB, int(stage), base_margin, scale, transform, out, out_cols);   \
  } while (0)
#define SCA_WHOLE_LAUNCH(DD) SCA_WHOLE_LAUNCH1(DD, 0, 1)
  if (la == 21 && depth >= 4 && depth <= 10) {
    switch (depth) {
      case 4: SCA_WHOLE_LAUNCH1(4, 2, 1); return;
      case 5: SCA_WHOLE_LAUNCH1(5, 2, 1); return;
      case 6: SCA_WHOLE_LAUNCH1(6, 2, 1); return;
      case 7: SCA_WHOLE_LAUNCH1(7, 2, 1); return;
      case 8: SCA_WHOLE_LAUNCH1(8, 2, 1); return;
      case 9: SCA_WHOLE_LAUNCH1(9, 2, 1); return;
      default: SCA_WHOLE_LAUNCH1(10, 2, 1); return;
    }
  }
  if (depth == 8 && la > 0) {
    switch (la) {
      case 21: SCA_WHOLE_LAUNCH1(8, 2, 1); return;
      case 22: SCA_WHOLE_LAUNCH1(8, 2, 2); return;
      case 31: SCA_WHOLE_LAUNCH1(8, 3, 1); return;
      case 32: SCA_WHOLE_LAUNCH1(8, 3, 2); return;
      case 41: SCA_WHOLE_LAUNCH1(8, 4, 1); return;
      case 42: SCA_WHOLE_LAUNCH1(8, 4, 2); return;
      default: break;
    }
  }
  switch (depth) {
    case 4: SCA_WHOLE_LAUNCH(4); break;
    case 5: SCA_WHOLE_LAUNCH(5); break;
    case 6: SCA_WHOLE_LAUNCH(6); break;
    case 7: SCA_WHOLE_LAUNCH(7); break;
    case 8: SCA_WHOLE_LAUNCH(8); break;
    case 9: SCA_WHOLE_LAUNCH(9); break;
    case 10: SCA_WHOLE_LAUNCH(10); break;
    default: SCA_WHOLE_LAUNCH1(0, 0, 1);
  }
#undef SCA_WHOLE_LAUNCH
#undef SCA_WHOLE_LAUNCH1
}

// SCA_TREE_SPLIT: workgroups per row tile (default 8; 0 = one workgroup, the
// perfect_whole kernel).  SCA_TREE_SPLIT_ROWS: largest batch split (default
// 32).  xgb1000 at 9 rows (profiles/r05sl_tree_split): 6.21 -> 5.27 us in the
// microbench, 7.17 -> 5.96 us serving with BAR-staged rows, 8.04 -> 7.04 us
// with host rows; serving batches of 17-32 rows 7.3 -> 5.8 us; in the
// microbench the single workgroup per row tile wins again at 128 rows.
// Round 6 (profiles/r06f_ab, one arrival counter per row tile): 16 parts
// win up to 16 rows (5.27 vs 5.58 us), 8 parts tie the whole kernel at 48-64
// rows and beat it at 96 (7.17 vs 7.37 us): defaults 16 / 8 parts, split up
// to 96 rows.
int tree_split_parts() {
  static const int v = [] {
    const char* e = std::getenv("SCA_TREE_SPLIT");
    const int p = e ? std::atoi(e) : 8;
    return p < 0 ? 0 : (p > 64 ? 64 : p);
  }();
  return v;
}

int tree_split_parts_for(int rows) {
  const int p = tree_split_parts();
  if (p <= 0) return 0;
  if (std::getenv("SCA_TREE_SPLIT")) return p;  // an explicit setting holds at every batch size
  return rows <= 16 ? 16 : p;
}

int tree_split_max_rows() {
  static const int v = [] {
    const char* e = std::getenv("SCA_TREE_SPLIT_ROWS");
    return e ? std::max(0, std::atoi(e)) : 96;
  }();
  return v;
}

void tree_perfect_split(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                        int cmp_le, int n_trees, int parts, const float* base_margin, float scale, int transform,
                        double* out, int out_cols, double* acc, int* counter, hipStream_t s, hipEvent_t stop) {
  if (rows <= 0 || n_trees <= 0 || parts <= 0 || depth < 4 || depth > 10) return;
  // rows per workgroup: one tree per lane of the part while the rows fit
  const int per_part = (n_trees + parts - 1) / parts;
  int RB = 1;
  while (RB < 16 && RB < rows && per_part * (RB * 2) <= kBlock) RB <<= 1;
  const bool stage = RB * F <= kMaxLdsFloats;
  const uint32_t lds = uint32_t((2 * kBlock + (stage ? ((RB * F + 3) & ~3) : 0)) * sizeof(float));
  const dim3 grid((rows + RB - 1) / RB, parts);
#define SCA_SPLIT_LAUNCH(DD)                                                                                      \
  do {                                                                                                            \
    if (stop)                                                                                                     \
      hipExtLaunchKernelGGL((perfect_split<DD>), grid, dim3(kBlock), lds, s, nullptr, stop, 0, X, rows, F, nodes,  \
                            leaves, cmp_le, n_trees, RB, int(stage), base_margin, scale, transform, out, out_cols,  \
                            acc, counter);                                                                        \
    else                                                                                                          \
      hipLaunchKernelGGL((perfect_split<DD>), grid, dim3(kBlock), lds, s, X, rows, F, nodes, leaves, cmp_le,       \
                         n_trees, RB, int(stage), base_margin, scale, transform, out, out_cols, acc, counter);    \
  } while (0)
  switch (depth) {
    case 4: SCA_SPLIT_LAUNCH(4); break;
    case 5: SCA_SPLIT_LAUNCH(5); break;
    case 6: SCA_SPLIT_LAUNCH(6); break;
    case 7: SCA_SPLIT_LAUNCH(7); break;
    case 8: SCA_SPLIT_LAUNCH(8); break;
    case 9: SCA_SPLIT_LAUNCH(9); break;
    default: SCA_SPLIT_LAUNCH(10); break;
  }
#undef SCA_SPLIT_LAUNCH
}

// Tile geometry for a batch: RB rows (16 / 32 / 64 as the batch grows) x
// TPW trees per workgroup, TPW the largest power of two (<= 16) whose trees
// fit 96 KB of LDS.  Returns false when the kernel does not apply.
bool tree_tile_plan(int rows, int F, int depth, int* RB, int* TPW, int* lds_bytes, int* stage_x) {
  if (depth < 4 || depth > 10 || rows <= 0) return false;
  constexpr int kLdsCap = 64 * 1024;  // dynamic LDS without a per-kernel attribute
  const int tb = tree_bytes(depth);
  int tpw = 16;
  while (tpw > 1 && tpw * tb > 56 * 1024) tpw >>= 1;
  int rb = rows > 96 ? 64 : (rows > 48 ? 32 : 16);
  if (rb * tpw > kTileMaxBlock) rb = kTileMaxBlock / tpw;
  const int red = (kTileMaxBlock / 64) * rb * int(sizeof(double));  // the fold reuses the tree area
  const int trees = std::max(tpw * tb, red);
  const int xt = ((rb * F + 3) & ~3) * int(sizeof(float));
  const int sx = trees + xt <= kLdsCap ? 1 : 0;
  *RB = rb;
  *TPW = tpw;
  *stage_x = sx;
  *lds_bytes = trees + (sx ? xt : 0);
  return *lds_bytes <= kLdsCap;
}

// Off by default (SCA_TREE_TILE_ROWS=N opts in for batches of 33..N rows):
// at the xgb1000 shape the tile kernel only beats the whole-ensemble kernel
// from ~192 rows (8.3 vs 8.8 us), loses below 128 (9.6 vs 6.3 us at 33 rows,
// the LDS staging of 16 trees per workgroup is not amortised), and serving
// batches are mostly small: 9.36 us mean vs 7.61 (profiles/r06e_tree_tile).
int tree_tile_max_rows() {
  static const int v = [] {
    const char* e = std::getenv("SCA_TREE_TILE_ROWS");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return v;
}

bool tree_perfect_tile(const double* X, int rows, int F, const TreeNode* nodes, const float* leaves, int depth,
                       int cmp_le, int n_trees, const float* base_margin, float scale, int transform, double* out,
                       int out_cols, double* acc, int* counter, hipStream_t s, hipEvent_t stop) {
  int RB, TPW, lds, sx;
  if (n_trees <= 0 || !tree_tile_plan(rows, F, depth, &RB, &TPW, &lds, &sx)) return false;
  const dim3 grid((rows + RB - 1) / RB, (n_trees + TPW - 1) / TPW), block(RB * TPW);
#define SCA_TILE_LAUNCH(DD)                                                                                       \
  do {                                                                                                            \
    if (stop)                                                                                                     \
      hipExtLaunchKernelGGL((perfect_tile<DD>), grid, block, uint32_t(lds), s, nullptr, stop, 0, X, rows, F, nodes, \
                            leaves, cmp_le, n_trees, RB, TPW, sx, base_margin, scale, transform, out, out_cols, acc,  \
                            counter);                                                                             \
    else                                                                                                          \
      hipLaunchKernelGGL((perfect_tile<DD>), grid, block, uint32_t(lds), s, X, rows, F, nodes, leaves, cmp_le,      \
                         n_trees, RB, TPW, sx, base_margin, scale, transform, out, out_cols, acc, counter);       \
  } while (0)
  switch (depth) {
    case 4: SCA_TILE_LAUNCH(4); break;
    case 5: SCA_TILE_LAUNCH(5); break;
    case 6: SCA_TILE_LAUNCH(6); break;
    case 7: SCA_TILE_LAUNCH(7); break;
    case 8: SCA_TILE_LAUNCH(8); break;
    case 9: SCA_TILE_LAUNCH(9); break;
    default: SCA_TILE_LAUNCH(10); break;
  }
#undef SCA_TILE_LAUNCH
  return true;
}

void tree_reduce(const double* partial, int rows, int n_chunks, const int* chunk_group, int groups,
                 const float* base_margin, float scale, int transform, double* out, int out_cols, hipStream_t s,
                 hipEvent_t stop) {
  if (rows <= 0) return;
  if (groups > kMaxGroups) groups = kMaxGroups;
  // Keep LDS <= 64 KB per block: 256 threads up to 32 groups, 64 beyond.
  const int nthr = groups > 32 ? 64 : kBlock;
  // Lanes per row: enough that each sums <= 4 slab entries (independent loads
  // in flight), the rest of the block takes more rows -> many small blocks
  // instead of a few long serial ones.
  int L = 1;
  while (L < nthr && L * 4 < n_chunks) L <<= 1;
  const int RB = nthr / L;
  const size_t lds = size_t(nthr) * groups * sizeof(double);
  if (stop)  // the batch's last kernel completes the batcher's event from its own dispatch
    hipExtLaunchKernelGGL(reduce_transform, dim3((rows + RB - 1) / RB), dim3(nthr), uint32_t(lds), s, nullptr, stop, 0,
                          partial, rows, n_chunks, chunk_group, groups, base_margin, scale, transform, out, out_cols,
                          RB);
  else
    hipLaunchKernelGGL(reduce_transform, dim3((rows + RB - 1) / RB), dim3(nthr), lds, s, partial, rows, n_chunks,
                       chunk_group, groups, base_margin, scale, transform, out, out_cols, RB);
}

}  // namespace sca::kern
