#include "mlp_model.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace sca::gpu {

namespace {

int round_up(int x, int m) { return (x + m - 1) / m * m; }
constexpr size_t kSlack = 4 * 16 + 64;  // workspace floats past each buffer (A look-ahead)
constexpr int kGemmRows = 512;          // rows_eff from which fp32 layers use the register-tiled GEMM
constexpr int kLdsGemmRows = 2048;      // ... and from which the LDS-tiled one (row-major weights)

uint16_t to_bf16(float f) {  // round to nearest even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return uint16_t((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

// Host twin of kern::Philox (csrc/kernels/philox.h): identical streams, so the
// CPU reference path draws the same reparameterisation noise as the GPU.
struct HostPhilox {
  uint32_t c[4], k[2], out[4];
  int used = 4;
  HostPhilox(uint64_t seed, uint64_t subseq) {
    k[0] = uint32_t(seed);
    k[1] = uint32_t(seed >> 32);
    c[0] = uint32_t(subseq);
    c[1] = uint32_t(subseq >> 32);
    c[2] = c[3] = 0;
  }
  void round() {
    uint32_t kk0 = k[0], kk1 = k[1], x0 = c[0], x1 = c[1], x2 = c[2], x3 = c[3];
    for (int i = 0; i < 10; ++i) {
      const uint64_t p0 = uint64_t(0xD2511F53u) * x0, p1 = uint64_t(0xCD9E8D57u) * x2;
      const uint32_t y0 = uint32_t(p1 >> 32) ^ x1 ^ kk0, y1 = uint32_t(p1);
      const uint32_t y2 = uint32_t(p0 >> 32) ^ x3 ^ kk1, y3 = uint32_t(p0);
      x0 = y0; x1 = y1; x2 = y2; x3 = y3;
      kk0 += 0x9E3779B9u;
      kk1 += 0xBB67AE85u;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
    if (++c[2] == 0) ++c[3];
    used = 0;
  }
  uint32_t next() {
    if (used == 4) round();
    return out[used++];
  }
  float uniform() { return (float(next() >> 8) + 1.0f) * (1.0f / 16777216.0f); }
  float normal() {
    const float u1 = uniform(), u2 = uniform();
    return std::sqrt(-2.0f * std::log(u1)) * float(std::cos(2.0 * M_PI * double(u2)));
  }
};

float act_host(float v, int a) {
  switch (a) {
    case kern::kMlpRelu: return std::max(v, 0.f);
    case kern::kMlpSigmoid: return 1.f / (1.f + std::exp(-v));
    case kern::kMlpTanh: return std::tanh(v);
    default: return v;
  }
}

void check_chain(const std::vector<DenseLayer>& ls, int in_dim, const char* what) {
  int k = in_dim;
  for (const auto& L : ls) {
    if (L.K != k) throw std::runtime_error(std::string("MlpModel: ") + what + " layer expects " + std::to_string(L.K) +
                                           " inputs but receives " + std::to_string(k));
    if (int64_t(L.W.size()) != int64_t(L.K) * L.N || int(L.b.size()) != L.N)
      throw std::runtime_error("MlpModel: layer weight / bias size mismatch");
    k = L.N;
  }
}

}  // namespace

MlpModel::MlpModel(std::vector<DenseLayer> layers, int out_mode) : enc_(std::move(layers)), out_mode_(out_mode) {
  if (enc_.empty()) throw std::runtime_error("MlpModel: no layers");
  F_ = enc_.front().K;
  check_chain(enc_, F_, "dense");
  if (out_mode_ == kOutBinary && enc_.back().N != 1) throw std::runtime_error("MlpModel: binary head needs one unit");
  out_dim_ = out_mode_ == kOutBinary ? 2 : enc_.back().N;
  build();
}

std::shared_ptr<MlpModel> MlpModel::vae(std::vector<DenseLayer> encoder, int latent, std::vector<DenseLayer> decoder,
                                        int samples, uint64_t seed) {
  std::shared_ptr<MlpModel> m(new MlpModel());
  m->enc_ = std::move(encoder);
  m->dec_ = std::move(decoder);
  m->vae_ = true;
  m->latent_ = latent;
  m->samples_ = samples;
  m->seed_ = seed;
  if (m->enc_.empty() || m->dec_.empty()) throw std::runtime_error("MlpModel::vae: empty encoder / decoder");
  m->F_ = m->enc_.front().K;
  check_chain(m->enc_, m->F_, "encoder");
  if (m->enc_.back().N != 2 * latent) throw std::runtime_error("MlpModel::vae: head must output 2 * latent");
  check_chain(m->dec_, latent, "decoder");
  if (m->dec_.back().N != m->F_) throw std::runtime_error("MlpModel::vae: decoder must reconstruct the input width");
  if (samples < 1) throw std::runtime_error("MlpModel::vae: samples must be >= 1");
  m->out_dim_ = 1;
  m->build();
  return m;
}

int MlpModel::add_layer(const DenseLayer& L, int type, int in_buf, int out_buf) {
  auto& p = prog_;
  const int n = p.n_pre + p.n_loop;
  if (n >= kern::kMlpMaxOps) throw std::runtime_error("MlpModel: too many layers");
  kern::MlpOp& op = p.ops[n];
  op.type = type;
  op.act = L.act;
  op.in_buf = in_buf;
  op.out_buf = out_buf;
  op.K = L.K;
  op.Kp = round_up(L.K, 16);
  op.N = L.N;
  op.Np = round_up(L.N, 16);
  // fragment-major Wt: [Np/16 tiles][Kp/16 blocks][64 lanes][4]; lane (kq, n)
  // of block kb holds Wt[16 kb + 4 kq + j][16 t + n], j = 0..3 (kernels.h)
  op.w_off = (long long)params_.size();
  params_.resize(params_.size() + size_t(op.Kp) * op.Np, 0.f);
  const int KB = op.Kp / 16;
  float* w = params_.data() + op.w_off;
  for (int t = 0; t < op.Np / 16; ++t)
    for (int kb = 0; kb < KB; ++kb)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 4; ++j) {
          const int nn = t * 16 + (lane & 15), k = kb * 16 + (lane >> 4) * 4 + j;
          w[((size_t(t) * KB + kb) * 64 + lane) * 4 + j] = (nn < L.N && k < L.K) ? L.W[size_t(nn) * L.K + k] : 0.f;
        }
  op.b_off = (long long)params_.size();
  params_.resize(params_.size() + size_t(op.Np), 0.f);
  for (int nn = 0; nn < L.N; ++nn) params_[size_t(op.b_off) + nn] = L.b[size_t(nn)];
  op.Kpb = round_up(L.K, 64);
  op.Npb = round_up(L.N, 64);
  op.wb_off = (long long)pbf_.size();
  if (precision_ == 0) {  // fp32 row-major [Npb][Kq], zero padded (gemm_lds_kernel<float>)
    const int Kq = round_up(L.K, 32);
    wr_off_[size_t(n)] = (long long)prm_.size();
    kq_[size_t(n)] = Kq;
    prm_.resize(prm_.size() + size_t(op.Npb) * Kq, 0.f);
    float* wr = prm_.data() + wr_off_[size_t(n)];
    for (int nn = 0; nn < L.N; ++nn)
      for (int k = 0; k < L.K; ++k) wr[size_t(nn) * Kq + k] = L.W[size_t(nn) * L.K + k];
  }
  if (precision_ == 1) {  // bf16 row-major [Npb][Kpb], zero padded (gemm_lds_kernel<__bf16>)
    pbf_.resize(pbf_.size() + size_t(op.Npb) * op.Kpb, 0);
    uint16_t* wb = pbf_.data() + op.wb_off;
    for (int nn = 0; nn < L.N; ++nn)
      for (int k = 0; k < L.K; ++k) wb[size_t(nn) * op.Kpb + k] = to_bf16(L.W[size_t(nn) * L.K + k]);
  }
  return n;
}

void MlpModel::set_precision(int p) {
  if (p != 0 && p != 1) throw std::runtime_error("MlpModel: precision must be fp32 (0) or bf16 (1)");
  precision_ = p;
  build();
}

void MlpModel::build() {
  if (const char* m = std::getenv("SCA_MLP_MODE"))
    mode_ = !std::strcmp(m, "fused") ? 1 : !std::strcmp(m, "layer") ? 2 : 0;
  prog_ = kern::MlpProgram();
  params_.clear();
  pbf_.clear();
  prm_.clear();
  wr_off_.assign(kern::kMlpMaxOps, -1);
  kq_.assign(kern::kMlpMaxOps, 0);
  auto& p = prog_;
  p.F = F_;
  p.Fp = round_up(F_, 16);
  int width[kern::kMlpMaxBufs] = {};
  width[0] = p.Fp;
  auto use = [&](int b, int w) { width[b] = std::max(width[b], w); };
  int cur = 0;
  if (!vae_) {
    for (size_t i = 0; i < enc_.size(); ++i) {
      const int out = (i % 2 == 0) ? 1 : 2;
      const int o = add_layer(enc_[i], kern::kMlpDense, cur, out);
      use(cur, p.ops[o].Kp);
      use(out, p.ops[o].Np);
      p.n_pre++;
      cur = out;
    }
    p.out_buf = cur;
    p.out_dim = enc_.back().N;
    p.out_softmax = out_mode_;
  } else {
    for (size_t i = 0; i < enc_.size(); ++i) {
      const bool head = i + 1 == enc_.size();
      const int out = head ? 3 : ((i % 2 == 0) ? 1 : 2);
      const int o = add_layer(enc_[i], kern::kMlpDense, cur, out);
      use(cur, p.ops[o].Kp);
      use(out, p.ops[o].Np);
      p.n_pre++;
      cur = out;
    }
    // loop: reparam 3 -> 4, decoder 4 -> 1 -> 2 -> ..., last layer fused with the MSE
    {
      const int n = p.n_pre + p.n_loop;
      kern::MlpOp& op = p.ops[n];
      op = kern::MlpOp();
      op.type = kern::kMlpReparam;
      op.in_buf = 3;
      op.out_buf = 4;
      op.N = latent_;
      op.Np = round_up(latent_, 16);
      use(4, op.Np);
      p.n_loop++;
    }
    cur = 4;
    for (size_t i = 0; i < dec_.size(); ++i) {
      const bool last = i + 1 == dec_.size();
      const int out = (i % 2 == 0) ? 1 : 2;
      const int o = add_layer(dec_[i], last ? kern::kMlpDenseMse : kern::kMlpDense, cur, out);
      use(cur, p.ops[o].Kp);
      if (!last) use(out, p.ops[o].Np);
      p.n_loop++;
      cur = out;
    }
    p.loops = samples_;
    p.mse_mode = 1;
    p.mse_dim = F_;
  }
  int off = 0;
  for (int b = 0; b < kern::kMlpMaxBufs; ++b) {
    if (!width[b]) continue;
    // ld = 8 (mod 16): ds_read_b128 A fragments (16 rows x 16 B per k quad)
    // are conflict-free in each of the instruction's four 16-lane groups
    p.buf_ld[b] = (width[b] + 15 - 8) / 16 * 16 + 8;
    p.buf_off[b] = off;
    off += kern::kMlpRows * p.buf_ld[b];
  }
  p.lds_floats = off;
  // 8 waves when a layer has >= 8 column tiles (more MFMA chains per tile of
  // rows at small batches; LDS-bound occupancy keeps ~1-2 workgroups per CU)
  int max_tiles = 0;
  for (int o = 0; o < p.n_pre + p.n_loop; ++o) max_tiles = std::max(max_tiles, p.ops[o].Np / 16);
  p.waves = max_tiles >= 8 ? 8 : 4;
  params_.resize(params_.size() + 4 * 64 * 4, 0.f);  // B look-ahead pad (4 blocks, mlp.hip dense())
  // A network whose activations do not fit one workgroup's 160 KiB of LDS
  // cannot use the fused kernel; it runs layer-wise (activations in HBM).
  fused_ok_ = (size_t(off) + kern::kMlpRows) * sizeof(float) <= 160 * 1024 && precision_ == 0;
  if (!fused_ok_) mode_ = 2;  // bf16 runs on the layer-wise GEMMs only
}

void MlpModel::to_device(int device) {
  d_params_.alloc(params_.size() * sizeof(float), device);
  d_params_.upload(params_.data(), params_.size() * sizeof(float));
  if (!pbf_.empty()) {
    d_pbf_.alloc(pbf_.size() * sizeof(uint16_t) + 64 * 16, device);  // + look-ahead pad
    d_pbf_.upload(pbf_.data(), pbf_.size() * sizeof(uint16_t));
  }
  if (!prm_.empty()) {
    d_prm_.alloc(prm_.size() * sizeof(float), device);
    d_prm_.upload(prm_.data(), prm_.size() * sizeof(float));
  }
}

// ------------------------------------------------------------ dispatch
// Cost model in CU-cycles (MI355X: 256 CUs x 4 MFMA pipes, one
// v_mfma_f32_16x16x4_f32 = 32 pipe cycles).  Fused: one workgroup per 16-row
// tile runs every layer, so a batch of few tiles leaves most CUs idle and
// the tile's MFMAs share one CU's 4 pipes.  Layer-wise: each layer spreads
// (row tiles x column tiles) single-wave tasks over all 1024 pipes, paying
// a launch gap and an L2 round trip per layer.
bool MlpModel::layerwise(int rows) const {
  if (mode_ == 1) return false;
  if (mode_ == 2) return true;
  const double row_tiles = std::ceil(rows / 16.0);
  const int S = vae_ ? samples_ : 1;
  double per_tile = 0, layer = 8000;  // convert + finish kernels
  for (int o = 0; o < prog_.n_pre + prog_.n_loop; ++o) {
    const auto& op = prog_.ops[o];
    if (op.type == kern::kMlpReparam) continue;
    const bool loop = o >= prog_.n_pre;
    const double mf = double(op.Np / 16) * (op.Kp / 16) * 4;
    per_tile += mf * (loop ? prog_.loops : 1);
    const double tasks = (loop ? std::ceil(rows * double(S) / 16.0) : row_tiles) * (op.Np / 16);
    layer += std::ceil(tasks / 1024.0) * (op.Kp / 16) * 4 * 32 + 1500 + 4000;
  }
  const double fused = std::max(1.0, row_tiles / 256.0) * per_tile * 8 + 2000;
  return layer < 0.9 * fused;
}

int MlpModel::max_np() const {
  int w = 16;
  for (int o = 0; o < prog_.n_pre + prog_.n_loop; ++o) w = std::max(w, prog_.ops[o].Np);
  return w;
}

size_t MlpModel::workspace_bytes(int max_rows, int) const {
  if (precision_ == 1) {
    const size_t R = size_t(round_up(std::max(max_rows, 1), 128)), S = vae_ ? size_t(samples_) : 1;
    size_t Wb = 64;
    for (int o = 0; o < prog_.n_pre + prog_.n_loop; ++o) Wb = std::max(Wb, size_t(prog_.ops[o].Npb));
    const size_t K0 = size_t(prog_.ops[0].Kpb), K0f = size_t(prog_.ops[0].Kp);
    // [x bf16 R x K0][buf0 bf16 R*S x Wb][buf1 bf16 R*S x Wb][x fp32 R x K0f][head/logits fp32 R x Wb][mse R]
    return (R * K0 + 2 * R * S * Wb) * 2 + (R * K0f + R * Wb + R) * 4 + 4 * 256;
  }
  if (mode_ == 1) return 0;
  if (mode_ == 0) {  // auto: only models the cost model ever sends layer-wise need one
    bool any = false;
    for (int r = 1; r <= std::max(max_rows, 1) && !any; r += (r < 64 ? 1 : 16)) any = layerwise(r);
    if (!any) return 0;
  }
  const size_t R = size_t(round_up(std::max(max_rows, 1), 16)), S = vae_ ? size_t(samples_) : 1;
  const size_t W = size_t(max_np()), K0 = size_t(round_up(prog_.ops[0].Kp, 32));
  // [X fp32 R x K0][buf0 R*S x W][buf1 R*S x W]([head R x W][mse R]), kSlack
  // floats after each: the layer kernel's A look-ahead reads up to 4 K-blocks
  // past the end of a row
  return (R * K0 + kSlack + 2 * (R * S * W + kSlack) + (vae_ ? R * W + kSlack + R : 0)) * sizeof(float);
}

void MlpModel::launch(const double* X, int rows, int, double* out, void* ws, hipStream_t s) {
  const uint64_t off = offset_.fetch_add(1);
  if (precision_ == 1) {
    if (!ws) throw std::runtime_error("MlpModel: bf16 network launched without a workspace");
    launch_layerwise_bf16(X, rows, out, static_cast<char*>(ws), seed_ ^ (off * 0x9E3779B97F4A7C15ULL), s);
    return;
  }
  if (!fused_ok_ && !ws) throw std::runtime_error("MlpModel: layer-wise network launched without a workspace");
  if (ws && layerwise(rows)) {
    launch_layerwise(X, rows, out, static_cast<float*>(ws), seed_ ^ (off * 0x9E3779B97F4A7C15ULL), s);
    return;
  }
  kern::mlp_forward(X, rows, prog_, d_params_.as<float>(), seed_, off, out, s);
}

void MlpModel::launch_layerwise(const double* X, int rows, double* out, float* ws, uint64_t key, hipStream_t s) {
  const float* P = d_params_.as<float>();
  const size_t R = size_t(round_up(rows, 16)), S = vae_ ? size_t(samples_) : 1, W = size_t(max_np());
  const size_t K0 = size_t(round_up(prog_.ops[0].Kp, 32));  // rows hold Kq readable floats (LDS-tiled GEMM)
  float* x32 = ws;
  float* buf[2] = {x32 + R * K0 + kSlack, x32 + R * K0 + kSlack + R * S * W + kSlack};
  float* head = buf[1] + R * S * W + kSlack;
  float* mse = head + R * W + kSlack;
  auto args = [&](const kern::MlpOp& op) {
    kern::MlpLayerArgs a;
    a.W = P + op.w_off;
    a.bias = P + op.b_off;
    a.K = op.K;
    a.Kp = op.Kp;
    a.N = op.N;
    a.Np = op.Np;
    a.act = op.act;
    a.rows = rows;
    a.rows_eff = rows;
    return a;
  };
  // encoder / plain stack: X -> x32 -> buf0 -> buf1 -> ...  A plain stack on
  // the LDS-tiled GEMM reads X (fp64) straight into its first layer's staging
  // (no convert pass; the VAE keeps x32 as its MSE reference) and writes the
  // model output from its last layer's epilogue (no mlp_finish).
  static const bool stage64 = [] { const char* v = std::getenv("SCA_MLP_DIRECT_IN"); return !v || atoi(v) != 0; }();
  const bool direct_in = stage64 && !vae_ && lds_layer(0, rows);
  if (!direct_in) kern::mlp_convert(X, rows, F_, int(K0), x32, s);
  const float* cur = x32;
  int cur_ld = int(K0), flip = 0;
  for (int o = 0; o < prog_.n_pre; ++o) {
    const auto& op = prog_.ops[o];
    kern::MlpLayerArgs a = args(op);
    a.A = cur;
    a.lda = cur_ld;
    const bool last = o + 1 == prog_.n_pre;
    a.O = vae_ && last ? head : buf[flip];
    a.ldo = op.Np;
    if (!vae_ && last && op.N <= 16 && lds_layer(o, rows) &&
        (prog_.out_softmax == 2 ? op.N == 1 && prog_.out_dim == 2 : prog_.out_dim == op.N)) {
      run_layer(a, o, s, o == 0 && direct_in ? X : nullptr, out);
      return;
    }
    run_layer(a, o, s, o == 0 && direct_in ? X : nullptr);
    cur = a.O;
    cur_ld = op.Np;
    flip ^= 1;
  }
  if (!vae_) {
    kern::mlp_finish(cur, cur_ld, rows, prog_.out_dim, prog_.out_softmax, out, s);
    return;
  }
  // decoder over rows x samples: reparam fused into the first layer's A, MSE into the last's epilogue
  (void)hipMemsetAsync(mse, 0, size_t(rows) * sizeof(float), s);
  const float* dcur = nullptr;
  int dld = 0;
  flip = 0;
  for (int o = prog_.n_pre; o < prog_.n_pre + prog_.n_loop; ++o) {
    const auto& op = prog_.ops[o];
    if (op.type == kern::kMlpReparam) continue;
    kern::MlpLayerArgs a = args(op);
    a.rows_eff = rows * int(S);
    if (!dcur) {
      a.H = head;
      a.ldh = prog_.ops[prog_.n_pre - 1].Np;
      a.latent = latent_;
      a.key = key;
    } else {
      a.A = dcur;
      a.lda = dld;
    }
    if (op.type == kern::kMlpDenseMse) {
      a.mse = mse;
      a.xref = x32;  // the fp32 input, as the fused kernel's LDS copy
      a.ldx = int(K0);
    } else {
      a.O = buf[flip];
      a.ldo = op.Np;
      dcur = a.O;
      dld = op.Np;
      flip ^= 1;
    }
    run_layer(a, o, s);
  }
  kern::mlp_mse_finish(mse, rows, 1.0 / (double(F_) * samples_), out, s);
}

// Large batches: the register-tiled GEMM (64 rows x up to 64 columns per
// wave); small ones: one 16x16 tile per wave (more waves for the chip).
bool MlpModel::lds_layer(int op, int rows_eff) const {
  return rows_eff >= kLdsGemmRows && wr_off_[size_t(op)] >= 0;
}

void MlpModel::run_layer(const kern::MlpLayerArgs& a, int op, hipStream_t s, const double* a64,
                         double* out64) const {
  if ((a64 || out64) && !lds_layer(op, a.rows_eff))
    throw std::logic_error("MlpModel::run_layer: fp64 A / fp64 output need the LDS-tiled GEMM");
  if (a.rows_eff < kGemmRows) {
    kern::mlp_layer(a, s);
    return;
  }
  kern::DenseGemmArgs g;
  const long long wr = wr_off_[size_t(op)];
  if (a.rows_eff >= kLdsGemmRows && !a.H && wr >= 0 && (a64 || (kq_[size_t(op)] <= a.lda && a.lda % 4 == 0))) {
    // A rows hold Kq floats (zeros past K), W row-major [Npb][Kq]: LDS-tiled exact-fp32 MFMA GEMM
    g.lds_f32 = 1;
    g.W = d_prm_.as<float>() + wr;
    g.Kp = kq_[size_t(op)];
    g.Np = prog_.ops[op].Npb;
    g.n_store = a.Np;  // the activation buffers are Np (16-padded) wide
  } else {
    g.W = a.W;
    g.Kp = a.Kp;
    g.Np = a.Np;
  }
  g.bias = a.bias;
  g.K = a.K;
  g.N = a.N;
  g.act = a.act;
  g.A = a.A;
  g.lda = a.lda;
  g.H = a.H;
  g.ldh = a.ldh;
  g.latent = a.latent;
  g.key = a.key;
  g.rows = a.rows;
  g.rows_eff = a.rows_eff;
  g.O = a.O;
  g.ldo = a.ldo;
  g.o_f32 = 1;
  g.mse = a.mse;
  g.xref = a.xref;
  g.ldx = a.ldx;
  if (a64) {  // fp64 rows [rows][K]: masked past K, converted to fp32 while staging
    g.A = a64;
    g.lda = F_;
    g.a_f64 = 1;
  }
  if (out64) {
    g.out64 = out64;
    g.out_mode = prog_.out_softmax;
  }
  kern::dense_gemm(g, s);
}

void MlpModel::launch_layerwise_bf16(const double* X, int rows, double* out, char* ws, uint64_t key, hipStream_t s) {
  const float* P = d_params_.as<float>();
  const uint16_t* Wb = d_pbf_.as<uint16_t>();
  const size_t R = size_t(round_up(rows, 128)), S = vae_ ? size_t(samples_) : 1;
  size_t Wmax = 64;
  for (int o = 0; o < prog_.n_pre + prog_.n_loop; ++o) Wmax = std::max(Wmax, size_t(prog_.ops[o].Npb));
  const size_t K0 = size_t(prog_.ops[0].Kpb), K0f = size_t(prog_.ops[0].Kp);
  uint16_t* xb = reinterpret_cast<uint16_t*>(ws);
  uint16_t* buf[2] = {xb + R * K0, xb + R * K0 + R * S * Wmax};
  float* x32 = reinterpret_cast<float*>(buf[1] + R * S * Wmax);
  float* head = x32 + R * K0f;
  float* mse = head + R * Wmax;
  auto args = [&](const kern::MlpOp& op) {
    kern::DenseGemmArgs a;
    a.bf16 = 1;
    a.W = Wb + op.wb_off;
    a.bias = P + op.b_off;
    a.K = op.K;
    a.Kp = op.Kpb;
    a.N = op.N;
    a.Np = op.Npb;
    a.act = op.act;
    a.rows = rows;
    a.rows_eff = rows;
    return a;
  };
  kern::convert_bf16(X, rows, F_, int(K0), xb, s);
  const void* cur = xb;
  int cur_ld = int(K0), flip = 0;
  for (int o = 0; o < prog_.n_pre; ++o) {
    const auto& op = prog_.ops[o];
    kern::DenseGemmArgs a = args(op);
    a.A = cur;
    a.lda = cur_ld;
    const bool last = o + 1 == prog_.n_pre;
    if (last && !vae_ && op.N <= 16 &&
        (prog_.out_softmax == 2 ? op.N == 1 && prog_.out_dim == 2 : prog_.out_dim == op.N)) {
      a.out64 = out;  // the epilogue writes the model output (mlp_finish fused)
      a.out_mode = prog_.out_softmax;
      kern::dense_gemm(a, s);
      return;
    }
    if (last) {  // plain MLP logits / VAE head [mu | log_var] in fp32
      a.O = head;
      a.o_f32 = 1;
    } else {
      a.O = buf[flip];
      a.o_f32 = 0;
      flip ^= 1;
    }
    a.ldo = op.Npb;
    kern::dense_gemm(a, s);
    cur = a.O;
    cur_ld = op.Npb;
  }
  if (!vae_) {
    kern::mlp_finish(head, cur_ld, rows, prog_.out_dim, prog_.out_softmax, out, s);
    return;
  }
  kern::mlp_convert(X, rows, F_, int(K0f), x32, s);  // fp32 reference rows for the MSE
  (void)hipMemsetAsync(mse, 0, size_t(rows) * sizeof(float), s);
  const void* dcur = nullptr;
  int dld = 0;
  flip = 0;
  for (int o = prog_.n_pre; o < prog_.n_pre + prog_.n_loop; ++o) {
    const auto& op = prog_.ops[o];
    if (op.type == kern::kMlpReparam) continue;
    kern::DenseGemmArgs a = args(op);
    a.rows_eff = rows * int(S);
    if (!dcur) {
      a.H = head;
      a.ldh = prog_.ops[prog_.n_pre - 1].Npb;
      a.latent = latent_;
      a.key = key;
    } else {
      a.A = dcur;
      a.lda = dld;
    }
    if (op.type == kern::kMlpDenseMse) {
      a.mse = mse;
      a.xref = x32;
      a.ldx = int(K0f);
    } else {
      a.O = buf[flip];
      a.o_f32 = 0;
      a.ldo = op.Npb;
      dcur = a.O;
      dld = op.Npb;
      flip ^= 1;
    }
    kern::dense_gemm(a, s);
  }
  kern::mlp_mse_finish(mse, rows, 1.0 / (double(F_) * samples_), out, s);
}

void MlpModel::cpu_dense(const DenseLayer& L, const std::vector<float>& in, std::vector<float>& out, int rows) const {
  out.assign(size_t(rows) * L.N, 0.f);
  for (int r = 0; r < rows; ++r)
    for (int n = 0; n < L.N; ++n) {
      float acc = 0.f;
      for (int k = 0; k < L.K; ++k) acc = std::fma(in[size_t(r) * L.K + k], L.W[size_t(n) * L.K + k], acc);
      out[size_t(r) * L.N + n] = act_host(acc + L.b[size_t(n)], L.act);
    }
}

void MlpModel::run_cpu(const double* X, int rows, int, double* out) const {
  std::vector<float> x(size_t(rows) * F_), a, b;
  for (size_t i = 0; i < x.size(); ++i) x[i] = float(X[i]);
  a = x;
  for (const auto& L : enc_) {
    cpu_dense(L, a, b, rows);
    a.swap(b);
  }
  if (!vae_) {
    const int N = enc_.back().N;
    for (int r = 0; r < rows; ++r) {
      const float* o = a.data() + size_t(r) * N;
      if (out_mode_ == kOutBinary) {
        out[size_t(r) * 2] = 1.0 - double(o[0]);
        out[size_t(r) * 2 + 1] = double(o[0]);
      } else if (out_mode_ == kOutSoftmax) {
        float m = *std::max_element(o, o + N), sum = 0.f;
        for (int c = 0; c < N; ++c) sum += std::exp(o[c] - m);
        for (int c = 0; c < N; ++c) out[size_t(r) * N + c] = double(std::exp(o[c] - m) / sum);
      } else {
        for (int c = 0; c < N; ++c) out[size_t(r) * N + c] = double(o[c]);
      }
    }
    return;
  }
  const uint64_t key = seed_ ^ (const_cast<std::atomic<uint64_t>&>(offset_).fetch_add(1) * 0x9E3779B97F4A7C15ULL);
  std::vector<double> mse(size_t(rows), 0.0);
  std::vector<float> z(size_t(rows) * latent_);
  for (int s = 0; s < samples_; ++s) {
    for (int r = 0; r < rows; ++r)
      for (int j = 0; j < latent_; ++j) {
        HostPhilox rng(key, (uint64_t(r) << 24) ^ (uint64_t(s) << 14) ^ uint64_t(j));
        const float eps = rng.normal();
        const float* h = a.data() + size_t(r) * 2 * latent_;
        z[size_t(r) * latent_ + j] = h[j] + std::exp(0.5f * h[latent_ + j]) * eps;
      }
    std::vector<float> d = z, e;
    for (const auto& L : dec_) {
      cpu_dense(L, d, e, rows);
      d.swap(e);
    }
    for (int r = 0; r < rows; ++r) {
      float acc = 0.f;
      for (int c = 0; c < F_; ++c) {
        const float diff = d[size_t(r) * F_ + c] - x[size_t(r) * F_ + c];
        acc += diff * diff;
      }
      mse[size_t(r)] += double(acc);
    }
  }
  for (int r = 0; r < rows; ++r) out[r] = mse[size_t(r)] / (double(F_) * samples_);
}

std::shared_ptr<RowModel> MlpModel::clone() const {
  std::shared_ptr<MlpModel> m = vae_ ? vae(enc_, latent_, dec_, samples_, seed_)
                                     : std::make_shared<MlpModel>(enc_, out_mode_);
  if (precision_) m->set_precision(precision_);
  return with_meta(m);
}

}  // namespace sca::gpu
