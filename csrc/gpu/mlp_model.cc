#include "mlp_model.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace sca::gpu {

namespace {

int round_up(int x, int m) { return (x + m - 1) / m * m; }

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
  op.Kp = round_up(L.K, 4);
  op.N = L.N;
  op.Np = round_up(L.N, 16);
  // Wt [Kp][Np] + b [Np], zero padded
  op.w_off = (long long)params_.size();
  params_.resize(params_.size() + size_t(op.Kp) * op.Np, 0.f);
  for (int nn = 0; nn < L.N; ++nn)
    for (int k = 0; k < L.K; ++k) params_[size_t(op.w_off) + size_t(k) * op.Np + nn] = L.W[size_t(nn) * L.K + k];
  op.b_off = (long long)params_.size();
  params_.resize(params_.size() + size_t(op.Np), 0.f);
  for (int nn = 0; nn < L.N; ++nn) params_[size_t(op.b_off) + nn] = L.b[size_t(nn)];
  return n;
}

void MlpModel::build() {
  prog_ = kern::MlpProgram();
  params_.clear();
  auto& p = prog_;
  p.F = F_;
  p.Fp = round_up(F_, 4);
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
    p.buf_ld[b] = width[b] | 1;  // odd stride: the 16 rows of a fragment land in distinct banks
    p.buf_off[b] = off;
    off += kern::kMlpRows * p.buf_ld[b];
  }
  p.lds_floats = off;
  if ((size_t(off) + kern::kMlpRows) * sizeof(float) > 160 * 1024)
    throw std::runtime_error("MlpModel: layer widths exceed the 160 KiB LDS budget of one workgroup");
}

void MlpModel::to_device(int device) {
  d_params_.alloc(params_.size() * sizeof(float), device);
  d_params_.upload(params_.data(), params_.size() * sizeof(float));
}

void MlpModel::launch(const double* X, int rows, int, double* out, void*, hipStream_t s) {
  kern::mlp_forward(X, rows, prog_, d_params_.as<float>(), seed_, offset_.fetch_add(1), out, s);
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
  if (vae_) {
    auto m = vae(enc_, latent_, dec_, samples_, seed_);
    return with_meta(m);
  }
  return with_meta(std::make_shared<MlpModel>(enc_, out_mode_));
}

}  // namespace sca::gpu
