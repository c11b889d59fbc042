#include "lstm_model.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace sca::gpu {

namespace {
int round_up(int x, int m) { return (x + m - 1) / m * m; }
// smallest stride >= k with stride == r (mod 32)
int stride_mod32(int k, int r) { return k + ((r - k) % 32 + 32) % 32; }
constexpr int kMaxLdsFloats = 160 * 1024 / 4;

void check_cell(const LstmWeights& w, int in, const char* what) {
  if (w.H <= 0 || w.in != in || w.W_ih.size() != size_t(4 * w.H) * in || w.W_hh.size() != size_t(4 * w.H) * w.H ||
      w.b.size() != size_t(4 * w.H))
    throw std::runtime_error(std::string("LstmSeqModel: bad ") + what + " weights");
}
}  // namespace

LstmSeqModel::LstmSeqModel(int T, int F, std::vector<std::pair<LstmWeights, LstmWeights>> enc,
                           std::vector<LstmWeights> dec, std::vector<float> dense_W, std::vector<float> dense_b,
                           int out_act)
    : T_(T), F_(F), out_act_(out_act), enc_(std::move(enc)), dec_(std::move(dec)), dW_(std::move(dense_W)),
      db_(std::move(dense_b)) {
  if (T_ < 1 || F_ < 1) throw std::runtime_error("LstmSeqModel: need T >= 1 and F >= 1");
  if (enc_.empty() || dec_.empty() || int(enc_.size()) > kern::kLstmMaxLayers ||
      int(dec_.size()) > kern::kLstmMaxLayers)
    throw std::runtime_error("LstmSeqModel: 1..4 encoder and decoder layers");
  int in = F_;
  for (auto& e : enc_) {
    check_cell(e.first, in, "encoder");
    check_cell(e.second, in, "encoder");
    if (e.first.H != e.second.H) throw std::runtime_error("LstmSeqModel: directions differ in width");
    in = 2 * e.first.H;
  }
  const int Hs = 2 * enc_.back().first.H;
  in = F_;
  for (auto& d : dec_) {
    check_cell(d, in, "decoder");
    if (d.H != Hs) throw std::runtime_error("LstmSeqModel: decoder units must equal 2 x encoder units");
    in = d.H;
  }
  if (dW_.size() != size_t(F_) * Hs || db_.size() != size_t(F_))
    throw std::runtime_error("LstmSeqModel: bad dense output weights");
  build();
}

void LstmSeqModel::build() {
  auto& p = prog_;
  p = kern::LstmProgram();
  p.T = T_;
  p.F = F_;
  p.n_enc = int(enc_.size());
  p.n_dec = int(dec_.size());
  p.D = dec_.back().H;
  p.out_act = out_act_;
  params_.clear();
  auto pad4 = [&] { params_.resize(size_t(round_up(int(params_.size()), 4)), 0.f); };
  // B fragments of one cell: frag[tile][ks][lane] = Wcat[tile*16 + lane%16][4 ks + lane/16]
  auto pack = [&](const LstmWeights& w, kern::LstmCell& c, long long phase) {
    c.in = w.in;
    c.H = w.H;
    c.Kp = round_up(w.in + w.H, 4);
    c.Np = round_up(4 * w.H, 16);
    c.lda = stride_mod32(c.Kp + 4, 2);  // + 4: the dense GEMM's A (h part) may read 3 past H
    c.ldg = c.Np + 4;
    c.w_off = int(params_.size() - size_t(phase));
    const int ntiles = c.Np / 16, ksteps = c.Kp / 4;
    for (int t = 0; t < ntiles; ++t)
      for (int ks = 0; ks < ksteps; ++ks)
        for (int lane = 0; lane < 64; ++lane) {
          const int col = t * 16 + (lane & 15), k = 4 * ks + (lane >> 4);
          float v = 0.f;
          if (col < 4 * w.H) {
            if (k < w.in) v = w.W_ih[size_t(col) * w.in + k];
            else if (k < w.in + w.H) v = w.W_hh[size_t(col) * w.H + (k - w.in)];
          }
          params_.push_back(v);
        }
    pad4();
    c.b_off = int(params_.size() - size_t(phase));
    params_.insert(params_.end(), w.b.begin(), w.b.end());
    params_.resize(params_.size() + size_t(c.Np - 4 * w.H), 0.f);
    pad4();
  };
  int wmax = 0;
  for (int l = 0; l < p.n_enc; ++l) {
    const long long ph = (long long)params_.size();
    p.enc_phase[l] = ph;
    pack(enc_[size_t(l)].first, p.enc[l][0], ph);
    pack(enc_[size_t(l)].second, p.enc[l][1], ph);
    p.enc_phase_floats[l] = int(params_.size() - size_t(ph));
    wmax = std::max(wmax, p.enc_phase_floats[l]);
  }
  {
    const long long ph = (long long)params_.size();
    p.dec_phase = ph;
    for (int l = 0; l < p.n_dec; ++l) pack(dec_[size_t(l)], p.dec[l], ph);
    p.dense_w = int(params_.size() - size_t(ph));
    p.dense_kp = round_up(p.D, 4);
    p.dense_np = round_up(F_, 16);
    for (int t = 0; t < p.dense_np / 16; ++t)
      for (int ks = 0; ks < p.dense_kp / 4; ++ks)
        for (int lane = 0; lane < 64; ++lane) {
          const int col = t * 16 + (lane & 15), k = 4 * ks + (lane >> 4);
          params_.push_back(col < F_ && k < p.D ? dW_[size_t(col) * p.D + k] : 0.f);
        }
    pad4();
    p.dense_b = int(params_.size() - size_t(ph));
    params_.insert(params_.end(), db_.begin(), db_.end());
    pad4();
    p.dec_phase_floats = int(params_.size() - size_t(ph));
    wmax = std::max(wmax, p.dec_phase_floats);
  }
  // LDS: [weights of the running phase][encoder A/G/C x 2 dirs, shared by all
  // encoder layers][decoder A/G/C per layer][mse]
  const int R = kern::kLstmRows;
  int enc_floats = 0;
  int a = 0, g = 0, cst = 0;
  for (int l = 0; l < p.n_enc; ++l) {
    a = std::max(a, R * p.enc[l][0].lda);
    g = std::max(g, R * p.enc[l][0].ldg);
    cst = std::max(cst, R * p.enc[l][0].H);
  }
  a = round_up(a, 4);
  g = round_up(g, 4);
  cst = round_up(cst, 4);
  enc_floats = 2 * (a + g + cst);
  int dec_floats = 0;
  for (int l = 0; l < p.n_dec; ++l)
    dec_floats += round_up(R * p.dec[l].lda, 4) + round_up(R * p.dec[l].ldg, 4) + round_up(R * p.dec[l].H, 4);
  const int rest = enc_floats + dec_floats + R + R * (round_up(F_, 16) + 4) + 8;
  p.w_lds = rest + wmax <= kMaxLdsFloats ? 1 : 0;
  p.w_region = p.w_lds ? round_up(wmax, 4) : 0;
  int off = p.w_region;
  for (int d = 0; d < 2; ++d) {
    for (int l = 0; l < p.n_enc; ++l) {
      p.enc[l][d].a_off = off;
      p.enc[l][d].g_off = off + a;
      p.enc[l][d].c_off = off + a + g;
    }
    off += a + g + cst;
  }
  for (int l = 0; l < p.n_dec; ++l) {
    auto& c = p.dec[l];
    c.a_off = off;
    off += round_up(R * c.lda, 4);
    c.g_off = off;
    off += round_up(R * c.ldg, 4);
    c.c_off = off;
    off += round_up(R * c.H, 4);
  }
  p.mse_off = off;
  off += R;
  p.y_off = round_up(off, 4);
  off = p.y_off + R * (p.dense_np + 4);
  const int xtile = R * T_ * F_;
  if (off + xtile <= kMaxLdsFloats) {  // input tile in LDS
    p.x_lds = 1;
    p.x_off = round_up(off, 4);
    off = p.x_off + xtile;
  }
  p.lds_floats = off;
  if (p.lds_floats > kMaxLdsFloats) throw std::runtime_error("LstmSeqModel: state does not fit the 160 KiB LDS");
  int hmax = 0;
  for (auto& e : enc_) hmax = std::max(hmax, e.first.H);
  p.Hmax2 = 2 * hmax;
  p.seq_ws_floats = p.n_enc > 1 ? 2LL * R * T_ * p.Hmax2 : 0;
  build_valu();
}

// Small-batch VALU programs (csrc/kernels/lstm_valu.hip), appended to the
// same parameter blob: per cell [H][Q][4][KPL] (k < H: W_hh, then W_ih, zero
// pad), bias [4][H]; Dense [F][Qy][KPL].  KPL is the smallest of 8/16/32 whose
// lane layout fits 1024 threads; R = 1, 2, 4 rows per workgroup.
void LstmSeqModel::build_valu() {
  for (auto& v : vprog_) v = kern::LstmvProgram();
  auto pow2 = [](int x) {
    int q = 1;
    while (q < x) q <<= 1;
    return q;
  };
  int kpl = 0;
  int threads = 0;
  for (int cand : {8, 16, 32}) {
    auto q_of = [&](int K) { return pow2((K + cand - 1) / cand); };
    int enc_t = 0;
    for (auto& e : enc_) enc_t = std::max(enc_t, 2 * round_up(e.first.H * q_of(e.first.H + e.first.in), 64));
    int dec_t = 0;
    for (auto& d : dec_) dec_t += round_up(d.H * q_of(d.H + d.in), 64);
    const int Qy = q_of(dec_.back().H);
    dec_t += round_up(F_ * Qy, 64);
    bool qok = Qy <= 64;
    for (auto& e : enc_) qok = qok && q_of(e.first.H + e.first.in) <= 64;
    for (auto& d : dec_) qok = qok && q_of(d.H + d.in) <= 64;
    if (qok && std::max(enc_t, dec_t) <= 1024) {
      kpl = cand;
      threads = std::max(enc_t, dec_t);
      break;
    }
  }
  if (!kpl) return;
  auto pad4 = [&] { params_.resize(size_t(round_up(int(params_.size()), 4)), 0.f); };
  auto q_of = [&](int K) { return pow2((K + kpl - 1) / kpl); };
  struct Packed {
    long long w_off, b_off;
    int Q;
  };
  auto pack = [&](const LstmWeights& w) {
    Packed r;
    const int K = w.H + w.in;
    r.Q = q_of(K);
    pad4();
    r.w_off = (long long)params_.size();
    for (int u = 0; u < w.H; ++u)
      for (int q = 0; q < r.Q; ++q)
        for (int g = 0; g < 4; ++g)
          for (int j = 0; j < kpl; ++j) {
            const int k = q * kpl + j, row = g * w.H + u;
            float v = 0.f;
            if (k < w.H) v = w.W_hh[size_t(row) * w.H + k];
            else if (k < K) v = w.W_ih[size_t(row) * w.in + (k - w.H)];
            params_.push_back(v);
          }
    pad4();
    r.b_off = (long long)params_.size();
    params_.insert(params_.end(), w.b.begin(), w.b.end());
    return r;
  };
  std::vector<std::pair<Packed, Packed>> penc;
  for (auto& e : enc_) penc.emplace_back(pack(e.first), pack(e.second));
  std::vector<Packed> pdec;
  for (auto& d : dec_) pdec.push_back(pack(d));
  const int D = dec_.back().H, Qy = q_of(D);
  pad4();
  const long long yw = (long long)params_.size();
  for (int f = 0; f < F_; ++f)
    for (int q = 0; q < Qy; ++q)
      for (int j = 0; j < kpl; ++j) {
        const int k = q * kpl + j;
        params_.push_back(k < D ? dW_[size_t(f) * D + k] : 0.f);
      }
  pad4();
  const long long yb = (long long)params_.size();
  params_.insert(params_.end(), db_.begin(), db_.end());
  pad4();

  const int Rs[3] = {1, 2, 4};
  for (int ri = 0; ri < 3; ++ri) {
    const int R = Rs[ri];
    kern::LstmvProgram& p = vprog_[ri];
    p.T = T_;
    p.F = F_;
    p.n_enc = int(enc_.size());
    p.n_dec = int(dec_.size());
    p.R = R;
    p.KPL = kpl;
    p.threads = threads;
    p.D = D;
    p.Qy = Qy;
    p.out_act = out_act_;
    p.yw_off = yw;
    p.yb_off = yb;
    int off = 0;
    p.x_off = off;
    off += round_up(R * T_ * F_, 4);
    auto set_cell = [&](kern::LstmvCell& c, const LstmWeights& w, const Packed& pk, int lane0) {
      c.in = w.in;
      c.H = w.H;
      c.Q = pk.Q;
      c.Kv = pk.Q * kpl;
      c.lane0 = lane0;
      c.w_off = pk.w_off;
      c.b_off = pk.b_off;
      c.v_off = off;
      off += 2 * R * c.Kv;
    };
    for (size_t l = 0; l < enc_.size(); ++l) {
      set_cell(p.enc[l][0], enc_[l].first, penc[l].first, 0);
      set_cell(p.enc[l][1], enc_[l].second, penc[l].second, round_up(enc_[l].first.H * penc[l].first.Q, 64));
    }
    int lane = 0;
    for (size_t l = 0; l < dec_.size(); ++l) {
      set_cell(p.dec[l], dec_[l], pdec[l], lane);
      lane += round_up(dec_[l].H * pdec[l].Q, 64);
    }
    p.y_lane0 = lane;
    int hmax = 0;
    for (auto& e : enc_) hmax = std::max(hmax, e.first.H);
    p.seq_ld = round_up(2 * hmax, 4);
    if (enc_.size() > 1) {
      p.seq_off[0] = off;
      off += R * T_ * p.seq_ld;
      p.seq_off[1] = off;
      off += R * T_ * p.seq_ld;
    }
    const int He2 = 2 * enc_.back().first.H;
    p.hfin_off = off;
    off += round_up(R * He2, 4);
    p.cfin_off = off;
    off += round_up(R * He2, 4);
    p.mse_off = off;
    off += round_up(R, 4);
    p.lds_floats = off;
    p.ok = off <= kMaxLdsFloats ? 1 : 0;
  }
}

std::string LstmSeqModel::path_for(int rows) const {
  if (const char* e = std::getenv("SCA_LSTM_PATH")) {
    if (!std::strcmp(e, "mfma")) return "mfma";
    if (!std::strcmp(e, "valu") && valu_program(4).ok) return "valu";
  }
  const int R = (rows + n_cu_ - 1) / n_cu_;
  return R <= kern::kLstmvMaxRows && valu_program(R).ok ? "valu" : "mfma";
}

void LstmSeqModel::to_device(int device) {
  d_params_.alloc(params_.size() * sizeof(float), device);
  d_params_.upload(params_.data(), params_.size() * sizeof(float));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    n_cu_ = prop.multiProcessorCount;
}

size_t LstmSeqModel::workspace_bytes(int max_rows, int) const {
  const size_t wgs = size_t((std::max(max_rows, 1) + kern::kLstmRows - 1) / kern::kLstmRows);
  return wgs * size_t(prog_.seq_ws_floats) * sizeof(float);
}

void LstmSeqModel::launch(const double* X, int rows, int, double* out, void* ws, hipStream_t s) {
  if (path_for(rows) == "valu") {
    // rows per workgroup: spread the batch over the CUs first (R = 1 up to one sequence per CU)
    int R = (rows + n_cu_ - 1) / n_cu_;
    R = R <= 1 ? 1 : R <= 2 ? 2 : 4;
    kern::lstm_valu_mse(X, rows, valu_program(R), d_params_.as<float>(), out, s);
    return;
  }
  kern::lstm_seq2seq_mse(X, rows, prog_, d_params_.as<float>(), static_cast<float*>(ws), out, s);
}

// ------------------------------------------------------------ CPU reference
namespace {
float sigm(float x) { return 1.f / (1.f + std::exp(-x)); }

// One LSTM step for one sequence: h, c updated in place.
void cell_step(const LstmWeights& w, const float* x, std::vector<float>& h, std::vector<float>& c) {
  const int H = w.H;
  std::vector<float> g(size_t(4 * H));
  for (int r = 0; r < 4 * H; ++r) {
    float acc = w.b[size_t(r)];
    for (int k = 0; k < w.in; ++k) acc += w.W_ih[size_t(r) * w.in + k] * x[k];
    for (int k = 0; k < H; ++k) acc += w.W_hh[size_t(r) * H + k] * h[size_t(k)];
    g[size_t(r)] = acc;
  }
  for (int u = 0; u < H; ++u) {
    const float i = sigm(g[size_t(u)]), f = sigm(g[size_t(H + u)]), gg = std::tanh(g[size_t(2 * H + u)]),
                o = sigm(g[size_t(3 * H + u)]);
    c[size_t(u)] = f * c[size_t(u)] + i * gg;
    h[size_t(u)] = o * std::tanh(c[size_t(u)]);
  }
}
}  // namespace

void LstmSeqModel::run_cpu(const double* X, int rows, int, double* out) const {
  const int T = T_, F = F_;
  for (int r = 0; r < rows; ++r) {
    std::vector<float> seq(size_t(T) * F);
    for (size_t i = 0; i < seq.size(); ++i) seq[i] = float(X[size_t(r) * T * F + i]);
    int in = F;
    std::vector<float> hf, cf, hb, cb;
    for (size_t l = 0; l < enc_.size(); ++l) {
      const auto& fw = enc_[l].first;
      const auto& bw = enc_[l].second;
      const int H = fw.H;
      hf.assign(size_t(H), 0.f);
      cf.assign(size_t(H), 0.f);
      hb.assign(size_t(H), 0.f);
      cb.assign(size_t(H), 0.f);
      std::vector<float> nxt(size_t(T) * 2 * H);
      for (int t = 0; t < T; ++t) {
        cell_step(fw, &seq[size_t(t) * in], hf, cf);
        std::copy(hf.begin(), hf.end(), nxt.begin() + size_t(t) * 2 * H);
      }
      for (int t = T - 1; t >= 0; --t) {
        cell_step(bw, &seq[size_t(t) * in], hb, cb);
        std::copy(hb.begin(), hb.end(), nxt.begin() + size_t(t) * 2 * H + H);
      }
      seq.swap(nxt);
      in = 2 * H;
    }
    std::vector<float> h0(hf), c0(cf);
    h0.insert(h0.end(), hb.begin(), hb.end());
    c0.insert(c0.end(), cb.begin(), cb.end());
    std::vector<std::vector<float>> hs(dec_.size(), h0), cs(dec_.size(), c0);
    std::vector<float> target(X + size_t(r) * T * F, X + size_t(r) * T * F + F);
    std::vector<float> inp;
    double err = 0.0;
    const int D = dec_.back().H;
    for (int t = 1; t < T; ++t) {
      inp = target;
      for (size_t l = 0; l < dec_.size(); ++l) {
        cell_step(dec_[l], inp.data(), hs[l], cs[l]);
        inp = hs[l];
      }
      for (int f = 0; f < F; ++f) {
        float acc = db_[size_t(f)];
        for (int k = 0; k < D; ++k) acc += dW_[size_t(f) * D + k] * inp[size_t(k)];
        float y = acc;
        if (out_act_ == 1) y = sigm(acc);
        else if (out_act_ == 2) y = std::tanh(acc);
        else if (out_act_ == 3) y = acc > 0.f ? acc : 0.f;
        target[size_t(f)] = y;
        const double d = double(float(X[(size_t(r) * T + t) * F + f])) - double(y);
        err += d * d;
      }
    }
    out[r] = err / double(T * F);
  }
}

std::shared_ptr<RowModel> LstmSeqModel::clone() const {
  return with_meta(std::make_shared<LstmSeqModel>(T_, F_, enc_, dec_, dW_, db_, out_act_));
}

}  // namespace sca::gpu
