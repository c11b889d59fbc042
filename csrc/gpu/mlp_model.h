// Dense networks served by the fused MLP kernel (csrc/kernels/mlp.hip).
//
// Two shapes:
//  * plain MLP -- sklearn MLPClassifier/Regressor, torch nn.Sequential of
//    Linear + activations, Keras Dense stacks: output = last layer (optional
//    row softmax, or binary-logistic [1 - p, p] expansion);
//  * VAE reconstruction error -- the VAE outlier detector's model
//    (components/outlier-detection/vae/model.py:23-91): encoder Dense layers,
//    a head layer with 2*latent outputs [z_mean | z_log_var], reparameterised
//    sampling, decoder Dense layers; output = mean over `samples` MC draws of the
//    row MSE between reconstruction and input (CoreVAE.py:131-137).
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "models.h"

namespace sca::gpu {

struct DenseLayer {
  std::vector<float> W;  // [N][K] row-major (torch Linear layout)
  std::vector<float> b;  // [N]
  int K = 0, N = 0;
  int act = 0;           // kern::MlpAct
};

class MlpModel : public RowModel {
 public:
  enum OutMode { kOutPlain = 0, kOutSoftmax = 1, kOutBinary = 2 };
  MlpModel(std::vector<DenseLayer> layers, int out_mode);
  static std::shared_ptr<MlpModel> vae(std::vector<DenseLayer> encoder, int latent, std::vector<DenseLayer> decoder,
                                       int samples, uint64_t seed);

  std::string name() const override { return vae_ ? "vae_mse" : "mlp"; }
  int in_cols() const override { return F_; }
  int out_cols(int) const override { return out_dim_; }
  void to_device(int device) override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  // Layer-wise path (one launch per layer over rows x column tiles) for
  // batches whose 16-row tiles cannot fill the chip; needs the workspace.
  size_t workspace_bytes(int max_rows, int cols) const override;
  bool layerwise(int rows) const;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  std::shared_ptr<RowModel> clone() const override;
  const kern::MlpProgram& program() const { return prog_; }
  // 0 = fp32 (exact f32 MFMA products, Keras / torch float32 numerics);
  // 1 = bf16 operands, fp32 accumulation (per-model opt-in, ~1e-2 relative).
  void set_precision(int p);
  int precision() const { return precision_; }
  void set_seed(uint64_t seed) { seed_ = seed; }

 private:
  MlpModel() = default;
  void build();
  int add_layer(const DenseLayer& L, int type, int in_buf, int out_buf);
  void cpu_dense(const DenseLayer& L, const std::vector<float>& in, std::vector<float>& out, int rows) const;
  void launch_layerwise(const double* X, int rows, double* out, float* ws, uint64_t key, hipStream_t s);
  void launch_layerwise_bf16(const double* X, int rows, double* out, char* ws, uint64_t key, hipStream_t s);
  // a64: fp64 request rows [rows][F] as A (converted while staging; LDS path only);
  // out64: write the model output from the epilogue (LDS path, N <= 16)
  void run_layer(const kern::MlpLayerArgs& a, int op, hipStream_t s, const double* a64 = nullptr,
                 double* out64 = nullptr) const;
  bool lds_layer(int op, int rows_eff) const;
  int max_np() const;

  std::vector<DenseLayer> enc_, dec_;  // plain: enc_ = all layers
  bool vae_ = false;
  int latent_ = 0, samples_ = 0, out_mode_ = 0;
  int F_ = 0, out_dim_ = 0;
  uint64_t seed_ = 0;
  std::atomic<uint64_t> offset_{0};  // advances per launch: fresh MC draws per request
  int mode_ = 0;                     // SCA_MLP_MODE: 0 auto, 1 fused, 2 layer-wise
  bool fused_ok_ = true;             // activations fit one workgroup's LDS
  int precision_ = 0;
  std::vector<uint16_t> pbf_;        // bf16 weights (precision_ == 1)
  DeviceBuffer d_pbf_;
  // fp32 weights row-major [Npb][Kq] (Kq = K rounded to 32) for the LDS-tiled
  // exact-fp32 GEMM of large batches; per op index, -1 = none
  std::vector<float> prm_;
  std::vector<long long> wr_off_;
  std::vector<int> kq_;
  DeviceBuffer d_prm_;
  kern::MlpProgram prog_;
  std::vector<float> params_;
  DeviceBuffer d_params_;
};

}  // namespace sca::gpu
