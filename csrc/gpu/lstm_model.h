// Seq2seq LSTM reconstruction-error model (seq2seq outlier detector, SURVEY
// K11; reference components/outlier-detection/seq2seq-lstm/model.py:6-92 and
// CoreSeq2SeqLSTM.py:107-174).  A row is one flattened [T, F] sequence; the
// output is its reconstruction MSE after the greedy T-1 step decode.  GPU
// path: one persistent MFMA kernel per batch (csrc/kernels/lstm.hip).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../kernels/kernels.h"
#include "hip_util.h"
#include "models.h"

namespace sca::gpu {

struct LstmWeights {  // one direction of one layer, torch layout (gate order i, f, g, o)
  std::vector<float> W_ih;  // [4H][in]
  std::vector<float> W_hh;  // [4H][H]
  std::vector<float> b;     // [4H] = b_ih + b_hh
  int in = 0, H = 0;
};

class LstmSeqModel : public RowModel {
 public:
  // enc[l] = {forward, backward}; dec[l]; dense W [F][D], b [F]; out_act 0 linear, 1 sigmoid, 2 tanh, 3 relu
  LstmSeqModel(int T, int F, std::vector<std::pair<LstmWeights, LstmWeights>> enc, std::vector<LstmWeights> dec,
               std::vector<float> dense_W, std::vector<float> dense_b, int out_act);

  std::string name() const override { return "lstm_seq2seq_mse"; }
  int in_cols() const override { return T_ * F_; }
  int out_cols(int) const override { return 1; }
  void to_device(int device) override;
  bool zero_copy_input() const override { return false; }  // every step re-reads x: stage it in HBM
  size_t workspace_bytes(int max_rows, int cols) const override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  std::shared_ptr<RowModel> clone() const override;
  const kern::LstmProgram& program() const { return prog_; }
  // Small-batch VALU program for R rows per workgroup (R = 1, 2, 4); ok == 0
  // when the model does not fit it (the MFMA kernel then serves every batch).
  const kern::LstmvProgram& valu_program(int R) const { return vprog_[R <= 1 ? 0 : R <= 2 ? 1 : 2]; }
  // Which kernel a batch of `rows` runs: "valu" or "mfma" (SCA_LSTM_PATH forces one).
  std::string path_for(int rows) const;

 private:
  void build();
  void build_valu();
  int T_, F_, out_act_;
  std::vector<std::pair<LstmWeights, LstmWeights>> enc_;
  std::vector<LstmWeights> dec_;
  std::vector<float> dW_, db_;
  kern::LstmProgram prog_;
  kern::LstmvProgram vprog_[3];
  int n_cu_ = 256;
  std::vector<float> params_;
  DeviceBuffer d_params_;
};

}  // namespace sca::gpu
