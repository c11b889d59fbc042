// RCCL fabric: cross-process (one process per MI355X) graph edges over xGMI.
//
// The reference fans a request out to child microservices over HTTP/gRPC
// (PredictiveUnitBean.java:170-183 -> InternalPredictionService.java:186-453)
// and joins their outputs for the combiner / returns the routed child's output.
// With one engine process per GPU, the front-end rank keeps the graph and the
// request queue; children placed on other ranks are reached with RCCL
// point-to-point transfers of whole micro-batches, GPU memory to GPU memory:
//
//   rank 0 (front end)                      rank r (worker)
//   ------------------                      ---------------
//   send header {op, model, rows, cols} --> recv header, spin until visible
//   send X [rows, cols] fp64 ------------> recv X
//                                          model.launch(X) on the worker's GPU
//   recv Y [rows, out_cols] <------------- send Y
//
// A fan-out to K ranks (COMBINER over replicas on K GPUs) is one RCCL group:
// the K sends are the scatter/broadcast, the K receives the gather, and the
// combine kernel runs on rank 0's GPU.  All fabric operations of a rank are
// issued from one stream in one order (a per-fabric mutex), so the sequence
// each worker observes is exactly header, payload, reply -- no deadlock, no
// tag matching needed.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../gpu/hip_util.h"
#include "../gpu/models.h"

namespace sca::par {

std::string rccl_unique_id();  // 128 opaque bytes; rank 0 creates, everyone receives it out of band

class Fabric {
 public:
  Fabric(int rank, int world, const std::string& unique_id, int device);
  ~Fabric();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  ncclComm_t comm() const { return comm_; }
  hipStream_t stream() const { return stream_.get(); }
  std::mutex& issue_mutex() { return mu_; }
  void close();

 private:
  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  gpu::Stream stream_;
  std::mutex mu_;
};
using FabricPtr = std::shared_ptr<Fabric>;

enum PeerOp : int32_t { kPeerStop = 0, kPeerRun = 1 };

// Front-end side: a row model whose computation happens on other ranks.
// `peers` = ranks holding a replica (model index `model_id` in each rank's
// PeerServer).  One peer: a remote MODEL node.  Several peers: COMBINER over
// replicas -- the batch is broadcast to every peer and the outputs gathered and
// averaged on this GPU.
class PeerRowModel : public gpu::RowModel {
 public:
  PeerRowModel(FabricPtr fabric, std::vector<int> peers, int model_id, int in_cols, int out_cols);
  ~PeerRowModel() override;
  std::string name() const override { return "rccl_peer"; }
  int in_cols() const override { return in_cols_; }
  int out_cols(int) const override { return out_cols_; }
  bool device_io_only() const override { return true; }
  void to_device(int device) override;
  size_t workspace_bytes(int max_rows, int cols) const override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void run_cpu(const double*, int, int, double*) const override;

 private:
  FabricPtr f_;
  std::vector<int> peers_;
  int model_id_, in_cols_, out_cols_;
  gpu::Event ev_in_, ev_done_;
  gpu::PinnedBuffer ptrs_;
};

// Worker side: serves the row models placed on this rank until rank 0 sends
// a stop header.
class PeerServer {
 public:
  explicit PeerServer(FabricPtr fabric);
  ~PeerServer();
  int add_model(gpu::RowModelPtr m);  // returns model_id (registration order)
  void start();
  void join();
  uint64_t batches() const { return batches_.load(); }
  uint64_t rows() const { return rows_.load(); }
  std::string error() const;

 private:
  void loop();
  FabricPtr f_;
  std::vector<gpu::RowModelPtr> models_;
  std::thread th_;
  std::atomic<uint64_t> batches_{0}, rows_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

// Front end: tell every worker rank to leave its serve loop.
void stop_peers(Fabric& f);

}  // namespace sca::par
