// Cross-process graph edges (one engine process per MI355X).
//
// The reference fans a request out to child microservices over HTTP/gRPC
// (PredictiveUnitBean.java:170-183 -> InternalPredictionService.java:186-453)
// and joins their outputs for the combiner / returns the routed child's output.
// With one engine process per GPU, the front-end rank keeps the graph and the
// request queue; children placed on other ranks are reached per micro-batch:
//
//   rank 0 (front end)                        rank r (worker)
//   ------------------                        ---------------
//   header {op, model, rows, cols} --ctrl-->  blocking read of the header (host)
//   X [rows, cols] fp64 ---------data------>  posted recv X (stream-ordered)
//                                             model.launch(X) on the worker's GPU
//   Y [rows, out_cols] <--------data-------   posted send Y (stream-ordered)
//
// Two planes behind one Transport:
//  * control: a host socket per (rank 0, worker) pair carries the 16-byte
//    headers, so the worker learns the batch geometry without a device round
//    trip -- it posts the payload receive, the kernel and the reply send on its
//    stream back to back and never waits for the GPU between batches;
//  * data: RCCL point-to-point on the fabric stream (GPU memory to GPU memory
//    over xGMI) for GPU fabrics, or the same sockets for CPU fabrics (device -1:
//    multi-process tests and CPU serving run the identical state machines).
//
// A fan-out to K ranks (COMBINER over replicas on K GPUs) is one RCCL group:
// the K sends are the broadcast, the K receives the gather, and the combine
// kernel runs on rank 0's GPU.  All fabric operations of a rank are issued
// from one thread at a time in one order (a per-fabric mutex), so the sequence
// each worker observes is exactly header, payload, reply.
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

struct PeerHeader {
  int32_t op = 0, model = 0, rows = 0, cols = 0;
};
enum PeerOp : int32_t { kPeerStop = 0, kPeerRun = 1 };

class Fabric {
 public:
  // ctrl_fds[r] = connected socket to rank r (-1 for self / no link): rank 0
  // holds one per worker, a worker one to rank 0.  The fabric owns them.
  // device >= 0: RCCL data plane (unique_id from rccl_unique_id on rank 0);
  // device < 0: the sockets carry the data too (unique_id ignored).
  Fabric(int rank, int world, const std::string& unique_id, int device, std::vector<int> ctrl_fds);
  ~Fabric();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  bool gpu() const { return device_ >= 0; }
  ncclComm_t comm() const { return comm_; }
  hipStream_t stream() const { return stream_.get(); }
  std::mutex& issue_mutex() { return mu_; }
  bool open() const { return open_; }
  void close();

  // control plane (host, blocking)
  void send_header(int peer, const PeerHeader& h);
  PeerHeader recv_header(int peer);
  // data plane: GPU fabrics enqueue on stream(); CPU fabrics block
  void send(const void* p, size_t bytes, int peer);
  void recv(void* p, size_t bytes, int peer);
  void group_start();
  void group_end();

 private:
  int fd(int peer) const;
  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  gpu::Stream stream_;
  std::vector<int> fds_;
  std::mutex mu_;
  bool open_ = true;
};
using FabricPtr = std::shared_ptr<Fabric>;

// Front-end side: a row model whose computation happens on other ranks.
// `peers` = ranks holding a replica (model index `model_id` in each rank's
// PeerServer).  One peer: a remote MODEL node.  Several peers: COMBINER over
// replicas -- the batch is broadcast to every peer and the outputs gathered and
// averaged on this GPU (or host, for CPU fabrics).
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
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  uint64_t batches() const { return batches_.load(); }

 private:
  void headers(int rows, int cols) const;
  FabricPtr f_;
  std::vector<int> peers_;
  int model_id_, in_cols_, out_cols_;
  gpu::Event ev_in_, ev_done_;
  mutable std::atomic<uint64_t> batches_{0};
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
  uint64_t host_syncs() const { return host_syncs_.load(); }  // device waits (buffer growth only)
  std::string error() const;

 private:
  void loop();
  void loop_cpu();
  FabricPtr f_;
  std::vector<gpu::RowModelPtr> models_;
  std::thread th_;
  std::atomic<uint64_t> batches_{0}, rows_{0}, host_syncs_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

// Front end: tell every worker rank to leave its serve loop.
void stop_peers(Fabric& f);

}  // namespace sca::par
