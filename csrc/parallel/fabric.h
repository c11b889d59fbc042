// Cross-process graph edges (one engine process per MI355X).
//
// The reference fans a request out to child microservices over HTTP/gRPC
// (PredictiveUnitBean.java:170-183 -> InternalPredictionService.java:186-453)
// and joins their outputs for the combiner / returns the routed child's output.
// With one engine process per GPU, the front-end rank keeps the graph and the
// request queue; children placed on other ranks are reached per micro-batch:
//
//   rank 0 (front end)                          rank r (worker)
//   ------------------                          ---------------
//   header {seq, op, model, rows, cols} ------> header ring (shared memory,
//     into the worker's header ring,             sequence-number doorbell)
//     no syscall                                 polled by the worker thread
//   X [rows, cols] fp64 --- comm_x / stream_x -> recv into slot k = seq % K
//                                                model.launch(slot k) on the
//                                                compute stream
//   Y [rows, out_cols] <--- comm_y / stream_y -- send from slot k
//
// Pipelining: the worker owns K batch slots; slot k's receive, kernel and
// reply are chained with events across three streams, and a slot is reused
// only once its previous reply has left (device-side waits -- the worker
// thread never blocks on the GPU).  X travels on one RCCL communicator and Y
// on a second one, each on its own stream, so the receive of batch k+1
// overlaps the kernel and reply of batch k, and the front end's send of the
// next batch is not queued behind the receive of the previous reply.
//
// Two planes:
//  * control: a shared-memory ring per (rank 0, worker) pair carries the
//    headers (the ranks share one host); the socket pair made at rendezvous
//    carries only the ring's name and serves as a liveness check;
//  * data: RCCL point-to-point (GPU memory to GPU memory over xGMI) for GPU
//    fabrics, or the sockets for CPU fabrics (device -1: multi-process tests
//    and CPU serving run the same header ring; a receiver thread per peer
//    hands replies to concurrent callers in order, and the worker reads
//    batches ahead of its compute thread, so K batches are in flight too).
//
// A fan-out to K ranks (COMBINER over replicas on K GPUs) is one RCCL group
// per direction: the sends are the broadcast, the receives the gather, and the
// combine kernel runs on rank 0's GPU.  All issues of a rank happen under one
// mutex, so every worker sees headers and payloads in one order.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../gpu/hip_util.h"
#include "../gpu/models.h"

namespace sca::par {

// Two 128-byte RCCL ids (X and Y communicators); rank 0 creates, everyone
// receives them out of band.
std::string rccl_unique_id();

struct PeerHeader {
  int32_t op = 0, model = 0, rows = 0, cols = 0;
};
enum PeerOp : int32_t { kPeerStop = 0, kPeerRun = 1 };

// Single-producer (rank 0) / single-consumer (one worker) header ring in a
// shared mapping.  Slot i holds header seq when slots[i].seq == seq + 1.
struct HeaderRing {
  static constexpr uint32_t kSlots = 256;
  struct alignas(64) Slot {
    std::atomic<uint64_t> seq;
    PeerHeader h;
  };
  alignas(64) std::atomic<uint64_t> consumed;  // headers taken by the worker
  Slot slots[kSlots];
};

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
  hipStream_t stream_x() const { return sx_.get(); }
  hipStream_t stream_y() const { return sy_.get(); }
  std::mutex& issue_mutex() { return mu_; }
  bool open() const { return open_.load(); }
  void close();

  // control plane: rank 0 publishes, the worker takes (spin, then back off;
  // throws once the peer's socket is gone)
  void publish(int peer, const PeerHeader& h);
  PeerHeader take();
  // data plane: GPU fabrics enqueue on stream_x (X) / stream_y (Y); CPU
  // fabrics write / read the sockets
  void send_x(const void* p, size_t bytes, int peer);
  void recv_x(void* p, size_t bytes, int peer);
  void send_y(const void* p, size_t bytes, int peer);
  void recv_y(void* p, size_t bytes, int peer);
  void group_start();
  void group_end();

  // CPU fabrics, rank 0: queue a reply read (bytes into `dst`) on the peer's
  // receiver thread; replies arrive in issue order.
  struct Waiter {
    std::mutex mu;
    std::condition_variable cv;
    int pending = 0;
    std::string error;
  };
  void expect_reply(int peer, void* dst, size_t bytes, std::shared_ptr<Waiter> w);

 private:
  int fd(int peer) const;
  void map_rings();
  bool peer_gone(int peer) const;
  void receiver(int peer);
  int rank_, world_, device_;
  ncclComm_t comm_x_ = nullptr, comm_y_ = nullptr;
  gpu::Stream sx_, sy_;
  std::vector<int> fds_;
  std::vector<HeaderRing*> rings_;  // rank 0: one per worker; worker: rings_[0]
  std::vector<uint64_t> next_;      // rank 0: next seq per worker; worker: next_[0] to take
  std::mutex mu_;
  std::atomic<bool> open_{true};
  // CPU reply receivers (rank 0)
  struct Pending {
    void* dst;
    size_t bytes;
    std::shared_ptr<Waiter> w;
  };
  struct RecvQ {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Pending> q;
    std::thread th;
  };
  std::vector<std::unique_ptr<RecvQ>> rq_;
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
// a stop header.  K = SCA_FABRIC_SLOTS (default 4) batches in flight.
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
  uint64_t max_inflight() const { return max_inflight_.load(); }  // most batches received but not yet answered
  int slots() const { return slots_; }
  std::string error() const;

 private:
  void loop();
  void loop_cpu();
  void note_inflight(uint64_t n);
  FabricPtr f_;
  std::vector<gpu::RowModelPtr> models_;
  std::thread th_;
  int slots_ = 4;
  std::atomic<uint64_t> batches_{0}, rows_{0}, host_syncs_{0}, max_inflight_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

// Front end: tell every worker rank to leave its serve loop.
void stop_peers(Fabric& f);

}  // namespace sca::par
