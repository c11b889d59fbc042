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
//   X [rows, cols] fp64 --- link r, X chan ---> recv into slot k = seq % K
//                                                model.launch(slot k) on the
//                                                compute stream
//   Y [rows, out_cols] <--- link r, Y chan ---- send from slot k
//
// Links: rank 0 holds one link per worker, each with its own X and Y streams,
// its own pair of 2-rank RCCL communicators and its own issue mutex, so
// batches bound for different workers (the two arms of an A/B test, the
// branches of a bandit, the replicas of a combiner) are issued and move over
// xGMI concurrently; only batches on the same link are ordered.  xGMI is
// point-to-point (one link per GPU pair), so per-pair communicators map 1:1
// onto the hardware instead of funnelling every peer through one ring.
//
// Pipelining: the worker owns K batch slots; slot k's receive, kernel and
// reply are chained with events across three streams, and a slot is reused
// only once its previous reply has left (device-side waits -- the worker
// thread never blocks on the GPU).  X travels on one communicator and Y on a
// second one, each on its own stream, so the receive of batch k+1 overlaps
// the kernel and reply of batch k.
//
// Planes:
//  * control: a shared-memory ring per (rank 0, worker) pair carries the
//    headers (the ranks share one host); the socket pair made at rendezvous
//    carries only the ring's name and serves as a liveness check;
//  * data, one of three transports behind send/recv:
//    - RCCL point-to-point (GPU memory to GPU memory over xGMI), GPU fabrics;
//    - loopback: every rank of the fabric lives in ONE process on ONE GPU
//      (LoopbackHub).  This runs the GPU code paths of both sides -- the
//      worker's slot pipeline, the front end's per-link streams, the fan-out
//      gather + combine kernel -- on a single device, so they are tested on
//      a 1-GPU box.  Eager protocol: a send copies into a hub-owned staging
//      buffer on the sender's stream (the sender's buffer is reusable in
//      stream order, as after ncclSend); a receive waits on the host until
//      the matching send is posted, then copies out on the receiver's stream
//      after the send's event.  No GPU-side wait on work not yet enqueued, so
//      the transport cannot wedge a hardware queue;
//    CPU gangs and the default GPU transport ("shm" / "ipc") are the mesh
//    (mesh.h): direct stage-to-stage edges over shared memory and HIP IPC.
//    This star fabric stays as the RCCL transport ("rccl": an X and a Y
//    communicator per link; "rccl1": one communicator and one stream per link,
//    the conservative fallback) and its in-process loopback rehearsal.
//
// A fan-out to K ranks (COMBINER over replicas on K GPUs) sends the batch on
// every link (the broadcast), receives every reply into its own slab (the
// gather) and averages them on rank 0's GPU once every link's Y event fired.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../gpu/hip_util.h"
#include "../gpu/models.h"

namespace sca::par {

// per_link * (world - 1) 128-byte RCCL ids (the X and Y communicators of
// every rank-0 <-> worker link, link r at [2(r-1), 2(r-1)+1]; or one per link
// when per_link == 1); rank 0 creates them, everyone receives them out of band.
std::string rccl_unique_ids(int world, int per_link = 2);

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

// In-process transport between the Fabric objects of one process (see the
// file comment).  Channels are keyed (src rank, dst rank, chan); messages on a
// channel match in posting order, like RCCL p2p on one communicator.
class LoopbackHub {
 public:
  explicit LoopbackHub(int device);
  ~LoopbackHub();
  int device() const { return device_; }
  void send(int src, int dst, int chan, const void* p, size_t bytes, hipStream_t s);
  void recv(int src, int dst, int chan, void* p, size_t bytes, hipStream_t s);
  void close_rank(int rank);  // wakes that rank's blocked receives (they throw)
  uint64_t messages() const { return messages_.load(); }
  uint64_t staging_buffers() const;
  // Receives that found their send already posted (the other case waited on
  // the host): the split shows whether the two sides ran concurrently.
  uint64_t matched_immediately() const { return immediate_.load(); }

 private:
  struct Stage {
    gpu::DeviceBuffer buf;
    gpu::Event ready, freed;
    bool busy = false;
  };
  struct Msg {
    Stage* st;
    size_t bytes;
  };
  struct Chan {
    std::deque<Msg> q;
  };
  Stage* acquire(size_t bytes);
  int device_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::tuple<int, int, int>, Chan> chans_;
  std::vector<std::unique_ptr<Stage>> pool_;
  std::vector<int> closed_;
  std::atomic<uint64_t> messages_{0}, immediate_{0};
  int recv_timeout_ms_ = 30000;
};
using LoopbackHubPtr = std::shared_ptr<LoopbackHub>;

class Fabric {
 public:
  // ctrl_fds[r] = connected socket to rank r (-1 for self / no link): rank 0
  // holds one per worker, a worker one to rank 0.  The fabric owns them.
  // GPU data plane: RCCL (unique_ids from rccl_unique_ids on rank 0, with
  // comms_per_link 2 = separate X and Y communicators and streams, 1 = one of
  // each per link) or, with `hub`, the in-process loopback transport.
  Fabric(int rank, int world, const std::string& unique_ids, int device, std::vector<int> ctrl_fds,
         LoopbackHubPtr hub = nullptr, int comms_per_link = 2);
  ~Fabric();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  bool gpu() const { return true; }
  bool loopback() const { return hub_ != nullptr; }
  std::string transport() const { return hub_ ? "loopback" : (per_link_ == 1 ? "rccl1" : "rccl"); }
  // Per-link resources (peer = the other end: a worker rank on rank 0, 0 on
  // a worker).
  hipStream_t stream_x(int peer) const { return link(peer).sx.get(); }
  hipStream_t stream_y(int peer) const { return per_link_ == 1 ? link(peer).sx.get() : link(peer).sy.get(); }
  std::mutex& link_mutex(int peer) { return link(peer).mu; }
  bool open() const { return open_.load(); }
  void close();

  // control plane: rank 0 publishes, the worker takes (spin, then back off;
  // throws once the peer's socket is gone)
  void publish(int peer, const PeerHeader& h);
  PeerHeader take();
  // data plane: enqueued on the link's X / Y stream
  void send_x(const void* p, size_t bytes, int peer);
  void recv_x(void* p, size_t bytes, int peer);
  void send_y(const void* p, size_t bytes, int peer);
  void recv_y(void* p, size_t bytes, int peer);

 private:
  struct Link {
    gpu::Stream sx, sy;
    ncclComm_t cx = nullptr, cy = nullptr;
    std::mutex mu;
  };
  Link& link(int peer) const;
  int fd(int peer) const;
  void map_rings();
  bool peer_gone(int peer) const;
  void xfer(bool send, int chan, void* p, size_t bytes, int peer);
  int rank_, world_, device_;
  LoopbackHubPtr hub_;
  std::vector<std::unique_ptr<Link>> links_;  // indexed by peer rank (null where there is no link)
  std::vector<int> fds_;
  std::vector<HeaderRing*> rings_;  // rank 0: one per worker; worker: rings_[0]
  std::vector<uint64_t> next_;      // rank 0: next seq per worker; worker: next_[0] to take
  std::mutex close_mu_;
  std::atomic<bool> open_{true};
  int per_link_ = 2;
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
  // The loopback transport's receive blocks on the host until the matching
  // send: those units need a pump of their own.  RCCL enqueues never block.
  bool exclusive_driver() const override { return f_->loopback(); }
  void to_device(int device) override;
  size_t workspace_bytes(int max_rows, int cols) const override;
  void launch(const double* X, int rows, int cols, double* out, void* ws, hipStream_t s) override;
  void run_cpu(const double* X, int rows, int cols, double* out) const override;
  uint64_t batches() const { return batches_.load(); }

 private:
  void header(int peer, int rows, int cols) const;
  FabricPtr f_;
  std::vector<int> peers_;
  int model_id_, in_cols_, out_cols_;
  std::mutex mu_;  // launch() state (the events) -- one batcher device thread in practice
  gpu::Event ev_in_;
  std::vector<gpu::Event> ev_y_;  // per peer: reply landed
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
  void note_inflight(uint64_t n);
  FabricPtr f_;
  std::vector<gpu::RowModelPtr> models_;
  std::thread th_;
  int slots_ = 4;
  int delay_us_ = 0;       // test knob (SCA_FABRIC_WORKER_DELAY_US): a slow model (GPU: a delay kernel)
  int host_delay_us_ = 0;  // test knob (SCA_FABRIC_WORKER_HOST_DELAY_US, GPU loop): a slow worker thread
  std::atomic<uint64_t> batches_{0}, rows_{0}, host_syncs_{0}, max_inflight_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

// Front end: tell every worker rank to leave its serve loop.
void stop_peers(Fabric& f);

}  // namespace sca::par
