// Mesh: the rank-placed graph data plane over shared memory and HIP IPC
// ("ipc" transport on GPU gangs, "shm" on CPU gangs).
//
// The reference reaches every graph node through its own pod: each hop is an
// HTTP/gRPC call from the engine (PredictiveUnitBean.java:128-138,170-192 ->
// InternalPredictionService.java:186-453), so a 3-stage pipeline costs three
// engine round trips.  Here a subtree placed on worker ranks is one PROGRAM:
// a small DAG of stages (a row model, a Python component, or an element-wise
// mean) with a rank each, agreed by every rank of the gang from the spec.
// Rank 0 writes the batch into the first stages' input slabs and rings a
// header doorbell on every rank of the program; each stage's output goes
// straight to the rank of the stage that consumes it, and only the program's
// output comes back to rank 0.  A pipeline r1 -> r2 -> r3 is 4 messages per
// batch (0->1, 1->2, 2->3, 3->0), not 6.
//
// Memory (consumer-owned slots; K = slots per program, seq = batch number):
//
//   rank c's REGION of program p: one shared-memory mapping created by c and
//   mapped (and, on GPU gangs, hipHostRegister'ed) by every rank of p:
//     header ring          rank 0 -> c: {seq, rows, cols}; doorbell = seq
//     flags, per slot k    ready[src] = seq (src's data for seq is in place),
//                          freed = seq (c has consumed its inputs of seq),
//                          err = seq (a stage failed; text beside it)
//     host slabs, per slot the program input X (written by rank 0's host),
//                          and every input of rank 0 (the program's output)
//   rank c's DEVICE SLAB allocation (GPU gangs): the inputs c receives from
//     stages on other workers; exported with hipIpcGetMemHandle, opened by
//     their producers, written with D2D copies (peer copies over xGMI when the
//     ranks sit on different GPUs).
//
// Ordering: a producer writes seq's data into the consumer's slot, then its
// ready flag (a host store, or hipStreamWriteValue64 behind the copy on the
// producer's stream).  Before it writes slot k for seq it waits until the
// consumer freed seq - K there.  Every cross-process wait is made by a HOST
// thread before it enqueues anything (tools/micro/ipc_probe: a stream waiting
// on another process could hold one of the process's 4 hardware queues that
// other streams share), so enqueued GPU work never waits on another process
// and a dead peer cannot wedge a queue.  A rank whose batch ends with exactly
// one remote write needs no freed flag of its own: that write's ready flag
// implies it.
//
// Threads: rank 0 has none -- ProgramModel::start_cpu / CpuCall::done run on
// the batcher's pump (one shared pump for every program unit).  A worker runs
// one thread per program it hosts stages of, with one stream each, so two
// programs on one rank overlap and cannot block each other.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../gpu/hip_util.h"
#include "../gpu/models.h"
#include "fabric.h"

namespace sca::par {

enum MeshStageKind : int { kMeshModel = 0, kMeshMean = 1, kMeshHost = 2 };

struct MeshStage {
  int rank = 0;
  int kind = kMeshModel;
  std::vector<int> inputs;  // stage indices (topological order); -1 = the program input
  int in_cols = 0, out_cols = 0;
  std::string node;
};

struct MeshProgram {
  int max_rows = 0;
  int in_cols = 0;                // width of the program input
  std::vector<MeshStage> stages;  // topological; the last one is the program output
};

// Host stage (a Python component): y[rows, out_cols] = f(x[rows, cols]).
using HostFn = std::function<void(const double* x, int rows, int cols, double* y, int out_cols)>;

struct MeshStats {
  uint64_t batches = 0, rows = 0, max_inflight = 0, host_waits = 0, stage_errors = 0;
};

class ProgramModel;

class Mesh : public std::enable_shared_from_this<Mesh> {
 public:
  // ctrl_fds: the gang's control sockets (rank 0: one per worker; a worker:
  // fds[0]) -- liveness only.  device < 0: CPU gang.
  Mesh(int rank, int world, int device, std::vector<int> ctrl_fds, int slots);
  ~Mesh();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  int slots() const { return K_; }
  bool gpu() const { return device_ >= 0; }
  std::string transport() const { return gpu() ? "ipc" : "shm"; }

  // Setup, identical order on every rank: add_program* -> set_* (own stages)
  // -> prepare() -> exchange blobs -> connect() -> barrier -> unlink() -> start().
  int add_program(MeshProgram p);
  void set_model(int prog, int stage, gpu::RowModelPtr m);
  void set_host_fn(int prog, int stage, HostFn f);
  std::string prepare();
  void connect(const std::vector<std::string>& blobs);
  void unlink();
  void start();  // worker threads
  void join();   // until every program thread left (stop header, close, error)
  // Rank 0: workers leave their loops; then the mesh closes.
  void stop_peers();
  void close();
  bool open() const { return open_.load(); }
  std::string error() const;
  MeshStats stats() const;
  // Messages one batch of `prog` moves between ranks (edges of its DAG).
  int messages_per_batch(int prog) const;

  // Peer readiness, before add_program (collective, same order everywhere):
  // probe_prepare() -> exchange blobs -> probe_connect() -> exchange the
  // rows -> set_peer_ok(matrix) -> barrier -> probe_finish().  Every GPU
  // worker exports a small fine-grained buffer; every worker opens every
  // other worker's buffer over HIP IPC, writes a canary into it with the
  // same device-to-device copy the programs use, reads it back with the
  // owner's pattern, and reports per rank: 1 ok, 0 failed, -1 not probed
  // (rank 0, CPU gangs).  SCA_MESH_FAULT=peer|canary injects a failure.
  // A worker -> worker edge whose probe failed gets a host-staged slab
  // ("ipc-host") instead of the consumer's HBM.
  std::string probe_prepare();
  std::vector<int> probe_connect(const std::vector<std::string>& blobs);
  std::string probe_error() const;
  void probe_finish();
  void set_peer_ok(const std::vector<std::vector<int>>& ok);  // [producer rank][consumer rank]
  // Per edge of `prog`: (producer stage, consumer rank, transport) with
  // transport "ipc" (consumer HBM over xGMI), "ipc-host" (host-staged after a
  // failed probe), "host" (rank 0 / program input slabs), "shm" (CPU gangs).
  std::vector<std::tuple<int, int, std::string>> edge_transports(int prog) const;

  // Rank 0: the front-end row model of a program (cpu_batching unit).
  gpu::RowModelPtr program_model(int prog, std::vector<std::string> class_names, bool flat);

  struct Impl;

 private:
  int rank_, world_, device_, K_;
  std::vector<int> fds_;
  std::atomic<bool> open_{true};
  std::unique_ptr<Impl> im_;
  friend class ProgramModel;
};
using MeshPtr = std::shared_ptr<Mesh>;

}  // namespace sca::par
