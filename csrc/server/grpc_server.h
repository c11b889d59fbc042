// Native gRPC (HTTP/2, h2c) front end: seldon.protos.Seldon/{Predict,SendFeedback}
// for the external API (reference engine/.../grpc/SeldonService.java:44-79,
// SeldonGrpcServer.java:37-143) plus the per-node services Generic / Model /
// Router / Transformer / OutputTransformer / Combiner (reference
// python/seldon_core/wrapper.py:98-142, proto/prediction.proto:93-128) for
// microservice mode.
//
// HTTP/2 framing, HPACK and flow control come from libnghttp2 (session API,
// memory I/O); the socket layer is the same epoll-per-worker / SO_REUSEPORT
// design as the HTTP/1.1 server.  Payloads are decoded by the hand-written
// protobuf codec straight into the engine's message struct.
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "../core/engine.h"

namespace sca {

struct GrpcOptions {
  std::string host = "0.0.0.0";
  int port = 5001;
  int threads = 4;
  std::string microservice_node;  // node for per-node services ("" = root)
  size_t max_message = size_t(64) << 20;  // seldon.io/grpc-max-message-size
};

class GrpcServer {
 public:
  GrpcServer(std::shared_ptr<Engine> engine, GrpcOptions opts);
  ~GrpcServer();
  void start();
  void stop();
  int bound_port() const { return bound_port_; }
  uint64_t requests_served() const { return served_.load(); }

  struct Worker;

 private:
  std::shared_ptr<Engine> engine_;
  GrpcOptions opts_;
  std::vector<std::shared_ptr<Worker>> workers_;
  int bound_port_ = 0;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> served_{0};
  friend struct Worker;
};

}  // namespace sca
