// Out-of-process predictive unit: the reference engine's internal
// microservice client (engine/.../service/InternalPredictionService.java:
// 78-453, grpc/GrpcChannelHandler.java:16-46) for graph nodes that run as a
// separate REST or gRPC microservice (e.g. a component started with
// `python -m seldon_core_amd.microservice`, or a remote proxy like SageMaker).
//
// REST: POST http://host:port/{predict|transform-input|transform-output|route|
// aggregate|send-feedback} with form body `json=<SeldonMessage>&isDefault=false`
// and Seldon-model-name/-image/-version headers; keep-alive connections per
// worker thread; retries on connect failure (seldon.io/rest-connect-retries);
// connect/read timeouts (seldon.io/rest-connection-timeout, rest-read-timeout).
// gRPC: unary calls on the node-type service (Model/Router/Transformer/
// OutputTransformer/Combiner, Generic for UNKNOWN_TYPE) over h2c (nghttp2).
// Calls run on a small worker pool so engine threads never block on sockets.
// ready(): TCP probe refreshed every 5 s (SeldonGraphReadyChecker.java:45-118).
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../core/engine.h"

namespace sca {

struct RemoteOptions {
  std::string host;
  int port = 0;
  bool grpc = false;
  std::string node_type = "MODEL";  // picks the gRPC service
  std::string model_name, model_image, model_version;
  int connect_timeout_ms = 200;
  int read_timeout_ms = 5000;
  int retries = 3;
  int threads = 8;
  size_t max_message = size_t(64) << 20;
};

class RemoteUnit : public Unit {
 public:
  explicit RemoteUnit(RemoteOptions o);
  ~RemoteUnit() override;
  std::string kind() const override { return std::string(opts_.grpc ? "grpc:" : "rest:") + opts_.host + ":" + std::to_string(opts_.port); }
  void predict(const CallCtx& c, MsgPtr in, Done k) override;
  void transform_input(const CallCtx& c, MsgPtr in, Done k) override;
  void transform_output(const CallCtx& c, MsgPtr in, Done k) override;
  void route(const CallCtx& c, MsgPtr in, Done k) override;
  void aggregate(const CallCtx& c, std::vector<MsgPtr> in, Done k) override;
  void send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) override;
  bool ready() const override;

  // Blocking single call (used by workers and tests): returns response body
  // (JSON for REST, protobuf for gRPC) or throws.
  std::string call_rest(const std::string& path, const std::string& json_body);
  std::string call_grpc(const std::string& method, const std::string& pb_body);

 private:
  void submit(std::function<void()> task);
  void call_message(const char* rest_path, const char* grpc_method, MsgPtr in, Done k);
  void probe_loop();

  RemoteOptions opts_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> tasks_;
  std::vector<std::thread> workers_;
  std::thread prober_;
  std::atomic<bool> running_{true};
  std::atomic<bool> reachable_{false};
};

}  // namespace sca
