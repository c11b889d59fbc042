// Native HTTP/1.1 front end for the engine.
//
// External API (reference engine/.../api/rest/RestClientController.java:76-291):
//   POST /api/v0.1/predictions   application/json | multipart/form-data
//   POST /api/v0.1/feedback
//   GET  /ping /ready /live /pause /unpause /  and /prometheus
// Internal microservice API (reference python/seldon_core/wrapper.py:33-89):
//   /predict /transform-input /transform-output /route /aggregate
//   /send-feedback /seldon.json   (form `json=`, query `?json=` or JSON body)
//
// One epoll loop per worker thread, SO_REUSEPORT listeners (the kernel
// spreads connections across workers), keep-alive, zero-copy request parse.
// Engine continuations that complete on another thread (GPU batcher) hand the
// serialized response back to the owning worker through a lock-protected
// queue + eventfd.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../core/engine.h"

namespace sca {

struct HttpOptions {
  std::string host = "0.0.0.0";
  std::vector<int> ports = {8000};
  int threads = 4;
  size_t max_body = 256u << 20;
  // Node served by the internal API routes; "" = graph root.
  std::string microservice_node;
  // Serve the internal microservice routes (/predict, ...).
  bool internal_api = true;
  std::string openapi_json;  // body for /seldon.json
};

class HttpServer {
 public:
  HttpServer(std::shared_ptr<Engine> engine, HttpOptions opts);
  ~HttpServer();
  void start();
  void stop();
  std::vector<int> bound_ports() const { return bound_ports_; }
  bool paused() const { return paused_.load(); }
  void set_paused(bool p) { paused_.store(p); }
  uint64_t requests_served() const { return served_.load(); }

  struct Worker;

 private:
  std::shared_ptr<Engine> engine_;
  HttpOptions opts_;
  std::vector<std::shared_ptr<Worker>> workers_;
  std::vector<int> bound_ports_;
  std::atomic<bool> paused_{false};
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> served_{0};
  int spin_us_ = 0;  // SCA_HTTP_SPIN_US: poll epoll this long before blocking
  friend struct Worker;
};

// Shared helpers (also used by the gRPC front end / tests).
std::string url_decode(std::string_view s);
bool form_value(std::string_view body, std::string_view key, std::string& out);

}  // namespace sca
