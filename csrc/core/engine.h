// In-process inference-graph executor.
//
// Semantics follow the reference engine's PredictiveUnitBean
// (engine/src/main/java/io/seldon/engine/predictors/PredictiveUnitBean.java:81-372):
// transform-input -> merge meta -> (leaf? return) -> route (-1 = all children)
// -> fan-out -> join -> aggregate -> merge meta -> transform-output -> merge
// meta, accumulating routing / requestPath / metrics for the final response
// meta, and feedback traversal along response.meta.routing.
//
// Unlike the reference (one HTTP hop + a thread hop per node, graph rebuilt
// from the spec on every request: PredictionService.java:113) the graph is
// compiled once and evaluated with continuations: a node bound to a GPU unit
// enqueues rows into that unit's micro-batcher and the request resumes on the
// batcher's completion thread, so no thread ever blocks on a device.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "message.h"
#include "metrics.h"
#include "spec.h"

namespace sca {

// ------------------------------------------------------------------ errors
// engine/src/main/java/io/seldon/engine/exception/APIException.java:28-38
enum class ApiError : int {
  INVALID_JSON,
  INVALID_ENDPOINT_URL,
  MICROSERVICE_ERROR,
  INVALID_ABTEST,
  INVALID_COMBINER_RESPONSE,
  INTERRUPTED,
  EXECUTION_FAILURE,
  INVALID_ROUTING,
  REQUEST_IO_EXCEPTION,
  // engine-native additions
  UNAVAILABLE,
  DEADLINE_EXCEEDED,
};

struct EngineError {
  int code = 206;
  std::string reason;
  std::string info;
  int http_status = 500;
  // Set by device units for failures of the device itself (launch / execution
  // error, hang, unhealthy replica), not of the request: a replica set may
  // re-run the request on another GPU.
  bool device_fault = false;
  // A component's own error reply (python/seldon_core/wrapper.py:22-31,
  // flask_utils.py:67-81): the JSON body its model_error_handler or
  // SeldonMicroserviceException.to_dict() produced, sent verbatim with
  // `http_status` (REST) or carried as the gRPC status message.
  std::string body;
};
using ErrPtr = std::shared_ptr<const EngineError>;

ErrPtr make_error(ApiError kind, std::string info);
// 203 MICROSERVICE_ERROR that answers with the component's status and body.
ErrPtr make_user_error(int http_status, std::string body, std::string info);
std::string error_to_json(const EngineError& e);

struct Outcome {
  MsgPtr msg;
  ErrPtr err;
  static Outcome ok(MsgPtr m) { return Outcome{std::move(m), nullptr}; }
  static Outcome fail(ErrPtr e) { return Outcome{nullptr, std::move(e)}; }
};
using Done = std::function<void(Outcome)>;
using FbDone = std::function<void(ErrPtr)>;

// --------------------------------------------------------------- node model
struct Node;

// Where a request's continuations should run: the front-end thread that
// owns its connection.  A unit that completes on a thread of its own (a GPU
// batcher's device thread) posts the rest of the request there, so graph
// walking, meta merging and serialisation spread over the front-end threads
// instead of piling onto the device thread.
class Executor {
 public:
  virtual ~Executor() = default;
  virtual void post(std::function<void()> fn) = 0;
};
using ExecPtr = std::shared_ptr<Executor>;

struct CallCtx {
  const Node* node;
  const std::string* puid;
  const ExecPtr* exec = nullptr;  // may be null: continue on the completing thread
};

// A unit implements a subset of the five predictive-unit methods.  Every
// method must invoke its continuation exactly once (on any thread).
class Unit {
 public:
  virtual ~Unit() = default;
  // For built-ins: the methods the implementation overrides (a built-in
  // implementation short-circuits the type table, PredictorConfigBean.java:84-107).
  // Return 0 to use the node's type/methods table.
  virtual uint32_t builtin_methods() const { return 0; }
  virtual void transform_input(const CallCtx& c, MsgPtr in, Done k) { (void)c; k(Outcome::ok(std::move(in))); }
  // MODEL nodes: the reference calls the component's /predict for a MODEL's
  // transform-input (InternalPredictionService.java:255-256).
  virtual void predict(const CallCtx& c, MsgPtr in, Done k) { transform_input(c, std::move(in), std::move(k)); }
  virtual void transform_output(const CallCtx& c, MsgPtr in, Done k) { (void)c; k(Outcome::ok(std::move(in))); }
  virtual void route(const CallCtx& c, MsgPtr in, Done k) { (void)c; (void)in; k(Outcome::ok(nullptr)); }
  virtual void aggregate(const CallCtx& c, std::vector<MsgPtr> in, Done k) { (void)c; k(Outcome::ok(in.empty() ? nullptr : in[0])); }
  virtual void send_feedback(const CallCtx& c, std::shared_ptr<const Feedback> fb, FbDone k) { (void)c; (void)fb; k(nullptr); }
  virtual bool ready() const { return true; }
  virtual std::string kind() const { return "unit"; }
  // Snapshot / restore of online state (routers, detectors); "" = stateless.
  virtual std::string snapshot() const { return ""; }
  virtual void restore(const std::string&) {}
  // Scrape-time export of unit-internal statistics (GPU batchers) into the
  // registry, labelled with the owning node's model labels.
  virtual void collect_metrics(MetricsRegistry& m, const Labels& labels) const { (void)m; (void)labels; }
};
using UnitPtr = std::shared_ptr<Unit>;

struct Node {
  const UnitSpec* spec = nullptr;
  std::string name;
  std::string image;
  uint32_t methods = 0;  // effective method mask
  bool builtin = false;
  bool is_model = false;  // MODEL type: transform-input is the component's predict
  std::vector<Node*> children;
  UnitPtr unit;
  Labels model_labels;    // deployment/predictor/model tags for metrics
  Series* client_timer[5] = {};
  Series* fb_reward = nullptr;
  Series* fb_count = nullptr;
  std::vector<Node*> fused;  // non-empty: this node evaluates the listed subtree (itself first)
  bool has(Method m) const { return methods & method_bit(m); }
};

struct EngineOptions {
  std::string deployment_name = "None";
  bool log_requests = false;
  bool log_responses = false;
  bool log_feedback = false;
  std::string message_logging_service;  // CloudEvents sink (SELDON_MESSAGE_LOGGING_SERVICE)
  bool log_messages_externally = false;  // SELDON_LOG_MESSAGES_EXTERNALLY
  std::string message_type = "seldon.message.pair";
  std::string deployment_name_env;       // DEPLOYMENT_NAME as set in the environment ("" = unset)
  std::string deployment_namespace;      // DEPLOYMENT_NAMESPACE
};

class MessageLogger;

// One finished span of the native tracer (E14; reference
// engine/.../tracing/TracingProvider.java:25-40 opens a Jaeger span per request
// and per microservice call).  Exported by the Python side as Zipkin v2 JSON.
struct TraceSpan {
  std::string trace_id;   // 32 hex
  std::string span_id;    // 16 hex
  std::string parent_id;  // "" for the request's root span
  std::string name;       // "predictions" or "<node>:<method>"
  std::string puid;
  int64_t start_us = 0, dur_us = 0;
  bool error = false;
};

class Engine {
 public:
  // `shared_metrics`: registry shared with sibling predictors (one /prometheus).
  Engine(PredictorSpecC spec, EngineOptions opts, std::shared_ptr<MetricsRegistry> shared_metrics = nullptr);
  ~Engine();

  const PredictorSpecC& spec() const { return spec_; }
  MetricsRegistry& metrics() { return metrics_; }
  // Prometheus text: unit collectors of this engine and its traffic peers /
  // shadows run first, then the (shared) registry renders.
  std::string render_metrics();
  std::shared_ptr<MetricsRegistry> metrics_ptr() const { return metrics_owner_; }

  // Split traffic between this predictor and sibling predictors by integer
  // weight (PredictorSpec.traffic; reference: Istio/Ambassador route weights,
  // seldondeployment_controller.go:180-215, ambassador.go:88) and mirror every
  // request to `shadows` (ambassador.go:119-122), discarding their responses.
  // `self_weight` is this predictor's own share.
  void set_traffic(int self_weight, std::vector<std::pair<std::shared_ptr<Engine>, int>> peers,
                   std::vector<std::shared_ptr<Engine>> shadows);
  // Header-match routing (reference ambassador `seldon.io/ambassador-header` /
  // `-regex-header`, operator/controllers/ambassador.go:99-118): a request
  // carrying header `name` whose value equals (or, regex, matches) `value` is
  // served by `target` regardless of the traffic weights.
  void add_header_route(const std::string& name, const std::string& value, bool regex, std::shared_ptr<Engine> target);
  bool has_header_routes() const { return !header_routes_.empty(); }
  bool is_route_header(std::string_view name) const;
  // predict() after header matching; `headers` = (name, value) pairs the front
  // end kept because is_route_header() was true for them.
  void predict_with_headers(MsgPtr request, Done k, ExecPtr exec,
                            const std::vector<std::pair<std::string, std::string>>& headers);
  // Graph evaluation on THIS predictor (no traffic split).
  void predict_local(MsgPtr request, Done k, ExecPtr exec = nullptr);
  void send_feedback_local(std::shared_ptr<Feedback> fb, FbDone k);
  const EngineOptions& options() const { return opts_; }

  // Bind an implementation to a node (before finalize()).
  void bind(const std::string& node, UnitPtr unit);
  // Bind `unit` to evaluate the whole subtree rooted at `root` in one call
  // (a device graph); `absorbed` are the subtree nodes it computes.  They keep
  // their place in the graph for meta (requestPath/routing) and feedback.
  void bind_fused(const std::string& root, UnitPtr unit, const std::vector<std::string>& absorbed);
  UnitPtr unit_of(const std::string& node) const;
  // Compile the graph. Throws std::runtime_error if a node is unbound.
  void finalize();
  bool finalized() const { return root_ != nullptr; }
  std::vector<std::string> node_names() const;
  const Node* node(const std::string& name) const;

  // Async API (thread-safe).  `exec`: the caller's executor (see Executor).
  void predict(MsgPtr request, Done k, ExecPtr exec = nullptr);
  void send_feedback(std::shared_ptr<Feedback> fb, FbDone k);
  // Reference "internal API" entry: call one node's method directly
  // (microservice mode: /predict, /route, ...).  `method` as in Method, or
  // kPredictMethod for /predict.
  static constexpr int kPredictMethod = 5;
  void call_node(const std::string& node, int method, std::vector<MsgPtr> in, Done k);

  bool ready() const;
  std::string new_puid();
  // Requests accepted by predict() and not yet answered (graceful drain).
  int64_t inflight() const { return inflight_.load(std::memory_order_acquire); }
  MessageLogger* message_logger() const { return msglog_.get(); }
  // Native tracing: sample `rate` of requests; spans are buffered (bounded)
  // until drain_spans().
  void enable_tracing(double rate) { trace_rate_ = rate; }
  std::vector<TraceSpan> drain_spans();

  // Hook invoked after each completed prediction (request, response) — used
  // by the async request logger.  Called on the completing thread.
  using PairHook = std::function<void(const SeldonMessage&, const SeldonMessage&)>;
  void set_pair_hook(PairHook h) { pair_hook_ = std::move(h); }

 private:
  struct ReqCtx;
  void eval(Node* n, MsgPtr input, std::shared_ptr<ReqCtx> ctx, Done k);
  void after_input(Node* n, MsgPtr input, MsgPtr ti, std::shared_ptr<ReqCtx> ctx, Done k);
  void fan_in(Node* n, std::vector<MsgPtr> outs, std::shared_ptr<ReqCtx> ctx, Done k);
  void dispatch_children(Node* n, std::shared_ptr<ReqCtx> ctx, Done k, MsgPtr ti, int routing);
  void after_aggregate(Node* n, MsgPtr agg_raw, const std::vector<const SeldonMessage*>& prev,
                       std::shared_ptr<ReqCtx> ctx, Done k);
  void feedback_node(Node* n, std::shared_ptr<const Feedback> fb, FbDone k);
  void add_metrics(Node* n, const SeldonMessage& m, ReqCtx* ctx);
  Node* compile(const UnitSpec& u);

  PredictorSpecC spec_;
  EngineOptions opts_;
  std::shared_ptr<MetricsRegistry> metrics_owner_;
  MetricsRegistry& metrics_;
  // Traffic split across predictors (ingress weights / shadow).
  std::vector<std::pair<Engine*, int>> routes_;
  int route_total_ = 0;
  std::vector<Engine*> shadows_;
  std::vector<std::shared_ptr<Engine>> peers_;
  struct HeaderRoute {
    std::string name_lc, value;
    bool regex = false;
    std::shared_ptr<void> re;  // std::regex, type-erased to keep <regex> out of the header
    Engine* target = nullptr;
  };
  std::vector<HeaderRoute> header_routes_;
  std::atomic<int64_t> inflight_{0};
  std::shared_ptr<MessageLogger> msglog_;
  double trace_rate_ = 0.0;
  std::mutex span_mu_;
  std::vector<TraceSpan> spans_;
  void push_span(TraceSpan s);
  Done traced(const std::shared_ptr<ReqCtx>& ctx, const Node* n, const char* what, Done k);
  std::unordered_map<std::string, UnitPtr> bound_;
  std::map<std::string, std::vector<std::string>> fused_;
  std::set<std::string> absorbed_;
  std::vector<std::unique_ptr<Node>> nodes_;
  Node* root_ = nullptr;
  Labels base_labels_;
  PairHook pair_hook_;
};

// Built-in implementations (engine/.../predictors/*Unit.java).
UnitPtr make_builtin_unit(UnitImpl impl, const UnitSpec& spec);

// Java's java.util.Random (48-bit LCG) so RANDOM_ABTEST reproduces the
// reference's branch sequence for a given seed (RandomABTestUnit.java:31-59).
class JavaRandom {
 public:
  explicit JavaRandom(int64_t seed) { set_seed(seed); }
  void set_seed(int64_t seed) { seed_ = (uint64_t(seed) ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
  int32_t next(int bits) {
    seed_ = (seed_ * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return int32_t(int64_t(seed_) >> (48 - bits));
  }
  float next_float() { return float(next(24)) / float(1 << 24); }
  uint64_t state() const { return seed_; }
  void set_state(uint64_t s) { seed_ = s; }

 private:
  uint64_t seed_;
};

// Dense branch index from a router response (PredictiveUnitBean.java:301-311).
bool branch_index(const SeldonMessage& m, int& out);

}  // namespace sca
