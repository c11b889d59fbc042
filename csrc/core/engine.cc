#include "engine.h"

#include "roctx.h"

#include "msglog.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <regex>
#include <stdexcept>

namespace sca {

// ------------------------------------------------------------------ errors
ErrPtr make_error(ApiError kind, std::string info) {
  auto e = std::make_shared<EngineError>();
  e->info = std::move(info);
  e->http_status = 500;
  switch (kind) {
    case ApiError::INVALID_JSON: e->code = 201; e->reason = "Invalid JSON"; break;
    case ApiError::INVALID_ENDPOINT_URL: e->code = 202; e->reason = "Invalid Endpoint URL"; break;
    case ApiError::MICROSERVICE_ERROR: e->code = 203; e->reason = "Microservice error"; break;
    case ApiError::INVALID_ABTEST: e->code = 204; e->reason = "Error happened in AB Test Routing"; break;
    case ApiError::INVALID_COMBINER_RESPONSE: e->code = 204; e->reason = "Invalid number of predictions from combiner"; break;
    case ApiError::INTERRUPTED: e->code = 205; e->reason = "API call interrupted"; break;
    case ApiError::EXECUTION_FAILURE: e->code = 206; e->reason = "Execution failure"; break;
    case ApiError::INVALID_ROUTING: e->code = 207; e->reason = "Invalid Routing"; break;
    case ApiError::REQUEST_IO_EXCEPTION: e->code = 208; e->reason = "IO Exception"; break;
    case ApiError::UNAVAILABLE: e->code = 209; e->reason = "Service unavailable"; e->http_status = 503; break;
    case ApiError::DEADLINE_EXCEEDED: e->code = 210; e->reason = "Deadline exceeded"; e->http_status = 504; break;
  }
  return e;
}

ErrPtr make_user_error(int http_status, std::string body, std::string info) {
  auto e = std::make_shared<EngineError>(*make_error(ApiError::MICROSERVICE_ERROR, std::move(info)));
  e->http_status = (http_status >= 100 && http_status <= 599) ? http_status : 500;
  e->body = std::move(body);
  return e;
}

std::string error_to_json(const EngineError& e) {
  if (!e.body.empty()) return e.body;
  Status s;
  s.code = e.code;
  s.info = e.info;
  s.reason = e.reason;
  s.status = 1;
  std::string out;
  status_to_json(s, out);
  return out;
}

bool branch_index(const SeldonMessage& m, int& out) {
  if (m.payload != Payload::Data) return false;
  std::vector<int64_t> shape;
  std::vector<double> vals;
  if (!m.data.dense(shape, vals, nullptr) || vals.empty()) return false;
  out = int(vals[0]);
  return true;
}

// ------------------------------------------------------------- puid (130b)
namespace {

struct Xoshiro {
  uint64_t s[4];
  Xoshiro() {
    std::random_device rd;
    for (auto& x : s) x = (uint64_t(rd()) << 32) ^ rd() ^ 0x9E3779B97F4A7C15ULL;
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
};

const uint32_t kTI = method_bit(Method::TRANSFORM_INPUT), kTO = method_bit(Method::TRANSFORM_OUTPUT),
               kRO = method_bit(Method::ROUTE), kAG = method_bit(Method::AGGREGATE),
               kSF = method_bit(Method::SEND_FEEDBACK);

// PredictorConfigBean.java:45-72
uint32_t type_methods(UnitType t) {
  switch (t) {
    case UnitType::MODEL: return kTI | kSF;
    case UnitType::TRANSFORMER: return kTI;
    case UnitType::OUTPUT_TRANSFORMER: return kTO;
    case UnitType::ROUTER: return kRO | kSF;
    case UnitType::COMBINER: return kAG;
    default: return 0;
  }
}

const char* method_uri(Method m) {
  switch (m) {
    case Method::TRANSFORM_INPUT: return "/transform-input";
    case Method::TRANSFORM_OUTPUT: return "/transform-output";
    case Method::ROUTE: return "/route";
    case Method::AGGREGATE: return "/aggregate";
    case Method::SEND_FEEDBACK: return "/send-feedback";
  }
  return "/";
}

using Clock = std::chrono::steady_clock;

// Wrap a continuation so it fires at most once even if a unit misbehaves,
// time the call, and turn thrown exceptions into engine errors.
template <class F>
void guarded(Series* timer, Done k, F&& body) {
  struct Once {
    std::atomic<bool> fired{false};
    Done k;
    Series* timer;
    Clock::time_point t0;
  };
  auto st = std::make_shared<Once>();
  st->k = std::move(k);
  st->timer = timer;
  st->t0 = Clock::now();
  auto fire = [](const std::shared_ptr<Once>& o1, Outcome o) {
    if (o1->fired.exchange(true)) return;
    if (o1->timer) o1->timer->observe_seconds(std::chrono::duration<double>(Clock::now() - o1->t0).count());
    o1->k(std::move(o));
  };
  try {
    body(Done([st, fire](Outcome o) { fire(st, std::move(o)); }));  // handed over, not copied
  } catch (const std::exception& e) {
    fire(st, Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, e.what())));
  }
}

MsgPtr merge_meta(MsgPtr latest, const std::vector<const SeldonMessage*>& prev, const std::string& puid) {
  Json::Object tags;
  auto put = [&](const Json::Object& src) {
    for (const auto& kv : src) {
      bool done = false;
      for (auto& t : tags)
        if (t.first == kv.first) { t.second = kv.second; done = true; break; }
      if (!done) tags.push_back(kv);
    }
  };
  for (const auto* p : prev) put(p->meta.tags);
  put(latest->meta.tags);
  MsgPtr out = latest.use_count() == 1 ? std::move(latest) : std::make_shared<SeldonMessage>(*latest);
  out->has_meta = true;
  out->meta = Meta();
  out->meta.puid = puid;
  out->meta.tags = std::move(tags);
  return out;
}

}  // namespace

std::string Engine::new_puid() {
  thread_local Xoshiro rng;
  // 130 random bits in base 32, no leading zeros (the reference's
  // BigInteger(130, random).toString(32)): 5-bit groups straight from a
  // 128-bit word plus the top 2 bits
  const uint64_t hi = rng.next() & 3;
  const unsigned __int128 x = (static_cast<unsigned __int128>(rng.next()) << 64) | rng.next();
  static const char* digits = "0123456789abcdefghijklmnopqrstuv";
  char buf[26];
  buf[0] = digits[uint32_t((x >> 125) | (hi << 3)) & 31];  // bits 125..129
  for (int g = 24; g >= 0; --g) buf[25 - g] = digits[uint32_t(x >> (5 * g)) & 31];
  int lead = 0;
  while (lead < 25 && buf[lead] == '0') ++lead;
  return std::string(buf + lead, size_t(26 - lead));
}

// ------------------------------------------------------------------ engine
struct Engine::ReqCtx {
  std::string puid;
  ExecPtr exec;
  bool traced = false;
  std::string trace_id, root_span;
  int64_t t0_us = 0;
  std::mutex mu;
  std::vector<std::pair<std::string, int32_t>> routing;
  StrMap request_path;
  std::vector<std::pair<std::string, std::vector<Metric>>> metrics;
};

Engine::Engine(PredictorSpecC spec, EngineOptions opts, std::shared_ptr<MetricsRegistry> shared_metrics)
    : spec_(std::move(spec)),
      opts_(std::move(opts)),
      metrics_owner_(shared_metrics ? std::move(shared_metrics) : std::make_shared<MetricsRegistry>()),
      metrics_(*metrics_owner_) {
  std::string pname = spec_.name.empty() ? "unknown" : spec_.name;
  auto it = spec_.labels.find("version");
  std::string pver = (it == spec_.labels.end() || it->second.empty()) ? "unknown" : it->second;
  base_labels_ = {{"deployment_name", opts_.deployment_name}, {"predictor_name", pname}, {"predictor_version", pver}};
  MessageLogOptions lo;
  lo.log_requests = opts_.log_requests;
  lo.log_responses = opts_.log_responses;
  lo.log_feedback = opts_.log_feedback;
  lo.external = opts_.log_messages_externally && !opts_.message_logging_service.empty();
  lo.url = opts_.message_logging_service;
  lo.message_type = opts_.message_type;
  lo.deployment_name = opts_.deployment_name_env;
  lo.deployment_namespace = opts_.deployment_namespace;
  if (lo.log_requests || lo.log_responses || lo.log_feedback || lo.external) msglog_ = std::make_shared<MessageLogger>(lo);
}

Engine::~Engine() = default;

void Engine::bind(const std::string& node, UnitPtr unit) {
  if (root_) throw std::runtime_error("engine already finalized");
  bound_[node] = std::move(unit);
}

UnitPtr Engine::unit_of(const std::string& node) const {
  for (const auto& n : nodes_)
    if (n->name == node) return n->unit;
  auto it = bound_.find(node);
  return it == bound_.end() ? nullptr : it->second;
}

Node* Engine::compile(const UnitSpec& u) {
  auto n = std::make_unique<Node>();
  n->spec = &u;
  n->name = u.name;
  n->image = u.image;
  auto it = bound_.find(u.name);
  if (it != bound_.end()) {
    n->unit = it->second;
  } else {
    n->unit = make_builtin_unit(u.implementation, u);
    if (!n->unit && absorbed_.count(u.name)) n->unit = std::make_shared<Unit>();  // computed by a fused ancestor
    if (!n->unit)
      throw std::runtime_error("no implementation bound for graph node '" + u.name + "' (implementation " +
                               (u.implementation_name.empty() ? "UNKNOWN_IMPLEMENTATION" : u.implementation_name) + ")");
  }
  if (uint32_t b = n->unit->builtin_methods()) {
    n->methods = b;
    n->builtin = true;
  } else if (!u.has_type || u.type == UnitType::UNKNOWN_TYPE) {
    for (Method m : u.methods) n->methods |= method_bit(m);
  } else {
    n->methods = type_methods(u.type);
  }
  n->is_model = u.has_type && u.type == UnitType::MODEL;
  n->model_labels = base_labels_;
  n->model_labels.push_back({"model_name", u.name.empty() ? "unknown" : u.name});
  n->model_labels.push_back({"model_image", u.image_name.empty() ? "unknown" : u.image_name});
  n->model_labels.push_back({"model_version", u.image_version.empty() ? "latest" : u.image_version});
  for (int m = 0; m < 5; ++m) {
    if (!(n->methods & (1u << m))) continue;
    Labels l = n->model_labels;
    l.push_back({"method", "POST"});
    l.push_back({"uri", (Method(m) == Method::TRANSFORM_INPUT && (u.type == UnitType::MODEL)) ? "/predict" : method_uri(Method(m))});
    n->client_timer[m] = metrics_.timer("seldon_api_engine_client_requests", std::move(l), true);
  }
  n->fb_reward = metrics_.counter("seldon_api_model_feedback_reward", n->model_labels);
  n->fb_count = metrics_.counter("seldon_api_model_feedback", n->model_labels);
  Node* raw = n.get();
  nodes_.push_back(std::move(n));
  for (const auto& c : u.children) raw->children.push_back(compile(c));
  return raw;
}

void Engine::finalize() {
  if (root_) return;
  root_ = compile(spec_.graph);
  for (const auto& f : fused_) {
    Node* r = nullptr;
    for (const auto& n : nodes_)
      if (n->name == f.first) r = n.get();
    if (!r) throw std::runtime_error("fused root '" + f.first + "' is not a graph node");
    // Pre-order walk of the subtree; every absorbed node must be inside it.
    std::vector<Node*> stack{r};
    std::set<std::string> want(f.second.begin(), f.second.end());
    while (!stack.empty()) {
      Node* v = stack.back();
      stack.pop_back();
      r->fused.push_back(v);
      want.erase(v->name);
      for (auto it = v->children.rbegin(); it != v->children.rend(); ++it) stack.push_back(*it);
    }
    if (!want.empty()) throw std::runtime_error("fused node '" + *want.begin() + "' is not below '" + f.first + "'");
  }
}

void Engine::bind_fused(const std::string& root, UnitPtr unit, const std::vector<std::string>& absorbed) {
  if (root_) throw std::runtime_error("engine already finalized");
  bound_[root] = std::move(unit);
  fused_[root] = absorbed;
  for (const auto& a : absorbed) absorbed_.insert(a);
}

std::vector<std::string> Engine::node_names() const {
  std::vector<std::string> v;
  for (const auto& n : nodes_) v.push_back(n->name);
  return v;
}

const Node* Engine::node(const std::string& name) const {
  for (const auto& n : nodes_)
    if (n->name == name) return n.get();
  return nullptr;
}

bool Engine::ready() const {
  if (!root_) return false;
  for (const auto& p : peers_)
    if (!p->ready()) return false;
  for (const auto& n : nodes_)
    if (!n->unit->ready()) return false;
  return true;
}

void Engine::add_metrics(Node* n, const SeldonMessage& m, ReqCtx* ctx) {
  if (!m.has_meta || m.meta.metrics.empty()) return;
  for (const auto& mt : m.meta.metrics) {
    Labels l = n->model_labels;
    for (const auto& t : mt.tags) l.push_back(t);
    switch (mt.type) {
      case MetricType::COUNTER: metrics_.counter(mt.key, std::move(l))->inc(mt.value); break;
      case MetricType::GAUGE: metrics_.gauge(mt.key, std::move(l))->set(mt.value); break;
      case MetricType::TIMER: metrics_.timer(mt.key, std::move(l))->observe_seconds(double(mt.value) / 1000.0); break;
    }
  }
  if (!ctx) return;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& e : ctx->metrics)
    if (e.first == n->name) {
      e.second.insert(e.second.end(), m.meta.metrics.begin(), m.meta.metrics.end());
      return;
    }
  ctx->metrics.emplace_back(n->name, m.meta.metrics);
}

// ------------------------------------------------------------------ tracing
namespace {
int64_t wall_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
std::string rand_hex(int bytes) {
  thread_local Xoshiro rng;
  static const char* hx = "0123456789abcdef";
  std::string s;
  s.reserve(size_t(bytes) * 2);
  uint64_t v = 0;
  for (int i = 0; i < bytes * 2; ++i) {
    if (i % 16 == 0) v = rng.next();
    s.push_back(hx[v & 15]);
    v >>= 4;
  }
  return s;
}
}  // namespace

void Engine::push_span(TraceSpan s) {
  std::lock_guard<std::mutex> g(span_mu_);
  if (spans_.size() >= 200000) spans_.erase(spans_.begin(), spans_.begin() + 100000);  // exporter stalled: keep recent
  spans_.push_back(std::move(s));
}

std::vector<TraceSpan> Engine::drain_spans() {
  std::vector<TraceSpan> out;
  std::lock_guard<std::mutex> g(span_mu_);
  out.swap(spans_);
  return out;
}

Done Engine::traced(const std::shared_ptr<ReqCtx>& ctx, const Node* n, const char* what, Done k) {
  if (trace::roctx_on()) {  // marker range around the node call, closed on whichever thread finishes it
    const uint64_t id = trace::range_start((n->name + ":" + what).c_str());
    k = [id, k = std::move(k)](Outcome o) {
      trace::range_stop(id);
      k(std::move(o));
    };
  }
  if (!ctx->traced) return k;
  const int64_t t0 = wall_us();
  std::string name = n->name + ":" + what;
  return [this, ctx, t0, name = std::move(name), k = std::move(k)](Outcome o) {
    TraceSpan s;
    s.trace_id = ctx->trace_id;
    s.span_id = rand_hex(8);
    s.parent_id = ctx->root_span;
    s.name = name;
    s.puid = ctx->puid;
    s.start_us = t0;
    s.dur_us = wall_us() - t0;
    s.error = bool(o.err);
    push_span(std::move(s));
    k(std::move(o));
  };
}

// ------------------------------------------------------------ traffic split
void Engine::set_traffic(int self_weight, std::vector<std::pair<std::shared_ptr<Engine>, int>> peers,
                         std::vector<std::shared_ptr<Engine>> shadows) {
  routes_.clear();
  shadows_.clear();
  peers_.clear();
  route_total_ = 0;
  if (self_weight > 0) { routes_.emplace_back(this, self_weight); route_total_ += self_weight; }
  for (auto& p : peers) {
    if (p.second > 0) { routes_.emplace_back(p.first.get(), p.second); route_total_ += p.second; }
    peers_.push_back(std::move(p.first));
  }
  for (auto& s : shadows) {
    shadows_.push_back(s.get());
    peers_.push_back(std::move(s));
  }
  if (route_total_ <= 0) throw std::runtime_error("traffic weights must sum to a positive value");
}

void Engine::add_header_route(const std::string& name, const std::string& value, bool regex,
                              std::shared_ptr<Engine> target) {
  HeaderRoute r;
  r.name_lc = name;
  for (auto& ch : r.name_lc) ch = char(std::tolower(static_cast<unsigned char>(ch)));
  r.value = value;
  r.regex = regex;
  if (regex) r.re = std::make_shared<std::regex>(value);
  r.target = target.get();
  peers_.push_back(std::move(target));
  header_routes_.push_back(std::move(r));
}

bool Engine::is_route_header(std::string_view name) const {
  for (const auto& r : header_routes_) {
    if (r.name_lc.size() != name.size()) continue;
    bool eq = true;
    for (size_t i = 0; i < name.size() && eq; ++i)
      eq = r.name_lc[i] == char(std::tolower(static_cast<unsigned char>(name[i])));
    if (eq) return true;
  }
  return false;
}

void Engine::predict_with_headers(MsgPtr req, Done k, ExecPtr exec,
                                  const std::vector<std::pair<std::string, std::string>>& headers) {
  for (const auto& r : header_routes_)
    for (const auto& h : headers) {
      std::string n = h.first;
      for (auto& ch : n) ch = char(std::tolower(static_cast<unsigned char>(ch)));
      if (n != r.name_lc) continue;
      const bool hit = r.regex ? std::regex_match(h.second, *std::static_pointer_cast<std::regex>(r.re))
                               : h.second == r.value;
      if (!hit) continue;
      inflight_.fetch_add(1, std::memory_order_relaxed);
      r.target->predict_local(std::move(req), [this, k = std::move(k)](Outcome o) {
        k(std::move(o));
        inflight_.fetch_sub(1, std::memory_order_release);
      }, std::move(exec));
      return;
    }
  predict(std::move(req), std::move(k), std::move(exec));
}

namespace {
uint32_t traffic_draw(int total) {
  thread_local uint64_t x = 0x9E3779B97F4A7C15ULL ^ uint64_t(reinterpret_cast<uintptr_t>(&x));
  x ^= x << 13;
  x ^= x >> 7;
  x ^= x << 17;
  return uint32_t((x >> 11) % uint64_t(total));
}
}  // namespace

void Engine::predict(MsgPtr req, Done k, ExecPtr exec) {
  inflight_.fetch_add(1, std::memory_order_relaxed);
  k = [this, k = std::move(k)](Outcome o) {
    k(std::move(o));
    inflight_.fetch_sub(1, std::memory_order_release);
  };
  if (routes_.empty() && shadows_.empty()) {
    predict_local(std::move(req), std::move(k), std::move(exec));
    return;
  }
  for (Engine* s : shadows_) s->predict_local(std::make_shared<SeldonMessage>(*req), [](Outcome) {});
  Engine* target = this;
  if (routes_.size() > 1) {
    int r = int(traffic_draw(route_total_));
    for (const auto& rt : routes_) {
      if (r < rt.second) { target = rt.first; break; }
      r -= rt.second;
    }
  } else if (!routes_.empty()) {
    target = routes_[0].first;
  }
  target->predict_local(std::move(req), std::move(k), std::move(exec));
}

void Engine::predict_local(MsgPtr req, Done k, ExecPtr exec) {
  if (!root_) {
    k(Outcome::fail(make_error(ApiError::UNAVAILABLE, "graph not finalized")));
    return;
  }
  if (!req->has_meta) {
    req->has_meta = true;
    req->meta.puid = new_puid();
  } else if (req->meta.puid.empty()) {
    req->meta.puid = new_puid();
  }
  auto ctx = std::make_shared<ReqCtx>();
  ctx->puid = req->meta.puid;
  ctx->exec = std::move(exec);
  if (trace_rate_ > 0.0) {
    thread_local Xoshiro rng;
    if (trace_rate_ >= 1.0 || double(rng.next() >> 11) * (1.0 / 9007199254740992.0) < trace_rate_) {
      ctx->traced = true;
      ctx->trace_id = rand_hex(16);
      ctx->root_span = rand_hex(8);
      ctx->t0_us = wall_us();
    }
  }
  const uint64_t roctx_id = trace::roctx_on() ? trace::range_start("predictions") : 0;
  const bool log_pair = msglog_ && msglog_->wants_pairs();
  MsgPtr request_copy = (pair_hook_ || log_pair ? req : nullptr);
  const auto t_req = log_pair ? std::chrono::system_clock::now() : std::chrono::system_clock::time_point();
  eval(root_, req, ctx, [this, ctx, k = std::move(k), request_copy, t_req, log_pair, roctx_id](Outcome o) {
    if (roctx_id) trace::range_stop(roctx_id);
    if (ctx->traced) {
      TraceSpan s;
      s.trace_id = ctx->trace_id;
      s.span_id = ctx->root_span;
      s.name = "predictions";
      s.puid = ctx->puid;
      s.start_us = ctx->t0_us;
      s.dur_us = wall_us() - ctx->t0_us;
      s.error = bool(o.err);
      push_span(std::move(s));
    }
    if (o.err) { k(std::move(o)); return; }
    MsgPtr r = o.msg.use_count() == 1 ? std::move(o.msg) : std::make_shared<SeldonMessage>(*o.msg);
    {
      std::lock_guard<std::mutex> g(ctx->mu);
      r->has_meta = true;
      for (auto& kv : ctx->routing) r->meta.put_routing(kv.first, kv.second);
      for (auto& kv : ctx->request_path) r->meta.put_request_path(kv.first, kv.second);
      for (auto& e : ctx->metrics) r->meta.metrics.insert(r->meta.metrics.end(), e.second.begin(), e.second.end());
    }
    r->meta.puid = ctx->puid;
    if (pair_hook_ && request_copy) pair_hook_(*request_copy, *r);
    if (log_pair) msglog_->pair(request_copy, r, t_req);
    k(Outcome::ok(std::move(r)));
  });
}

void Engine::eval(Node* n, MsgPtr input, std::shared_ptr<ReqCtx> ctx, Done k) {
  auto visit = [&ctx](const Node* v) {
    bool found = false;
    for (auto& kv : ctx->request_path)
      if (kv.first == v->name) { kv.second = v->image; found = true; break; }
    if (!found) ctx->request_path.emplace_back(v->name, v->image);
  };
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    visit(n);
    // A fused device graph evaluates its whole subtree in one unit call; record
    // the per-node meta the unfused walk would have produced.
    for (const Node* f : n->fused) {
      if (f != n) visit(f);
      if (!f->children.empty()) ctx->routing.emplace_back(f->name, -1);
    }
  }
  if (!n->fused.empty()) {
    CallCtx cc{n, &ctx->puid, &ctx->exec};
    guarded(n->client_timer[int(Method::TRANSFORM_INPUT)],
            traced(ctx, n, "device-graph", [this, n, input, ctx, k = std::move(k)](Outcome o) mutable {
              if (o.err) { k(std::move(o)); return; }
              if (!o.msg) { k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "empty response from " + n->name))); return; }
              add_metrics(n, *o.msg, ctx.get());
              k(Outcome::ok(merge_meta(std::move(o.msg), {input.get()}, ctx->puid)));
            }),
            [&](Done kk) { n->unit->transform_input(cc, input, std::move(kk)); });
    return;
  }
  if (!n->has(Method::TRANSFORM_INPUT)) {
    after_input(n, input, input, std::move(ctx), std::move(k));
    return;
  }
  CallCtx cc{n, &ctx->puid, &ctx->exec};
  guarded(n->client_timer[int(Method::TRANSFORM_INPUT)],
          traced(ctx, n, n->is_model ? "predict" : "transform-input",
                 [this, n, input, ctx, k = std::move(k)](Outcome o) mutable {
            if (o.err) { k(std::move(o)); return; }
            if (!o.msg) { k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "empty response from " + n->name))); return; }
            after_input(n, std::move(input), std::move(o.msg), std::move(ctx), std::move(k));
          }),
          [&](Done kk) {
            if (n->is_model) n->unit->predict(cc, input, std::move(kk));
            else n->unit->transform_input(cc, input, std::move(kk));
          });
}

void Engine::after_input(Node* n, MsgPtr input, MsgPtr ti, std::shared_ptr<ReqCtx> ctx, Done k) {
  add_metrics(n, *ti, ctx.get());
  const SeldonMessage* in_raw = input.get();
  MsgPtr keep_in = std::move(input);
  // a node without transform-input passes its input through: then `ti` IS the
  // input and the extra reference would force merge_meta to copy the message
  // (merge_meta reads every tag before it rewrites the meta)
  if (keep_in.get() == ti.get()) keep_in.reset();
  ti = merge_meta(std::move(ti), {in_raw}, ctx->puid);
  keep_in.reset();
  if (n->children.empty()) {
    k(Outcome::ok(std::move(ti)));
    return;
  }
  if (!n->has(Method::ROUTE)) {
    dispatch_children(n, std::move(ctx), std::move(k), std::move(ti), -1);
    return;
  }
  CallCtx cc{n, &ctx->puid, &ctx->exec};
  MsgPtr ti_keep = ti;
  guarded(n->client_timer[int(Method::ROUTE)],
          traced(ctx, n, "route", [this, n, ctx, ti_keep, k = std::move(k)](Outcome o) mutable {
            if (o.err) { k(std::move(o)); return; }
            int routing = -1;
            if (o.msg) {
              if (!branch_index(*o.msg, routing)) {
                k(Outcome::fail(make_error(ApiError::INVALID_ROUTING, "Router that caused the exception: id=" + n->name + " name=" + n->name)));
                return;
              }
              if (routing < -1 || routing >= int(n->children.size())) {
                k(Outcome::fail(make_error(ApiError::INVALID_ROUTING,
                                           "Invalid branch index. Router that caused the exception: id=" + n->name + " name=" + n->name)));
                return;
              }
              add_metrics(n, *o.msg, ctx.get());
            }
            dispatch_children(n, ctx, std::move(k), std::move(ti_keep), routing);
          }),
          [&](Done kk) { n->unit->route(cc, ti, std::move(kk)); });
}

void Engine::dispatch_children(Node* n, std::shared_ptr<ReqCtx> ctx, Done k, MsgPtr ti2, int routing) {
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    bool found = false;
    for (auto& kv : ctx->routing)
      if (kv.first == n->name) { kv.second = routing; found = true; break; }
    if (!found) ctx->routing.emplace_back(n->name, routing);
  }
  std::vector<Node*> selected;
  if (routing == -1) selected = n->children;
  else selected.push_back(n->children[size_t(routing)]);
  struct Fan {
    std::vector<MsgPtr> outs;
    std::atomic<int> remaining;
    std::atomic<bool> failed{false};
  };
  auto fan = std::make_shared<Fan>();
  fan->outs.resize(selected.size());
  fan->remaining.store(int(selected.size()));
  for (size_t i = 0; i < selected.size(); ++i) {
    eval(selected[i], ti2, ctx, [this, n, ctx, k, fan, i](Outcome o) {
      if (o.err) {
        if (!fan->failed.exchange(true)) k(std::move(o));
        return;
      }
      fan->outs[i] = std::move(o.msg);
      if (fan->remaining.fetch_sub(1, std::memory_order_acq_rel) == 1 && !fan->failed.load())
        fan_in(n, std::move(fan->outs), ctx, k);
    });
  }
}

void Engine::fan_in(Node* n, std::vector<MsgPtr> outs, std::shared_ptr<ReqCtx> ctx, Done k) {
  std::vector<const SeldonMessage*> prev;
  prev.reserve(outs.size());
  for (const auto& m : outs) prev.push_back(m.get());
  if (!n->has(Method::AGGREGATE)) {
    // identity aggregate: hand the first child's reply over without another
    // reference so merge_meta rewrites it in place (prev[0] stays valid: the
    // message lives on in `first`)
    MsgPtr first = std::move(outs[0]);
    after_aggregate(n, std::move(first), prev, std::move(ctx), std::move(k));
    return;
  }
  CallCtx cc{n, &ctx->puid, &ctx->exec};
  auto held = std::make_shared<std::vector<MsgPtr>>(std::move(outs));
  guarded(n->client_timer[int(Method::AGGREGATE)],
          traced(ctx, n, "aggregate", [this, n, ctx, k, held, prev = std::move(prev)](Outcome o) mutable {
            if (o.err) { k(std::move(o)); return; }
            if (!o.msg) { k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "empty aggregate from " + n->name))); return; }
            after_aggregate(n, std::move(o.msg), prev, std::move(ctx), std::move(k));
          }),
          [&](Done kk) { n->unit->aggregate(cc, *held, std::move(kk)); });
}

void Engine::after_aggregate(Node* n, MsgPtr agg_raw, const std::vector<const SeldonMessage*>& prev,
                             std::shared_ptr<ReqCtx> ctx, Done k) {
  add_metrics(n, *agg_raw, ctx.get());
  MsgPtr agg = merge_meta(std::move(agg_raw), prev, ctx->puid);
  if (!n->has(Method::TRANSFORM_OUTPUT)) {  // identity transform: meta already merged
    k(Outcome::ok(std::move(agg)));
    return;
  }
  CallCtx cc{n, &ctx->puid, &ctx->exec};
  guarded(n->client_timer[int(Method::TRANSFORM_OUTPUT)],
          traced(ctx, n, "transform-output", [this, n, ctx, k = std::move(k), agg](Outcome o2) mutable {
            if (o2.err) { k(std::move(o2)); return; }
            if (!o2.msg) { k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, "empty response from " + n->name))); return; }
            add_metrics(n, *o2.msg, ctx.get());
            k(Outcome::ok(merge_meta(std::move(o2.msg), {agg.get()}, ctx->puid)));
          }),
          [&](Done kk) { n->unit->transform_output(cc, agg, std::move(kk)); });
}

// ----------------------------------------------------------------- feedback
void Engine::send_feedback(std::shared_ptr<Feedback> fb, FbDone k) {
  // The reference routes /feedback through the same weighted ingress mapping.
  if (routes_.size() > 1) {
    // Sticky when the response identifies its predictor: a node (name and
    // image) in meta.requestPath that only one predictor has.
    Engine* owner = nullptr;
    for (const auto& kv : fb->response.meta.request_path) {
      Engine* only = nullptr;
      int hits = 0;
      for (const auto& rt : routes_) {
        const Node* nd = rt.first->node(kv.first);
        if (nd && nd->image == kv.second) { only = rt.first; ++hits; }
      }
      if (hits == 1) { owner = only; break; }
    }
    if (!owner) {
      int r = int(traffic_draw(route_total_));
      for (const auto& rt : routes_) {
        if (r < rt.second) { owner = rt.first; break; }
        r -= rt.second;
      }
    }
    if (owner) {
      owner->send_feedback_local(std::move(fb), std::move(k));
      return;
    }
  }
  send_feedback_local(std::move(fb), std::move(k));
}

void Engine::send_feedback_local(std::shared_ptr<Feedback> fb, FbDone k) {
  if (!root_) {
    k(make_error(ApiError::UNAVAILABLE, "graph not finalized"));
    return;
  }
  if (msglog_ && msglog_->wants_feedback()) msglog_->feedback(fb);
  feedback_node(root_, std::move(fb), std::move(k));
}

void Engine::feedback_node(Node* n, std::shared_ptr<const Feedback> fb, FbDone k) {
  int32_t routing = -1;
  fb->response.meta.routing_of(n->name, routing);
  std::vector<Node*> children;
  if (routing == -1) children = n->children;
  else if (routing >= 0) {
    if (size_t(routing) >= n->children.size()) {
      k(make_error(ApiError::INVALID_ROUTING, "Invalid feedback routing " + std::to_string(routing) + " for node " + n->name));
      return;
    }
    children.push_back(n->children[size_t(routing)]);
  }
  struct Join {
    std::atomic<int> remaining;
    std::mutex mu;
    ErrPtr err;
  };
  auto join = std::make_shared<Join>();
  join->remaining.store(int(children.size()) + 1);
  auto arrive = [this, n, fb, join, k](ErrPtr e) {
    if (e) {
      std::lock_guard<std::mutex> g(join->mu);
      if (!join->err) join->err = e;
    }
    if (join->remaining.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    if (!join->err) {  // PredictiveUnitBean.java:313-316
      n->fb_reward->inc(double(fb->reward));
      n->fb_count->inc(1.0);
    }
    k(join->err);
  };
  for (Node* c : children) feedback_node(c, fb, arrive);
  if (!n->has(Method::SEND_FEEDBACK)) {
    arrive(nullptr);
    return;
  }
  CallCtx cc{n, &fb->response.meta.puid};
  Series* timer = n->client_timer[int(Method::SEND_FEEDBACK)];
  auto t0 = Clock::now();
  auto once = std::make_shared<std::atomic<bool>>(false);
  FbDone kk = [arrive, once, timer, t0](ErrPtr e) {
    if (once->exchange(true)) return;
    if (timer) timer->observe_seconds(std::chrono::duration<double>(Clock::now() - t0).count());
    arrive(std::move(e));
  };
  try {
    n->unit->send_feedback(cc, fb, kk);
  } catch (const std::exception& e) {
    kk(make_error(ApiError::MICROSERVICE_ERROR, e.what()));
  }
}

// ---------------------------------------------------------- direct node call
void Engine::call_node(const std::string& name, int method, std::vector<MsgPtr> in, Done k) {
  Node* n = nullptr;
  for (auto& x : nodes_)
    if (x->name == name) { n = x.get(); break; }
  if (!n) {
    k(Outcome::fail(make_error(ApiError::EXECUTION_FAILURE, "unknown node " + name)));
    return;
  }
  if ((method != kPredictMethod && method != int(Method::SEND_FEEDBACK) && in.empty()) ||
      (method == kPredictMethod && in.empty())) {
    k(Outcome::fail(make_error(ApiError::INVALID_JSON, "missing request")));
    return;
  }
  static const std::string empty;
  CallCtx cc{n, in.empty() ? &empty : &in[0]->meta.puid};
  const Method m = method == kPredictMethod ? Method::TRANSFORM_INPUT : Method(method);
  guarded(n->client_timer[int(m)], std::move(k), [&](Done kk) {
    if (method == kPredictMethod) {
      n->unit->predict(cc, in.at(0), std::move(kk));
      return;
    }
    switch (m) {
      case Method::TRANSFORM_INPUT: n->unit->transform_input(cc, in.at(0), std::move(kk)); break;
      case Method::TRANSFORM_OUTPUT: n->unit->transform_output(cc, in.at(0), std::move(kk)); break;
      case Method::ROUTE: n->unit->route(cc, in.at(0), std::move(kk)); break;
      case Method::AGGREGATE: n->unit->aggregate(cc, std::move(in), std::move(kk)); break;
      case Method::SEND_FEEDBACK: kk(Outcome::fail(make_error(ApiError::EXECUTION_FAILURE, "use send_feedback"))); break;
    }
  });
}

std::string Engine::render_metrics() {
  std::vector<const Engine*> engines{this};
  for (auto& [e, w] : routes_) {
    (void)w;
    if (e != this) engines.push_back(e);
  }
  for (Engine* e : shadows_) engines.push_back(e);
  std::vector<const Unit*> seen;
  for (const Engine* e : engines) {
    for (const auto& n : e->nodes_) {
      const Unit* u = n->unit.get();
      if (!u || std::find(seen.begin(), seen.end(), u) != seen.end()) continue;
      seen.push_back(u);
      u->collect_metrics(metrics_, n->model_labels);
    }
  }
  return metrics_.render();
}

}  // namespace sca
