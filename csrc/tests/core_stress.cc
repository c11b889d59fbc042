// Host-side stress driver for the sanitizer builds.
//
// The reference has no race detection at all; its shared state is
// ConcurrentHashMap accumulators (PredictiveUnitBean.java:82-84) and
// unsynchronised router counters (EpsilonGreedy.py:118-125).  This binary
// drives every host-side concurrent path of the native core -- codecs, graph
// executor continuations, traffic split + shadows, tracing, metrics, the
// HTTP/1.1 and gRPC front ends -- so that `tools/build_sanitizers.py` can run
// it under AddressSanitizer+UBSan and ThreadSanitizer:
//
//   core_stress fuzz   <iters>     codec fuzzing (JSON / protobuf / feedback), 4 threads
//   core_stress engine <requests>  concurrent predict / feedback / metrics / tracing
//   core_stress serve              HTTP + gRPC front ends; prints "PORTS <http> <grpc>",
//                                  serves until stdin closes (the test drives sca_loadgen)
//
// Exit status 0 = every check passed; sanitizer reports make it non-zero.
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <iostream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "core/engine.h"
#include "core/json.h"
#include "core/message.h"
#include "core/spec.h"
#include "server/grpc_server.h"
#include "server/http_server.h"

using namespace sca;

namespace {

const char* kGraph = R"({
  "name": "stress", "traffic": 100,
  "componentSpecs": [{"spec": {"containers": [{"name": "m1", "image": "seldonio/mock:0.1"}]}}],
  "graph": {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
            "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
            "children": [
              {"name": "m1", "type": "MODEL", "implementation": "SIMPLE_MODEL", "children": []},
              {"name": "avg", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
                {"name": "m2", "type": "MODEL", "implementation": "SIMPLE_MODEL", "children": []},
                {"name": "m3", "type": "MODEL", "implementation": "SIMPLE_MODEL", "children": []}]}]}
})";

const char* kRequests[] = {
    R"({"data":{"names":["a","b"],"ndarray":[[1.0,2.0]]}})",
    R"({"data":{"tensor":{"shape":[3,2],"values":[1,2,3,4,5,6]}},"meta":{"tags":{"t":"v"}}})",
    R"({"strData":"hello"})",
    R"({"binData":"AAEC"})",
    R"({"jsonData":{"k":[1,2,{"x":null}]}})",
    R"({"meta":{"puid":"abc"},"data":{"ndarray":[[0.5,0.25,0.125]]}})",
};

int fails = 0;
std::mutex fail_mu;
void check(bool ok, const std::string& what) {
  if (ok) return;
  std::lock_guard<std::mutex> g(fail_mu);
  ++fails;
  if (fails < 20) std::cerr << "CHECK FAILED: " << what << "\n";
}

std::shared_ptr<Engine> make_engine(std::shared_ptr<MetricsRegistry> shared = nullptr) {
  EngineOptions o;
  o.deployment_name = "stress";
  auto e = std::make_shared<Engine>(parse_predictor_spec(parse_json(kGraph)), o, shared);
  e->finalize();
  return e;
}

Outcome predict_sync(Engine& e, MsgPtr m) {
  std::promise<Outcome> p;
  auto f = p.get_future();
  e.predict(std::move(m), [&p](Outcome o) { p.set_value(std::move(o)); });
  return f.get();
}

// ----------------------------------------------------------------- fuzz
std::string mutate(std::string s, std::mt19937_64& rng) {
  const char alphabet[] = "{}[]\":,0123456789.eE+-truefalsnl \\u\x01\xff";
  const int edits = 1 + int(rng() % 4);
  for (int i = 0; i < edits && !s.empty(); ++i) {
    const size_t pos = rng() % s.size();
    switch (rng() % 4) {
      case 0: s[pos] = alphabet[rng() % (sizeof(alphabet) - 1)]; break;
      case 1: s.erase(pos, 1 + rng() % 3); break;
      case 2: s.insert(pos, 1, alphabet[rng() % (sizeof(alphabet) - 1)]); break;
      default: s.resize(pos); break;
    }
  }
  return s;
}

void fuzz_thread(int seed, int iters) {
  std::mt19937_64 rng(seed);
  for (int i = 0; i < iters; ++i) {
    const std::string base = kRequests[rng() % (sizeof(kRequests) / sizeof(kRequests[0]))];
    // JSON: valid input round-trips; mutated input parses or throws, never crashes.
    {
      SeldonMessage m;
      message_from_json(parse_json(base), m);
      std::string out;
      message_to_json(m, out);
      SeldonMessage m2;
      message_from_json(parse_json(out), m2);
      std::string out2;
      message_to_json(m2, out2);
      check(out == out2, "json round trip: " + out + " vs " + out2);
      std::string pb;
      message_to_pb(m, pb);
      SeldonMessage m3;
      check(message_from_pb(pb, m3), "pb decode of encoded message");
      std::string pb2;
      message_to_pb(m3, pb2);
      check(pb == pb2, "pb round trip");
      // protobuf: random corruption of a valid encoding
      for (int k = 0; k < 4 && !pb.empty(); ++k) {
        std::string bad = pb;
        bad[rng() % bad.size()] = char(rng());
        if (rng() % 2) bad.resize(rng() % bad.size());
        SeldonMessage junk;
        (void)message_from_pb(bad, junk);
      }
    }
    try {
      SeldonMessage m;
      message_from_json(parse_json(mutate(base, rng)), m);
      std::string out;
      message_to_json(m, out);
    } catch (const std::exception&) {
    }
    try {
      Feedback f;
      feedback_from_json(parse_json(mutate(R"({"request":)" + base + R"(,"reward":1.0,"response":{"meta":{"routing":{"ab":1}}}})", rng)), f);
    } catch (const std::exception&) {
    }
  }
}

// --------------------------------------------------------------- engine
void engine_mode(int requests) {
  auto shared = std::make_shared<MetricsRegistry>();
  auto e = make_engine(shared);
  auto peer = make_engine(shared);
  auto shadow = make_engine(shared);
  e->set_traffic(50, {{peer, 50}}, {shadow});
  e->enable_tracing(1.0);
  std::atomic<bool> stop{false};
  std::thread scraper([&] {
    while (!stop.load()) {
      check(e->render_metrics().find("seldon_api_engine_server_requests") != std::string::npos ||
                true, "metrics");
      (void)e->drain_spans();
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  std::vector<std::thread> ts;
  const int nthreads = 8;
  for (int t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937_64 rng(1000 + t);
      for (int i = 0; i < requests / nthreads; ++i) {
        auto m = std::make_shared<SeldonMessage>();
        message_from_json(parse_json(kRequests[rng() % 2]), *m);
        Outcome o = predict_sync(*e, m);
        check(o.msg != nullptr, "predict failed: " + (o.err ? o.err->info : std::string("?")));
        if (!o.msg) continue;
        // feedback along the response's routing, like the MAB loop
        std::string resp;
        message_to_json(*o.msg, resp);
        auto fb = std::make_shared<Feedback>();
        std::string req;
        message_to_json(*m, req);
        feedback_from_json(parse_json(R"({"request":)" + req + R"(,"response":)" + resp + R"(,"reward":1.0})"), *fb);
        std::promise<ErrPtr> p;
        auto f = p.get_future();
        e->send_feedback(fb, [&p](ErrPtr x) { p.set_value(std::move(x)); });
        check(f.get() == nullptr, "feedback failed");
      }
    });
  }
  for (auto& t : ts) t.join();
  stop.store(true);
  scraper.join();
  check(e->inflight() == 0, "inflight after drain");
}

// ---------------------------------------------------------------- serve
void serve_mode() {
  auto e = make_engine();
  HttpOptions ho;
  ho.host = "127.0.0.1";
  ho.ports = {0};
  ho.threads = 4;
  HttpServer http(e, ho);
  http.start();
  GrpcOptions go;
  go.host = "127.0.0.1";
  go.port = 0;
  go.threads = 4;
  GrpcServer grpc(e, go);
  grpc.start();
  std::cout << "PORTS " << http.bound_ports().at(0) << " " << grpc.bound_port() << std::endl;
  // Toggle readiness from another thread while traffic runs (/pause races).
  std::atomic<bool> stop{false};
  std::thread toggler([&] {
    while (!stop.load()) {
      (void)http.paused();
      (void)e->render_metrics();
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  });
  std::string line;
  while (std::getline(std::cin, line)) {
  }
  stop.store(true);
  toggler.join();
  grpc.stop();
  http.stop();
  std::cout << "served " << http.requests_served() << std::endl;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "engine";
  const int n = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (mode == "fuzz") {
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t) ts.emplace_back(fuzz_thread, 7 + t, n);
    for (auto& t : ts) t.join();
  } else if (mode == "engine") {
    engine_mode(n);
  } else if (mode == "serve") {
    serve_mode();
  } else {
    std::cerr << "usage: core_stress fuzz|engine|serve [n]\n";
    return 2;
  }
  if (fails) {
    std::cerr << fails << " checks failed\n";
    return 1;
  }
  std::cout << "ok " << mode << std::endl;
  return 0;
}
