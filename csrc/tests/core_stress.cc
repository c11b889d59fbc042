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
//   core_stress batcher <requests> the GPU micro-batcher's host machinery on its CPU
//                                  path (cpu_batching): per-thread submission shards,
//                                  device thread, hand-off thread, recycled response
//                                  parcels posted to 8 executors by 8 producer threads
//   core_stress mesh <requests>    a CPU gang's mesh (csrc/parallel/mesh.cc) with rank 0
//                                  and rank 1 in this one process: 8 producer threads
//                                  through a cpu_batching unit over the program model
//                                  (async pump, chunked issue, reap, doorbells), the
//                                  worker's program thread, and calls abandoned mid-flight
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

#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>

#include <sys/socket.h>

#include "core/engine.h"
#include "gpu/batcher.h"
#include "kernels/kernels.h"
#include "parallel/mesh.h"
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

// ---------------------------------------------------------------- batcher
// y = [sum(x), 2 * x0, rows_in_batch-independent id]: each request can check
// its own answer.
class FakeRowModel : public gpu::RowModel {
 public:
  std::string name() const override { return "fake"; }
  int in_cols() const override { return 4; }
  int out_cols(int) const override { return 3; }
  void to_device(int) override {}
  void launch(const double*, int, int, double*, void*, hipStream_t) override {
    throw std::runtime_error("fake model has no device path");
  }
  void run_cpu(const double* X, int rows, int cols, double* out) const override {
    for (int r = 0; r < rows; ++r) {
      const double* x = X + size_t(r) * cols;
      out[r * 3 + 0] = x[0] + x[1] + x[2] + x[3];
      out[r * 3 + 1] = 2.0 * x[0];
      out[r * 3 + 2] = x[3];
    }
  }
};

// One thread draining posted continuations (a front-end worker stand-in).
class ThreadExecutor : public Executor {
 public:
  ThreadExecutor() : th_([this] { run(); }) {}
  ~ThreadExecutor() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void post(std::function<void()> fn) override {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(fn));
    }
    cv_.notify_one();
  }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      auto fn = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      fn();
      lk.lock();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;
};

void batcher_mode(int n) {
  gpu::BatcherOptions o;
  o.device = -1;
  o.cpu_batching = true;
  o.slots = 3;
  o.max_batch = 64;
  auto unit = std::make_shared<gpu::BatchedUnit>(std::make_shared<FakeRowModel>(), o);
  constexpr int kThreads = 8;
  std::vector<ExecPtr> execs;
  for (int i = 0; i < kThreads; ++i) execs.push_back(std::make_shared<ThreadExecutor>());
  std::atomic<int> done{0}, wrong{0};
  std::vector<std::thread> producers;
  const std::string puid = "stress";
  for (int t = 0; t < kThreads; ++t) {
    producers.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      for (int i = 0; i < n; ++i) {
        const int rows = 1 + int(rng() % 3);
        auto m = std::make_shared<SeldonMessage>();
        m->payload = Payload::Data;
        std::vector<double> vals;
        for (int r = 0; r < rows; ++r) {
          const double id = double(t) * 1e6 + i * 10 + r;
          vals.insert(vals.end(), {1.0 * r, 0.5, 0.25, id});
        }
        m->data.set_dense(DataKind::Tensor, {int64_t(rows), 4}, std::move(vals));
        // a third of the requests finish on the completing thread (no executor)
        const ExecPtr* ex = (i % 3 == 0) ? nullptr : &execs[size_t((t + i) % kThreads)];
        CallCtx c{nullptr, &puid, ex};
        unit->transform_input(c, m, [&, t, i, rows](Outcome o) {
          bool ok = !o.err && o.msg && o.msg->data.values.size() == size_t(rows) * 3;
          if (ok)
            for (int r = 0; r < rows; ++r) {
              const double id = double(t) * 1e6 + i * 10 + r;
              const double* y = o.msg->data.values.data() + r * 3;
              ok = ok && y[0] == 1.0 * r + 0.75 + id && y[1] == 2.0 * r && y[2] == id;
            }
          if (!ok) wrong.fetch_add(1);
          done.fetch_add(1);
        });
      }
    });
  }
  for (auto& p : producers) p.join();
  for (int spin = 0; done.load() < kThreads * n && spin < 30000; ++spin) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  const auto st = unit->stats();
  unit->stop();
  execs.clear();
  check(done.load() == kThreads * n, "every batched request answered exactly once");
  check(wrong.load() == 0, "every batched request got its own rows back");
  check(st.requests == uint64_t(kThreads) * n, "batcher counted every request");
  check(st.batches < st.requests, "requests shared batches");
  std::cout << "batches " << st.batches << " requests " << st.requests << std::endl;
}

void mesh_mode(int n) {
  // control sockets: rank 0 holds one end per worker, the worker the other
  int sp[2];
  check(socketpair(AF_UNIX, SOCK_STREAM, 0, sp) == 0, "socketpair");
  constexpr int kSlots = 4;
  auto m0 = std::make_shared<par::Mesh>(0, 2, -1, std::vector<int>{-1, sp[0]}, kSlots);
  auto m1 = std::make_shared<par::Mesh>(1, 2, -1, std::vector<int>{sp[1], -1}, kSlots);
  par::MeshProgram prog;
  prog.max_rows = 16;  // small: multi-row batches are issued in chunks
  prog.in_cols = 4;
  par::MeshStage st;
  st.rank = 1;
  st.kind = par::kMeshModel;
  st.inputs = {-1};
  st.in_cols = 4;
  st.out_cols = 3;
  st.node = "fake";
  prog.stages.push_back(st);
  m0->add_program(prog);
  m1->add_program(prog);
  m1->set_model(0, 0, std::make_shared<FakeRowModel>());
  const std::vector<std::string> blobs{m0->prepare(), m1->prepare()};
  m0->connect(blobs);
  m1->connect(blobs);
  m0->unlink();
  m1->unlink();
  m1->start();
  m0->start();
  gpu::BatcherOptions o;
  o.device = -1;
  o.cpu_batching = true;
  o.slots = kSlots;
  o.max_batch = 64;
  auto unit = std::make_shared<gpu::BatchedUnit>(m0->program_model(0, {}, false), o);
  constexpr int kThreads = 8;
  std::vector<ExecPtr> execs;
  for (int i = 0; i < kThreads; ++i) execs.push_back(std::make_shared<ThreadExecutor>());
  std::atomic<int> done{0}, wrong{0};
  std::vector<std::thread> producers;
  const std::string puid = "stress";
  for (int t = 0; t < kThreads; ++t) {
    producers.emplace_back([&, t] {
      std::mt19937 rng(4321 + t);
      for (int i = 0; i < n; ++i) {
        const int rows = 1 + int(rng() % 5);
        auto m = std::make_shared<SeldonMessage>();
        m->payload = Payload::Data;
        std::vector<double> vals;
        for (int r = 0; r < rows; ++r) {
          const double id = double(t) * 1e6 + i * 10 + r;
          vals.insert(vals.end(), {1.0 * r, 0.5, 0.25, id});
        }
        m->data.set_dense(DataKind::Tensor, {int64_t(rows), 4}, std::move(vals));
        const ExecPtr* ex = (i % 3 == 0) ? nullptr : &execs[size_t((t + i) % kThreads)];
        CallCtx c{nullptr, &puid, ex};
        unit->transform_input(c, m, [&, t, i, rows](Outcome out) {
          bool ok = !out.err && out.msg && out.msg->data.values.size() == size_t(rows) * 3;
          if (ok)
            for (int r = 0; r < rows; ++r) {
              const double id = double(t) * 1e6 + i * 10 + r;
              const double* y = out.msg->data.values.data() + r * 3;
              ok = ok && y[0] == 1.0 * r + 0.75 + id && y[1] == 2.0 * r && y[2] == id;
            }
          if (!ok) wrong.fetch_add(1);
          done.fetch_add(1);
        });
      }
    });
  }
  // direct callers of the program model on the side, half of them giving up
  // mid-flight (their batches complete and free their slots, `out` untouched)
  auto pm = m0->program_model(0, {}, false);
  std::atomic<int> direct_ok{0};
  std::thread side([&] {
    std::vector<double> x(4 * 7), y(3 * 7);
    for (int i = 0; i < n / 4; ++i) {
      for (int r = 0; r < 7; ++r) {
        x[size_t(r) * 4 + 0] = r;
        x[size_t(r) * 4 + 1] = 0.5;
        x[size_t(r) * 4 + 2] = 0.25;
        x[size_t(r) * 4 + 3] = 7e6 + i;
      }
      auto call = pm->start_cpu(x.data(), 7, 4, y.data());
      if (i % 2) {
        call.reset();  // abandoned
        continue;
      }
      while (!call->done()) call->wait_us(100);
      bool ok = call->error().empty();
      for (int r = 0; r < 7 && ok; ++r) ok = y[size_t(r) * 3 + 2] == 7e6 + i && y[size_t(r) * 3 + 1] == 2.0 * r;
      if (ok) direct_ok.fetch_add(1);
    }
  });
  for (auto& p : producers) p.join();
  side.join();
  for (int spin = 0; done.load() < kThreads * n && spin < 60000; ++spin)
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  const auto stu = unit->stats();
  unit->stop();
  execs.clear();
  m0->stop_peers();
  m1->join();
  const auto ms = m1->stats();
  check(done.load() == kThreads * n, "every mesh request answered exactly once");
  check(wrong.load() == 0, "every mesh request got its own rows back");
  check(direct_ok.load() == (n / 4 + 1) / 2, "every direct (not abandoned) call got its rows");
  check(m0->error().empty() && m1->error().empty(), "no mesh error");
  check(stu.batches < stu.requests, "mesh requests shared batches");
  std::cout << "mesh batches " << ms.batches << " rows " << ms.rows << " max_inflight " << ms.max_inflight << std::endl;
  ::close(sp[0]);
  ::close(sp[1]);
}

}  // namespace

// The mesh's GPU-gang path references two device helpers; a CPU gang never
// calls them, and the sanitizer build has no device code.
namespace sca::kern {
void combine_mean_f64(const double* const*, int, int64_t, double*, hipStream_t) { std::abort(); }
void device_delay_us(int, hipStream_t) { std::abort(); }
}  // namespace sca::kern

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
  } else if (mode == "batcher") {
    batcher_mode(n);
  } else if (mode == "mesh") {
    mesh_mode(n);
  } else {
    std::cerr << "usage: core_stress fuzz|engine|serve|batcher|mesh [n]\n";
    return 2;
  }
  if (fails) {
    std::cerr << fails << " checks failed\n";
    return 1;
  }
  std::cout << "ok " << mode << std::endl;
  return 0;
}
