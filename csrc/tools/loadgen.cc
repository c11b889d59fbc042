// sca_loadgen: closed-loop load generator for the engine's REST and gRPC
// front ends (MI355X-native replacement for the reference's locust setup:
// util/loadtester/scripts/predict_rest_locust.py, predict_grpc_locust.py;
// helm-charts/seldon-core-loadtesting).
//
// N concurrent "users" (connections x streams) each keep exactly one request
// in flight, like locust users with no wait time.  Work is divided into steps
// of R completed requests; per-step wall time and every request's latency are
// reported as one JSON object on stdout.
//
//   sca_loadgen --mode rest --host 127.0.0.1 --port 8000 --path /api/v0.1/predictions
//               --body '{"data":{"ndarray":[[1,2]]}}' --users 256 --threads 8
//               --steps 10 --warmup 2 --step-requests 20000
//   sca_loadgen --mode grpc --port 5001 --path /seldon.protos.Seldon/Predict
//               --body-file req.pb ...
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

using Clock = std::chrono::steady_clock;

struct Args {
  std::string mode = "rest";
  std::string host = "127.0.0.1";
  int port = 8000;
  std::string path = "/api/v0.1/predictions";
  std::string body;
  std::string content_type = "application/json";
  int users = 256;
  int threads = 8;
  int streams_per_conn = 1;  // grpc: concurrent streams per connection
  int steps = 5;
  int warmup = 1;
  long step_requests = 10000;
  bool keepalive = true;
  // Sampled reply check: every `check_every`-th reply of a worker must contain
  // `expect` (e.g. the DefaultData bytes of a reference reply); a 200 whose
  // body differs counts as an error, so a wrong answer inside the timed
  // region fails the run instead of counting as a prediction.
  std::string expect;
  long check_every = 16;
  // Poll epoll without blocking for up to this many microseconds before a
  // blocking wait (0 = always block): a client thread that never sleeps costs
  // the server no wake-up in its send path.
  int spin_us = 0;
};

// epoll_wait that polls (timeout 0) for up to spin_us before blocking.
static int wait_events(int epfd, epoll_event* evs, int max, int spin_us) {
  if (spin_us > 0) {
    const auto until = Clock::now() + std::chrono::microseconds(spin_us);
    do {
      const int n = epoll_wait(epfd, evs, max, 0);
      if (n != 0) return n;
    } while (Clock::now() < until);
  }
  return epoll_wait(epfd, evs, max, 1000);
}

static std::string read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) {
    fprintf(stderr, "cannot read %s\n", p.c_str());
    exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static int connect_to(const std::string& host, int port) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  inet_pton(AF_INET, host.c_str(), &a.sin_addr);
  for (int attempt = 0; attempt < 200; ++attempt) {
    if (connect(fd, (sockaddr*)&a, sizeof a) == 0) break;
    if (attempt == 199) {
      perror("connect");
      exit(3);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    close(fd);
    fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  return fd;
}

// ------------------------------------------------------------- step control
struct StepCtl {
  std::atomic<long> issued{0};
  long limit = 0;
  std::atomic<long> errors{0};
  std::atomic<long> completed{0};
  std::atomic<long> checked{0};
  std::atomic<long> bad_body{0};
  bool try_issue() { return issued.fetch_add(1, std::memory_order_relaxed) < limit; }
};

// ------------------------------------------------------------- REST client
struct RestConn {
  int fd;
  std::string in;
  size_t sent = 0;
  bool busy = false;
  Clock::time_point t0;
};

struct Worker {
  const Args* a;
  std::string request;  // full HTTP request bytes (REST)
  std::vector<float> lat_us;
  bool record = false;
  long replies = 0;  // this worker's replies so far (check sampling)

  // true when this reply is sampled and its body lacks the expected bytes
  bool body_bad(const char* p, size_t n, StepCtl& st) {
    if (a->expect.empty() || (replies++ % a->check_every) != 0) return false;
    st.checked.fetch_add(1, std::memory_order_relaxed);
    if (memmem(p, n, a->expect.data(), a->expect.size()) != nullptr) return false;
    st.bad_body.fetch_add(1, std::memory_order_relaxed);
    return true;
  }

  // REST
  std::vector<RestConn> rconns;
  int epfd = -1;

  void init_rest(int nconn) {
    epfd = epoll_create1(0);
    std::ostringstream r;
    r << "POST " << a->path << " HTTP/1.1\r\nHost: " << a->host << ":" << a->port
      << "\r\nContent-Type: " << a->content_type << "\r\nContent-Length: " << a->body.size() << "\r\n\r\n"
      << a->body;
    request = r.str();
    rconns.resize(size_t(nconn));
    for (int i = 0; i < nconn; ++i) {
      rconns[size_t(i)].fd = connect_to(a->host, a->port);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLET;
      ev.data.u32 = uint32_t(i);
      epoll_ctl(epfd, EPOLL_CTL_ADD, rconns[size_t(i)].fd, &ev);
    }
  }

  bool rest_send(RestConn& c) {
    while (c.sent < request.size()) {
      ssize_t w = ::send(c.fd, request.data() + c.sent, request.size() - c.sent, MSG_NOSIGNAL);
      if (w > 0) { c.sent += size_t(w); continue; }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;
      return false;
    }
    return true;
  }

  // Returns true when a full response was consumed.
  bool rest_parse(RestConn& c, StepCtl& st) {
    size_t he = c.in.find("\r\n\r\n");
    if (he == std::string::npos) return false;
    size_t cl = 0;
    size_t p = c.in.find("Content-Length:");
    if (p == std::string::npos) p = c.in.find("content-length:");
    if (p != std::string::npos && p < he) cl = size_t(strtoul(c.in.c_str() + p + 15, nullptr, 10));
    if (c.in.size() < he + 4 + cl) return false;
    int status = atoi(c.in.c_str() + 9);
    const bool bad = status == 200 && body_bad(c.in.data() + he + 4, cl, st);
    c.in.erase(0, he + 4 + cl);
    if (status != 200 || bad) st.errors.fetch_add(1, std::memory_order_relaxed);
    st.completed.fetch_add(1, std::memory_order_relaxed);
    if (record) lat_us.push_back(float(std::chrono::duration<double, std::micro>(Clock::now() - c.t0).count()));
    c.busy = false;
    return true;
  }

  void rest_step(StepCtl& st) {
    int active = 0;
    for (auto& c : rconns) {
      if (st.try_issue()) {
        c.busy = true;
        c.sent = 0;
        c.t0 = Clock::now();
        rest_send(c);
        ++active;
      }
    }
    epoll_event evs[512];
    char buf[65536];
    while (active > 0) {
      int n = wait_events(epfd, evs, 512, a->spin_us);
      for (int i = 0; i < n; ++i) {
        RestConn& c = rconns[evs[i].data.u32];
        if (!c.busy) {
          // drain stray data
          while (::recv(c.fd, buf, sizeof buf, 0) > 0) {}
          continue;
        }
        if (evs[i].events & EPOLLOUT) rest_send(c);
        if (evs[i].events & EPOLLIN) {
          while (true) {
            ssize_t r = ::recv(c.fd, buf, sizeof buf, 0);
            if (r > 0) {
              c.in.append(buf, size_t(r));
              if (size_t(r) < sizeof buf) break;  // drained (edge-triggered epoll)
              continue;
            }
            if (r == 0) { fprintf(stderr, "server closed connection\n"); exit(4); }
            break;
          }
          while (c.busy && rest_parse(c, st)) {
            if (st.try_issue()) {
              c.busy = true;
              c.sent = 0;
              c.t0 = Clock::now();
              rest_send(c);
            } else {
              --active;
            }
          }
        }
      }
    }
  }

  // ------------------------------------------------------------ gRPC client
  struct GStream {
    Clock::time_point t0;
    int grpc_status = -1;
    size_t off = 0;
    std::string body;  // reply bytes (only while checking bodies)
  };
  struct GConn {
    int fd;
    nghttp2_session* s = nullptr;
    Worker* w;
    StepCtl* st = nullptr;
    int inflight = 0;
    std::unordered_map<int32_t, GStream> streams;
    std::string out;
  };
  std::vector<std::unique_ptr<GConn>> gconns;
  std::string grpc_msg;  // length-prefixed
  nghttp2_session_callbacks* cbs = nullptr;

  static ssize_t g_read(nghttp2_session*, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags,
                        nghttp2_data_source* src, void*) {
    auto* c = static_cast<GConn*>(src->ptr);
    auto& gs = c->streams[sid];
    const std::string& m = c->w->grpc_msg;
    size_t n = std::min(len, m.size() - gs.off);
    memcpy(buf, m.data() + gs.off, n);
    gs.off += n;
    if (gs.off == m.size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
    return ssize_t(n);
  }
  static int g_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* v,
                      size_t vl, uint8_t, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    if (nl == 11 && !memcmp(name, "grpc-status", 11)) c->streams[f->hd.stream_id].grpc_status = atoi(std::string((const char*)v, vl).c_str());
    return 0;
  }
  static int g_chunk(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    if (!c->w->a->expect.empty()) {
      auto it = c->streams.find(sid);
      if (it != c->streams.end()) it->second.body.append(reinterpret_cast<const char*>(data), len);
    }
    return 0;
  }
  static int g_close(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    auto it = c->streams.find(sid);
    if (it == c->streams.end()) return 0;
    const bool bad = it->second.grpc_status == 0 &&
                     c->w->body_bad(it->second.body.data(), it->second.body.size(), *c->st);
    if (it->second.grpc_status != 0 || bad) c->st->errors.fetch_add(1, std::memory_order_relaxed);
    c->st->completed.fetch_add(1, std::memory_order_relaxed);
    if (c->w->record)
      c->w->lat_us.push_back(float(std::chrono::duration<double, std::micro>(Clock::now() - it->second.t0).count()));
    c->streams.erase(it);
    --c->inflight;
    if (c->st->try_issue()) c->w->g_submit(*c);
    return 0;
  }

  void g_submit(GConn& c) {
    std::string auth = a->host + ":" + std::to_string(a->port);
    nghttp2_nv hdrs[] = {
        {(uint8_t*)":method", (uint8_t*)"POST", 7, 4, 0},
        {(uint8_t*)":scheme", (uint8_t*)"http", 7, 4, 0},
        {(uint8_t*)":path", (uint8_t*)a->path.c_str(), 5, a->path.size(), 0},
        {(uint8_t*)":authority", (uint8_t*)auth.c_str(), 10, auth.size(), 0},
        {(uint8_t*)"content-type", (uint8_t*)"application/grpc", 12, 16, 0},
        {(uint8_t*)"te", (uint8_t*)"trailers", 2, 8, 0},
    };
    nghttp2_data_provider prd;
    prd.source.ptr = &c;
    prd.read_callback = g_read;
    int32_t sid = nghttp2_submit_request(c.s, nullptr, hdrs, 6, &prd, nullptr);
    if (sid < 0) { fprintf(stderr, "submit_request failed\n"); exit(5); }
    c.streams[sid].t0 = Clock::now();
    ++c.inflight;
  }

  void g_flush(GConn& c) {
    const uint8_t* data;
    ssize_t n;
    while ((n = nghttp2_session_mem_send(c.s, &data)) > 0) c.out.append((const char*)data, size_t(n));
    size_t off = 0;
    while (off < c.out.size()) {
      ssize_t w = ::send(c.fd, c.out.data() + off, c.out.size() - off, MSG_NOSIGNAL);
      if (w > 0) { off += size_t(w); continue; }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      fprintf(stderr, "send failed\n");
      exit(4);
    }
    c.out.erase(0, off);
  }

  void init_grpc(int nconn) {
    epfd = epoll_create1(0);
    uint32_t n = htonl(uint32_t(a->body.size()));
    grpc_msg.assign(1, '\0');
    grpc_msg.append((const char*)&n, 4);
    grpc_msg += a->body;
    nghttp2_session_callbacks_new(&cbs);
    nghttp2_session_callbacks_set_on_header_callback(cbs, g_header);
    nghttp2_session_callbacks_set_on_stream_close_callback(cbs, g_close);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, g_chunk);
    for (int i = 0; i < nconn; ++i) {
      auto c = std::make_unique<GConn>();
      c->fd = connect_to(a->host, a->port);
      c->w = this;
      nghttp2_session_client_new(&c->s, cbs, c.get());
      nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16 << 20}};
      nghttp2_submit_settings(c->s, NGHTTP2_FLAG_NONE, iv, 1);
      nghttp2_session_set_local_window_size(c->s, NGHTTP2_FLAG_NONE, 0, 256 << 20);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLET;
      ev.data.u32 = uint32_t(i);
      epoll_ctl(epfd, EPOLL_CTL_ADD, c->fd, &ev);
      g_flush(*c);
      gconns.push_back(std::move(c));
    }
  }

  void grpc_step(StepCtl& st) {
    for (auto& c : gconns) {
      c->st = &st;
      for (int s = 0; s < a->streams_per_conn; ++s)
        if (st.try_issue()) g_submit(*c);
      g_flush(*c);
    }
    epoll_event evs[512];
    uint8_t buf[65536];
    auto total_inflight = [&] {
      int t = 0;
      for (auto& c : gconns) t += c->inflight;
      return t;
    };
    while (total_inflight() > 0) {
      int n = wait_events(epfd, evs, 512, a->spin_us);
      for (int i = 0; i < n; ++i) {
        GConn& c = *gconns[evs[i].data.u32];
        if (evs[i].events & EPOLLIN) {
          while (true) {
            ssize_t r = ::recv(c.fd, buf, sizeof buf, 0);
            if (r > 0) {
              if (nghttp2_session_mem_recv(c.s, buf, size_t(r)) < 0) { fprintf(stderr, "h2 recv error\n"); exit(4); }
              if (size_t(r) < sizeof buf) break;  // drained (edge-triggered epoll)
              continue;
            }
            if (r == 0) { fprintf(stderr, "server closed connection\n"); exit(4); }
            break;
          }
        }
        g_flush(c);
      }
    }
  }
};

static double pct(std::vector<float>& v, double q) {
  if (v.empty()) return 0;
  size_t k = size_t(q * double(v.size() - 1) + 0.5);
  std::nth_element(v.begin(), v.begin() + long(k), v.end());
  return double(v[k]) / 1000.0;
}

int main(int argc, char** argv) {
  Args a;
  std::string body_file;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto v = [&]() -> std::string {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); exit(2); }
      return argv[++i];
    };
    if (k == "--mode") a.mode = v();
    else if (k == "--host") a.host = v();
    else if (k == "--port") a.port = std::stoi(v());
    else if (k == "--path") a.path = v();
    else if (k == "--body") a.body = v();
    else if (k == "--body-file") body_file = v();
    else if (k == "--content-type") a.content_type = v();
    else if (k == "--users") a.users = std::stoi(v());
    else if (k == "--threads") a.threads = std::stoi(v());
    else if (k == "--streams-per-conn") a.streams_per_conn = std::stoi(v());
    else if (k == "--steps") a.steps = std::stoi(v());
    else if (k == "--warmup") a.warmup = std::stoi(v());
    else if (k == "--step-requests") a.step_requests = std::stol(v());
    else if (k == "--expect") a.expect = v();
    else if (k == "--expect-file") a.expect = read_file(v());
    else if (k == "--check-every") a.check_every = std::max(1L, std::stol(v()));
    else if (k == "--spin-us") a.spin_us = std::max(0, std::stoi(v()));
    else if (k == "--cpus") {  // comma-separated CPU ids: pin this process (bench placement A/B)
      cpu_set_t set;
      CPU_ZERO(&set);
      const std::string list = v();
      size_t pos = 0;
      while (pos < list.size()) {
        const size_t e = list.find(',', pos);
        CPU_SET(std::stoi(list.substr(pos, e == std::string::npos ? std::string::npos : e - pos)), &set);
        if (e == std::string::npos) break;
        pos = e + 1;
      }
      if (sched_setaffinity(0, sizeof set, &set) != 0) { perror("sched_setaffinity"); return 2; }
    }
    else { fprintf(stderr, "unknown arg %s\n", k.c_str()); return 2; }
  }
  if (!body_file.empty()) a.body = read_file(body_file);
  const bool grpc = a.mode == "grpc";
  const int nthreads = std::max(1, std::min(a.threads, a.users));
  int conns_total = grpc ? std::max(1, a.users / std::max(1, a.streams_per_conn)) : a.users;
  std::vector<Worker> workers(static_cast<size_t>(nthreads));
  for (int t = 0; t < nthreads; ++t) {
    workers[size_t(t)].a = &a;
    int nc = conns_total / nthreads + (t < conns_total % nthreads ? 1 : 0);
    if (grpc) workers[size_t(t)].init_grpc(std::max(1, nc));
    else workers[size_t(t)].init_rest(std::max(1, nc));
  }
  std::vector<double> step_ms;
  long total_ok = 0, total_err = 0, total_checked = 0, total_bad = 0;
  double timed_s = 0;
  for (int step = 0; step < a.warmup + a.steps; ++step) {
    const bool timed = step >= a.warmup;
    StepCtl st;
    st.limit = a.step_requests;
    for (auto& w : workers) w.record = timed;
    auto t0 = Clock::now();
    std::vector<std::thread> th;
    for (auto& w : workers) th.emplace_back([&w, &st, grpc] { grpc ? w.grpc_step(st) : w.rest_step(st); });
    for (auto& t : th) t.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    if (timed) {
      step_ms.push_back(dt * 1000.0);
      timed_s += dt;
      total_ok += st.completed.load() - st.errors.load();
      total_err += st.errors.load();
    }
    total_checked += st.checked.load();  // warmup replies are checked too
    total_bad += st.bad_body.load();
  }
  std::vector<float> lat;
  for (auto& w : workers) lat.insert(lat.end(), w.lat_us.begin(), w.lat_us.end());
  double mean = 0, mx = 0;
  for (float x : lat) { mean += x; mx = std::max(mx, double(x)); }
  mean = lat.empty() ? 0 : mean / double(lat.size()) / 1000.0;
  printf("{\"mode\":\"%s\",\"users\":%d,\"threads\":%d,\"steps\":%d,\"step_requests\":%ld,\"ok\":%ld,\"errors\":%ld,"
         "\"seconds\":%.6f,\"rps\":%.2f,\"p50_ms\":%.4f,\"p90_ms\":%.4f,\"p99_ms\":%.4f,\"p999_ms\":%.4f,"
         "\"mean_ms\":%.4f,\"max_ms\":%.4f,\"checked\":%ld,\"bad_body\":%ld,\"step_ms\":[",
         a.mode.c_str(), a.users, nthreads, a.steps, a.step_requests, total_ok, total_err, timed_s,
         timed_s > 0 ? double(total_ok) / timed_s : 0.0, pct(lat, 0.5), pct(lat, 0.9), pct(lat, 0.99),
         pct(lat, 0.999), mean, mx / 1000.0, total_checked, total_bad);
  for (size_t i = 0; i < step_ms.size(); ++i) printf("%s%.4f", i ? "," : "", step_ms[i]);
  printf("]}\n");
  return (total_err > 0 || total_bad > 0) ? 1 : 0;
}
