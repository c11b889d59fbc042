#include "grpc_server.h"

#include <arpa/inet.h>
#include <nghttp2/nghttp2.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <unordered_map>

namespace sca {

namespace {

// gRPC status codes
enum : int { kOk = 0, kUnknown = 2, kInvalidArgument = 3, kDeadline = 4, kResourceExhausted = 8,
             kUnimplemented = 12, kInternal = 13, kUnavailable = 14 };

struct GStream {
  int32_t id = 0;
  std::string path;
  std::string body;
  std::string resp;  // length-prefixed gRPC message
  size_t resp_off = 0;
  bool compressed_enc = false;
  bool too_big = false;
};

struct GConn {
  int fd = -1;
  uint64_t gen = 0;
  nghttp2_session* session = nullptr;
  std::string out;
  size_t out_off = 0;
  bool dead = false;
  std::unordered_map<int32_t, std::unique_ptr<GStream>> streams;
  GrpcServer::Worker* w = nullptr;
  ~GConn() {
    if (session) nghttp2_session_del(session);
  }
};

struct GCompletion {
  int fd;
  uint64_t gen;
  int32_t stream;
  int grpc_status;
  std::string message;  // grpc-message on error
  std::string payload;  // serialized protobuf on success
};

std::string pct_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') o.push_back(char(c));
    else { o.push_back('%'); o.push_back(hex[c >> 4]); o.push_back(hex[c & 15]); }
  }
  return o;
}

nghttp2_nv make_nv(const char* n, const char* v, size_t vlen) {
  nghttp2_nv nv;
  nv.name = (uint8_t*)n;
  nv.value = (uint8_t*)v;
  nv.namelen = strlen(n);
  nv.valuelen = vlen;
  nv.flags = NGHTTP2_NV_FLAG_NONE;
  return nv;
}

int grpc_status_of(const EngineError& e) {
  if (!e.body.empty()) {  // a component's own error: its HTTP status in gRPC terms
    switch (e.http_status) {
      case 400: return kInvalidArgument;
      case 401: return 16;  // UNAUTHENTICATED
      case 403: return 7;   // PERMISSION_DENIED
      case 404: return 5;   // NOT_FOUND
      case 409: return 10;  // ABORTED
      case 429: return kResourceExhausted;
      case 501: return kUnimplemented;
      case 503: return kUnavailable;
      case 504: return kDeadline;
      default: return kUnknown;
    }
  }
  switch (e.code) {
    case 201: return kInvalidArgument;
    case 209: return kUnavailable;
    case 210: return kDeadline;
    default: return kUnknown;
  }
}

}  // namespace

struct GrpcServer::Worker : Executor, std::enable_shared_from_this<GrpcServer::Worker> {
  GrpcServer* srv = nullptr;
  int epfd = -1, evfd = -1, lfd = -1;
  std::thread th;
  std::thread::id tid;
  std::atomic<bool> stop{false};
  std::unordered_map<int, std::unique_ptr<GConn>> conns;
  uint64_t next_gen = 1;
  std::mutex qmu;
  std::vector<GCompletion> q;
  std::vector<std::function<void()>> tasks;  // continuations posted by GPU units
  bool running_tasks = false;                // worker thread only
  // Wake-ups: an enqueue writes the eventfd only while the worker is (about to
  // be) blocked in epoll_wait; an awake worker picks the work up at the top of
  // its loop.  polling / has_work pair up seq_cst (no lost wake-up), which
  // saves an eventfd write + epoll wake + read per hand-off under load.
  std::atomic<bool> polling{false};
  std::atomic<bool> has_work{false};
  bool need_wake() {  // caller holds qmu, has just queued work
    has_work.store(true, std::memory_order_seq_cst);
    if (wake_pending || !polling.load(std::memory_order_seq_cst)) return false;
    wake_pending = true;
    return true;
  }
  bool wake_pending = false;                 // eventfd written and not yet drained (guarded by qmu)
  nghttp2_session_callbacks* cbs = nullptr;

  // Executor: run a request's continuation on this I/O thread.
  void post(std::function<void()> fn) override {
    if (std::this_thread::get_id() == tid || stop.load(std::memory_order_relaxed)) {
      fn();
      return;
    }
    bool wake;
    {
      std::lock_guard<std::mutex> g(qmu);
      tasks.push_back(std::move(fn));
      wake = need_wake();
    }
    if (wake) {
      uint64_t one = 1;
      ssize_t w = ::write(evfd, &one, 8);
      (void)w;
    }
  }

  ~Worker() {
    for (auto& kv : conns)
      if (!kv.second->dead) ::close(kv.first);
    conns.clear();
    if (lfd >= 0) ::close(lfd);
    if (evfd >= 0) ::close(evfd);
    if (epfd >= 0) ::close(epfd);
    if (cbs) nghttp2_session_callbacks_del(cbs);
  }

  // ------------------------------------------------------------ callbacks
  static int on_begin_headers(nghttp2_session*, const nghttp2_frame* frame, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    if (frame->hd.type != NGHTTP2_HEADERS || frame->headers.cat != NGHTTP2_HCAT_REQUEST) return 0;
    auto s = std::make_unique<GStream>();
    s->id = frame->hd.stream_id;
    c->streams[frame->hd.stream_id] = std::move(s);
    return 0;
  }
  static int on_header(nghttp2_session*, const nghttp2_frame* frame, const uint8_t* name, size_t namelen,
                       const uint8_t* value, size_t valuelen, uint8_t, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    if (frame->hd.type != NGHTTP2_HEADERS) return 0;
    auto it = c->streams.find(frame->hd.stream_id);
    if (it == c->streams.end()) return 0;
    std::string_view n((const char*)name, namelen), v((const char*)value, valuelen);
    if (n == ":path") it->second->path = std::string(v);
    else if (n == "grpc-encoding" && v != "identity") it->second->compressed_enc = true;
    return 0;
  }
  static int on_data_chunk(nghttp2_session*, uint8_t, int32_t stream_id, const uint8_t* data, size_t len, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    auto it = c->streams.find(stream_id);
    if (it == c->streams.end()) return 0;
    GStream* s = it->second.get();
    if (s->body.size() + len > c->w->srv->opts_.max_message + 5) {
      s->too_big = true;
      return 0;
    }
    s->body.append((const char*)data, len);
    return 0;
  }
  static int on_frame_recv(nghttp2_session*, const nghttp2_frame* frame, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    if ((frame->hd.type == NGHTTP2_DATA || frame->hd.type == NGHTTP2_HEADERS) &&
        (frame->hd.flags & NGHTTP2_FLAG_END_STREAM)) {
      auto it = c->streams.find(frame->hd.stream_id);
      if (it != c->streams.end()) c->w->dispatch(c, it->second.get());
    }
    return 0;
  }
  static int on_stream_close(nghttp2_session*, int32_t stream_id, uint32_t, void* ud) {
    auto* c = static_cast<GConn*>(ud);
    c->streams.erase(stream_id);
    return 0;
  }
  static ssize_t read_body(nghttp2_session* session, int32_t stream_id, uint8_t* buf, size_t length,
                           uint32_t* data_flags, nghttp2_data_source* src, void*) {
    auto* s = static_cast<GStream*>(src->ptr);
    const size_t n = std::min(length, s->resp.size() - s->resp_off);
    memcpy(buf, s->resp.data() + s->resp_off, n);
    s->resp_off += n;
    if (s->resp_off == s->resp.size()) {
      *data_flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
      nghttp2_nv tr[] = {make_nv("grpc-status", "0", 1)};
      nghttp2_submit_trailer(session, stream_id, tr, 1);
    }
    return ssize_t(n);
  }

  // ------------------------------------------------------------ responses
  void send_error(GConn* c, int32_t stream_id, int status, const std::string& msg) {
    std::string st = std::to_string(status), m = pct_encode(msg);
    nghttp2_nv hdrs[] = {make_nv(":status", "200", 3), make_nv("content-type", "application/grpc", 16),
                         make_nv("grpc-status", st.c_str(), st.size()), make_nv("grpc-message", m.c_str(), m.size())};
    nghttp2_submit_response(c->session, stream_id, hdrs, 4, nullptr);
  }

  void send_ok(GConn* c, int32_t stream_id, std::string&& pb) {
    auto it = c->streams.find(stream_id);
    if (it == c->streams.end()) return;
    GStream* s = it->second.get();
    s->resp.resize(5 + pb.size());
    s->resp[0] = 0;
    const uint32_t n = htonl(uint32_t(pb.size()));
    memcpy(&s->resp[1], &n, 4);
    memcpy(&s->resp[5], pb.data(), pb.size());
    s->resp_off = 0;
    nghttp2_nv hdrs[] = {make_nv(":status", "200", 3), make_nv("content-type", "application/grpc", 16)};
    nghttp2_data_provider prd;
    prd.source.ptr = s;
    prd.read_callback = read_body;
    nghttp2_submit_response(c->session, stream_id, hdrs, 2, &prd);
  }

  void deliver(GCompletion&& d) {
    if (std::this_thread::get_id() == tid && running_tasks) {  // flushed after the task batch
      std::lock_guard<std::mutex> g(qmu);
      q.push_back(std::move(d));
      return;
    }
    if (std::this_thread::get_id() == tid) {
      complete(std::move(d), false);
      return;
    }
    bool wake;
    {
      std::lock_guard<std::mutex> g(qmu);
      q.push_back(std::move(d));
      wake = need_wake();
    }
    if (wake) {  // one wakeup per drained batch of completions
      uint64_t one = 1;
      ssize_t w = ::write(evfd, &one, 8);
      (void)w;
    }
  }

  void complete(GCompletion&& d, bool flush_now) {
    auto it = conns.find(d.fd);
    if (it == conns.end() || it->second->gen != d.gen || it->second->dead) return;
    GConn* c = it->second.get();
    if (d.grpc_status == kOk) send_ok(c, d.stream, std::move(d.payload));
    else send_error(c, d.stream, d.grpc_status, d.message);
    srv->served_.fetch_add(1, std::memory_order_relaxed);
    if (flush_now) flush(c);
  }

  void drain_queue(bool evfd_ready) {
    if (evfd_ready) {
      uint64_t v;
      ssize_t r = ::read(evfd, &v, 8);
      (void)r;
    }
    std::vector<GCompletion> items;
    std::vector<std::function<void()>> run;
    {
      std::lock_guard<std::mutex> g(qmu);
      if (evfd_ready) wake_pending = false;  // anything queued from now on signals again
      has_work.store(false, std::memory_order_relaxed);
      run.swap(tasks);
    }
    running_tasks = true;
    for (auto& fn : run) fn();
    running_tasks = false;
    {
      std::lock_guard<std::mutex> g(qmu);
      items.swap(q);
    }
    std::vector<int> touched;
    for (auto& d : items) {
      int fd = d.fd;
      complete(std::move(d), false);
      touched.push_back(fd);
    }
    for (int fd : touched) {
      auto it = conns.find(fd);
      if (it != conns.end() && !it->second->dead) {
        flush(it->second.get());
        if (it->second->dead) conns.erase(it);
      }
    }
  }

  // ------------------------------------------------------------ dispatch
  void dispatch(GConn* c, GStream* s) {
    const int32_t sid = s->id;
    if (s->too_big) {
      send_error(c, sid, kResourceExhausted, "message larger than max");
      return;
    }
    if (s->body.size() < 5) {
      send_error(c, sid, kInvalidArgument, "missing gRPC message");
      return;
    }
    if (s->body[0] != 0) {
      send_error(c, sid, kUnimplemented, "compressed messages are not supported");
      return;
    }
    uint32_t len;
    memcpy(&len, s->body.data() + 1, 4);
    len = ntohl(len);
    if (size_t(len) + 5 > s->body.size()) {
      send_error(c, sid, kInvalidArgument, "truncated gRPC message");
      return;
    }
    std::string_view pb(s->body.data() + 5, len);
    const std::string& path = s->path;
    const size_t slash = path.rfind('/');
    std::string service = slash == std::string::npos ? "" : path.substr(0, slash);
    std::string method = slash == std::string::npos ? path : path.substr(slash + 1);
    int fd = c->fd;
    uint64_t gen = c->gen;
    auto self = shared_from_this();
    auto on_msg = [self, fd, gen, sid](Outcome o) {
      GCompletion d{fd, gen, sid, kOk, "", ""};
      if (o.err) {
        d.grpc_status = grpc_status_of(*o.err);
        d.message = error_to_json(*o.err);
      } else if (o.msg) {
        message_to_pb(*o.msg, d.payload);
      }
      self->deliver(std::move(d));
    };
    auto on_fb = [self, fd, gen, sid](ErrPtr e) {
      GCompletion d{fd, gen, sid, kOk, "", ""};
      if (e) {
        d.grpc_status = grpc_status_of(*e);
        d.message = error_to_json(*e);
      }
      self->deliver(std::move(d));
    };
    Engine& eng = *srv->engine_;
    if (method == "SendFeedback") {
      auto fb = std::make_shared<Feedback>();
      if (!feedback_from_pb(pb, *fb)) { send_error(c, sid, kInvalidArgument, "invalid Feedback"); return; }
      eng.send_feedback(fb, on_fb);
      return;
    }
    if (service == "/seldon.protos.Seldon" && method == "Predict") {
      auto msg = std::make_shared<SeldonMessage>();
      if (!message_from_pb(pb, *msg)) { send_error(c, sid, kInvalidArgument, "invalid SeldonMessage"); return; }
      eng.predict(msg, on_msg, self);
      return;
    }
    int m;
    if (method == "Predict") m = Engine::kPredictMethod;
    else if (method == "TransformInput") m = int(Method::TRANSFORM_INPUT);
    else if (method == "TransformOutput") m = int(Method::TRANSFORM_OUTPUT);
    else if (method == "Route") m = int(Method::ROUTE);
    else if (method == "Aggregate") m = int(Method::AGGREGATE);
    else { send_error(c, sid, kUnimplemented, "unknown method " + path); return; }
    if (service.rfind("/seldon.protos.", 0) != 0) { send_error(c, sid, kUnimplemented, "unknown service " + path); return; }
    std::vector<MsgPtr> in;
    if (m == int(Method::AGGREGATE)) {
      std::vector<SeldonMessage> list;
      if (!message_list_from_pb(pb, list)) { send_error(c, sid, kInvalidArgument, "invalid SeldonMessageList"); return; }
      for (auto& x : list) in.push_back(std::make_shared<SeldonMessage>(std::move(x)));
    } else {
      auto msg = std::make_shared<SeldonMessage>();
      if (!message_from_pb(pb, *msg)) { send_error(c, sid, kInvalidArgument, "invalid SeldonMessage"); return; }
      in.push_back(msg);
    }
    const std::string node = srv->opts_.microservice_node.empty() ? eng.spec().graph.name : srv->opts_.microservice_node;
    eng.call_node(node, m, std::move(in), on_msg);
  }

  // ------------------------------------------------------------ socket I/O
  void run() {
    tid = std::this_thread::get_id();
    epoll_event evs[256];
    while (!stop.load(std::memory_order_relaxed)) {
      if (has_work.load(std::memory_order_acquire)) drain_queue(false);
      polling.store(true, std::memory_order_seq_cst);
      if (has_work.load(std::memory_order_seq_cst)) {  // queued after the check above
        polling.store(false, std::memory_order_relaxed);
        continue;
      }
      int n = epoll_wait(epfd, evs, 256, 200);
      polling.store(false, std::memory_order_relaxed);
      for (int i = 0; i < n; ++i) {
        int fd = evs[i].data.fd;
        uint32_t e = evs[i].events;
        if (fd == evfd) { drain_queue(true); continue; }
        if (fd == lfd) { accept_all(); continue; }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        GConn* c = it->second.get();
        if (e & (EPOLLERR | EPOLLHUP)) close_conn(c);
        if (!c->dead && (e & EPOLLIN)) on_readable(c);
        if (!c->dead && (e & EPOLLOUT)) flush(c);
        if (c->dead) conns.erase(fd);
      }
    }
  }

  void accept_all() {
    while (true) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<GConn>();
      c->fd = fd;
      c->gen = next_gen++;
      c->w = this;
      nghttp2_session_server_new(&c->session, cbs, c.get());
      nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
                                     {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16 << 20},
                                     {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1 << 20}};
      nghttp2_submit_settings(c->session, NGHTTP2_FLAG_NONE, iv, 3);
      nghttp2_session_set_local_window_size(c->session, NGHTTP2_FLAG_NONE, 0, 256 << 20);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLET | EPOLLRDHUP;
      ev.data.fd = fd;
      epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &ev);
      GConn* raw = c.get();
      conns[fd] = std::move(c);
      flush(raw);
    }
  }

  void close_conn(GConn* c) {
    if (c->dead) return;
    c->dead = true;
    epoll_ctl(epfd, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
  }

  void on_readable(GConn* c) {
    uint8_t buf[65536];
    while (true) {
      ssize_t r = ::read(c->fd, buf, sizeof buf);
      if (r > 0) {
        ssize_t rv = nghttp2_session_mem_recv(c->session, buf, size_t(r));
        if (rv < 0) { close_conn(c); return; }
        if (size_t(r) < sizeof buf) break;  // drained (edge-triggered: the next arrival is reported)
        continue;
      }
      if (r == 0) { close_conn(c); return; }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      close_conn(c);
      return;
    }
    flush(c);
  }

  void flush(GConn* c) {
    if (c->dead) return;
    while (true) {
      const uint8_t* data;
      ssize_t n = nghttp2_session_mem_send(c->session, &data);
      if (n < 0) { close_conn(c); return; }
      if (n == 0) break;
      c->out.append((const char*)data, size_t(n));
    }
    while (c->out_off < c->out.size()) {
      ssize_t w = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
      if (w > 0) { c->out_off += size_t(w); continue; }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;
      close_conn(c);
      return;
    }
    c->out.clear();
    c->out_off = 0;
    if (!nghttp2_session_want_read(c->session) && !nghttp2_session_want_write(c->session)) close_conn(c);
  }
};

GrpcServer::GrpcServer(std::shared_ptr<Engine> engine, GrpcOptions opts)
    : engine_(std::move(engine)), opts_(std::move(opts)) {}

GrpcServer::~GrpcServer() { stop(); }

void GrpcServer::start() {
  if (running_.exchange(true)) return;
  const int nthreads = std::max(1, opts_.threads);
  for (int t = 0; t < nthreads; ++t) {
    auto w = std::make_shared<Worker>();
    w->srv = this;
    nghttp2_session_callbacks_new(&w->cbs);
    nghttp2_session_callbacks_set_on_begin_headers_callback(w->cbs, Worker::on_begin_headers);
    nghttp2_session_callbacks_set_on_header_callback(w->cbs, Worker::on_header);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(w->cbs, Worker::on_data_chunk);
    nghttp2_session_callbacks_set_on_frame_recv_callback(w->cbs, Worker::on_frame_recv);
    nghttp2_session_callbacks_set_on_stream_close_callback(w->cbs, Worker::on_stream_close);
    w->epfd = epoll_create1(EPOLL_CLOEXEC);
    w->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = w->evfd;
    epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->evfd, &ev);
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(t == 0 ? opts_.port : bound_port_));
    if (inet_pton(AF_INET, opts_.host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 4096) < 0) {
      ::close(fd);
      running_.store(false);
      throw std::runtime_error("gRPC bind/listen failed on port " + std::to_string(opts_.port) + ": " + strerror(errno));
    }
    socklen_t len = sizeof a;
    getsockname(fd, (sockaddr*)&a, &len);
    if (t == 0) bound_port_ = ntohs(a.sin_port);
    w->lfd = fd;
    epoll_event lev{};
    lev.events = EPOLLIN;
    lev.data.fd = fd;
    epoll_ctl(w->epfd, EPOLL_CTL_ADD, fd, &lev);
    workers_.push_back(std::move(w));
  }
  for (auto& w : workers_) {
    Worker* raw = w.get();
    w->th = std::thread([raw] { raw->run(); });
  }
}

void GrpcServer::stop() {
  if (!running_.exchange(false)) return;
  for (auto& w : workers_) w->stop.store(true);
  for (auto& w : workers_)
    if (w->th.joinable()) w->th.join();
  workers_.clear();
}

}  // namespace sca
