#include "http_server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>

#include <deque>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <unordered_map>

namespace sca {

using Clock = std::chrono::steady_clock;

// ------------------------------------------------------------------ helpers
static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

std::string url_decode(std::string_view s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '+') o.push_back(' ');
    else if (c == '%' && i + 2 < s.size() && hexval(s[i + 1]) >= 0 && hexval(s[i + 2]) >= 0) {
      o.push_back(char(hexval(s[i + 1]) * 16 + hexval(s[i + 2])));
      i += 2;
    } else o.push_back(c);
  }
  return o;
}

bool form_value(std::string_view body, std::string_view key, std::string& out) {
  size_t pos = 0;
  while (pos <= body.size()) {
    size_t amp = body.find('&', pos);
    if (amp == std::string_view::npos) amp = body.size();
    std::string_view kv = body.substr(pos, amp - pos);
    size_t eq = kv.find('=');
    std::string_view k = kv.substr(0, eq);
    if (url_decode(k) == key) {
      out = eq == std::string_view::npos ? std::string() : url_decode(kv.substr(eq + 1));
      return true;
    }
    pos = amp + 1;
  }
  return false;
}

static inline char ascii_lower(char c) { return c >= 'A' && c <= 'Z' ? char(c | 0x20) : c; }
static bool iequals(std::string_view a, std::string_view b) {  // ASCII case folding (header names, tokens)
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (ascii_lower(a[i]) != ascii_lower(b[i])) return false;
  return true;
}

static std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

static const char* status_text(int code) {
  switch (code) {
    case 100: return "Continue";
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Unknown";
  }
}

// Parse a multipart/form-data body into the JSON object the reference builds
// (RestClientController.java:156-198): strData -> string, file parts ->
// binData (base64), other fields -> parsed JSON.
static bool multipart_to_json(std::string_view body, std::string_view boundary, Json& out, std::string& err) {
  out = Json::object();
  std::string delim = "--" + std::string(boundary);
  size_t pos = body.find(delim);
  if (pos == std::string_view::npos) { err = "multipart boundary not found"; return false; }
  pos += delim.size();
  while (true) {
    if (body.substr(pos, 2) == "--") break;
    if (body.substr(pos, 2) == "\r\n") pos += 2;
    size_t hend = body.find("\r\n\r\n", pos);
    if (hend == std::string_view::npos) { err = "bad multipart headers"; return false; }
    std::string_view headers = body.substr(pos, hend - pos);
    size_t cstart = hend + 4;
    size_t next = body.find("\r\n" + delim, cstart);
    if (next == std::string_view::npos) { err = "unterminated multipart part"; return false; }
    std::string_view content = body.substr(cstart, next - cstart);
    std::string name, filename;
    bool has_file = false;
    size_t hp = 0;
    while (hp < headers.size()) {
      size_t le = headers.find("\r\n", hp);
      if (le == std::string_view::npos) le = headers.size();
      std::string_view line = headers.substr(hp, le - hp);
      size_t colon = line.find(':');
      if (colon != std::string_view::npos && iequals(trim(line.substr(0, colon)), "content-disposition")) {
        std::string_view v = line.substr(colon + 1);
        auto grab = [&](std::string_view key, std::string& dst) {
          size_t k = v.find(key);
          while (k != std::string_view::npos && k > 0 && v[k - 1] != ' ' && v[k - 1] != ';') k = v.find(key, k + 1);
          if (k == std::string_view::npos) return false;
          size_t s = k + key.size();
          if (s < v.size() && v[s] == '"') {
            size_t e = v.find('"', s + 1);
            dst = std::string(v.substr(s + 1, e - s - 1));
          } else {
            size_t e = v.find(';', s);
            dst = std::string(trim(v.substr(s, e == std::string_view::npos ? v.size() - s : e - s)));
          }
          return true;
        };
        grab("name=", name);
        has_file = grab("filename=", filename);
      }
      hp = le + 2;
    }
    if (iequals(name, "strData")) {
      out.set(name, Json(std::string(content)));
    } else if (has_file) {
      out.set(name, Json(base64_encode(content)));
    } else {
      try {
        out.set(name, parse_json(content));
      } catch (const std::exception& e) {
        err = e.what();
        return false;
      }
    }
    pos = next + 2 + delim.size();
  }
  return true;
}

// ------------------------------------------------------------------ worker
namespace {

struct Request {
  std::string_view method, target, path, query, content_type, body;
  bool keep_alive = true;
  std::vector<std::pair<std::string, std::string>> route_headers;  // only when the engine routes on headers
};

struct Conn {
  int fd = -1;
  uint64_t gen = 0;
  std::string in;
  size_t in_off = 0;
  std::string out;
  size_t out_off = 0;
  bool busy = false;
  bool close_after = false;
  bool sent_continue = false;
  bool dead = false;
};

struct Completion {
  int fd;
  uint64_t gen;
  int status;
  std::string ctype;
  std::string body;
  bool keep_alive;
  // Deferred serialization: the I/O worker renders the outcome.
  bool has_outcome = false;
  Outcome outcome;
  int kind = 0;  // 0 external predict, 1 internal call
  const std::string* uri = nullptr;  // interned by the worker (Worker::intern)
  Clock::time_point t0;
};

enum class Route { Predict, Feedback, Internal, Other };

}  // namespace

struct HttpServer::Worker : Executor, std::enable_shared_from_this<HttpServer::Worker> {
  HttpServer* srv;
  int epfd = -1;
  int evfd = -1;
  std::vector<int> listen_fds;
  std::thread th;
  std::thread::id tid;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  uint64_t next_gen = 1;
  std::mutex qmu;
  std::vector<Completion> q;
  std::vector<std::function<void()>> tasks;  // continuations posted by GPU units
  bool running_tasks = false;               // worker thread only
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
  bool wake_pending = false;                // eventfd written and not yet drained (guarded by qmu)
  std::atomic<bool> stop{false};
  std::unordered_map<std::string, Series*> timers;
  Series* last_timer = nullptr;
  int last_status = 0;
  const std::string* last_uri = nullptr;

  ~Worker() {
    for (auto& kv : conns)
      if (!kv.second->dead) ::close(kv.first);
    for (int fd : listen_fds) ::close(fd);
    if (evfd >= 0) ::close(evfd);
    if (epfd >= 0) ::close(epfd);
  }

  // Request paths seen by this worker, interned so a request's completion
  // carries a pointer instead of two heap copies of the path.  Bounded: past
  // kMaxUris distinct paths the rest share one "other" entry (metrics label).
  static constexpr size_t kMaxUris = 64;
  std::deque<std::string> uris;
  const std::string* intern(std::string_view path) {
    for (const auto& u : uris)
      if (u == path) return &u;
    if (uris.size() >= kMaxUris) {
      static const std::string other = "other";
      return &other;
    }
    uris.emplace_back(path);
    return &uris.back();
  }

  Series* server_timer(const std::string* up, int status) {
    // hot path: the last (uri, status) seen by this worker (interned: a pointer compare)
    if (last_timer && status == last_status && up == last_uri) return last_timer;
    const std::string& uri = *up;
    std::string key = uri + "#" + std::to_string(status);
    auto it = timers.find(key);
    if (it != timers.end()) {
      last_timer = it->second;
      last_status = status;
      last_uri = up;
      return it->second;
    }
    Labels l = {{"deployment_name", srv->engine_->options().deployment_name},
                {"predictor_name", srv->engine_->spec().name.empty() ? "unknown" : srv->engine_->spec().name},
                {"predictor_version", [&] {
                   auto v = srv->engine_->spec().labels.find("version");
                   return v == srv->engine_->spec().labels.end() || v->second.empty() ? std::string("unknown") : v->second;
                 }()},
                {"exception", "None"},
                {"method", "POST"},
                {"status", std::to_string(status)},
                {"uri", uri}};
    Series* s = srv->engine_->metrics().timer("seldon_api_engine_server_requests", std::move(l), true);
    timers.emplace(key, s);
    last_timer = s;
    last_status = status;
    last_uri = up;
    return s;
  }

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
      int n = 0;
      if (srv->spin_us_ > 0) {  // poll briefly before sleeping: the next request usually arrives within microseconds
        polling.store(false, std::memory_order_relaxed);
        const auto until = Clock::now() + std::chrono::microseconds(srv->spin_us_);
        do {
          n = epoll_wait(epfd, evs, 256, 0);
        } while (n == 0 && !has_work.load(std::memory_order_acquire) && Clock::now() < until);
        if (n == 0 && has_work.load(std::memory_order_acquire)) continue;
        if (n == 0) {
          polling.store(true, std::memory_order_seq_cst);
          if (has_work.load(std::memory_order_seq_cst)) {
            polling.store(false, std::memory_order_relaxed);
            continue;
          }
          n = epoll_wait(epfd, evs, 256, 200);
        }
      } else {
        n = epoll_wait(epfd, evs, 256, 200);
      }
      polling.store(false, std::memory_order_relaxed);
      for (int i = 0; i < n; ++i) {
        int fd = evs[i].data.fd;
        uint32_t e = evs[i].events;
        if (fd == evfd) { drain_queue(true); continue; }
        bool is_listen = false;
        for (int lf : listen_fds)
          if (lf == fd) { is_listen = true; break; }
        if (is_listen) { accept_all(fd); continue; }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn* c = it->second.get();
        if (e & (EPOLLERR | EPOLLHUP)) { close_conn(c); continue; }
        if (e & EPOLLIN) on_readable(c);
        if (c->dead) { reap(fd); continue; }
        if (e & EPOLLOUT) flush(c);
        if (c->dead) reap(fd);
      }
    }
  }

  void accept_all(int lfd) {
    while (true) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->gen = next_gen++;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLET | EPOLLRDHUP;
      ev.data.fd = fd;
      epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &ev);
      conns[fd] = std::move(c);
    }
  }

  void close_conn(Conn* c) {
    if (c->dead) return;
    c->dead = true;
    epoll_ctl(epfd, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
  }
  void reap(int fd) { conns.erase(fd); }

  void on_readable(Conn* c) {
    char buf[65536];
    while (true) {
      ssize_t r = ::read(c->fd, buf, sizeof buf);
      if (r > 0) {
        if (c->in_off > 0 && c->in_off == c->in.size()) { c->in.clear(); c->in_off = 0; }
        c->in.append(buf, size_t(r));
        // A short read drained the socket: edge-triggered epoll reports the
        // next arrival (or the peer's FIN), so skip the read that would
        // only return EAGAIN -- one syscall less per request.
        if (size_t(r) < sizeof buf) break;
        continue;
      }
      if (r == 0) {  // peer closed: finish in-flight work, then close
        if (!c->busy && c->out_off == c->out.size()) { close_conn(c); return; }
        c->close_after = true;
        break;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      close_conn(c);
      return;
    }
    process(c);
  }

  void flush(Conn* c) {
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
    if (c->close_after && !c->busy) close_conn(c);
  }

  void write_response(Conn* c, int status, std::string_view ctype, std::string_view body, bool keep_alive) {
    std::string& o = c->out;
    o += "HTTP/1.1 ";
    o += std::to_string(status);
    o.push_back(' ');
    o += status_text(status);
    o += "\r\nContent-Type: ";
    o += ctype;
    o += "\r\nAccess-Control-Allow-Origin: *\r\nContent-Length: ";
    o += std::to_string(body.size());
    o += keep_alive ? "\r\n\r\n" : "\r\nConnection: close\r\n\r\n";
    o.append(body.data(), body.size());
    if (!keep_alive) c->close_after = true;
    srv->served_.fetch_add(1, std::memory_order_relaxed);
  }

  // Parse as many complete requests as possible (one in flight at a time).
  // Nothing thrown while parsing one client's bytes may reach the epoll loop:
  // answer 400 and drop that connection instead.
  void process(Conn* c) {
    try {
      process_requests(c);
    } catch (const std::exception& e) {
      if (c->dead) return;
      c->busy = false;
      c->in.clear();
      c->in_off = 0;
      write_response(c, 400, "text/plain", std::string("bad request: ") + e.what(), false);
      flush(c);
    }
  }

  void process_requests(Conn* c) {
    while (!c->busy && !c->dead) {
      std::string_view buf(c->in.data() + c->in_off, c->in.size() - c->in_off);
      if (buf.empty()) break;
      size_t hend = buf.find("\r\n\r\n");
      if (hend == std::string_view::npos) {
        if (buf.size() > 65536) { write_response(c, 431, "text/plain", "header too large", false); }
        break;
      }
      Request rq;
      std::string_view head = buf.substr(0, hend);
      size_t le = head.find("\r\n");
      std::string_view line = head.substr(0, le);
      size_t s1 = line.find(' ');
      size_t s2 = line.find(' ', s1 + 1);
      if (s1 == std::string_view::npos || s2 == std::string_view::npos) {
        write_response(c, 400, "text/plain", "bad request line", false);
        break;
      }
      rq.method = line.substr(0, s1);
      rq.target = line.substr(s1 + 1, s2 - s1 - 1);
      std::string_view version = line.substr(s2 + 1);
      rq.keep_alive = version != "HTTP/1.0";
      size_t qm = rq.target.find('?');
      rq.path = rq.target.substr(0, qm);
      if (qm != std::string_view::npos) rq.query = rq.target.substr(qm + 1);
      size_t content_length = 0;
      bool chunked = false, expect_continue = false;
      size_t hp = le == std::string_view::npos ? head.size() : le + 2;
      while (hp < head.size()) {
        size_t e = head.find("\r\n", hp);
        if (e == std::string_view::npos) e = head.size();
        std::string_view h = head.substr(hp, e - hp);
        size_t colon = h.find(':');
        if (colon != std::string_view::npos) {
          std::string_view name = h.substr(0, colon), val = trim(h.substr(colon + 1));
          if (iequals(name, "content-length")) content_length = size_t(strtoull(std::string(val).c_str(), nullptr, 10));
          else if (iequals(name, "transfer-encoding")) chunked = val.find("chunked") != std::string_view::npos;
          else if (iequals(name, "connection")) {
            if (iequals(val, "close")) rq.keep_alive = false;
            else if (iequals(val, "keep-alive")) rq.keep_alive = true;
          } else if (iequals(name, "content-type")) rq.content_type = val;
          else if (iequals(name, "expect")) expect_continue = iequals(val, "100-continue");
          else if (srv->engine_->has_header_routes() && srv->engine_->is_route_header(name))
            rq.route_headers.emplace_back(std::string(name), std::string(val));
        }
        hp = e + 2;
      }
      size_t body_start = hend + 4;
      std::string chunk_body;
      size_t consumed;
      if (chunked) {
        size_t p = body_start;
        bool complete = false;
        bool bad = false, too_large = false;
        while (true) {
          size_t ce = buf.find("\r\n", p);
          if (ce == std::string_view::npos) break;
          // chunk-size = 1*HEXDIG [ ";" chunk-ext ]; reject anything else and
          // compare without adding to the untrusted size (no wrap-around).
          std::string_view szs = buf.substr(p, ce - p);
          size_t semi = szs.find(';');
          if (semi != std::string_view::npos) szs = szs.substr(0, semi);
          szs = trim(szs);
          if (szs.empty() || szs.size() > 15 ||
              szs.find_first_not_of("0123456789abcdefABCDEF") != std::string_view::npos) { bad = true; break; }
          size_t sz = size_t(strtoull(std::string(szs).c_str(), nullptr, 16));
          if (sz > srv->opts_.max_body || chunk_body.size() > srv->opts_.max_body - sz) { too_large = true; break; }
          if (sz == 0) {
            size_t te = buf.find("\r\n", ce + 2);
            if (te == std::string_view::npos) break;
            p = te + 2;
            complete = true;
            break;
          }
          if (buf.size() - (ce + 2) < sz + 2) break;
          if (buf.substr(ce + 2 + sz, 2) != "\r\n") { bad = true; break; }
          chunk_body.append(buf.data() + ce + 2, sz);
          p = ce + 2 + sz + 2;
        }
        if (bad) { write_response(c, 400, "text/plain", "bad chunked encoding", false); break; }
        if (too_large) { write_response(c, 413, "text/plain", "payload too large", false); break; }
        if (!complete) {
          // an incomplete chunked body may not grow past the body limit
          if (buf.size() - body_start > srv->opts_.max_body + 65536) {
            write_response(c, 413, "text/plain", "payload too large", false);
            break;
          }
          if (expect_continue && !c->sent_continue) { c->out += "HTTP/1.1 100 Continue\r\n\r\n"; c->sent_continue = true; flush(c); }
          break;
        }
        consumed = p;
        rq.body = chunk_body;
      } else {
        if (content_length > srv->opts_.max_body) { write_response(c, 413, "text/plain", "payload too large", false); break; }
        if (buf.size() < body_start + content_length) {
          if (expect_continue && !c->sent_continue) { c->out += "HTTP/1.1 100 Continue\r\n\r\n"; c->sent_continue = true; flush(c); }
          break;
        }
        rq.body = buf.substr(body_start, content_length);
        consumed = body_start + content_length;
      }
      c->sent_continue = false;
      // The request views point into c->in; handle() must finish using them
      // before c->in is modified (it copies what async work needs).
      handle(c, rq);
      c->in_off += consumed;
      if (c->in_off == c->in.size()) { c->in.clear(); c->in_off = 0; }
    }
    if (!c->dead) flush(c);
  }

  void respond_now(Conn* c, int status, std::string_view ctype, std::string_view body, bool keep_alive) {
    write_response(c, status, ctype, body, keep_alive);
  }

  // Extract the SeldonMessage JSON text from an internal-API request.
  bool internal_payload(const Request& rq, std::string& json_text, std::string& err) {
    if (rq.content_type.find("application/x-www-form-urlencoded") != std::string_view::npos) {
      if (form_value(rq.body, "json", json_text)) return true;
    }
    if (rq.content_type.find("multipart/form-data") != std::string_view::npos) {
      size_t b = rq.content_type.find("boundary=");
      Json obj;
      if (b == std::string_view::npos || !multipart_to_json(rq.body, rq.content_type.substr(b + 9), obj, err)) return false;
      json_text = obj.dump();
      return true;
    }
    if (!rq.query.empty() && form_value(rq.query, "json", json_text)) return true;
    if (!rq.body.empty()) { json_text = std::string(rq.body); return true; }
    err = "Empty json parameter in data";
    return false;
  }

  void handle(Conn* c, const Request& rq) {
    std::string_view p = rq.path;
    // Gateway-style paths (Ambassador/Istio prefix routing, reference
    // operator/controllers/ambassador.go:81): /seldon/[<ns>/]<sdep>/api/...
    if (p.rfind("/seldon/", 0) == 0) {
      const size_t api = p.find("/api/");
      if (api != std::string_view::npos) p = p.substr(api);
    }
    Engine& eng = *srv->engine_;
    if (p == "/api/v0.1/predictions" || p == "/api/v1.0/predictions") { predict_external(c, rq); return; }
    if (p == "/api/v0.1/feedback" || p == "/api/v1.0/feedback") { feedback_external(c, rq); return; }
    if (p == "/ping") { respond_now(c, 200, "text/plain", "pong", rq.keep_alive); return; }
    if (p == "/live") { respond_now(c, 200, "text/plain", "live", rq.keep_alive); return; }
    if (p == "/ready") {
      bool ok = !srv->paused_.load() && eng.ready();
      respond_now(c, ok ? 200 : 503, "text/plain", ok ? "ready" : "Service unavailable", rq.keep_alive);
      return;
    }
    if (p == "/pause") { srv->paused_.store(true); respond_now(c, 200, "text/plain", "paused", rq.keep_alive); return; }
    if (p == "/unpause") { srv->paused_.store(false); respond_now(c, 200, "text/plain", "unpaused", rq.keep_alive); return; }
    if (p == "/prometheus" || p == "/metrics") {
      std::string body = eng.render_metrics();
      respond_now(c, 200, "text/plain; version=0.0.4", body, rq.keep_alive);
      return;
    }
    if (p == "/") { respond_now(c, 200, "text/plain", "Hello World!!", rq.keep_alive); return; }
    if (srv->opts_.internal_api) {
      if (p == "/seldon.json") {
        respond_now(c, 200, "application/json", srv->opts_.openapi_json.empty() ? "{}" : srv->opts_.openapi_json, rq.keep_alive);
        return;
      }
      int m = 0;
      bool internal = true;
      if (p == "/predict") m = Engine::kPredictMethod;
      else if (p == "/transform-input") m = int(Method::TRANSFORM_INPUT);
      else if (p == "/transform-output") m = int(Method::TRANSFORM_OUTPUT);
      else if (p == "/route") m = int(Method::ROUTE);
      else if (p == "/aggregate") m = int(Method::AGGREGATE);
      else if (p == "/send-feedback") m = int(Method::SEND_FEEDBACK);
      else internal = false;
      if (internal) { internal_call(c, rq, m); return; }
    }
    respond_now(c, 404, "text/plain", "not found", rq.keep_alive);
  }

  // Engine continuation -> this worker (inline when already on it).
  void deliver(Completion&& done) {
    if (std::this_thread::get_id() == tid && running_tasks) {  // finish after the task batch (may resume the conn)
      std::lock_guard<std::mutex> g(qmu);
      q.push_back(std::move(done));
      return;
    }
    if (std::this_thread::get_id() == tid) {
      auto it = conns.find(done.fd);
      if (it != conns.end() && it->second->gen == done.gen && !it->second->dead) finish(it->second.get(), std::move(done), false);
      return;
    }
    bool wake;
    {
      std::lock_guard<std::mutex> g(qmu);
      q.push_back(std::move(done));
      wake = need_wake();
    }
    if (wake) {  // one wakeup per drained batch of completions
      uint64_t one = 1;
      ssize_t w = ::write(evfd, &one, 8);
      (void)w;
    }
  }

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

  void drain_queue(bool evfd_ready) {
    if (evfd_ready) {
      uint64_t v;
      ssize_t r = ::read(evfd, &v, 8);
      (void)r;
    }
    std::vector<Completion> items;
    std::vector<std::function<void()>> run;
    {
      std::lock_guard<std::mutex> g(qmu);
      if (evfd_ready) wake_pending = false;  // anything queued from now on signals again
      has_work.store(false, std::memory_order_relaxed);
      items.swap(q);
      run.swap(tasks);
    }
    running_tasks = true;
    for (auto& fn : run) fn();  // completions they produce are queued in q
    running_tasks = false;
    {
      std::lock_guard<std::mutex> g(qmu);  // completions queued by other threads meanwhile
      for (auto& d : q) items.push_back(std::move(d));
      q.clear();
    }
    for (auto& d : items) {
      auto it = conns.find(d.fd);
      if (it == conns.end() || it->second->gen != d.gen || it->second->dead) continue;
      Conn* c = it->second.get();
      finish(c, std::move(d), true);
      if (c->dead) reap(c->fd);
    }
  }

  void finish(Conn* c, Completion&& d, bool resume) {
    if (d.has_outcome) {
      std::string body;
      int status = 200;
      if (d.outcome.err) {
        if (!d.outcome.err->body.empty()) {  // the component's own status + body (wrapper.py:22-31)
          status = d.outcome.err->http_status;
          body = d.outcome.err->body;
        } else if (d.kind == 1) {  // wrapper-style error (flask_utils.py:67-82)
          status = 400;
          body = "{\"status\":{\"status\":1,\"info\":";
          append_quoted(body, d.outcome.err->info);
          body += ",\"code\":-1,\"reason\":\"MICROSERVICE_BAD_DATA\"}}";
        } else {
          status = d.outcome.err->http_status;
          body = error_to_json(*d.outcome.err);
        }
      } else if (d.outcome.msg) {
        body.reserve(512);
        message_to_json(*d.outcome.msg, body);
      } else {
        body = "{}";
      }
      if (d.kind == 0 && d.uri) server_timer(d.uri, status)->observe_seconds(std::chrono::duration<double>(Clock::now() - d.t0).count());
      write_response(c, status, "application/json", body, d.keep_alive);
    } else {
      if (d.kind == 0 && d.uri)
        server_timer(d.uri, d.status)->observe_seconds(std::chrono::duration<double>(Clock::now() - d.t0).count());
      write_response(c, d.status, d.ctype, d.body, d.keep_alive);
    }
    c->busy = false;
    if (resume) process(c);
  }

  bool parse_external_body(const Request& rq, Json& out, std::string& err) {
    try {
      if (rq.content_type.find("multipart/form-data") != std::string_view::npos) {
        size_t b = rq.content_type.find("boundary=");
        if (b == std::string_view::npos) { err = "missing multipart boundary"; return false; }
        std::string_view bd = rq.content_type.substr(b + 9);
        if (!bd.empty() && bd.front() == '"') bd = bd.substr(1, bd.find('"', 1) - 1);
        return multipart_to_json(rq.body, bd, out, err);
      }
      if (rq.content_type.find("application/x-www-form-urlencoded") != std::string_view::npos) {
        std::string j;
        if (form_value(rq.body, "json", j)) { out = parse_json(j); return true; }
      }
      if (rq.body.empty() && !rq.query.empty()) {
        std::string j;
        if (form_value(rq.query, "json", j)) { out = parse_json(j); return true; }
      }
      out = parse_json(rq.body);
      return true;
    } catch (const std::exception& e) {
      err = e.what();
      return false;
    }
  }

  void predict_external(Conn* c, const Request& rq) {
    const auto t0 = Clock::now();
    const std::string* uri = intern(rq.path);
    auto msg = std::make_shared<SeldonMessage>();
    Json j;
    std::string err;
    bool ok;
    static const bool fast = [] { const char* v = getenv("SCA_REST_FAST_JSON"); return !v || atoi(v) != 0; }();
    if (fast && !rq.body.empty() && rq.content_type.find("form") == std::string_view::npos &&
        fast_dense_message(rq.body, *msg)) {
      ok = true;  // dense ndarray request parsed without a JSON tree
    } else if ((ok = parse_external_body(rq, j, err))) {
      try {
        message_from_json(j, *msg);
      } catch (const std::exception& e) {
        ok = false;
        err = e.what();
      }
    }
    if (!ok) {
      auto e = make_error(ApiError::INVALID_JSON, std::string(rq.body));
      Completion d{c->fd, c->gen, e->http_status, "application/json", error_to_json(*e), rq.keep_alive};
      d.uri = uri;
      d.t0 = t0;
      c->busy = true;
      finish(c, std::move(d), false);
      return;
    }
    c->busy = true;
    int fd = c->fd;
    uint64_t gen = c->gen;
    bool ka = rq.keep_alive;
    auto self = shared_from_this();
    Done done = [self, fd, gen, ka, uri, t0](Outcome o) {
      Completion d{fd, gen, 200, "", "", ka};
      d.has_outcome = true;
      d.outcome = std::move(o);
      d.kind = 0;
      d.uri = uri;
      d.t0 = t0;
      self->deliver(std::move(d));
    };
    if (!rq.route_headers.empty()) srv->engine_->predict_with_headers(msg, std::move(done), self, rq.route_headers);
    else srv->engine_->predict(msg, std::move(done), self);
  }

  void feedback_external(Conn* c, const Request& rq) {
    const auto t0 = Clock::now();
    const std::string* uri = intern(rq.path);
    auto fb = std::make_shared<Feedback>();
    try {
      Json j = parse_json(rq.body);
      feedback_from_json(j, *fb);
    } catch (const std::exception&) {
      auto e = make_error(ApiError::INVALID_JSON, std::string(rq.body));
      Completion d{c->fd, c->gen, e->http_status, "application/json", error_to_json(*e), rq.keep_alive};
      d.uri = uri;
      d.t0 = t0;
      c->busy = true;
      finish(c, std::move(d), false);
      return;
    }
    c->busy = true;
    int fd = c->fd;
    uint64_t gen = c->gen;
    bool ka = rq.keep_alive;
    srv->engine_->send_feedback(fb, [self = shared_from_this(), fd, gen, ka, uri, t0](ErrPtr e) {
      Completion d{fd, gen, e ? e->http_status : 200, "application/json", e ? error_to_json(*e) : "{}", ka};
      d.uri = uri;
      d.t0 = t0;
      self->deliver(std::move(d));
    });
  }

  void internal_call(Conn* c, const Request& rq, int m) {
    std::string text, err;
    auto bad = [&](const std::string& info) {
      std::string body = "{\"status\":{\"status\":1,\"info\":";
      append_quoted(body, info);
      body += ",\"code\":-1,\"reason\":\"MICROSERVICE_BAD_DATA\"}}";
      respond_now(c, 400, "application/json", body, rq.keep_alive);
    };
    if (!internal_payload(rq, text, err)) { bad(err); return; }
    std::string node = srv->opts_.microservice_node.empty() ? srv->engine_->spec().graph.name : srv->opts_.microservice_node;
    int fd = c->fd;
    uint64_t gen = c->gen;
    bool ka = rq.keep_alive;
    auto cb = [self = shared_from_this(), fd, gen, ka](Outcome o) {
      Completion d{fd, gen, 200, "", "", ka};
      d.has_outcome = true;
      d.outcome = std::move(o);
      d.kind = 1;
      self->deliver(std::move(d));
    };
    try {
      Json j = parse_json(text);
      if (m == int(Method::SEND_FEEDBACK)) {
        auto fb = std::make_shared<Feedback>();
        feedback_from_json(j, *fb);
        c->busy = true;
        srv->engine_->send_feedback(fb, [cb](ErrPtr e) {
          if (e) cb(Outcome::fail(e));
          else {
            auto empty = std::make_shared<SeldonMessage>();
            cb(Outcome::ok(empty));
          }
        });
        return;
      }
      std::vector<MsgPtr> in;
      if (m == int(Method::AGGREGATE)) {
        std::vector<SeldonMessage> list;
        message_list_from_json(j, list);
        for (auto& x : list) in.push_back(std::make_shared<SeldonMessage>(std::move(x)));
      } else {
        auto msg = std::make_shared<SeldonMessage>();
        message_from_json(j, *msg);
        in.push_back(msg);
      }
      c->busy = true;
      srv->engine_->call_node(node, m, std::move(in), cb);
    } catch (const std::exception& e) {
      c->busy = false;
      bad(e.what());
    }
  }
};

// ------------------------------------------------------------------ server
static int make_listener(const std::string& host, int port, int* bound_port) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(fd, (sockaddr*)&a, sizeof a) < 0) {
    ::close(fd);
    throw std::runtime_error("bind() failed on port " + std::to_string(port) + ": " + strerror(errno));
  }
  if (listen(fd, 4096) < 0) {
    ::close(fd);
    throw std::runtime_error("listen() failed");
  }
  socklen_t len = sizeof a;
  getsockname(fd, (sockaddr*)&a, &len);
  *bound_port = ntohs(a.sin_port);
  return fd;
}

HttpServer::HttpServer(std::shared_ptr<Engine> engine, HttpOptions opts)
    : engine_(std::move(engine)), opts_(std::move(opts)) {
  if (const char* e = std::getenv("SCA_HTTP_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
}

HttpServer::~HttpServer() { stop(); }

void HttpServer::start() {
  if (running_.exchange(true)) return;
  int nthreads = std::max(1, opts_.threads);
  bound_ports_.assign(opts_.ports.size(), 0);
  for (int t = 0; t < nthreads; ++t) {
    auto w = std::make_shared<Worker>();
    w->srv = this;
    w->epfd = epoll_create1(EPOLL_CLOEXEC);
    w->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = w->evfd;
    epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->evfd, &ev);
    for (size_t p = 0; p < opts_.ports.size(); ++p) {
      int want = t == 0 ? opts_.ports[p] : bound_ports_[p];
      int got = 0;
      int lfd = make_listener(opts_.host, want, &got);
      if (t == 0) bound_ports_[p] = got;
      epoll_event lev{};
      lev.events = EPOLLIN;
      lev.data.fd = lfd;
      epoll_ctl(w->epfd, EPOLL_CTL_ADD, lfd, &lev);
      w->listen_fds.push_back(lfd);
    }
    workers_.push_back(std::move(w));
  }
  for (auto& w : workers_) {
    Worker* raw = w.get();
    w->th = std::thread([raw] { raw->run(); });
  }
}

void HttpServer::stop() {
  if (!running_.exchange(false)) return;
  for (auto& w : workers_) w->stop.store(true);
  for (auto& w : workers_)
    if (w->th.joinable()) w->th.join();
  workers_.clear();
}

}  // namespace sca
