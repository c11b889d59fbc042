#include "remote_unit.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <unordered_map>

#include "http_server.h"

namespace sca {

namespace {

struct NetError : std::runtime_error {
  bool connect_failure;
  NetError(const std::string& m, bool c) : std::runtime_error(m), connect_failure(c) {}
};

struct RemoteUserError : std::runtime_error {
  int status;
  std::string body;
  RemoteUserError(int s, std::string b)
      : std::runtime_error("Bad return code " + std::to_string(s) + ": " + b), status(s), body(std::move(b)) {}
};

int connect_timeout(const std::string& host, int port, int connect_ms, int io_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw NetError("cannot resolve " + host, true);
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  int rc = connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc < 0 && errno != EINPROGRESS) {
    ::close(fd);
    throw NetError("connect to " + host + ":" + std::to_string(port) + " failed: " + strerror(errno), true);
  }
  if (rc < 0) {
    pollfd p{fd, POLLOUT, 0};
    if (poll(&p, 1, connect_ms) <= 0) {
      ::close(fd);
      throw NetError("connect timeout to " + host + ":" + std::to_string(port), true);
    }
    int err = 0;
    socklen_t len = sizeof err;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err) {
      ::close(fd);
      throw NetError("connect to " + host + ":" + std::to_string(port) + " failed: " + strerror(err), true);
    }
  }
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) & ~O_NONBLOCK);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  timeval tv{io_ms / 1000, (io_ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  return fd;
}

void write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w <= 0) {
      if (w < 0 && errno == EINTR) continue;
      throw NetError("send failed", false);
    }
    p += w;
    n -= size_t(w);
  }
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  o.reserve(s.size() * 3 / 2);
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') o.push_back(char(c));
    else { o.push_back('%'); o.push_back(hex[c >> 4]); o.push_back(hex[c & 15]); }
  }
  return o;
}

// One keep-alive REST connection per (thread, endpoint).
thread_local std::unordered_map<std::string, int> tl_rest;

// Synchronous h2c client session per (thread, endpoint).
struct H2Client {
  int fd = -1;
  nghttp2_session* s = nullptr;
  std::string body;
  int grpc_status = -1;
  std::string grpc_message;
  bool closed = false;
  std::string req;
  size_t req_off = 0;
  ~H2Client() {
    if (s) nghttp2_session_del(s);
    if (fd >= 0) ::close(fd);
  }
};
thread_local std::unordered_map<std::string, std::unique_ptr<H2Client>> tl_h2;

int h2_on_data(nghttp2_session*, uint8_t, int32_t, const uint8_t* d, size_t n, void* ud) {
  static_cast<H2Client*>(ud)->body.append((const char*)d, n);
  return 0;
}
int h2_on_header(nghttp2_session*, const nghttp2_frame*, const uint8_t* name, size_t nl, const uint8_t* v, size_t vl,
                 uint8_t, void* ud) {
  auto* c = static_cast<H2Client*>(ud);
  std::string_view n((const char*)name, nl);
  if (n == "grpc-status") c->grpc_status = atoi(std::string((const char*)v, vl).c_str());
  else if (n == "grpc-message") c->grpc_message = url_decode(std::string_view((const char*)v, vl));
  return 0;
}
int h2_on_close(nghttp2_session*, int32_t, uint32_t, void* ud) {
  static_cast<H2Client*>(ud)->closed = true;
  return 0;
}
ssize_t h2_read(nghttp2_session*, int32_t, uint8_t* buf, size_t len, uint32_t* flags, nghttp2_data_source* src, void*) {
  auto* c = static_cast<H2Client*>(src->ptr);
  size_t n = std::min(len, c->req.size() - c->req_off);
  memcpy(buf, c->req.data() + c->req_off, n);
  c->req_off += n;
  if (c->req_off == c->req.size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
  return ssize_t(n);
}

void h2_pump_out(H2Client& c) {
  const uint8_t* data;
  ssize_t n;
  while ((n = nghttp2_session_mem_send(c.s, &data)) > 0) write_all(c.fd, (const char*)data, size_t(n));
  if (n < 0) throw NetError("h2 send error", false);
}

const char* grpc_service_for(const std::string& type) {
  if (type == "MODEL") return "Model";
  if (type == "ROUTER") return "Router";
  if (type == "TRANSFORMER") return "Transformer";
  if (type == "OUTPUT_TRANSFORMER") return "OutputTransformer";
  if (type == "COMBINER") return "Combiner";
  return "Generic";
}

}  // namespace

RemoteUnit::RemoteUnit(RemoteOptions o) : opts_(std::move(o)) {
  const int n = std::max(1, opts_.threads);
  for (int i = 0; i < n; ++i)
    workers_.emplace_back([this] {
      while (true) {
        std::function<void()> t;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return !tasks_.empty() || !running_.load(); });
          if (tasks_.empty()) {
            for (auto& kv : tl_rest) ::close(kv.second);
            tl_rest.clear();
            tl_h2.clear();
            return;
          }
          t = std::move(tasks_.front());
          tasks_.pop_front();
        }
        t();
      }
    });
  prober_ = std::thread([this] { probe_loop(); });
}

RemoteUnit::~RemoteUnit() {
  running_.store(false);
  cv_.notify_all();
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  if (prober_.joinable()) prober_.join();
}

void RemoteUnit::probe_loop() {
  while (running_.load()) {
    bool ok = false;
    for (int i = 0; i < 3 && !ok; ++i) {
      try {
        int fd = connect_timeout(opts_.host, opts_.port, 500, 500);
        ::close(fd);
        ok = true;
      } catch (...) {
      }
    }
    reachable_.store(ok);
    for (int i = 0; i < 50 && running_.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
}

bool RemoteUnit::ready() const { return reachable_.load(); }

void RemoteUnit::submit(std::function<void()> task) {
  {
    std::lock_guard<std::mutex> g(mu_);
    tasks_.push_back(std::move(task));
  }
  cv_.notify_one();
}

std::string RemoteUnit::call_rest(const std::string& path, const std::string& json_body) {
  const std::string key = opts_.host + ":" + std::to_string(opts_.port);
  const std::string form = "json=" + url_encode(json_body) + "&isDefault=false";
  std::string req = "POST /" + path + " HTTP/1.1\r\nHost: " + key +
                    "\r\nContent-Type: application/x-www-form-urlencoded\r\nSeldon-model-name: " + opts_.model_name +
                    "\r\nSeldon-model-image: " + opts_.model_image + "\r\nSeldon-model-version: " + opts_.model_version +
                    "\r\nContent-Length: " + std::to_string(form.size()) + "\r\n\r\n" + form;
  std::string last_err;
  for (int attempt = 0; attempt < std::max(1, opts_.retries) + 1; ++attempt) {
    int fd = -1;
    bool reused = false;
    try {
      auto it = tl_rest.find(key);
      if (it != tl_rest.end()) { fd = it->second; reused = true; }
      else {
        fd = connect_timeout(opts_.host, opts_.port, opts_.connect_timeout_ms, opts_.read_timeout_ms);
        tl_rest[key] = fd;
      }
      write_all(fd, req.data(), req.size());
      std::string in;
      char buf[16384];
      size_t hend;
      while ((hend = in.find("\r\n\r\n")) == std::string::npos) {
        ssize_t r = ::recv(fd, buf, sizeof buf, 0);
        if (r <= 0) throw NetError(r == 0 ? "connection closed" : "read timeout", false);
        in.append(buf, size_t(r));
      }
      const int status = atoi(in.c_str() + 9);
      std::string head = in.substr(0, hend);
      for (auto& ch : head) ch = char(tolower(ch));
      size_t cl = 0;
      bool chunked = head.find("transfer-encoding: chunked") != std::string::npos;
      size_t p = head.find("content-length:");
      if (p != std::string::npos) cl = size_t(strtoull(head.c_str() + p + 15, nullptr, 10));
      std::string body = in.substr(hend + 4);
      if (chunked) {
        std::string out;
        while (true) {
          size_t le;
          while ((le = body.find("\r\n")) == std::string::npos) {
            ssize_t r = ::recv(fd, buf, sizeof buf, 0);
            if (r <= 0) throw NetError("connection closed", false);
            body.append(buf, size_t(r));
          }
          size_t sz = strtoull(body.substr(0, le).c_str(), nullptr, 16);
          while (body.size() < le + 2 + sz + 2) {
            ssize_t r = ::recv(fd, buf, sizeof buf, 0);
            if (r <= 0) throw NetError("connection closed", false);
            body.append(buf, size_t(r));
          }
          if (sz == 0) break;
          out.append(body, le + 2, sz);
          body.erase(0, le + 2 + sz + 2);
        }
        body.swap(out);
      } else {
        while (body.size() < cl) {
          ssize_t r = ::recv(fd, buf, sizeof buf, 0);
          if (r <= 0) throw NetError("connection closed", false);
          body.append(buf, size_t(r));
        }
        body.resize(cl);
      }
      if (head.find("connection: close") != std::string::npos) {
        ::close(fd);
        tl_rest.erase(key);
      }
      if (status < 200 || status >= 300) {
        // A component's own error reply (a JSON object, e.g. its
        // model_error_handler's body) travels back to the client with its
        // status; anything else is the reference's "Bad return code"
        // (InternalPredictionService.java:426-427).
        bool obj = false;
        try {
          obj = parse_json(body).is_object();
        } catch (const std::exception&) {
        }
        if (obj) throw RemoteUserError(status, body);
        throw std::runtime_error("Bad return code " + std::to_string(status) + ": " + body);
      }
      return body;
    } catch (const NetError& e) {
      if (fd >= 0) {
        ::close(fd);
        tl_rest.erase(key);
      }
      last_err = e.what();
      if (reused) { --attempt; continue; }  // stale keep-alive connection: not a retry
      if (!e.connect_failure) break;        // reference retries only resource-access errors
    }
  }
  throw std::runtime_error("Failed to retrieve predictions from " + key + ": " + last_err);
}

std::string RemoteUnit::call_grpc(const std::string& method, const std::string& pb_body) {
  const std::string key = opts_.host + ":" + std::to_string(opts_.port);
  const std::string path = std::string("/seldon.protos.") + grpc_service_for(opts_.node_type) + "/" + method;
  for (int attempt = 0; attempt < 2; ++attempt) {
    auto& slot = tl_h2[key];
    try {
      if (!slot) {
        slot = std::make_unique<H2Client>();
        slot->fd = connect_timeout(opts_.host, opts_.port, opts_.connect_timeout_ms, opts_.read_timeout_ms);
        nghttp2_session_callbacks* cbs;
        nghttp2_session_callbacks_new(&cbs);
        nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, h2_on_data);
        nghttp2_session_callbacks_set_on_header_callback(cbs, h2_on_header);
        nghttp2_session_callbacks_set_on_stream_close_callback(cbs, h2_on_close);
        nghttp2_session_client_new(&slot->s, cbs, slot.get());
        nghttp2_session_callbacks_del(cbs);
        nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16 << 20}};
        nghttp2_submit_settings(slot->s, NGHTTP2_FLAG_NONE, iv, 1);
        nghttp2_session_set_local_window_size(slot->s, NGHTTP2_FLAG_NONE, 0, 256 << 20);
      }
      H2Client& c = *slot;
      c.body.clear();
      c.grpc_status = -1;
      c.grpc_message.clear();
      c.closed = false;
      c.req.assign(1, '\0');
      const uint32_t n = htonl(uint32_t(pb_body.size()));
      c.req.append((const char*)&n, 4);
      c.req += pb_body;
      c.req_off = 0;
      const std::string auth = key;
      nghttp2_nv hdrs[] = {
          {(uint8_t*)":method", (uint8_t*)"POST", 7, 4, 0},
          {(uint8_t*)":scheme", (uint8_t*)"http", 7, 4, 0},
          {(uint8_t*)":path", (uint8_t*)path.c_str(), 5, path.size(), 0},
          {(uint8_t*)":authority", (uint8_t*)auth.c_str(), 10, auth.size(), 0},
          {(uint8_t*)"content-type", (uint8_t*)"application/grpc", 12, 16, 0},
          {(uint8_t*)"te", (uint8_t*)"trailers", 2, 8, 0},
      };
      nghttp2_data_provider prd;
      prd.source.ptr = &c;
      prd.read_callback = h2_read;
      if (nghttp2_submit_request(c.s, nullptr, hdrs, 6, &prd, nullptr) < 0) throw NetError("submit failed", false);
      h2_pump_out(c);
      uint8_t buf[65536];
      while (!c.closed) {
        ssize_t r = ::recv(c.fd, buf, sizeof buf, 0);
        if (r <= 0) throw NetError(r == 0 ? "connection closed" : "read timeout", false);
        if (nghttp2_session_mem_recv(c.s, buf, size_t(r)) < 0) throw NetError("h2 protocol error", false);
        h2_pump_out(c);
      }
      if (c.grpc_status != 0)
        throw std::runtime_error("gRPC status " + std::to_string(c.grpc_status) + ": " + c.grpc_message);
      if (c.body.size() < 5) return std::string();
      uint32_t len;
      memcpy(&len, c.body.data() + 1, 4);
      len = ntohl(len);
      return c.body.substr(5, len);
    } catch (const NetError& e) {
      tl_h2.erase(key);
      if (attempt == 1) throw std::runtime_error(std::string("gRPC call to ") + key + " failed: " + e.what());
    }
  }
  throw std::runtime_error("unreachable");
}

void RemoteUnit::call_message(const char* rest_path, const char* grpc_method, MsgPtr in, Done k) {
  std::string rp = rest_path, gm = grpc_method;
  submit([this, rp, gm, in, k]() {
    try {
      auto m = std::make_shared<SeldonMessage>();
      if (opts_.grpc) {
        std::string pb;
        message_to_pb(*in, pb);
        if (!message_from_pb(call_grpc(gm, pb), *m)) throw std::runtime_error("invalid protobuf response");
      } else {
        std::string js;
        message_to_json(*in, js);
        message_from_json(parse_json(call_rest(rp, js)), *m);
      }
      k(Outcome::ok(std::move(m)));
    } catch (const RemoteUserError& e) {
      k(Outcome::fail(make_user_error(e.status, e.body, e.what())));
    } catch (const std::exception& e) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, e.what())));
    }
  });
}

void RemoteUnit::predict(const CallCtx&, MsgPtr in, Done k) { call_message("predict", "Predict", std::move(in), std::move(k)); }
void RemoteUnit::transform_input(const CallCtx&, MsgPtr in, Done k) {
  call_message("transform-input", "TransformInput", std::move(in), std::move(k));
}
void RemoteUnit::transform_output(const CallCtx&, MsgPtr in, Done k) {
  call_message("transform-output", "TransformOutput", std::move(in), std::move(k));
}
void RemoteUnit::route(const CallCtx&, MsgPtr in, Done k) { call_message("route", "Route", std::move(in), std::move(k)); }

void RemoteUnit::aggregate(const CallCtx&, std::vector<MsgPtr> in, Done k) {
  submit([this, in, k]() {
    try {
      std::vector<const SeldonMessage*> v;
      for (auto& m : in) v.push_back(m.get());
      auto m = std::make_shared<SeldonMessage>();
      if (opts_.grpc) {
        std::string pb;
        message_list_to_pb(v, pb);
        if (!message_from_pb(call_grpc("Aggregate", pb), *m)) throw std::runtime_error("invalid protobuf response");
      } else {
        std::string js;
        message_list_to_json(v, js);
        message_from_json(parse_json(call_rest("aggregate", js)), *m);
      }
      k(Outcome::ok(std::move(m)));
    } catch (const RemoteUserError& e) {
      k(Outcome::fail(make_user_error(e.status, e.body, e.what())));
    } catch (const std::exception& e) {
      k(Outcome::fail(make_error(ApiError::MICROSERVICE_ERROR, e.what())));
    }
  });
}

void RemoteUnit::send_feedback(const CallCtx&, std::shared_ptr<const Feedback> fb, FbDone k) {
  submit([this, fb, k]() {
    try {
      if (opts_.grpc) {
        std::string pb;
        feedback_to_pb(*fb, pb);
        call_grpc("SendFeedback", pb);
      } else {
        std::string js;
        feedback_to_json(*fb, js);
        call_rest("send-feedback", js);
      }
      k(nullptr);
    } catch (const RemoteUserError& e) {
      k(make_user_error(e.status, e.body, e.what()));
    } catch (const std::exception& e) {
      k(make_error(ApiError::MICROSERVICE_ERROR, e.what()));
    }
  });
}

}  // namespace sca
