#include "msglog.h"

#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "json.h"

namespace sca {

namespace {

bool parse_url(const std::string& url, std::string& host, int& port, std::string& path) {
  std::string u = url;
  if (u.rfind("http://", 0) == 0) u = u.substr(7);
  else if (u.find("://") != std::string::npos) return false;  // https etc. unsupported
  const size_t slash = u.find('/');
  std::string hp = slash == std::string::npos ? u : u.substr(0, slash);
  path = slash == std::string::npos ? "/" : u.substr(slash);
  const size_t colon = hp.rfind(':');
  port = 80;
  if (colon != std::string::npos) {
    port = std::atoi(hp.c_str() + colon + 1);
    hp = hp.substr(0, colon);
  }
  host = hp;
  return !host.empty() && port > 0;
}

int dial(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (connect(fd, a->ai_addr, a->ai_addrlen) == 0) break;
    close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  return fd;
}

bool send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n <= 0) {
      if (n < 0 && errno == EINTR) continue;
      return false;
    }
    off += size_t(n);
  }
  return true;
}

// Reads one HTTP/1.1 response (Content-Length or chunked ignored: we only need
// the status line and to consume the body for keep-alive). Returns status or -1.
int read_response(int fd, bool& keep_alive) {
  std::string buf;
  char tmp[4096];
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
    if (n <= 0) return -1;
    buf.append(tmp, size_t(n));
  }
  int status = -1;
  if (buf.size() > 12) status = std::atoi(buf.c_str() + 9);
  std::string head = buf.substr(0, hdr_end);
  for (auto& c : head) c = char(std::tolower(static_cast<unsigned char>(c)));
  keep_alive = head.find("connection: close") == std::string::npos;
  size_t len = 0;
  const size_t cl = head.find("content-length:");
  if (cl != std::string::npos) len = size_t(std::atoll(head.c_str() + cl + 15));
  else keep_alive = false;  // unknown framing: don't reuse
  size_t have = buf.size() - hdr_end - 4;
  while (have < len) {
    ssize_t n = ::recv(fd, tmp, std::min(sizeof tmp, len - have), 0);
    if (n <= 0) return status;
    have += size_t(n);
  }
  return status;
}

}  // namespace

MessageLogger::MessageLogger(MessageLogOptions o) : o_(std::move(o)) {
  if (o_.external && !parse_url(o_.url, host_, port_, path_)) {
    std::fprintf(stderr, "[seldon-amd] message logging service URL not supported: %s\n", o_.url.c_str());
    o_.external = false;
  }
  th_ = std::thread([this] { loop(); });
}

MessageLogger::~MessageLogger() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  if (fd_ >= 0) close(fd_);
}

std::string MessageLogger::iso_time(std::chrono::system_clock::time_point t) {
  const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(t.time_since_epoch()).count();
  const time_t secs = time_t(ms / 1000);
  tm g{};
  gmtime_r(&secs, &g);
  char b[40];
  std::snprintf(b, sizeof b, "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ", g.tm_year + 1900, g.tm_mon + 1, g.tm_mday, g.tm_hour,
                g.tm_min, g.tm_sec, int(ms % 1000));
  return b;
}

void MessageLogger::pair(std::shared_ptr<const SeldonMessage> req, std::shared_ptr<const SeldonMessage> resp,
                         std::chrono::system_clock::time_point t_req) {
  Job j;
  j.req = std::move(req);
  j.resp = std::move(resp);
  j.t_req = t_req;
  j.t_resp = std::chrono::system_clock::now();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= o_.max_queue) { dropped_++; return; }
    q_.push_back(std::move(j));
  }
  cv_.notify_one();
}

void MessageLogger::feedback(std::shared_ptr<const Feedback> fb) {
  Job j;
  j.fb = std::move(fb);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= o_.max_queue) { dropped_++; return; }
    q_.push_back(std::move(j));
  }
  cv_.notify_one();
}

void MessageLogger::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_idle_.wait(lk, [&] { return q_.empty() && !busy_; });
}

std::string MessageLogger::pair_json(const SeldonMessage& req, const SeldonMessage& resp, const std::string& t_req,
                                     const std::string& t_resp) const {
  auto with_date = [](const SeldonMessage& m, const std::string& date) {
    std::string s;
    message_to_json(m, s);
    // message_to_json always renders an object; splice "date" in before '}'.
    const size_t end = s.rfind('}');
    std::string tail = ",\"date\":";
    append_quoted(tail, date);
    s.insert(end, s.size() > 2 ? tail : tail.substr(1));
    return s;
  };
  std::string out = "{\"request\":" + with_date(req, t_req) + ",\"response\":" + with_date(resp, t_resp);
  if (!o_.deployment_name.empty()) {
    out += ",\"sdepName\":";
    append_quoted(out, o_.deployment_name);
  }
  if (!o_.deployment_namespace.empty()) {
    out += ",\"namespace\":";
    append_quoted(out, o_.deployment_namespace);
  }
  out += "}";
  return out;
}

void MessageLogger::post(const std::string& body, const std::string& puid, const std::string& t_req) {
  std::string req = "POST " + path_ + " HTTP/1.1\r\nHost: " + host_ + ":" + std::to_string(port_) +
                    "\r\nContent-Type: application/json\r\nX-B3-Flags: 1\r\nCE-SpecVersion: 0.2\r\nCE-Type: " +
                    o_.message_type + "\r\nCE-Time: " + t_req + "\r\nCE-EventID: " + puid +
                    "\r\nCE-Source: " + (o_.deployment_name.empty() ? "seldon" : "application/json") +
                    "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (fd_ < 0) fd_ = dial(host_, port_, o_.timeout_ms);
    if (fd_ < 0) break;
    bool keep = false;
    int status = -1;
    if (send_all(fd_, req)) status = read_response(fd_, keep);
    if (status < 0 || !keep) {
      close(fd_);
      fd_ = -1;
    }
    if (status >= 200 && status < 300) { sent_++; return; }
    if (status >= 0) break;  // the sink answered with an error: don't resend
  }
  failed_++;
}

void MessageLogger::loop() {
  while (true) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(mu_);
      busy_ = false;
      if (q_.empty()) cv_idle_.notify_all();
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ and drained
      j = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
    }
    if (j.fb) {
      std::string s;
      feedback_to_json(*j.fb, s);
      std::fprintf(stdout, "%s\n", s.c_str());
      std::fflush(stdout);
      continue;
    }
    if (o_.log_requests || o_.log_responses) {
      std::string s;
      if (o_.log_requests) { message_to_json(*j.req, s); std::fprintf(stdout, "%s\n", s.c_str()); }
      if (o_.log_responses) { s.clear(); message_to_json(*j.resp, s); std::fprintf(stdout, "%s\n", s.c_str()); }
      std::fflush(stdout);
    }
    if (o_.external) {
      const std::string tr = iso_time(j.t_req);
      post(pair_json(*j.req, *j.resp, tr, iso_time(j.t_resp)), j.req->meta.puid, tr);
    }
  }
}

}  // namespace sca
