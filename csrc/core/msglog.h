// Request/response logging off the hot path.
//
// Reference: engine/.../service/PredictionService.java:98-191 -- optional
// stdout JSON logging of requests / responses / feedback
// (SELDON_LOG_REQUESTS, SELDON_LOG_RESPONSES, SELDON_LOG_FEEDBACK_REQUESTS) and
// a CloudEvents 0.2 POST of each {request, response} pair to
// SELDON_MESSAGE_LOGGING_SERVICE (headers CE-SpecVersion / CE-Type
// seldon.message.pair / CE-Time / CE-EventID=puid / CE-Source).  The reference
// does this synchronously on the request thread; here the completing thread
// only enqueues the two messages and a background thread serialises and ships
// them (bounded queue, drops counted rather than back-pressuring serving).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "message.h"

namespace sca {

struct MessageLogOptions {
  bool log_requests = false;
  bool log_responses = false;
  bool log_feedback = false;
  bool external = false;               // SELDON_LOG_MESSAGES_EXTERNALLY
  std::string url;                     // SELDON_MESSAGE_LOGGING_SERVICE
  std::string message_type = "seldon.message.pair";
  std::string deployment_name;         // DEPLOYMENT_NAME ("" = unset)
  std::string deployment_namespace;    // DEPLOYMENT_NAMESPACE
  size_t max_queue = 65536;
  int timeout_ms = 2000;
};

class MessageLogger {
 public:
  explicit MessageLogger(MessageLogOptions o);
  ~MessageLogger();
  bool wants_pairs() const { return o_.log_requests || o_.log_responses || o_.external; }
  bool wants_feedback() const { return o_.log_feedback; }
  void pair(std::shared_ptr<const SeldonMessage> req, std::shared_ptr<const SeldonMessage> resp,
            std::chrono::system_clock::time_point t_req);
  void feedback(std::shared_ptr<const Feedback> fb);
  void flush();  // wait until the queue is drained (tests / shutdown)
  uint64_t sent() const { return sent_.load(); }
  uint64_t dropped() const { return dropped_.load(); }
  uint64_t failed() const { return failed_.load(); }

  // {"request": {...,"date"}, "response": {...,"date"}, "sdepName", "namespace"}
  std::string pair_json(const SeldonMessage& req, const SeldonMessage& resp, const std::string& t_req,
                        const std::string& t_resp) const;
  static std::string iso_time(std::chrono::system_clock::time_point t);

 private:
  struct Job {
    std::shared_ptr<const SeldonMessage> req, resp;
    std::shared_ptr<const Feedback> fb;
    std::chrono::system_clock::time_point t_req, t_resp;
  };
  void loop();
  void post(const std::string& body, const std::string& puid, const std::string& t_req);

  MessageLogOptions o_;
  std::mutex mu_;
  std::condition_variable cv_, cv_idle_;
  std::deque<Job> q_;
  bool busy_ = false;
  bool stop_ = false;
  std::atomic<uint64_t> sent_{0}, dropped_{0}, failed_{0};
  std::string host_, path_;
  int port_ = 80;
  int fd_ = -1;  // keep-alive connection to the sink
  std::thread th_;
};

}  // namespace sca
