// mxstream — socket text source core (Flink SocketTextStreamFunction semantics: '\n'
// delimiter, trailing '\r' stripped, remainder flushed at EOF, maxRetry = 0 by default). A
// background thread reads the connection; the consumer polls batches of lines. No Python here
// (csrc/runtime.cpp binds it; csrc/tests/tsan_main.cpp runs it under ThreadSanitizer).
//
// Back-pressure: the queue between the reader and the consumer holds at most `max_queue` lines.
// A full queue blocks the reader thread, which stops draining the socket, so the kernel's
// receive buffer fills and TCP flow control slows the sender -- a slow job throttles its source
// instead of growing host memory without bound (Flink's credit-based network stack, F-net).
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "mxs_log.h"

namespace mxs {

class SocketReaderCore {
 public:
  SocketReaderCore(std::string host, int port, std::string delimiter, int max_retry, int64_t retry_ms,
                   size_t max_queue = 1 << 22)
      : host_(std::move(host)), port_(port), delim_(std::move(delimiter)), max_retry_(max_retry),
        retry_ms_(retry_ms), max_queue_(max_queue ? max_queue : 1) {
    if (delim_.empty()) throw std::invalid_argument("empty delimiter");
  }

  // Times the reader waited for queue space (back-pressure events) -- for metrics and tests.
  int64_t blocked() const { return blocked_.load(); }
  ~SocketReaderCore() { close(); }

  void start() {
    if (th_.joinable()) return;
    th_ = std::thread([this] { run(); });
  }

  // Up to max_lines queued lines ('\n'-terminated) into *joined; waits up to timeout_ms for
  // the first one. *eof: the connection is closed and everything was handed out.
  void poll(size_t max_lines, int timeout_ms, std::string* joined, size_t* n, bool* eof,
            std::string* err) {
    joined->clear();
    *n = 0;
    std::unique_lock<std::mutex> lk(mu_);
    // system_clock deadline: pthread_cond_timedwait, which ThreadSanitizer intercepts
    // (steady_clock waits use pthread_cond_clockwait, invisible to GCC 11's TSan).
    cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), [&] { return !q_.empty() || eof_; });
    while (!q_.empty() && *n < max_lines) {
      *joined += q_.front();
      joined->push_back('\n');
      q_.pop_front();
      ++*n;
    }
    *eof = eof_ && q_.empty();
    *err = err_;
    if (*n) space_.notify_all();
  }

  // Stops the reader: shutdown() wakes a recv() blocked on the connection; the reader thread
  // itself closes the descriptor (closing it here would race with that recv and could hit a
  // reused descriptor number). fd_ changes only under mu_.
  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
      space_.notify_all();  // a reader blocked on a full queue
    }
    if (th_.joinable()) th_.join();
  }

 private:
  void push(std::string line) {
    std::unique_lock<std::mutex> lk(mu_);
    if (q_.size() >= max_queue_) {
      blocked_.fetch_add(1);
      space_.wait(lk, [&] { return q_.size() < max_queue_ || stop_; });
    }
    q_.push_back(std::move(line));
    cv_.notify_one();
  }
  void finish(const std::string& err) {
    std::lock_guard<std::mutex> g(mu_);
    eof_ = true;
    err_ = err;
    cv_.notify_all();
  }
  int connect_once() {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0) return -1;
    int fd = -1;
    for (addrinfo* p = res; p; p = p->ai_next) {
      fd = ::socket(p->ai_family, p->ai_socktype, p->ai_protocol);
      if (fd < 0) continue;
      if (::connect(fd, p->ai_addr, p->ai_addrlen) == 0) break;
      ::close(fd);
      fd = -1;
    }
    freeaddrinfo(res);
    return fd;
  }
  void run() {
    int attempt = 0;
    std::string buffer;
    while (!stop_) {
      const int fd = connect_once();
      if (fd < 0) {
        if (max_retry_ >= 0 && attempt >= max_retry_) {
          mxs_log(kError, "socket", "could not connect to " + host_ + ":" + std::to_string(port_));
          finish("ConnectException: could not connect to " + host_ + ":" + std::to_string(port_));
          return;
        }
        ++attempt;
        mxs_log(kWarn, "socket", "connect to " + host_ + ":" + std::to_string(port_) +
                                     " failed, retry " + std::to_string(attempt));
        std::this_thread::sleep_for(std::chrono::milliseconds(retry_ms_));
        continue;
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        fd_ = fd;
      }
      mxs_log(kInfo, "socket", "connected to " + host_ + ":" + std::to_string(port_));
      char chunk[8192];
      while (!stop_) {
        const ssize_t r = ::recv(fd, chunk, sizeof(chunk), 0);
        if (r <= 0) break;
        buffer.append(chunk, (size_t)r);
        size_t pos;
        while ((pos = buffer.find(delim_)) != std::string::npos) {
          std::string line = buffer.substr(0, pos);
          if (delim_ == "\n" && !line.empty() && line.back() == '\r') line.pop_back();
          push(std::move(line));
          buffer.erase(0, pos + delim_.size());
        }
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        fd_ = -1;
        ::close(fd);
      }
      ++attempt;
      if (stop_ || max_retry_ == 0 || (max_retry_ > 0 && attempt > max_retry_)) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(retry_ms_));
    }
    if (!buffer.empty()) push(buffer);
    finish("");
  }

  std::string host_;
  int port_;
  std::string delim_;
  int max_retry_;
  int64_t retry_ms_;
  std::thread th_;
  std::mutex mu_;
  size_t max_queue_;
  std::condition_variable cv_;     // consumer: lines available / end of stream
  std::condition_variable space_;  // reader: room in the queue (back-pressure)
  std::deque<std::string> q_;
  std::atomic<int64_t> blocked_{0};
  bool eof_ = false;
  std::string err_;
  std::atomic<bool> stop_{false};
  int fd_ = -1;  // guarded by mu_
};

}  // namespace mxs
