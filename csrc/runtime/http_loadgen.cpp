// Closed-loop HTTP/1.1 load generator; see http_loadgen.h.
#include "runtime/http_loadgen.h"

#include <arpa/inet.h>
#include <pthread.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <unordered_map>

namespace arena {

namespace {

using Clock = std::chrono::steady_clock;

double now_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }

int count_of(const std::string& s, size_t from, size_t to, const char* pat) {
  const size_t n = std::strlen(pat);
  int k = 0;
  for (size_t p = s.find(pat, from); p != std::string::npos && p + n <= to; p = s.find(pat, p + n)) ++k;
  return k;
}

}  // namespace

struct HttpLoadGen::Conn {
  int fd = -1;
  const std::string* out = nullptr;  // request being sent
  size_t off = 0;
  std::string in;
  double t_send = 0;
  bool waiting = false;  // a request is in flight on this connection
};

HttpLoadGen::HttpLoadGen(LoadGenConfig cfg, std::vector<std::string> requests)
    : cfg_(std::move(cfg)), reqs_(std::move(requests)) {
  if (reqs_.empty()) throw std::runtime_error("HttpLoadGen: no requests");
  if (cfg_.users < 1) throw std::runtime_error("HttpLoadGen: users < 1");
  cfg_.threads = std::max(1, std::min(cfg_.threads, cfg_.users));
}

HttpLoadGen::~HttpLoadGen() { stop(0.0); }

static int connect_to(const std::string& host, int port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
    ::close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  return fd;
}

void HttpLoadGen::start() {
  if (!threads_.empty()) return;
  t0_ = now_s();
  issuing_.store(true);
  for (int t = 0; t < cfg_.threads; ++t) epfds_.push_back(epoll_create1(EPOLL_CLOEXEC));
  for (int t = 0; t < cfg_.threads; ++t) threads_.emplace_back([this, t] { loop(t); });
}

void HttpLoadGen::loop(int idx) {
  pthread_setname_np(pthread_self(), "arena-loadgen");
  const int ep = epfds_[idx];
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  auto arm = [&](Conn* c, bool want_out) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | (want_out ? EPOLLOUT : 0u);
    ev.data.fd = c->fd;
    epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
  };
  auto send_some = [&](Conn* c) -> bool {  // false: connection broken
    while (c->off < c->out->size()) {
      const ssize_t k = ::send(c->fd, c->out->data() + c->off, c->out->size() - c->off, MSG_NOSIGNAL);
      if (k > 0) {
        c->off += (size_t)k;
        continue;
      }
      if (k < 0 && errno == EINTR) continue;
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        arm(c, true);
        return true;
      }
      return false;
    }
    arm(c, false);
    return true;
  };
  auto issue = [&](Conn* c) -> bool {  // false: nothing issued (stopped or request budget spent)
    if (!issuing_.load()) return false;
    const int64_t k = next_req_.fetch_add(1);
    if (cfg_.max_requests > 0 && k >= cfg_.max_requests) return false;
    c->out = &reqs_[(size_t)(k % (int64_t)reqs_.size())];
    c->off = 0;
    c->in.clear();
    c->t_send = now_s();
    c->waiting = true;
    in_flight_.fetch_add(1);
    return true;
  };
  auto record = [&](Conn* c, int status, int dets) {
    c->waiting = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      const double t = now_s();  // under the lock: records are in completion order across threads
      recs_.push_back({t - t0_, (float)(t - c->t_send), (int16_t)status, (int16_t)std::min(dets, 32767)});
    }
    in_flight_.fetch_sub(1);
    cv_.notify_all();
  };
  auto open_conn = [&]() -> Conn* {
    const int fd = connect_to(cfg_.host, cfg_.port);
    if (fd < 0) {
      connect_failures_.fetch_add(1);
      return nullptr;
    }
    auto c = std::make_unique<Conn>();
    c->fd = fd;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.fd = fd;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    Conn* raw = c.get();
    conns[fd] = std::move(c);
    live_conns_.fetch_add(1);
    return raw;
  };
  auto drop = [&](Conn* c) {
    epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
    live_conns_.fetch_sub(1);
    conns.erase(c->fd);
  };
  // (re)open a connection for one user and send its next request; a few attempts, then the user is dropped
  auto reopen = [&]() {
    for (int attempt = 0; attempt < 3 && issuing_.load(); ++attempt) {
      Conn* n = open_conn();
      if (n == nullptr) continue;
      if (!issue(n)) return;
      if (send_some(n)) return;
      record(n, -1, 0);
      drop(n);
    }
  };
  auto restart = [&](Conn* c) {  // the server closed the connection: reconnect and continue the user's loop
    if (c->waiting) record(c, -1, 0);
    drop(c);
    reopen();
  };

  for (int u = idx; u < cfg_.users; u += cfg_.threads) reopen();
  std::vector<epoll_event> evs(256);
  char buf[16384];
  while (!stop_.load()) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 50);
    for (int i = 0; i < n; ++i) {
      auto it = conns.find(evs[i].data.fd);
      if (it == conns.end()) continue;
      Conn* c = it->second.get();
      if ((evs[i].events & EPOLLOUT) && c->out && c->off < c->out->size()) {
        if (!send_some(c)) {
          restart(c);
          continue;
        }
      }
      if (!(evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) continue;
      bool eof = false;
      while (true) {
        const ssize_t k = ::recv(c->fd, buf, sizeof buf, 0);
        if (k > 0) {
          c->in.append(buf, (size_t)k);
          continue;
        }
        if (k == 0) eof = true;
        else if (errno == EINTR) continue;
        else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
        break;
      }
      // complete responses (one per request; the server answers in order)
      bool broken = false;
      while (c->waiting) {
        const size_t hend = c->in.find("\r\n\r\n");
        if (hend == std::string::npos) break;
        int status = 0;
        if (c->in.compare(0, 5, "HTTP/") == 0) {
          const size_t sp = c->in.find(' ');
          if (sp != std::string::npos) status = std::atoi(c->in.c_str() + sp + 1);
        }
        int64_t clen = 0;
        bool close_after = false;
        for (size_t p = c->in.find("\r\n") + 2; p < hend;) {
          size_t e = c->in.find("\r\n", p);
          if (e == std::string::npos || e > hend) e = hend;
          std::string h = c->in.substr(p, e - p);
          std::transform(h.begin(), h.end(), h.begin(), [](unsigned char ch) { return (char)std::tolower(ch); });
          if (h.rfind("content-length:", 0) == 0) clen = std::atoll(h.c_str() + 15);
          else if (h.rfind("connection:", 0) == 0 && h.find("close") != std::string::npos) close_after = true;
          p = e + 2;
        }
        const size_t total = hend + 4 + (size_t)std::max<int64_t>(0, clen);
        if (c->in.size() < total) break;
        record(c, status, count_of(c->in, hend + 4, total, "\"class_name\""));
        c->in.erase(0, total);
        if (close_after) {
          broken = true;
          break;
        }
        if (issue(c) && !send_some(c)) {
          broken = true;
          break;
        }
      }
      if (broken || eof) restart(c);
    }
  }
  for (auto& kv : conns) {
    ::close(kv.first);
    live_conns_.fetch_sub(1);
  }
  conns.clear();
}

void HttpLoadGen::stop(double timeout_s) {
  if (threads_.empty()) return;
  issuing_.store(false);
  const auto deadline = Clock::now() + std::chrono::duration<double>(std::max(0.0, timeout_s));
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_until(lk, deadline, [this] { return in_flight_.load() <= 0; });
  }
  stop_.store(true);
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (int ep : epfds_) ::close(ep);
  epfds_.clear();
}

int64_t HttpLoadGen::completed() {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)recs_.size();
}

bool HttpLoadGen::wait_completed(int64_t n, double timeout_s) {
  const auto deadline = Clock::now() + std::chrono::duration<double>(std::max(0.0, timeout_s));
  std::unique_lock<std::mutex> lk(mu_);
  while ((int64_t)recs_.size() < n) {
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout && (int64_t)recs_.size() < n) return false;
    if (live_conns_.load() == 0 && in_flight_.load() == 0 && connect_failures_.load() > 0 &&
        (int64_t)recs_.size() < n)
      return false;
  }
  return true;
}

std::vector<LoadGenRecord> HttpLoadGen::records(int64_t from, int64_t to) {
  std::lock_guard<std::mutex> lk(mu_);
  from = std::max<int64_t>(0, from);
  to = std::min<int64_t>((int64_t)recs_.size(), to < 0 ? (int64_t)recs_.size() : to);
  if (to <= from) return {};
  return std::vector<LoadGenRecord>(recs_.begin() + from, recs_.begin() + to);
}

}  // namespace arena
