// Native HTTP/1.1 front end (see http_front.h).
#include "http_front.h"

#include <arpa/inet.h>
#include <cstdlib>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <ctime>
#include <stdexcept>

#include "jpeg_decode.h"

namespace arena {

const std::vector<double> kLatencyBucketsMs = {1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000};
const std::vector<std::string> kStages = {"decode", "queue", "gpu", "detection", "classification", "total"};

namespace {

using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// CPU time of the calling thread (ms): the per-stage host cost breakdown of FrontStats
double thread_cpu_ms() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

thread_local bool t_predict_dispatched = false;  // parse_one dispatched a /predict (its CPU counts as "parse")

std::string lower(std::string s) {
  for (auto& ch : s) ch = (char)std::tolower((unsigned char)ch);
  return s;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
  return s.substr(a, b - a);
}

void json_escape(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char ch : s) {
    if (ch == '"') out += "\\\"";
    else if (ch == '\\') out += "\\\\";
    else if (ch < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", ch);
      out += b;
    } else out.push_back((char)ch);
  }
  out.push_back('"');
}

void json_num(std::string& out, double v) {
  if (!std::isfinite(v)) {
    out += "null";
    return;
  }
  char b[32];
  snprintf(b, sizeof b, "%.9g", v);
  out += b;
}

std::string detail_json(const std::string& msg) {
  std::string s = "{\"detail\":";
  json_escape(s, msg);
  s += "}";
  return s;
}

std::string uuid4() {
  thread_local std::mt19937_64 rng(std::random_device{}() ^ (uint64_t)Clock::now().time_since_epoch().count());
  uint64_t a = rng(), b = rng();
  a = (a & 0xffffffffffff0fffULL) | 0x0000000000004000ULL;  // version 4
  b = (b & 0x3fffffffffffffffULL) | 0x8000000000000000ULL;  // variant 10
  char s[40];
  snprintf(s, sizeof s, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xffff),
           (unsigned)(a & 0xffff), (unsigned)(b >> 48), (unsigned long long)(b & 0xffffffffffffULL));
  return s;
}

// The reference /predict body (architectures/monolithic/app/models.py PredictResponse): request id, detections
// with their top-1 classification (raw logit, or the softmax probability with ARENA_CONFIDENCE=softmax), timing.
std::string predict_json(const RequestResult& r, const std::vector<std::string>& labels, bool softmax,
                         double queue_ms, double gpu_ms, double det_ms, double cls_ms, double inference_ms,
                         double decode_ms, double total_ms) {
  std::string s;
  s.reserve(512 + 256 * r.det.size());
  s += "{\"request_id\":";
  json_escape(s, uuid4());
  s += ",\"detections\":[";
  for (size_t i = 0; i < r.det.size(); ++i) {
    const Detection& d = r.det[i];
    if (i) s += ',';
    s += "{\"detection\":{\"x1\":";
    json_num(s, d.x1);
    s += ",\"y1\":";
    json_num(s, d.y1);
    s += ",\"x2\":";
    json_num(s, d.x2);
    s += ",\"y2\":";
    json_num(s, d.y2);
    s += ",\"confidence\":";
    json_num(s, d.conf);
    s += ",\"class_id\":" + std::to_string(d.cls) + "},\"classification\":{\"class_id\":";
    int cid = -1;
    double conf = 0.0;
    if (i < r.topk.size()) {
      cid = r.topk[i].idx[0];
      conf = softmax ? r.topk[i].prob[0] : r.topk[i].logit[0];
    }
    s += std::to_string(cid) + ",\"class_name\":";
    json_escape(s, (cid >= 0 && cid < (int)labels.size()) ? labels[cid] : std::string());
    s += ",\"confidence\":";
    json_num(s, conf);
    s += "}}";
  }
  s += "],\"timing\":{\"queue_ms\":";
  json_num(s, queue_ms);
  s += ",\"gpu_ms\":";
  json_num(s, gpu_ms);
  s += ",\"batch_size\":";
  json_num(s, r.batch_size);
  s += ",\"detection_ms\":";
  json_num(s, det_ms);
  s += ",\"classification_ms\":";
  json_num(s, cls_ms);
  s += ",\"inference_ms\":";
  json_num(s, inference_ms);
  s += ",\"decode_ms\":";
  json_num(s, decode_ms);
  s += ",\"total_ms\":";
  json_num(s, total_ms);
  s += "}}";
  return s;
}

const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 422: return "Unprocessable Entity";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Unknown";
  }
}

bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n > 0) {
    const ssize_t k = ::write(fd, c, n);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n > 0) {
    const ssize_t k = ::read(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

// multipart/form-data: the part named `field`; returns false when absent / malformed
bool multipart_field(const std::string& body, const std::string& ctype, const std::string& field, size_t& off,
                     size_t& len, std::string& err) {
  const std::string lc = lower(ctype);
  size_t bp = lc.find("boundary=");
  if (bp == std::string::npos) {
    err = "multipart body without a boundary";
    return false;
  }
  std::string boundary = ctype.substr(bp + 9);
  const size_t semi = boundary.find(';');
  if (semi != std::string::npos) boundary = boundary.substr(0, semi);
  boundary = trim(boundary);
  if (boundary.size() >= 2 && boundary.front() == '"' && boundary.back() == '"')
    boundary = boundary.substr(1, boundary.size() - 2);
  if (boundary.empty()) {
    err = "multipart body without a boundary";
    return false;
  }
  const std::string delim = "--" + boundary;
  size_t pos = body.find(delim);
  while (pos != std::string::npos) {
    pos += delim.size();
    if (body.compare(pos, 2, "--") == 0) break;  // closing delimiter
    if (body.compare(pos, 2, "\r\n") == 0) pos += 2;
    const size_t hend = body.find("\r\n\r\n", pos);
    if (hend == std::string::npos) break;
    const std::string headers = lower(body.substr(pos, hend - pos));
    const size_t dstart = hend + 4;
    const size_t dend = body.find("\r\n" + delim, dstart);
    if (dend == std::string::npos) break;
    const std::string want = "name=\"" + lower(field) + "\"";
    if (headers.find("content-disposition") != std::string::npos && headers.find(want) != std::string::npos) {
      off = dstart;
      len = dend - dstart;
      return true;
    }
    pos = dend + 2;
  }
  err = "missing form field '" + field + "'";
  return false;
}

}  // namespace

struct HttpFrontEnd::Conn {
  int fd = -1, ep = -1;
  std::mutex mu;             // out / closed / busy / paused (the response may come from any thread)
  std::string in;            // I/O thread only
  std::string out;
  size_t out_off = 0;
  bool closed = false, busy = false, close_after = false;
  bool paused = false;       // input buffer at its cap: EPOLLIN off until the in-flight response is written
  // I/O thread only: timeouts and the incremental chunked-body parse (a body arriving over many reads is
  // scanned once, not from its start on every read)
  Clock::time_point last_rx, req_start;
  bool in_request = false;
  size_t chunk_pos = 0;      // next chunk-size line (0: not started)
  std::string chunk_body;
  HttpFrontEnd::LocalDone local;  // in-process request (submit_local): the answer goes here, not to a socket
};

struct HttpFrontEnd::Pending {
  std::shared_ptr<Conn> conn;
  int worker = 0;
  int kind = 0;  // 0 /predict, 1 KServe infer
  Clock::time_point t0, t_dec;
};

struct HttpFrontEnd::HandlerPending {
  std::shared_ptr<Conn> conn;
  Clock::time_point t0;
};

struct HttpFrontEnd::DecodeTask {
  std::shared_ptr<Conn> conn;
  Clock::time_point t0, t_queued;
  std::string body;  // the request body (moved in); the upload is body[off, off + len)
  size_t off = 0, len = 0;
  int kind = 0;      // 0 /predict, 1 KServe infer
};

namespace {
// A split-decoded upload in flight: its parsed header (the device descriptor's source) and the buffer holding
// its coefficients (or, host-only mode, its RGB frame); kept alive by the batcher until the request completes.
struct NativeUpload {
  JpegInfo info;
  std::shared_ptr<uint8_t> buf;
};
}  // namespace

HttpFrontEnd::HttpFrontEnd(DynamicBatcher* batcher, DecodeChannel dc, std::vector<std::string> labels,
                           FrontConfig cfg)
    : batcher_(batcher), dc_(std::move(dc)), labels_(std::move(labels)), cfg_(std::move(cfg)) {
  const bool proxy = cfg_.upstream_port > 0;
  if (proxy) {
    if (cfg_.handler_mode) throw std::runtime_error("HttpFrontEnd: proxy mode and handler mode exclude each other");
    std::vector<KServeUpstream> ups{KServeUpstream{cfg_.upstream_host, cfg_.upstream_port}};
    size_t p = 0;
    while (p < cfg_.upstreams.size()) {  // "host:port,host:port"
      size_t e = cfg_.upstreams.find(',', p);
      if (e == std::string::npos) e = cfg_.upstreams.size();
      const std::string item = cfg_.upstreams.substr(p, e - p);
      p = e + 1;
      if (item.empty()) continue;
      const size_t colon = item.rfind(':');
      if (colon == std::string::npos) throw std::runtime_error("HttpFrontEnd: upstream '" + item + "' is not host:port");
      KServeUpstream u{item.substr(0, colon), std::atoi(item.c_str() + colon + 1)};
      if (u.host.empty()) u.host = "127.0.0.1";
      if (u.port <= 0) throw std::runtime_error("HttpFrontEnd: upstream '" + item + "' has no port");
      if (u.host == ups[0].host && u.port == ups[0].port) continue;
      ups.push_back(u);
    }
    proxy_.reset(new KServeProxy(std::move(ups), cfg_.upstream_model, cfg_.upstream_conns));
    proxy_->set_recycler(&bodies_);
    cfg_.decode_threads = 0;
  }
  if (!cfg_.handler_mode && !proxy) {
    if (batcher_ == nullptr) throw std::runtime_error("HttpFrontEnd: no batcher");
    has_pool_ = dc_.shm != nullptr;
    if (has_pool_ || cfg_.decode_threads <= 0) {
      if (dc_.shm == nullptr || dc_.slots <= 0 || dc_.task_fds.empty() || dc_.result_fd < 0 || dc_.result_wfd < 0)
        throw std::runtime_error("HttpFrontEnd: incomplete decode channel");
      if (dc_.big_fds.size() != dc_.task_fds.size())
        throw std::runtime_error("HttpFrontEnd: big_fds / task_fds mismatch");
    }
    if (cfg_.decode_threads > 0)
      host_pool_ = HostBufferPool::create(cfg_.decode_buffer_cap, cfg_.host_alloc, cfg_.host_free);
  }
  stats_.latency_hist.assign(kLatencyBucketsMs.size() + 1, 0);
  stats_.stage_hist.assign(kStages.size(), std::vector<int64_t>(kLatencyBucketsMs.size() + 1, 0));
  stats_.stage_sum_ms.assign(kStages.size(), 0.0);
  for (int s = dc_.slots - 1; s >= 0; --s) free_slots_.push_back(s);
  for (size_t i = 0; i < dc_.task_fds.size(); ++i) task_mu_.emplace_back(new std::mutex);
  load_ = std::vector<std::atomic<int>>(dc_.task_fds.size());
  for (auto& l : load_) l.store(0);

  listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) throw std::runtime_error("HttpFrontEnd: socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (cfg_.reuse_port) setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)cfg_.port);
  if (inet_pton(AF_INET, cfg_.host.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(listen_fd_, (sockaddr*)&addr, sizeof addr) != 0 || ::listen(listen_fd_, 1024) != 0) {
    const std::string e = strerror(errno);
    ::close(listen_fd_);
    throw std::runtime_error("HttpFrontEnd: cannot listen on port " + std::to_string(cfg_.port) + ": " + e);
  }
  socklen_t al = sizeof addr;
  getsockname(listen_fd_, (sockaddr*)&addr, &al);
  port_ = ntohs(addr.sin_port);
  stop_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);

  const int n = std::max(1, cfg_.io_threads);
  for (int i = 0; i < n; ++i) {
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLEXCLUSIVE;
    ev.data.fd = listen_fd_;
    epoll_ctl(ep, EPOLL_CTL_ADD, listen_fd_, &ev);
    epoll_event sv{};
    sv.events = EPOLLIN;
    sv.data.fd = stop_efd_;
    epoll_ctl(ep, EPOLL_CTL_ADD, stop_efd_, &sv);
    epfds_.push_back(ep);
  }
  for (int i = 0; i < n; ++i) io_threads_.emplace_back([this, i] { io_loop(i); });
  if (!cfg_.handler_mode && has_pool_) collector_ = std::thread([this] { collector_loop(); });
  if (!cfg_.handler_mode && !proxy)
    for (int i = 0; i < cfg_.decode_threads; ++i) decode_threads_.emplace_back([this, i] { decode_loop(i); });
}

HttpFrontEnd::~HttpFrontEnd() { stop(); }

void HttpFrontEnd::stop() {
  if (stop_.exchange(true)) return;
  if (proxy_) proxy_->stop();  // answers what it still holds; no upstream request outlives the front end
  uint64_t one = 1;
  if (write(stop_efd_, &one, sizeof one) < 0) { /* the flag alone stops the loops on their next wakeup */ }
  if (cfg_.handler_mode) {
    std::lock_guard<std::mutex> lk(hq_mu_);
    hq_cv_.notify_all();  // wake take()
  } else if (has_pool_) {
    // wake the collector with a sentinel completion record (key < 0)
    int64_t rec[4] = {-1, 0, 0, 0};
    write_all(dc_.result_wfd, rec, sizeof rec);
  }
  {
    std::lock_guard<std::mutex> lk(dq_mu_);
    dq_cv_.notify_all();
  }
  for (auto& t : io_threads_)
    if (t.joinable()) t.join();
  for (auto& t : decode_threads_)
    if (t.joinable()) t.join();
  if (collector_.joinable()) collector_.join();
  {
    std::lock_guard<std::mutex> lk(dq_mu_);
    dq_.clear();  // never started: their connections are closing with the front end
  }
  {
    // requests already handed to the batcher answer through callbacks that capture `this`; the batcher
    // completes (or fails, on its own shutdown) every one of them, so wait here rather than free under them
    std::unique_lock<std::mutex> lk(cb_mu_);
    if (!cb_cv_.wait_for(lk, std::chrono::seconds(30), [this] { return cb_outstanding_ == 0; }))
      std::fprintf(stderr, "http_front: %lld batcher callbacks still outstanding at stop()\n",
                   (long long)cb_outstanding_);
  }
  for (int ep : epfds_) ::close(ep);
  epfds_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  if (stop_efd_ >= 0) ::close(stop_efd_);
  stop_efd_ = -1;
  {
    std::lock_guard<std::mutex> lk(hq_mu_);
    hq_.clear();
    hpend_.clear();
  }
  std::lock_guard<std::mutex> lk(pend_mu_);
  pending_.clear();
}

void HttpFrontEnd::callback_done() {
  std::lock_guard<std::mutex> lk(cb_mu_);
  if (--cb_outstanding_ == 0) cb_cv_.notify_all();
}

void HttpFrontEnd::drain() {
  std::lock_guard<std::mutex> lk(drain_mu_);
  if (drained_ || listen_fd_ < 0) return;
  drained_ = true;
  for (int ep : epfds_) epoll_ctl(ep, EPOLL_CTL_DEL, listen_fd_, nullptr);
  ::shutdown(listen_fd_, SHUT_RDWR);  // the fd itself is closed by stop(), after the I/O threads joined
}

int HttpFrontEnd::handler_pending() {
  std::lock_guard<std::mutex> lk(hq_mu_);
  return (int)hpend_.size();
}

std::vector<HandlerRequest> HttpFrontEnd::take(int max_n, int timeout_ms) {
  std::vector<HandlerRequest> out;
  std::unique_lock<std::mutex> lk(hq_mu_);
  hq_cv_.wait_for(lk, std::chrono::milliseconds(std::max(0, timeout_ms)),
                  [this] { return !hq_.empty() || stop_.load(); });
  while (!hq_.empty() && (int)out.size() < std::max(1, max_n)) {
    out.push_back(std::move(hq_.front()));
    hq_.pop_front();
  }
  return out;
}

bool HttpFrontEnd::complete(uint64_t key, int code, const std::string& body, int n_det) {
  std::shared_ptr<HandlerPending> hp;
  {
    std::lock_guard<std::mutex> lk(hq_mu_);
    auto it = hpend_.find(key);
    if (it == hpend_.end()) return false;
    hp = it->second;
    hpend_.erase(it);
  }
  const double total_ms = ms_since(hp->t0);
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++stats_.requests;
    if (code == 200) {
      ++stats_.ok;
      stats_.detections += n_det;
      stats_.sum_total_ms += total_ms;
      size_t b = 0;
      while (b < kLatencyBucketsMs.size() && total_ms > kLatencyBucketsMs[b]) ++b;
      ++stats_.latency_hist[b];
    } else if (code == 413) {
      ++stats_.too_large;
    } else if (code == 503) {
      ++stats_.unavailable;
    } else if (code >= 500) {
      ++stats_.errors;
    } else {
      ++stats_.bad_request;
    }
  }
  respond(hp->conn, code, "application/json", body);
  return true;
}

void HttpFrontEnd::set_metrics_text(std::string text) {
  std::lock_guard<std::mutex> lk(metrics_mu_);
  metrics_text_ = std::move(text);
}

FrontStats HttpFrontEnd::stats() {
  FrontStats s;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    s = stats_;
  }
  s.bodies_recycled = (int64_t)bodies_.hits();
  s.bodies_allocated = (int64_t)bodies_.misses();
  return s;
}

void HttpFrontEnd::io_loop(int idx) {
  pthread_setname_np(pthread_self(), "arena-http-io");
  const int ep = epfds_[idx];
  std::unordered_map<int, std::shared_ptr<Conn>> conns;
  std::vector<epoll_event> evs(256);
  auto last_sweep = Clock::now();
  while (!stop_.load()) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 200);
    const auto now = Clock::now();
    if (now - last_sweep > std::chrono::milliseconds(500) && (cfg_.idle_timeout_ms > 0 || cfg_.read_timeout_ms > 0)) {
      last_sweep = now;
      std::vector<std::shared_ptr<Conn>> expired;
      for (auto& kv : conns) {
        const auto& c = kv.second;
        bool busy;
        {
          std::lock_guard<std::mutex> lk(c->mu);
          busy = c->busy || c->out_off < c->out.size();
        }
        if (busy) continue;  // a request in flight is answered, never cut off
        const double idle = std::chrono::duration<double, std::milli>(now - c->last_rx).count();
        const double reading = std::chrono::duration<double, std::milli>(now - c->req_start).count();
        if ((c->in_request && cfg_.read_timeout_ms > 0 && reading > cfg_.read_timeout_ms) ||
            (!c->in_request && cfg_.idle_timeout_ms > 0 && idle > cfg_.idle_timeout_ms))
          expired.push_back(c);
      }
      for (auto& c : expired) {
        conns.erase(c->fd);
        close_conn(ep, c);
        std::lock_guard<std::mutex> sl(stats_mu_);
        ++stats_.timeouts;
      }
    }
    for (int i = 0; i < n && !stop_.load(); ++i) {
      const int fd = evs[i].data.fd;
      if (fd == stop_efd_) continue;
      if (fd == listen_fd_) {
        while (true) {
          const int c = accept4(listen_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (c < 0) break;
          int one = 1;
          setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          auto conn = std::make_shared<Conn>();
          conn->fd = c;
          conn->ep = ep;
          conn->last_rx = Clock::now();
          conns[c] = conn;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = c;
          epoll_ctl(ep, EPOLL_CTL_ADD, c, &ev);
          std::lock_guard<std::mutex> lk(stats_mu_);
          ++stats_.connections;
          ++stats_.open_connections;
        }
        continue;
      }
      auto it = conns.find(fd);
      if (it == conns.end()) continue;
      auto c = it->second;
      if (evs[i].events & EPOLLOUT) handle_writable(ep, c);
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) handle_readable(ep, c);
      bool closed;
      {
        std::lock_guard<std::mutex> lk(c->mu);
        closed = c->closed;
      }
      if (closed) conns.erase(fd);
    }
  }
  for (auto& kv : conns) close_conn(ep, kv.second);
}

void HttpFrontEnd::close_conn(int ep, const std::shared_ptr<Conn>& c) {
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->closed) return;
  c->closed = true;
  epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);  // under the lock: a response thread never touches a reused descriptor
  std::lock_guard<std::mutex> sl(stats_mu_);
  --stats_.open_connections;
}

void HttpFrontEnd::handle_readable(int ep, const std::shared_ptr<Conn>& c) {
  {
    // handle_writable of the same event may have closed it: its descriptor number can already belong to a
    // connection another I/O thread accepted (found by tests/test_native_http.py's TSAN stress)
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->closed) return;
  }
  char buf[65536];
  bool eof = false;
  // Buffer at most one maximal request (body + headers) plus one read: a client pipelining while a request
  // is in flight, or streaming an endless chunked body, cannot grow the buffer without bound.
  const size_t cap = (size_t)cfg_.max_body + (64u << 10);
  while (c->in.size() < cap) {
    const ssize_t k = ::read(c->fd, buf, std::min(sizeof buf, cap - c->in.size() + 1));
    if (k > 0) {
      c->in.append(buf, (size_t)k);
      c->last_rx = Clock::now();
      if (!c->in_request) {
        c->in_request = true;
        c->req_start = c->last_rx;
      }
      continue;
    }
    if (k == 0) eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
    break;
  }
  if (c->in.size() >= cap) {  // stop reading until the connection's response is out (handle_writable re-arms)
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->closed && !c->paused) {
      c->paused = true;
      epoll_event ev{};
      // no EPOLLIN / EPOLLRDHUP (both level-triggered: a half-closed peer would spin the loop); a vanished
      // peer shows up as a failed send of the response
      ev.events = c->out_off < c->out.size() ? EPOLLOUT : 0u;
      ev.data.fd = c->fd;
      epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
    }
  }
  while (true) {
    {
      std::lock_guard<std::mutex> lk(c->mu);
      if (c->busy || c->closed) break;
    }
    if (!parse_one(c)) break;
  }
  if (c->in.size() >= cap) {
    // a full buffer that still holds no complete request (a chunked body of many tiny chunks costs more wire
    // bytes than its decoded size): nothing in flight will ever re-arm the connection, so answer now
    bool idle;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      idle = !c->busy && !c->closed;
      if (idle) {
        c->busy = true;
        c->close_after = true;
      }
    }
    if (idle) {
      c->in.clear();
      c->in_request = false;
      c->chunk_pos = 0;
      c->chunk_body.clear();
      fail_request(c, 413, "request body too large");
    }
  }
  if (eof) {
    bool busy;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      busy = c->busy;
      c->close_after = true;
    }
    if (!busy) close_conn(ep, c);
    else {  // the peer half-closed with a request in flight: answer it, then close
      epoll_event ev{};
      ev.events = 0;
      ev.data.fd = c->fd;
      std::lock_guard<std::mutex> lk(c->mu);
      if (!c->closed) epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
    }
  }
}

void HttpFrontEnd::handle_writable(int ep, const std::shared_ptr<Conn>& c) {
  bool done = false, close_now = false;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->closed) return;
    while (c->out_off < c->out.size()) {
      const ssize_t k = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
      if (k > 0) {
        c->out_off += (size_t)k;
        continue;
      }
      if (k < 0 && errno == EINTR) continue;
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      close_now = true;  // peer gone
      break;
    }
    if (!close_now && c->out_off >= c->out.size()) {
      c->out.clear();
      c->out_off = 0;
      c->busy = false;
      c->paused = false;
      done = true;
      if (c->close_after) close_now = true;
      else {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP;
        ev.data.fd = c->fd;
        epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
      }
    }
  }
  if (close_now) {
    close_conn(ep, c);
    return;
  }
  if (done) {
    while (true) {  // requests the client sent ahead (pipelining)
      {
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->busy || c->closed) break;
      }
      if (!parse_one(c)) break;
    }
  }
}

bool HttpFrontEnd::parse_one(const std::shared_ptr<Conn>& c) {
  t_predict_dispatched = false;
  const double c0 = thread_cpu_ms();
  const bool r = parse_one_impl(c);
  if (t_predict_dispatched) {
    const double dt = thread_cpu_ms() - c0;
    std::lock_guard<std::mutex> sl(stats_mu_);
    stats_.cpu_parse_ms += dt;
  }
  return r;
}

bool HttpFrontEnd::parse_one_impl(const std::shared_ptr<Conn>& c) {
  std::string& in = c->in;
  const size_t hend = in.find("\r\n\r\n");
  if (hend == std::string::npos || hend > 65536) {  // the header block is capped whether or not it is complete
    if (in.size() > 65536) {
      {
        std::lock_guard<std::mutex> lk(c->mu);
        c->busy = true;
        c->close_after = true;
      }
      in.clear();
      respond(c, 431, "application/json", detail_json("request headers too large"));
      return true;
    }
    return false;
  }
  const size_t le = in.find("\r\n");
  const std::string line = in.substr(0, le);
  const size_t s1 = line.find(' '), s2 = line.rfind(' ');
  auto bad = [&](int code, const std::string& msg) {
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->busy = true;
      c->close_after = true;
    }
    in.clear();
    c->in_request = false;
    c->chunk_pos = 0;
    c->chunk_body.clear();
    {
      std::lock_guard<std::mutex> sl(stats_mu_);
      ++stats_.requests;
      ++stats_.bad_request;
    }
    respond(c, code, "application/json", detail_json(msg));
    return true;
  };
  if (s1 == std::string::npos || s2 == s1) return bad(400, "malformed request line");
  const std::string method = line.substr(0, s1);
  std::string path = line.substr(s1 + 1, s2 - s1 - 1);
  const std::string version = line.substr(s2 + 1);
  const size_t q = path.find('?');
  if (q != std::string::npos) path = path.substr(0, q);
  int64_t clen = -1, ihcl = -1;
  bool chunked = false, close_req = version == "HTTP/1.0";
  std::string ctype;
  size_t p = le + 2;
  while (p < hend) {
    size_t e = in.find("\r\n", p);
    if (e == std::string::npos || e > hend) e = hend;
    const std::string h = in.substr(p, e - p);
    const size_t colon = h.find(':');
    if (colon != std::string::npos) {
      const std::string name = lower(trim(h.substr(0, colon)));
      const std::string val = trim(h.substr(colon + 1));
      if (name == "content-length") clen = std::atoll(val.c_str());
      else if (name == "transfer-encoding") chunked = lower(val).find("chunked") != std::string::npos;
      else if (name == "content-type") ctype = val;
      else if (name == "inference-header-content-length") ihcl = std::atoll(val.c_str());
      else if (name == "connection") {
        const std::string v = lower(val);
        if (v.find("close") != std::string::npos) close_req = true;
        else if (v.find("keep-alive") != std::string::npos) close_req = false;
      }
    }
    p = e + 2;
  }
  const size_t body0 = hend + 4;
  std::string body;
  size_t consumed;
  if (chunked) {
    // resume where the previous read stopped: chunks already appended stay in chunk_body
    size_t pos = c->chunk_pos ? c->chunk_pos : body0;
    body = c->chunk_pos ? std::move(c->chunk_body) : bodies_.get();
    auto suspend = [&]() {
      c->chunk_pos = pos;
      c->chunk_body = std::move(body);
      return false;
    };
    while (true) {
      const size_t e = in.find("\r\n", pos);
      if (e == std::string::npos) {
        if (in.size() - pos > 64) return bad(400, "malformed chunk size");
        return suspend();
      }
      errno = 0;
      char* endp = nullptr;
      const std::string field = in.substr(pos, e - pos);
      const long long n = std::strtoll(field.c_str(), &endp, 16);
      if (n < 0 || endp == field.c_str()) return bad(400, "malformed chunk size");
      if (errno == ERANGE) return bad(413, "request body too large");  // saturated: beyond any limit
      // compare without overflow: n may be up to LLONG_MAX
      if (n > cfg_.max_body - (int64_t)body.size()) return bad(413, "request body too large");
      if (in.size() < e + 2 + (size_t)n + 2) return suspend();
      if (n == 0) {  // last chunk, then optional trailers ending with an empty line
        const size_t tend = in.find("\r\n\r\n", e);
        if (in.compare(e + 2, 2, "\r\n") == 0) consumed = e + 4;
        else if (tend != std::string::npos) consumed = tend + 4;
        else return suspend();
        break;
      }
      body.append(in, e + 2, (size_t)n);
      pos = e + 2 + (size_t)n + 2;
    }
    c->chunk_pos = 0;
    c->chunk_body.clear();
  } else {
    if (clen < 0) clen = 0;
    if (clen > cfg_.max_body) return bad(413, "request body too large");
    if (in.size() < body0 + (size_t)clen) return false;
    body = bodies_.get();  // a recycled body's capacity: no allocation in steady state
    body.assign(in, body0, (size_t)clen);
    consumed = body0 + (size_t)clen;
  }
  in.erase(0, consumed);
  c->in_request = !in.empty();  // a pipelined request's bytes already count from now
  if (c->in_request) c->req_start = Clock::now();
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->busy = true;
    c->close_after = close_req;
  }
  dispatch(c, method, path, ctype, std::move(body), ihcl);
  return true;
}

void HttpFrontEnd::dispatch(const std::shared_ptr<Conn>& c, const std::string& method, const std::string& path,
                            const std::string& ctype, std::string&& body, int64_t ihcl) {
  if (!cfg_.kserve_model.empty() && path.rfind("/v2", 0) == 0 && kserve_route(c, method, path, std::move(body), ihcl))
    return;
  if (path == "/predict") {
    if (method != "POST") {
      respond(c, 405, "application/json", detail_json("Method Not Allowed"));
      return;
    }
    predict(c, std::move(body), ctype);
    return;
  }
  if (path == "/health" && method == "GET") {
    if (healthy_.load())
      respond(c, 200, "application/json", "{\"status\":\"healthy\",\"models_loaded\":true}");
    else
      respond(c, 503, "application/json", "{\"status\":\"unhealthy\",\"models_loaded\":false}");
    return;
  }
  if (path == "/metrics" && method == "GET") {
    std::string t;
    {
      std::lock_guard<std::mutex> lk(metrics_mu_);
      t = metrics_text_;
    }
    respond(c, 200, "text/plain; version=0.0.4; charset=utf-8", t);
    return;
  }
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++stats_.not_found;
  }
  respond(c, 404, "application/json", detail_json("Not Found"));
}

void HttpFrontEnd::respond(const std::shared_ptr<Conn>& c, int code, const std::string& ctype,
                           const std::string& body, bool, const std::string& extra_headers) {
  if (c->local) {
    c->local(code, body);
    return;
  }
  std::string r;
  r.reserve(body.size() + 160);
  char head[256];
  bool close_after;
  {
    std::lock_guard<std::mutex> lk(c->mu);
    close_after = c->close_after;
  }
  snprintf(head, sizeof head, "HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %zu\r\n%s", code,
           reason(code), ctype.c_str(), body.size(), close_after ? "Connection: close\r\n" : "");
  r += head;
  if (!cfg_.replica_tag.empty()) r += "x-arena-replica: " + cfg_.replica_tag + "\r\n";
  r += extra_headers;
  r += "\r\n";
  r += body;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->closed) return;
  c->out += r;
  epoll_event ev{};
  ev.events = c->paused ? EPOLLOUT : (EPOLLIN | EPOLLOUT | EPOLLRDHUP);  // the connection's I/O thread writes it
  ev.data.fd = c->fd;
  epoll_ctl(c->ep, EPOLL_CTL_MOD, c->fd, &ev);
}

void HttpFrontEnd::release_slot(int slot) {
  std::lock_guard<std::mutex> lk(slot_mu_);
  free_slots_.push_back(slot);
}

void HttpFrontEnd::predict(const std::shared_ptr<Conn>& c, std::string&& body, const std::string& ctype) {
  const auto t0 = Clock::now();
  auto fail = [&](int code, const std::string& msg) {
    {
      std::lock_guard<std::mutex> sl(stats_mu_);
      ++stats_.requests;
      if (code == 413) ++stats_.too_large;
      else if (code == 503) ++stats_.unavailable;
      else if (code >= 500) ++stats_.errors;
      else ++stats_.bad_request;
    }
    respond(c, code, "application/json", detail_json(msg));
  };
  if (!healthy_.load()) return fail(503, "Service not ready");
  size_t off = 0, len = body.size();
  if (lower(ctype).rfind("multipart/form-data", 0) == 0) {
    std::string err;
    if (!multipart_field(body, ctype, "file", off, len, err)) return fail(422, err);
  }
  if (len == 0) return fail(422, "empty request body");
  if (cfg_.handler_mode) {
    const uint64_t key = next_key_.fetch_add(1);
    auto hp = std::make_shared<HandlerPending>();
    hp->conn = c;
    hp->t0 = t0;
    {
      std::lock_guard<std::mutex> lk(hq_mu_);
      if ((int)hpend_.size() >= cfg_.max_handler_queue) {
        hp.reset();
      } else {
        hpend_[key] = hp;
        HandlerRequest r;
        r.key = key;
        r.data.assign(body, off, len);
        hq_.push_back(std::move(r));
      }
    }
    if (!hp) return fail(503, "request queue is full");
    hq_cv_.notify_one();
    return;
  }
  t_predict_dispatched = true;
  if (proxy_) {
    std::string upload = bodies_.get();
    upload.assign(body, off, len);
    bodies_.put(std::move(body));
    return proxy_predict(c, t0, std::move(upload));  // the proxy worker recycles it once forwarded
  }
  start_upload(c, t0, std::move(body), off, len, 0);
}

void HttpFrontEnd::start_upload(const std::shared_ptr<Conn>& c, Clock_tp t0, std::string&& body, size_t off,
                                size_t len, int kind) {
  if (cfg_.decode_threads > 0) {
    auto t = std::make_unique<DecodeTask>();
    t->conn = c;
    t->t0 = t0;
    t->t_queued = Clock::now();
    t->body = std::move(body);
    t->off = off;
    t->len = len;
    t->kind = kind;
    {
      std::lock_guard<std::mutex> lk(dq_mu_);
      dq_.push_back(std::move(t));
    }
    dq_cv_.notify_one();
    return;
  }
  pool_submit(c, t0, body, off, len, kind);
}

bool HttpFrontEnd::kserve_route(const std::shared_ptr<Conn>& c, const std::string& method, const std::string& path,
                                std::string&& body, int64_t ihcl) {
  const std::string& m = cfg_.kserve_model;
  const std::string mpre = "/v2/models/" + m;
  auto err_json = [](const std::string& msg) {
    std::string s = "{\"error\":";
    json_escape(s, msg);
    return s + "}";
  };
  if (method == "GET") {
    if (path == "/v2/health/live") {
      respond(c, 200, "application/json", "{\"live\":true}");
      return true;
    }
    if (path == "/v2/health/ready" || path == mpre + "/ready" || path == mpre + "/versions/1/ready") {
      const bool ok = healthy_.load();
      respond(c, ok ? 200 : 503, "application/json", ok ? "{\"ready\":true}" : "{\"ready\":false}");
      return true;
    }
    if (path == "/v2") {
      respond(c, 200, "application/json",
              "{\"name\":\"arena-modelserver-native\",\"version\":\"2.0.0\",\"extensions\":[\"binary_tensor_data\"]}");
      return true;
    }
    if (path == mpre || path == mpre + "/versions/1") {
      respond(c, 200, "application/json", kserve_model_metadata(m));
      return true;
    }
    return false;
  }
  if (method != "POST") return false;
  const bool infer = path == mpre + "/infer" || path == mpre + "/versions/1/infer";
  if (!infer) {
    if (path.size() > 6 && path.compare(path.size() - 6, 6, "/infer") == 0) {
      respond(c, 404, "application/json", err_json("Request for unknown model: '" + path + "' is not found"));
      return true;
    }
    return false;
  }
  const auto t0 = Clock::now();
  size_t off = 0, len = 0;
  std::string err;
  if (!healthy_.load()) {
    fail_request(c, 503, "Server not ready", 1);
    return true;
  }
  if (!kserve_parse_bytes_input(body, ihcl, "IMAGE_BYTES", off, len, err) || len == 0) {
    fail_request(c, 400, err.empty() ? "empty IMAGE_BYTES" : err, 1);
    return true;
  }
  t_predict_dispatched = true;
  start_upload(c, t0, std::move(body), off, len, 1);
  return true;
}

std::vector<int64_t> HttpFrontEnd::upstream_forwarded() const {
  std::vector<int64_t> v;
  if (proxy_)
    for (int i = 0; i < proxy_->num_upstreams(); ++i) v.push_back(proxy_->forwarded_to(i));
  return v;
}

void HttpFrontEnd::proxy_predict(const std::shared_ptr<Conn>& c, Clock_tp t0, std::string upload) {
  const auto t_inf = Clock::now();
  {
    std::lock_guard<std::mutex> lk(cb_mu_);
    ++cb_outstanding_;
  }
  proxy_->submit(std::move(upload), [this, c, t0, t_inf](ProxyReply&& rep) {
    struct Done {
      HttpFrontEnd* f;
      ~Done() { f->callback_done(); }
    } done{this};
    if (rep.status != 200 || !rep.error.empty()) {
      const int code = rep.status == 0 ? 502 : rep.status == 200 ? 502 : rep.status;
      fail_request(c, code, "model server: " + (rep.error.empty() ? std::string("error") : rep.error));
      return;
    }
    const double cj = thread_cpu_ms();
    const RequestResult& r = rep.result;
    const double inference_ms = ms_since(t_inf);
    const double queue_ms = r.queue_us / 1e3, gpu_ms = r.compute_us / 1e3;
    const double det_ms = r.det_ms >= 0 ? r.det_ms : 0.0, cls_ms = r.cls_ms >= 0 ? r.cls_ms : 0.0;
    const double total_ms = ms_since(t0);
    const std::string s = predict_json(r, labels_, cfg_.softmax_confidence, queue_ms, gpu_ms, det_ms, cls_ms,
                                       inference_ms, 0.0, total_ms);
    record_ok(total_ms, 0.0, queue_ms, gpu_ms, det_ms, cls_ms, (int64_t)r.det.size(), thread_cpu_ms() - cj);
    respond(c, 200, "application/json", s);
  });
}

void HttpFrontEnd::submit_local(std::string upload, LocalDone done) {
  auto c = std::make_shared<Conn>();
  c->local = std::move(done);
  c->busy = true;
  const auto t0 = Clock::now();
  if (upload.empty()) return fail_request(c, 422, "empty request body");
  if (cfg_.decode_threads <= 0) return pool_submit(c, t0, upload, 0, upload.size());
  auto t = std::make_unique<DecodeTask>();
  t->conn = c;
  t->t0 = t0;
  t->t_queued = t0;
  t->len = upload.size();
  t->body = std::move(upload);
  {
    std::lock_guard<std::mutex> lk(dq_mu_);
    dq_.push_back(std::move(t));
  }
  dq_cv_.notify_one();
}

LocalLoadGen::LocalLoadGen(HttpFrontEnd* fe, std::vector<std::string> uploads, int users)
    : fe_(fe), uploads_(std::move(uploads)), users_(std::max(1, users)) {
  if (uploads_.empty()) throw std::runtime_error("LocalLoadGen: no uploads");
}

LocalLoadGen::~LocalLoadGen() { stop(30.0); }

void LocalLoadGen::start() {
  t0_ = Clock::now();
  issuing_.store(true);
  for (int i = 0; i < users_; ++i) issue();
}

void LocalLoadGen::issue() {
  if (!issuing_.load()) return;
  const int64_t k = next_.fetch_add(1);
  in_flight_.fetch_add(1);
  const auto t_send = Clock::now();
  fe_->submit_local(uploads_[(size_t)(k % (int64_t)uploads_.size())], [this, t_send](int code, const std::string& body) {
    LoadGenRecord r;
    const auto now = Clock::now();
    r.t_done = std::chrono::duration<double>(now - t0_).count();
    r.latency = (float)std::chrono::duration<double>(now - t_send).count();
    r.status = (int16_t)code;
    int n = 0;
    for (size_t p = body.find("\"class_name\""); p != std::string::npos; p = body.find("\"class_name\"", p + 1)) ++n;
    r.dets = (int16_t)n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      recs_.push_back(r);
    }
    cv_.notify_all();
    // a synchronous failure would recurse through issue() -> submit_local -> this callback: cap the depth
    thread_local int depth = 0;
    if (depth < 16) {
      ++depth;
      issue();
      --depth;
    }
    std::lock_guard<std::mutex> lk(mu_);  // stop() / the destructor cannot return before this unlocks
    in_flight_.fetch_sub(1);
    cv_.notify_all();
  });
}

void LocalLoadGen::stop(double timeout_s) {
  issuing_.store(false);
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), [this] { return in_flight_.load() == 0; });
}

int64_t LocalLoadGen::completed() {
  std::lock_guard<std::mutex> lk(mu_);
  return (int64_t)recs_.size();
}

bool LocalLoadGen::wait_completed(int64_t n, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  return cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return (int64_t)recs_.size() >= n; });
}

std::vector<LoadGenRecord> LocalLoadGen::records(int64_t from, int64_t to) {
  std::lock_guard<std::mutex> lk(mu_);
  from = std::max<int64_t>(0, from);
  to = to < 0 ? (int64_t)recs_.size() : std::min<int64_t>((int64_t)recs_.size(), to);
  if (to <= from) return {};
  return std::vector<LoadGenRecord>(recs_.begin() + from, recs_.begin() + to);
}

void HttpFrontEnd::fail_request(const std::shared_ptr<Conn>& c, int code, const std::string& msg, int kind) {
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++stats_.requests;
    if (code == 413) ++stats_.too_large;
    else if (code == 503) ++stats_.unavailable;
    else if (code >= 500) ++stats_.errors;
    else ++stats_.bad_request;
  }
  if (kind == 1) {  // KServe error body
    std::string e = "{\"error\":";
    json_escape(e, msg);
    respond(c, code, "application/json", e + "}");
    return;
  }
  respond(c, code, "application/json", detail_json(msg));
}

void HttpFrontEnd::pool_submit(const std::shared_ptr<Conn>& c, Clock_tp t0, const std::string& body, size_t off,
                               size_t len, int kind) {
  if (!has_pool_)
    return fail_request(c, 500, "Failed to decode image: format not supported by the native decoder", kind);
  int slot;
  {
    std::lock_guard<std::mutex> lk(slot_mu_);
    if (free_slots_.empty()) slot = -1;
    else {
      slot = free_slots_.back();
      free_slots_.pop_back();
    }
  }
  if (slot < 0) return fail_request(c, 503, "decode pool is saturated", kind);
  auto pend = std::make_shared<Pending>();
  pend->conn = c;
  pend->kind = kind;
  pend->t0 = t0;
  pend->t_dec = Clock::now();
  const uint64_t key = next_key_.fetch_add(1);
  // task record (server/decode_pool.py _TASK "<qii": key, slot, payload length or -1 = inline)
  struct __attribute__((packed)) Task {
    int64_t key;
    int32_t slot, n;
  } task{(int64_t)key, slot, (int32_t)len};
  std::string msg;
  if ((int64_t)len <= dc_.in_bytes) {
    std::memcpy(dc_.shm + (size_t)slot * dc_.stride, body.data() + off, len);
    msg.assign((const char*)&task, sizeof task);
  } else {
    task.n = -1;
    msg.assign((const char*)&task, sizeof task);
    msg.append(body, off, len);
  }
  int w = 0;
  for (int i = 1; i < (int)load_.size(); ++i)
    if (load_[i].load() < load_[w].load()) w = i;
  load_[w].fetch_add(1);
  pend->worker = w;
  {
    std::lock_guard<std::mutex> lk(pend_mu_);
    pending_[key] = pend;
  }
  const uint32_t be = htonl((uint32_t)msg.size());  // multiprocessing Connection framing
  bool ok;
  {
    std::lock_guard<std::mutex> lk(*task_mu_[w]);
    ok = write_all(dc_.task_fds[w], &be, 4) && write_all(dc_.task_fds[w], msg.data(), msg.size());
  }
  if (!ok) {
    load_[w].fetch_sub(1);
    {
      std::lock_guard<std::mutex> lk(pend_mu_);
      pending_.erase(key);
    }
    release_slot(slot);
    return fail_request(c, 503, "decode workers unavailable", kind);
  }
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++stats_.fallback_decoded;
  }
  // the worker's load is released when its completion record arrives (finish_decode)
}

void HttpFrontEnd::decode_loop(int idx) {
  pthread_setname_np(pthread_self(), "arena-jpeg");
  (void)idx;
  for (;;) {
    std::unique_ptr<DecodeTask> t;
    {
      std::unique_lock<std::mutex> lk(dq_mu_);
      dq_cv_.wait(lk, [this] { return stop_.load() || !dq_.empty(); });
      if (stop_.load()) return;
      t = std::move(dq_.front());
      dq_.pop_front();
    }
    native_decode(*t);
    bodies_.put(std::move(t->body));  // back to the I/O threads' next requests, not to this thread's allocator
  }
}

void HttpFrontEnd::native_decode(DecodeTask& t) {
  const double c0 = thread_cpu_ms();
  const uint8_t* data = (const uint8_t*)t.body.data() + t.off;
  auto up = std::make_shared<NativeUpload>();
  std::string err;
  JpegStatus st = jpeg_parse(data, t.len, up->info, err, cfg_.max_image_pixels);
  if (st == JpegStatus::Unsupported) return pool_submit(t.conn, t.t0, t.body, t.off, t.len, t.kind);  // PIL fallback
  if (st == JpegStatus::Corrupt)
    return fail_request(t.conn, err.find("image too large") != std::string::npos ? 413 : 500, err, t.kind);
  const JpegInfo& ji = up->info;
  InputImage in{nullptr, ji.height, ji.width};
  // Device reconstruction needs the coefficients, the sample planes and the RGB frame in one batch's staging
  // pool (staged_bytes) and the coefficients in one pooled buffer.  A frame too large for either (about
  // > 15 MP at 4:2:0 with the default pool) is reconstructed on the host instead and staged as RGB, as the PIL
  // path would stage it: the split decoder never turns away an upload the reference's decoder accepts.
  const int64_t cap = batcher_->staging_cap();
  InputImage probe = in;
  probe.jpeg = &ji;
  bool device = cfg_.jpeg_device && (cap <= 0 || staged_bytes(probe) <= cap);
  // compact coefficients (ARENA_JPEG_COMPACT, default 1): about a third of the dense blocks' bytes at q90, so a
  // third of the pack copy and of the batch's H2D
  const bool compact = jpeg_compact_enabled();
  if (device) {
    up->buf = host_pool_->get(compact ? (size_t)jpeg_compact_capacity(ji) : (size_t)ji.coef_count * 2);
    device = (bool)up->buf;
  }
  if (device) {
    st = compact ? jpeg_decode_compact(data, t.len, up->info, up->buf.get(), err)
                 : jpeg_decode_coefs(data, t.len, ji, (int16_t*)up->buf.get(), err);
    in.data = up->buf.get();
    in.jpeg = &up->info;
  } else {
    thread_local std::vector<int16_t> coef;
    coef.resize((size_t)ji.coef_count);
    st = jpeg_decode_coefs(data, t.len, ji, coef.data(), err);
    if (st == JpegStatus::Ok) {
      const size_t rgb_bytes = (size_t)ji.width * ji.height * 3;
      up->buf = host_pool_->get(rgb_bytes);
      if (!up->buf) {  // beyond the largest size class or the pool's cap: a buffer of its own
        uint8_t* raw = static_cast<uint8_t*>(std::malloc(rgb_bytes));
        if (raw == nullptr) return fail_request(t.conn, 503, "decode buffers exhausted", t.kind);
        up->buf = std::shared_ptr<uint8_t>(raw, [](uint8_t* q) { std::free(q); });
      }
      jpeg_coefs_to_rgb(ji, coef.data(), up->buf.get());
      in.data = up->buf.get();
    }
    if (coef.capacity() > ((size_t)16 << 20)) std::vector<int16_t>().swap(coef);  // do not pin a huge frame's
  }
  if (st != JpegStatus::Ok) return fail_request(t.conn, 500, err, t.kind);
  const double decode_ms = ms_since(t.t_queued);
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++stats_.native_decoded;
    stats_.cpu_decode_ms += thread_cpu_ms() - c0;
  }
  {
    std::lock_guard<std::mutex> lk(cb_mu_);
    ++cb_outstanding_;
  }
  const int64_t id = batcher_->enqueue_input(in, up, make_result_cb(t.conn, t.t0, Clock::now(), decode_ms, t.kind));
  if (id < 0) callback_done();  // rejected: the batcher never calls back
  if (id == -1) return fail_request(t.conn, 503, "request queue is full", t.kind);
  if (id == -2) return fail_request(t.conn, 413, "image exceeds the staging capacity of one batch", t.kind);
}

void HttpFrontEnd::collector_loop() {
  pthread_setname_np(pthread_self(), "arena-collect");
  // completion record (server/decode_pool.py _DONE "<qiiiiq": key, slot, h, w, status, aux)
  struct __attribute__((packed)) Done {
    int64_t key;
    int32_t slot, h, w, status;
    int64_t aux;
  };
  static_assert(sizeof(Done) == 32, "completion record is 32 bytes");
  Done d;
  while (read_all(dc_.result_fd, &d, sizeof d)) {
    if (d.key < 0 || stop_.load()) break;
    finish_decode((uint64_t)d.key, d.slot, d.h, d.w, d.status, d.aux);
  }
}

void HttpFrontEnd::record_ok(double total_ms, double decode_ms, double queue_ms, double gpu_ms, double det_ms,
                             double cls_ms, int64_t n_det, double json_cpu_ms) {
  std::lock_guard<std::mutex> sl(stats_mu_);
  ++stats_.requests;
  ++stats_.ok;
  stats_.cpu_json_ms += json_cpu_ms;
  stats_.detections += n_det;
  stats_.sum_total_ms += total_ms;
  stats_.sum_decode_ms += decode_ms;
  stats_.sum_queue_ms += queue_ms;
  stats_.sum_gpu_ms += gpu_ms;
  size_t b = 0;
  while (b < kLatencyBucketsMs.size() && total_ms > kLatencyBucketsMs[b]) ++b;
  ++stats_.latency_hist[b];
  const double stage_ms[] = {decode_ms, queue_ms, gpu_ms, det_ms, cls_ms, total_ms};
  for (size_t k = 0; k < kStages.size(); ++k) {
    size_t bb = 0;
    while (bb < kLatencyBucketsMs.size() && stage_ms[k] > kLatencyBucketsMs[bb]) ++bb;
    ++stats_.stage_hist[k][bb];
    stats_.stage_sum_ms[k] += stage_ms[k];
  }
}

ResultCallback HttpFrontEnd::make_result_cb(const std::shared_ptr<Conn>& conn, Clock_tp t0, Clock_tp t_inf,
                                            double decode_ms, int kind) {
  HttpFrontEnd* self = this;
  return [self, conn, t0, t_inf, decode_ms, kind](RequestResult&& r) {
    struct Done {
      HttpFrontEnd* f;
      ~Done() { f->callback_done(); }
    } done{self};
    if (!r.error.empty()) {
      self->fail_request(conn, 500, r.error, kind);
      return;
    }
    const double queue_ms = r.queue_us / 1e3, gpu_ms = r.compute_us / 1e3;
    const double inference_ms = ms_since(t_inf);
    // device time of the detection network (+ decode / NMS / crop plan) and of the classification network
    // (crop gather -> top-5) of this request's batch, from the program's wall-clock stamps (OP_STAMP); with
    // the batch's H2D / D2H they make up gpu_ms (reference timing keys, architectures/monolithic/app/
    // inference.py:180,224-225; there the per-request CPU time of each network)
    const double det_ms = r.det_ms >= 0 ? r.det_ms : 0.0, cls_ms = r.cls_ms >= 0 ? r.cls_ms : 0.0;
    const double cj = thread_cpu_ms();
    if (kind == 1) {  // KServe infer: the ensemble's output tensors (binary tensor extension)
      int64_t ihcl = -1;
      const std::string body = kserve_build_response(self->cfg_.kserve_model, "", r, true, &ihcl);
      const double total_ms = ms_since(t0);
      self->record_ok(total_ms, decode_ms, queue_ms, gpu_ms, det_ms, cls_ms, (int64_t)r.det.size(),
                      thread_cpu_ms() - cj);
      self->respond(conn, 200, "application/octet-stream", body, false,
                    "Inference-Header-Content-Length: " + std::to_string(ihcl) + "\r\n");
      return;
    }
    const double total_ms = ms_since(t0);
    const std::string s = predict_json(r, self->labels_, self->cfg_.softmax_confidence, queue_ms, gpu_ms, det_ms,
                                       cls_ms, inference_ms, decode_ms, total_ms);
    self->record_ok(total_ms, decode_ms, queue_ms, gpu_ms, det_ms, cls_ms, (int64_t)r.det.size(),
                    thread_cpu_ms() - cj);
    self->respond(conn, 200, "application/json", s);
  };
}

void HttpFrontEnd::finish_decode(uint64_t key, int slot, int h, int w, int status, int64_t aux) {
  std::shared_ptr<Pending> pend;
  {
    std::lock_guard<std::mutex> lk(pend_mu_);
    auto it = pending_.find(key);
    if (it != pending_.end()) {
      pend = it->second;
      pending_.erase(it);
    }
  }
  if (pend) load_[pend->worker].fetch_sub(1);
  const uint8_t* out = dc_.shm + (size_t)slot * dc_.stride + dc_.in_bytes;
  std::vector<uint8_t> big;
  if (status == 2) {  // oversize result on worker `aux`'s pipe: Connection framing (4-byte BE length)
    const int fd = dc_.big_fds[(size_t)aux];
    uint32_t be = 0;
    if (read_all(fd, &be, 4)) {
      int64_t n = (int32_t)ntohl(be);
      if (n == -1) {
        uint64_t be8 = 0;
        read_all(fd, &be8, 8);
        n = (int64_t)__builtin_bswap64(be8);
      }
      big.resize((size_t)std::max<int64_t>(n, 0));
      read_all(fd, big.data(), big.size());
    }
    out = big.data();
  }
  if (!pend) {
    release_slot(slot);
    return;
  }
  auto conn = pend->conn;
  auto fail = [&](int code, const std::string& msg) {
    {
      std::lock_guard<std::mutex> sl(stats_mu_);
      ++stats_.requests;
      if (code == 413) ++stats_.too_large;
      else if (code == 503) ++stats_.unavailable;
      else ++stats_.errors;
    }
    if (pend->kind == 1) {
      std::string e = "{\"error\":";
      json_escape(e, msg);
      respond(conn, code, "application/json", e + "}");
      return;
    }
    respond(conn, code, "application/json", detail_json(msg));
  };
  if (status == 1) {
    const std::string text((const char*)out, (size_t)std::max<int64_t>(0, std::min<int64_t>(aux, dc_.slot_bytes)));
    release_slot(slot);
    // a header declaring more pixels than the decoder accepts (processing/transforms.py ImageTooLargeError)
    return fail(text.find("image too large") != std::string::npos ? 413 : 500, text);
  }
  if (status == 2 && big.size() != (size_t)h * w * 3) {
    release_slot(slot);
    return fail(500, "decode worker result lost");
  }
  const double decode_ms = ms_since(pend->t_dec);
  ResultCallback cb = make_result_cb(conn, pend->t0, Clock::now(), decode_ms, pend->kind);
  {
    std::lock_guard<std::mutex> lk(cb_mu_);
    ++cb_outstanding_;
  }
  const int64_t id = batcher_->enqueue(out, h, w, std::move(cb));
  release_slot(slot);  // the batcher copied the pixels
  if (id < 0) callback_done();  // rejected: the batcher never calls back
  if (id == -1) return fail(503, "request queue is full");
  if (id == -2) return fail(413, "image exceeds the staging capacity of one batch");
}

}  // namespace arena
