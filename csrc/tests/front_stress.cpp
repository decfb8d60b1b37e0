// Concurrency / robustness stress of the native HTTP front end (csrc/runtime/http_front.cpp) over the
// dynamic batcher and CPU EchoInstances, with in-process fake decode workers speaking the decode pool's
// pipe protocol (server/decode_pool.py: 16-byte task records with Connection framing, 32-byte completion
// records on one shared pipe, oversize results on a per-worker pipe).  Built and run under ThreadSanitizer
// and AddressSanitizer by tests/test_native_http.py (host code only; no GPU).
//
// Clients race the I/O threads, the collector and the batcher threads with:
//   * keep-alive request loops (raw and multipart bodies) whose answers are checked against the echo
//     instance's deterministic detections for the uploaded "image";
//   * pipelined bursts (several requests written before any answer is read);
//   * half-closed connections (shutdown(SHUT_WR) right after the request);
//   * oversized headers (431), malformed request lines (400), unknown paths (404), bodies the fake decoder
//     rejects (500 with its message) and results too large for a shared-memory slot (the worker's pipe);
//   * connections dropped mid-body and mid-response;
//   * drain() and then stop() while requests are still in flight;
// and a handler-mode front end (take() / complete() from two owner threads) under the same client mix.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/echo_instance.h"
#include "../runtime/http_front.h"

using namespace arena;

namespace {

std::atomic<int> fails{0};
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "CHECK failed: %s: ", #cond);   \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      fails.fetch_add(1);                                  \
    }                                                      \
  } while (0)

constexpr int kMaxDet = 4;

bool read_all(int fd, void* p, size_t n) {
  auto* c = (char*)p;
  while (n) {
    const ssize_t k = ::read(fd, c, n);
    if (k > 0) {
      c += k;
      n -= (size_t)k;
    } else if (k < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

bool write_all(int fd, const void* p, size_t n) {
  auto* c = (const char*)p;
  while (n) {
    const ssize_t k = ::write(fd, c, n);
    if (k > 0) {
      c += k;
      n -= (size_t)k;
    } else if (k < 0 && errno == EINTR) {
      continue;
    } else {
      return false;
    }
  }
  return true;
}

// Fake "image" upload: "FAKE" h(uint16) w(uint16) seed(uint8); the decoder fills h x w x 3 with seed.
std::string fake_image(int h, int w, uint8_t seed) {
  std::string s = "FAKE";
  s.push_back((char)(h & 0xff));
  s.push_back((char)(h >> 8));
  s.push_back((char)(w & 0xff));
  s.push_back((char)(w >> 8));
  s.push_back((char)seed);
  return s;
}

struct FakeDecodePool {
  DecodeChannel dc;
  std::vector<uint8_t> shm;
  std::vector<int> task_r, big_w;
  int result_r = -1, result_w = -1;
  std::vector<std::thread> workers;

  FakeDecodePool(int n_workers, int slots, int64_t in_bytes, int64_t slot_bytes) {
    dc.slots = slots;
    dc.in_bytes = in_bytes;
    dc.slot_bytes = slot_bytes;
    dc.stride = in_bytes + slot_bytes;
    shm.assign((size_t)(slots * dc.stride), 0);
    dc.shm = shm.data();
    int rp[2];
    if (pipe(rp) != 0) std::abort();
    result_r = rp[0];
    result_w = rp[1];
    dc.result_fd = result_r;
    dc.result_wfd = result_w;
    for (int i = 0; i < n_workers; ++i) {
      int tp[2], bp[2];
      if (pipe(tp) != 0 || pipe(bp) != 0) std::abort();
      dc.task_fds.push_back(tp[1]);
      task_r.push_back(tp[0]);
      dc.big_fds.push_back(bp[0]);
      big_w.push_back(bp[1]);
    }
    for (int i = 0; i < n_workers; ++i) workers.emplace_back([this, i] { work(i); });
  }

  void work(int idx) {
    struct __attribute__((packed)) Task {
      int64_t key;
      int32_t slot, n;
    };
    struct __attribute__((packed)) Done {
      int64_t key;
      int32_t slot, h, w, status;
      int64_t aux;
    };
    while (true) {
      uint32_t be = 0;
      if (!read_all(task_r[idx], &be, 4)) return;  // task pipe closed: the pool is shutting down
      std::string msg(ntohl(be), '\0');
      if (!read_all(task_r[idx], msg.data(), msg.size())) return;
      Task t;
      std::memcpy(&t, msg.data(), sizeof t);
      uint8_t* slot = dc.shm + (size_t)t.slot * dc.stride;
      std::string up = t.n >= 0 ? std::string((const char*)slot, (size_t)t.n) : msg.substr(sizeof t);
      Done d{t.key, t.slot, 0, 0, 0, 0};
      if (up.size() < 9 || up.compare(0, 4, "FAKE") != 0) {
        const std::string err = "cannot identify image file";
        std::memcpy(slot + dc.in_bytes, err.data(), err.size());
        d.status = 1;
        d.aux = (int64_t)err.size();
        write_all(result_w, &d, sizeof d);
        continue;
      }
      const int h = (uint8_t)up[4] | ((uint8_t)up[5] << 8), w = (uint8_t)up[6] | ((uint8_t)up[7] << 8);
      const uint8_t seed = (uint8_t)up[8];
      const size_t n = (size_t)h * w * 3;
      d.h = h;
      d.w = w;
      if ((int64_t)n <= dc.slot_bytes) {
        std::memset(slot + dc.in_bytes, seed, n);
        write_all(result_w, &d, sizeof d);
      } else {  // oversize: the record first, then the pixels with Connection framing on this worker's pipe
        d.status = 2;
        d.aux = idx;
        std::vector<uint8_t> px(n, seed);
        const uint32_t len = htonl((uint32_t)n);
        write_all(result_w, &d, sizeof d);
        write_all(big_w[idx], &len, 4);
        write_all(big_w[idx], px.data(), px.size());
      }
    }
  }

  // after the front end stopped: close the task pipes (workers exit), then every remaining descriptor
  void shutdown() {
    for (int fd : dc.task_fds) ::close(fd);
    for (auto& t : workers) t.join();
    for (int fd : task_r) ::close(fd);
    for (int fd : dc.big_fds) ::close(fd);
    for (int fd : big_w) ::close(fd);
    ::close(result_r);
    ::close(result_w);
  }
};

int connect_port(int port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
    ::close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  timeval tv{10, 0};  // a lost response fails the check instead of hanging the test
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  return fd;
}

std::string predict_request(const std::string& img, bool multipart) {
  std::string body, ctype;
  if (multipart) {
    const std::string b = "stressboundary42";
    body = "--" + b + "\r\nContent-Disposition: form-data; name=\"file\"; filename=\"x.jpg\"\r\n"
           "Content-Type: image/jpeg\r\n\r\n" + img + "\r\n--" + b + "--\r\n";
    ctype = "multipart/form-data; boundary=" + b;
  } else {
    body = img;
    ctype = "application/octet-stream";
  }
  return "POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: " + ctype +
         "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
}

// Reads one response; returns the status (-1: connection closed / timeout) and the body.
int read_response(int fd, std::string& buf, std::string& body) {
  char tmp[8192];
  while (true) {
    const size_t hend = buf.find("\r\n\r\n");
    if (hend != std::string::npos) {
      const int status = std::atoi(buf.c_str() + 9);
      size_t clen = 0;
      const size_t p = buf.find("Content-Length: ");
      if (p != std::string::npos && p < hend) clen = (size_t)std::atoll(buf.c_str() + p + 16);
      if (buf.size() >= hend + 4 + clen) {
        body = buf.substr(hend + 4, clen);
        buf.erase(0, hend + 4 + clen);
        return status;
      }
    }
    const ssize_t k = ::recv(fd, tmp, sizeof tmp, 0);
    if (k <= 0) return -1;
    buf.append(tmp, (size_t)k);
  }
}

int count_of(const std::string& s, const char* pat) {
  int n = 0;
  for (size_t p = s.find(pat); p != std::string::npos; p = s.find(pat, p + 1)) ++n;
  return n;
}

struct Tally {
  std::atomic<int64_t> ok{0}, checked{0}, errors{0}, closed{0};
};

// One client: a mix of the behaviours above, checking every answer it can attribute.
void client(int port, int id, int rounds, bool handler_mode, std::atomic<bool>& draining, Tally& t) {
  std::mt19937 rng(1234 + id);
  int fd = -1;
  std::string buf, body;
  auto reconnect = [&]() {
    if (fd >= 0) ::close(fd);
    buf.clear();
    fd = connect_port(port);
    return fd >= 0;
  };
  for (int r = 0; r < rounds; ++r) {
    if (fd < 0 && !reconnect()) {
      if (draining.load()) return;  // the listener is gone
      t.closed.fetch_add(1);
      continue;
    }
    const int kind = (int)(rng() % 100);
    const uint8_t seed = (uint8_t)(rng() % 251);
    const int expect_det = 1 + seed % kMaxDet;
    if (kind < 55) {  // keep-alive request, checked
      const bool big = rng() % 10 == 0;  // result larger than a shared-memory slot
      const std::string req = predict_request(fake_image(big ? 128 : 8 + (int)(rng() % 24), 16, seed), rng() % 2);
      if (!write_all(fd, req.data(), req.size())) { reconnect(); continue; }
      const int st = read_response(fd, buf, body);
      if (st < 0) { t.closed.fetch_add(1); reconnect(); continue; }
      if (st == 200) {
        t.ok.fetch_add(1);
        if (!handler_mode) {
          CHECK(count_of(body, "\"class_name\"") == expect_det, "detections %d != %d for seed %d: %s",
                count_of(body, "\"class_name\""), expect_det, seed, body.c_str());
          t.checked.fetch_add(1);
        }
      } else {
        CHECK(st == 503, "unexpected status %d: %s", st, body.c_str());
      }
    } else if (kind < 70) {  // pipelined burst of 3
      std::string reqs;
      uint8_t seeds[3];
      for (int k = 0; k < 3; ++k) {
        seeds[k] = (uint8_t)(rng() % 251);
        reqs += predict_request(fake_image(12, 12, seeds[k]), k == 1);
      }
      if (!write_all(fd, reqs.data(), reqs.size())) { reconnect(); continue; }
      for (int k = 0; k < 3; ++k) {
        const int st = read_response(fd, buf, body);
        if (st < 0) { t.closed.fetch_add(1); reconnect(); break; }
        if (st == 200 && !handler_mode) {
          CHECK(count_of(body, "\"class_name\"") == 1 + seeds[k] % kMaxDet,
                "pipelined answer %d out of order or wrong: %s", k, body.c_str());
          t.checked.fetch_add(1);
        }
        if (st == 200) t.ok.fetch_add(1);
      }
    } else if (kind < 75) {  // half-close after the request: the answer must still arrive
      const std::string req = predict_request(fake_image(10, 10, seed), false);
      write_all(fd, req.data(), req.size());
      ::shutdown(fd, SHUT_WR);
      const int st = read_response(fd, buf, body);
      CHECK(st == 200 || st == 503 || st == -1, "half-close status %d", st);
      if (st == 200) t.ok.fetch_add(1);
      reconnect();
    } else if (kind < 79) {  // oversized headers
      std::string req = "GET /health HTTP/1.1\r\nX-Big: " + std::string(70000, 'a') + "\r\n\r\n";
      write_all(fd, req.data(), req.size());
      const int st = read_response(fd, buf, body);
      CHECK(st == 431 || st == -1, "oversized headers status %d", st);
      reconnect();
    } else if (kind < 83) {  // malformed request line, unknown path
      const std::string req = rng() % 2 ? std::string("GARBAGE\r\n\r\n") : std::string("GET /nope HTTP/1.1\r\n\r\n");
      write_all(fd, req.data(), req.size());
      const int st = read_response(fd, buf, body);
      CHECK(st == 400 || st == 404 || st == -1, "malformed request status %d", st);
      reconnect();
    } else if (kind < 88) {  // a body the decoder rejects
      const std::string req = predict_request("NOTANIMAGE", rng() % 2);
      write_all(fd, req.data(), req.size());
      const int st = read_response(fd, buf, body);
      if (st < 0) { reconnect(); continue; }
      CHECK(st == 500 || st == 503 || (handler_mode && st == 200), "bad image status %d: %s", st, body.c_str());
      t.errors.fetch_add(1);
    } else if (kind < 93) {  // drop the connection mid-body
      const std::string req = predict_request(fake_image(20, 20, seed), false);
      write_all(fd, req.data(), req.size() / 2);
      reconnect();
    } else {  // drop the connection right after the request (the answer is discarded by the server)
      const std::string req = predict_request(fake_image(20, 20, seed), rng() % 2);
      write_all(fd, req.data(), req.size());
      reconnect();
    }
  }
  if (fd >= 0) ::close(fd);
}

void run_batcher_mode() {
  auto inst = std::make_shared<EchoInstance>(2, 8, kMaxDet, 300);
  BatcherConfig bc;
  bc.max_batch = 8;
  bc.max_queue_delay_us = 400;
  bc.max_queue_size = 256;
  auto batcher = std::make_unique<DynamicBatcher>(std::vector<std::shared_ptr<BatchInstance>>{inst}, bc);
  FakeDecodePool pool(3, 24, 4096, 16 * 16 * 3 * 8);  // 128 x 16 images overflow a slot
  FrontConfig cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.io_threads = 3;
  cfg.max_body = 1 << 20;
  cfg.idle_timeout_ms = 2000;
  cfg.read_timeout_ms = 2000;
  std::vector<std::string> labels(1000);
  for (size_t i = 0; i < labels.size(); ++i) labels[i] = "class" + std::to_string(i);
  auto front = std::make_unique<HttpFrontEnd>(batcher.get(), pool.dc, labels, cfg);
  const int port = front->port();
  std::atomic<bool> draining{false};
  Tally t;
  std::vector<std::thread> clients;
  for (int i = 0; i < 12; ++i) clients.emplace_back([&, i] { client(port, i, 150, false, draining, t); });
  std::thread stats_reader([&] {  // stats() and set_metrics_text() race the I/O threads
    for (int i = 0; i < 50; ++i) {
      front->set_metrics_text("# metrics " + std::to_string(i) + "\n");
      FrontStats s = front->stats();
      CHECK(s.ok <= s.requests, "stats ok %lld > requests %lld", (long long)s.ok, (long long)s.requests);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  draining.store(true);
  front->drain();  // new connections are refused; open ones keep being served
  for (auto& c : clients) c.join();
  stats_reader.join();
  front->stop();
  front.reset();
  batcher->shutdown();
  batcher.reset();
  pool.shutdown();
  CHECK(t.checked.load() > 50, "only %lld answers were checked", (long long)t.checked.load());
  std::printf("batcher mode: %lld ok, %lld checked, %lld decode errors, %lld closed\n", (long long)t.ok.load(),
              (long long)t.checked.load(), (long long)t.errors.load(), (long long)t.closed.load());
}

void run_handler_mode() {
  FrontConfig cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.io_threads = 2;
  cfg.handler_mode = true;
  cfg.max_handler_queue = 64;
  cfg.idle_timeout_ms = 2000;
  cfg.read_timeout_ms = 2000;
  auto front = std::make_unique<HttpFrontEnd>(nullptr, DecodeChannel{}, std::vector<std::string>{}, cfg);
  const int port = front->port();
  std::atomic<bool> stop{false}, draining{false};
  std::vector<std::thread> owners;
  for (int o = 0; o < 2; ++o)
    owners.emplace_back([&] {  // the Python owner's loop: take a few, answer each (some late, some twice)
      std::mt19937 rng(99);
      while (!stop.load()) {
        for (auto& r : front->take(8, 20)) {
          if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
          const bool ok = front->complete(r.key, 200, "{\"detections\": []}", 0);
          (void)ok;  // false when the client is gone
          CHECK(!front->complete(r.key, 200, "{}", 0), "key %llu answered twice", (unsigned long long)r.key);
        }
      }
    });
  Tally t;
  std::vector<std::thread> clients;
  for (int i = 0; i < 8; ++i) clients.emplace_back([&, i] { client(port, 100 + i, 120, true, draining, t); });
  for (auto& c : clients) c.join();
  front->drain();
  CHECK(front->handler_pending() >= 0, "pending count");
  stop.store(true);
  for (auto& o : owners) o.join();
  front->stop();
  front.reset();
  CHECK(t.ok.load() > 50, "handler mode answered only %lld", (long long)t.ok.load());
  std::printf("handler mode: %lld ok, %lld closed\n", (long long)t.ok.load(), (long long)t.closed.load());
}

}  // namespace

int main() {
  run_batcher_mode();
  run_handler_mode();
  if (fails.load() != 0) {
    std::printf("front_stress: %d failures\n", fails.load());
    return 1;
  }
  std::printf("front_stress: ok\n");
  return 0;
}
