// Closed-loop HTTP/1.1 load generator (native): the reference's load protocol is Locust users that each
// send one /predict upload, wait for the answer and send the next (reference experiment.yaml:178-181,
// 300-318; the locustfile itself is not in the reference).  bench.py and the serving sweeps drive the
// native front end with it over loopback: `users` keep-alive connections spread over a few epoll
// threads, pre-built request bytes (headers + multipart body), one completion record per response
// (latency, status, detections in the JSON), GIL-free waits.  A Python client pool cost about a core
// per 2-3k requests/s and competed with the server for the same CPUs.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace arena {

struct LoadGenConfig {
  std::string host = "127.0.0.1";
  int port = 8100;
  int users = 1;
  int threads = 1;
  int64_t max_requests = 0;  // stop issuing after this many (0 = until stop())
};

struct LoadGenRecord {
  double t_done = 0;   // seconds since start()
  float latency = 0;   // seconds, request sent -> response complete
  int16_t status = 0;  // HTTP status, or -1: connection failed / closed mid-request
  int16_t dets = 0;    // detections in the response body (occurrences of "class_name")
};

class HttpLoadGen {
 public:
  HttpLoadGen(LoadGenConfig cfg, std::vector<std::string> requests);
  ~HttpLoadGen();
  HttpLoadGen(const HttpLoadGen&) = delete;
  HttpLoadGen& operator=(const HttpLoadGen&) = delete;

  void start();
  // stop issuing new requests; waits up to timeout_s for the in-flight ones, then closes every connection
  void stop(double timeout_s = 30.0);
  int64_t completed();
  // waits until at least n responses completed (false on timeout or when every connection failed)
  bool wait_completed(int64_t n, double timeout_s);
  std::vector<LoadGenRecord> records(int64_t from, int64_t to);
  int64_t connect_failures() const { return connect_failures_.load(); }

  struct Conn;

 private:
  void loop(int idx);

  LoadGenConfig cfg_;
  std::vector<std::string> reqs_;
  std::vector<int> epfds_;
  std::vector<std::thread> threads_;
  std::atomic<bool> issuing_{false}, stop_{false};
  std::atomic<int64_t> next_req_{0}, in_flight_{0}, connect_failures_{0};
  std::atomic<int> live_conns_{0};
  double t0_ = 0;

  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<LoadGenRecord> recs_;
};

}  // namespace arena
