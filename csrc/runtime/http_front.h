// Native HTTP/1.1 front end for the monolithic arm: POST /predict end to end
// without the Python request path.
//
// The reference serves /predict from FastAPI (architectures/monolithic/app/
// main.py:120-190: multipart upload -> cv2 decode -> ONNX detection ->
// crops -> ONNX classification -> JSON).  The Python port of that handler
// (server/monolithic.py) measured ~0.7-1.4 ms of interpreter time per request
// (h11 parsing, starlette/fastapi dispatch, pydantic, logging; tools/
// http_overhead.py), which capped one serving process far below the engine.
// Here the whole request path is C++:
//
//   epoll I/O threads: accept, HTTP/1.1 keep-alive parsing (Content-Length or
//   chunked), multipart/form-data field "file" or a raw image body
//     -> native decode (FrontConfig.decode_threads > 0, the default of the serving
//        paths): the upload goes to a pool of C++ decode threads running the host
//        half of the split JPEG decoder (runtime/jpeg_decode.h): marker parse +
//        Huffman decode straight into a pinned buffer of the HostBufferPool
//        (runtime/host_pool.h) -> DynamicBatcher::enqueue_input, zero-copy; the
//        executor DMAs the coefficients and reconstructs the frame on the GPU
//        (kernels/jpeg_idct.hip).  Uploads the split decoder does not cover
//        (progressive JPEG, PNG, ...) fall through to:
//     -> the PIL decode pool: the bytes go into a slot of the pool's shared memory
//        and a 16-byte task record to the least-loaded decode worker (the spawned
//        PIL processes of server/decode_pool.py)
//   collector thread: completion records from the workers' shared pipe
//     -> DynamicBatcher::enqueue straight from the shared-memory pixels
//   batcher instance threads: results
//     -> the reference's JSON schema (request_id, detections[{detection,
//        classification}], timing) -> the connection's I/O thread writes it.
//
// Handler mode (FrontConfig.handler_mode, no batcher / decode channel): the
// same HTTP/1.1 + multipart layer in front of a Python topology whose request
// path is not one batcher (microservices detection service, model-server
// gateway).  predict() queues (key, upload bytes); the owner drains the queue
// with take() (GIL released while waiting), runs its async handler and hands
// the finished JSON back with complete(key, status, body).  The Python HTTP
// stack (uvicorn/h11 + starlette + multipart parsing, ~0.7-1.4 ms of
// interpreter time per request) is what capped those arms' processes.
//
// GET /health (503 once set_healthy(false)), GET /metrics (text supplied by
// the Python owner, which renders Prometheus from stats()).  Errors follow the
// FastAPI handler: 422 bad upload, 413 too large, 503 queue full / not ready,
// 500 decode or device failure, each with {"detail": ...}.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "batcher.h"
#include "kserve.h"
#include "host_pool.h"
#include "http_loadgen.h"
#include "string_pool.h"

namespace arena {

// The decode pool's transport (server/decode_pool.py ProcessDecodePool): shared memory of `slots` slots of
// `stride` bytes (upload region of `in_bytes`, then the decoded pixels), one task pipe per worker
// (multiprocessing Connection framing: 4-byte big-endian length + payload), the workers' shared completion
// pipe (raw 32-byte records) and its write end (to wake the collector on stop), one pipe per worker for
// oversize results (Connection framing).
struct DecodeChannel {
  uint8_t* shm = nullptr;
  int64_t stride = 0, in_bytes = 0, slot_bytes = 0;
  int slots = 0;
  std::vector<int> task_fds, big_fds;
  int result_fd = -1, result_wfd = -1;
};

struct FrontConfig {
  std::string host = "0.0.0.0";
  int port = 8100;
  int io_threads = 4;
  bool reuse_port = true;
  bool softmax_confidence = false;  // ARENA_CONFIDENCE=softmax (default: the top-1 logit, as the reference)
  int64_t max_body = 64 << 20;
  std::string replica_tag;  // non-empty: an "x-arena-replica" header on every response (server/replica.py)
  bool handler_mode = false;  // uploads go to take() / complete() instead of decode pool + batcher
  int max_handler_queue = 4096;  // queued + in-handler requests before 503
  // A keep-alive connection with nothing in flight and no bytes received for idle_timeout_ms is closed; so is
  // one whose request has been arriving for longer than read_timeout_ms (a client trickling its headers or
  // body would otherwise hold a descriptor and its buffer forever).  0 disables the check.
  int64_t idle_timeout_ms = 60000;
  int64_t read_timeout_ms = 30000;
  // Native decode threads (0: every upload goes to the PIL decode pool of the DecodeChannel).
  int decode_threads = 0;
  // true: split decode (host Huffman -> device reconstruction); false: the whole decode on the host threads
  // (same arithmetic, RGB staged like a PIL decode) — for instances without the device half and for A/B runs.
  bool jpeg_device = true;
  int64_t max_image_pixels = 50000000;     // decode-bomb guard (processing/transforms.py max_image_pixels)
  int64_t decode_buffer_cap = 2LL << 30;   // host buffers of decoded uploads in flight (HostBufferPool cap)
  HostBufferPool::AllocFn host_alloc;      // pinning allocator for those buffers (empty: plain memory)
  HostBufferPool::FreeFn host_free;
  // KServe-v2 REST for this ensemble model (runtime/kserve.h; empty: off): POST /v2/models/<m>/infer with the
  // binary tensor extension takes the /predict path and answers the ensemble's output tensors; GET /v2,
  // /v2/health/{live,ready}, /v2/models/<m>[/ready] answer the protocol's metadata / health routes
  std::string kserve_model;
  // Native gateway ("proxy mode", upstream_port > 0): /predict uploads are forwarded to a model server's KServe
  // endpoint over upstream_conns keep-alive connections and its output tensors answered as the reference JSON;
  // no batcher or decoder in this process
  std::string upstream_host = "127.0.0.1";
  int upstream_port = 0;
  std::string upstream_model = "arena_pipeline";
  int upstream_conns = 64;
  // more model servers ("host:port,host:port", e.g. one per GPU): with it the proxy spreads requests over
  // upstream_host:upstream_port and these, least-outstanding first (KServeProxy)
  std::string upstreams;
};

// One upload handed to the Python handler (handler mode).
struct HandlerRequest {
  uint64_t key = 0;
  std::string data;  // the multipart "file" field (or the raw body)
};

struct FrontStats {
  int64_t requests = 0, ok = 0, bad_request = 0, too_large = 0, unavailable = 0, errors = 0, not_found = 0;
  int64_t connections = 0, open_connections = 0, detections = 0, timeouts = 0;
  int64_t native_decoded = 0, fallback_decoded = 0;  // uploads decoded by the split decoder / the PIL pool
  int64_t bodies_recycled = 0, bodies_allocated = 0;  // request bodies served by the body pool / newly grown
  double sum_total_ms = 0, sum_decode_ms = 0, sum_queue_ms = 0, sum_gpu_ms = 0;
  // host CPU time (thread CPU clock) of request stages, summed: HTTP + multipart parse on the I/O threads, the
  // native decode (marker parse + entropy decode), the JSON response built in the batcher callback
  double cpu_parse_ms = 0, cpu_decode_ms = 0, cpu_json_ms = 0;
  std::vector<int64_t> latency_hist;  // counts per bucket of kLatencyBucketsMs (last = +Inf)
  // per-stage latency histograms of the successful requests (arena_request_latency_seconds{stage=...}):
  // kStages order, each counts per bucket of kLatencyBucketsMs (last = +Inf), with its sum in ms
  std::vector<std::vector<int64_t>> stage_hist;
  std::vector<double> stage_sum_ms;
};

// decode, queue (dynamic batcher), gpu (batch submit -> results), detection / classification (device time of
// the two networks, from the program's wall-clock stamps), total (request received -> response queued)
extern const std::vector<std::string> kStages;

extern const std::vector<double> kLatencyBucketsMs;

class HttpFrontEnd;

// Closed-loop in-process users of HttpFrontEnd::submit_local (the HTTP layer left out): `users` requests in
// flight, each completion issues the next upload (round robin over `uploads`).  Same record format as the HTTP
// load generator (http_loadgen.h).
class LocalLoadGen {
 public:
  LocalLoadGen(HttpFrontEnd* fe, std::vector<std::string> uploads, int users);
  ~LocalLoadGen();
  void start();
  void stop(double timeout_s = 30.0);
  int64_t completed();
  bool wait_completed(int64_t n, double timeout_s);
  std::vector<LoadGenRecord> records(int64_t from, int64_t to);

 private:
  void issue();
  HttpFrontEnd* fe_;
  std::vector<std::string> uploads_;
  int users_;
  std::atomic<bool> issuing_{false};
  std::atomic<int64_t> next_{0}, in_flight_{0};
  std::chrono::steady_clock::time_point t0_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<LoadGenRecord> recs_;
};

class HttpFrontEnd {
 public:
  HttpFrontEnd(DynamicBatcher* batcher, DecodeChannel dc, std::vector<std::string> labels, FrontConfig cfg);
  ~HttpFrontEnd();
  HttpFrontEnd(const HttpFrontEnd&) = delete;
  HttpFrontEnd& operator=(const HttpFrontEnd&) = delete;

  int port() const { return port_; }
  void set_healthy(bool h) { healthy_.store(h); }
  void set_metrics_text(std::string text);
  FrontStats stats();
  // proxy mode: requests forwarded to each upstream so far (empty otherwise)
  std::vector<int64_t> upstream_forwarded() const;
  void stop();

  // handler mode: up to max_n queued uploads; waits up to timeout_ms for the first one (empty on timeout / stop)
  std::vector<HandlerRequest> take(int max_n, int timeout_ms);
  // handler mode: answer request `key` (status code, JSON body); n_det counts into the detections total.
  // Returns false when the key is unknown (connection gone, already answered).
  bool complete(uint64_t key, int code, const std::string& body, int n_det = 0);
  bool handler_mode() const { return cfg_.handler_mode; }
  // Stop accepting: the listening socket leaves the epoll sets and is shut down (Linux unhashes it, so an
  // SO_REUSEPORT group stops routing new connections here); open connections keep being served.
  void drain();
  // handler mode: requests queued or inside the Python handler
  int handler_pending();
  // In-process request (no socket, no HTTP parse): `upload` takes the /predict path from the decode stage on
  // (split decoder or PIL pool, batcher, device, JSON) and `done(status, json)` receives what a client would.
  // Drives LocalLoadGen, the control that isolates the cost of the HTTP layer.
  using LocalDone = std::function<void(int, const std::string&)>;
  void submit_local(std::string upload, LocalDone done);

  struct Conn;
  struct Pending;
  using Clock_tp = std::chrono::steady_clock::time_point;

 private:
  void io_loop(int idx);
  void collector_loop();
  void handle_readable(int ep, const std::shared_ptr<Conn>& c);
  void handle_writable(int ep, const std::shared_ptr<Conn>& c);
  bool parse_one(const std::shared_ptr<Conn>& c);  // true: a full request was consumed
  bool parse_one_impl(const std::shared_ptr<Conn>& c);
  void dispatch(const std::shared_ptr<Conn>& c, const std::string& method, const std::string& path,
                const std::string& ctype, std::string&& body, int64_t ihcl = -1);
  void predict(const std::shared_ptr<Conn>& c, std::string&& body, const std::string& ctype);
  bool kserve_route(const std::shared_ptr<Conn>& c, const std::string& method, const std::string& path,
                    std::string&& body, int64_t ihcl);
  void start_upload(const std::shared_ptr<Conn>& c, Clock_tp t0, std::string&& body, size_t off, size_t len,
                    int kind);
  void proxy_predict(const std::shared_ptr<Conn>& c, Clock_tp t0, std::string upload);
  void record_ok(double total_ms, double decode_ms, double queue_ms, double gpu_ms, double det_ms, double cls_ms,
                 int64_t n_det, double json_cpu_ms);
  void respond(const std::shared_ptr<Conn>& c, int code, const std::string& ctype, const std::string& body,
               bool count_latency = false, const std::string& extra_headers = "");
  void close_conn(int ep, const std::shared_ptr<Conn>& c);
  void finish_decode(uint64_t key, int slot, int h, int w, int status, int64_t aux);
  struct DecodeTask;
  void decode_loop(int idx);
  void native_decode(DecodeTask& t);
  // hand an upload to the PIL decode pool (also the split decoder's fallback); answers the error itself
  // kind: 0 = /predict (reference JSON), 1 = KServe infer (binary output tensors)
  void pool_submit(const std::shared_ptr<Conn>& c, Clock_tp t0, const std::string& body, size_t off, size_t len,
                   int kind = 0);
  ResultCallback make_result_cb(const std::shared_ptr<Conn>& c, Clock_tp t0, Clock_tp t_inf, double decode_ms,
                                int kind = 0);
  void fail_request(const std::shared_ptr<Conn>& c, int code, const std::string& msg, int kind = 0);
  void release_slot(int slot);
  void callback_done();

  DynamicBatcher* batcher_;
  // request bodies: filled on the I/O threads, released on the decode threads / proxy workers, recycled here
  // instead of freed (runtime/string_pool.h); declared before proxy_, so it outlives the proxy's workers
  StringPool bodies_;
  std::unique_ptr<KServeProxy> proxy_;  // proxy mode (cfg_.upstream_port > 0)
  DecodeChannel dc_;
  std::vector<std::string> labels_;
  FrontConfig cfg_;
  int listen_fd_ = -1, port_ = 0, stop_efd_ = -1;
  std::atomic<bool> stop_{false}, healthy_{true};
  std::vector<std::thread> io_threads_;
  std::thread collector_;
  std::vector<int> epfds_;

  std::mutex slot_mu_;
  std::vector<int> free_slots_;
  std::vector<std::unique_ptr<std::mutex>> task_mu_;
  std::vector<std::atomic<int>> load_;

  std::mutex pend_mu_;
  std::unordered_map<uint64_t, std::shared_ptr<Pending>> pending_;
  std::atomic<uint64_t> next_key_{1};

  // handler mode
  struct HandlerPending;
  std::mutex hq_mu_;
  std::condition_variable hq_cv_;
  std::deque<HandlerRequest> hq_;
  std::unordered_map<uint64_t, std::shared_ptr<HandlerPending>> hpend_;  // queued or in the handler

  std::mutex drain_mu_;
  bool drained_ = false;

  // native decode
  std::mutex dq_mu_;
  std::condition_variable dq_cv_;
  std::deque<std::unique_ptr<DecodeTask>> dq_;
  std::vector<std::thread> decode_threads_;
  std::shared_ptr<HostBufferPool> host_pool_;
  bool has_pool_ = false;  // a PIL decode channel is attached

  std::mutex metrics_mu_;
  std::string metrics_text_;
  std::mutex stats_mu_;
  FrontStats stats_;

  // batcher callbacks capture `this`: stop() waits for the ones still outstanding before tearing down
  std::mutex cb_mu_;
  std::condition_variable cb_cv_;
  int64_t cb_outstanding_ = 0;
};

}  // namespace arena
