// KServe-v2 REST with the binary tensor extension, for the "triton" arm's hot path
// (reference: architectures/triton/gateway/app/triton_client.py:70-144 calls Triton's ModelInfer; the arena
// gateway sends the whole upload to the model server's `arena_pipeline` ensemble in one request).
//
//   server side (HttpFrontEnd, FrontConfig.kserve_model): POST /v2/models/<model>[/versions/<v>]/infer with
//     `Inference-Header-Content-Length: n`, a JSON header naming one BYTES input IMAGE_BYTES
//     (parameters.binary_data_size) and its binary element (4-byte little-endian length + the encoded image);
//     the upload takes the /predict path (split decoder, dynamic batcher, device program) and the answer is the
//     ensemble's outputs DETECTIONS [n,6] FP32, CLASS_IDS [n,5] INT32, CLASS_LOGITS / CLASS_PROBS [n,5] FP32,
//     STAGE_MS [4] FP32 as binary tensors (JSON "data" arrays when the request carried no binary extension);
//   client side (KServeProxy, the native gateway): a pool of keep-alive connections that forward /predict
//     uploads that way and turn the binary outputs back into a RequestResult for the reference JSON.
//
// The JSON handled here is the small, fixed vocabulary of these messages; a purpose-built scanner (strings,
// numbers, arrays, objects) reads it without a general JSON library.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "batcher.h"
#include "string_pool.h"

namespace arena {

// Request body -> the byte range of the first element of BYTES input `input` inside `body`.  `ihcl` is the
// Inference-Header-Content-Length header (< 0: absent -> an error: a JPEG does not travel as a JSON string).
bool kserve_parse_bytes_input(const std::string& body, int64_t ihcl, const std::string& input, size_t& off,
                              size_t& len, std::string& err);

// The ensemble's outputs of one request.  binary: (JSON header, binary tensors) and *ihcl = header length;
// else a plain JSON body with "data" arrays and *ihcl = -1.
std::string kserve_build_response(const std::string& model, const std::string& id, const RequestResult& r,
                                  bool binary, int64_t* ihcl);

// A request carrying `upload` as IMAGE_BYTES (binary extension, binary outputs requested).
std::string kserve_build_request(const std::string& upload, const std::string& id, int64_t* ihcl);

// Binary-extension response -> detections, top-5 and stage times (RequestResult.det / topk / det_ms / cls_ms /
// queue_us / compute_us).
bool kserve_parse_response(const std::string& body, int64_t ihcl, RequestResult& r, std::string& err);

// Model metadata JSON of the ensemble (GET /v2/models/<model>).
std::string kserve_model_metadata(const std::string& model);

struct ProxyReply {
  int status = 0;          // upstream HTTP status (0: no answer)
  std::string error;       // transport / protocol error or the upstream's error body
  RequestResult result;    // parsed outputs (status 200)
};

// Keep-alive client pool: `conns` worker threads, each with one persistent TCP connection to host:port,
// forward uploads as KServe infer requests for `model`.  A request is resent once, on a new connection, only
// when the send failed or the kept-alive connection closed before any answer byte (the server cannot have
// started it); a poll timeout answers 504 without a resend.  Callbacks run on the worker threads.
enum class RoundtripFail { None, Send, ClosedEarly, Timeout, Protocol };
//
// Several upstreams (one model-server process per GPU, each with its own native endpoint): every request goes to
// the upstream with the fewest requests in flight from this proxy (ties: the worker's own rotation), each worker
// keeping one connection per upstream.
struct KServeUpstream {
  std::string host;
  int port = 0;
};
class KServeProxy {
 public:
  KServeProxy(std::string host, int port, std::string model, int conns, int timeout_ms = 60000);
  KServeProxy(std::vector<KServeUpstream> ups, std::string model, int conns, int timeout_ms = 60000);
  ~KServeProxy();
  KServeProxy(const KServeProxy&) = delete;
  KServeProxy& operator=(const KServeProxy&) = delete;
  void submit(std::string upload, std::function<void(ProxyReply&&)> done);
  void stop();
  // true when GET /v2/health/ready answers 200 on every upstream (fresh connections; used before the front end
  // turns healthy)
  bool upstream_ready();
  int64_t forwarded() const { return forwarded_.load(); }
  int64_t reconnects() const { return reconnects_.load(); }
  int num_upstreams() const { return (int)ups_.size(); }
  // requests forwarded to upstream i so far
  int64_t forwarded_to(int i) const { return ups_[(size_t)i].forwarded.load(); }
  // uploads go back to this pool once forwarded (the front end's body pool: no cross-thread frees)
  void set_recycler(StringPool* pool) { recycle_ = pool; }

 private:
  struct Task {
    std::string upload;
    std::function<void(ProxyReply&&)> done;
  };
  struct Up {
    std::string host;
    int port = 0;
    std::atomic<int> inflight{0};
    std::atomic<int64_t> forwarded{0};
  };
  void worker(int index);
  int pick(int rotation) const;
  int connect_upstream(int u, std::string& err) const;
  bool roundtrip(int& fd, const std::string& req, int& status, int64_t& ihcl, std::string& body, std::string& err,
                 RoundtripFail* fail = nullptr);

  std::deque<Up> ups_;  // deque: Up holds atomics (not movable)
  std::string model_;
  int timeout_ms_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Task> q_;
  bool stop_ = false;
  std::vector<std::thread> threads_;
  std::atomic<int64_t> forwarded_{0}, reconnects_{0};
  StringPool* recycle_ = nullptr;
};

}  // namespace arena
