// Split-decoder ingest for request paths that are not the native HTTP front end: the model server's ensemble
// (arm C, IMAGE_BYTES inputs of arena_pipeline) and any caller holding encoded uploads.
//
// submit(upload, done, fallback) hands the bytes to a pool of C++ decode threads that run the host half of the
// split JPEG decoder (runtime/jpeg_decode.h: marker parse + Huffman decode into a pinned HostBufferPool buffer)
// and enqueue the result into the DynamicBatcher without a copy (enqueue_input); the instance reconstructs the
// frame on the GPU.  `done` receives the batch result (or an error: a corrupt upload, a full queue).  Uploads the
// split decoder does not cover (progressive JPEG, PNG, ...) are handed back through `fallback` untouched — the
// caller decodes them its own way (PIL) and enqueues the pixels.  The reference decodes on the request thread
// (architectures/triton/gateway/app/pipeline.py:131-139 via cv2; here the ensemble's server process).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "batcher.h"
#include "host_pool.h"

namespace arena {

struct IngestConfig {
  int threads = 4;
  bool jpeg_device = true;  // false: reconstruct on the host threads (instances without the device half)
  int64_t max_image_pixels = 50000000;
  int64_t buffer_cap = 1LL << 30;
  HostBufferPool::AllocFn host_alloc;
  HostBufferPool::FreeFn host_free;
};

struct IngestStats {
  int64_t native = 0, fallback = 0, errors = 0;
  double cpu_decode_ms = 0;
};

class JpegIngest {
 public:
  using Fallback = std::function<void(std::string&& upload)>;
  JpegIngest(DynamicBatcher* batcher, IngestConfig cfg);
  ~JpegIngest();
  JpegIngest(const JpegIngest&) = delete;
  JpegIngest& operator=(const JpegIngest&) = delete;

  // export_dst: device address that receives the reconstructed frame (InputImage::export_dst)
  void submit(std::string upload, ResultCallback done, Fallback fallback, uint8_t* export_dst = nullptr);
  IngestStats stats();
  void stop();

 private:
  struct Task {
    std::string upload;
    ResultCallback done;
    Fallback fallback;
    uint8_t* export_dst = nullptr;
  };
  void loop();
  void run(Task& t);

  DynamicBatcher* batcher_;
  IngestConfig cfg_;
  std::shared_ptr<HostBufferPool> pool_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Task> q_;
  bool stop_ = false;
  std::vector<std::thread> threads_;
  std::mutex stats_mu_;
  IngestStats stats_;
};

}  // namespace arena
