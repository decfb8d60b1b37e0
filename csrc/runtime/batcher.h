// Native dynamic batcher (the scheduler half of the Triton replacement).
//
// The reference's Triton deployment runs the default scheduler with
// `max_batch_size: 0` (infrastructure/minio/triton_config.py:98-128), i.e. no
// batching, one request per ONNX Runtime call.  This batcher implements the
// `dynamic_batching { preferred_batch_size, max_queue_delay_microseconds }`
// semantics of a model-repository config.pbtxt on top of Executor instances
// (one per `instance_group` count on the GPU):
//
//   * requests wait in one FIFO shared by all instances of the model;
//   * an idle instance takes a batch as soon as the queue holds max_batch
//     requests, or a preferred size is available and no larger one can form,
//     or the oldest request has waited max_queue_delay;
//   * each instance keeps one batch in flight per staging slot (the executor
//     runs each slot on its own stream), so packing/H2D of the next batch
//     overlaps the graphs of the previous ones;
//   * completion callbacks run on the instance thread.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "instance.h"

namespace arena {

struct RequestResult {
  int64_t id = 0;
  int det_count = 0;
  std::vector<Detection> det;    // min(det_count, max_det) rows
  std::vector<TopkResult> topk;  // one per kept detection
  std::vector<uint8_t> raw;      // raw tensor output (raw-output programs)
  int batch_size = 0;
  double queue_us = 0, compute_us = 0;
  double det_ms = -1, cls_ms = -1;  // device stage times of the request's batch (BatchResult)
  std::string error;
};

using ResultCallback = std::function<void(RequestResult&&)>;

struct BatcherConfig {
  int max_batch = 32;
  std::vector<int> preferred;          // preferred batch sizes (ascending)
  int64_t max_queue_delay_us = 500;
  int64_t max_queue_size = 4096;       // 0 = unbounded
  // Delay used while the instance has no batch in flight (-1: max_queue_delay_us).  A short idle delay keeps
  // the single-request latency low while a longer max_queue_delay_us still grows the batches once the device
  // is busy (arrivals during device work merge into the next batch).
  int64_t idle_queue_delay_us = -1;
  // While a batch is in flight and a slot is free: 0 = collect (wait for) the oldest batch first, arrivals merge
  // into the batch after it; 1 = admit a batch as soon as it is due (max_queue_delay_us / size) into the free
  // slot, so batches overlap on the device (instances that answer BatchInstance::ready).  -1 = ARENA_BATCH_OVERLAP
  // from the environment (default 0).
  int overlap = -1;
};

struct BatcherStats {
  int64_t requests = 0, batches = 0, rejected = 0, failed = 0;
  int64_t queue_depth = 0;
  double sum_batch = 0;
  double sum_queue_us = 0, sum_compute_us = 0;
  std::vector<int64_t> batch_hist;  // index = batch size
  int64_t device_faults = 0;        // failed batches whose error is a HIP runtime error ("HIP error ...")
  std::string last_error;           // text of the most recent failed batch
};

class DynamicBatcher {
 public:
  // smallest staging capacity of the instances in bytes (0 = unlimited): inputs whose staged_bytes exceed it
  // are rejected by enqueue (-2)
  int64_t staging_cap() const { return staging_cap_; }
  DynamicBatcher(std::vector<std::shared_ptr<BatchInstance>> instances, const BatcherConfig& cfg);
  ~DynamicBatcher();
  DynamicBatcher(const DynamicBatcher&) = delete;
  DynamicBatcher& operator=(const DynamicBatcher&) = delete;

  // Copies the input; returns the request id, -1 when the queue is full, -2 when the input is larger than
  // an instance can stage in one batch (the caller answers 413 / INVALID_ARGUMENT).
  // `bytes` == 0: RGB uint8 HxWx3 image; otherwise an fp32 [3, h, w] tensor of
  // that many bytes (reference tensor contract of the model server).
  int64_t enqueue(const uint8_t* data, int h, int w, ResultCallback cb, int64_t bytes = 0,
                  uint8_t* export_dst = nullptr);
  // Zero-copy: the request references `in` (pixels, tensor or split-decoded JPEG coefficients) and keeps
  // `owner` alive until its callback has run — the native front end's decode threads hand over pinned
  // buffers the executor DMAs from directly.  Same return codes as enqueue().
  int64_t enqueue_input(const InputImage& in, std::shared_ptr<const void> owner, ResultCallback cb);
  BatcherStats stats();
  void shutdown();

 private:
  struct Request {
    int64_t id;
    InputImage in;
    std::shared_ptr<const void> owner;  // keeps in.data (and in.jpeg) alive
    int64_t staged;                     // staged_bytes(in)
    ResultCallback cb;
    std::chrono::steady_clock::time_point t_enq;
  };
  int64_t push(std::unique_ptr<Request> r);
  using Batch = std::vector<std::unique_ptr<Request>>;

  void instance_loop(int idx);
  // can_wait: block until a batch is due.  Otherwise, with `until` in the future, wait for new requests or the
  // queue delay to expire up to that time; return false when nothing is due by then.
  bool take_batch(Batch& out, bool can_wait,
                  std::chrono::steady_clock::time_point until = std::chrono::steady_clock::time_point::min());
  void finish(Batch& batch, const BatchResult& r, std::chrono::steady_clock::time_point t_submit, size_t raw_bytes);
  void fail(Batch& batch, const std::string& err);

  std::vector<std::shared_ptr<BatchInstance>> inst_;
  BatcherConfig cfg_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::unique_ptr<Request>> q_;
  bool stop_ = false;
  int64_t staging_cap_ = 0;  // smallest staging capacity of the instances (0 = unlimited)
  bool overlap_ = false;     // BatcherConfig::overlap resolved
  int64_t next_id_ = 1;
  BatcherStats stats_;
  std::vector<std::thread> threads_;
};

}  // namespace arena
