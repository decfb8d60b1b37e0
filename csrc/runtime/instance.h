// The interface the dynamic batcher schedules onto: one "model instance"
// (Triton's instance_group entry) that accepts batches of requests into a
// fixed number of in-flight slots.  The GPU Executor (executor.h) is the
// production implementation; tests drive the batcher with CPU fakes under
// ThreadSanitizer / AddressSanitizer (csrc/tests/batcher_stress.cpp).
#pragma once
#include <cstdint>
#include <vector>

#include "../kernels/launch.h"

namespace arena {

struct JpegInfo;  // runtime/jpeg_decode.h

struct InputImage {
  const uint8_t* data;  // RGB uint8 HWC, contiguous (or an fp32 tensor when bytes != 0, or JPEG coefficients)
  int h, w;
  int64_t bytes = 0;    // explicit payload size (tensor inputs); 0 = h*w*3
  // Entropy-decoded JPEG (split decoder, runtime/jpeg_decode.h): `data` holds jpeg->coef_count int16
  // coefficients (ideally pinned host memory: the executor DMAs them straight from there) and the instance
  // reconstructs the RGB frame on the device.
  const JpegInfo* jpeg = nullptr;
  // Optional device address (on the instance's GPU) that receives a copy of the staged RGB frame, device to
  // device on the batch's stream (arm B device transport: the detector exports the frame it already uploaded
  // into the IPC ring slot the classification service reads; no second host -> device copy).
  uint8_t* export_dst = nullptr;
};

// Staging-pool bytes an input occupies in one batch (each region rounded up to 256 B): the RGB frame, plus for a
// split-decoded JPEG its coefficient blocks and the reconstruction's sample planes.
int64_t staged_bytes(const InputImage& im);

// Per-slot results copied back to pinned memory after the slot's graph.
struct BatchResult {
  int n_images = 0;
  int bucket = 0;
  int total_crops = 0;
  std::vector<int> det_count;        // [n]
  std::vector<Detection> det;        // [n * max_det]
  std::vector<TopkResult> topk;      // [total crops], in crop-plan order
  std::vector<int> crop_offset;      // [n + 1] first crop of each image
  double gpu_ms = 0.0;               // graph wall time from events
  // device time of the detection part (program start -> classifier start) and of the classification part
  // (classifier start -> end), from OP_STAMP wall-clock stamps; -1 when the program has no stamps
  double det_ms = -1.0, cls_ms = -1.0;
  std::vector<uint8_t> raw;          // [n * raw_out_bytes] when the program exports raw tensors
};

class BatchInstance {
 public:
  virtual ~BatchInstance() = default;
  virtual std::vector<int> buckets() const = 0;  // batch capacities, ascending (last = largest)
  virtual int num_slots() const = 0;             // batches that may be in flight at once
  virtual int max_det() const = 0;               // detection rows per image in BatchResult::det
  virtual int64_t raw_out_bytes() const = 0;     // raw output bytes per image (0 = none)
  // Bytes one batch may stage in total (each input rounded up to 256); 0 = unlimited.  The batcher
  // closes a batch before it would exceed this and rejects an input that can never fit.
  virtual int64_t staging_bytes() const { return 0; }
  // Start a batch; returns the slot id.  Throws when every slot is in flight.
  virtual int submit(const std::vector<InputImage>& imgs) = 0;
  // Wait for a slot's batch and return its results (the slot becomes free).
  virtual BatchResult collect(int slot) = 0;
  // Non-blocking completion test of a slot's batch: 1 done (collect will not wait), 0 still running, -1 the
  // instance cannot tell (the batcher then collects, i.e. waits).  With 0 the batcher keeps admitting new
  // batches into free slots while the oldest one runs.
  virtual int ready(int slot) { (void)slot; return -1; }
  // Estimated microseconds until a running slot's batch completes (<= 0: unknown or due now).
  virtual double remaining_us(int slot) { (void)slot; return 0.0; }
};

}  // namespace arena
