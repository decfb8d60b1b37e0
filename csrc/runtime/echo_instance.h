// A host-only BatchInstance: answers every image with a deterministic set of
// detections derived from its size and first pixel, without a GPU.  It lets
// the dynamic batcher and the native HTTP front end (http_front.h) be tested
// end to end on CPU machines (tests/test_native_http.py) and measured for
// their own host cost (tools/http_overhead.py --native).
#pragma once
#include <algorithm>
#include <cstring>
#include <chrono>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <vector>

#include "instance.h"
#include "jpeg_decode.h"

namespace arena {

class EchoInstance : public BatchInstance {
 public:
  // latency_us: collect() returns no earlier than this long after submit (a stand-in for device time)
  // staging_cap: the staging_bytes() it reports (0 = unlimited), as an Executor reports its slot's image pool
  EchoInstance(int slots, int max_batch, int max_det = 4, int latency_us = 0, int64_t staging_cap = 0)
      : slots_(slots), max_batch_(max_batch), max_det_(max_det), latency_us_(latency_us), staging_cap_(staging_cap),
        results_(slots),
        busy_(slots, false), t_submit_(slots) {}
  std::vector<int> buckets() const override {
    std::vector<int> b;
    for (int v = 1; v < max_batch_; v *= 2) b.push_back(v);
    b.push_back(max_batch_);
    return b;
  }
  int num_slots() const override { return slots_; }
  int max_det() const override { return max_det_; }
  int64_t raw_out_bytes() const override { return 0; }
  int64_t staging_bytes() const override { return staging_cap_; }

  // Image i of a batch gets min(max_det, 1 + first_byte % max_det) detections: box k spans
  // (k, k, w - k, h - k), confidence 0.9 - 0.1 k, COCO class k; crop top-5 = classes 10k .. 10k + 4.
  int submit(const std::vector<InputImage>& imgs) override {
    if (imgs.empty() || (int)imgs.size() > max_batch_) throw std::runtime_error("EchoInstance: bad batch size");
    std::lock_guard<std::mutex> lk(mu_);
    int s = -1;
    for (int i = 0; i < slots_; ++i)
      if (!busy_[i]) { s = i; break; }
    if (s < 0) throw std::runtime_error("EchoInstance: all slots busy");
    BatchResult r;
    const int n = (int)imgs.size();
    r.n_images = n;
    r.det_count.resize(n);
    r.det.resize((size_t)n * max_det_);
    r.crop_offset.resize(n + 1);
    int total = 0;
    for (int i = 0; i < n; ++i) {
      uint8_t first = imgs[i].data[0];
      if (imgs[i].jpeg != nullptr) {  // split-decoded JPEG: reconstruct like the device would (host reference)
        std::vector<uint8_t> rgb((size_t)imgs[i].h * imgs[i].w * 3);
        std::vector<int16_t> dense;
        jpeg_coefs_to_rgb(*imgs[i].jpeg, jpeg_dense_coefs(*imgs[i].jpeg, imgs[i].data, dense), rgb.data());
        first = rgb[0];
      }
      const int k_n = std::min(max_det_, 1 + first % max_det_);
      r.det_count[i] = k_n;
      r.crop_offset[i] = total;
      for (int k = 0; k < k_n; ++k) {
        Detection& d = r.det[(size_t)i * max_det_ + k];
        d.x1 = (float)k;
        d.y1 = (float)k;
        d.x2 = (float)(imgs[i].w - k);
        d.y2 = (float)(imgs[i].h - k);
        d.conf = 0.9f - 0.1f * (float)k;
        d.cls = k;
        TopkResult t{};
        for (int j = 0; j < 5; ++j) {
          t.idx[j] = 10 * k + j;
          t.logit[j] = 5.0f - (float)j;
          t.prob[j] = 0.5f / (float)(j + 1);
        }
        r.topk.push_back(t);
      }
      total += k_n;
    }
    r.crop_offset[n] = total;
    r.total_crops = total;
    results_[s] = std::move(r);
    busy_[s] = true;
    t_submit_[s] = std::chrono::steady_clock::now();
    return s;
  }

  // completion tests as the Executor answers them (the batcher's interruptible wait runs on CPU too)
  int ready(int slot) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot < 0 || slot >= slots_ || !busy_[slot]) return 1;
    return std::chrono::steady_clock::now() >= t_submit_[slot] + std::chrono::microseconds(latency_us_) ? 1 : 0;
  }
  double remaining_us(int slot) override {
    std::lock_guard<std::mutex> lk(mu_);
    if (slot < 0 || slot >= slots_ || !busy_[slot]) return 0.0;
    return std::chrono::duration<double, std::micro>(t_submit_[slot] + std::chrono::microseconds(latency_us_) -
                                                     std::chrono::steady_clock::now())
        .count();
  }

  BatchResult collect(int slot) override {
    std::chrono::steady_clock::time_point due;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (slot < 0 || slot >= slots_ || !busy_[slot]) throw std::runtime_error("EchoInstance: bad slot");
      due = t_submit_[slot] + std::chrono::microseconds(latency_us_);
    }
    std::this_thread::sleep_until(due);
    std::lock_guard<std::mutex> lk(mu_);
    busy_[slot] = false;
    // stand-in stage times (the executor derives them from the program's wall-clock stamps): 60 % / 30 % of
    // the simulated device latency, so the stage plumbing is testable without a GPU
    results_[slot].det_ms = 0.6e-3 * latency_us_;
    results_[slot].cls_ms = 0.3e-3 * latency_us_;
    return std::move(results_[slot]);
  }

 private:
  int slots_, max_batch_, max_det_, latency_us_;
  int64_t staging_cap_;
  std::vector<BatchResult> results_;
  std::vector<bool> busy_;
  std::vector<std::chrono::steady_clock::time_point> t_submit_;
  std::mutex mu_;
};

}  // namespace arena
