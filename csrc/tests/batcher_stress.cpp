// Concurrency stress test of the native DynamicBatcher (csrc/runtime/batcher.cpp)
// against CPU fake instances — built and run under ThreadSanitizer and
// AddressSanitizer by tests/test_batcher_native.py (host code only; no GPU).
//
// Checks, with many producer threads racing the instance threads:
//   * every accepted request gets exactly one callback, with ITS result
//     (the fake encodes the request's first pixel into the detections);
//   * batches never exceed max_batch, and no instance ever has more than
//     num_slots() batches in flight;
//   * a submit() failure is reported to every request of that batch;
//   * a full queue rejects (enqueue returns -1) instead of blocking;
//   * shutdown() drains queued work and joins cleanly;
//   * batches never stage more bytes than the instance's staging capacity, and an
//     input that can never fit is rejected at enqueue (-2) (a large
//     image must not fail the small requests it shares a batch with).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/batcher.h"

using namespace arena;

namespace {

constexpr int kMaxDet = 4;
constexpr uint8_t kPoison = 250;  // first pixel value that makes submit() throw

std::atomic<int> fails{0};
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++fails;                                             \
    }                                                      \
  } while (0)

class FakeInstance : public BatchInstance {
 public:
  FakeInstance(int slots, int max_batch, int64_t staging = 0)
      : slots_(slots), max_batch_(max_batch), staging_(staging), busy_(slots, false), work_(slots) {}
  int64_t staging_bytes() const override { return staging_; }
  std::vector<int> buckets() const override { return {1, 2, 4, max_batch_}; }
  int num_slots() const override { return slots_; }
  int max_det() const override { return kMaxDet; }
  int64_t raw_out_bytes() const override { return 0; }

  int submit(const std::vector<InputImage>& imgs) override {
    CHECK(!imgs.empty() && (int)imgs.size() <= max_batch_, "batch size %zu", imgs.size());
    if (staging_ > 0) {
      int64_t sum = 0;
      for (auto& im : imgs) sum += ((int64_t)im.h * im.w * 3 + 255) / 256 * 256;
      CHECK(sum <= staging_, "batch stages %lld bytes > capacity %lld", (long long)sum, (long long)staging_);
      if (sum > staging_) throw std::runtime_error("batch exceeds the staging pool");
      max_staged_ = std::max(max_staged_, sum);
    }
    int s = -1;
    for (int i = 0; i < slots_; ++i)
      if (!busy_[i]) { s = i; break; }
    CHECK(s >= 0, "submit with every slot busy");
    if (s < 0) throw std::runtime_error("all slots busy");
    for (auto& im : imgs)
      if (im.data[0] == kPoison) throw std::runtime_error("poisoned batch");
    std::vector<uint8_t> firsts;
    for (auto& im : imgs) firsts.push_back(im.data[(size_t)im.h * im.w * 3 - 1]);  // last byte = first byte
    busy_[s] = true;
    ++in_flight_;
    max_in_flight_ = std::max(max_in_flight_, in_flight_);
    // the "device": completes the batch asynchronously on another thread
    work_[s] = std::async(std::launch::async, [firsts, seed = seed_++]() {
      std::mt19937 rng(seed);
      std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
      BatchResult r;
      const int n = (int)firsts.size();
      r.n_images = n;
      r.det_count.resize(n);
      r.det.resize((size_t)n * kMaxDet);
      r.crop_offset.resize(n + 1);
      int total = 0;
      for (int i = 0; i < n; ++i) {
        const int v = firsts[i];
        r.det_count[i] = v % (kMaxDet + 2);  // may exceed max_det: kept rows are clipped
        r.crop_offset[i] = total;
        const int kept = std::min(r.det_count[i], kMaxDet);
        for (int k = 0; k < kept; ++k) {
          Detection& d = r.det[(size_t)i * kMaxDet + k];
          d.x1 = (float)v;
          d.y1 = (float)k;
          TopkResult t{};
          t.idx[0] = v;
          r.topk.push_back(t);
        }
        total += kept;
      }
      r.crop_offset[n] = total;
      r.total_crops = total;
      return r;
    });
    return s;
  }

  int ready(int slot) override {  // the batcher's overlap path (non-blocking completion test)
    CHECK(slot >= 0 && slot < slots_ && busy_[slot], "ready() of idle slot %d", slot);
    return work_[slot].wait_for(std::chrono::seconds(0)) == std::future_status::ready ? 1 : 0;
  }
  double remaining_us(int) override { return 100.0; }

  BatchResult collect(int slot) override {
    CHECK(slot >= 0 && slot < slots_ && busy_[slot], "collect of idle slot %d", slot);
    BatchResult r = work_[slot].get();
    busy_[slot] = false;
    --in_flight_;
    return r;
  }

  int max_in_flight() const { return max_in_flight_; }
  int64_t max_staged() const { return max_staged_; }

 private:
  int slots_, max_batch_;
  int64_t staging_ = 0, max_staged_ = 0;
  std::vector<bool> busy_;
  std::vector<std::future<BatchResult>> work_;
  int in_flight_ = 0, max_in_flight_ = 0;
  unsigned seed_ = 1;
};

struct Outcome {
  std::atomic<int> calls{0};
  int det_count = -1;
  float x1 = -1.f;
  int top = -1;
  int batch = 0;
  std::string error;
};

void run_stress(int overlap) {
  const int producers = 8, per = 1500, max_batch = 8;
  auto a = std::make_shared<FakeInstance>(3, max_batch);
  auto b = std::make_shared<FakeInstance>(2, max_batch);
  BatcherConfig cfg;
  cfg.max_batch = max_batch;
  cfg.preferred = {4, 8};
  cfg.max_queue_delay_us = 200;
  cfg.max_queue_size = 0;
  cfg.overlap = overlap;
  std::vector<Outcome> out((size_t)producers * per);
  std::vector<uint8_t> expect(out.size());
  {
    DynamicBatcher bat({a, b}, cfg);
    std::vector<std::thread> ts;
    for (int p = 0; p < producers; ++p) {
      ts.emplace_back([&, p]() {
        std::mt19937 rng(p + 100);
        for (int i = 0; i < per; ++i) {
          const size_t k = (size_t)p * per + i;
          uint8_t v = (uint8_t)((p * 37 + i * 11) % 240);  // never the poison value
          expect[k] = v;
          const int h = 1 + (int)(rng() % 4), w = 1 + (int)(rng() % 4);
          std::vector<uint8_t> img((size_t)h * w * 3, 7);
          img[0] = v;
          img.back() = v;
          Outcome* o = &out[k];
          const int64_t id = bat.enqueue(img.data(), h, w, [o](RequestResult&& r) {
            o->det_count = r.det_count;
            o->x1 = r.det.empty() ? -1.f : r.det[0].x1;
            o->top = r.topk.empty() ? -1 : r.topk[0].idx[0];
            o->batch = r.batch_size;
            o->error = r.error;
            o->calls.fetch_add(1);
          });
          CHECK(id > 0, "unbounded queue rejected a request");
          if (rng() % 64 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 500));
        }
      });
    }
    // stats() races the instance threads on purpose
    std::atomic<bool> done{false};
    std::thread poll([&]() {
      while (!done.load()) {
        auto s = bat.stats();
        CHECK(s.requests <= (int64_t)out.size(), "stats overflow");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    });
    for (auto& t : ts) t.join();
    // wait until every callback ran, then shut down
    for (int spin = 0; spin < 20000; ++spin) {
      if (bat.stats().requests + bat.stats().failed >= (int64_t)out.size()) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    done = true;
    poll.join();
    auto s = bat.stats();
    CHECK(s.requests == (int64_t)out.size(), "requests %lld", (long long)s.requests);
    CHECK(s.batches > 0 && s.sum_batch / s.batches >= 1.0, "batches");
    bat.shutdown();
  }
  for (size_t k = 0; k < out.size(); ++k) {
    const Outcome& o = out[k];
    CHECK(o.calls.load() == 1, "request %zu got %d callbacks", k, o.calls.load());
    CHECK(o.error.empty(), "request %zu error %s", k, o.error.c_str());
    const int v = expect[k];
    CHECK(o.det_count == v % (kMaxDet + 2), "request %zu det_count %d (v=%d)", k, o.det_count, v);
    if (std::min(v % (kMaxDet + 2), kMaxDet) > 0) {
      CHECK(o.x1 == (float)v && o.top == v, "request %zu got another request's result", k);
    }
    CHECK(o.batch >= 1 && o.batch <= max_batch, "batch size %d", o.batch);
  }
  CHECK(a->max_in_flight() <= a->num_slots() && b->max_in_flight() <= b->num_slots(), "slot overcommit");
  CHECK(a->max_in_flight() + b->max_in_flight() >= 2, "no pipelining observed");
}

void run_failures_and_rejection() {
  auto a = std::make_shared<FakeInstance>(2, 4);
  BatcherConfig cfg;
  cfg.max_batch = 4;
  cfg.max_queue_delay_us = 1000000;  // no batch can form (2 < max_batch) before shutdown
  cfg.max_queue_size = 2;
  std::vector<Outcome> out(16);
  int accepted = 0, rejected = 0;
  {
    DynamicBatcher bat({a}, cfg);
    for (int i = 0; i < 16; ++i) {
      std::vector<uint8_t> img(3, (uint8_t)(i == 0 ? kPoison : 1 + i));
      Outcome* o = &out[i];
      const int64_t id = bat.enqueue(img.data(), 1, 1, [o](RequestResult&& r) {
        o->error = r.error;
        o->det_count = r.det_count;
        o->calls.fetch_add(1);
      });
      if (id > 0) ++accepted; else ++rejected;
    }
    bat.shutdown();  // drains what was accepted
    auto s = bat.stats();
    CHECK(s.rejected == rejected, "rejected stat %lld vs %d", (long long)s.rejected, rejected);
  }
  CHECK(rejected > 0, "bounded queue never rejected");
  int called = 0, errored = 0;
  for (auto& o : out) {
    called += o.calls.load();
    errored += !o.error.empty();
  }
  CHECK(called == accepted, "callbacks %d for %d accepted requests", called, accepted);
  CHECK(errored >= 1 && out[0].error.find("poisoned") != std::string::npos, "poisoned batch not reported");
}

void run_staging_capacity() {
  // capacity = 4 x 1 KiB-aligned small images; "large" 20x20 images (1200 B -> 1280 staged) fill 3 slots
  const int64_t cap = 4096;
  auto a = std::make_shared<FakeInstance>(2, 8, cap);
  BatcherConfig cfg;
  cfg.max_batch = 8;
  cfg.max_queue_delay_us = 100;
  cfg.max_queue_size = 0;
  std::vector<Outcome> out(64);
  {
    DynamicBatcher bat({a}, cfg);
    std::vector<uint8_t> big((size_t)40 * 40 * 3, 9);  // 4800 B: can never fit
    Outcome dummy;
    const int64_t rej = bat.enqueue(big.data(), 40, 40, [&](RequestResult&&) { dummy.calls.fetch_add(1); });
    CHECK(rej == -2, "oversized input not rejected (%lld)", (long long)rej);
    for (int i = 0; i < 64; ++i) {
      const int side = (i % 3 == 0) ? 20 : 4;
      std::vector<uint8_t> img((size_t)side * side * 3, (uint8_t)(1 + i % 200));
      Outcome* o = &out[i];
      const int64_t id = bat.enqueue(img.data(), side, side, [o](RequestResult&& r) {
        o->error = r.error;
        o->calls.fetch_add(1);
      });
      CHECK(id > 0, "request %d rejected", i);
    }
    for (int spin = 0; spin < 20000 && bat.stats().requests + bat.stats().failed < 64; ++spin)
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    bat.shutdown();
    CHECK(dummy.calls.load() == 0, "rejected request got a callback");
  }
  for (int i = 0; i < 64; ++i) {
    CHECK(out[i].calls.load() == 1, "request %d got %d callbacks", i, out[i].calls.load());
    CHECK(out[i].error.empty(), "request %d failed: %s", i, out[i].error.c_str());
  }
  CHECK(a->max_staged() > 0 && a->max_staged() <= cap, "staged %lld", (long long)a->max_staged());
}

}  // namespace

int main() {
  run_staging_capacity();
  run_stress(0);
  run_stress(1);  // overlap: ready() tests and timed takes interleaved with collects
  run_failures_and_rejection();
  if (fails.load()) {
    std::fprintf(stderr, "batcher_stress: %d check(s) failed\n", fails.load());
    return 1;
  }
  std::printf("batcher_stress: ok\n");
  return 0;
}
