// Native dynamic batcher; see batcher.h.
#include "batcher.h"

#include <sys/prctl.h>

#include <pthread.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "jpeg_decode.h"
#include "trace.h"

namespace arena {

using clk = std::chrono::steady_clock;

DynamicBatcher::DynamicBatcher(std::vector<std::shared_ptr<BatchInstance>> instances, const BatcherConfig& cfg)
    : inst_(std::move(instances)), cfg_(cfg) {
  if (inst_.empty()) throw std::runtime_error("DynamicBatcher: no executor instances");
  int largest = 0;
  for (auto& e : inst_) {
    auto b = e->buckets();
    if (b.empty()) throw std::runtime_error("DynamicBatcher: executor has no buckets");
    largest = largest == 0 ? b.back() : std::min(largest, b.back());
  }
  cfg_.max_batch = std::max(1, std::min(cfg_.max_batch, largest));
  if (cfg_.overlap < 0) {
    const char* e = std::getenv("ARENA_BATCH_OVERLAP");
    cfg_.overlap = e != nullptr && std::atoi(e) > 0 ? 1 : 0;
  }
  overlap_ = cfg_.overlap > 0;
  std::sort(cfg_.preferred.begin(), cfg_.preferred.end());
  cfg_.preferred.erase(std::remove_if(cfg_.preferred.begin(), cfg_.preferred.end(),
                                      [&](int v) { return v <= 0 || v > cfg_.max_batch; }),
                       cfg_.preferred.end());
  stats_.batch_hist.assign(cfg_.max_batch + 1, 0);
  for (auto& e : inst_) {
    const int64_t cap = e->staging_bytes();
    if (cap > 0) staging_cap_ = staging_cap_ > 0 ? std::min(staging_cap_, cap) : cap;
  }
  for (size_t i = 0; i < inst_.size(); ++i) threads_.emplace_back([this, i]() { instance_loop((int)i); });
}

DynamicBatcher::~DynamicBatcher() { shutdown(); }

void DynamicBatcher::shutdown() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ && threads_.empty()) return;
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

int64_t staged_bytes(const InputImage& im) {
  auto a = [](int64_t v) { return (v + 255) / 256 * 256; };
  if (im.jpeg != nullptr)
    return a((int64_t)im.h * im.w * 3) +
           a(im.jpeg->compact_bytes >= 0 ? im.jpeg->compact_bytes
                                         : std::max(im.jpeg->coef_count * 2, jpeg_compact_capacity(*im.jpeg))) +
           a(im.jpeg->plane_bytes);
  return a(im.bytes > 0 ? im.bytes : (int64_t)im.h * im.w * 3);
}

int64_t DynamicBatcher::enqueue(const uint8_t* data, int h, int w, ResultCallback cb, int64_t bytes,
                                uint8_t* export_dst) {
  InputImage in{nullptr, h, w};
  in.bytes = bytes;
  in.export_dst = export_dst;
  const int64_t staged = staged_bytes(in);
  if (staging_cap_ > 0 && staged > staging_cap_) {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.rejected;
    return -2;
  }
  auto copy = std::make_shared<std::vector<uint8_t>>(data, data + (bytes > 0 ? (size_t)bytes : (size_t)h * w * 3));
  in.data = copy->data();
  auto r = std::make_unique<Request>();
  r->in = in;
  r->owner = std::move(copy);
  r->staged = staged;
  r->cb = std::move(cb);
  return push(std::move(r));
}

int64_t DynamicBatcher::enqueue_input(const InputImage& in, std::shared_ptr<const void> owner, ResultCallback cb) {
  const int64_t staged = staged_bytes(in);
  if (staging_cap_ > 0 && staged > staging_cap_) {
    std::lock_guard<std::mutex> lk(mu_);
    ++stats_.rejected;
    return -2;
  }
  auto r = std::make_unique<Request>();
  r->in = in;
  r->owner = std::move(owner);
  r->staged = staged;
  r->cb = std::move(cb);
  return push(std::move(r));
}

int64_t DynamicBatcher::push(std::unique_ptr<Request> r) {
  r->t_enq = clk::now();
  int64_t id;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_) return -1;
    if (cfg_.max_queue_size > 0 && (int64_t)q_.size() >= cfg_.max_queue_size) {
      ++stats_.rejected;
      return -1;
    }
    id = next_id_++;
    r->id = id;
    q_.push_back(std::move(r));
    stats_.queue_depth = (int64_t)q_.size();
  }
  cv_.notify_one();
  return id;
}

bool DynamicBatcher::take_batch(Batch& out, bool can_wait, clk::time_point until) {
  std::unique_lock<std::mutex> lk(mu_);
  // can_wait == no batch of this instance in flight: the idle delay applies
  const auto delay = std::chrono::microseconds(can_wait && cfg_.idle_queue_delay_us >= 0 ? cfg_.idle_queue_delay_us
                                                                                         : cfg_.max_queue_delay_us);
  for (;;) {
    if (q_.empty()) {
      if (stop_) return false;
      if (!can_wait) {
        if (clk::now() >= until) return false;
        cv_.wait_until(lk, until);
        if (q_.empty()) return false;
        continue;
      }
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      continue;
    }
    // Requests that fit the staging pool together (in FIFO order, at least one): a batch of large
    // images is cut short instead of failing every request in it at submit.
    int n = (int)q_.size();
    if (staging_cap_ > 0) {
      int64_t sum = 0;
      int fit = 0;
      for (auto& rq : q_) {
        if (fit >= cfg_.max_batch) break;
        const int64_t b = rq->staged;
        if (fit > 0 && sum + b > staging_cap_) break;
        sum += b;
        ++fit;
      }
      if (fit < n && fit < cfg_.max_batch) {
        for (int i = 0; i < fit; ++i) {
          out.push_back(std::move(q_.front()));
          q_.pop_front();
        }
        stats_.queue_depth = (int64_t)q_.size();
        return true;
      }
    }
    int take = 0;
    if (n >= cfg_.max_batch) {
      take = cfg_.max_batch;
    } else if (!cfg_.preferred.empty() && n >= cfg_.preferred.back()) {
      take = cfg_.preferred.back();
    } else if (stop_ || clk::now() - q_.front()->t_enq >= delay) {
      take = n;  // delay expired: run what is queued
    }
    if (take > 0) {
      for (int i = 0; i < take; ++i) {
        out.push_back(std::move(q_.front()));
        q_.pop_front();
      }
      stats_.queue_depth = (int64_t)q_.size();
      return true;
    }
    const auto due = q_.front()->t_enq + delay;
    if (!can_wait) {
      if (clk::now() >= until) return false;
      cv_.wait_until(lk, std::min(until, due));
      continue;
    }
    cv_.wait_until(lk, due);
  }
}

void DynamicBatcher::finish(Batch& batch, const BatchResult& r, clk::time_point t_submit, size_t raw_bytes) {
  const auto t_done = clk::now();
  const int max_det = (int)(r.det.size() / std::max<size_t>(1, batch.size()));
  const double compute_us = std::chrono::duration<double, std::micro>(t_done - t_submit).count();
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.batches += 1;
    stats_.requests += (int64_t)batch.size();
    stats_.sum_batch += (double)batch.size();
    stats_.sum_compute_us += compute_us;
    if ((int)batch.size() < (int)stats_.batch_hist.size()) stats_.batch_hist[batch.size()] += 1;
    for (auto& rq : batch)
      stats_.sum_queue_us += std::chrono::duration<double, std::micro>(t_submit - rq->t_enq).count();
  }
  for (size_t i = 0; i < batch.size(); ++i) {
    RequestResult rr;
    rr.id = batch[i]->id;
    rr.det_count = i < r.det_count.size() ? r.det_count[i] : 0;
    const int kept = std::min(rr.det_count, max_det);
    if (kept > 0)
      rr.det.assign(r.det.begin() + (size_t)i * max_det, r.det.begin() + (size_t)i * max_det + kept);
    if (i + 1 < r.crop_offset.size())
      rr.topk.assign(r.topk.begin() + r.crop_offset[i], r.topk.begin() + r.crop_offset[i + 1]);
    if (raw_bytes > 0 && r.raw.size() >= (i + 1) * raw_bytes)
      rr.raw.assign(r.raw.begin() + i * raw_bytes, r.raw.begin() + (i + 1) * raw_bytes);
    rr.batch_size = (int)batch.size();
    rr.queue_us = std::chrono::duration<double, std::micro>(t_submit - batch[i]->t_enq).count();
    rr.compute_us = compute_us;
    rr.det_ms = r.det_ms;
    rr.cls_ms = r.cls_ms;
    batch[i]->cb(std::move(rr));
  }
}

void DynamicBatcher::fail(Batch& batch, const std::string& err) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stats_.failed += (int64_t)batch.size();
    stats_.last_error = err;
    // a HIP runtime error (ARENA_HIP_CHECK) poisons the device context; anything else (an input the staging
    // pool cannot take, an empty image) fails only this batch (server/batching.py is_device_fault)
    if (err.rfind("HIP error", 0) == 0) ++stats_.device_faults;
  }
  for (auto& rq : batch) {
    RequestResult rr;
    rr.id = rq->id;
    rr.error = err;
    rq->cb(std::move(rr));
  }
}

void DynamicBatcher::instance_loop(int idx) {
  pthread_setname_np(pthread_self(), "arena-batcher");
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us: its short timed waits must not stretch to 50 us
  BatchInstance& ex = *inst_[idx];
  struct InFlight {
    int slot;
    Batch batch;
    clk::time_point t_submit;
  };
  std::deque<InFlight> pending;
  for (;;) {
    if ((int)pending.size() < ex.num_slots()) {
      Batch b;
      if (take_batch(b, pending.empty())) {
        std::vector<InputImage> imgs;
        imgs.reserve(b.size());
        for (auto& rq : b) imgs.push_back(rq->in);
        try {
          trace::mark("arena.batch");
          const auto t = clk::now();
          const int slot = ex.submit(imgs);
          pending.push_back(InFlight{slot, std::move(b), t});
        } catch (const std::exception& e) {
          fail(b, e.what());
        }
        continue;
      }
      if (pending.empty()) {
        std::lock_guard<std::mutex> lk(mu_);
        if (stop_ && q_.empty()) return;
        continue;
      }
      // A slot is free and the oldest batch runs: wait for whichever comes first, a batch coming due (submitted
      // at once, so batches overlap on the device instead of queueing behind this wait) or the oldest batch's
      // completion (sleeping until shortly before its expected end, then polling every kPollUs).
      const int rd = overlap_ ? ex.ready(pending.front().slot) : -1;
      if (rd == 0) {
        // naps of half the expected remaining time, 20-200 us (Executor::wait_done): an early completion is
        // seen within one nap, and a new arrival ends the nap at once (take_batch waits on the queue)
        constexpr double kPollUs = 20.0, kMaxNapUs = 200.0;
        const double nap = std::min(kMaxNapUs, std::max(kPollUs, 0.5 * ex.remaining_us(pending.front().slot)));
        const auto until = clk::now() + std::chrono::microseconds((int64_t)nap);
        if (take_batch(b, false, until)) {
          std::vector<InputImage> imgs;
          imgs.reserve(b.size());
          for (auto& rq : b) imgs.push_back(rq->in);
          try {
            trace::mark("arena.batch");
            const auto t = clk::now();
            const int slot = ex.submit(imgs);
            pending.push_back(InFlight{slot, std::move(b), t});
          } catch (const std::exception& e) {
            fail(b, e.what());
          }
        }
        bool stopping;
        {
          std::lock_guard<std::mutex> lk(mu_);
          stopping = stop_;
        }
        if (!stopping || !b.empty()) continue;
        // stopping with nothing queued: collect (wait for) the in-flight batches below
      }
    }
    InFlight f = std::move(pending.front());
    pending.pop_front();
    try {
      BatchResult r = ex.collect(f.slot);
      trace::Range tf("arena.batcher.callbacks");
      finish(f.batch, r, f.t_submit, (size_t)std::max<int64_t>(0, ex.raw_out_bytes()));
    } catch (const std::exception& e) {
      fail(f.batch, e.what());
    }
  }
}

BatcherStats DynamicBatcher::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

}  // namespace arena
