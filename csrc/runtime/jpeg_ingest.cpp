// See jpeg_ingest.h.
#include "runtime/jpeg_ingest.h"

#include <pthread.h>

#include <cstdlib>
#include <ctime>

#include "runtime/jpeg_decode.h"

namespace arena {

namespace {

double thread_cpu_ms() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// the decoded upload in flight: parsed header + the buffer its coefficients (or RGB frame) live in
struct Upload {
  JpegInfo info;
  std::shared_ptr<uint8_t> buf;
};

void fail(const ResultCallback& done, const std::string& msg) {
  RequestResult r;
  r.error = msg;
  done(std::move(r));
}

}  // namespace

JpegIngest::JpegIngest(DynamicBatcher* batcher, IngestConfig cfg) : batcher_(batcher), cfg_(std::move(cfg)) {
  if (batcher_ == nullptr) throw std::runtime_error("JpegIngest: no batcher");
  pool_ = HostBufferPool::create(cfg_.buffer_cap, cfg_.host_alloc, cfg_.host_free);
  for (int i = 0; i < std::max(1, cfg_.threads); ++i) threads_.emplace_back([this] { loop(); });
}

JpegIngest::~JpegIngest() { stop(); }

void JpegIngest::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ && threads_.empty()) return;
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  std::deque<Task> left;
  {
    std::lock_guard<std::mutex> lk(mu_);
    left.swap(q_);
  }
  for (auto& t : left) fail(t.done, "ingest stopped");
}

void JpegIngest::submit(std::string upload, ResultCallback done, Fallback fallback, uint8_t* export_dst) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!stop_) {
      q_.push_back(Task{std::move(upload), std::move(done), std::move(fallback), export_dst});
      cv_.notify_one();
      return;
    }
  }
  fail(done, "ingest stopped");
}

IngestStats JpegIngest::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return stats_;
}

void JpegIngest::loop() {
  pthread_setname_np(pthread_self(), "arena-jpeg");
  for (;;) {
    Task t;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stopping
      t = std::move(q_.front());
      q_.pop_front();
    }
    run(t);
  }
}

void JpegIngest::run(Task& t) {
  const double c0 = thread_cpu_ms();
  const uint8_t* data = (const uint8_t*)t.upload.data();
  auto up = std::make_shared<Upload>();
  std::string err;
  JpegStatus st = t.upload.empty() ? JpegStatus::Corrupt : jpeg_parse(data, t.upload.size(), up->info, err,
                                                                      cfg_.max_image_pixels);
  if (t.upload.empty()) err = "Failed to decode image: empty payload";
  if (st == JpegStatus::Unsupported) {
    {
      std::lock_guard<std::mutex> lk(stats_mu_);
      ++stats_.fallback;
    }
    t.fallback(std::move(t.upload));
    return;
  }
  const JpegInfo& ji = up->info;
  InputImage in{nullptr, ji.height, ji.width};
  in.export_dst = t.export_dst;
  if (st == JpegStatus::Ok) {
    // device reconstruction when the frame's coefficients, planes and RGB fit one batch's staging pool and a
    // pooled buffer; otherwise the host reconstructs it (bit-exact, jpeg_coefs_to_rgb) and it is staged as RGB
    const int64_t cap = batcher_->staging_cap();
    InputImage probe = in;
    probe.jpeg = &ji;
    bool device = cfg_.jpeg_device && (cap <= 0 || staged_bytes(probe) <= cap);
    const bool compact = jpeg_compact_enabled();
    if (device) {
      up->buf = pool_->get(compact ? (size_t)jpeg_compact_capacity(ji) : (size_t)ji.coef_count * 2);
      device = (bool)up->buf;
    }
    if (device) {
      st = compact ? jpeg_decode_compact(data, t.upload.size(), up->info, up->buf.get(), err)
                   : jpeg_decode_coefs(data, t.upload.size(), ji, (int16_t*)up->buf.get(), err);
      in.data = up->buf.get();
      in.jpeg = &up->info;
    } else {
      std::vector<int16_t> coef((size_t)ji.coef_count);
      st = jpeg_decode_coefs(data, t.upload.size(), ji, coef.data(), err);
      if (st == JpegStatus::Ok) {
        const size_t rgb_bytes = (size_t)ji.width * ji.height * 3;
        up->buf = pool_->get(rgb_bytes);
        if (!up->buf) {  // beyond the largest size class or the pool's cap: a buffer of its own
          uint8_t* raw = static_cast<uint8_t*>(std::malloc(rgb_bytes));
          if (raw != nullptr) up->buf = std::shared_ptr<uint8_t>(raw, [](uint8_t* q) { std::free(q); });
        }
        if (!up->buf) {
          st = JpegStatus::Corrupt;
          err = "decode buffers exhausted";
        } else {
          jpeg_coefs_to_rgb(ji, coef.data(), up->buf.get());
          in.data = up->buf.get();
        }
      }
    }
  }
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    if (st == JpegStatus::Ok) ++stats_.native;
    else ++stats_.errors;
    stats_.cpu_decode_ms += thread_cpu_ms() - c0;
  }
  if (st != JpegStatus::Ok) return fail(t.done, err);
  ResultCallback done = t.done;  // enqueue_input consumes its copy; keep one for a rejection
  const int64_t id = batcher_->enqueue_input(in, up, std::move(t.done));
  if (id == -1) fail(done, "request queue is full");
  else if (id == -2) fail(done, "image exceeds the staging capacity of one batch");
}

}  // namespace arena
