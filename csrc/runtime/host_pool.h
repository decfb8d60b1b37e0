// Size-classed pool of host buffers for request payloads the device DMAs from (the split JPEG decoder's
// coefficient blocks, csrc/runtime/jpeg_decode.h).
//
// The native front end's decode threads write each upload's coefficients straight into one of these buffers
// and the executor copies them host -> device from there (Executor::submit), so a frame is written once on
// the host and never packed again.  With a pinning allocator (hipHostMalloc, installed by the bindings on a
// GPU box) the copy is a true async DMA; without one (CPU tests) plain aligned memory is used.
//
// Buffers are carved from chunks of >= 16 MiB into power-of-two classes (64 KiB .. 64 MiB) and recycled through
// per-class free lists; a buffer is handed out as a shared_ptr whose deleter returns it, and every buffer keeps
// the pool alive.  `cap_bytes` bounds the reserved total: get() returns nullptr beyond it (the caller answers
// 503, like a full request queue).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

namespace arena {

class HostBufferPool : public std::enable_shared_from_this<HostBufferPool> {
 public:
  using AllocFn = std::function<void*(size_t)>;
  using FreeFn = std::function<void(void*)>;

  static std::shared_ptr<HostBufferPool> create(int64_t cap_bytes, AllocFn alloc = {}, FreeFn free_fn = {}) {
    return std::shared_ptr<HostBufferPool>(new HostBufferPool(cap_bytes, std::move(alloc), std::move(free_fn)));
  }
  ~HostBufferPool() {
    for (void* c : chunks_) free_(c);
  }
  HostBufferPool(const HostBufferPool&) = delete;
  HostBufferPool& operator=(const HostBufferPool&) = delete;

  std::shared_ptr<uint8_t> get(size_t bytes) {
    int cls = 0;
    while (cls < kClasses - 1 && class_bytes(cls) < bytes) ++cls;
    if (class_bytes(cls) < bytes) return nullptr;  // larger than the largest class
    uint8_t* p = nullptr;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (free_list_[cls].empty() && !grow(cls)) return nullptr;
      p = free_list_[cls].back();
      free_list_[cls].pop_back();
      ++in_use_;
    }
    auto self = shared_from_this();
    return std::shared_ptr<uint8_t>(p, [self, cls](uint8_t* q) { self->put(cls, q); });
  }
  int64_t reserved() {
    std::lock_guard<std::mutex> lk(mu_);
    return reserved_;
  }
  int64_t in_use() {
    std::lock_guard<std::mutex> lk(mu_);
    return in_use_;
  }
  bool pinned() const { return pinned_; }

 private:
  static constexpr int kClasses = 11;
  static constexpr size_t kMinClass = 64 << 10;
  static constexpr size_t kChunk = 16 << 20;
  static size_t class_bytes(int cls) { return kMinClass << cls; }

  HostBufferPool(int64_t cap, AllocFn a, FreeFn f) : cap_(cap), pinned_((bool)a) {
    alloc_ = a ? std::move(a) : AllocFn([](size_t n) { return std::aligned_alloc(4096, (n + 4095) / 4096 * 4096); });
    free_ = f ? std::move(f) : FreeFn([](void* p) { std::free(p); });
    free_list_.resize(kClasses);
  }
  bool grow(int cls) {  // under mu_
    const size_t cb = class_bytes(cls);
    const size_t chunk = cb > kChunk ? cb : kChunk;
    if (cap_ > 0 && reserved_ + (int64_t)chunk > cap_) return false;
    void* c = alloc_(chunk);
    if (c == nullptr) return false;
    chunks_.push_back(c);
    reserved_ += (int64_t)chunk;
    for (size_t o = 0; o + cb <= chunk; o += cb) free_list_[cls].push_back((uint8_t*)c + o);
    return true;
  }
  void put(int cls, uint8_t* p) {
    std::lock_guard<std::mutex> lk(mu_);
    free_list_[cls].push_back(p);
    --in_use_;
  }

  int64_t cap_;
  bool pinned_;
  AllocFn alloc_;
  FreeFn free_;
  std::mutex mu_;
  std::vector<std::vector<uint8_t*>> free_list_;
  std::vector<void*> chunks_;
  int64_t reserved_ = 0, in_use_ = 0;
};

}  // namespace arena
