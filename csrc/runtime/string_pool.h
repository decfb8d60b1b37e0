// Recycled request-body buffers for the serving front ends.
//
// A request body is filled on the connection's I/O thread and released on another thread (a decode thread, or a
// proxy worker for the gateway).  Allocated with malloc and freed that way, every request moved a ~100-600 KB
// chunk between glibc arenas: the I/O threads' arenas fragmented and held ~115 MB after a protocol sweep until a
// periodic malloc_trim returned it (round 5).  Here the body's storage goes back to a shared
// free list instead of to the allocator, and the I/O thread's next request reuses its capacity: in steady state
// no body is allocated or freed at all, on any thread.
//
// The pool is bounded in count (`max_keep`) and in the capacity it keeps per string (`max_capacity`): a burst
// beyond it, or one very large upload, is freed normally.
#pragma once

#include <cstddef>
#include <mutex>
#include <string>
#include <vector>

namespace arena {

class StringPool {
 public:
  explicit StringPool(size_t max_keep = 1024, size_t max_capacity = (size_t)8 << 20)
      : max_keep_(max_keep), max_capacity_(max_capacity) {
    free_.reserve(max_keep_);
  }

  // an empty string, with the capacity of a recycled one when there is one
  std::string get() {
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.empty()) {
      ++misses_;
      return std::string();
    }
    std::string s = std::move(free_.back());
    free_.pop_back();
    ++hits_;
    return s;
  }

  // return a string's storage (its contents are dropped); called from any thread
  void put(std::string&& s) {
    if (s.capacity() <= 64 || s.capacity() > max_capacity_) return;  // SSO / outsized: let it go
    s.clear();
    std::lock_guard<std::mutex> lk(mu_);
    if (free_.size() >= max_keep_) return;  // full: the caller's string keeps (and frees) its storage
    free_.push_back(std::move(s));
  }

  size_t hits() const {
    std::lock_guard<std::mutex> lk(mu_);
    return hits_;
  }
  size_t misses() const {
    std::lock_guard<std::mutex> lk(mu_);
    return misses_;
  }
  size_t kept() const {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.size();
  }

 private:
  mutable std::mutex mu_;
  std::vector<std::string> free_;
  size_t max_keep_, max_capacity_;
  size_t hits_ = 0, misses_ = 0;
};

}  // namespace arena
