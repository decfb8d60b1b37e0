// Race / memory check for the front end's request-body pool (csrc/runtime/string_pool.h), built host-only under
// ThreadSanitizer and AddressSanitizer by tests/test_batcher_native.py.  As in the server: "I/O" threads take a
// body from the pool and fill it, hand it to "decode" threads through a queue, and those put it back; some bodies
// are oversized (freed, not kept) and the pool is bounded.
//
//   string_pool_stress [iterations per producer]
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/string_pool.h"

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  constexpr int kProducers = 4, kConsumers = 4;
  arena::StringPool pool(64, 1 << 20);
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::string> q;
  std::atomic<int> producers_left{kProducers};
  std::atomic<long> checked{0}, bad{0};
  std::vector<std::thread> th;
  for (int p = 0; p < kProducers; ++p)
    th.emplace_back([&, p]() {
      for (int i = 0; i < iters; ++i) {
        std::string body = pool.get();
        if (!body.empty()) bad.fetch_add(1);  // a recycled body must come back empty
        const size_t n = (i % 97 == 0) ? (size_t)(2 << 20) : (size_t)(1000 + (i * 131 + p * 17) % 150000);
        body.assign(n, (char)('a' + (i + p) % 26));
        {
          std::lock_guard<std::mutex> lk(mu);
          q.push_back(std::move(body));
        }
        cv.notify_one();
      }
      producers_left.fetch_sub(1);
      cv.notify_all();
    });
  for (int c = 0; c < kConsumers; ++c)
    th.emplace_back([&]() {
      for (;;) {
        std::string body;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return !q.empty() || producers_left.load() == 0; });
          if (q.empty()) return;
          body = std::move(q.front());
          q.pop_front();
        }
        // every byte is the producer's fill: no other thread wrote into a body in flight
        for (size_t k = 1; k < body.size(); k += 4093)
          if (body[k] != body[0]) bad.fetch_add(1);
        checked.fetch_add(1);
        pool.put(std::move(body));
      }
    });
  for (auto& t : th) t.join();
  const long want = (long)kProducers * iters;
  if (bad.load() != 0 || checked.load() != want || pool.kept() > 64) {
    std::printf("string_pool_stress: FAILED (bad %ld, checked %ld of %ld, kept %zu)\n", bad.load(), checked.load(),
                want, pool.kept());
    return 1;
  }
  std::printf("string_pool_stress: ok (%ld bodies, %zu recycled, %zu allocated, %zu kept)\n", checked.load(),
              pool.hits(), pool.misses(), pool.kept());
  return 0;
}
