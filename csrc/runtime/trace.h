// Host-side tracing ranges for rocprofv3 (--marker-trace): the reference's
// only "tracing" is a per-request id and inline perf_counter deltas
// (architectures/monolithic/app/logger.py:17,54-57; inference.py:150-225).
// Here the native runtime also emits roctx ranges around its host phases
// (batch formation, staging copies, graph launch, result wait), so a
// rocprofv3 timeline shows host work next to the kernels it feeds.
//
// The roctx library is opened lazily with dlopen (no link-time dependency);
// without it, or with ARENA_ROCTX=0, every call is a no-op costing one
// predictable branch.
#pragma once

namespace arena {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

struct Range {
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace arena
