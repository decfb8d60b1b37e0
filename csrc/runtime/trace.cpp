// Lazy roctx binding; see trace.h.
#include "trace.h"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace arena {
namespace trace {

namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

struct Api {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
  bool on = false;
};

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("ARENA_ROCTX");
    if (e != nullptr && e[0] == '0') return;
    void* h = nullptr;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                            "libroctx64.so"}) {
      h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
      if (h != nullptr) break;
    }
    if (h == nullptr) return;
    a.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
    a.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
    a.mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
    a.on = a.push != nullptr && a.pop != nullptr;
  });
  return a;
}

}  // namespace

bool enabled() { return api().on; }
void push(const char* name) {
  if (api().on) api().push(name);
}
void pop() {
  if (api().on) api().pop();
}
void mark(const char* name) {
  if (api().mark != nullptr) api().mark(name);
}

}  // namespace trace
}  // namespace arena
