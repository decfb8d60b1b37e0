// Host-only check of the cross-device guard (csrc/runtime/peer.h) with a fake peer-access table: 4 "GPUs", GPU 3
// has no peer path to 0 and 1.  Built and run by tests/test_split_gpu.py (CPU part).
#include <cstdio>
#include <stdexcept>
#include <string>

#include "runtime/peer.h"

int main() {
  auto can = [](int dst, int src) { return !((dst == 3 && src < 2) || (src == 3 && dst < 2)); };
  int fails = 0;
  auto expect_ok = [&](int d, int s) {
    try {
      arena::require_peer_access(d, s, "test", can);
    } catch (const std::exception& e) {
      std::printf("unexpected refusal %d<-%d: %s\n", d, s, e.what());
      ++fails;
    }
  };
  auto expect_refused = [&](int d, int s) {
    try {
      arena::require_peer_access(d, s, "SplitInstance", can);
      std::printf("missing refusal %d<-%d\n", d, s);
      ++fails;
    } catch (const std::runtime_error& e) {
      const std::string m = e.what();
      if (m.find("GPU " + std::to_string(d)) == std::string::npos || m.find("SplitInstance") == std::string::npos) {
        std::printf("unclear message: %s\n", m.c_str());
        ++fails;
      }
    }
  };
  expect_ok(0, 0);
  expect_ok(0, 1);
  expect_ok(2, 3);
  expect_ok(-1, 3);  // unknown source device: nothing to check
  expect_refused(3, 0);
  expect_refused(1, 3);
  if (fails) return 1;
  std::printf("peer_check: ok\n");
  return 0;
}
