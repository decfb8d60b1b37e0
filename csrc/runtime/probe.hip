// Diagnostic probe for hipGraph kernel-argument lifetime (no memory faults possible).
//
// A one-kernel graph whose only inputs are by-value scalars writes them into a
// __device__ array (address not taken from the kernel arguments).  Relaunching
// the graph after other work and reading the array back shows whether the
// graph's captured kernel arguments survived.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/common.h"

namespace arena {

__device__ int g_probe[16];

struct ProbeArgs {
  int v[16];
};

__global__ void probe_kernel(const ProbeArgs a) {
  if (threadIdx.x < 16) g_probe[threadIdx.x] = a.v[threadIdx.x];
}

struct GraphProbe {
  hipGraphExec_t exec = nullptr;
  hipStream_t stream = nullptr;
};

void* probe_create(int base) {
  auto* p = new GraphProbe();
  ARENA_HIP_CHECK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
  ProbeArgs a;
  for (int i = 0; i < 16; ++i) a.v[i] = base + i;
  hipGraph_t g = nullptr;
  ARENA_HIP_CHECK(hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, p->stream, a);
  ARENA_HIP_CHECK(hipStreamEndCapture(p->stream, &g));
  ARENA_HIP_CHECK(hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0));
  ARENA_HIP_CHECK(hipGraphDestroy(g));
  return p;
}

std::vector<int> probe_launch(void* h) {
  auto* p = (GraphProbe*)h;
  int zero[16] = {0};
  ARENA_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), zero, sizeof(zero)));
  ARENA_HIP_CHECK(hipGraphLaunch(p->exec, p->stream));
  ARENA_HIP_CHECK(hipStreamSynchronize(p->stream));
  std::vector<int> out(16);
  ARENA_HIP_CHECK(hipMemcpyFromSymbol(out.data(), HIP_SYMBOL(g_probe), sizeof(int) * 16));
  return out;
}

void probe_destroy(void* h) {
  auto* p = (GraphProbe*)h;
  hipGraphExecDestroy(p->exec);
  hipStreamDestroy(p->stream);
  delete p;
}

}  // namespace arena
