// Classifier tail: global average pool (K13 first half) and the per-row
// argmax / softmax / top-5 reduction (K14).
//
// Reference semantics: architectures/monolithic/app/inference.py:201-203 and
// architectures/triton/gateway/app/pipeline.py:181-183 report the top-1 raw
// logit; architectures/microservices/classification/app/inference.py:112-132
// reports softmax probabilities and a top-5 list.  The kernel returns both so
// each topology can reproduce its own reference field.
#include "common.h"
#include "launch.h"

namespace arena {

template <typename T>
__global__ __launch_bounds__(256) void avgpool_kernel(const AvgPoolParams p) {
  const int B = live_batch(p.B, p.bdev);
  const int cg = p.C >> 3;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)B * cg) return;
  const int b = (int)(tid / cg), g = (int)(tid % cg);
  const T* x = (const T*)p.x + (size_t)b * p.HW * p.C + g * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < p.HW; ++i) {
    float v[8];
    load8(x + (size_t)i * p.C, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k];
  }
  if constexpr (sizeof(T) == 4) {  // exact-fp32 pipeline: mean as sum / HW (torch adaptive_avg_pool2d)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] /= (float)p.HW;
  } else {
    const float inv = 1.0f / (float)p.HW;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
  }
  store8((T*)p.y + (size_t)b * p.C + g * 8, acc);
}

void global_avgpool(const AvgPoolParams& p, hipStream_t s) {
  if (p.C % 8 != 0) throw std::runtime_error("global_avgpool: C % 8 != 0");
  const long total = (long)p.B * (p.C / 8);
  if (total <= 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (p.f32)
    hipLaunchKernelGGL(avgpool_kernel<float>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(avgpool_kernel<bf16>, grid, dim3(256), 0, s, p);
}

constexpr int kTopkPer = 16;  // row elements per lane held in registers

// One wave per row.  Each round finds the (value, first index) maximum over
// the row with the previously chosen indices excluded.
__global__ __launch_bounds__(256) void topk_kernel(const TopkParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  int B = p.B;
  if (p.ctrl != nullptr) B = live_batch(p.B, &p.ctrl->n_crops);
  else if (p.bdev != nullptr) B = live_batch(p.B, p.bdev);
  if (row >= B) return;
  const float* x = p.logits + (size_t)row * p.ld;
  TopkResult res;
  if (p.N <= 64 * kTopkPer) {
    // Whole row in registers (16 values per lane for N <= 1024): the seven passes over it (max, sum,
    // 5 selection rounds) read no memory, so one load latency per row instead of seven chains.
    float v[kTopkPer];
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j) {
      const int i = lane + 64 * j;
      v[j] = i < p.N ? x[i] : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j) mx = fmaxf(mx, v[j]);
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j)
      if (lane + 64 * j < p.N) se += __expf(v[j] - mx);
    se = wave_sum(se);
    const float inv = 1.0f / se;
    unsigned taken = 0;  // bit j: element lane + 64 j already chosen
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < kTopkPer; ++j) {
        const int i = lane + 64 * j;
        if (i < p.N && !((taken >> j) & 1u) && (v[j] > bv || (v[j] == bv && i < bi))) { bv = v[j]; bi = i; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if ((bi & 63) == lane) taken |= 1u << (bi >> 6);
      res.idx[k] = bi;
      res.logit[k] = bv;
      res.prob[k] = __expf(bv - mx) * inv;
    }
  } else {
    float mx = -INFINITY;
    for (int i = lane; i < p.N; i += 64) mx = fmaxf(mx, x[i]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int i = lane; i < p.N; i += 64) se += __expf(x[i] - mx);
    se = wave_sum(se);
    const float inv = 1.0f / se;
    int chosen[5] = {-1, -1, -1, -1, -1};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int i = lane; i < p.N; i += 64) {
        bool skip = false;
#pragma unroll
        for (int q = 0; q < 5; ++q) skip |= (q < k) && (chosen[q] == i);
        const float v = x[i];
        if (!skip && (v > bv || (v == bv && i < bi))) { bv = v; bi = i; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      chosen[k] = bi;
      res.idx[k] = bi;
      res.logit[k] = bv;
      res.prob[k] = __expf(bv - mx) * inv;
    }
  }
  res.pad_ = 0;
  if (lane == 0) {
    const int base = p.ctrl != nullptr ? p.ctrl->crop_base : 0;
    p.out[base + row] = res;
  }
}

void topk_softmax(const TopkParams& p, hipStream_t s) {
  if (p.N < 5) throw std::runtime_error("topk_softmax: N < 5");
  if (p.B <= 0) return;
  hipLaunchKernelGGL(topk_kernel, dim3((p.B + 3) / 4), dim3(256), 0, s, p);
}

}  // namespace arena

namespace arena {

// Zero-fill used inside captured graphs instead of hipMemsetAsync: memset
// nodes of a hipGraph captured before PyTorch's first H2D copies stopped
// taking effect afterwards on ROCm 7.0 (kernel nodes were unaffected), so
// the executor's graphs contain kernel nodes only.
__global__ __launch_bounds__(256) void zero_fill_kernel(uint4* p, size_t n16, uint8_t* tail, int n_tail) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) p[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i < (size_t)n_tail) tail[i] = 0;
}

// Stage timestamp (planner OP_STAMP): the device's constant-rate wall clock (wall_clock64, the 100 MHz
// REALTIME counter; rate from hipDeviceAttributeWallClockRate) written where the graph reaches this op, so the
// executor reports detection / classification device time per batch without breaking the graph up.
__global__ void stamp_kernel(unsigned long long* dst) {
  const unsigned long long t = wall_clock64();
  if (threadIdx.x == 0) dst[threadIdx.x] = t;
}

void stamp(void* dst, hipStream_t s) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, (unsigned long long*)dst);
}

void zero_fill(void* ptr, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  if (((uintptr_t)ptr & 15) != 0) throw std::runtime_error("zero_fill: pointer must be 16-byte aligned");
  const size_t n16 = bytes / 16;
  const int n_tail = (int)(bytes - n16 * 16);
  const size_t threads = n16 > (size_t)n_tail ? n16 : (size_t)n_tail;
  hipLaunchKernelGGL(zero_fill_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, (uint4*)ptr, n16,
                     (uint8_t*)ptr + n16 * 16, n_tail);
}

}  // namespace arena
