// Fully connected layer (1x1 conv on a 1x1 map: MobileNetV2's classifier
// 1280 -> 1000, K13 second half) as a split-K MFMA GEMM.
//
// Reference: torchvision mobilenet_v2 classifier Linear(1280, 1000) per crop
// (architectures/monolithic/app/inference.py:196).  M = crops (<= a few
// hundred), N = 1000, K = 1280: too little M for the tiled conv kernels,
// whose workgroups walked all 40 K slabs with a dependent load per slab
// (27 us for 126 crops).  Here a workgroup owns 16 crops x 32 classes and
// its 4 waves split K in quarters: every wave issues all of its weight and
// activation loads up front (one memory latency), runs KQS x 2 MFMAs, and
// the four partial tiles are summed through LDS by wave 0, which applies
// bias / activation and stores fp32 logits (or bf16).
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace arena {

template <int KQS>  // 32-deep K slabs per wave (K = 4 * KQS * 32)
__global__ __launch_bounds__(256) void fc_splitk_kernel(const ConvParams p) {
  __shared__ f32x4 red[3][2][64];
  const int ntn = (p.Cout + 31) / 32;
  const int mt = blockIdx.x / ntn;
  const int n0 = (blockIdx.x - mt * ntn) * 32, m0 = mt * 16;
  const int live = p.bdev ? live_batch(p.B, p.bdev) : p.B;
  if (m0 >= live) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int k0 = wave * KQS * 32;

  const bf16* w = (const bf16*)p.w;
  const bf16* x = (const bf16*)p.x;
  bf16x8 wa[KQS][2], xv[KQS];
  const int m = m0 + row;
  const bool mok = m < live;
#pragma unroll
  for (int s = 0; s < KQS; ++s) {
    const int k = k0 + s * 32 + kq * 8;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int n = n0 + f * 16 + row;
      wa[s][f] = n < p.Cout_pad ? *(const bf16x8*)(w + (size_t)n * p.Kpad + k) : bf16x8{};
    }
    xv[s] = __builtin_bit_cast(bf16x8, load16_or_zero(x + (size_t)m * p.xs + k, x, mok && k < p.Cin));
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < KQS; ++s)
#pragma unroll
    for (int f = 0; f < 2; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s][f], xv[s], acc[f], 0, 0, 0);

  if (wave > 0) {
    red[wave - 1][0][lane] = acc[0];
    red[wave - 1][1][lane] = acc[1];
  }
  __syncthreads();
  if (wave != 0 || !mok) return;
  // acc[f][i]: class n0 + f*16 + kq*4 + i, crop m
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    f32x4 a = acc[f] + red[0][f][lane] + red[1][f][lane] + red[2][f][lane];
    const int cb = n0 + f * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bb = *(const float4*)(p.bias + cb);
    float v[4] = {apply_act(a[0] + bb.x, p.act), apply_act(a[1] + bb.y, p.act), apply_act(a[2] + bb.z, p.act),
                  apply_act(a[3] + bb.w, p.act)};
    if (p.f32out)
      *(float4*)((float*)p.y + (size_t)m * p.ys + cb) = make_float4(v[0], v[1], v[2], v[3]);
    else
      *(uint2*)((bf16*)p.y + (size_t)m * p.ys + cb) = pack4(v);
  }
}

static const bool g_conv_fc = [] {
  const char* e = std::getenv("ARENA_CONV_FC");
  return e ? std::atoi(e) != 0 : true;
}();

// 1x1 conv over a 1x1 map with K = 1280 (4 waves x 10 slabs); false when the shape does not apply.
bool conv_fc(const ConvParams& p, hipStream_t s) {
  if (!g_conv_fc || p.KH != 1 || p.KW != 1 || p.H != 1 || p.W != 1 || p.Ho != 1 || p.Wo != 1 || p.stride != 1 ||
      p.res != nullptr || p.y2 != nullptr || p.pw_w != nullptr || p.Kpad != 1280 || p.Cin > p.Kpad ||
      p.xs % 8 != 0 || p.ys % 4 != 0)
    return false;
  const long grid = (long)((p.B + 15) / 16) * ((p.Cout + 31) / 32);
  if (grid <= 0) return true;
  hipLaunchKernelGGL(fc_splitk_kernel<10>, dim3((unsigned)grid), dim3(256), 0, s, p);
  return true;
}

}  // namespace arena
