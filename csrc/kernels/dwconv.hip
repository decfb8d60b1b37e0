// Depthwise 3x3 convolution (+ folded BN bias + ReLU6) in NHWC bf16.
//
// Replaces the 17 grouped Conv nodes of MobileNetV2's inverted-residual
// blocks that ONNX Runtime runs on the CPU in the reference
// (architectures/microservices/classification/app/inference.py:110 and
// architectures/monolithic/app/inference.py:196 call session.run).
// Depthwise convs have no reduction across channels, so they are VALU work:
// each thread owns 8 consecutive channels (one 16-byte vector) of one output
// pixel; consecutive threads take consecutive channel groups of the same
// pixel, so every tap load of a wave is one coalesced NHWC row segment.
#include "common.h"
#include "launch.h"

namespace arena {

// Each thread computes a vertical strip of R output rows for one pixel column
// and one 8-channel group: the (R-1)*S+3 input rows it needs are loaded and
// converted once and reused by every output row they touch, and the 9 taps'
// weights stay in registers (fp32) for the whole strip.  All index math is
// 32-bit (v1 used 64-bit div/mod per thread).
template <int R, int S>
__global__ __launch_bounds__(256) void dwconv3x3_kernel(const DwParams p) {
  const int B = live_batch(p.B, p.bdev);
  const int cg = p.C >> 3;
  const int strips = (p.Ho + R - 1) / R;
  const int total = B * strips * p.Wo * cg;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int g = tid % cg;
  int t = tid / cg;
  const int ox = t % p.Wo;
  t /= p.Wo;
  const int st = t % strips;
  const int b = t / strips;
  const int c0 = g * 8;
  const int oy0 = st * R;

  const bf16* x = (const bf16*)p.x + (size_t)b * p.H * p.W * p.xs + c0;
  const bf16* w = (const bf16*)p.w + c0;
  float wt[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k) unpack8(*(const uint4*)(w + k * p.C), wt[k]);
  float acc[R][8];
  {
    const float4 b0 = *(const float4*)(p.bias + c0);
    const float4 b1 = *(const float4*)(p.bias + c0 + 4);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc[r][0] = b0.x; acc[r][1] = b0.y; acc[r][2] = b0.z; acc[r][3] = b0.w;
      acc[r][4] = b1.x; acc[r][5] = b1.y; acc[r][6] = b1.z; acc[r][7] = b1.w;
    }
  }
  constexpr int NIN = (R - 1) * S + 3;
  const int iy0 = oy0 * S - 1, ix0 = ox * S - 1;
#pragma unroll
  for (int ri = 0; ri < NIN; ++ri) {
    const int iy = iy0 + ri;
    if ((unsigned)iy >= (unsigned)p.H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ix0 + kx;
      if ((unsigned)ix >= (unsigned)p.W) continue;
      float xv[8];
      unpack8(*(const uint4*)(x + (iy * p.W + ix) * p.xs), xv);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ky = ri - r * S;
        if (ky < 0 || ky > 2) continue;  // compile-time after unrolling
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[r][i] = fmaf(xv[i], wt[ky * 3 + kx][i], acc[r][i]);
      }
    }
  }
  bf16* y = (bf16*)p.y + (size_t)b * p.Ho * p.Wo * p.ys + c0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int oy = oy0 + r;
    if (oy >= p.Ho) break;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[r][i] = apply_act(acc[r][i], p.act);
    *(uint4*)(y + (oy * p.Wo + ox) * p.ys) = pack8(acc[r]);
  }
}

template <int R, int S>
static void dw_launch(const DwParams& p, hipStream_t s) {
  const long total = (long)p.B * ((p.Ho + R - 1) / R) * p.Wo * (p.C / 8);
  if (total <= 0) return;
  if (total >= (1L << 31) || (long)p.H * p.W * p.xs >= (1L << 31)) throw std::runtime_error("dwconv3x3: too large");
  hipLaunchKernelGGL((dwconv3x3_kernel<R, S>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

void dwconv3x3(const DwParams& p, hipStream_t s) {
  if (p.C % 8 != 0 || p.xs % 8 != 0 || p.ys % 8 != 0)
    throw std::runtime_error("dwconv3x3: C, xs, ys must be multiples of 8");
  if (p.stride == 1)
    dw_launch<4, 1>(p, s);  // 14x14: 4+4+4+2 strips, 7x7: 4+3
  else
    dw_launch<2, 2>(p, s);
}

}  // namespace arena
