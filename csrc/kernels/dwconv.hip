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

__global__ __launch_bounds__(256) void dwconv3x3_kernel(const DwParams p) {
  const int B = live_batch(p.B, p.bdev);
  const int cg = p.C >> 3;
  const long total = (long)B * p.Ho * p.Wo * cg;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int g = (int)(tid % cg);
  const long pix = tid / cg;
  const int ox = (int)(pix % p.Wo);
  const long t2 = pix / p.Wo;
  const int oy = (int)(t2 % p.Ho);
  const int b = (int)(t2 / p.Ho);
  const int c0 = g * 8;

  const bf16* x = (const bf16*)p.x;
  const bf16* w = (const bf16*)p.w;
  float acc[8];
  {
    const float4 b0 = *(const float4*)(p.bias + c0);
    const float4 b1 = *(const float4*)(p.bias + c0 + 4);
    acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w;
    acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
  }
  const int iy0 = oy * p.stride - 1, ix0 = ox * p.stride - 1;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int iy = iy0 + kh;
    if ((unsigned)iy >= (unsigned)p.H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ix = ix0 + kw;
      if ((unsigned)ix >= (unsigned)p.W) continue;
      float xv[8], wv[8];
      unpack8(*(const uint4*)(x + ((size_t)(b * p.H + iy) * p.W + ix) * p.xs + c0), xv);
      unpack8(*(const uint4*)(w + (size_t)(kh * 3 + kw) * p.C + c0), wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(xv[i], wv[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = apply_act(acc[i], p.act);
  *(uint4*)((bf16*)p.y + ((size_t)(b * p.Ho + oy) * p.Wo + ox) * p.ys + c0) = pack8(acc);
}

void dwconv3x3(const DwParams& p, hipStream_t s) {
  if (p.C % 8 != 0 || p.xs % 8 != 0 || p.ys % 8 != 0)
    throw std::runtime_error("dwconv3x3: C, xs, ys must be multiples of 8");
  const long total = (long)p.B * p.Ho * p.Wo * (p.C / 8);
  if (total <= 0) return;
  hipLaunchKernelGGL(dwconv3x3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

}  // namespace arena
