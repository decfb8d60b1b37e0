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
// and one 8-channel group: the (R-1)*S+3 input rows it needs are loaded once
// and reused by every output row they touch, and the 9 taps' weights stay in
// registers for the whole strip.  Horizontal tap pairs (kx = 0, 1) run as
// v_dot2c_f32_bf16 on channel-regrouped bf16 pairs (v_perm), kx = 2 as an fp32
// FMA.  All index math is 32-bit (v1 used 64-bit div/mod per thread).
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
  // Per kernel row ky: taps (kx=0, kx=1) as bf16 pairs per channel for v_dot2c_f32_bf16,
  // tap kx=2 as fp32.
  unsigned wp[3][8];
  float w2[3][8];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const uint4 a = *(const uint4*)(w + (ky * 3 + 0) * p.C);
    const uint4 bq = *(const uint4*)(w + (ky * 3 + 1) * p.C);
    const unsigned av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wp[ky][2 * j] = __builtin_amdgcn_perm(bv[j], av[j], 0x05040100u);
      wp[ky][2 * j + 1] = __builtin_amdgcn_perm(bv[j], av[j], 0x07060302u);
    }
    unpack8(*(const uint4*)(w + (ky * 3 + 2) * p.C), w2[ky]);
  }
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
    const bf16* row = x + iy * p.W * p.xs;
    // the three input pixels of this row (zero outside the image: padding)
    const uint4 v0 = load16_or_zero(row + ix0 * p.xs, x, (unsigned)ix0 < (unsigned)p.W);
    const uint4 v1 = load16_or_zero(row + (ix0 + 1) * p.xs, x, (unsigned)(ix0 + 1) < (unsigned)p.W);
    const uint4 v2 = load16_or_zero(row + (ix0 + 2) * p.xs, x, (unsigned)(ix0 + 2) < (unsigned)p.W);
    const unsigned a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
    unsigned pr[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pr[2 * j] = __builtin_amdgcn_perm(a1[j], a0[j], 0x05040100u);
      pr[2 * j + 1] = __builtin_amdgcn_perm(a1[j], a0[j], 0x07060302u);
    }
    float x2[8];
    unpack8(v2, x2);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int ky = ri - r * S;
      if (ky < 0 || ky > 2) continue;  // compile-time after unrolling
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[r][i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, pr[i]),
                                                    __builtin_bit_cast(bf16x2, wp[ky][i]), acc[r][i], false);
        acc[r][i] = fmaf(x2[i], w2[ky][i], acc[r][i]);
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
