// MobileNetV2 head conv (1x1, 320 -> 1280, ReLU6) fused with the global
// average pool (K13 first half).
//
// Reference (torchvision mobilenet_v2 under ONNX Runtime, per crop:
// architectures/monolithic/app/inference.py:196): features[-1] is a
// Conv1x1+BN+ReLU6 to 1280 channels at 7x7, followed by
// adaptive_avg_pool2d(1).  Unfused, the 7x7x1280 map (125 KB per crop) is
// written to HBM and read back once by a separate pooling kernel; here every
// workgroup owns all HW pixels of one crop for a 256-channel slice, so the
// pool is a register / cross-lane reduction of its own MFMA accumulators.
//
// Per workgroup (256 threads = 4 waves): crop b, channels n0 .. n0+127.
//   stage   x[b] (HW <= 64 pixels x K channels, bf16) -> LDS, rows padded by
//           16 B (stride 656 B for K = 320: conflict-free 16-B row reads);
//           pixels HW..63 are zero.
//   MFMA    wave w owns 32 output channels (2 N-fragments) x 64 pixels
//           (4 M-fragments); A = weight rows, all 10 K slabs loaded into
//           registers up front (issued before the staging loads, so the
//           whole workgroup pays one memory latency), B = pixel rows (LDS).
//           8 v_mfma_f32_16x16x32_bf16 per 32-deep K slab.
//   pool    bias + activation per element, sum over the valid pixels (in-lane
//           over M-fragments, then xor-shuffles over the 16 pixel lanes),
//           scale by 1/HW, bf16 store of 4 channels per lane group.
// The pooled vector is summed in fp32 before a single bf16 rounding (the
// unfused path rounds every 7x7 activation to bf16 first).
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {
constexpr int kNS = 128;  // output channels per workgroup
constexpr int kNF = 2;    // 16-channel N-fragments per wave
constexpr int kMaxHW = 64;
}  // namespace

template <int KSLABS>
__global__ __launch_bounds__(256) void head_pool_kernel(const HeadPoolParams p) {
  constexpr int K = KSLABS * 32;
  constexpr int PITCH = K * 2 + 16;  // bytes per staged pixel row
  __shared__ __align__(16) uint8_t xs[kMaxHW * PITCH];

  const int nslices = (p.N + kNS - 1) / kNS;
  const int b = blockIdx.x / nslices;
  const int n0 = (blockIdx.x - b * nslices) * kNS;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;

  // ---- all weights of this wave's channels -> registers (one latency for the whole K loop)
  const bf16* w = (const bf16*)p.w;
  const int nw = n0 + wave * (16 * kNF);
  bf16x8 wa[KSLABS][kNF];
#pragma unroll
  for (int s = 0; s < KSLABS; ++s)
#pragma unroll
    for (int f = 0; f < kNF; ++f) {
      const int n = nw + f * 16 + row;
      wa[s][f] = n < p.Npad ? *(const bf16x8*)(w + (size_t)n * p.Kpad + s * 32 + kq * 8) : bf16x8{};
    }

  // ---- stage the crop's pixels (16-B pieces)
  const bf16* xb = (const bf16*)p.x + (size_t)b * p.HW * p.xs;
  constexpr int CPR = K / 8;
  for (int i = tid; i < kMaxHW * CPR; i += 256) {
    const int px = i / CPR, c = i - px * CPR;
    const bool ok = px < p.HW && c * 8 < p.K;
    *(uint4*)(xs + px * PITCH + c * 16) = load16_or_zero(xb + (size_t)px * p.xs + c * 8, xb, ok);
  }
  __syncthreads();

  f32x4 acc[kNF][4];  // [N-fragment][M-fragment]
#pragma unroll
  for (int f = 0; f < kNF; ++f)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < KSLABS; ++s) {
    bf16x8 xv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) xv[m] = *(const bf16x8*)(xs + (m * 16 + row) * PITCH + s * 64 + kq * 16);
#pragma unroll
    for (int f = 0; f < kNF; ++f)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        acc[f][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s][f], xv[m], acc[f][m], 0, 0, 0);
  }

  // ---- epilogue: bias + act, mean over the valid pixels, one bf16 store per 4 channels
  // acc[f][m][i]: channel nw + f*16 + kq*4 + i, pixel m*16 + row
  const float inv = 1.0f / (float)p.HW;
  bf16* y = (bf16*)p.y + (size_t)b * p.ys;
#pragma unroll
  for (int f = 0; f < kNF; ++f) {
    const int cb = nw + f * 16 + kq * 4;
    const bool cok = cb < p.N;
    const float4 bias = cok ? *(const float4*)(p.bias + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (m * 16 + row < p.HW) {
        sum[0] += apply_act(acc[f][m][0] + bias.x, p.act);
        sum[1] += apply_act(acc[f][m][1] + bias.y, p.act);
        sum[2] += apply_act(acc[f][m][2] + bias.z, p.act);
        sum[3] += apply_act(acc[f][m][3] + bias.w, p.act);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) sum[i] += __shfl_xor(sum[i], o, 64);
      sum[i] *= inv;
    }
    if (row == 0 && cok) *(uint2*)(y + cb) = pack4(sum);
  }
}

void head_pool(const HeadPoolParams& p, hipStream_t s) {
  if (p.HW <= 0 || p.HW > kMaxHW) throw std::runtime_error("head_pool: HW must be 1..64");
  if (p.Kpad != 320 || p.K > p.Kpad) throw std::runtime_error("head_pool: instantiated for Kpad 320");
  if (p.N % 4 || p.Npad % 16 || p.Npad < p.N) throw std::runtime_error("head_pool: bad output channel geometry");
  if (p.xs % 8 || p.ys % 4) throw std::runtime_error("head_pool: strides must keep 16-B / 8-B alignment");
  const long grid = (long)p.B * ((p.N + kNS - 1) / kNS);
  if (grid <= 0) return;
  hipLaunchKernelGGL(head_pool_kernel<10>, dim3((unsigned)grid), dim3(256), 0, s, p);
}


// ---------------------------------------------------------------------------
// fp32 programs: the same fusion at fp32 accuracy on the bf16 matrix cores (triple-bf16 split, six partial
// products per MFMA step, conv_f32.hip).  Unfused, the fp32 head was a 1x1 conv writing the 7x7x1280 fp32 map
// (251 KB per crop) plus an avgpool kernel reading it back: 73 + 17 us for 128 crops
// (profiles/r2_fp32_stream2_ops.md ops 109-110).  The crop's pixels are split into [h|m|l] bf16 planes in LDS
// once (64 rows x 1952 B: a pitch of 2 (mod 4) 16-B slots); each wave splits its weight fragments in
// registers, one K slab ahead of use.
// 8 waves x 32 channels = 256 output channels per workgroup (5 per crop for 1280): the staged, split pixel
// block (the workgroup's fixed cost) is shared by twice the channels of a 4-wave workgroup.
constexpr int kNSF = 256, kHeadF32Threads = 512;

// The split pixel block is staged in two K halves of 160 channels (64 rows x 992 B = 62 KiB, a pitch of 2 (mod 4)
// 16-B slots): two workgroups fit a CU instead of one (the whole-K block took 122 KiB), so one workgroup's staging
// and its weight-load latency overlap the other's MFMAs.
template <int KSLABS>
__global__ __launch_bounds__(kHeadF32Threads) void head_pool_f32_kernel(const HeadPoolParams p) {
  constexpr int K = KSLABS * 32;
  static_assert(KSLABS % 2 == 0, "two K halves of whole slabs");
  constexpr int KH = K / 2, SH = KSLABS / 2;  // channels / slabs per staged half
  constexpr int PITCH = 6 * KH + 32;          // bytes per staged pixel row: three bf16 planes + pad
  extern __shared__ __align__(16) uint8_t xsf[];

  const int nslices = (p.N + kNSF - 1) / kNSF;
  const int b = blockIdx.x / nslices;
  const int n0 = (blockIdx.x - b * nslices) * kNSF;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const float* w = (const float*)p.w;
  const int nw = n0 + wave * (16 * kNF);

  float4 wr[kNF][2];
  auto load_w = [&](int s) {
#pragma unroll
    for (int f = 0; f < kNF; ++f) {
      const int n = nw + f * 16 + row;
      const float* src = w + (size_t)(n < p.Npad ? n : 0) * p.Kpad + s * 32 + kq * 8;
      wr[f][0] = *(const float4*)src;
      wr[f][1] = *(const float4*)(src + 4);
      if (n >= p.Npad) wr[f][0] = wr[f][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  load_w(0);

  const float* xb = (const float*)p.x + (size_t)b * p.HW * p.xs;
  constexpr int CPR = KH / 4;
  // stage K half h of the crop's pixels as split planes (pixels HW..63 and channels past K are zero)
  auto stage = [&](int h) {
    for (int i = tid; i < kMaxHW * CPR; i += kHeadF32Threads) {
      const int px = i / CPR, c = i - px * CPR;
      const int ch = h * KH + c * 4;
      const bool ok = px < p.HW && ch < p.K;
      float4 v = *(const float4*)(ok ? xb + (size_t)px * p.xs + ch : xb);
      if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
      const float f[4] = {v.x, v.y, v.z, v.w};
      bf16x4 hh, m, l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hh[j] = (bf16)f[j];
        const float r = f[j] - (float)hh[j];
        m[j] = (bf16)r;
        l[j] = (bf16)(r - (float)m[j]);
      }
      uint8_t* d = xsf + px * PITCH + c * 8;
      *(bf16x4*)d = hh;
      *(bf16x4*)(d + 2 * KH) = m;
      *(bf16x4*)(d + 4 * KH) = l;
    }
  };

  f32x4 acc[kNF][4];
#pragma unroll
  for (int f = 0; f < kNF; ++f)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) acc[f][mm] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();  // every wave is done with the first half before it is replaced
    stage(h);
    __syncthreads();
#pragma unroll 1
    for (int s = h * SH; s < (h + 1) * SH; ++s) {
      bf16x8 ah[kNF], am[kNF], al[kNF];
#pragma unroll
      for (int f = 0; f < kNF; ++f) {
        const float v[8] = {wr[f][0].x, wr[f][0].y, wr[f][0].z, wr[f][0].w, wr[f][1].x, wr[f][1].y, wr[f][1].z, wr[f][1].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ah[f][j] = (bf16)v[j];
          const float r = v[j] - (float)ah[f][j];
          am[f][j] = (bf16)r;
          al[f][j] = (bf16)(r - (float)am[f][j]);
        }
      }
      if (s + 1 < KSLABS) load_w(s + 1);  // next slab's weights in flight during this slab's MFMAs
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        const uint8_t* r = xsf + (mm * 16 + row) * PITCH + (s - h * SH) * 64 + kq * 16;
        const bf16x8 bh = *(const bf16x8*)r, bm = *(const bf16x8*)(r + 2 * KH), bl = *(const bf16x8*)(r + 4 * KH);
#pragma unroll
        for (int f = 0; f < kNF; ++f) {
          f32x4 c = acc[f][mm];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[f], bm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[f], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[f], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bm, c, 0, 0, 0);
          acc[f][mm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[f], bh, c, 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: bias + act, mean over the valid pixels, fp32 store of 4 channels per lane group
  const float inv = 1.0f / (float)p.HW;
  float* y = (float*)p.y + (size_t)b * p.ys;
#pragma unroll
  for (int f = 0; f < kNF; ++f) {
    const int cb = nw + f * 16 + kq * 4;
    const bool cok = cb < p.N;
    const float4 bias = cok ? *(const float4*)(p.bias + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      if (mm * 16 + row < p.HW) {
        sum[0] += apply_act(acc[f][mm][0] + bias.x, p.act);
        sum[1] += apply_act(acc[f][mm][1] + bias.y, p.act);
        sum[2] += apply_act(acc[f][mm][2] + bias.z, p.act);
        sum[3] += apply_act(acc[f][mm][3] + bias.w, p.act);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) sum[i] += __shfl_xor(sum[i], o, 64);
      sum[i] *= inv;
    }
    if (row == 0 && cok) *(float4*)(y + cb) = make_float4(sum[0], sum[1], sum[2], sum[3]);
  }
}

constexpr int kHeadF32Lds = kMaxHW * (6 * 160 + 32);  // one staged K half (head_pool_f32_kernel)

void head_pool_f32_prepare() {
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)head_pool_f32_kernel<10>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kHeadF32Lds));
}

void head_pool_f32(const HeadPoolParams& p, hipStream_t s) {
  if (p.HW <= 0 || p.HW > kMaxHW) throw std::runtime_error("head_pool_f32: HW must be 1..64");
  if (p.Kpad != 320 || p.K > p.Kpad || p.K % 4) throw std::runtime_error("head_pool_f32: instantiated for Kpad 320");
  if (p.N % 4 || p.Npad % 16 || p.Npad < p.N) throw std::runtime_error("head_pool_f32: bad output channel geometry");
  if (p.xs % 4 || p.ys % 4) throw std::runtime_error("head_pool_f32: strides must keep 16-B alignment");
  const long grid = (long)p.B * ((p.N + kNSF - 1) / kNSF);
  if (grid <= 0) return;
  hipLaunchKernelGGL(head_pool_f32_kernel<10>, dim3((unsigned)grid), dim3(kHeadF32Threads), kHeadF32Lds, s, p);
}

}  // namespace arena
