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

}  // namespace arena
