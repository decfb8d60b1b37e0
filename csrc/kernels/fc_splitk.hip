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
namespace {
__device__ __forceinline__ float f4_get(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}
__device__ __forceinline__ float4 load_f4_or_zero(const float* p, const float* safe, bool ok) {
  const float4 v = *(const float4*)(ok ? p : safe);
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}
}  // namespace
}  // namespace arena

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


// ---------------------------------------------------------------------------
// Exact-fp32 counterpart (fp32 programs): same tiling (16 crops x 32 classes per workgroup, 4 waves split K in
// quarters, partial tiles summed through LDS in wave order = deterministic), fp32 activations / weights and
// v_mfma_f32_16x16x4_f32 (one rounding per product).  The fp32 program ran this layer through the tiled
// implicit-GEMM conv: 96 workgroups walking 40 K chunks each, 38 us for 128 crops
// (profiles/r2_fp32_stream2_ops.md op 111).  Lane l supplies k = 16 c + 4 (l >> 4) + s in MFMA step s of
// chunk c: one float4 of the weight row / activation row per 16-deep chunk.
template <int KQC>  // 16-deep K chunks per wave (K = 4 * KQC * 16)
__global__ __launch_bounds__(256) void fc_splitk_f32_kernel(const ConvParams p) {
  __shared__ f32x4 red[3][2][64];
  const int ntn = (p.Cout + 31) / 32;
  const int mt = blockIdx.x / ntn;
  const int n0 = (blockIdx.x - mt * ntn) * 32, m0 = mt * 16;
  const int live = p.bdev ? live_batch(p.B, p.bdev) : p.B;
  if (m0 >= live) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int k0 = wave * KQC * 16;
  const float* w = (const float*)p.w;
  const float* x = (const float*)p.x;
  const int m = m0 + row;
  const bool mok = m < live;
  const float* wr0 = w + (size_t)min(n0 + row, p.Cout_pad - 1) * p.Kpad + k0 + kq * 4;
  const float* wr1 = w + (size_t)min(n0 + 16 + row, p.Cout_pad - 1) * p.Kpad + k0 + kq * 4;
  const float* xr = x + (size_t)(mok ? m : 0) * p.xs + k0 + kq * 4;

  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  constexpr int G = 5;  // chunks whose loads are issued together (KQC % G == 0)
  static_assert(KQC % G == 0, "fc_splitk_f32: chunk grouping");
#pragma unroll 1
  for (int c0 = 0; c0 < KQC; c0 += G) {
    float4 a0[G], a1[G], xv[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int k = (c0 + g) * 16;
      a0[g] = *(const float4*)(wr0 + k);
      a1[g] = *(const float4*)(wr1 + k);
      xv[g] = load_f4_or_zero(xr + k, x, mok && k0 + k + kq * 4 < p.Cin);
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const float xs = f4_get(xv[g], s4);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4_get(a0[g], s4), xs, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4_get(a1[g], s4), xs, acc[1], 0, 0, 0);
      }
  }

  if (wave > 0) {
    red[wave - 1][0][lane] = acc[0];
    red[wave - 1][1][lane] = acc[1];
  }
  __syncthreads();
  if (wave != 0 || !mok) return;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    f32x4 a = acc[f] + red[0][f][lane] + red[1][f][lane] + red[2][f][lane];
    const int cb = n0 + f * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bb = *(const float4*)(p.bias + cb);
    *(float4*)((float*)p.y + (size_t)m * p.ys + cb) =
        make_float4(apply_act(a[0] + bb.x, p.act), apply_act(a[1] + bb.y, p.act), apply_act(a[2] + bb.z, p.act),
                    apply_act(a[3] + bb.w, p.act));
  }
}

// fp32 FC (impl kF32Fc, and the fp32 default for this shape): 1x1 conv over a 1x1 map, Kpad == 1280.
bool conv_fc_f32(const ConvParams& p, hipStream_t s) {
  if (p.KH != 1 || p.KW != 1 || p.H != 1 || p.W != 1 || p.Ho != 1 || p.Wo != 1 || p.stride != 1 ||
      p.res != nullptr || p.y2 != nullptr || p.Kpad != 1280 || p.Cin > p.Kpad || p.xs % 4 != 0 || p.ys % 4 != 0 ||
      p.Cout % 4 != 0)
    return false;
  const long grid = (long)((p.B + 15) / 16) * ((p.Cout + 31) / 32);
  if (grid <= 0) return true;
  hipLaunchKernelGGL(fc_splitk_f32_kernel<20>, dim3((unsigned)grid), dim3(256), 0, s, p);
  return true;
}

}  // namespace arena
