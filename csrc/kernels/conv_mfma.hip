// Implicit-GEMM NHWC convolution on CDNA4 matrix cores.
//
// Replaces the ONNX Runtime CPU Conv(+BN folded)+Sigmoid*Mul (SiLU) / Clip
// (ReLU6) / Add / Concat / Resize nodes that the reference executes for
// YOLOv5nu and MobileNetV2 (reference: src/shared/model/registry.py:194-224
// builds the ORT sessions; architectures/monolithic/app/inference.py:164,196
// runs them).  One kernel family covers every dense conv of both networks
// (stem, 3x3 s1/s2, 1x1 pointwise expand/project, detect-head 1x1, the FC
// layer as a 1x1 conv on a 1x1 map).
//
// GEMM mapping (v_mfma_f32_16x16x32_bf16, wave64):
//   A = weights  [Cout][K]  row = output channel   (lane&15), k = 8*(lane>>4)+j
//   B = im2col   [K][M]     col = output pixel     (lane&15), same k mapping
//   D = [Cout][M]: lane holds 4 consecutive output channels of one pixel, so
//       the epilogue writes 8 contiguous bytes of an NHWC row per lane.
// K is ordered (kh, kw, ci) so a lane's 8 k-values are 8 consecutive input
// channels of one tap: one 16-byte load straight from the NHWC activation.
// Both operands are loaded global->VGPR (weights are tiny and L2 resident,
// activations are re-read by the taps of neighbouring pixels through L1/L2).
//
// Block = 256 threads (4 waves).  Wave tile = WC x 16 output channels by
// WP x 16 pixels; the four waves of a block share the channel tile and cover
// 4*WP*16 consecutive pixels, so weight fragments are L1 hits for 3 of 4 waves.
#include "common.h"
#include "launch.h"

namespace arena {

template <int WC, int WP, bool F32OUT>
__global__ __launch_bounds__(256) void conv_mfma_kernel(const ConvParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int kq = lane >> 4;

  const int B = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = B * HWo;
  const int blk_pix = blockIdx.x * (4 * WP * 16);
  if (blk_pix >= M) return;
  const int pix0 = blk_pix + wave * (WP * 16);
  const int cout0 = blockIdx.y * (WC * 16);

  const bf16* __restrict__ x = (const bf16*)p.x;
  const int H = p.H, W = p.W, xs = p.xs, Cin = p.Cin, KW = p.KW;
  const int taps = p.KH * p.KW;

  int pbase[WP], iy0[WP], ix0[WP];
  bool pv[WP];
#pragma unroll
  for (int q = 0; q < WP; ++q) {
    const int pix = pix0 + q * 16 + col;
    pv[q] = pix < M;
    const int pp = pv[q] ? pix : 0;
    const int b = pp / HWo;
    const int r = pp - b * HWo;
    const int oy = r / p.Wo;
    const int ox = r - oy * p.Wo;
    pbase[q] = b * H * W;
    iy0[q] = oy * p.stride - p.pad_t;
    ix0[q] = ox * p.stride - p.pad_l;
  }

  const bf16* wrow[WC];
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    int row = cout0 + c * 16 + col;
    row = row < p.Cout_pad ? row : p.Cout_pad - 1;
    wrow[c] = (const bf16*)p.w + (size_t)row * p.Kpad + kq * 8;
  }

  f32x4 acc[WC][WP];
#pragma unroll
  for (int c = 0; c < WC; ++c)
#pragma unroll
    for (int q = 0; q < WP; ++q) acc[c][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // (tap, ci) of this lane's first k-group, then advanced by 32 per k-step.
  int ci = (kq * 8) % Cin;
  int tap = (kq * 8) / Cin;
  int kh = tap / KW, kw = tap - (tap / KW) * KW;

  const int nks = p.Kpad >> 5;
  const uint4 zero = {0u, 0u, 0u, 0u};
  for (int ks = 0; ks < nks; ++ks) {
    uint4 a[WC];
#pragma unroll
    for (int c = 0; c < WC; ++c) a[c] = *(const uint4*)(wrow[c] + ks * 32);
    uint4 bv[WP];
    const bool tv = tap < taps;
#pragma unroll
    for (int q = 0; q < WP; ++q) {
      const int iy = iy0[q] + kh;
      const int ix = ix0[q] + kw;
      const bool ok = pv[q] && tv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const size_t off = (size_t)(pbase[q] + iy * W + ix) * xs + ci;
      bv[q] = ok ? *(const uint4*)(x + off) : zero;
    }
#pragma unroll
    for (int c = 0; c < WC; ++c) {
      const bf16x8 av = __builtin_bit_cast(bf16x8, a[c]);
#pragma unroll
      for (int q = 0; q < WP; ++q)
        acc[c][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, bv[q]),
                                                          acc[c][q], 0, 0, 0);
    }
    ci += 32;
    while (ci >= Cin) {
      ci -= Cin;
      ++tap;
      if (++kw == KW) { kw = 0; ++kh; }
    }
  }

  // Epilogue: bias -> activation -> residual -> store (+ upsampled copy).
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    const int cb = cout0 + c * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int q = 0; q < WP; ++q) {
      if (!pv[q]) continue;
      const int pix = pix0 + q * 16 + col;
      float v[4] = {acc[c][q][0] + bias.x, acc[c][q][1] + bias.y, acc[c][q][2] + bias.z,
                    acc[c][q][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        float rv[4];
        unpack4(*(const uint2*)((const bf16*)p.res + (size_t)pix * p.rs + cb), rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      if constexpr (F32OUT) {
        *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const uint2 pk = pack4(v);
        *(uint2*)((bf16*)p.y + (size_t)pix * p.ys + cb) = pk;
        if (p.y2 != nullptr) {
          const int b = pix / HWo;
          const int r = pix - b * HWo;
          const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
          const int W2 = 2 * p.Wo;
          bf16* y2 = (bf16*)p.y2;
          const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
          *(uint2*)(y2 + base * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + 1) * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + W2) * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + W2 + 1) * p.y2s + cb) = pk;
        }
      }
    }
  }
}

template <int WC, int WP>
static void launch_wc_wp(const ConvParams& p, hipStream_t s, int M) {
  dim3 grid((M + 4 * WP * 16 - 1) / (4 * WP * 16), (p.Cout_pad + WC * 16 - 1) / (WC * 16));
  if (p.f32out)
    hipLaunchKernelGGL((conv_mfma_kernel<WC, WP, true>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<WC, WP, false>), grid, dim3(256), 0, s, p);
}

template <int WC>
static void launch_wc(const ConvParams& p, hipStream_t s, int M) {
  const int ny = (p.Cout_pad + WC * 16 - 1) / (WC * 16);
  // Prefer the widest pixel tile that still gives >= 2 blocks per CU.
  const long blocks4 = (long)((M + 255) / 256) * ny;
  const long blocks2 = (long)((M + 127) / 128) * ny;
  if (blocks4 >= 512)
    launch_wc_wp<WC, 4>(p, s, M);
  else if (blocks2 >= 512)
    launch_wc_wp<WC, 2>(p, s, M);
  else
    launch_wc_wp<WC, 1>(p, s, M);
}

void conv2d(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 8 != 0 || p.xs % 8 != 0 || p.Kpad % 32 != 0 || p.Cout_pad % 16 != 0 ||
      p.Cout % 4 != 0 || p.Cout > p.Cout_pad)
    throw std::runtime_error("conv2d: unsupported geometry (Cin/xs %8, Kpad %32, Cout_pad %16, Cout %4)");
  if (p.Kpad < p.KH * p.KW * p.Cin) throw std::runtime_error("conv2d: Kpad < KH*KW*Cin");
  if (p.y2 != nullptr && p.f32out) throw std::runtime_error("conv2d: upsampled copy needs bf16 output");
  const long M = (long)p.B * p.Ho * p.Wo;
  if (M <= 0) return;
  if (M > 0x7fffffffL) throw std::runtime_error("conv2d: M overflows int");
  const int ncf = p.Cout_pad / 16;
  if (ncf % 4 == 0)
    launch_wc<4>(p, s, (int)M);
  else if (ncf % 5 == 0)
    launch_wc<5>(p, s, (int)M);
  else if (ncf % 3 == 0)
    launch_wc<3>(p, s, (int)M);
  else if (ncf % 2 == 0)
    launch_wc<2>(p, s, (int)M);
  else
    launch_wc<1>(p, s, (int)M);
}

}  // namespace arena
