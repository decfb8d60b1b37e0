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
#include <cstdlib>

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

// ---------------------------------------------------------------------------
// v2 (default): weight-stationary LDS kernel.
//
// Profile of the direct kernel (v1) on the YOLO 3x3 layers: every wave
// re-streams the whole [Cout][K] weight matrix from L2 (a 64x576 tile is
// 74 KB, larger than the 32 KB vector L1), so the kernel runs at the L2
// bandwidth, ~4x below the MFMA rate.  A fully LDS-staged im2col GEMM (both
// operands, one barrier per 32/64-deep K tile) was measured 1.5-4x *slower*:
// at 3 blocks/CU the per-tile global-load latency is exposed.  This variant
// keeps v1's high-occupancy, barrier-free activation stream (each lane loads
// its im2col fragment straight from NHWC global memory, with the next K-step
// prefetched into registers) and moves only the weights into LDS: the block
// copies a [BN][KC] weight chunk once (one barrier pair per chunk, usually a
// single chunk) and all four waves read their A fragments with ds_read_b128.
// Weight rows are XOR-swizzled per 16-byte chunk (row & 7).
template <int MF, int NF>
__global__ __launch_bounds__(256) void conv_wlds_kernel(const ConvParams p, const int kc) {
  extern __shared__ __attribute__((aligned(16))) uint4 wl[];  // [NF*16][kc/8] chunks
  constexpr int BN = NF * 16;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int col = lane & 15;
  const int kq = lane >> 4;

  const int B = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = B * HWo;
  const int nx = gridDim.x;
  int bx = blockIdx.x;
  {  // bijective XCD-aware remap: neighbouring pixel tiles share an L2
    const int q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
    bx = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int blk_pix = bx * (4 * MF * 16);
  if (blk_pix >= M) return;
  const int pix0 = blk_pix + wave * (MF * 16);
  const int cout0 = blockIdx.y * BN;

  const bf16* __restrict__ x = (const bf16*)p.x;
  const bf16* __restrict__ w = (const bf16*)p.w;
  const int H = p.H, W = p.W, xs = p.xs, Cin = p.Cin, KW = p.KW;
  const int taps = p.KH * p.KW;

  int pbase[MF], iy0[MF], ix0[MF];
  bool pv[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int pix = pix0 + f * 16 + col;
    pv[f] = pix < M;
    const int pp = pv[f] ? pix : 0;
    const int b = pp / HWo;
    const int r = pp - b * HWo;
    const int oy = r / p.Wo;
    const int ox = r - oy * p.Wo;
    pbase[f] = b * H * W;
    iy0[f] = oy * p.stride - p.pad_t;
    ix0[f] = ox * p.stride - p.pad_l;
  }

  f32x4 acc[NF][MF];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int f = 0; f < MF; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  int ci = (kq * 8) % Cin;
  int tap = (kq * 8) / Cin;
  int kh = tap / KW, kw = tap - (tap / KW) * KW;
  const uint4 zero = {0u, 0u, 0u, 0u};

  auto load_b = [&](uint4* bv) {
    const bool tv = tap < taps;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int iy = iy0[f] + kh, ix = ix0[f] + kw;
      const bool ok = pv[f] && tv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      bv[f] = ok ? *(const uint4*)(x + (size_t)(pbase[f] + iy * W + ix) * xs + ci) : zero;
    }
    ci += 32;
    while (ci >= Cin) {
      ci -= Cin;
      ++tap;
      if (++kw == KW) { kw = 0; ++kh; }
    }
  };

  // 16-byte chunks per weight row in LDS, padded to a multiple of 8 so the
  // (row & 7) XOR swizzle never leaves its row
  const int nch = ((kc >> 3) + 7) & ~7;
  uint4 bcur[MF], bnext[MF];
  load_b(bcur);
  for (int k0 = 0; k0 < p.Kpad; k0 += kc) {
    const int klen = min(kc, p.Kpad - k0);
    const int lch = klen >> 3;
    if (k0 > 0) __syncthreads();  // previous chunk fully consumed
    for (int q = tid; q < BN * lch; q += 256) {
      const int n = q / lch, c = q - n * lch;
      int row = cout0 + n;
      row = row < p.Cout_pad ? row : p.Cout_pad - 1;
      wl[n * nch + (c ^ (n & 7))] = *(const uint4*)(w + (size_t)row * p.Kpad + k0 + c * 8);
    }
    __syncthreads();
    const int nks = klen >> 5;
    for (int ks = 0; ks < nks; ++ks) {
      const bool more = (k0 + (ks + 1) * 32) < p.Kpad;
      if (more) load_b(bnext);
      const int ch = ks * 4 + kq;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int n = j * 16 + col;
        const bf16x8 a = __builtin_bit_cast(bf16x8, wl[n * nch + (ch ^ (n & 7))]);
#pragma unroll
        for (int f = 0; f < MF; ++f)
          acc[j][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bcur[f]), acc[j][f],
                                                            0, 0, 0);
      }
      if (more) {
#pragma unroll
        for (int f = 0; f < MF; ++f) bcur[f] = bnext[f];
      }
    }
  }

#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = cout0 + j * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      if (!pv[f]) continue;
      const int pix = pix0 + f * 16 + col;
      float v[4] = {acc[j][f][0] + bias.x, acc[j][f][1] + bias.y, acc[j][f][2] + bias.z, acc[j][f][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        float rv[4];
        unpack4(*(const uint2*)((const bf16*)p.res + (size_t)pix * p.rs + cb), rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      if (p.f32out) {
        *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const uint2 pk = pack4(v);
        *(uint2*)((bf16*)p.y + (size_t)pix * p.ys + cb) = pk;
        if (p.y2 != nullptr) {
          const int b = pix / HWo;
          const int rr = pix - b * HWo;
          const int oy = rr / p.Wo, ox = rr - (rr / p.Wo) * p.Wo;
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

constexpr int kWldsBytes = 64 * 1024;  // weight chunk budget per block (2+ blocks/CU)

template <int MF, int NF>
static void launch_wlds(const ConvParams& p, hipStream_t s, int M) {
  constexpr int BN = NF * 16;
  int kc = (kWldsBytes / (BN * 2)) / 64 * 64;
  if (kc > p.Kpad) kc = p.Kpad;
  const size_t lds = (size_t)BN * (((kc >> 3) + 7) & ~7) * 16;
  dim3 grid((M + 4 * MF * 16 - 1) / (4 * MF * 16), (p.Cout_pad + BN - 1) / BN);
  hipLaunchKernelGGL((conv_wlds_kernel<MF, NF>), grid, dim3(256), lds, s, p, kc);
}

template <int NF>
static void launch_wlds_nf(const ConvParams& p, hipStream_t s, int M) {
  const int ny = (p.Cout_pad + NF * 16 - 1) / (NF * 16);
  const long b4 = (long)((M + 255) / 256) * ny, b2 = (long)((M + 127) / 128) * ny;
  if (b4 >= 1024)
    launch_wlds<4, NF>(p, s, M);
  else if (b2 >= 512)
    launch_wlds<2, NF>(p, s, M);
  else
    launch_wlds<1, NF>(p, s, M);
}

static void launch_wlds_any(const ConvParams& p, hipStream_t s, int M) {
  const int ncf = p.Cout_pad / 16;
  if (ncf % 4 == 0)
    launch_wlds_nf<4>(p, s, M);
  else if (ncf % 5 == 0)
    launch_wlds_nf<5>(p, s, M);
  else if (ncf % 3 == 0)
    launch_wlds_nf<3>(p, s, M);
  else if (ncf % 2 == 0)
    launch_wlds_nf<2>(p, s, M);
  else
    launch_wlds_nf<1>(p, s, M);
}

// ---------------------------------------------------------------------------
// 3x3 spatial-tile kernel (stride 1 or 2, Cin % 32 == 0): the YOLO workhorse.
//
// The implicit-GEMM kernels above re-read every input pixel once per tap
// (9x) from L1/L2 and re-stream the weights per wave.  Here a block owns an
// output tile of (4*MF) rows x 16 columns x BN channels of one image; per
// 32-channel input slice it stages the halo'd input tile
// [(TH-1)*S+3][15*S+3][32] and that slice's weights [9][BN][32] in LDS once
// (one barrier pair per slice), then each wave runs 9 taps x MF x NF MFMAs
// reading both operands with ds_read_b128.  Per 16-byte chunk the LDS image
// is XOR-swizzled by ((pixel or row) >> 2) & 3 so the 16 lanes of a fragment
// read land on distinct bank groups.
template <int S, int MF, int NF>
__global__ __launch_bounds__(256) void conv3x3_tile_kernel(const ConvParams p) {
  constexpr int TH = 4 * MF;
  constexpr int BN = NF * 16;
  constexpr int IR = (TH - 1) * S + 3;   // staged input rows
  constexpr int IC = 15 * S + 3;         // staged input cols
  constexpr int IN_CH = IR * IC * 4;     // 16-byte chunks of the input tile
  constexpr int W_CH = 9 * BN * 4;       // 16-byte chunks of the weight slice
  __shared__ uint4 sin[IN_CH];
  __shared__ uint4 sw[W_CH];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + 15) >> 4, tiles_y = (p.Ho + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;
  const int b = blockIdx.x / per_img;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = blockIdx.x - b * per_img;
  const int ty0 = (t / tiles_x) * TH, tx0 = (t % tiles_x) * 16;
  const int cout0 = blockIdx.y * BN;
  const int iy_base = ty0 * S - p.pad_t, ix_base = tx0 * S - p.pad_l;
  const bf16* __restrict__ x = (const bf16*)p.x + (size_t)b * p.H * p.W * p.xs;
  const bf16* __restrict__ w = (const bf16*)p.w;
  const int Cin = p.Cin;

  f32x4 acc[NF][MF];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int f = 0; f < MF; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint4 zero = {0u, 0u, 0u, 0u};

  for (int c0 = 0; c0 < Cin; c0 += 32) {
    if (c0 > 0) __syncthreads();
    for (int q = tid; q < IN_CH; q += 256) {
      const int pix = q >> 2, ch = q & 3;
      const int r = pix / IC, c = pix - (pix / IC) * IC;
      const int iy = iy_base + r, ix = ix_base + c;
      uint4 v = zero;
      if ((unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)
        v = *(const uint4*)(x + ((size_t)iy * p.W + ix) * p.xs + c0 + ch * 8);
      sin[pix * 4 + (ch ^ ((pix >> 2) & 3))] = v;
    }
    for (int q = tid; q < W_CH; q += 256) {
      const int row = q >> 2, ch = q & 3;  // row = tap*BN + n
      const int tap = row / BN, n = row - (row / BN) * BN;
      int co = cout0 + n;
      co = co < p.Cout_pad ? co : p.Cout_pad - 1;
      sw[row * 4 + (ch ^ ((n >> 2) & 3))] = *(const uint4*)(w + (size_t)co * p.Kpad + tap * Cin + c0 + ch * 8);
    }
    __syncthreads();
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
        bf16x8 a[NF], bb[MF];
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int n = j * 16 + col;
          a[j] = __builtin_bit_cast(bf16x8, sw[(tap * BN + n) * 4 + (kq ^ ((n >> 2) & 3))]);
        }
#pragma unroll
        for (int f = 0; f < MF; ++f) {
          const int pix = ((wave * MF + f) * S + kh) * IC + col * S + kw;
          bb[f] = __builtin_bit_cast(bf16x8, sin[pix * 4 + (kq ^ ((pix >> 2) & 3))]);
        }
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < MF; ++f)
            acc[j][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bb[f], acc[j][f], 0, 0, 0);
      }
    }
  }

  const int ox = tx0 + col;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = cout0 + j * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int oy = ty0 + wave * MF + f;
      if (oy >= p.Ho || ox >= p.Wo) continue;
      const size_t pix = ((size_t)b * p.Ho + oy) * p.Wo + ox;
      float v[4] = {acc[j][f][0] + bias.x, acc[j][f][1] + bias.y, acc[j][f][2] + bias.z, acc[j][f][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        float rv[4];
        unpack4(*(const uint2*)((const bf16*)p.res + pix * p.rs + cb), rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      const uint2 pk = pack4(v);
      *(uint2*)((bf16*)p.y + pix * p.ys + cb) = pk;
      if (p.y2 != nullptr) {
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

template <int S, int MF, int NF>
static void launch_tile(const ConvParams& p, hipStream_t s) {
  constexpr int TH = 4 * MF;
  const int tiles = ((p.Wo + 15) / 16) * ((p.Ho + TH - 1) / TH);
  dim3 grid(p.B * tiles, (p.Cout_pad + NF * 16 - 1) / (NF * 16));
  hipLaunchKernelGGL((conv3x3_tile_kernel<S, MF, NF>), grid, dim3(256), 0, s, p);
}

template <int S, int NF>
static void launch_tile_nf(const ConvParams& p, hipStream_t s) {
  // MF=2 (8-row tiles) when the map is tall enough and there are enough blocks
  const long blocks2 = (long)p.B * ((p.Wo + 15) / 16) * ((p.Ho + 7) / 8) * ((p.Cout_pad + NF * 16 - 1) / (NF * 16));
  if (S == 1 && p.Ho >= 16 && blocks2 >= 512)
    launch_tile<S, 2, NF>(p, s);
  else
    launch_tile<S, 1, NF>(p, s);
}

template <int S>
static void launch_tile_s(const ConvParams& p, hipStream_t s) {
  const int ncf = p.Cout_pad / 16;
  if (ncf % 4 == 0)
    launch_tile_nf<S, 4>(p, s);
  else if (ncf % 3 == 0)
    launch_tile_nf<S, 3>(p, s);
  else if (ncf % 5 == 0)
    launch_tile_nf<S, 5>(p, s);
  else if (ncf % 2 == 0)
    launch_tile_nf<S, 2>(p, s);
  else
    launch_tile_nf<S, 1>(p, s);
}

static bool tile_ok(const ConvParams& p) {
  return p.KH == 3 && p.KW == 3 && (p.stride == 1 || p.stride == 2) && p.Cin % 32 == 0 && !p.f32out &&
         p.Kpad >= 9 * p.Cin;
}

static int g_conv_impl = [] {
  const char* e = std::getenv("ARENA_CONV_IMPL");
  return e ? std::atoi(e) : 2;
}();
static int conv_impl() { return g_conv_impl; }
static bool g_conv_pw = [] {
  const char* e = std::getenv("ARENA_CONV_PW");
  return e ? std::atoi(e) != 0 : true;
}();
static bool conv_pw_enabled() { return g_conv_pw; }
static bool g_conv_v3 = [] {
  const char* e = std::getenv("ARENA_CONV_V3");
  return e ? std::atoi(e) != 0 : true;
}();
void set_conv_v3(bool v) { g_conv_v3 = v; }
void set_conv_pw(bool v) { g_conv_pw = v; }

void set_conv_impl(int v) {
  if (v < 1 || v > 3) throw std::runtime_error("conv impl must be 1 (direct), 2 (LDS tiles) or 3 (igemm)");
  g_conv_impl = v;
}
int get_conv_impl() { return g_conv_impl; }

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

static void launch_v1(const ConvParams& p, hipStream_t s, int M);

void conv2d(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 8 != 0 || p.xs % 8 != 0 || p.Kpad % 32 != 0 || p.Cout_pad % 16 != 0 ||
      p.Cout % 4 != 0 || p.Cout > p.Cout_pad)
    throw std::runtime_error("conv2d: unsupported geometry (Cin/xs %8, Kpad %32, Cout_pad %16, Cout %4)");
  if (p.Kpad < p.KH * p.KW * p.Cin) throw std::runtime_error("conv2d: Kpad < KH*KW*Cin");
  if (p.y2 != nullptr && p.f32out) throw std::runtime_error("conv2d: upsampled copy needs bf16 output");
  const long M = (long)p.B * p.Ho * p.Wo;
  if (M <= 0) return;
  if (M > 0x7fffffffL) throw std::runtime_error("conv2d: M overflows int");
  if (p.pw_w != nullptr) {  // fused pointwise epilogue: only the v3 halo-tile kernel implements it
    if (!conv3x3_v3(p, s)) throw std::runtime_error("conv2d: fused pointwise epilogue needs a v3-eligible 3x3 conv");
    return;
  }
  if (conv_fc(p, s)) return;  // classifier FC: split-K GEMM, whatever the family
  const int impl = p.impl ? p.impl : conv_impl();
  if (impl == 3) {
    conv_igemm(p, s);
    return;
  }
  if (impl == 2) {
    if (conv_pw_enabled() && conv_pw(p, s)) return;
    if (g_conv_v3 && conv3x3_v3(p, s)) return;
    if (tile_ok(p)) {
      if (p.stride == 1)
        launch_tile_s<1>(p, s);
      else
        launch_tile_s<2>(p, s);
    } else if (p.Kpad >= 256) {
      launch_wlds_any(p, s, (int)M);
    } else {
      launch_v1(p, s, (int)M);
    }
    return;
  }
  launch_v1(p, s, (int)M);
}

static void launch_v1(const ConvParams& p, hipStream_t s, int M) {
  const int ncf = p.Cout_pad / 16;
  if (ncf % 4 == 0)
    launch_wc<4>(p, s, M);
  else if (ncf % 5 == 0)
    launch_wc<5>(p, s, M);
  else if (ncf % 3 == 0)
    launch_wc<3>(p, s, M);
  else if (ncf % 2 == 0)
    launch_wc<2>(p, s, M);
  else
    launch_wc<1>(p, s, M);
}

}  // namespace arena
