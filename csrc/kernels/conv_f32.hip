// Exact-fp32 pipeline kernels: implicit-GEMM convolution on the fp32-input
// matrix cores, depthwise 3x3 and SPPF pooling over fp32 NHWC activations.
//
// The reference executes both networks as fp32 ONNX graphs on ONNX Runtime's
// CPU EP (reference: experiment.yaml:202,207,220,225 declare float32 I/O;
// src/shared/model/registry.py:220-224 creates the sessions).  This file is
// the MI355X counterpart at the same precision: every product is an fp32
// product with fp32 accumulation (v_mfma_f32_16x16x4_f32: one rounding per
// product, a k-ordered fma chain — bit-for-bit an fp32 dot product in a
// different summation order), activations are stored as fp32.
//
// GEMM mapping (v_mfma_f32_16x16x4_f32, wave64): lane l supplies
//   A[i = l&15][k = l>>4]  (weights: row = output channel)
//   B[k = l>>4][j = l&15]  (im2col: column = output pixel)
// and receives D[row = 4*(l>>4) + r][col = l&15], r = 0..3.  A K-chunk of 16
// is four MFMAs: in step s lane l supplies k = 16*chunk + 4*(l>>4) + s, so a
// lane's four k-values of a chunk are four consecutive input channels of one
// tap (K is ordered (kh, kw, ci)) — one 16-byte float4 load from NHWC memory,
// and the weight fragment is one float4 of the weight row.  The accumulator
// holds 4 consecutive output channels of one pixel: one float4 NHWC store.
//
// fp32 MFMA issues at 1/16 of the bf16 rate (32 cycles per 16x16x4 per SIMD),
// so these kernels are matrix-core bound at realistic occupancy: each wave
// keeps WC x WP independent 16x16 accumulators (>= 2 hide the 40-cycle
// dependent latency) and prefetches the next K-chunk's operands into
// registers while the current chunk's MFMAs run.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"
#include "letterbox.h"

namespace arena {

__device__ __forceinline__ float4 load_f4_or_zero(const float* p, const float* safe, bool ok) {
  const float4 v = *(const float4*)(ok ? p : safe);
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float f4_get(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

// Bijective XCD-aware block remap (8 XCDs, round-robin dispatch): consecutive
// logical tiles land on the same XCD so neighbouring pixel tiles share its L2.
__device__ __forceinline__ int xcd_remap(int bx, int nx) {
  const int q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
}

template <int WC, int WP>
__global__ __launch_bounds__(256) void conv_f32_kernel(const ConvParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int kq = lane >> 4;

  const int B = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = B * HWo;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int blk_pix = bx * (4 * WP * 16);
  if (blk_pix >= M) return;
  const int pix0 = blk_pix + wave * (WP * 16);
  const int cout0 = blockIdx.y * (WC * 16);

  const float* __restrict__ x = (const float*)p.x;
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

  const float* wrow[WC];
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    int row = cout0 + c * 16 + col;
    row = row < p.Cout_pad ? row : p.Cout_pad - 1;
    wrow[c] = (const float*)p.w + (size_t)row * p.Kpad + kq * 4;
  }

  f32x4 acc[WC][WP];
#pragma unroll
  for (int c = 0; c < WC; ++c)
#pragma unroll
    for (int q = 0; q < WP; ++q) acc[c][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // (tap, ci) of this lane's k-group in the current chunk
  int ci = (kq * 4) % Cin;
  int tap = (kq * 4) / Cin;
  int kh = tap / KW, kw = tap - (tap / KW) * KW;

  float4 a[WC], bv[WP];
  auto load_chunk = [&](int ks, float4* av, float4* bq) {
#pragma unroll
    for (int c = 0; c < WC; ++c) av[c] = *(const float4*)(wrow[c] + ks * 16);
    const bool tv = tap < taps;
#pragma unroll
    for (int q = 0; q < WP; ++q) {
      const int iy = iy0[q] + kh;
      const int ix = ix0[q] + kw;
      const bool ok = pv[q] && tv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      bq[q] = load_f4_or_zero(x + (size_t)(pbase[q] + iy * W + ix) * xs + ci, x, ok);
    }
    ci += 16;
    while (ci >= Cin) {
      ci -= Cin;
      ++tap;
      if (++kw == KW) { kw = 0; ++kh; }
    }
  };

  const int nks = p.Kpad >> 4;
  load_chunk(0, a, bv);
  for (int ks = 0; ks < nks; ++ks) {
    float4 an[WC], bn[WP];
    if (ks + 1 < nks) load_chunk(ks + 1, an, bn);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int c = 0; c < WC; ++c) {
        const float av = f4_get(a[c], s);
#pragma unroll
        for (int q = 0; q < WP; ++q)
          acc[c][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, f4_get(bv[q], s), acc[c][q], 0, 0, 0);
      }
    }
    if (ks + 1 < nks) {
#pragma unroll
      for (int c = 0; c < WC; ++c) a[c] = an[c];
#pragma unroll
      for (int q = 0; q < WP; ++q) bv[q] = bn[q];
    }
  }

  // Epilogue: bias -> activation -> residual -> store (+ 2x nearest-upsampled copy).
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    const int cb = cout0 + c * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int q = 0; q < WP; ++q) {
      if (!pv[q]) continue;
      const int pix = pix0 + q * 16 + col;
      float v[4] = {acc[c][q][0] + bias.x, acc[c][q][1] + bias.y, acc[c][q][2] + bias.z, acc[c][q][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + (size_t)pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int b = pix / HWo;
        const int r = pix - b * HWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int WC, int WP>
static void launch_f32(const ConvParams& p, hipStream_t s, long M) {
  dim3 grid((unsigned)((M + 4 * WP * 16 - 1) / (4 * WP * 16)), (unsigned)((p.Cout_pad + WC * 16 - 1) / (WC * 16)));
  hipLaunchKernelGGL((conv_f32_kernel<WC, WP>), grid, dim3(256), 0, s, p);
}

template <int WC>
static void launch_f32_wc(const ConvParams& p, hipStream_t s, long M) {
  const long ny = (p.Cout_pad + WC * 16 - 1) / (WC * 16);
  // widest pixel tile that still gives >= 2 workgroups per CU (256 CUs)
  if (((M + 255) / 256) * ny >= 512)
    launch_f32<WC, 4>(p, s, M);
  else if (((M + 127) / 128) * ny >= 512)
    launch_f32<WC, 2>(p, s, M);
  else
    launch_f32<WC, 1>(p, s, M);
}

// ---------------------------------------------------------------------------
// LDS-tiled implicit GEMM (default).  The direct kernel above re-reads each
// wave's weight rows and im2col fragments from L1/L2 for every K-chunk; here a
// workgroup stages a [BM pixels x 32 k] activation tile and a [BN channels x
// 32 k] weight tile in LDS once per K-chunk (double-buffered: the next chunk's
// global loads are in flight while the current chunk's MFMAs run, one barrier
// per chunk) and its four waves (WM x WN layout) read their fragments with
// ds_read_b128.  The staging assignment gives each thread a fixed k-group (4
// consecutive k = 4 input channels of one tap) and BM/32 fixed pixels, so the
// im2col address math is one (tap, ci) split per chunk plus a bounds test per
// pixel.  LDS rows are padded to KC + 8 floats (see the pitch note below).

template <int MF, int NF, int WM, int WN, int KC = 32>
__global__ __launch_bounds__(256) void conv_f32_lds_kernel(const ConvParams p) {
  constexpr int BM = WM * MF * 16, BN = WN * NF * 16;
  // k per LDS chunk; floats per LDS row: KC + 8 makes the row pitch 2 (mod 4) 16-byte slots, which puts the
  // 16 rows x 4 k-groups of every ds_read_b128 lane group on 16 distinct slots of the 256-B bank row
  // (KC + 4, an odd slot count, is 2-way: 31-36 % SQ_LDS_BANK_CONFLICT in profiles/r2_fp32_pmc_ops.md)
  constexpr int F32_KC = KC, F32_PITCH = KC + 8;
  constexpr int GROUPS = KC / 4;                    // float4 k-groups per row
  constexpr int RPP = 256 / GROUPS;                 // rows staged per pass of the workgroup
  constexpr int PPT = BM / RPP;                     // staged pixels per thread
  constexpr int WPT = (BN * GROUPS + 255) / 256;    // staged weight float4 per thread
  static_assert(BM % RPP == 0, "pixel tile must be a multiple of the staging pass");
  __shared__ __attribute__((aligned(16))) float sB[2][BM * F32_PITCH];
  __shared__ __attribute__((aligned(16))) float sA[2][BN * F32_PITCH];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;

  const int Bl = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = Bl * HWo;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = bx * BM;
  if (m0 >= M) return;
  const int n0 = blockIdx.y * BN;

  const float* __restrict__ x = (const float*)p.x;
  const float* __restrict__ w = (const float*)p.w;
  const int H = p.H, W = p.W, xs = p.xs, Cin = p.Cin, KW = p.KW, Kpad = p.Kpad;
  const int taps = p.KH * p.KW;

  // staging roles: k-group g (4 consecutive k), pixels tid/GROUPS + RPP*j
  const int g = tid % GROUPS;
  int pb[PPT], py[PPT], px[PPT];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int m = m0 + tid / GROUPS + RPP * j;
    if (m < M) {
      const int b = m / HWo, r = m - b * HWo;
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      pb[j] = b * H * W;
      py[j] = oy * p.stride - p.pad_t;
      px[j] = ox * p.stride - p.pad_l;
    } else {
      pb[j] = 0;
      py[j] = -(1 << 20);  // fails the bounds test: zero fill
      px[j] = 0;
    }
  }
  float4 rb[PPT], ra[WPT];
  auto gload = [&](int kc) {
    const int k = kc * F32_KC + 4 * g;
    const int tap = k / Cin, ci = k - tap * Cin;
    const int kh = tap / KW, kw = tap - kh * KW;
    const bool tv = tap < taps;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int iy = py[j] + kh, ix = px[j] + kw;
      const bool ok = tv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      rb[j] = load_f4_or_zero(x + (size_t)(pb[j] + iy * W + ix) * xs + ci, x, ok);
    }
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = tid + 256 * j;  // (row, group) of the weight tile
      const int row = e / GROUPS, gg = e % GROUPS;
      const int kk = kc * F32_KC + 4 * gg;
      const bool ok = e < BN * GROUPS && n0 + row < p.Cout_pad && kk < Kpad;
      ra[j] = load_f4_or_zero(w + (size_t)(n0 + row) * Kpad + kk, w, ok);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PPT; ++j)
      *(float4*)&sB[buf][(tid / GROUPS + RPP * j) * F32_PITCH + 4 * g] = rb[j];
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = tid + 256 * j;
      if (e < BN * GROUPS) *(float4*)&sA[buf][(e / GROUPS) * F32_PITCH + 4 * (e % GROUPS)] = ra[j];
    }
  };

  f32x4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (Kpad + F32_KC - 1) / F32_KC;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) gload(kc + 1);
#pragma unroll
    for (int u = 0; u < F32_KC / 16; ++u) {
      float4 af[NF], bf[MF];
#pragma unroll
      for (int j = 0; j < NF; ++j)
        af[j] = *(const float4*)&sA[cur][((wn * NF + j) * 16 + col) * F32_PITCH + 16 * u + 4 * kq];
#pragma unroll
      for (int f = 0; f < MF; ++f)
        bf[f] = *(const float4*)&sB[cur][((wm * MF + f) * 16 + col) * F32_PITCH + 16 * u + 4 * kq];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < MF; ++f)
            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4_get(af[j], t), f4_get(bf[f], t), acc[f][j], 0, 0, 0);
    }
    if (kc + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // Epilogue: lane holds 4 consecutive output channels (rows 4*kq..+3 of the 16x16 tile) of pixel col.
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + (wn * NF + j) * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int pix = m0 + (wm * MF + f) * 16 + col;
      if (pix >= M) continue;
      float v[4] = {acc[f][j][0] + bias.x, acc[f][j][1] + bias.y, acc[f][j][2] + bias.z, acc[f][j][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + (size_t)pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int b = pix / HWo;
        const int r = pix - b * HWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int MF, int NF, int WM, int WN, int KC = 32>
static void launch_lds(const ConvParams& p, hipStream_t s, long M) {
  constexpr int BM = WM * MF * 16, BN = WN * NF * 16;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((p.Cout_pad + BN - 1) / BN));
  hipLaunchKernelGGL((conv_f32_lds_kernel<MF, NF, WM, WN, KC>), grid, dim3(256), 0, s, p);
}

// ---------------------------------------------------------------------------
// fp32-accurate implicit GEMM on the bf16 matrix cores ("x3": triple-bf16
// split).  fp32 MFMA issues at 1/16 of the bf16 rate, so the fp32 kernels above
// are matrix-core bound.  Every fp32 operand is split exactly into three bf16
// terms, v = h + m + l (h = rn_bf16(v), m = rn_bf16(v - h), l = rn_bf16(v - h
// - m); each residual is exact in fp32 and 3 x 8 significant bits cover fp32's
// 24), and the product is formed from the six partial products whose order is
// <= 2^-16 of |a||b|:
//   a*b ~= ah*bh + ah*bm + am*bh + ah*bl + al*bh + am*bm
// The dropped terms (am*bl, al*bm, al*bl) are below 2^-24 |a||b| — the size of
// fp32's own product rounding — and bf16 products are exact in the fp32
// accumulator, so the result has fp32-level error (tests/test_fp32_gpu.py
// compares it to fp64 next to the exact-fp32 kernel).  Six 16x16x32 bf16 MFMAs
// (16 cycles each) replace eight 16x16x4 fp32 MFMAs (32 cycles each) per 32-deep
// k chunk: 2.7x less matrix-core time.
//
// Staging is the fp32 LDS kernel's (float4 of 4 consecutive k per thread, same
// fp32 weight blob), split on the way into LDS: a row holds the chunk's 32 k as
// three bf16 planes [h | m | l] (96 bf16 + 16 pad = 224 B = 14 x 16-B slots:
// a pitch of 2 (mod 4) slots keeps each ds_read_b128 lane group on 16
// distinct slots).  Lane l reads its bf16x8 fragment (k = 8*(l>>4)..+7 of row l&15) of
// each plane with one ds_read_b128.
constexpr int X3_KC = 32;
constexpr int X3_PITCH = 3 * X3_KC + 16;  // bf16 per LDS row: 14 slots = 2 (mod 4), conflict-free b128 reads

__device__ __forceinline__ void split3(float v, bf16& h, bf16& m, bf16& l) {
  h = (bf16)v;
  const float r = v - (float)h;
  m = (bf16)r;
  l = (bf16)(r - (float)m);
}

__device__ __forceinline__ void store_split4(bf16* row, int k, const float4& v) {
  bf16x4 h, m, l;
  bf16 th, tm, tl;
  split3(v.x, th, tm, tl); h[0] = th; m[0] = tm; l[0] = tl;
  split3(v.y, th, tm, tl); h[1] = th; m[1] = tm; l[1] = tl;
  split3(v.z, th, tm, tl); h[2] = th; m[2] = tm; l[2] = tl;
  split3(v.w, th, tm, tl); h[3] = th; m[3] = tm; l[3] = tl;
  *(bf16x4*)(row + k) = h;
  *(bf16x4*)(row + X3_KC + k) = m;
  *(bf16x4*)(row + 2 * X3_KC + k) = l;
}

template <int MF, int NF, int WM, int WN>
__global__ __launch_bounds__(256) void conv_x3_lds_kernel(const ConvParams p) {
  constexpr int BM = WM * MF * 16, BN = WN * NF * 16;
  constexpr int GROUPS = X3_KC / 4;              // float4 k-groups per row
  constexpr int RPP = 256 / GROUPS;              // rows staged per pass of the workgroup
  constexpr int PPT = BM / RPP;                  // staged pixels per thread
  constexpr int WPT = (BN * GROUPS + 255) / 256; // staged weight float4 per thread
  static_assert(BM % RPP == 0, "pixel tile must be a multiple of the staging pass");
  __shared__ __attribute__((aligned(16))) bf16 sB[2][BM * X3_PITCH];
  __shared__ __attribute__((aligned(16))) bf16 sA[2][BN * X3_PITCH];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;

  const int Bl = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = Bl * HWo;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = bx * BM;
  if (m0 >= M) return;
  const int n0 = blockIdx.y * BN;

  const float* __restrict__ x = (const float*)p.x;
  const float* __restrict__ w = (const float*)p.w;
  const int H = p.H, W = p.W, xs = p.xs, Cin = p.Cin, KW = p.KW, Kpad = p.Kpad;
  const int taps = p.KH * p.KW;

  const int g = tid % GROUPS;
  int pb[PPT], py[PPT], px[PPT];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int m = m0 + tid / GROUPS + RPP * j;
    if (m < M) {
      const int b = m / HWo, r = m - b * HWo;
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      pb[j] = b * H * W;
      py[j] = oy * p.stride - p.pad_t;
      px[j] = ox * p.stride - p.pad_l;
    } else {
      pb[j] = 0;
      py[j] = -(1 << 20);  // fails the bounds test: zero fill
      px[j] = 0;
    }
  }
  float4 rb[PPT], ra[WPT];
  auto gload = [&](int kc) {
    const int k = kc * X3_KC + 4 * g;
    const int tap = k / Cin, ci = k - tap * Cin;
    const int kh = tap / KW, kw = tap - kh * KW;
    const bool tv = tap < taps;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int iy = py[j] + kh, ix = px[j] + kw;
      const bool ok = tv && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      rb[j] = load_f4_or_zero(x + (size_t)(pb[j] + iy * W + ix) * xs + ci, x, ok);
    }
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = tid + 256 * j;
      const int row = e / GROUPS, gg = e % GROUPS;
      const int kk = kc * X3_KC + 4 * gg;
      const bool ok = e < BN * GROUPS && n0 + row < p.Cout_pad && kk < Kpad;
      ra[j] = load_f4_or_zero(w + (size_t)(n0 + row) * Kpad + kk, w, ok);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < PPT; ++j) store_split4(&sB[buf][(tid / GROUPS + RPP * j) * X3_PITCH], 4 * g, rb[j]);
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = tid + 256 * j;
      if (e < BN * GROUPS) store_split4(&sA[buf][(e / GROUPS) * X3_PITCH], 4 * (e % GROUPS), ra[j]);
    }
  };

  f32x4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (Kpad + X3_KC - 1) / X3_KC;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) gload(kc + 1);
    bf16x8 ah[NF], am[NF], al[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const bf16* r = &sA[cur][((wn * NF + j) * 16 + col) * X3_PITCH + 8 * kq];
      ah[j] = *(const bf16x8*)r;
      am[j] = *(const bf16x8*)(r + X3_KC);
      al[j] = *(const bf16x8*)(r + 2 * X3_KC);
    }
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const bf16* r = &sB[cur][((wm * MF + f) * 16 + col) * X3_PITCH + 8 * kq];
      const bf16x8 bh = *(const bf16x8*)r;
      const bf16x8 bm = *(const bf16x8*)(r + X3_KC);
      const bf16x8 bl = *(const bf16x8*)(r + 2 * X3_KC);
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        // smallest terms first: they are added while the accumulator is smallest
        f32x4 c = acc[f][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bm, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[j], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bm, c, 0, 0, 0);
        acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bh, c, 0, 0, 0);
      }
    }
    if (kc + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + (wn * NF + j) * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int pix = m0 + (wm * MF + f) * 16 + col;
      if (pix >= M) continue;
      float v[4] = {acc[f][j][0] + bias.x, acc[f][j][1] + bias.y, acc[f][j][2] + bias.z, acc[f][j][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + (size_t)pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int b = pix / HWo;
        const int r = pix - b * HWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int MF, int NF, int WM, int WN>
static void launch_x3(const ConvParams& p, hipStream_t s, long M) {
  constexpr int BM = WM * MF * 16, BN = WN * NF * 16;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((p.Cout_pad + BN - 1) / BN));
  hipLaunchKernelGGL((conv_x3_lds_kernel<MF, NF, WM, WN>), grid, dim3(256), 0, s, p);
}

// x3 tile variants (ConvParams.impl = kF32X3 + index)
static bool launch_x3_variant(const ConvParams& p, hipStream_t s, long M, int v) {
  switch (v) {
    case 0: launch_x3<2, 2, 2, 2>(p, s, M); return true;  // 64 x 64
    case 1: launch_x3<4, 2, 2, 2>(p, s, M); return true;  // 128 x 64
    case 2: launch_x3<2, 4, 2, 2>(p, s, M); return true;  // 64 x 128
    case 3: launch_x3<4, 4, 2, 2>(p, s, M); return true;  // 128 x 128
    case 4: launch_x3<2, 2, 4, 1>(p, s, M); return true;  // 128 x 32
    case 5: launch_x3<1, 4, 4, 1>(p, s, M); return true;  // 64 x 64 (4 x 1 waves)
    case 6: launch_x3<2, 4, 4, 1>(p, s, M); return true;  // 128 x 64 (4 x 1 waves)
    case 7: launch_x3<1, 2, 2, 2>(p, s, M); return true;  // 32 x 64
    case 8: launch_x3<2, 3, 4, 1>(p, s, M); return true;  // 128 x 48
    case 9: launch_x3<2, 5, 4, 1>(p, s, M); return true;  // 128 x 80
    case 10: launch_x3<1, 1, 4, 1>(p, s, M); return true; // 64 x 16
    case 11: launch_x3<2, 1, 4, 1>(p, s, M); return true; // 128 x 16
    default: return false;
  }
}

// Explicit tile variants (ConvParams.impl = 10 + index): the sweep table of tools/bench_f32_convs.py.
// (MF, NF, WM, WN, KC): BM = WM*MF*16 pixels x BN = WN*NF*16 channels, KC k per LDS chunk.
static bool launch_lds_variant(const ConvParams& p, hipStream_t s, long M, int v) {
  switch (v) {
    case 0: launch_lds<2, 2, 2, 2, 32>(p, s, M); return true;   // 64 x 64
    case 1: launch_lds<4, 2, 2, 2, 32>(p, s, M); return true;   // 128 x 64
    case 2: launch_lds<2, 4, 2, 2, 32>(p, s, M); return true;   // 64 x 128
    case 3: launch_lds<4, 4, 2, 2, 32>(p, s, M); return true;   // 128 x 128
    case 4: launch_lds<2, 2, 2, 2, 64>(p, s, M); return true;   // 64 x 64, K64
    case 5: launch_lds<4, 2, 2, 2, 64>(p, s, M); return true;   // 128 x 64, K64
    case 6: launch_lds<2, 4, 2, 2, 64>(p, s, M); return true;   // 64 x 128, K64
    case 7: launch_lds<2, 2, 4, 1, 32>(p, s, M); return true;   // 128 x 32
    case 8: launch_lds<4, 1, 4, 1, 32>(p, s, M); return true;   // 256 x 16
    case 9: launch_lds<2, 3, 4, 1, 32>(p, s, M); return true;   // 128 x 48
    case 10: launch_lds<2, 5, 4, 1, 32>(p, s, M); return true;  // 128 x 80
    case 11: launch_lds<1, 4, 4, 1, 32>(p, s, M); return true;  // 64 x 64 (4 x 1 waves)
    case 12: launch_lds<2, 4, 4, 1, 32>(p, s, M); return true;  // 128 x 64 (4 x 1 waves)
    case 13: launch_lds<1, 2, 2, 2, 32>(p, s, M); return true;  // 32 x 64
    case 14: launch_lds<2, 2, 4, 1, 64>(p, s, M); return true;  // 128 x 32, K64
    case 15: launch_lds<2, 3, 4, 1, 64>(p, s, M); return true;  // 128 x 48, K64
    default: return false;
  }
}

// Pixel-tile depth: the largest MF that still launches >= 2 workgroups per CU.  BM is capped at 128 pixels
// (WM = 4 layouts stop at MF = 2): a 256-pixel tile needs 74+ KB of LDS and drops to one wave per SIMD.
template <int NF, int WM, int WN>
static void launch_lds_m(const ConvParams& p, hipStream_t s, long M) {
  constexpr int BN = WN * NF * 16;
  const long ny = (p.Cout_pad + BN - 1) / BN;
  if (WM * 64 <= 128 && ((M + WM * 64 - 1) / (WM * 64)) * ny >= 512)
    launch_lds<(WM * 64 <= 128 ? 4 : 2), NF, WM, WN>(p, s, M);
  else if (((M + WM * 32 - 1) / (WM * 32)) * ny >= 512)
    launch_lds<2, NF, WM, WN>(p, s, M);
  else
    launch_lds<1, NF, WM, WN>(p, s, M);
}

static int f32_conv_family() {
  static const int v = [] {
    const char* e = std::getenv("ARENA_F32_CONV");  // "direct" = the register-streamed kernel
    return (e != nullptr && std::string(e) == "direct") ? 1 : 2;
  }();
  return v;
}

// ---------------------------------------------------------------------------
// 3x3 halo-tile kernel (stride 1 or 2): a workgroup owns TH output rows x 16
// output columns of one image and BN = NF*16 output channels.  Per 16-channel
// input chunk it stages the input halo ((TH-1)*S+3 rows x 15*S+3 columns) and
// the chunk's [BN][9][16] weights in LDS once, then runs all nine taps from
// LDS: the im2col kernel above re-fetched each input pixel once per tap (9x
// the global/L2 traffic for 3x3 convs; these convs are 2.4 ms of the fp32
// detector, profiles/r2_fp32_irfused_ops.md).  Wave w computes output rows
// w, w+4, ... (MF = TH/4 rows of 16 pixels) x NF channel tiles.
// LDS pitches (floats) chosen so every ds_read_b128 lane group (16 lanes: 16 consecutive pixels or weight
// rows x 4 k-groups) lands on 16 distinct 16-B slots of the 256-B bank row: the stride between the lanes'
// rows must be 2 (mod 4) slots — 6 slots per halo pixel at stride 1 (2 x 5 = 10 slots between the pixels
// read by neighbouring lanes at stride 2), 38 slots per weight row.
constexpr int HALO_CK = 16;             // input channels per chunk
constexpr int HALO_WP = 9 * HALO_CK + 8;  // LDS pitch of a weight row (floats)
__host__ __device__ constexpr int halo_cp(int S) { return S == 1 ? HALO_CK + 8 : HALO_CK + 4; }

template <int S, int TH, int NF>
__global__ __launch_bounds__(256) void conv_f32_halo_kernel(const ConvParams p) {
  constexpr int TW = 16, MF = TH / 4, BN = NF * 16;
  constexpr int HR = (TH - 1) * S + 3, HC = (TW - 1) * S + 3, HPIX = HR * HC;
  constexpr int HALO_CP = halo_cp(S);
  __shared__ __attribute__((aligned(16))) float sX[HPIX * HALO_CP];
  __shared__ __attribute__((aligned(16))) float sW[BN * HALO_WP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles = tiles_x * tiles_y;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = bx - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - p.pad_t, ix0 = ox0 * S - p.pad_l;
  const int n0 = blockIdx.y * BN;
  const float* __restrict__ x = (const float*)p.x + (size_t)b * p.H * p.W * p.xs;
  const float* __restrict__ w = (const float*)p.w;

  f32x4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < p.Cin; c0 += HALO_CK) {
    // stage the halo (zero outside the image) and the chunk's weights
    for (int i = tid; i < HPIX * 4; i += 256) {
      const int px = i >> 2, g = i & 3;
      const int hy = px / HC, hx = px - hy * HC;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      *(float4*)&sX[px * HALO_CP + 4 * g] = load_f4_or_zero(x + ((size_t)iy * p.W + ix) * p.xs + c0 + 4 * g, x, ok);
    }
    for (int i = tid; i < BN * 36; i += 256) {  // [BN][9 taps][4 groups] float4
      const int row = i / 36, e = i - row * 36;
      const int tap = e >> 2, g = e & 3;
      const int n = n0 + row;
      const bool ok = n < p.Cout_pad;
      *(float4*)&sW[row * HALO_WP + tap * HALO_CK + 4 * g] =
          load_f4_or_zero(w + (size_t)n * p.Kpad + tap * p.Cin + c0 + 4 * g, w, ok);
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - ky * 3;
      float4 af[NF], bf[MF];
#pragma unroll
      for (int j = 0; j < NF; ++j) af[j] = *(const float4*)&sW[(j * 16 + col) * HALO_WP + tap * HALO_CK + 4 * kq];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int oy = wave + 4 * f;
        bf[f] = *(const float4*)&sX[((oy * S + ky) * HC + col * S + kx) * HALO_CP + 4 * kq];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < MF; ++f)
            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4_get(af[j], u), f4_get(bf[f], u), acc[f][j], 0, 0, 0);
    }
    __syncthreads();
  }

  const int HWo = p.Ho * p.Wo;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + j * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int oy = oy0 + wave + 4 * f, ox = ox0 + col;
      if (oy >= p.Ho || ox >= p.Wo) continue;
      const size_t pix = (size_t)b * HWo + (size_t)oy * p.Wo + ox;
      float v[4] = {acc[f][j][0] + bias.x, acc[f][j][1] + bias.y, acc[f][j][2] + bias.z, acc[f][j][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int S, int TH, int NF>
static void launch_halo(const ConvParams& p, hipStream_t s) {
  constexpr int BN = NF * 16;
  const int tiles = ((p.Wo + 15) / 16) * ((p.Ho + TH - 1) / TH);
  dim3 grid((unsigned)(p.B * tiles), (unsigned)((p.Cout_pad + BN - 1) / BN));
  hipLaunchKernelGGL((conv_f32_halo_kernel<S, TH, NF>), grid, dim3(256), 0, s, p);
}

template <int S, int TH>
static bool launch_halo_n(const ConvParams& p, hipStream_t s) {
  const int ncf = p.Cout_pad / 16;
  if (ncf == 1) launch_halo<S, TH, 1>(p, s);
  else if (ncf == 2) launch_halo<S, TH, 2>(p, s);
  else if (ncf == 3 || ncf == 9) launch_halo<S, TH, 3>(p, s);
  else if (ncf == 5) launch_halo<S, TH, 5>(p, s);
  else if (ncf % 4 == 0) launch_halo<S, TH, 4>(p, s);
  else return false;
  return true;
}

// ---------------------------------------------------------------------------
// 3x3 stride-1 halo tiles on the bf16 matrix cores with the triple-bf16 split
// (x3, see conv_x3_lds_kernel): the large detect-head / neck 3x3 convs are the
// one place the fp32 kernels are matrix-core bound (50-65 % MFMA busy,
// profiles/r2_fp32_pmc_ops.md), and here each staged input element feeds nine
// taps, so splitting it on the way into LDS costs 1/9 per use.
//
// Workgroup: TH = 8 output rows x 16 columns of one image x BN = NF*16 output
// channels; wave w computes rows w and w+4 (MF = 2).  Per 32-channel input
// chunk the (10 x 18)-pixel halo is staged once (three bf16 planes per pixel,
// 224-B pitch = 14 slots: conflict-free ds_read_b128 for 16 consecutive
// pixels); the chunk's weights are staged one kernel row (ky) at a time —
// [BN][3 taps][3 planes x 32] at a 608-B (38-slot) pitch — so LDS stays at
// 40 KB + BN x 0.6 KB.  The next stage's global loads (the next ky's weights,
// and at ky = 2 the next chunk's halo) are issued into registers before the
// current stage's 3 taps x MF x NF x 6 MFMAs run.  Cin need not be a multiple
// of 32: the tail chunk's missing channels stage as zeros.
// TH = 8 output rows per workgroup (4 waves) or 16 (8 waves, x3h16 variants): the stage's weights are
// re-read from L2 by every workgroup, and at 8 x 16 output pixels per stage that stream (~25 KB per
// 2.3k MFMA cycles) runs the L2 near its bandwidth; 16 x 16 tiles halve it per pixel (and the halo
// overhead drops from 1.41x to 1.27x) at one workgroup of 8 waves per CU.
constexpr int X3H_TW = 16, X3H_HC = X3H_TW + 2;
constexpr int X3H_XP = 3 * 32 + 16;      // bf16 per halo pixel (224 B)
constexpr int X3H_WP = 3 * 3 * 32 + 16;  // bf16 per weight row of one ky (3 taps x 3 planes x 32 k; 608 B)
__host__ __device__ constexpr int x3h_lds_bytes(int NF, int TH) {
  return ((TH + 2) * X3H_HC * X3H_XP + NF * 16 * X3H_WP) * 2;
}

template <int NF, int X3H_TH = 8>
__global__ __launch_bounds__(X3H_TH * 32) void conv_x3_halo_kernel(const ConvParams p) {
  constexpr int NT = X3H_TH * 32, NW = X3H_TH / 2;     // threads, waves (wave w: rows w and w + NW)
  constexpr int X3H_HR = X3H_TH + 2, X3H_HPIX = X3H_HR * X3H_HC;
  constexpr int X3H_XV = (X3H_HPIX * 8 + NT - 1) / NT;  // halo float4 per thread
  constexpr int BN = NF * 16, MF = 2;
  constexpr int WV = (BN * 3 * 8 + NT - 1) / NT;  // weight float4 per thread per ky stage
  extern __shared__ __attribute__((aligned(16))) bf16 x3h_lds[];
  bf16* sX = x3h_lds;                              // [HPIX][X3H_XP]
  bf16* sW = x3h_lds + X3H_HPIX * X3H_XP;          // [BN][X3H_WP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + X3H_TW - 1) / X3H_TW, tiles_y = (p.Ho + X3H_TH - 1) / X3H_TH;
  const int tiles = tiles_x * tiles_y;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = bx - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * X3H_TH, ox0 = tx * X3H_TW;
  const int iy0 = oy0 - p.pad_t, ix0 = ox0 - p.pad_l;
  const int n0 = blockIdx.y * BN;
  const int Cin = p.Cin;
  const float* __restrict__ x = (const float*)p.x + (size_t)b * p.H * p.W * p.xs;
  const float* __restrict__ w = (const float*)p.w;

  float4 rx[X3H_XV], rw[WV];
  auto load_x = [&](int c0) {
#pragma unroll
    for (int j = 0; j < X3H_XV; ++j) {
      const int i = tid + NT * j;
      const int px = i >> 3, g = i & 7;
      const int hy = px / X3H_HC, hx = px - hy * X3H_HC;
      const int iy = iy0 + hy, ix = ix0 + hx, c = c0 + 4 * g;
      const bool ok = i < X3H_HPIX * 8 && c < Cin && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      rx[j] = load_f4_or_zero(x + ((size_t)iy * p.W + ix) * p.xs + c, x, ok);
    }
  };
  auto load_w = [&](int c0, int ky) {
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int i = tid + NT * j;  // (row, kx, g)
      const int row = i / 24, e = i - row * 24;
      const int kx = e >> 3, g = e & 7;
      const int n = n0 + row, c = c0 + 4 * g;
      const bool ok = i < BN * 24 && n < p.Cout_pad && c < Cin;
      rw[j] = load_f4_or_zero(w + (size_t)n * p.Kpad + (ky * 3 + kx) * Cin + c, w, ok);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int j = 0; j < X3H_XV; ++j) {
      const int i = tid + NT * j;
      if (i < X3H_HPIX * 8) store_split4(&sX[(i >> 3) * X3H_XP], 4 * (i & 7), rx[j]);
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int i = tid + NT * j;
      if (i < BN * 24) {
        const int row = i / 24, e = i - row * 24;
        store_split4(&sW[row * X3H_WP + (e >> 3) * 96], 4 * (e & 7), rw[j]);
      }
    }
  };

  f32x4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nstage = ((Cin + 31) / 32) * 3;
  load_x(0);
  load_w(0, 0);
  for (int st = 0; st < nstage; ++st) {
    const int c0 = (st / 3) * 32, ky = st - (st / 3) * 3;
    if (ky == 0) store_x();
    store_w();
    __syncthreads();
    if (st + 1 < nstage) {  // next stage's global loads overlap this stage's MFMAs
      const int nc0 = ((st + 1) / 3) * 32, nky = (st + 1) - ((st + 1) / 3) * 3;
      if (nky == 0) load_x(nc0);
      load_w(nc0, nky);
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      bf16x8 ah[NF], am[NF], al[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const bf16* r = &sW[(j * 16 + col) * X3H_WP + kx * 96 + 8 * kq];
        ah[j] = *(const bf16x8*)r;
        am[j] = *(const bf16x8*)(r + 32);
        al[j] = *(const bf16x8*)(r + 64);
      }
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int oy = wave + NW * f;
        const bf16* r = &sX[((oy + ky) * X3H_HC + col + kx) * X3H_XP + 8 * kq];
        const bf16x8 bh = *(const bf16x8*)r;
        const bf16x8 bm = *(const bf16x8*)(r + 32);
        const bf16x8 bl = *(const bf16x8*)(r + 64);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          f32x4 c = acc[f][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[j], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bm, c, 0, 0, 0);
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bh, c, 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  const int HWo = p.Ho * p.Wo;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + j * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int oy = oy0 + wave + NW * f, ox = ox0 + col;
      if (oy >= p.Ho || ox >= p.Wo) continue;
      const size_t pix = (size_t)b * HWo + (size_t)oy * p.Wo + ox;
      float v[4] = {acc[f][j][0] + bias.x, acc[f][j][1] + bias.y, acc[f][j][2] + bias.z, acc[f][j][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int NF, int TH = 8>
static void launch_x3_halo(const ConvParams& p, hipStream_t s) {
  constexpr int BN = NF * 16;
  const int tiles = ((p.Wo + X3H_TW - 1) / X3H_TW) * ((p.Ho + TH - 1) / TH);
  dim3 grid((unsigned)(p.B * tiles), (unsigned)((p.Cout_pad + BN - 1) / BN));
  hipLaunchKernelGGL((conv_x3_halo_kernel<NF, TH>), grid, dim3(TH * 32), x3h_lds_bytes(NF, TH), s, p);
}

void x3_halo_prepare() {
#define X3H_ATTR(NF_, TH_)                                                                            \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3_halo_kernel<NF_, TH_>,                       \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  X3H_ATTR(1, 8) X3H_ATTR(2, 8) X3H_ATTR(3, 8) X3H_ATTR(4, 8) X3H_ATTR(5, 8)
  X3H_ATTR(2, 16) X3H_ATTR(3, 16) X3H_ATTR(4, 16)
#undef X3H_ATTR
}

// ---------------------------------------------------------------------------
// 3x3 stride-1 conv over 16 input channels (the YOLO space-to-depth stem's 320x320 and 160x160 layers) on the
// bf16 matrix cores with the triple-bf16 split.  The generic halo kernel runs a 16-channel input as a 32-deep
// chunk half zero (9 slabs of 32 per output tile); here one kernel row's three taps x 16 channels (48 k, laid
// out contiguously in the [Cout][ky][kx][c] weight row) fill 2 slabs: kx 0-1 in the first, kx 2 plus zeros in
// the second (6 slabs, 1.5x fewer MFMAs), and the whole input halo (10 x 18 pixels x 16 channels x 3 planes =
// 17 KB) and all weights (BN x 3 rows x 416 B) are staged once: no K loop, one barrier.  Lane (col, kq) of
// slab s reads channels c0..c0+7 of tap kx = (32 s + 8 kq) / 16 at pixel column col + kx (kx = 3 is the zero
// half: it re-reads a valid pixel, its weights are zero).  Pitches (LDS bank model of MI355X_MICROARCH.md
// §LDS): 96 B per halo pixel and 3 x 416 B per weight row are conflict-free for these ds_read_b128 patterns.
constexpr int H16_TH = 8, H16_TW = 16, H16_HR = H16_TH + 2, H16_HC = H16_TW + 2, H16_HPIX = H16_HR * H16_HC;
constexpr int H16_XP = 48;    // bf16 per halo pixel: [h|m|l][16]
constexpr int H16_WPK = 208;  // bf16 per (row, ky): [2 slabs][h|m|l][32] = 192 + 16 pad (416 B)

//
// LB: the input is the letterboxed space-to-depth image itself (the stem conv of the fp32 detector): each halo
// pixel is sampled from the uint8 image (letterbox_s2d_px, the letterbox kernel's own sampler, so the values
// are bitwise those of the unfused program) and the 320x320x16 fp32 s2d tensor is never written or re-read.
template <int NF, bool LB>
__global__ __launch_bounds__(256) void conv_x3_h16_kernel(const ConvParams p) {
  constexpr int BN = NF * 16, MF = 2;
  __shared__ __attribute__((aligned(16))) bf16 sX[H16_HPIX * H16_XP];
  __shared__ __attribute__((aligned(16))) bf16 sW[BN * 3 * H16_WPK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + H16_TW - 1) / H16_TW, tiles_y = (p.Ho + H16_TH - 1) / H16_TH;
  const int tiles = tiles_x * tiles_y;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = bx - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * H16_TH, ox0 = tx * H16_TW;
  const int iy0 = oy0 - p.pad_t, ix0 = ox0 - p.pad_l;
  const int n0 = blockIdx.y * BN;
  const float* __restrict__ x = (const float*)p.x + (size_t)b * p.H * p.W * p.xs;
  const float* __restrict__ w = (const float*)p.w;

  if constexpr (LB) {
    // one thread per halo pixel: 12 live channels sampled from the image, 4 zero; conv padding is zero.  The
    // letterboxed values are uint8 integers k (/255 follows): k is exact in bf16, so only the h plane is
    // staged and the weights carry the /255 (w' = w / 255 split in three planes): k * w'_h + k * w'_m + k * w'_l
    // is k * w / 255 to fp32 accuracy in three MFMAs instead of six, and the halo needs no split arithmetic
    const ImageMeta m = p.lb_meta[b];
    for (int px = tid; px < H16_HPIX; px += 256) {
      const int hy = px / H16_HC, hx = px - hy * H16_HC;
      const int iy = iy0 + hy, ix = ix0 + hx;
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = 0.f;
      if ((unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W) letterbox_s2d_px_u8(p.lb_pool, m, iy, ix, v);
      bf16x8 h[2];
#pragma unroll
      for (int c = 0; c < 16; ++c) h[c >> 3][c & 7] = (bf16)v[c];
      bf16* d = &sX[px * H16_XP];
      *(bf16x8*)d = h[0];
      *(bf16x8*)(d + 8) = h[1];
    }
  } else {
  // input halo: 4 float4 (16 channels) per pixel, split into three planes
  for (int i = tid; i < H16_HPIX * 4; i += 256) {
    const int px = i >> 2, g = i & 3;
    const int hy = px / H16_HC, hx = px - hy * H16_HC;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    const float4 v = load_f4_or_zero(x + ((size_t)iy * p.W + ix) * p.xs + 4 * g, x, ok);
    bf16x4 h, m, l;
    bf16 th, tm, tl;
    split3(v.x, th, tm, tl); h[0] = th; m[0] = tm; l[0] = tl;
    split3(v.y, th, tm, tl); h[1] = th; m[1] = tm; l[1] = tl;
    split3(v.z, th, tm, tl); h[2] = th; m[2] = tm; l[2] = tl;
    split3(v.w, th, tm, tl); h[3] = th; m[3] = tm; l[3] = tl;
    bf16* d = &sX[px * H16_XP + 4 * g];
    *(bf16x4*)d = h;
    *(bf16x4*)(d + 16) = m;
    *(bf16x4*)(d + 32) = l;
  }
  }
  // weights: row n, kernel row ky -> 64 k (48 real: kx 0..2 x 16 channels) in two 32-deep slabs
  for (int i = tid; i < BN * 3 * 16; i += 256) {
    const int row = i / 48, e = i - row * 48;
    const int ky = e >> 4, q = e & 15;  // q: float4 index within the 64-k row (12..15 are the zero half)
    const int n = n0 + row, k = ky * 48 + 4 * q;
    const bool ok = n < p.Cout_pad && q < 12;
    float4 v = load_f4_or_zero(w + (size_t)n * p.Kpad + k, w, ok);
    if constexpr (LB) v = make_float4(v.x / 255.0f, v.y / 255.0f, v.z / 255.0f, v.w / 255.0f);
    bf16x4 h, m, l;
    bf16 th, tm, tl;
    split3(v.x, th, tm, tl); h[0] = th; m[0] = tm; l[0] = tl;
    split3(v.y, th, tm, tl); h[1] = th; m[1] = tm; l[1] = tl;
    split3(v.z, th, tm, tl); h[2] = th; m[2] = tm; l[2] = tl;
    split3(v.w, th, tm, tl); h[3] = th; m[3] = tm; l[3] = tl;
    const int slab = q >> 3, kk = 4 * (q & 7);
    bf16* d = &sW[(row * 3 + ky) * H16_WPK + slab * 96 + kk];
    *(bf16x4*)d = h;
    *(bf16x4*)(d + 32) = m;
    *(bf16x4*)(d + 64) = l;
  }
  __syncthreads();

  f32x4 acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int kabs = sl * 32 + kq * 8;
      const int kx = kabs >> 4 < 3 ? kabs >> 4 : 2, c0 = kabs & 15;
      bf16x8 ah[NF], am[NF], al[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const bf16* r = &sW[((j * 16 + col) * 3 + ky) * H16_WPK + sl * 96 + 8 * kq];
        ah[j] = *(const bf16x8*)r;
        am[j] = *(const bf16x8*)(r + 32);
        al[j] = *(const bf16x8*)(r + 64);
      }
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int oy = wave + 4 * f;
        const bf16* r = &sX[((oy + ky) * H16_HC + col + kx) * H16_XP + c0];
        if constexpr (LB) {  // exact integer activations: one plane
          const bf16x8 bh = *(const bf16x8*)r;
#pragma unroll
          for (int j = 0; j < NF; ++j) {
            f32x4 c = acc[f][j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[j], bh, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bh, c, 0, 0, 0);
            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bh, c, 0, 0, 0);
          }
          continue;
        }
        const bf16x8 bh = *(const bf16x8*)r, bm = *(const bf16x8*)(r + 16), bl = *(const bf16x8*)(r + 32);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          f32x4 c = acc[f][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bm, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[j], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[j], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bm, c, 0, 0, 0);
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bh, c, 0, 0, 0);
        }
      }
    }
  }

  const int HWo = p.Ho * p.Wo;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + j * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int oy = oy0 + wave + 4 * f, ox = ox0 + col;
      if (oy >= p.Ho || ox >= p.Wo) continue;
      const size_t pix = (size_t)b * HWo + (size_t)oy * p.Wo + ox;
      float v[4] = {acc[f][j][0] + bias.x, acc[f][j][1] + bias.y, acc[f][j][2] + bias.z, acc[f][j][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int NF>
static void launch_x3_h16(const ConvParams& p, hipStream_t s) {
  constexpr int BN = NF * 16;
  const int tiles = ((p.Wo + H16_TW - 1) / H16_TW) * ((p.Ho + H16_TH - 1) / H16_TH);
  dim3 grid((unsigned)(p.B * tiles), (unsigned)((p.Cout_pad + BN - 1) / BN));
  if (p.lb_meta != nullptr)
    hipLaunchKernelGGL((conv_x3_h16_kernel<NF, true>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_x3_h16_kernel<NF, false>), grid, dim3(256), 0, s, p);
}

// impl kF32X3H16: 3x3 stride-1 pad-1 convs over exactly 16 input channels (Kpad 144)
static bool x3_h16(const ConvParams& p, hipStream_t s) {
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.Cin != 16 || p.Kpad != 144 || p.pad_t != 1 || p.pad_l != 1 ||
      p.xs % 4 != 0)
    return false;
  const int ncf = p.Cout_pad / 16;
  if (ncf == 1) launch_x3_h16<1>(p, s);
  else if (ncf % 2 == 0) launch_x3_h16<2>(p, s);
  else launch_x3_h16<1>(p, s);
  return true;
}

// impl kF32X3Halo: 3x3 stride-1 convs with Kpad == 9 * Cin (tap-major K) and Cin % 4 == 0.  nf > 0 forces the
// channel tile (impl kF32X3HaloN3 / N2: BN 48 / 32): the 80-channel detect-head convs at NF = 5 need 89 KB of
// LDS (one workgroup, one wave per SIMD); two 48-channel tiles fit twice per CU at 17 % padded channels.
static bool x3_halo(const ConvParams& p, hipStream_t s, int nf = 0, int th = 8) {
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.Kpad != 9 * p.Cin || p.Cin % 4 != 0) return false;
  const int ncf = p.Cout_pad / 16;
  if (th == 16) {  // 16-row tiles (8 waves): 48 / 64-channel tiles, or 32 for narrow layers
    if (nf == 3 || (nf == 0 && (ncf == 3 || ncf == 5 || ncf == 9))) launch_x3_halo<3, 16>(p, s);
    else if (nf == 2 || (nf == 0 && ncf <= 2)) launch_x3_halo<2, 16>(p, s);
    else launch_x3_halo<4, 16>(p, s);
    return true;
  }
  if (nf == 3) {
    launch_x3_halo<3>(p, s);
    return true;
  }
  if (nf == 2) {
    launch_x3_halo<2>(p, s);
    return true;
  }
  if (ncf == 1) launch_x3_halo<1>(p, s);
  else if (ncf == 2) launch_x3_halo<2>(p, s);
  else if (ncf == 3 || ncf == 9) launch_x3_halo<3>(p, s);
  else if (ncf == 5) launch_x3_halo<5>(p, s);
  else if (ncf % 4 == 0) launch_x3_halo<4>(p, s);
  else return false;
  return true;
}

// Where the halo kernel runs (measured per layer on MI355X, profiles/r2_fp32_halo_ops.md vs
// r2_fp32_irfused_ops.md): stride-1 3x3 convs on >= 40-wide maps with <= 128 input channels — the
// s2d stem 333 -> 199 us, the 160x160 C3 bottleneck 89 -> 54 us, the 80x80 detect-head convs 375 -> 332
// and 196 -> 171 us.  Stride-2 convs (2-3x the halo per output pixel) and the 20x20 maps (16-wide tiles
// waste 37 % of a 20-wide row) stay on the im2col kernel, which was faster there.
// ARENA_F32_HALO=0 disables it, =2 forces it for every eligible 3x3 conv.
static bool halo_f32(const ConvParams& p, hipStream_t s, bool force = false) {
  static const int env_mode = [] {
    const char* e = std::getenv("ARENA_F32_HALO");
    return e == nullptr ? 1 : std::atoi(e);
  }();
  const int mode = force ? 2 : env_mode;
  if (mode == 0 || p.KH != 3 || p.KW != 3 || p.Cin % HALO_CK != 0 || p.Kpad != 9 * p.Cin) return false;
  if (mode == 1 && !(p.stride == 1 && p.Wo >= 40 && p.Cin <= 128)) return false;
  if (p.stride == 1) return launch_halo_n<1, 8>(p, s);
  if (p.stride == 2) return launch_halo_n<2, 4>(p, s);
  return false;
}

// ---------------------------------------------------------------------------
// Weight-stationary streaming small-K conv, fp32-accurate on the bf16 matrix cores (triple-bf16 split).
// The small-K 1x1 convs (K <= 192: YOLO C3 / neck pointwise layers, MobileNetV2 expand GEMMs) ran 2-10x
// off their memory floor in the tiled kernels above (profiles/r2_fp32_irprefetch_ops.md: 10-30 % MFMA
// busy, each workgroup's life one load latency + 2-6 k-chunks + its stores): here a workgroup splits its
// BN x K weight tile into three bf16 planes in LDS once, then its four waves stream 16-pixel tiles through
// a grid-stride loop, the next tile's activations loaded into registers while the current tile's
// 6 x KS x NF MFMAs run.  Lane l takes pixel (l & 15) and k = 8 (l >> 4) .. +7 of each 32-deep slab (two
// float4 of the NHWC row), splits them in registers, and reads the weight fragment of every channel tile
// from LDS (row pitch 6K + 32 B = 2 (mod 4) 16-B slots: conflict-free ds_read_b128).
constexpr int STR_THREADS = 256;

__device__ __forceinline__ f32x4 mfma_x3f(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                          const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

template <int NF, int KS>
__global__ __launch_bounds__(STR_THREADS) void conv_x3_stream_kernel(const ConvParams p) {
  constexpr int BN = NF * 16, K = KS * 32, WP = 6 * K + 32;
  __shared__ __attribute__((aligned(16))) uint8_t sW[BN * WP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int n0 = blockIdx.y * BN;
  const int HWo = p.Ho * p.Wo;
  const int M = live_batch(p.B, p.bdev) * HWo;
  const int tiles = (M + 15) / 16;
  int t = blockIdx.x * 4 + wave;
  if (blockIdx.x * 4 >= tiles) return;

  // weight tile -> three bf16 planes (zero past Cout_pad / Kpad)
  const float* __restrict__ w = (const float*)p.w;
  for (int i = tid; i < BN * K / 4; i += STR_THREADS) {
    const int row = i / (K / 4), k = 4 * (i - row * (K / 4));
    const bool ok = n0 + row < p.Cout_pad && k < p.Kpad;
    float4 v = *(const float4*)(ok ? w + (size_t)(n0 + row) * p.Kpad + k : w);
    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
    bf16x4 h, m, l;
    bf16 th, tm, tl;
    split3(v.x, th, tm, tl); h[0] = th; m[0] = tm; l[0] = tl;
    split3(v.y, th, tm, tl); h[1] = th; m[1] = tm; l[1] = tl;
    split3(v.z, th, tm, tl); h[2] = th; m[2] = tm; l[2] = tl;
    split3(v.w, th, tm, tl); h[3] = th; m[3] = tm; l[3] = tl;
    uint8_t* r = sW + row * WP + k * 2;
    *(bf16x4*)r = h;
    *(bf16x4*)(r + 2 * K) = m;
    *(bf16x4*)(r + 4 * K) = l;
  }
  float4 bias[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + j * 16 + 4 * kq;
    bias[j] = cb < p.Cout ? *(const float4*)(p.bias + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();

  const float* __restrict__ x = (const float*)p.x;
  const int tstride = gridDim.x * 4;
  // implicit im2col: this lane's 8 k of slab sl are input channels ci..ci+7 of one tap (Cin % 8 == 0)
  int tdy[KS], tdx[KS], tci[KS];
#pragma unroll
  for (int sl = 0; sl < KS; ++sl) {
    const int k0 = sl * 32 + kq * 8, tap = k0 / p.Cin;
    const int kh = tap / p.KW;
    tci[sl] = k0 - tap * p.Cin;
    tdy[sl] = tap < p.KH * p.KW ? kh - p.pad_t : -(1 << 20);  // past the last tap: zero (fails the bounds test)
    tdx[sl] = tap - kh * p.KW - p.pad_l;
  }
  float4 b0[KS], b1[KS];
  auto load_b = [&](int tt) {
    const int pix = tt * 16 + col;
    const int b = pix / HWo, r = pix - b * HWo;
    const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
    const float* xb = x + (size_t)b * p.H * p.W * p.xs;
#pragma unroll
    for (int sl = 0; sl < KS; ++sl) {
      const int iy = oy * p.stride + tdy[sl], ix = ox * p.stride + tdx[sl];
      const bool ok = pix < M && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const float* ptr = xb + ((size_t)iy * p.W + ix) * p.xs + tci[sl];
      b0[sl] = load_f4_or_zero(ptr, x, ok);
      b1[sl] = load_f4_or_zero(ptr + 4, x, ok);
    }
  };
  if (t < tiles) load_b(t);
  for (; t < tiles; t += tstride) {
    float4 c0[KS], c1[KS];
#pragma unroll
    for (int sl = 0; sl < KS; ++sl) {
      c0[sl] = b0[sl];
      c1[sl] = b1[sl];
    }
    if (t + tstride < tiles) load_b(t + tstride);  // next tile's activations in flight during this tile
    f32x4 acc[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < KS; ++sl) {
      const float v[8] = {c0[sl].x, c0[sl].y, c0[sl].z, c0[sl].w, c1[sl].x, c1[sl].y, c1[sl].z, c1[sl].w};
      bf16x8 bh, bm, bl;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bf16 th, tm, tl;
        split3(v[i], th, tm, tl);
        bh[i] = th;
        bm[i] = tm;
        bl[i] = tl;
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const uint8_t* ra = sW + (j * 16 + col) * WP + sl * 64 + kq * 16;
        acc[j] = mfma_x3f(*(const bf16x8*)ra, *(const bf16x8*)(ra + 2 * K), *(const bf16x8*)(ra + 4 * K), bh, bm,
                          bl, acc[j]);
      }
    }
    const int pix = t * 16 + col;
    if (pix >= M) continue;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int cb = n0 + j * 16 + kq * 4;
      if (cb >= p.Cout) continue;
      float v[4] = {acc[j][0] + bias[j].x, acc[j][1] + bias[j].y, acc[j][2] + bias[j].z, acc[j][3] + bias[j].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + (size_t)pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int b = pix / HWo;
        const int r = pix - b * HWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int NF, int KS>
static void launch_stream(const ConvParams& p, hipStream_t s) {
  constexpr int BN = NF * 16;
  const int ny = (p.Cout_pad + BN - 1) / BN;
  const long tiles = ((long)p.B * p.Ho * p.Wo + 15) / 16;
  // ~1024 resident workgroups over the chip (4 per CU), each streaming tiles of 16 pixels per wave
  const long gx = std::max(1L, std::min((tiles + 3) / 4, (long)std::max(1, 1024 / ny)));
  hipLaunchKernelGGL((conv_x3_stream_kernel<NF, KS>), dim3((unsigned)gx, (unsigned)ny), dim3(STR_THREADS), 0, s, p);
}

template <int NF>
static bool launch_stream_k(const ConvParams& p, hipStream_t s) {
  switch ((p.Kpad + 31) / 32) {
    case 1: launch_stream<NF, 1>(p, s); return true;
    case 2: launch_stream<NF, 2>(p, s); return true;
    case 3: launch_stream<NF, 3>(p, s); return true;
    case 4: launch_stream<NF, 4>(p, s); return true;
    case 5: launch_stream<NF, 5>(p, s); return true;
    case 6: launch_stream<NF, 6>(p, s); return true;
    default: return false;
  }
}

// Exact-fp32 streaming variant (impl kF32StreamExact): the same weight-stationary pixel stream on
// v_mfma_f32_16x16x4_f32 with fp32 operands and no split.  The split variant ran VALU-bound on the small-K
// layers (profiles/r2_fp32_pmc_ops_v2.md: 10-30 VALU per MFMA — eight splits per lane per 32-deep slab plus the
// SiLU epilogue for a K = 32 conv's 12 MFMAs): at K <= 64 the 4x-slower fp32 MFMA costs less than the split.
// Lane l supplies k = 16 c + 4 (l >> 4) + s in step s of chunk c (one float4 per chunk: Cin % 4 == 0 keeps the 4
// channels in one tap); weight rows are fp32 in LDS at a K + 8 float pitch (2 (mod 4) 16-B slots).
template <int NF, int KC>
__global__ __launch_bounds__(STR_THREADS) void conv_f32_stream_kernel(const ConvParams p) {
  constexpr int BN = NF * 16, K = KC * 16, WPF = K + 8;
  __shared__ __attribute__((aligned(16))) float sW[BN * WPF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int n0 = blockIdx.y * BN;
  const int HWo = p.Ho * p.Wo;
  const int M = live_batch(p.B, p.bdev) * HWo;
  const int tiles = (M + 15) / 16;
  int t = blockIdx.x * 4 + wave;
  if (blockIdx.x * 4 >= tiles) return;

  const float* __restrict__ w = (const float*)p.w;
  for (int i = tid; i < BN * K / 4; i += STR_THREADS) {
    const int row = i / (K / 4), k = 4 * (i - row * (K / 4));
    const bool ok = n0 + row < p.Cout_pad && k < p.Kpad;
    *(float4*)&sW[row * WPF + k] = load_f4_or_zero(w + (size_t)(n0 + row) * p.Kpad + k, w, ok);
  }
  float4 bias[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int cb = n0 + j * 16 + 4 * kq;
    bias[j] = cb < p.Cout ? *(const float4*)(p.bias + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();

  const float* __restrict__ x = (const float*)p.x;
  const int tstride = gridDim.x * 4;
  int tdy[KC], tdx[KC], tci[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const int k0 = c * 16 + kq * 4, tap = k0 / p.Cin;
    const int kh = tap / p.KW;
    tci[c] = k0 - tap * p.Cin;
    tdy[c] = (tap < p.KH * p.KW && k0 < p.Kpad) ? kh - p.pad_t : -(1 << 20);
    tdx[c] = tap - kh * p.KW - p.pad_l;
  }
  float4 bnext[KC];
  auto load_b = [&](int tt) {
    const int pix = tt * 16 + col;
    const int b = pix / HWo, r = pix - b * HWo;
    const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
    const float* xb = x + (size_t)b * p.H * p.W * p.xs;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int iy = oy * p.stride + tdy[c], ix = ox * p.stride + tdx[c];
      const bool ok = pix < M && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      bnext[c] = load_f4_or_zero(xb + ((size_t)iy * p.W + ix) * p.xs + tci[c], x, ok);
    }
  };
  if (t < tiles) load_b(t);
  for (; t < tiles; t += tstride) {
    float4 bc[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) bc[c] = bnext[c];
    if (t + tstride < tiles) load_b(t + tstride);
    f32x4 acc[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const float4 a = *(const float4*)&sW[(j * 16 + col) * WPF + c * 16 + kq * 4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4_get(a, s4), f4_get(bc[c], s4), acc[j], 0, 0, 0);
      }
    }
    const int pix = t * 16 + col;
    if (pix >= M) continue;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int cb = n0 + j * 16 + kq * 4;
      if (cb >= p.Cout) continue;
      float v[4] = {acc[j][0] + bias[j].x, acc[j][1] + bias[j].y, acc[j][2] + bias[j].z, acc[j][3] + bias[j].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        const float4 rv = *(const float4*)((const float*)p.res + (size_t)pix * p.rs + cb);
        v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
      }
      const float4 o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = o;
      if (p.y2 != nullptr) {
        const int b = pix / HWo;
        const int r = pix - b * HWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int W2 = 2 * p.Wo;
        float* y2 = (float*)p.y2;
        const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
        *(float4*)(y2 + base * p.y2s + cb) = o;
        *(float4*)(y2 + (base + 1) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2) * p.y2s + cb) = o;
        *(float4*)(y2 + (base + W2 + 1) * p.y2s + cb) = o;
      }
    }
  }
}

template <int NF, int KC>
static void launch_stream_exact(const ConvParams& p, hipStream_t s) {
  constexpr int BN = NF * 16;
  const int ny = (p.Cout_pad + BN - 1) / BN;
  const long tiles = ((long)p.B * p.Ho * p.Wo + 15) / 16;
  const long gx = std::max(1L, std::min((tiles + 3) / 4, (long)std::max(1, 1024 / ny)));
  hipLaunchKernelGGL((conv_f32_stream_kernel<NF, KC>), dim3((unsigned)gx, (unsigned)ny), dim3(STR_THREADS), 0, s, p);
}

template <int NF>
static bool launch_stream_exact_k(const ConvParams& p, hipStream_t s) {
  const int kc = p.Kpad / 16;  // chunk counts rounded up to an instantiated one (weights / taps past Kpad are zero)
  if (kc <= 1) launch_stream_exact<NF, 1>(p, s);
  else if (kc <= 2) launch_stream_exact<NF, 2>(p, s);
  else if (kc <= 4) launch_stream_exact<NF, 4>(p, s);
  else if (kc <= 6) launch_stream_exact<NF, 6>(p, s);
  else if (kc <= 8) launch_stream_exact<NF, 8>(p, s);
  else if (kc <= 10) launch_stream_exact<NF, 10>(p, s);
  else if (kc <= 12) launch_stream_exact<NF, 12>(p, s);
  else return false;
  return true;
}

static bool f32_stream(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 4 != 0 || p.Kpad > 192 || p.Kpad % 16 != 0 || p.Kpad < p.KH * p.KW * p.Cin || p.xs % 4 != 0)
    return false;
  const int ncf = p.Cout_pad / 16;
  const int nf = ncf <= 5 ? ncf : ncf % 4 == 0 ? 4 : ncf % 3 == 0 ? 3 : ncf % 5 == 0 ? 5 : ncf % 2 == 0 ? 2 : 1;
  switch (nf) {
    case 1: return launch_stream_exact_k<1>(p, s);
    case 2: return launch_stream_exact_k<2>(p, s);
    case 3: return launch_stream_exact_k<3>(p, s);
    case 4: return launch_stream_exact_k<4>(p, s);
    case 5: return launch_stream_exact_k<5>(p, s);
    default: return false;
  }
}

// impl kF32Stream (channel tile by Cout) / kF32StreamN2 (32-channel tiles): any conv with Cin % 8 == 0 and
// Kpad <= 192 (1x1 pointwise layers, and the 3x3 / 2x2 convs over 16-channel space-to-depth stems, whose
// taps are gathered per lane: 8 k of a slab never straddle two taps)
static bool x3_stream(const ConvParams& p, hipStream_t s, int nf_force) {
  if (p.Cin % 8 != 0 || p.Kpad > 192 || p.Kpad < p.KH * p.KW * p.Cin || p.xs % 4 != 0) return false;
  const int ncf = p.Cout_pad / 16;
  const int nf = nf_force ? nf_force
                          : ncf <= 5 ? ncf : ncf % 4 == 0 ? 4 : ncf % 3 == 0 ? 3 : ncf % 5 == 0 ? 5 : ncf % 2 == 0 ? 2 : 1;
  switch (nf) {
    case 1: return launch_stream_k<1>(p, s);
    case 2: return launch_stream_k<2>(p, s);
    case 3: return launch_stream_k<3>(p, s);
    case 4: return launch_stream_k<4>(p, s);
    case 5: return launch_stream_k<5>(p, s);
    default: return false;
  }
}

void conv2d_f32(const ConvParams& p, hipStream_t s) {
  if (p.Cin % 4 != 0 || p.xs % 4 != 0 || p.Kpad % 16 != 0 || p.Cout_pad % 16 != 0 || p.Cout % 4 != 0 ||
      p.Cout > p.Cout_pad || p.ys % 4 != 0)
    throw std::runtime_error("conv2d_f32: unsupported geometry (Cin/xs/ys %4, Kpad %16, Cout_pad %16, Cout %4)");
  if (p.Cin < 16) throw std::runtime_error("conv2d_f32: Cin must be >= 16");
  if (p.Kpad < p.KH * p.KW * p.Cin) throw std::runtime_error("conv2d_f32: Kpad < KH*KW*Cin");
  if (p.pw_w != nullptr) {  // fused Detect-head 1x1: only the x3hg epilogue variants implement it
    if (p.impl >= kF32X3HRPw && p.impl < kF32X3HRPw + kF32X3HRPwVariants) {
      if (!conv_x3hr_pw(p, s, p.impl - kF32X3HRPw))
        throw std::runtime_error("conv2d_f32: a fused pointwise epilogue needs an x3hr-pw variant that fits the conv");
      return;
    }
    const int v = p.impl >= kF32X3HGPw && p.impl < kF32X3HGPw + kF32X3HGPwVariants ? p.impl - kF32X3HGPw
                  : p.impl >= kF32X3HGPwSmall && p.impl < kF32X3HGPwSmall + kF32X3HGPwSmallVariants
                      ? kF32X3HGPwVariants + p.impl - kF32X3HGPwSmall
                  : p.impl == 0 ? (p.Cout_pad <= 64 ? 0 : 2)
                                : -1;
    if (v < 0 || !conv_x3hg_pw(p, s, v))
      throw std::runtime_error("conv2d_f32: a fused pointwise epilogue needs an x3hg-pw variant that fits the conv");
    return;
  }
  if (p.res != nullptr && p.rs % 4 != 0) throw std::runtime_error("conv2d_f32: residual stride % 4");
  if (p.y2 != nullptr && p.y2s % 4 != 0) throw std::runtime_error("conv2d_f32: upsampled stride % 4");
  const long M = (long)p.B * p.Ho * p.Wo;
  if (M <= 0) return;
  if (M > 0x7fffffffL || (long)p.B * p.H * p.W * p.xs > 0x7fffffffL) throw std::runtime_error("conv2d_f32: too large");
  const int ncf = p.Cout_pad / 16;
  if (p.lb_meta != nullptr) {  // letterbox source: only the x3-h16 stem kernel samples images
    if (p.lb_pool == nullptr || !x3_h16(p, s))
      throw std::runtime_error("conv2d_f32: a letterbox-source conv must be a 3x3 s1 pad-1 conv over 16 channels");
    return;
  }
  if (p.impl >= 10) {  // explicit variant (autotune table / microbenchmarks)
    if (p.impl >= kF32X3G && p.impl < kF32X3G + kF32X3GVariants) {
      if (!conv_x3g(p, s, p.impl - kF32X3G))
        throw std::runtime_error("conv2d_f32: not an x3g-eligible conv (needs pre-split weights)");
      return;
    }
    if (p.impl >= kF32X3GSK && p.impl < kF32X3GSK + kF32X3GSKVariants) {
      if (!conv_x3g_sk(p, s, p.impl - kF32X3GSK))
        throw std::runtime_error("conv2d_f32: not a split-K x3g-eligible conv (pre-split weights, workspace)");
      return;
    }
    if (p.impl >= kF32X3HG && p.impl < kF32X3HG + kF32X3HGVariants) {
      if (!conv_x3hg(p, s, p.impl - kF32X3HG))
        throw std::runtime_error("conv2d_f32: not an x3hg-eligible conv (3x3 s1 with pre-split weights)");
      return;
    }
    if (p.impl >= kF32X3HR && p.impl < kF32X3HR + kF32X3HRVariants) {
      if (!conv_x3hr(p, s, p.impl - kF32X3HR))
        throw std::runtime_error("conv2d_f32: not an x3hr-eligible conv (3x3 s1 with pre-split weights)");
      return;
    }
    if (p.impl == kF32X3H16) {
      if (!x3_h16(p, s)) throw std::runtime_error("conv2d_f32: not an x3-h16-eligible conv (3x3 s1 over 16 channels)");
      return;
    }
    if (p.impl == kF32Fc) {
      if (!conv_fc_f32(p, s)) throw std::runtime_error("conv2d_f32: not an FC-eligible conv (1x1 map, Kpad 1280)");
      return;
    }
    if (p.impl == kF32StreamExact) {
      if (!f32_stream(p, s)) throw std::runtime_error("conv2d_f32: not a stream-eligible conv (Cin % 4, Kpad <= 192)");
      return;
    }
    if (p.impl == kF32Stream || p.impl == kF32StreamN2) {
      if (!x3_stream(p, s, p.impl == kF32StreamN2 ? 2 : 0))
        throw std::runtime_error("conv2d_f32: not a stream-eligible conv (Cin % 8, Kpad <= 192)");
      return;
    }
    if (p.impl == kF32X3Halo || p.impl == kF32X3HaloN3 || p.impl == kF32X3HaloN2 || p.impl == kF32X3Halo16 ||
        p.impl == kF32X3Halo16N3) {
      const int nf = (p.impl == kF32X3HaloN3 || p.impl == kF32X3Halo16N3) ? 3 : p.impl == kF32X3HaloN2 ? 2 : 0;
      const int th = (p.impl == kF32X3Halo16 || p.impl == kF32X3Halo16N3) ? 16 : 8;
      if (!x3_halo(p, s, nf, th)) throw std::runtime_error("conv2d_f32: not an x3-halo-eligible conv");
      return;
    }
    if (p.impl == kF32Halo) {
      if (!halo_f32(p, s, true)) throw std::runtime_error("conv2d_f32: not a halo-eligible conv");
      return;
    }
    if (p.impl >= kF32X3) {
      if (p.impl >= kF32X3 + kF32X3Variants || !launch_x3_variant(p, s, M, p.impl - kF32X3))
        throw std::runtime_error("conv2d_f32: unknown x3 variant");
      return;
    }
    if (p.impl >= 10 + kF32Variants || !launch_lds_variant(p, s, M, p.impl - 10)) throw std::runtime_error("conv2d_f32: unknown variant");
    return;
  }
  if (p.impl == 0 && conv_fc_f32(p, s)) return;  // classifier FC: split-K over the 1x1 map
  const int impl = p.impl == 1 ? 1 : p.impl >= 2 ? 2 : f32_conv_family();
  if (impl == 2 && halo_f32(p, s)) return;
  if (impl == 2) {
    // channel tile per workgroup (BN = WN*NF*16) by output-channel count
    if (ncf == 1)
      launch_lds_m<1, 4, 1>(p, s, M);   // BN 16
    else if (ncf == 2)
      launch_lds_m<2, 4, 1>(p, s, M);   // BN 32
    else if (ncf == 3 || ncf == 9)
      launch_lds_m<3, 4, 1>(p, s, M);   // BN 48 (144 = 3 x 48: the stacked detect-head convs)
    else if (ncf == 5)
      launch_lds_m<5, 4, 1>(p, s, M);   // BN 80 (the 80-class branch)
    else if (ncf == 6)
      launch_lds_m<3, 2, 2>(p, s, M);   // BN 96
    else
      launch_lds_m<2, 2, 2>(p, s, M);   // BN 64
    return;
  }
  // channel tile: the widest of 4/3/2 x 16 channels that wastes no more than the narrower ones
  if (ncf % 4 == 0 || ncf > 12)
    launch_f32_wc<4>(p, s, M);
  else if (ncf % 3 == 0)
    launch_f32_wc<3>(p, s, M);
  else if (ncf % 2 == 0)
    launch_f32_wc<2>(p, s, M);
  else if (ncf == 5)
    launch_f32_wc<5>(p, s, M);
  else
    launch_f32_wc<1>(p, s, M);
}

// ---------------------------------------------------------------- depthwise 3x3 (fp32)
// One thread = 4 consecutive channels (one float4) of an R-row x CX-column
// output block; each of the (R-1)*S+3 input rows is loaded once per block as
// (CX-1)*S+3 float4 columns (CX = 2 at stride 1: 24 loads for 8 outputs instead
// of 18 for 4), and the 9 taps' weights stay in registers.  Consecutive
// threads take consecutive channel groups of the same pixel (coalesced NHWC
// rows).  Every output sums bias + taps in (ky, kx) order, as a plain 3x3 loop.
template <int R, int S, int CX>
__global__ __launch_bounds__(256) void dwconv_f32_kernel(const DwParams p) {
  const int B = live_batch(p.B, p.bdev);
  const int cg = p.C >> 2;
  const int strips = (p.Ho + R - 1) / R;
  const int colb = (p.Wo + CX - 1) / CX;
  const int total = B * strips * colb * cg;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int g = tid % cg;
  int t = tid / cg;
  const int ox0 = (t % colb) * CX;
  t /= colb;
  const int st = t % strips;
  const int b = t / strips;
  const int c0 = g * 4;
  const int oy0 = st * R;
  const float* x = (const float*)p.x + (size_t)b * p.H * p.W * p.xs + c0;
  const float* w = (const float*)p.w + c0;
  float4 wt[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wt[k] = *(const float4*)(w + k * p.C);
  const float4 bias = *(const float4*)(p.bias + c0);
  float4 acc[R][CX];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < CX; ++c) acc[r][c] = bias;
  constexpr int NIN = (R - 1) * S + 3, NCOL = (CX - 1) * S + 3;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
#pragma unroll
  for (int ri = 0; ri < NIN; ++ri) {
    const int iy = iy0 + ri;
    if ((unsigned)iy >= (unsigned)p.H) continue;
    const float* row = x + (size_t)iy * p.W * p.xs;
    float4 v[NCOL];
#pragma unroll
    for (int q = 0; q < NCOL; ++q)
      v[q] = load_f4_or_zero(row + (ix0 + q) * p.xs, x, (unsigned)(ix0 + q) < (unsigned)p.W);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int ky = ri - r * S;
      if (ky < 0 || ky > 2) continue;  // compile-time after unrolling
#pragma unroll
      for (int c = 0; c < CX; ++c)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const float4 ww = wt[ky * 3 + kx];
          const float4 vv = v[c * S + kx];
          acc[r][c].x = fmaf(vv.x, ww.x, acc[r][c].x);
          acc[r][c].y = fmaf(vv.y, ww.y, acc[r][c].y);
          acc[r][c].z = fmaf(vv.z, ww.z, acc[r][c].z);
          acc[r][c].w = fmaf(vv.w, ww.w, acc[r][c].w);
        }
    }
  }
  float* y = (float*)p.y + (size_t)b * p.Ho * p.Wo * p.ys + c0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int oy = oy0 + r;
    if (oy >= p.Ho) break;
#pragma unroll
    for (int c = 0; c < CX; ++c) {
      const int ox = ox0 + c;
      if (ox >= p.Wo) break;
      const float4 a = acc[r][c];
      *(float4*)(y + (size_t)(oy * p.Wo + ox) * p.ys) =
          make_float4(apply_act(a.x, p.act), apply_act(a.y, p.act), apply_act(a.z, p.act), apply_act(a.w, p.act));
    }
  }
}

template <int R, int S, int CX>
static void dw_f32_launch(const DwParams& p, hipStream_t s) {
  const long total = (long)p.B * ((p.Ho + R - 1) / R) * ((p.Wo + CX - 1) / CX) * (p.C / 4);
  if (total <= 0) return;
  if (total >= (1L << 31) || (long)p.B * p.H * p.W * p.xs >= (1L << 31))
    throw std::runtime_error("dwconv3x3_f32: too large");
  hipLaunchKernelGGL((dwconv_f32_kernel<R, S, CX>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

static int dw_f32_cols() {  // ARENA_DW_CX=1: the one-column variant (A/B switch)
  static const int v = [] {
    const char* e = std::getenv("ARENA_DW_CX");
    return (e != nullptr && std::atoi(e) == 1) ? 1 : 2;
  }();
  return v;
}

void dwconv3x3_f32(const DwParams& p, hipStream_t s) {
  if (p.C % 4 != 0 || p.xs % 4 != 0 || p.ys % 4 != 0)
    throw std::runtime_error("dwconv3x3_f32: C, xs, ys must be multiples of 4");
  const bool two = dw_f32_cols() == 2;
  if (p.stride == 1)
    two ? dw_f32_launch<4, 1, 2>(p, s) : dw_f32_launch<4, 1, 1>(p, s);
  else if (p.stride == 2)
    two ? dw_f32_launch<2, 2, 2>(p, s) : dw_f32_launch<2, 2, 1>(p, s);
  else
    throw std::runtime_error("dwconv3x3_f32: stride must be 1 or 2");
}

// ---------------------------------------------------------------- SPPF (fp32)
// Cascaded 5x5 stride-1 max pools (== 5/9/13 windows, -inf padding) as two
// separable passes through LDS; one workgroup = one image x 4 channels.
constexpr int SPPF_F32_MAX_PIX = 512;  // YOLO: 20x20 = 400

__global__ __launch_bounds__(256) void sppf_f32_kernel(const SppfParams p) {
  __shared__ float4 in[SPPF_F32_MAX_PIX];
  __shared__ float4 h5[SPPF_F32_MAX_PIX], h9[SPPF_F32_MAX_PIX], h13[SPPF_F32_MAX_PIX];
  const int B = live_batch(p.B, p.bdev);
  const int groups = p.C >> 2;
  const int b = blockIdx.x / groups;
  if (b >= B) return;
  const int c0 = (blockIdx.x - b * groups) * 4;
  const int H = p.H, W = p.W, HW = H * W;
  float* buf = (float*)p.buf + (size_t)b * HW * p.xs;
  for (int i = threadIdx.x; i < HW; i += 256) in[i] = *(const float4*)(buf + (size_t)i * p.xs + c0);
  __syncthreads();
  auto mx = [](float4 a, float4 v) {
    return make_float4(fmaxf(a.x, v.x), fmaxf(a.y, v.y), fmaxf(a.z, v.z), fmaxf(a.w, v.w));
  };
  const float4 ninf = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int i = threadIdx.x; i < HW; i += 256) {
    const int y = i / W, xx = i - y * W;
    float4 m5 = ninf, m9 = ninf, m13 = ninf;
#pragma unroll
    for (int dx = -6; dx <= 6; ++dx) {
      const int ix = xx + dx;
      if ((unsigned)ix >= (unsigned)W) continue;
      const float4 v = in[y * W + ix];
      const int a = dx < 0 ? -dx : dx;
      m13 = mx(m13, v);
      if (a <= 4) m9 = mx(m9, v);
      if (a <= 2) m5 = mx(m5, v);
    }
    h5[i] = m5;
    h9[i] = m9;
    h13[i] = m13;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HW; i += 256) {
    const int y = i / W, xx = i - y * W;
    float4 m5 = ninf, m9 = ninf, m13 = ninf;
#pragma unroll
    for (int dy = -6; dy <= 6; ++dy) {
      const int iy = y + dy;
      if ((unsigned)iy >= (unsigned)H) continue;
      const int j = iy * W + xx;
      const int a = dy < 0 ? -dy : dy;
      m13 = mx(m13, h13[j]);
      if (a <= 4) m9 = mx(m9, h9[j]);
      if (a <= 2) m5 = mx(m5, h5[j]);
    }
    float* o = buf + (size_t)i * p.xs + c0;
    *(float4*)(o + p.C) = m5;
    *(float4*)(o + 2 * p.C) = m9;
    *(float4*)(o + 3 * p.C) = m13;
  }
}

void sppf_pool_f32(const SppfParams& p, hipStream_t s) {
  if (p.C % 4 != 0 || p.xs < 4 * p.C || p.xs % 4 != 0 || p.H * p.W > SPPF_F32_MAX_PIX)
    throw std::runtime_error("sppf_pool_f32: bad geometry (C % 4, xs >= 4C, H*W <= 512)");
  if (p.B <= 0) return;
  hipLaunchKernelGGL(sppf_f32_kernel, dim3((unsigned)(p.B * (p.C / 4))), dim3(256), 0, s, p);
}

}  // namespace arena
