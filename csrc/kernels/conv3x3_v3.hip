// 3x3 convolution (stride 1 or 2, Cin % 16 == 0) — halo-tile kernel, v3.
//
// Block = 4 waves; output tile = (4*MF) rows x 16 columns of one image, BN =
// NF*16 output channels.  Per 32-channel input slab the block stages
//   * the input halo tile  [(4MF-1)S+3 rows][ICP pitch][32 ch]  (ICP = 32 / 48,
//     a multiple of 16 pixels: the XOR swizzle term of a pixel then depends
//     only on its column, so every fragment address is a per-lane base plus a
//     compile-time immediate), and
//   * the weight slice     [9 taps][BN][32 ch]
// and runs 9 * NF * MF MFMAs per wave out of LDS.  The next slab's input and
// weights are fetched into registers before the current slab is multiplied,
// so global latency hides behind MFMA; staging addresses are computed once.
//
// Counters on v2 (same tiling, addresses recomputed per access, no prefetch)
// showed ~11 VALU instructions per MFMA: address/index math, not MFMA, set
// the pace.  v3 cuts that to a few per slab.
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace arena {

template <int S, int MF, int NF>
struct V3Geom {
  static constexpr int TH = 4 * MF;
  static constexpr int BN = NF * 16;
  static constexpr int IR = (TH - 1) * S + 3;
  static constexpr int IC = 15 * S + 3;
  static constexpr int ICP = S == 1 ? 32 : 48;
  static constexpr int IN_BYTES = IR * ICP * 64;
  static constexpr int W_BYTES = 9 * BN * 64;
  static constexpr int IN_PIX = IR * IC;
  static constexpr int IN_IT = (IN_PIX + 63) / 64;  // staging iterations (64 pixels x 4 chunks each)
  static constexpr int W_IT = (9 * BN + 63) / 64;
};

__device__ __forceinline__ int v3swz(int pix, int chunk) {
  return (chunk ^ ((0x78 >> (((pix >> 2) & 3) * 2)) & 3)) << 4;
}

// PWNF > 0: a pointwise conv (PWNF*16 -> PWNF*16 channels, K = PWNF*16 padded to 32) runs on the
// activated 3x3 tile in the epilogue (Detect head: 3x3 -> 1x1 without the intermediate round trip).
template <int S, int MF, int NF, int PWNF = 0>
__global__ __launch_bounds__(256) void conv3x3_v3_kernel(const ConvParams p) {
  using G = V3Geom<S, MF, NF>;
  constexpr int TH = G::TH, BN = G::BN, IC = G::IC, ICP = G::ICP;
  __shared__ __align__(16) uint8_t sin[G::IN_BYTES];
  __shared__ __align__(16) uint8_t sw[G::W_BYTES];

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

  // ---- staging maps (computed once): thread -> chunk c = tid & 3, 64 pixels / rows per iteration
  const int sc = tid & 3, sq = tid >> 2;
  int in_goff[G::IN_IT];   // element offset into x of (pixel, chunk), -1 = zero / unused
  int in_loff[G::IN_IT];   // LDS byte offset
#pragma unroll
  for (int i = 0; i < G::IN_IT; ++i) {
    const int pix = sq + 64 * i;
    const int r = pix / IC, c = pix - r * IC;
    const int iy = iy_base + r, ix = ix_base + c;
    const bool ok = pix < G::IN_PIX && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    in_goff[i] = ok ? (iy * p.W + ix) * p.xs + sc * 8 : -1;
    const int lp = r * ICP + c;
    in_loff[i] = pix < G::IN_PIX ? lp * 64 + v3swz(lp, sc) : -1;
  }
  int w_goff[G::W_IT], w_loff[G::W_IT];
#pragma unroll
  for (int i = 0; i < G::W_IT; ++i) {
    const int R = sq + 64 * i;  // R = tap * BN + n
    const int tap = R / BN, n = R - tap * BN;
    int co = cout0 + n;
    co = co < p.Cout_pad ? co : p.Cout_pad - 1;
    w_goff[i] = R < 9 * BN ? co * p.Kpad + tap * Cin + sc * 8 : -1;
    w_loff[i] = R < 9 * BN ? R * 64 + v3swz(n, sc) : -1;  // masked chunks still store zeros
  }

  uint4 rin[G::IN_IT], rw[G::W_IT];
  auto fetch = [&](int c0) {
    const bool cv = c0 + sc * 8 < Cin;  // this thread's 8-channel chunk exists in slab c0 (Cin % 32 == 16: half slab)
#pragma unroll
    for (int i = 0; i < G::IN_IT; ++i) rin[i] = load16_or_zero(x + in_goff[i] + c0, x, cv && in_goff[i] >= 0);
#pragma unroll
    for (int i = 0; i < G::W_IT; ++i) rw[i] = load16_or_zero(w + w_goff[i] + c0, w, cv && w_goff[i] >= 0);
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < G::IN_IT; ++i)
      if (in_loff[i] >= 0) *(uint4*)(sin + in_loff[i]) = rin[i];
#pragma unroll
    for (int i = 0; i < G::W_IT; ++i)
      if (w_loff[i] >= 0) *(uint4*)(sw + w_loff[i]) = rw[i];
  };

  // ---- fragment read bases: B (input) per kw, A (weights) per lane
  int bbase[3];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int lp = (wave * MF * S) * ICP + col * S + kw;
    bbase[kw] = lp * 64 + v3swz(col * S + kw, kq);
  }
  const int abase = col * 64 + v3swz(col, kq);

  f32x4 acc[NF][MF];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int f = 0; f < MF; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  fetch(0);
  for (int c0 = 0; c0 < Cin; c0 += 32) {
    __syncthreads();  // previous slab fully consumed
    stash();
    __syncthreads();
    if (c0 + 32 < Cin) fetch(c0 + 32);  // next slab in flight during the MFMAs
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        bf16x8 a[NF], bb[MF];
#pragma unroll
        for (int j = 0; j < NF; ++j)
          a[j] = *(const bf16x8*)(sw + abase + ((kh * 3 + kw) * BN + j * 16) * 64);
#pragma unroll
        for (int f = 0; f < MF; ++f) bb[f] = *(const bf16x8*)(sin + bbase[kw] + (f * S + kh) * ICP * 64);
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < MF; ++f)
            acc[j][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bb[f], acc[j][f], 0, 0, 0);
      }
    }
  }

  if constexpr (PWNF > 0) {
    // ---- fused pointwise: H = act(acc + bias) -> LDS [slab][pixel][32 ch] (swizzled 64-B rows, reusing the
    // weight area), then pw_y = W2 . H + b2 with this wave's own pixels as the B operand.
    static_assert(NF == PWNF, "the 3x3 tile must cover every input channel of the pointwise conv");
    constexpr int NPX = TH * 16, SL2 = (PWNF * 16 + 31) / 32;
    static_assert(SL2 * NPX * 64 <= G::W_BYTES, "H tile must fit the weight area");
    __syncthreads();  // every wave is done with the last slab's weights
    for (int i = tid; i < SL2 * NPX * 4; i += 256) *(uint4*)(sw + i * 16) = uint4{0u, 0u, 0u, 0u};
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int cb = j * 16 + kq * 4;
      const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int P = (wave * MF + f) * 16 + col;
        float v[4] = {acc[j][f][0] + bias.x, acc[j][f][1] + bias.y, acc[j][f][2] + bias.z, acc[j][f][3] + bias.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
        *(uint2*)(sw + (cb >> 5) * NPX * 64 + P * 64 + ((((cb & 31) >> 3) ^ ((0x78 >> (((P >> 2) & 3) * 2)) & 3)) << 4) +
                  (cb & 7) * 2) = pack4(v);
      }
    }
    __syncthreads();
    const bf16* __restrict__ w2 = (const bf16*)p.pw_w;
    f32x4 acc2[PWNF][MF];
#pragma unroll
    for (int n = 0; n < PWNF; ++n)
#pragma unroll
      for (int f = 0; f < MF; ++f) acc2[n][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < SL2; ++sl) {
      bf16x8 hb[MF];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int P = (wave * MF + f) * 16 + col;
        hb[f] = *(const bf16x8*)(sw + sl * NPX * 64 + P * 64 + ((kq ^ ((0x78 >> (((P >> 2) & 3) * 2)) & 3)) << 4));
      }
#pragma unroll
      for (int n = 0; n < PWNF; ++n) {
        const bf16x8 a = *(const bf16x8*)(w2 + (size_t)(n * 16 + col) * p.pw_kpad + sl * 32 + kq * 8);
#pragma unroll
        for (int f = 0; f < MF; ++f) acc2[n][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, hb[f], acc2[n][f], 0, 0, 0);
      }
    }
    const int oxp = tx0 + col;
#pragma unroll
    for (int n = 0; n < PWNF; ++n) {
      const int oc = n * 16 + kq * 4;
      if (oc >= p.pw_cout) continue;
      const float4 b2 = *(const float4*)(p.pw_bias + oc);
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int oy = ty0 + wave * MF + f;
        if (oy >= p.Ho || oxp >= p.Wo) continue;
        const size_t pix = ((size_t)b * p.Ho + oy) * p.Wo + oxp;
        float v[4] = {acc2[n][f][0] + b2.x, acc2[n][f][1] + b2.y, acc2[n][f][2] + b2.z, acc2[n][f][3] + b2.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.pw_act);
        *(uint2*)((bf16*)p.pw_y + pix * p.pw_ys + oc) = pack4(v);
      }
    }
    return;
  }

  // ---- epilogue
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
static void v3_launch(const ConvParams& p, hipStream_t s) {
  constexpr int TH = 4 * MF;
  const int tiles = ((p.Wo + 15) / 16) * ((p.Ho + TH - 1) / TH);
  dim3 grid(p.B * tiles, (p.Cout_pad + NF * 16 - 1) / (NF * 16));
  if (p.pw_w != nullptr) {
    if constexpr (S == 1 && MF <= 2 && (NF == 4 || NF == 5)) {
      if (grid.y != 1 || p.pw_cout > NF * 16 || p.pw_kpad != (NF * 16 + 31) / 32 * 32 || p.res != nullptr ||
          p.y2 != nullptr || p.f32out)
        throw std::runtime_error("conv3x3_v3: unsupported fused pointwise geometry");
      hipLaunchKernelGGL((conv3x3_v3_kernel<S, MF, NF, NF>), grid, dim3(256), 0, s, p);
      return;
    }
    throw std::runtime_error("conv3x3_v3: fused pointwise needs stride 1 and 64 or 80 channels");
  }
  hipLaunchKernelGGL((conv3x3_v3_kernel<S, MF, NF>), grid, dim3(256), 0, s, p);
}

static int v3_max_mf() {
  static const int v = [] {
    const char* e = std::getenv("ARENA_V3_MF");
    return e != nullptr ? std::atoi(e) : 2;
  }();
  return v;
}

template <int S, int NF>
static void v3_nf(const ConvParams& p, hipStream_t s) {
  const long ngrp = (p.Cout_pad + NF * 16 - 1) / (NF * 16);
  const long blocks2 = (long)p.B * ((p.Wo + 15) / 16) * ((p.Ho + 7) / 8) * ngrp;
  const long blocks4 = (long)p.B * ((p.Wo + 15) / 16) * ((p.Ho + 15) / 16) * ngrp;
  if constexpr (S == 1) {
    // 4 output rows per wave: ~2x the MFMAs per staged slab, fewer halo re-reads (LDS 36 KB input tile)
    if (v3_max_mf() >= 4 && p.pw_w == nullptr && p.Ho >= 32 && blocks4 >= 512) {
      v3_launch<S, 4, NF>(p, s);
      return;
    }
    if (p.Ho >= 16 && blocks2 >= 512) {
      v3_launch<S, 2, NF>(p, s);
      return;
    }
  }
  v3_launch<S, 1, NF>(p, s);
}

bool conv3x3_v3(const ConvParams& p, hipStream_t s) {
  // Cin % 32 == 16 (s2d stems, YOLO's first C3, the 80-class detect branch) ends in a half-empty slab
  if (!(p.KH == 3 && p.KW == 3 && (p.stride == 1 || p.stride == 2) && p.Cin % 16 == 0 &&
        !p.f32out && p.Kpad >= 9 * p.Cin))
    return false;
  if ((long)p.H * p.W * p.xs >= (1L << 31)) return false;  // 32-bit staging offsets
  const int ncf = p.Cout_pad / 16;
  const int nf = ncf % 4 == 0 ? 4 : ncf % 3 == 0 ? 3 : ncf % 5 == 0 ? 5 : ncf % 2 == 0 ? 2 : 1;
#define V3(S_, NF_) if (p.stride == S_ && nf == NF_) { v3_nf<S_, NF_>(p, s); return true; }
  V3(1, 1) V3(1, 2) V3(1, 3) V3(1, 4) V3(1, 5)
  V3(2, 1) V3(2, 2) V3(2, 3) V3(2, 4) V3(2, 5)
#undef V3
  return false;
}

}  // namespace arena
