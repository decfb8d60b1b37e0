// Fused inverted residual: one output tile per WAVE (no block barriers).
//
// The block-cooperative kernel (ir_block.hip) splits each tile's expand /
// depthwise / project phases across 4 waves with three __syncthreads per
// 32-channel hidden chunk; on the 112..14 px stride-1 blocks those barriers
// and the short per-chunk phases left the CUs latency-bound.  Here each wave
// owns a whole TH x TW tile: it stages its input halo tile in its own LDS
// region and walks the hidden chunks alone — expand (MFMA, weights as direct
// 16-B global loads), depthwise (tap pairs via v_perm + v_dot2c_f32_bf16,
// weights in registers), project (MFMA, accumulators in VGPRs).  LDS traffic
// between phases is ordered by the wave's own instruction stream.
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace arena {

__device__ __forceinline__ int wswz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}
__device__ __forceinline__ float relu6w(float v) { return relu6f(v); }
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have completed
  __builtin_amdgcn_wave_barrier();
}

#ifndef IRW_XREG_S1
#define IRW_XREG_S1 1
#endif

template <int S, int TH, int TW, int MP, int NS, bool EXPAND>
__global__ __launch_bounds__(256) void ir_wave_kernel(const IrParams p) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int PIN = PH * PW, PIN_PAD = (PIN + 15) / 16 * 16;
  constexpr int POUT = TH * TW, POUT_PAD = (POUT + 15) / 16 * 16;
  constexpr int NE = PIN_PAD / 16, NP = POUT_PAD / 16;
  // Stride-2 expand blocks (one input slab, no residual): each lane keeps its expand B operands (halo
  // pixel j*16+row, channels kq*8..+8) in NE VGPR quads instead of staging the tile in LDS; LDS per
  // workgroup 53 -> 28 KB, so occupancy is no longer LDS-bound at 3 waves per SIMD
  constexpr bool XREG = NS == 1 && EXPAND && (S == 2 || IRW_XREG_S1);
  constexpr int XB = XREG ? 0 : NS * PIN_PAD * 64, EB = EXPAND ? PIN_PAD * 64 : 0, DB = POUT_PAD * 64;
  constexpr int WAVE_BYTES = XB + EB + DB;
  // unroll depth per shape (measured: full unroll is best for 7x7 tiles; the 8x8 tile
  // needs the lighter unroll to stay at 2 waves/SIMD without AGPR spills)
  constexpr int E_UNROLL = TH == 8 && !XREG ? 2 : NE;  // xr[j] needs static indices
  constexpr int D_UNROLL = TH == 8 ? 1 : POUT_PAD / 16;
  extern __shared__ __align__(16) uint8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kq = lane >> 4;
  uint8_t* Xs = lds + wave * WAVE_BYTES;
  uint8_t* Es = Xs + XB;
  uint8_t* Ds = Es + EB;

  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles = tiles_x * tiles_y;
  const int gt = blockIdx.x * 4 + wave;  // global tile index
  const int b = gt / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;  // whole wave exits; no block barrier follows
  const int t = gt - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const bf16* xb = (const bf16*)p.x + (size_t)b * p.H * p.W * p.x_cs;

  // ---- input halo tile -> this wave's LDS (zero outside the image / past inp), or -> xr (XREG)
  bf16x8 xr[XREG ? NE : 1];
  if constexpr (XREG) {
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int pix = j * 16 + row;
      const int py = pix / PW, px = pix - py * PW;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = pix < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && kq * 8 < p.inp;
      xr[j] = __builtin_bit_cast(bf16x8, load16_or_zero(xb + ((size_t)iy * p.W + ix) * p.x_cs + kq * 8, xb, ok));
    }
  }
  constexpr int CPR = NS * 4;
  for (int i = lane; !XREG && i < PIN_PAD * CPR; i += 64) {
    const int pix = i / CPR, c = i - pix * CPR;  // CPR is a compile-time power of two
    const int py = pix / PW, px = pix - py * PW;
    const int iy = iy0 + py, ix = ix0 + px;
    const bool ok = pix < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && c * 8 < p.inp;
    const uint4 v = load16_or_zero(xb + ((size_t)iy * p.W + ix) * p.x_cs + c * 8, xb, ok);
    *(uint4*)(Xs + (c >> 2) * PIN_PAD * 64 + wswz(pix, c & 3)) = v;
  }
  wave_lds_sync();

  // chunk-invariant: which expand rows (halo pixels) are inside the image
  unsigned e_inb = 0;  // bit j: halo pixel j*16+row inside the image
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int pix = j * 16 + row;
    const int py = pix / PW, px = pix - py * PW;
    if (pix < PIN && (unsigned)(iy0 + py) < (unsigned)p.H && (unsigned)(ix0 + px) < (unsigned)p.W) e_inb |= 1u << j;
  }

  f32x4 acc[NP][MP];
#pragma unroll
  for (int q = 0; q < NP; ++q)
#pragma unroll
    for (int m = 0; m < MP; ++m) acc[q][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* we = (const bf16*)p.we;
  const bf16* wd = (const bf16*)p.wd;
  const bf16* wp = (const bf16*)p.wp;
  const int dc = lane & 3;  // this lane's 8-channel group in the depthwise phase
  const int nchunks = p.hid_pad >> 5;
  for (int h = 0; h < nchunks; ++h) {
    const int h0 = h * 32;
    // depthwise weights of this lane's channels: tap pairs (2p, 2p+1) as bf16x2, tap 8 fp32
    unsigned wpair[4][8];
    float w8[8], bd[8];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const uint4 a = *(const uint4*)(wd + (2 * pp) * p.hid_pad + h0 + dc * 8);
      const uint4 c2 = *(const uint4*)(wd + (2 * pp + 1) * p.hid_pad + h0 + dc * 8);
      const unsigned av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c2.x, c2.y, c2.z, c2.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wpair[pp][2 * j] = __builtin_amdgcn_perm(cv[j], av[j], 0x05040100u);
        wpair[pp][2 * j + 1] = __builtin_amdgcn_perm(cv[j], av[j], 0x07060302u);
      }
    }
    unpack8(*(const uint4*)(wd + 8 * p.hid_pad + h0 + dc * 8), w8);
    {
      const float4 b0 = *(const float4*)(p.bd + h0 + dc * 8);
      const float4 b1 = *(const float4*)(p.bd + h0 + dc * 8 + 4);
      bd[0] = b0.x; bd[1] = b0.y; bd[2] = b0.z; bd[3] = b0.w;
      bd[4] = b1.x; bd[5] = b1.y; bd[6] = b1.z; bd[7] = b1.w;
    }
    // project weights (A operand): rows m*16+row, columns h0 + kq*8
    bf16x8 wpa[MP];
#pragma unroll
    for (int m = 0; m < MP; ++m) wpa[m] = *(const bf16x8*)(wp + (size_t)(m * 16 + row) * p.hid_pad + h0 + kq * 8);

    const uint8_t* Esrc;
    if constexpr (EXPAND) {
      bf16x8 wa0[NS], wa1[NS];
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        wa0[sl] = *(const bf16x8*)(we + (size_t)(h0 + row) * p.inp_pad + sl * 32 + kq * 8);
        wa1[sl] = *(const bf16x8*)(we + (size_t)(h0 + 16 + row) * p.inp_pad + sl * 32 + kq * 8);
      }
      const float4 be0 = *(const float4*)(p.be + h0 + kq * 4);
      const float4 be1 = *(const float4*)(p.be + h0 + 16 + kq * 4);
#pragma unroll E_UNROLL
      for (int j = 0; j < NE; ++j) {
        f32x4 e0 = {be0.x, be0.y, be0.z, be0.w}, e1 = {be1.x, be1.y, be1.z, be1.w};  // bias folded into init
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
          const bf16x8 bv = XREG ? xr[j] : *(const bf16x8*)(Xs + sl * PIN_PAD * 64 + wswz(j * 16 + row, kq));
          e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa0[sl], bv, e0, 0, 0, 0);
          e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa1[sl], bv, e1, 0, 0, 0);
        }
        const int pix = j * 16 + row;
        float v0[4] = {relu6w(e0[0]), relu6w(e0[1]), relu6w(e0[2]), relu6w(e0[3])};
        float v1[4] = {relu6w(e1[0]), relu6w(e1[1]), relu6w(e1[2]), relu6w(e1[3])};
        if (!((e_inb >> j) & 1u)) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v0[k] = v1[k] = 0.f;
        }
        const int h4 = kq * 4;  // hidden rows kq*4..+3 (tile 0) and 16+kq*4.. (tile 1)
        *(uint2*)(Es + wswz(pix, h4 >> 3) + (h4 & 7) * 2) = pack4(v0);
        *(uint2*)(Es + wswz(pix, (16 + h4) >> 3) + (h4 & 7) * 2) = pack4(v1);
      }
      wave_lds_sync();
      Esrc = Es;
    } else {
      Esrc = Xs + h * PIN_PAD * 64;
    }

    // depthwise: this lane handles pixels q = (lane >> 2) + 16 k, channel group dc
#pragma unroll D_UNROLL
    for (int k = 0; k < POUT_PAD / 16; ++k) {
      const int q = (lane >> 2) + 16 * k;
      uint4 outv = {0u, 0u, 0u, 0u};
      if (q < POUT) {
        const int oy = q / TW, ox = q - oy * TW;
        float a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = bd[i];
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int t0 = 2 * pp, t1 = 2 * pp + 1;
          const uint4 e0 = *(const uint4*)(Esrc + wswz((oy * S + t0 / 3) * PW + ox * S + t0 % 3, dc));
          const uint4 e1 = *(const uint4*)(Esrc + wswz((oy * S + t1 / 3) * PW + ox * S + t1 % 3, dc));
          const unsigned x0[4] = {e0.x, e0.y, e0.z, e0.w}, x1[4] = {e1.x, e1.y, e1.z, e1.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const unsigned lo = __builtin_amdgcn_perm(x1[j], x0[j], 0x05040100u);
            const unsigned hi = __builtin_amdgcn_perm(x1[j], x0[j], 0x07060302u);
            a[2 * j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, lo),
                                                       __builtin_bit_cast(bf16x2, wpair[pp][2 * j]), a[2 * j], false);
            a[2 * j + 1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hi),
                                                           __builtin_bit_cast(bf16x2, wpair[pp][2 * j + 1]),
                                                           a[2 * j + 1], false);
          }
        }
        float e8[8];
        unpack8(*(const uint4*)(Esrc + wswz((oy * S + 2) * PW + ox * S + 2, dc)), e8);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = relu6w(fmaf(e8[i], w8[i], a[i]));
        outv = pack8(a);
      }
      *(uint4*)(Ds + wswz(q, dc)) = outv;
    }
    wave_lds_sync();

    // project: acc[pixel tile q][oup tile m] += Wp[m][chunk] . D[chunk][q]
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const bf16x8 bv = *(const bf16x8*)(Ds + wswz(q * 16 + row, kq));
#pragma unroll
      for (int m = 0; m < MP; ++m) acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wpa[m], bv, acc[q][m], 0, 0, 0);
    }
    // E and D are rewritten next chunk: the MFMA operand reads above are issued
    // (and ordered in the LDS queue) before the next chunk's writes.
  }

  // ---- epilogue: bias (+ residual from the staged input tile) -> NHWC bf16
  bf16* yb = (bf16*)p.y + (size_t)b * p.Ho * p.Wo * p.y_cs;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int pix = q * 16 + row;
    if (pix >= POUT) continue;
    const int ly = pix / TW, lx = pix - (pix / TW) * TW;
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy >= p.Ho || ox >= p.Wo) continue;
    bf16* yp = yb + ((size_t)oy * p.Wo + ox) * p.y_cs;
    const int rpix = (ly + 1) * PW + lx + 1;
#pragma unroll
    for (int m = 0; m < MP; ++m) {
      const int oc = m * 16 + kq * 4;
      if (oc >= p.oup) continue;
      const float4 bb = *(const float4*)(p.bp + oc);
      float v[4] = {acc[q][m][0] + bb.x, acc[q][m][1] + bb.y, acc[q][m][2] + bb.z, acc[q][m][3] + bb.w};
      if (S == 1 && p.res) {
        float r[4];
        if constexpr (XREG)  // the tile was never staged: residual straight from global (L2-hot)
          unpack4(*(const uint2*)(xb + ((size_t)oy * p.W + ox) * p.x_cs + oc), r);
        else
          unpack4(*(const uint2*)(Xs + (oc >> 5) * PIN_PAD * 64 + wswz(rpix, (oc & 31) >> 3) + (oc & 7) * 2), r);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += r[k];
      }
      *(uint2*)(yp + oc) = pack4(v);
    }
  }
}

template <int S, int TH, int TW, int MP, int NS, bool EXPAND>
static void irw_launch(const IrParams& p, hipStream_t s) {
  constexpr int PIN_PAD = (((TH - 1) * S + 3) * ((TW - 1) * S + 3) + 15) / 16 * 16, POUT_PAD = (TH * TW + 15) / 16 * 16;
  constexpr bool XREG = NS == 1 && EXPAND && (S == 2 || IRW_XREG_S1);
  constexpr size_t lds = 4 * (size_t)((XREG ? 0 : NS * PIN_PAD * 64) + (EXPAND ? PIN_PAD * 64 : 0) + POUT_PAD * 64);
  static_assert(lds <= 160 * 1024, "LDS");
  const long tiles = (long)((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B;
  if (tiles <= 0) return;
  hipLaunchKernelGGL((ir_wave_kernel<S, TH, TW, MP, NS, EXPAND>), dim3((unsigned)((tiles + 3) / 4)), dim3(256), lds, s,
                     p);
}

// Measured (profiles/r1_irwave_ops.md): the wave kernel wins on the 56x56 and 28x28
// expand blocks; block 1 (no expand) and the 14x14 blocks stay block-cooperative.
// Stride 2 uses 4x4 output tiles (9x9 halo).  Single-slab expand blocks keep the halo in VGPRs
// (IRW_XREG_S1=0 at build time restores LDS staging for stride 1: profiles/r1_irwave_xreg_ops.md).
#define ARENA_IRW_CONFIGS(X) \
  X(1, 8, 8, 2, 1, true)     \
  X(1, 7, 7, 2, 1, true)     \
  X(2, 4, 4, 2, 1, true)

void ir_wave_prepare() {
#define X(S, TH, TW, MP, NS, E)                                                                       \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_wave_kernel<S, TH, TW, MP, NS, E>,                 \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ARENA_IRW_CONFIGS(X)
#undef X
}

// Stride-1 blocks with a supported (tile, oup tiles, input slabs) shape; false otherwise.
static const bool g_irw_s2 = [] {
  const char* e = std::getenv("ARENA_IRW_S2");
  return e ? std::atoi(e) != 0 : true;
}();

bool ir_block_wave(const IrParams& p, int tile, hipStream_t s) {
  if (p.stride == 2) {
    if (!g_irw_s2 || p.Ho % 4 || p.Wo % 4) return false;
    tile = 4;
  } else if (p.stride != 1) {
    return false;
  }
  const int MP = p.oup_pad / 16, NS = p.inp_pad / 32;
  const bool E = p.expand != 0;
#define X(S_, TH_, TW_, MP_, NS_, E_)                                              \
  if (p.stride == S_ && tile == TH_ && MP == MP_ && NS == NS_ && E == E_) {        \
    irw_launch<S_, TH_, TW_, MP_, NS_, E_>(p, s);                                  \
    return true;                                                                   \
  }
  ARENA_IRW_CONFIGS(X)
#undef X
  return false;
}

}  // namespace arena
