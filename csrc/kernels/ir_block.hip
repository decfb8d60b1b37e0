// Fused MobileNetV2 inverted-residual block on CDNA4 matrix cores.
//
// Reference computation (ONNX Runtime, per crop, architectures/monolithic/
// app/inference.py:196 running torchvision's mobilenet_v2): Conv1x1+BN+Clip
// (expand) -> depthwise Conv3x3+BN+Clip -> Conv1x1+BN (project) [-> Add].
// Unfused, the expanded tensor is the largest activation of the network
// (112x112x96 per crop in block 2) and is written to and re-read from HBM
// twice.  Here one workgroup owns a TH x TW output tile of one crop:
//
//   X tile (input + 1-px halo, stride-aware) ........ LDS, loaded once
//   for each chunk of 32 hidden channels:
//     E = relu6(X . We^T + be)   MFMA 16x16x32 ...... LDS (zero outside the image:
//                                                      the depthwise pads the *expanded* map)
//     D = relu6(dw3x3_S(E) + bd)  VALU, 8 ch / lane .. LDS
//     acc += Wp[:, chunk] . D     MFMA, accumulators stay in VGPRs
//   y = acc + bp (+ x)  -> NHWC bf16, 8-byte stores
//
// All LDS images use 64-byte rows (32 bf16 channels) whose 16-byte chunks are
// XOR-swizzled with g[(row>>2)&3], g = {0,2,3,1}: for the 16x16x32 operand
// read (lane l: row l&15, chunk l>>4) every ds_read_b128 lane group
// ({0-3,12-15,20-27}, ...) then touches 16 distinct 16-byte bank slots.
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace arena {

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}

__device__ __forceinline__ float relu6(float v) { return relu6f(v); }

// i / d for small non-negative ints via a float reciprocal (1/d rounds up for every
// divisor used here, and i * 1e-7 relative error stays far below 1/d for i < 2^20).
__device__ __forceinline__ int fdiv(int i, float inv_d) { return (int)((float)i * inv_d); }

template <int S, int TH, int TW, int MP, bool EXPAND>
__global__ __launch_bounds__(256) void ir_block_kernel(const IrParams p) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int PIN = PH * PW, PIN_PAD = (PIN + 15) / 16 * 16;
  constexpr int POUT = TH * TW, POUT_PAD = (POUT + 15) / 16 * 16;
  constexpr int NE = PIN_PAD / 16, NP = POUT_PAD / 16, NPW = (NP + 3) / 4;
  constexpr int WP_PER_T = (MP * 64 + 255) / 256;  // 16-B pieces of a Wp chunk per thread
  constexpr int WE_PER_T = 3;                       // inp_pad <= 192 -> 32*24/256
  constexpr int WD_BYTES = 768;  // per chunk: tap pairs [4][32] bf16x2, tap 8 [32] fp32, bias [32] fp32
  extern __shared__ __align__(16) uint8_t lds[];
  const int nslab = p.inp_pad >> 5;
  const int cpr = p.inp_pad >> 3;
  uint8_t* Xs = lds;                                    // [nslab][PIN_PAD] rows
  uint8_t* Es = Xs + nslab * PIN_PAD * 64;              // [PIN_PAD] rows (EXPAND)
  uint8_t* Ds = Es + (EXPAND ? PIN_PAD * 64 : 0);       // [POUT_PAD] rows
  uint8_t* Wps = Ds + POUT_PAD * 64;                    // 2 x [MP*16] rows
  uint8_t* Wds = Wps + 2 * MP * 16 * 64;                // 2 x dw taps (packed pairs) + bias
  uint8_t* Wes = Wds + 2 * WD_BYTES;                    // 2 x [nslab][32] rows (EXPAND)
  const int we_buf = nslab * 32 * 64;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles = tiles_x * tiles_y;
  const int b = blockIdx.x / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = blockIdx.x - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const bf16* xb = (const bf16*)p.x + (size_t)b * p.H * p.W * p.x_cs;
  const bf16* wp = (const bf16*)p.wp;
  const bf16* we = (const bf16*)p.we;
  const bf16* wd = (const bf16*)p.wd;

  // Per-chunk weights (Wp columns, We rows, dw taps + bias) are prefetched into
  // registers one chunk ahead and written to the idle LDS buffer after the
  // current chunk's last read of it, so their global latency hides behind MFMA.
  uint4 rwp[WP_PER_T], rwe[WE_PER_T], rwd;
  const float inv_cpr_w = 1.0f / (float)cpr;
  auto fetch = [&](int h0) {
#pragma unroll
    for (int k = 0; k < WP_PER_T; ++k) {
      const int i = tid + k * 256;
      rwp[k] = load16_or_zero(wp + (size_t)(i >> 2) * p.hid_pad + h0 + (i & 3) * 8, wp, i < MP * 64);
    }
    if constexpr (EXPAND) {
#pragma unroll
      for (int k = 0; k < WE_PER_T; ++k) {
        const int i = tid + k * 256;
        const int r = fdiv(i, inv_cpr_w), c = i - r * cpr;
        rwe[k] = load16_or_zero(we + (size_t)(h0 + r) * p.inp_pad + c * 8, we, i < 32 * cpr);
      }
    }
    const void* pd = tid < 36 ? (const void*)(wd + (tid >> 2) * p.hid_pad + h0 + (tid & 3) * 8)
                              : (const void*)(p.bd + h0 + (tid - 36) * 4);
    rwd = load16_or_zero(pd, wd, tid < 44);
  };
  auto stash = [&](int buf) {
    uint8_t* wps = Wps + buf * MP * 16 * 64;
#pragma unroll
    for (int k = 0; k < WP_PER_T; ++k) {
      const int i = tid + k * 256;
      if (i < MP * 64) *(uint4*)(wps + swz(i >> 2, i & 3)) = rwp[k];
    }
    if constexpr (EXPAND) {
      uint8_t* wes = Wes + buf * we_buf;
#pragma unroll
      for (int k = 0; k < WE_PER_T; ++k) {
        const int i = tid + k * 256;
        if (i < 32 * cpr) {
          const int r = fdiv(i, inv_cpr_w), c = i - r * cpr;
          *(uint4*)(wes + (c >> 2) * 32 * 64 + swz(r, c & 3)) = rwe[k];
        }
      }
    }
    // Depthwise taps are stored as bf16 PAIRS (tap 2p, tap 2p+1) per channel, the layout
    // v_dot2c_f32_bf16 consumes: thread tid (< 36) holds tap tid>>2, channels (tid&3)*8..+8;
    // its partner tap sits 4 lanes up in the same wave.  Tap 8 is kept as fp32.
    uint8_t* wdl = Wds + buf * WD_BYTES;
    if (tid < 64) {
      uint4 nb;
      nb.x = __shfl_down(rwd.x, 4, 64);
      nb.y = __shfl_down(rwd.y, 4, 64);
      nb.z = __shfl_down(rwd.z, 4, 64);
      nb.w = __shfl_down(rwd.w, 4, 64);
      const int tap = tid >> 2, c = tid & 3;
      if (tid < 32 && (tap & 1) == 0) {
        const unsigned a[4] = {rwd.x, rwd.y, rwd.z, rwd.w}, b2[4] = {nb.x, nb.y, nb.z, nb.w};
        unsigned q[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          q[2 * j] = __builtin_amdgcn_perm(b2[j], a[j], 0x05040100u);      // (ch 2j: tap, tap+1)
          q[2 * j + 1] = __builtin_amdgcn_perm(b2[j], a[j], 0x07060302u);  // (ch 2j+1: tap, tap+1)
        }
        uint4* dst = (uint4*)(wdl + (tap >> 1) * 128 + c * 32);
        dst[0] = make_uint4(q[0], q[1], q[2], q[3]);
        dst[1] = make_uint4(q[4], q[5], q[6], q[7]);
      } else if (tap == 8) {
        float f[8];
        unpack8(rwd, f);
        *(float4*)(wdl + 512 + c * 32) = make_float4(f[0], f[1], f[2], f[3]);
        *(float4*)(wdl + 512 + c * 32 + 16) = make_float4(f[4], f[5], f[6], f[7]);
      } else if (tid >= 36 && tid < 44) {
        *(uint4*)(wdl + 640 + (tid - 36) * 16) = rwd;
      }
    }
  };

  // ---- input tile (with halo) -> LDS, zero outside the image / past inp
  fetch(0);
  const float inv_cpr = 1.0f / (float)cpr;
  for (int i = tid; i < PIN_PAD * cpr; i += 256) {
    const int pix = fdiv(i, inv_cpr), c = i - pix * cpr;
    const int py = pix / PW, px = pix - py * PW;
    const int iy = iy0 + py, ix = ix0 + px;
    const bool ok = pix < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && c * 8 < p.inp;
    const uint4 v = load16_or_zero(xb + ((size_t)iy * p.W + ix) * p.x_cs + c * 8, xb, ok);
    *(uint4*)(Xs + (c >> 2) * PIN_PAD * 64 + swz(pix, c & 3)) = v;
  }
  stash(0);

  f32x4 acc[NPW][MP];
#pragma unroll
  for (int q = 0; q < NPW; ++q)
#pragma unroll
    for (int m = 0; m < MP; ++m) acc[q][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Expand-epilogue row info is chunk-invariant: per owned N-tile, whether the
  // pixel is inside the image (the depthwise zero-pads the EXPANDED map) and the
  // swizzled LDS addresses of this lane's two 4-channel groups.
  constexpr int NEW = (NE + 3) / 4;
  bool e_inb[NEW];
  int e_addr[NEW][2];
#pragma unroll
  for (int q = 0; q < NEW; ++q) {
    const int pix = (wave + 4 * q) * 16 + row;
    const int py = pix / PW, px = pix - py * PW;
    const int iy = iy0 + py, ix = ix0 + px;
    e_inb[q] = pix < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int hc = mt * 16 + kq * 4;
      e_addr[q][mt] = swz(pix, hc >> 3) + (hc & 7) * 2;
    }
  }

  const int nchunks = p.hid_pad >> 5;
  __syncthreads();
  for (int h = 0; h < nchunks; ++h) {
    const int cur = h & 1;
    const bool more = h + 1 < nchunks;
    if (more) fetch((h + 1) * 32);

    const uint8_t* Esrc;
    if constexpr (EXPAND) {
      const uint8_t* wes = Wes + cur * we_buf;
      const float* be = p.be + h * 32;
#pragma unroll
      for (int q = 0; q < NEW; ++q) {
        const int j = wave + 4 * q;
        if (j >= NE) break;
        const float4 bq0 = *(const float4*)(be + kq * 4);
        const float4 bq1 = *(const float4*)(be + 16 + kq * 4);
        f32x4 e0 = {bq0.x, bq0.y, bq0.z, bq0.w}, e1 = {bq1.x, bq1.y, bq1.z, bq1.w};  // bias folded into init
        for (int sl = 0; sl < nslab; ++sl) {
          const bf16x8 bv = *(const bf16x8*)(Xs + sl * PIN_PAD * 64 + swz(j * 16 + row, kq));
          const bf16x8 a0 = *(const bf16x8*)(wes + sl * 32 * 64 + swz(row, kq));
          const bf16x8 a1 = *(const bf16x8*)(wes + sl * 32 * 64 + swz(16 + row, kq));
          e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bv, e0, 0, 0, 0);
          e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bv, e1, 0, 0, 0);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int hc = mt * 16 + kq * 4;
          const f32x4 e = mt ? e1 : e0;
          float v[4] = {relu6(e[0]), relu6(e[1]), relu6(e[2]), relu6(e[3])};
          if (!e_inb[q]) v[0] = v[1] = v[2] = v[3] = 0.f;
          *(uint2*)(Es + e_addr[q][mt]) = pack4(v);
        }
      }
      __syncthreads();
      Esrc = Es;
    } else {
      Esrc = Xs + h * PIN_PAD * 64;  // hidden == input channels
    }

    // depthwise 3x3 stride S: one (output pixel, 8-channel chunk) per item
    const uint8_t* wdl = Wds + cur * WD_BYTES;
    for (int i = tid; i < POUT_PAD * 4; i += 256) {
      const int q = i >> 2, c = i & 3;
      uint4 outv = {0u, 0u, 0u, 0u};
      if (q < POUT) {
        const int oy = q / TW, ox = q - oy * TW;
        float a[8];
        const float4 b0 = *(const float4*)(wdl + 640 + c * 32);
        const float4 b1 = *(const float4*)(wdl + 640 + c * 32 + 16);
        a[0] = b0.x; a[1] = b0.y; a[2] = b0.z; a[3] = b0.w;
        a[4] = b1.x; a[5] = b1.y; a[6] = b1.z; a[7] = b1.w;
        // taps (2p, 2p+1): regroup each channel's two taps with v_perm, multiply-add with v_dot2c
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int t0 = 2 * pp, t1 = 2 * pp + 1;
          const int pin0 = (oy * S + t0 / 3) * PW + ox * S + t0 % 3;
          const int pin1 = (oy * S + t1 / 3) * PW + ox * S + t1 % 3;
          const uint4 e0 = *(const uint4*)(Esrc + swz(pin0, c));
          const uint4 e1 = *(const uint4*)(Esrc + swz(pin1, c));
          const uint4 wa = *(const uint4*)(wdl + pp * 128 + c * 32);
          const uint4 wb = *(const uint4*)(wdl + pp * 128 + c * 32 + 16);
          const unsigned x0[4] = {e0.x, e0.y, e0.z, e0.w}, x1[4] = {e1.x, e1.y, e1.z, e1.w};
          const unsigned wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const unsigned lo = __builtin_amdgcn_perm(x1[j], x0[j], 0x05040100u);
            const unsigned hi = __builtin_amdgcn_perm(x1[j], x0[j], 0x07060302u);
            a[2 * j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, lo),
                                                       __builtin_bit_cast(bf16x2, wv[2 * j]), a[2 * j], false);
            a[2 * j + 1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hi),
                                                           __builtin_bit_cast(bf16x2, wv[2 * j + 1]), a[2 * j + 1],
                                                           false);
          }
        }
        {  // tap 8 (ky = kx = 2)
          const int pin = (oy * S + 2) * PW + ox * S + 2;
          float e[8];
          unpack8(*(const uint4*)(Esrc + swz(pin, c)), e);
          const float4 w0 = *(const float4*)(wdl + 512 + c * 32);
          const float4 w1 = *(const float4*)(wdl + 512 + c * 32 + 16);
          a[0] = fmaf(e[0], w0.x, a[0]); a[1] = fmaf(e[1], w0.y, a[1]);
          a[2] = fmaf(e[2], w0.z, a[2]); a[3] = fmaf(e[3], w0.w, a[3]);
          a[4] = fmaf(e[4], w1.x, a[4]); a[5] = fmaf(e[5], w1.y, a[5]);
          a[6] = fmaf(e[6], w1.z, a[6]); a[7] = fmaf(e[7], w1.w, a[7]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = relu6(a[k]);
        outv = pack8(a);
      }
      *(uint4*)(Ds + swz(q, c)) = outv;
    }
    __syncthreads();

    // project: acc[pixel tile][oup tile] += Wp[oup][chunk] . D[chunk][pixels]
    const uint8_t* wps = Wps + cur * MP * 16 * 64;
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const int j = wave + 4 * q;
      if (j < NP) {
        const bf16x8 bv = *(const bf16x8*)(Ds + swz(j * 16 + row, kq));
#pragma unroll
        for (int m = 0; m < MP; ++m) {
          const bf16x8 av = *(const bf16x8*)(wps + swz(m * 16 + row, kq));
          acc[q][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[q][m], 0, 0, 0);
        }
      }
    }
    if (more) stash(cur ^ 1);
    __syncthreads();  // next chunk: weights visible, E/D free
  }

  // ---- epilogue: bias (+ residual from the staged input tile) -> NHWC bf16
  bf16* yb = (bf16*)p.y + (size_t)b * p.Ho * p.Wo * p.y_cs;
#pragma unroll
  for (int q = 0; q < NPW; ++q) {
    const int j = wave + 4 * q;
    if (j >= NP) continue;
    const int pix = j * 16 + row;
    if (pix >= POUT) continue;
    const int ly = pix / TW, lx = pix - (pix / TW) * TW;
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy >= p.Ho || ox >= p.Wo) continue;
    bf16* yp = yb + ((size_t)oy * p.Wo + ox) * p.y_cs;
    const int rpix = (ly * S + 1) * PW + lx * S + 1;  // same pixel in the input tile (S == 1 when res)
#pragma unroll
    for (int m = 0; m < MP; ++m) {
      const int oc = m * 16 + kq * 4;
      if (oc >= p.oup) continue;
      const float4 bb = *(const float4*)(p.bp + oc);
      float v[4] = {acc[q][m][0] + bb.x, acc[q][m][1] + bb.y, acc[q][m][2] + bb.z, acc[q][m][3] + bb.w};
      if (p.res) {
        float r[4];
        unpack4(*(const uint2*)(Xs + (oc >> 5) * PIN_PAD * 64 + swz(rpix, (oc & 31) >> 3) + (oc & 7) * 2), r);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += r[k];
      }
      *(uint2*)(yp + oc) = pack4(v);
    }
  }
}

template <int S, int TH, int TW, int MP, bool EXPAND>
static size_t ir_lds_bytes(int inp_pad) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int PIN_PAD = (PH * PW + 15) / 16 * 16, POUT_PAD = (TH * TW + 15) / 16 * 16;
  const int nslab = inp_pad / 32;
  return (size_t)nslab * PIN_PAD * 64 + (EXPAND ? PIN_PAD * 64 : 0) + POUT_PAD * 64 + 2 * MP * 16 * 64 +
         2 * 768 + (EXPAND ? 2 * nslab * 32 * 64 : 0);
}

template <int S, int TH, int TW, int MP, bool EXPAND>
static void ir_launch(const IrParams& p, hipStream_t s) {
  const size_t lds = ir_lds_bytes<S, TH, TW, MP, EXPAND>(p.inp_pad);
  if (lds > 160 * 1024) throw std::runtime_error("ir_block: LDS budget exceeded");
  const int tiles = ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW);
  const long grid = (long)p.B * tiles;
  if (grid <= 0) return;
  hipLaunchKernelGGL((ir_block_kernel<S, TH, TW, MP, EXPAND>), dim3((unsigned)grid), dim3(256), lds, s, p);
}

template <int S, int TH, int TW, int MP, bool EXPAND>
static void ir_set_attr() {
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_block_kernel<S, TH, TW, MP, EXPAND>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

// Supported (stride, tile, oup tiles, expand) combinations: the 17 blocks of
// MobileNetV2 at 224 (8x8 tiles at 112/56, 7x7 tiles from 28 down).
#define ARENA_IR_CONFIGS(X)                                          \
  X(1, 16, 16, 1, false)                                             \
  X(1, 8, 8, 1, false)                                               \
  X(2, 8, 8, 2, true)                                                \
  X(1, 8, 8, 2, true)                                                \
  X(2, 7, 7, 2, true)                                                \
  X(1, 7, 7, 2, true)                                                \
  X(2, 7, 7, 4, true)                                                \
  X(1, 7, 7, 4, true)                                                \
  X(1, 7, 7, 6, true)                                                \
  X(2, 7, 7, 10, true)                                               \
  X(1, 7, 7, 10, true)                                               \
  X(1, 7, 7, 20, true)                                               \
  X(1, 14, 14, 4, true)                                              \
  X(1, 14, 14, 6, true)

void ir_wave_prepare();
void ir_crop_prepare();
void ir_crop_f32_prepare();
void ir_f32_prepare();
bool ir_block_crop(const IrParams& p, hipStream_t s);
bool ir_block_wave(const IrParams& p, int tile, hipStream_t s);
static bool g_ir_wave = [] {
  const char* e = std::getenv("ARENA_IR_WAVE");
  return e ? std::atoi(e) != 0 : true;
}();
void set_ir_wave(bool v) { g_ir_wave = v; }

void ir_prepare() {
  ir_wave_prepare();
  ir_crop_prepare();
  ir_crop_f32_prepare();
  ir_f32_prepare();
#define X(S, TH, TW, MP, E) ir_set_attr<S, TH, TW, MP, E>();
  ARENA_IR_CONFIGS(X)
#undef X
}

// 16x16 output tiles for the 112x112 block (no expand: 42 KB of LDS, 4x the work per workgroup and
// 1.27x instead of 1.56x halo re-reads); ARENA_IR_T16=0 keeps 8x8.
static const bool g_ir_t16 = [] {
  const char* e = std::getenv("ARENA_IR_T16");
  return e ? std::atoi(e) != 0 : true;
}();
// Whole-crop 14x14 tiles for the stride-1 14x14 blocks (ARENA_IR_T14=1): one workgroup per crop, 16
// output N-tiles per hidden chunk instead of 4, and no 9x9-for-7x7 halo recompute of the expansion.
static bool g_ir_t14 = [] {
  const char* e = std::getenv("ARENA_IR_T14");
  return e ? std::atoi(e) != 0 : false;
}();
void set_ir_t14(bool v) { g_ir_t14 = v; }
int ir_tile(int Ho, int stride) {
  if (g_ir_t14 && Ho == 14 && stride == 1) return 14;
  return (g_ir_t16 && Ho >= 112 && Ho % 16 == 0) ? 16 : (Ho % 8 == 0 && Ho >= 56) ? 8 : 7;
}

void ir_block(const IrParams& p, hipStream_t s) {
  if (p.inp_pad % 32 || p.hid_pad % 32 || p.oup_pad % 16 || p.inp % 8 || p.oup % 4 || p.oup > p.oup_pad ||
      p.inp > p.inp_pad)
    throw std::runtime_error("ir_block: bad channel geometry");
  if (p.inp_pad > 192) throw std::runtime_error("ir_block: inp_pad > 192");
  if (!p.expand && p.hid_pad != p.inp_pad) throw std::runtime_error("ir_block: no-expand needs hid_pad == inp_pad");
  if (p.res && (p.stride != 1 || p.inp != p.oup)) throw std::runtime_error("ir_block: residual needs s1, inp == oup");
  if (p.Ho != (p.H + 2 - 3) / p.stride + 1 || p.Wo != (p.W + 2 - 3) / p.stride + 1)
    throw std::runtime_error("ir_block: output size mismatch");
  if (ir_block_crop(p, s)) return;
  const int T = ir_tile(p.Ho, p.stride);
  if (g_ir_wave && ir_block_wave(p, T, s)) return;
  const int MP = p.oup_pad / 16;
  const bool E = p.expand != 0;
#define X(S_, TH_, TW_, MP_, E_)                                                     \
  if (p.stride == S_ && T == TH_ && MP == MP_ && E == E_) {                         \
    ir_launch<S_, TH_, TW_, MP_, E_>(p, s);                                         \
    return;                                                                         \
  }
  ARENA_IR_CONFIGS(X)
#undef X
  throw std::runtime_error("ir_block: unsupported configuration (stride " + std::to_string(p.stride) + ", tile " +
                           std::to_string(T) + ", oup_pad " + std::to_string(p.oup_pad) + ", expand " +
                           std::to_string(p.expand) + ")");
}

}  // namespace arena
