// Whole YOLOv5 C3 block at fp32 accuracy, for the 160x160 level (C1 = 32, c_ = 16, one Bottleneck with shortcut):
//
//   T  = SiLU(W12 . x + b12)                    cv1 | cv2 (1x1, 32 -> 32)
//   U  = SiLU(W1 . T[:, :16] + b1)              Bottleneck cv1 (1x1, 16 -> 16), zero outside the image
//   T1 = T[:, :16] + SiLU(conv3x3(U) + b2)      Bottleneck cv2 (3x3, 16 -> 16) + shortcut
//   y  = SiLU(W3 . [T1, T[:, 16:]] + b3)        cv3 (1x1, 32 -> 32)
//
// The reference runs these as four fp32 ONNX convs (architectures/monolithic/app/inference.py:158-225 via
// ultralytics' C3); unfused here they were four kernels whose 52-105 MB intermediates crossed HBM: ~680 MB of
// traffic per batch of 32 requests, 155 us (ops 2-5 of profiles/r4d/ops_s6t0_bs32.md).  Here one workgroup
// owns an 8 x 16 output tile, recomputes the 1x1 stages on a one-pixel halo ring (10 x 18 = 180 pixels, 1.4x
// their MACs) and keeps T and U in LDS as triple-bf16 planes (v = h + m + l exactly to fp32 rounding, the x3
// scheme of ir_tile_x3.hip): HBM sees the block input once and the output once.
//
// Every GEMM runs on the matrix cores with the six-product split (am bm, al bh, ah bl, am bh, ah bm, ah bh;
// fp32 accumulation): rows = output channels (A = weights, pre-split at plan time), columns = pixels
// (B = activations).  v_mfma_f32_16x16x32_bf16 for K = 32 steps; the 16-deep Bottleneck 1x1 uses
// v_mfma_f32_16x16x16_bf16 instead of padding K.  The 3x3 packs two taps (2 x 16 channels) per 32-deep K step:
// 9 taps in 5 steps, the tenth tap's weights are zero.
//
// Weights (engine/planner.py ProgramBuilder.c3_fused, fp32): w12 bf16 [32][3][32], wb1 [16][3][16],
// wb2 [16][3][160] (k = tap * 16 + channel), w3 [32][3][32] — planes h, m, l of each fp32 row; biases fp32.
#include <stdexcept>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int C3X_TH = 8, C3X_TW = 16;                       // output tile
constexpr int C3X_PH = C3X_TH + 2, C3X_PW = C3X_TW + 2;      // halo tile
constexpr int C3X_NPIX = C3X_PH * C3X_PW;                    // 180
constexpr int C3X_ROWS = (C3X_NPIX + 15) / 16 * 16;          // 192 (12 pixel tiles)
constexpr int C3X_TPB = 3 * 32 * 2 + 16;                     // T row: [h 32 | m 32 | l 32] bf16 + pad (13 slots)
constexpr int C3X_UPB = 3 * 16 * 2 + 16;                     // U row: [h 16 | m 16 | l 16] bf16 + pad (7 slots)
constexpr int C3X_LDS = C3X_ROWS * (C3X_TPB + C3X_UPB) + 96 * 4;  // + the four bias vectors

__device__ __forceinline__ void c3x_split4(const float* v, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16 th = (bf16)v[i];
    const float r = v[i] - (float)th;
    const bf16 tm = (bf16)r;
    h[i] = th;
    m[i] = tm;
    l[i] = (bf16)(r - (float)tm);
  }
}

__device__ __forceinline__ void c3x_split8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bf16 th = (bf16)v[i];
    const float r = v[i] - (float)th;
    const bf16 tm = (bf16)r;
    h[i] = th;
    m[i] = tm;
    l[i] = (bf16)(r - (float)tm);
  }
}

__device__ __forceinline__ f32x4 c3x_mfma32(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                            const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 c3x_mfma16(const bf16x4& ah, const bf16x4& am, const bf16x4& al, const bf16x4& bh,
                                            const bf16x4& bm, const bf16x4& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, c, 0, 0, 0);
}

// one lane's 16-byte piece of each plane of a pre-split weight row (row stride 3 * K bf16)
__device__ __forceinline__ void c3x_wload8(const bf16* w, int K, int row, int k, bf16x8& h, bf16x8& m, bf16x8& l) {
  const bf16* r = w + (size_t)row * 3 * K + k;
  h = *(const bf16x8*)r;
  m = *(const bf16x8*)(r + K);
  l = *(const bf16x8*)(r + 2 * K);
}

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void c3_x3_kernel(const C3Params p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t c3x_lds[];
  uint8_t* Tp = c3x_lds;                          // [ROWS][TPB]
  uint8_t* Up = c3x_lds + C3X_ROWS * C3X_TPB;     // [ROWS][UPB]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = p.W / C3X_TW, tiles = (p.H / C3X_TH) * tiles_x;
  const int total = live_batch(p.B, p.bdev) * tiles;  // tiles of the live images, image-major
  int tile = blockIdx.x;
  if (tile >= total) return;
  const bf16* w12 = (const bf16*)p.w12;
  const bf16* wb1 = (const bf16*)p.wb1[0];
  const bf16* wb2 = (const bf16*)p.wb2[0];
  const bf16* w3 = (const bf16*)p.w3;

  // Every weight fragment and bias this lane needs is requested up front (one global-latency wait, overlapping
  // the input loads) and kept in registers across the four stages: fetched per stage, each stage's dependent
  // weight loads were a serial chain of L2 round trips per wave (the first version ran 154 us per batch of 32,
  // no faster than the four unfused convs).
  bf16x8 w1h[2], w1m[2], w1l[2], w4h[2], w4m[2], w4l[2], w3h[5], w3m[5], w3l[5];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    c3x_wload8(w12, 32, nt * 16 + col, 8 * kq, w1h[nt], w1m[nt], w1l[nt]);
    c3x_wload8(w3, 32, nt * 16 + col, 8 * kq, w4h[nt], w4m[nt], w4l[nt]);
  }
#pragma unroll
  for (int st = 0; st < 5; ++st) c3x_wload8(wb2, 160, col, 32 * st + 8 * kq, w3h[st], w3m[st], w3l[st]);
  const bf16* r1 = wb1 + (size_t)col * 3 * 16 + 4 * kq;
  const bf16x4 w2h = *(const bf16x4*)r1, w2m = *(const bf16x4*)(r1 + 16), w2l = *(const bf16x4*)(r1 + 32);
  // biases in LDS (registers are the limit at two waves per SIMD): [b12 32 | b3 32 | bb1 16 | bb2 16]
  float* Bs = (float*)(Up + C3X_ROWS * C3X_UPB);
  if (tid < 24) {
    const float* src = tid < 8 ? p.b12 + 4 * tid : tid < 16 ? p.b3 + 4 * (tid - 8)
                     : tid < 20 ? p.bb1[0] + 4 * (tid - 16) : p.bb2[0] + 4 * (tid - 20);
    *(float4*)(Bs + 4 * tid) = *(const float4*)src;
  }
  __syncthreads();

  // Persistent workgroups (grid <= 2 per CU): each walks tiles blockIdx.x, + gridDim.x, ...; the next tile's
  // input is requested right after this tile's is split, so its HBM latency hides behind this tile's four stages.
  float4 xa[3], xb[3];
  bool xin[3];
#define C3X_FETCH(tile_)                                                                                   \
  {                                                                                                        \
    const int fb = (tile_) / tiles, ft = (tile_) - fb * tiles;                                             \
    const int fy0 = (ft / tiles_x) * C3X_TH, fx0 = (ft - (ft / tiles_x) * tiles_x) * C3X_TW;               \
    const float* fx = (const float*)p.x + (size_t)fb * p.H * p.W * p.xs;                                   \
    _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                                        \
      const int r = (wave + 4 * i) * 16 + col;                                                             \
      const int iy = fy0 - 1 + r / C3X_PW, ix = fx0 - 1 + r % C3X_PW;                                      \
      xin[i] = r < C3X_NPIX && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;               \
      const float* src = fx + ((size_t)(xin[i] ? iy : 0) * p.W + (xin[i] ? ix : 0)) * p.xs + 8 * kq;       \
      xa[i] = *(const float4*)src;                                                                         \
      xb[i] = *(const float4*)(src + 4);                                                                   \
    }                                                                                                      \
  }
  C3X_FETCH(tile)
  for (; tile < total; tile += gridDim.x) {
  const int b = tile / tiles, t = tile - (tile / tiles) * tiles;
  const int y0 = (t / tiles_x) * C3X_TH, x0 = (t - (t / tiles_x) * tiles_x) * C3X_TW;

  // ---- stage 1: T = SiLU(W12 . x + b12) on the halo tile (12 pixel tiles, 3 per wave; both 16-channel halves)
  {
    bf16x8 xh[3], xm[3], xl[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const bool in = xin[i];
      float v[8] = {in ? xa[i].x : 0.f, in ? xa[i].y : 0.f, in ? xa[i].z : 0.f, in ? xa[i].w : 0.f,
                    in ? xb[i].x : 0.f, in ? xb[i].y : 0.f, in ? xb[i].z : 0.f, in ? xb[i].w : 0.f};
      c3x_split8(v, xh[i], xm[i], xl[i]);
    }
    if (tile + (int)gridDim.x < total) C3X_FETCH(tile + (int)gridDim.x)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int r = (wave + 4 * i) * 16 + col;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 acc = c3x_mfma32(w1h[nt], w1m[nt], w1l[nt], xh[i], xm[i], xl[i], f32x4{0.f, 0.f, 0.f, 0.f});
        // lane holds channels nt * 16 + 4 kq .. +3 of halo pixel r
        const float4 bb = *(const float4*)(Bs + nt * 16 + 4 * kq);
        float o[4] = {silu(acc[0] + bb.x), silu(acc[1] + bb.y), silu(acc[2] + bb.z), silu(acc[3] + bb.w)};
        bf16x4 h, m, l;
        c3x_split4(o, h, m, l);
        uint8_t* d = Tp + r * C3X_TPB + (nt * 16 + 4 * kq) * 2;
        *(bf16x4*)d = h;
        *(bf16x4*)(d + 64) = m;
        *(bf16x4*)(d + 128) = l;
      }
    }
  }
  __syncthreads();

  // ---- stage 2: U = SiLU(W1 . T[:, :16] + b1) on the halo tile, zero outside the image (the 3x3's padding)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = (wave + 4 * i) * 16 + col;
    const uint8_t* s = Tp + r * C3X_TPB + 8 * kq;
    const f32x4 acc = c3x_mfma16(w2h, w2m, w2l, *(const bf16x4*)s, *(const bf16x4*)(s + 64),
                                 *(const bf16x4*)(s + 128), f32x4{0.f, 0.f, 0.f, 0.f});
    const int iy = y0 - 1 + r / C3X_PW, ix = x0 - 1 + r % C3X_PW;
    const bool in = r < C3X_NPIX && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    const float4 bias2 = *(const float4*)(Bs + 64 + 4 * kq);
    float o[4] = {silu(acc[0] + bias2.x), silu(acc[1] + bias2.y), silu(acc[2] + bias2.z), silu(acc[3] + bias2.w)};
    if (!in) o[0] = o[1] = o[2] = o[3] = 0.f;
    bf16x4 h, m, l;
    c3x_split4(o, h, m, l);
    uint8_t* d = Up + r * C3X_UPB + 8 * kq;
    *(bf16x4*)d = h;
    *(bf16x4*)(d + 32) = m;
    *(bf16x4*)(d + 64) = l;
  }
  __syncthreads();

  // ---- stage 3: T1 = T1 + SiLU(conv3x3(U) + b2) on the output tile (8 pixel tiles = 8 rows, 2 per wave), in
  // place in T: a lane reads and writes only its own pixel's channels there; every lane reads U, not written now
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oy = wave + 4 * i, ox = col;  // a 16-pixel tile is one output row
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      int tap = 2 * st + (kq >> 1);
      if (tap > 8) tap = 4;  // the tenth tap: zero weight columns, any valid pixel
      const uint8_t* s = Up + ((oy + tap / 3) * C3X_PW + ox + tap % 3) * C3X_UPB + 16 * (kq & 1);
      acc = c3x_mfma32(w3h[st], w3m[st], w3l[st], *(const bf16x8*)s, *(const bf16x8*)(s + 32),
                       *(const bf16x8*)(s + 64), acc);
    }
    uint8_t* d = Tp + ((oy + 1) * C3X_PW + ox + 1) * C3X_TPB + 8 * kq;
    const bf16x4 th = *(const bf16x4*)d, tm = *(const bf16x4*)(d + 64), tl = *(const bf16x4*)(d + 128);
    const float4 bias3 = *(const float4*)(Bs + 80 + 4 * kq);
    const float bb[4] = {bias3.x, bias3.y, bias3.z, bias3.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ((float)th[j] + (float)tm[j] + (float)tl[j]) + silu(acc[j] + bb[j]);
    bf16x4 h, m, l;
    c3x_split4(o, h, m, l);
    *(bf16x4*)d = h;
    *(bf16x4*)(d + 64) = m;
    *(bf16x4*)(d + 128) = l;
  }
  __syncthreads();

  // ---- stage 4: y = SiLU(W3 . [T1, T2] + b3) on the output tile (8 rows x 2 channel halves, 4 per wave)
  {
    float* __restrict__ y = (float*)p.y + (size_t)b * p.H * p.W * p.ys;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pr = wave + 4 * i, oy = pr >> 1, nt = pr & 1, ox = col;
      const uint8_t* s = Tp + ((oy + 1) * C3X_PW + ox + 1) * C3X_TPB + 16 * kq;
      const f32x4 acc = c3x_mfma32(w4h[nt], w4m[nt], w4l[nt], *(const bf16x8*)s, *(const bf16x8*)(s + 64),
                                   *(const bf16x8*)(s + 128), f32x4{0.f, 0.f, 0.f, 0.f});
      const int co = nt * 16 + 4 * kq;
      const float4 bias = *(const float4*)(Bs + 32 + co);
      *(float4*)(y + ((size_t)(y0 + oy) * p.W + x0 + ox) * p.ys + co) =
          make_float4(silu(acc[0] + bias.x), silu(acc[1] + bias.y), silu(acc[2] + bias.z), silu(acc[3] + bias.w));
    }
  }
  __syncthreads();  // the next tile's stage 1 overwrites T
  }
#undef C3X_FETCH
}

bool c3_x3_supported(int C1, int CH, int NB, bool res, int H, int W) {
  return C1 == 32 && CH == 16 && NB == 1 && res && H % C3X_TH == 0 && W % C3X_TW == 0;
}

void c3_x3_prepare() {
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)c3_x3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      C3X_LDS));
}

void c3_x3(const C3Params& p, hipStream_t s) {
  if (!c3_x3_supported(p.C1, p.CH, p.NB, p.res != 0, p.H, p.W))
    throw std::runtime_error("c3_x3: unsupported geometry (the 160x160 C3 block: C1 32, c_ 16, one bottleneck)");
  if (p.xs % 4 != 0 || p.ys % 4 != 0 || p.xs < 32 || p.ys < 32)
    throw std::runtime_error("c3_x3: pixel strides must be multiples of 4 covering 32 channels");
  const long tiles = (long)p.B * (p.H / C3X_TH) * (p.W / C3X_TW);
  if (tiles <= 0) return;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    ARENA_HIP_CHECK(hipGetDevice(&dev));
    ARENA_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long grid = tiles < 2L * cus ? tiles : 2L * cus;  // two resident workgroups per CU (60 KB LDS each)
  hipLaunchKernelGGL(c3_x3_kernel, dim3((unsigned)grid), dim3(256), C3X_LDS, s, p);
}

}  // namespace arena
