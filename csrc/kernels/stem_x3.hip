// fp32-accurate detector front end in one kernel: letterbox sampling -> YOLO s2d stem conv (3x3, 16 -> 16,
// SiLU) -> the following 3x3 stride-2 conv (16 -> 32, SiLU).  The reference runs this as the first two
// Conv nodes of the fp32 ONNX graph after cv2 letterboxing (architectures/monolithic/app/inference.py:158-180,
// src/shared/processing/yolo_preprocess.py); the unfused fp32 program wrote the 320x320x16 stem map (210 MB
// per batch of 32) and read it back in the s2 conv: 157 + 122 us (profiles/r3c_rt1_ops.md ops 1-2).  Here
// the stem map of a tile exists only in LDS.
//
// Workgroup: NW waves, one TH x 16 tile of the 160x160 output of one image.
//   1. sample the (2 TH + 3) x 35 s2d input pixels of the tile from the uint8 image (letterbox_s2d_px_u8: the
//      letterbox op's own sampler) into LDS as one bf16 plane: the values are integers k <= 255, exact in
//      bf16, and the stem weights carry the 1/255 (pre-split into three planes on the host, so the stem's
//      products are k * w/255 to fp32 accuracy in three MFMAs);
//   2. stem GEMM on v_mfma_f32_16x16x32_bf16 over the (2 TH + 1) x 33 stem pixels the tile needs, as a flat
//      list in fragments of 16 (the kernel row ky's three taps x 16 channels are 48 k: kx 0-1 fill one
//      32-deep slab, kx 2 plus zero weights the second); + bias, SiLU, zero outside the 320x320 map (the s2
//      conv's padding), split into h | m | l planes in LDS;
//   3. the stride-2 conv on v_mfma_f32_32x32x16_bf16, one 16-deep K step per tap, six partial products per
//      operand pair (the x3 scheme of halo_x3g.hip); stem columns are stored even-then-odd so that the
//      stride-2 fragment reads of 16 consecutive lanes hit consecutive LDS rows;
//   4. + bias, SiLU, fp32 NHWC store.
// Weights are read straight from global memory (L2-resident, 41 KB) into fragment registers at each GEMM's start.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"
#include "letterbox.h"

namespace arena {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int SX_TW = 16;                   // output columns per tile
constexpr int SX_SC = 2 * SX_TW + 1;        // stem columns per tile (33)
constexpr int SX_SCS = 2 * ((SX_SC + 1) / 2);  // stored stem columns: 17 even, then 16 odd + 1 pad (34)
constexpr int SX_IC = SX_SC + 2;            // s2d input columns (35)
// LDS strides, chosen with a bank model of the three access patterns (ds_read_b128 lane groups, 64 banks; wide
// writes, 32 banks): 32-B input pixels (no pad) make the stem GEMM's fragment reads 1.5-way instead of 2.3-way,
// and 16 bf16 of pad per stored stem row make the stride-2 conv's reads conflict-free (were 2-way: the two output
// rows of a fragment sat 68 pixel slots apart, i.e. 48 banks)
constexpr int SX_IP = 16;                   // bf16 per input pixel: 12 s2d channels + 4 zero (32 B)
constexpr int SX_SP = 56;                   // bf16 per stem pixel: 3 planes x 16 channels + 8 pad (112 B)
constexpr int SX_SRS = SX_SCS * SX_SP + 16; // bf16 per stored stem row

__host__ __device__ constexpr int sx_sr(int TH) { return 2 * TH + 1; }  // stem rows per tile
__host__ __device__ constexpr int sx_lds_bytes(int TH) {
  return ((sx_sr(TH) + 2) * SX_IC * SX_IP + sx_sr(TH) * SX_SRS) * 2;
}

__device__ __forceinline__ int sx_xcd_remap(int bx, int nx) {
  const int q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
}

}  // namespace

template <int TH, int NW>
__global__ __launch_bounds__(NW * 64) void stem_s2_x3_kernel(const StemFusedParams p) {
  constexpr int NT = NW * 64;
  constexpr int SR = sx_sr(TH), IR = SR + 2;
  constexpr int NSP = SR * SX_SC;            // stem pixels of the tile
  constexpr int NSF = (NSP + 15) / 16;       // 16-pixel stem fragments
  constexpr int NOF = TH / 2;                // 32-pixel output fragments (2 rows x 16 columns)
  static_assert(TH % 2 == 0, "output fragments are two rows");
  extern __shared__ __attribute__((aligned(16))) bf16 sx_lds[];
  bf16* sIn = sx_lds;                        // [IR][35][SX_IP]
  bf16* sSt = sx_lds + IR * SX_IC * SX_IP;   // [SR][SX_SRS]: 34 pixels of SX_SP + pad

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T2 = p.S / 2, Ho = p.S / 4, Wo = p.S / 4;  // s2d / stem map side, output side
  const int tiles_x = Wo / SX_TW, tiles = (Ho / TH) * tiles_x;
  const int bx = sx_xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / tiles;
  const int n_live = p.ctrl != nullptr ? min(p.ctrl->n_images, p.cap) : p.cap;
  if (b >= n_live) return;
  const int t = bx - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * SX_TW;
  const int sy0 = 2 * oy0 - 1, sx0 = 2 * ox0 - 1;  // stem map origin of the tile (s2 conv pad 1)
  const int iy0 = sy0 - 1, ix0 = sx0 - 1;          // s2d input origin (stem conv pad 1)

  const int col = lane & 15, kq = lane >> 4, fr = lane & 31, fh = lane >> 5;

  // ---- 1. letterboxed s2d input, uint8 values as one bf16 plane (zero outside the map: the stem's padding)
  {
    // every sample of this thread is issued before the first is stored: the byte loads of all PXT pixels are in
    // flight together (one pixel per pass waited out a global-load latency per pass)
    constexpr int NPX = IR * SX_IC, PXT = (NPX + NT - 1) / NT;
    const ImageMeta m = p.meta[b];
    float v[PXT][12];
    if (m.new_h == m.h && m.new_w == m.w) {
      // unit scale (the bench's COCO-shaped 640x480 / 640x427 images; uniform per workgroup): the letterboxed
      // pixel is the source pixel or the gray 114 border.  Branch-free: every address is clamped into the
      // image and loaded unconditionally, then selected, so all 4 x 4 x 3 byte loads of a thread are in flight
      // together (the per-sub-pixel branches of letterbox_s2d_px_u8 waited out one load latency each)
      const uint8_t* img = p.pool + m.offset;
      uint8_t u[PXT][12];
      bool ok[PXT][4];
#pragma unroll
      for (int j = 0; j < PXT; ++j) {
        const int px = tid + NT * j;
        const int hy = px / SX_IC, hx = px - hy * SX_IC;
        const int iy = iy0 + hy, ix = ix0 + hx;
        const bool live = px < NPX && (unsigned)iy < (unsigned)T2 && (unsigned)ix < (unsigned)T2;
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int dy = 2 * iy + (pq >> 1) - m.pad_h, dx = 2 * ix + (pq & 1) - m.pad_w;
          ok[j][pq] = live && dy >= 0 && dy < m.h && dx >= 0 && dx < m.w;
          const int cy = min(max(dy, 0), m.h - 1), cx = min(max(dx, 0), m.w - 1);
          const uint8_t* s = img + ((size_t)cy * m.w + cx) * 3;
          u[j][pq * 3] = s[0];
          u[j][pq * 3 + 1] = s[1];
          u[j][pq * 3 + 2] = s[2];
        }
      }
#pragma unroll
      for (int j = 0; j < PXT; ++j) {
        const int px = tid + NT * j;
        const int hy = px / SX_IC, hx = px - hy * SX_IC;
        const bool live = px < NPX && (unsigned)(iy0 + hy) < (unsigned)T2 && (unsigned)(ix0 + hx) < (unsigned)T2;
#pragma unroll
        for (int pq = 0; pq < 4; ++pq)
#pragma unroll
          for (int c = 0; c < 3; ++c)
            v[j][pq * 3 + c] = !live ? 0.f : ok[j][pq] ? (float)u[j][pq * 3 + c] : 114.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < PXT; ++j) {
        const int px = tid + NT * j;
        const int hy = px / SX_IC, hx = px - hy * SX_IC;
        const int iy = iy0 + hy, ix = ix0 + hx;
#pragma unroll
        for (int c = 0; c < 12; ++c) v[j][c] = 0.f;
        if (px < NPX && (unsigned)iy < (unsigned)T2 && (unsigned)ix < (unsigned)T2) {
          float t[16];
          letterbox_s2d_px_u8(p.pool, m, iy, ix, t);
#pragma unroll
          for (int c = 0; c < 12; ++c) v[j][c] = t[c];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < PXT; ++j) {
      const int px = tid + NT * j;
      if (px < NPX) {
        bf16x8 h0, h1;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          h0[c] = (bf16)v[j][c];
          h1[c] = c < 4 ? (bf16)v[j][8 + c] : (bf16)0.f;
        }
        bf16* d = sIn + px * SX_IP;
        *(bf16x8*)d = h0;
        *(bf16x8*)(d + 8) = h1;
      }
    }
  }
  __syncthreads();

  // ---- 2. stem GEMM (16x16x32): A = weights [16 ch][32 k] per (ky, slab), B = input [32 k][16 stem px]
  {
    const bf16* __restrict__ w0 = (const bf16*)p.w;  // [3 ky][2 slabs][16 ch][3 planes][32 k]
    bf16x8 ah[6], am[6], al[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const bf16* r = w0 + ((s * 16 + col) * 3) * 32 + 8 * kq;
      ah[s] = *(const bf16x8*)r;
      am[s] = *(const bf16x8*)(r + 32);
      al[s] = *(const bf16x8*)(r + 64);
    }
    const float4 bias = *(const float4*)(p.bias + 4 * kq);
    const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
    for (int f = wave; f < NSF; f += NW) {
      int sp = f * 16 + col;
      const bool live = sp < NSP;
      sp = live ? sp : NSP - 1;
      const int sr = sp / SX_SC, sc = sp - sr * SX_SC;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const int kabs = sl * 32 + kq * 8;
          const int kx = kabs >> 4 < 3 ? kabs >> 4 : 2, c0 = kabs & 15;  // kx 3: zero weights
          const bf16x8 x = *(const bf16x8*)(sIn + ((sr + ky) * SX_IC + sc + kx) * SX_IP + c0);
          const int s = ky * 2 + sl;
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s], x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[s], x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s], x, acc, 0, 0, 0);
        }
      if (!live) continue;
      // lane holds channels 4 kq .. 4 kq + 3 of stem pixel (sr, sc)
      const int gy = sy0 + sr, gx = sx0 + sc;
      const bool in = (unsigned)gy < (unsigned)T2 && (unsigned)gx < (unsigned)T2;
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = in ? silu(acc[e] + bb[e]) : 0.f;
        const bf16 th = (bf16)v;
        const float rr = v - (float)th;
        const bf16 tm = (bf16)rr;
        h[e] = th;
        m[e] = tm;
        l[e] = (bf16)(rr - (float)tm);
      }
      bf16* d = sSt + sr * SX_SRS + ((sc & 1) * (SX_SCS / 2) + (sc >> 1)) * SX_SP + 4 * kq;
      *(bf16x4*)d = h;
      *(bf16x4*)(d + 16) = m;
      *(bf16x4*)(d + 32) = l;
    }
  }
  __syncthreads();

  // ---- 3. stride-2 conv (32x32x16): A = weights [32 ch][16 k] per tap, B = stem planes [16 k][32 px]
  const bf16* __restrict__ w1 = (const bf16*)p.w2;  // [9 taps][32 ch][3 planes][16 k]
  bf16x8 bwh[9], bwm[9], bwl[9];  // all nine taps' fragments in flight before the first MFMA
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const bf16* wr = w1 + ((tap * 32 + fr) * 3) * 16 + 8 * fh;
    bwh[tap] = *(const bf16x8*)wr;
    bwm[tap] = *(const bf16x8*)(wr + 16);
    bwl[tap] = *(const bf16x8*)(wr + 32);
  }
  // With NW >= 2 NOF waves, two waves share an output fragment: one takes taps 0-4, the other 5-8, and the second
  // hands its partial sums over through LDS (the s2d input region is free after the stem GEMM).
  constexpr bool SPLIT = NW >= 2 * NOF;
  auto conv_taps = [&](int f, int t0, int t1, f32x16& acc) {
    const int r = 2 * f + (fr >> 4), c = fr & 15;  // output pixel of this lane within the tile
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap < t0 || tap >= t1) continue;  // wave-uniform
      const int ky = tap / 3, kx = tap - ky * 3;
      const bf16x8 wh = bwh[tap], wm = bwm[tap], wl = bwl[tap];
      const int sr = 2 * r + ky, sc = 2 * c + kx;
      const bf16* xr = sSt + sr * SX_SRS + ((sc & 1) * (SX_SCS / 2) + (sc >> 1)) * SX_SP + 8 * fh;
      const bf16x8 xh = *(const bf16x8*)xr, xm = *(const bf16x8*)(xr + 16), xl = *(const bf16x8*)(xr + 32);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc, 0, 0, 0);
    }
  };
  // ---- 4. epilogue: lane holds channels 8 g + 4 fh + {0..3} of its pixel
  auto store = [&](int f, const f32x16& acc) {
    const int r = 2 * f + (fr >> 4), c = fr & 15;
    const int oy = oy0 + r, ox = ox0 + c;
    float* y = (float*)p.y2 + (((size_t)b * Ho + oy) * Wo + ox) * p.y2s;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = 8 * g + 4 * fh;
      const float4 bias = *(const float4*)(p.bias2 + ch);
      *(float4*)(y + ch) = make_float4(apply_act(acc[4 * g] + bias.x, p.act2), apply_act(acc[4 * g + 1] + bias.y, p.act2),
                                       apply_act(acc[4 * g + 2] + bias.z, p.act2),
                                       apply_act(acc[4 * g + 3] + bias.w, p.act2));
    }
  };
  if constexpr (SPLIT) {
    static_assert(NOF * 16 * 64 * 4 <= (2 * TH + 3) * SX_IC * SX_IP * 2, "partials must fit the input region");
    float* part = (float*)sIn;  // [NOF][16][64]
    const int f = wave % NOF, half = wave / NOF;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (half < 2) conv_taps(f, half == 0 ? 0 : 5, half == 0 ? 5 : 9, acc);
    if (half == 1)
#pragma unroll
      for (int e = 0; e < 16; ++e) part[(f * 16 + e) * 64 + lane] = acc[e];
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] += part[(f * 16 + e) * 64 + lane];
      store(f, acc);
    }
  } else {
    for (int f = wave; f < NOF; f += NW) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      conv_taps(f, 0, 9, acc);
      store(f, acc);
    }
  }
}

namespace {

template <int TH, int NW>
void sx_launch(const StemFusedParams& p, hipStream_t s) {
  const int tiles = (p.S / 4 / TH) * (p.S / 4 / SX_TW);
  hipLaunchKernelGGL((stem_s2_x3_kernel<TH, NW>), dim3((unsigned)(p.cap * tiles)), dim3(NW * 64), sx_lds_bytes(TH),
                     s, p);
}

}  // namespace

// Geometry the kernel assumes (checked here, on the host, before any launch): letterbox source, 16 -> 16 stem,
// 16 -> 32 stride-2 conv, output side S / 4 a multiple of the 16-wide tile and of TH, fp32 output with a
// float4-aligned pixel stride.  STEM_X3_TH (4 default / 8) picks the tile height.
void stem_s2_f32(const StemFusedParams& p, hipStream_t s) {
  if (p.src != 0 || p.KS != 3 || p.Cout != 16 || p.w2 == nullptr || p.Cout2 != 32 || p.y2 == nullptr ||
      p.y2s % 4 != 0 || p.y2s < 32 || p.S % 64 != 0 || p.pool == nullptr || p.meta == nullptr)
    throw std::runtime_error("stem_s2_f32: needs letterbox src, 3x3 16->16 stem, 3x3 s2 16->32, S % 64 == 0");
  if (p.cap <= 0) return;
  // ARENA_STEM_X3_TH: tile rows (4 default, 8); ARENA_STEM_X3_NW: waves per workgroup (TH 4: 2 or 4; TH 8: 4)
  const char* e = std::getenv("ARENA_STEM_X3_TH");  // read per enqueue: graphs capture it once
  const char* n = std::getenv("ARENA_STEM_X3_NW");
  const int th = e != nullptr && std::atoi(e) == 8 ? 8 : 4;
  const int nw = n != nullptr ? std::atoi(n) : 4;
  if (th == 8)
    sx_launch<8, 4>(p, s);
  else if (nw == 2)
    sx_launch<4, 2>(p, s);
  else
    sx_launch<4, 4>(p, s);
}

void stem_s2_f32_prepare() {
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)stem_s2_x3_kernel<4, 2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, sx_lds_bytes(4)));
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)stem_s2_x3_kernel<4, 4>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, sx_lds_bytes(4)));
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)stem_s2_x3_kernel<8, 4>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, sx_lds_bytes(8)));
}

}  // namespace arena
