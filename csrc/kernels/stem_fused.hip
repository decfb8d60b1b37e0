// Fused preprocessing + stem convolution (K1+K2 for YOLOv5nu, K9+K10 for
// MobileNetV2): the space-to-depth input tile of one workgroup is computed
// straight from the uint8 source image into LDS (letterbox for the detector,
// crop gather + ImageNet normalisation for the classifier) and the stem conv
// runs on it with MFMA, so the bf16 s2d tensor never goes to HBM.
//
// Unfused, the detector's front end wrote a [B,320,320,16] bf16 letterbox
// tensor (105 MB at B = 32) and the stem conv read it back ~9x through L2;
// here each workgroup recomputes its halo ring instead (10x34 input pixels
// for an 8x32 output tile: 1.33x the bilinear work, no round trip).
//
// Per workgroup (256 threads = 4 waves): one output tile of TH x TW pixels
// (256) x NF*16 channels of one image / crop.
//   phase 1  every thread builds s2d pixels of the (TH+KS-1) x (TW+KS-1)
//            halo tile: 4 sub-pixels x RGB by cv2-INTER_LINEAR bilinear
//            sampling, 16 bf16 channels (12 live) = 32 B per pixel in LDS;
//            pixels outside the map are the conv's zero padding.
//   phase 2  each wave owns 4 fragments of 16 pixels; K = KS*KS taps x 16
//            channels in 32-deep slabs, weights held in registers; one
//            v_mfma_f32_16x16x32_bf16 per (fragment, N-fragment, slab).
//   epilogue bias + activation, 8-byte stores of 4 channels per lane.
// Blocks are mapped so that all tiles of an image run on one XCD (the
// source image's rows are re-read by neighbouring tiles from that L2).
//
// Numerics are identical to letterbox_s2d / crop_gather_s2d followed by the
// stem conv: the same float ops produce the same bf16 s2d values.
#include "common.h"
#include "launch.h"

namespace arena {

namespace {

struct LinTap2 {
  int i0, i1;
  float f;
};

__device__ __forceinline__ LinTap2 tap_of(int d, float scale, int n) {
  float fx = ((float)d + 0.5f) * scale - 0.5f;
  int s0 = (int)floorf(fx);
  float f = fx - (float)s0;
  if (s0 < 0) { s0 = 0; f = 0.f; }
  if (s0 >= n - 1) { s0 = n - 1; f = 0.f; }
  LinTap2 t;
  t.i0 = s0;
  t.i1 = s0 + 1 < n ? s0 + 1 : n - 1;
  t.f = f;
  return t;
}

struct RowTap {
  int o0, o1;  // byte offsets of the two taps (o0 < 0: outside the sampled area)
  float f;     // weight of tap 1
};

typedef float float2v __attribute__((ext_vector_type(2)));

// Both sub-pixel columns of one sub-pixel row (the pair shares the row taps),
// in packed fp32 (v_pk_fma_f32 / v_pk_add_f32).  `ident` (scale exactly 1,
// so every lerp weight is 0): the sample is the source byte itself, as
// cv2.resize copies at equal sizes.  Columns outside the sampled area keep
// `pad`.
__device__ __forceinline__ void bilinear_pair(const uint8_t* base, const RowTap& ry, const RowTap& c0,
                                              const RowTap& c1, bool ident, float pad, float2v* rgb) {
  const bool v0 = c0.o0 >= 0, v1 = c1.o0 >= 0;
  if (!v0 && !v1) return;
  const int a0 = v0 ? c0.o0 : c1.o0, a1 = v1 ? c1.o0 : c0.o0;  // an invalid column reads its valid neighbour
  const uint8_t* p0 = base + ry.o0;
  if (ident) {
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = float2v{(float)p0[a0 + c], (float)p0[a1 + c]};
  } else {
    const int b0 = v0 ? c0.o1 : c1.o1, b1 = v1 ? c1.o1 : c0.o1;
    const uint8_t* p1 = base + ry.o1;
    const float2v fx = {c0.f, c1.f}, fy = {ry.f, ry.f}, half = {0.5f, 0.5f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float2v va = {(float)p0[a0 + c], (float)p0[a1 + c]}, vb = {(float)p0[b0 + c], (float)p0[b1 + c]};
      const float2v vd = {(float)p1[a0 + c], (float)p1[a1 + c]}, ve = {(float)p1[b0 + c], (float)p1[b1 + c]};
      const float2v top = va + (vb - va) * fx;
      const float2v bot = vd + (ve - vd) * fx;
      const float2v r = top + (bot - top) * fy + half;
      rgb[c] = float2v{floorf(r.x), floorf(r.y)};  // cv2 returns uint8
    }
  }
  if (!v0 || !v1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = float2v{v0 ? rgb[c].x : pad, v1 ? rgb[c].y : pad};
  }
}

// Source geometry of one batch item, uniform over the workgroup.
struct Src {
  const uint8_t* img;  // top-left of the sampled region
  int stride_px;       // image row stride in pixels
  int h, w;            // sampled region size (letterbox: new_h/new_w of the resized image)
  int rh, rw;          // region size the taps clamp to (source pixels)
  int pad_h, pad_w;    // letterbox padding (0 for crops)
  float sy, sx;
  bool empty;          // zero-area crop -> black
};

}  // namespace

// Source pixels a tile samples are first copied into LDS with aligned dword
// loads (a 640x480 image at scale 1 needs ~21 rows x 69 px = 4.3 KB per
// 8x32 tile), then the bilinear taps read LDS bytes: one global dword load
// per 4 source bytes instead of 12 byte loads per sub-pixel.  Regions above
// the budget (strongly downscaled images, large crops) sample global memory.
constexpr int kSrcBudget = 8192;  // 16 KB measured slower: LDS held occupancy at 5 workgroups / CU

// Source geometry of batch item `item` (image letterboxed to p.S, or crop resized to p.S x p.S).
template <int SRC>
__device__ __forceinline__ Src make_src(const StemFusedParams& p, int item) {
  Src g;
  if constexpr (SRC == 0) {
    const ImageMeta m = p.meta[item];
    g.img = p.pool + m.offset;
    g.stride_px = m.w;
    g.h = m.new_h;
    g.w = m.new_w;
    g.rh = m.h;
    g.rw = m.w;
    g.pad_h = m.pad_h;
    g.pad_w = m.pad_w;
    g.sy = (float)((double)m.h / (double)m.new_h);
    g.sx = (float)((double)m.w / (double)m.new_w);
    g.empty = false;
  } else {
    const CropRef cr = p.crops[p.ctrl->crop_base + item];
    const ImageMeta m = p.meta[cr.img];
    const int cw = cr.x2 - cr.x1, ch = cr.y2 - cr.y1;
    g.empty = cw <= 0 || ch <= 0;
    g.img = p.pool + m.offset + ((size_t)cr.y1 * m.w + cr.x1) * 3;
    g.stride_px = m.w;
    g.h = g.rh = ch;
    g.w = g.rw = cw;
    g.pad_h = g.pad_w = 0;
    g.sy = g.empty ? 1.f : (float)((double)ch / (double)p.S);
    g.sx = g.empty ? 1.f : (float)((double)cw / (double)p.S);
  }

  return g;
}

// Space-to-depth halo tile of HH x HW s2d pixels starting at s2d position (sY0, sX0): phase 0
// stages the source bytes it samples in `region` (when they fit in BUDGET bytes), the tap tables
// are built, and phase 1 writes 32 B (16 bf16 channels, 12 live) per s2d pixel into `tile`;
// pixels outside the S/2 x S/2 map are zero (the stem conv's padding).  Ends with the tile
// written by this thread (callers barrier before reading it).
template <int SRC, int HH, int HW, int BUDGET>
__device__ __forceinline__ void build_s2d_tile(const StemFusedParams& p, const Src& g, int sY0, int sX0, uint4* tile,
                                               uint32_t* region, RowTap* rtab, RowTap* ctab) {
  constexpr int NPIX = HH * HW;
  static_assert(2 * HH <= 64 && 2 * HW <= 192, "tap tables are built by waves 0 / 1-3");
  const int S2 = p.S >> 1;
  // ---- phase 0: source rows / columns this tile samples -> LDS (when they fit)
  // sub-pixel rows/cols of the halo tile, clamped to the sampled area
  const int lim_y = SRC == 0 ? g.h : p.S, lim_x = SRC == 0 ? g.w : p.S;
  const int sy_lo = max(2 * sY0 - g.pad_h, 0), sy_hi = min(2 * (sY0 + HH - 1) + 1 - g.pad_h, lim_y - 1);
  const int sx_lo = max(2 * sX0 - g.pad_w, 0), sx_hi = min(2 * (sX0 + HW - 1) + 1 - g.pad_w, lim_x - 1);
  bool staged = false;
  int r_lo = 0, c_lo = 0, pitch = 0;
  const size_t row_bytes = (size_t)g.stride_px * 3;
  if (!g.empty && sy_lo <= sy_hi && sx_lo <= sx_hi) {
    r_lo = tap_of(sy_lo, g.sy, g.rh).i0;
    c_lo = tap_of(sx_lo, g.sx, g.rw).i0;
    const int r_hi = tap_of(sy_hi, g.sy, g.rh).i1, c_hi = tap_of(sx_hi, g.sx, g.rw).i1;
    const int nrows = r_hi - r_lo + 1, rbytes = (c_hi - c_lo + 1) * 3;
    const int ndw = (rbytes + 3 + 3) >> 2;  // up to 3 bytes of alignment shift in front
    pitch = ndw * 4;
    staged = nrows * pitch <= BUDGET;
    if (staged) {
      const uint8_t* base = g.img + (size_t)r_lo * row_bytes + (size_t)c_lo * 3;
      for (int i = threadIdx.x; i < nrows * ndw; i += 256) {
        const int r = i / ndw, k = i - (i / ndw) * ndw;
        const uint8_t* src = base + (size_t)r * row_bytes;
        const uint32_t* a = (const uint32_t*)((uintptr_t)src & ~(uintptr_t)3);
        region[r * ndw + k] = a[k];
      }
    }
  }
  const uint8_t* reg = (const uint8_t*)region;
  const uintptr_t base_addr = (uintptr_t)(g.img + (size_t)r_lo * row_bytes + (size_t)c_lo * 3);

  // ---- tap tables: one entry per sub-pixel row / column of the halo tile
  // (byte offsets of both source rows / pixels in the staged region or the
  // image, and the lerp weight), so the per-sub-pixel work below is lookups,
  // 12 byte loads and the lerps.  o0 < 0 marks a row / column outside the
  // sampled area (letterbox border -> 114, empty crop -> 0).
  if (threadIdx.x < 2 * HH) {
    const int d = 2 * sY0 + (int)threadIdx.x - g.pad_h;
    RowTap e{-1, -1, 0.f};
    if (!g.empty && d >= 0 && d < (SRC == 0 ? g.h : p.S)) {
      const LinTap2 t = tap_of(d, g.sy, g.rh);
      if (staged) {
        const int r0 = t.i0 - r_lo, r1 = t.i1 - r_lo;
        e.o0 = r0 * pitch + (int)((base_addr + (size_t)r0 * row_bytes) & 3);
        e.o1 = r1 * pitch + (int)((base_addr + (size_t)r1 * row_bytes) & 3);
      } else {
        e.o0 = (int)((size_t)t.i0 * row_bytes);
        e.o1 = (int)((size_t)t.i1 * row_bytes);
      }
      e.f = t.f;
    }
    rtab[threadIdx.x] = e;
  } else if (threadIdx.x >= 64 && threadIdx.x < 64 + 2 * HW) {
    const int k = (int)threadIdx.x - 64;
    const int d = 2 * sX0 + k - g.pad_w;
    RowTap e{-1, -1, 0.f};
    if (!g.empty && d >= 0 && d < (SRC == 0 ? g.w : p.S)) {
      const LinTap2 t = tap_of(d, g.sx, g.rw);
      const int c0 = staged ? c_lo : 0;
      e.o0 = (t.i0 - c0) * 3;
      e.o1 = (t.i1 - c0) * 3;
      e.f = t.f;
    }
    ctab[k] = e;
  }
  __syncthreads();

  // ---- phase 1: s2d halo tile into LDS
  const float pad_val = SRC == 0 ? 114.f : 0.f;
  const bool ident = g.sy == 1.f && g.sx == 1.f;
  for (int i = threadIdx.x; i < NPIX; i += 256) {
    const int hy = i / HW, hx = i - (i / HW) * HW;
    const int Y = sY0 + hy, X = sX0 + hx;
    float out[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) out[k] = 0.f;
    if ((unsigned)Y < (unsigned)S2 && (unsigned)X < (unsigned)S2) {
      const RowTap c0 = ctab[2 * hx], c1 = ctab[2 * hx + 1];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const RowTap ry = rtab[2 * hy + a];
        float2v rgb[3] = {{pad_val, pad_val}, {pad_val, pad_val}, {pad_val, pad_val}};  // (column 0, column 1)
        if (ry.o0 >= 0) {
          // separate calls keep the staged path on ds_read (not flat) loads
          if (staged) bilinear_pair(reg, ry, c0, c1, ident, pad_val, rgb);
          else bilinear_pair(g.img, ry, c0, c1, ident, pad_val, rgb);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const float v = b ? rgb[c].y : rgb[c].x;
            if constexpr (SRC == 0) out[(a * 2 + b) * 3 + c] = v * (1.0f / 255.0f);
            else out[(a * 2 + b) * 3 + c] = (v * (1.0f / 255.0f) - p.mean[c]) * p.inv_std[c];
          }
        }
      }
    }
    tile[i * 2] = pack8(out);
    tile[i * 2 + 1] = pack8(out + 8);
  }

}

template <int SRC, int KS, int NF, int TH, int TW>
__global__ __launch_bounds__(256) void stem_fused_kernel(const StemFusedParams p) {
  constexpr int HH = TH + KS - 1, HW = TW + KS - 1, NPIX = HH * HW;
  constexpr int SLABS = (KS * KS * 16 + 31) / 32;
  static_assert(TH * TW == 256, "one 256-pixel tile per workgroup (4 waves x 4 fragments)");
  __shared__ __align__(16) uint4 tile[NPIX * 2];  // 32 B per s2d pixel
  __shared__ __align__(16) uint32_t region[kSrcBudget / 4];

  const int S2 = p.S >> 1;
  const int tiles_x = (S2 + TW - 1) / TW, tiles_y = (S2 + TH - 1) / TH, ntiles = tiles_x * tiles_y;
  const int id = blockIdx.x, xcd = id & 7, j = id >> 3;
  const int item = (j / ntiles) * 8 + xcd;  // every tile of one item lands on one XCD
  const int t = j - (j / ntiles) * ntiles;
  const int n_live = live_batch(p.cap, SRC == 0 ? &p.ctrl->n_images : &p.ctrl->n_crops);
  if (item >= n_live) return;
  const int ty0 = (t / tiles_x) * TH, tx0 = (t % tiles_x) * TW;

  const Src g = make_src<SRC>(p, item);
  __shared__ RowTap rtab[2 * HH];
  __shared__ RowTap ctab[2 * HW];
  build_s2d_tile<SRC, HH, HW, kSrcBudget>(p, g, ty0 - 1, tx0 - 1, tile, region, rtab, ctab);

  // ---- weights of this lane's rows into registers (overlaps the barrier)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const bf16* __restrict__ w = (const bf16*)p.w;
  bf16x8 wf[NF][SLABS];
#pragma unroll
  for (int a = 0; a < NF; ++a)
#pragma unroll
    for (int s = 0; s < SLABS; ++s) wf[a][s] = *(const bf16x8*)(w + (size_t)(a * 16 + row) * p.Kpad + s * 32 + kq * 8);
  __syncthreads();

  // ---- phase 2: MFMA over the LDS tile
  f32x4 acc[NF][4];
#pragma unroll
  for (int a = 0; a < NF; ++a)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[a][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < SLABS; ++s) {
    int tap = 2 * s + (kq >> 1);
    if (tap >= KS * KS) tap = 0;  // zero weight rows; any finite LDS value will do
    const int kh = tap / KS, kw = tap - (tap / KS) * KS, chunk = kq & 1;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int P = (wave * 4 + f) * 16 + row;
      const int py = P / TW, px = P - (P / TW) * TW;
      const bf16x8 bv = *(const bf16x8*)&tile[((py + kh) * HW + px + kw) * 2 + chunk];
#pragma unroll
      for (int a = 0; a < NF; ++a) acc[a][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a][s], bv, acc[a][f], 0, 0, 0);
    }
  }

  // ---- epilogue
  bf16* __restrict__ y = (bf16*)p.y;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int P = (wave * 4 + f) * 16 + row;
    const int oy = ty0 + P / TW, ox = tx0 + (P - (P / TW) * TW);
    if (oy >= S2 || ox >= S2) continue;
    const size_t base = ((size_t)item * S2 * S2 + (size_t)oy * S2 + ox) * p.ys;
#pragma unroll
    for (int a = 0; a < NF; ++a) {
      const int cb = a * 16 + kq * 4;
      const float4 bias = *(const float4*)(p.bias + cb);
      float v[4] = {acc[a][f][0] + bias.x, acc[a][f][1] + bias.y, acc[a][f][2] + bias.z, acc[a][f][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      *(uint2*)(y + base + cb) = pack4(v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Detector front end in one kernel: letterbox -> stem (3x3 s1 over s2d, 16 ch, SiLU) -> second conv
// (3x3 s2, 16 -> 32, SiLU).  The 320x320x16 stem output (105 MB at B = 32, written once and read
// back ~2.3x by the next conv) never leaves LDS.  Per workgroup: a TH2 x TW2 tile of the second
// conv's output needs a (2TH2+1) x (2TW2+1) stem-output tile, which needs a (2TH2+3) x (2TW2+3)
// s2d tile: the s2d work per image equals the single-stage kernel's (665 vs 2 x 340 halo pixels
// per 256 stem outputs), the stem MFMA work grows 1.1x for the halo.
constexpr int kSrc2Budget = 12288;  // ~8.4 KB source bytes per tile at scale 1 (aliases the stem output)

template <int TH2, int TW2>
__global__ __launch_bounds__(256) void stem2_kernel(const StemFusedParams p) {
  constexpr int SR = 2 * TH2 + 1, SC = 2 * TW2 + 1;  // stem-output tile
  constexpr int HH = SR + 2, HW = SC + 2;            // s2d tile
  constexpr int NS = SR * SC, NSF = (NS + 15) / 16;  // stem-output pixels / 16-pixel fragments
  constexpr int SLABS = 5;                           // 9 taps x 16 channels in 32-deep slabs (both convs)
  static_assert(TH2 * TW2 == 128, "8 second-conv fragments: 2 per wave");
  // The staged source bytes are dead once the s2d tile is built, so they share LDS with the stem
  // output: 40.5 KB per workgroup = 4 workgroups per CU (53 KB without the alias: 3).
  constexpr int SCRATCH = NS * 2 > kSrc2Budget / 16 ? NS * 2 : kSrc2Budget / 16;  // uint4 units
  __shared__ __align__(16) uint4 tile[HH * HW * 2];
  __shared__ __align__(16) uint4 scratch[SCRATCH];
  uint4* sout = scratch;                   // stem output, 32 B per pixel (after the s2d tile is built)
  uint32_t* region = (uint32_t*)scratch;  // staged source bytes (while the s2d tile is built)
  __shared__ RowTap rtab[2 * HH];
  __shared__ RowTap ctab[2 * HW];

  const int S2 = p.S >> 1, S4 = S2 >> 1;
  const int tiles_x = S4 / TW2, ntiles = tiles_x * (S4 / TH2);
  const int id = blockIdx.x, xcd = id & 7, j = id >> 3;
  const int item = (j / ntiles) * 8 + xcd;  // every tile of one image lands on one XCD
  const int t = j - (j / ntiles) * ntiles;
  if (item >= live_batch(p.cap, &p.ctrl->n_images)) return;
  const int oy0 = (t / tiles_x) * TH2, ox0 = (t % tiles_x) * TW2;
  const int Y0 = 2 * oy0 - 1, X0 = 2 * ox0 - 1;  // stem-output tile origin (second conv: pad 1)

  const Src g = make_src<0>(p, item);
  build_s2d_tile<0, HH, HW, kSrc2Budget>(p, g, Y0 - 1, X0 - 1, tile, region, rtab, ctab);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const bf16* __restrict__ w = (const bf16*)p.w;
  const bf16* __restrict__ w2 = (const bf16*)p.w2;
  bf16x8 wf[SLABS], w2f[2][SLABS];
#pragma unroll
  for (int s = 0; s < SLABS; ++s) {
    wf[s] = *(const bf16x8*)(w + (size_t)row * p.Kpad + s * 32 + kq * 8);
#pragma unroll
    for (int a = 0; a < 2; ++a) w2f[a][s] = *(const bf16x8*)(w2 + (size_t)(a * 16 + row) * p.Kpad2 + s * 32 + kq * 8);
  }
  const float4 sb = *(const float4*)(p.bias + kq * 4);
  __syncthreads();

  // ---- stem conv over the s2d tile -> sout (zero outside the S/2 map: the second conv's padding)
  for (int fr = wave; fr < NSF; fr += 4) {
    const int P = fr * 16 + row;
    const int Pc = P < NS ? P : NS - 1;  // padded rows read a valid pixel; their results are unused
    const int sy = Pc / SC, sx = Pc - (Pc / SC) * SC;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SLABS; ++s) {
      int tap = 2 * s + (kq >> 1);
      if (tap >= 9) tap = 0;  // zero weight rows
      const int kh = tap / 3, kw = tap - (tap / 3) * 3;
      const bf16x8 bv = *(const bf16x8*)&tile[((sy + kh) * HW + sx + kw) * 2 + (kq & 1)];
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], bv, acc, 0, 0, 0);
    }
    const bool inside = (unsigned)(Y0 + sy) < (unsigned)S2 && (unsigned)(X0 + sx) < (unsigned)S2;
    float v[4] = {apply_act(acc[0] + sb.x, p.act), apply_act(acc[1] + sb.y, p.act), apply_act(acc[2] + sb.z, p.act),
                  apply_act(acc[3] + sb.w, p.act)};
    if (!inside) v[0] = v[1] = v[2] = v[3] = 0.f;
    if (P < NS) *(uint2*)((uint8_t*)sout + P * 32 + kq * 8) = pack4(v);
  }
  __syncthreads();

  // ---- second conv (3x3 stride 2) over sout -> global
  bf16* __restrict__ y2 = (bf16*)p.y2;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int Q = (wave * 2 + q) * 16 + row;
    const int qy = Q / TW2, qx = Q - (Q / TW2) * TW2;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < SLABS; ++s) {
      int tap = 2 * s + (kq >> 1);
      if (tap >= 9) tap = 0;
      const int kh = tap / 3, kw = tap - (tap / 3) * 3;
      const bf16x8 bv = *(const bf16x8*)&sout[((2 * qy + kh) * SC + 2 * qx + kw) * 2 + (kq & 1)];
#pragma unroll
      for (int a = 0; a < 2; ++a) acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[a][s], bv, acc[a], 0, 0, 0);
    }
    const size_t base = ((size_t)item * S4 * S4 + (size_t)(oy0 + qy) * S4 + ox0 + qx) * p.y2s;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int cb = a * 16 + kq * 4;
      const float4 bias = *(const float4*)(p.bias2 + cb);
      float v[4] = {acc[a][0] + bias.x, acc[a][1] + bias.y, acc[a][2] + bias.z, acc[a][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act2);
      *(uint2*)(y2 + base + cb) = pack4(v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Classifier front end in one kernel: crop gather (resize 224, ImageNet normalisation) -> stem
// (2x2 over s2d, 32 ch, ReLU6) -> MobileNetV2 block 1 (t = 1: depthwise 3x3 + ReLU6, project
// 32 -> 16).  The 112x112x32 stem output (101 MB for 126 crops, written once and read once) only
// exists in LDS.  Per workgroup: a T x T tile of block 1's output needs a (T+2)^2 stem-output tile,
// which needs a (T+3)^2 s2d tile.
constexpr int kSrcIrBudget = 8192;

__device__ __forceinline__ int ir_swz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}

template <int T>
__global__ __launch_bounds__(256) void stem_ir_kernel(const StemFusedParams p) {
  constexpr int FT = T + 2, HT = FT + 1;                  // stem-output tile, s2d tile
  constexpr int NFP = FT * FT, NFF = (NFP + 15) / 16;     // stem-output pixels / fragments
  constexpr int NOUT = T * T;
  static_assert(NOUT % 64 == 0 && 2 * HT <= 64, "tile geometry");
  // LDS A: s2d tile, later the depthwise output D; LDS B: staged source bytes, later the stem output F.
  constexpr int A_BYTES = HT * HT * 32 > NOUT * 64 ? HT * HT * 32 : NOUT * 64;
  constexpr int B_BYTES = NFP * 64 > kSrcIrBudget ? NFP * 64 : kSrcIrBudget;
  __shared__ __align__(16) uint8_t lA[A_BYTES];
  __shared__ __align__(16) uint8_t lB[B_BYTES];
  __shared__ RowTap rtab[2 * HT];
  __shared__ RowTap ctab[2 * HT];
  uint4* tile = (uint4*)lA;
  uint8_t* Ds = lA;
  uint32_t* region = (uint32_t*)lB;
  uint8_t* Fs = lB;

  const int S2 = p.S >> 1;
  const int tiles_x = S2 / T, ntiles = tiles_x * tiles_x;
  const int id = blockIdx.x, xcd = id & 7, j = id >> 3;
  const int item = (j / ntiles) * 8 + xcd;  // every tile of one crop lands on one XCD
  const int t = j - (j / ntiles) * ntiles;
  if (item >= live_batch(p.cap, &p.ctrl->n_crops)) return;
  const int oy0 = (t / tiles_x) * T, ox0 = (t % tiles_x) * T;
  const int Y0 = oy0 - 1, X0 = ox0 - 1;  // stem-output tile origin (depthwise pad 1)

  const Src g = make_src<1>(p, item);
  build_s2d_tile<1, HT, HT, kSrcIrBudget>(p, g, Y0 - 1, X0 - 1, tile, region, rtab, ctab);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const bf16* __restrict__ w = (const bf16*)p.w;
  bf16x8 wf[2][2];  // [N-fragment][slab]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int s = 0; s < 2; ++s) wf[a][s] = *(const bf16x8*)(w + (size_t)(a * 16 + row) * p.Kpad + s * 32 + kq * 8);
  const float4 sb0 = *(const float4*)(p.bias + kq * 4), sb1 = *(const float4*)(p.bias + 16 + kq * 4);
  // depthwise taps of this thread's 8-channel group (items tid + 256 k keep tid & 3), as bf16 tap pairs
  const int dc = tid & 3;
  const bf16* wd = (const bf16*)p.ir_wd;
  unsigned wpair[4][8];
  float w8[8], bd[8];
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) {
    const uint4 a = *(const uint4*)(wd + (2 * pp) * 32 + dc * 8);
    const uint4 c2 = *(const uint4*)(wd + (2 * pp + 1) * 32 + dc * 8);
    const unsigned av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c2.x, c2.y, c2.z, c2.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      wpair[pp][2 * q] = __builtin_amdgcn_perm(cv[q], av[q], 0x05040100u);
      wpair[pp][2 * q + 1] = __builtin_amdgcn_perm(cv[q], av[q], 0x07060302u);
    }
  }
  unpack8(*(const uint4*)(wd + 8 * 32 + dc * 8), w8);
  {
    const float4 b0 = *(const float4*)(p.ir_bd + dc * 8), b1 = *(const float4*)(p.ir_bd + dc * 8 + 4);
    bd[0] = b0.x; bd[1] = b0.y; bd[2] = b0.z; bd[3] = b0.w;
    bd[4] = b1.x; bd[5] = b1.y; bd[6] = b1.z; bd[7] = b1.w;
  }
  const bf16x8 wpa = *(const bf16x8*)((const bf16*)p.ir_wp + row * 32 + kq * 8);
  __syncthreads();

  // ---- stem conv (2x2 over s2d, 32 channels, ReLU6) -> F (zero outside the S/2 map: depthwise padding)
  for (int fr = wave; fr < NFF; fr += 4) {
    const int P = fr * 16 + row;
    const int Pc = P < NFP ? P : NFP - 1;
    const int sy = Pc / FT, sx = Pc - (Pc / FT) * FT;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int tap = 2 * s + (kq >> 1), kh = tap >> 1, kw = tap & 1;
      const bf16x8 bv = *(const bf16x8*)&tile[((sy + kh) * HT + sx + kw) * 2 + (kq & 1)];
#pragma unroll
      for (int a = 0; a < 2; ++a) acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a][s], bv, acc[a], 0, 0, 0);
    }
    const bool inside = (unsigned)(Y0 + sy) < (unsigned)S2 && (unsigned)(X0 + sx) < (unsigned)S2;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float4 bb = a ? sb1 : sb0;
      float v[4] = {apply_act(acc[a][0] + bb.x, p.act), apply_act(acc[a][1] + bb.y, p.act),
                    apply_act(acc[a][2] + bb.z, p.act), apply_act(acc[a][3] + bb.w, p.act)};
      if (!inside) v[0] = v[1] = v[2] = v[3] = 0.f;
      if (P < NFP) *(uint2*)(Fs + P * 64 + (a * 16 + kq * 4) * 2) = pack4(v);
    }
  }
  __syncthreads();

  // ---- depthwise 3x3 + ReLU6 -> D (swizzled rows for the project MFMA)
#pragma unroll
  for (int k = 0; k < NOUT * 4 / 256; ++k) {
    const int q = (tid + 256 * k) >> 2;
    const int oy = q / T, ox = q - (q / T) * T;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = bd[i];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int t0 = 2 * pp, t1 = 2 * pp + 1;
      const uint4 e0 = *(const uint4*)(Fs + ((oy + t0 / 3) * FT + ox + t0 % 3) * 64 + dc * 16);
      const uint4 e1 = *(const uint4*)(Fs + ((oy + t1 / 3) * FT + ox + t1 % 3) * 64 + dc * 16);
      const unsigned x0[4] = {e0.x, e0.y, e0.z, e0.w}, x1[4] = {e1.x, e1.y, e1.z, e1.w};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const unsigned lo = __builtin_amdgcn_perm(x1[jj], x0[jj], 0x05040100u);
        const unsigned hi = __builtin_amdgcn_perm(x1[jj], x0[jj], 0x07060302u);
        acc[2 * jj] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, lo),
                                                      __builtin_bit_cast(bf16x2, wpair[pp][2 * jj]), acc[2 * jj], false);
        acc[2 * jj + 1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hi),
                                                          __builtin_bit_cast(bf16x2, wpair[pp][2 * jj + 1]),
                                                          acc[2 * jj + 1], false);
      }
    }
    float e8[8];
    unpack8(*(const uint4*)(Fs + ((oy + 2) * FT + ox + 2) * 64 + dc * 16), e8);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = relu6f(fmaf(e8[i], w8[i], acc[i]));
    *(uint4*)(Ds + ir_swz(q, dc)) = pack8(acc);
  }
  __syncthreads();

  // ---- project 32 -> 16 (+ bias, no activation) -> global
  bf16* __restrict__ y = (bf16*)p.ir_y;
  const float4 pb = *(const float4*)(p.ir_bp + kq * 4);
#pragma unroll
  for (int f = 0; f < NOUT / 64; ++f) {
    const int fr = wave * (NOUT / 64) + f;
    const bf16x8 bv = *(const bf16x8*)(Ds + ir_swz(fr * 16 + row, kq));
    f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wpa, bv, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const int q = fr * 16 + row, oy = q / T, ox = q - (q / T) * T;
    float v[4] = {acc[0] + pb.x, acc[1] + pb.y, acc[2] + pb.z, acc[3] + pb.w};
    *(uint2*)(y + ((size_t)item * S2 * S2 + (size_t)(oy0 + oy) * S2 + ox0 + ox) * p.ir_ys + kq * 4) = pack4(v);
  }
}

template <int SRC, int KS, int NF, int TH, int TW>
static void stem_launch(const StemFusedParams& p, hipStream_t s) {
  const int S2 = p.S / 2;
  const int ntiles = ((S2 + TW - 1) / TW) * ((S2 + TH - 1) / TH);
  const long blocks = (long)((p.cap + 7) / 8) * 8 * ntiles;
  hipLaunchKernelGGL((stem_fused_kernel<SRC, KS, NF, TH, TW>), dim3((unsigned)blocks), dim3(256), 0, s, p);
}

void stem_fused(const StemFusedParams& p, hipStream_t s) {
  if (p.S % 2 != 0 || p.S <= 0) throw std::runtime_error("stem_fused: S must be positive and even");
  if (p.ctrl == nullptr) throw std::runtime_error("stem_fused: needs the control block (live counts)");
  if (p.ys % 4 != 0) throw std::runtime_error("stem_fused: output pixel stride must be a multiple of 4");
  if (p.cap <= 0) return;
  if (p.src == 0) {  // YOLOv5nu: letterbox -> 6x6/s2 stem as 3x3/s1 over s2d, 16 channels, SiLU
    if (p.KS != 3 || p.Cout != 16 || p.Kpad != 160)
      throw std::runtime_error("stem_fused: detector stem must be 3x3 (s2d) x 16 -> 16, Kpad 160");
    if (p.w2 != nullptr) {
      if (p.Cout2 != 32 || p.Kpad2 != 160 || p.S % 64 != 0 || p.y2s % 4 != 0 || p.y2 == nullptr)
        throw std::runtime_error("stem_fused: second conv must be 3x3 s2 16 -> 32 (Kpad 160) with S % 64 == 0");
      const int S4 = p.S / 4;
      const long blocks = (long)((p.cap + 7) / 8) * 8 * (S4 / 8) * (S4 / 16);
      hipLaunchKernelGGL((stem2_kernel<8, 16>), dim3((unsigned)blocks), dim3(256), 0, s, p);
      return;
    }
    stem_launch<0, 3, 1, 8, 32>(p, s);
  } else if (p.src == 1) {  // MobileNetV2: crop gather -> 3x3/s2 stem as 2x2/s1 over s2d, 32 channels, ReLU6
    if (p.KS != 2 || p.Cout != 32 || p.Kpad != 64 || p.crops == nullptr)
      throw std::runtime_error("stem_fused: classifier stem must be 2x2 (s2d) x 16 -> 32, Kpad 64");
    if (p.ir_wd != nullptr) {
      if (p.S % 32 != 0 || p.ir_ys % 4 != 0 || p.ir_y == nullptr || p.ir_bd == nullptr || p.ir_wp == nullptr ||
          p.ir_bp == nullptr)
        throw std::runtime_error("stem_fused: fused first block needs S % 32 == 0 and its weights / output");
      const int S2 = p.S / 2;
      const long blocks = (long)((p.cap + 7) / 8) * 8 * (S2 / 16) * (S2 / 16);
      hipLaunchKernelGGL((stem_ir_kernel<16>), dim3((unsigned)blocks), dim3(256), 0, s, p);
      return;
    }
    stem_launch<1, 2, 2, 16, 16>(p, s);
  } else {
    throw std::runtime_error("stem_fused: unknown source");
  }
}

}  // namespace arena
