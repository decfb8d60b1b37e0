// Fused MobileNetV2 inverted residual, fp32-accurate on the bf16 matrix cores (triple-bf16 split), for the
// tiled 112x112 .. 28x28 stages (torchvision mobilenet_v2 features[2..7]; the reference runs them as fp32
// ONNX per crop, architectures/monolithic/app/inference.py:196).
//
// Same tiling and phase structure as ir_f32.hip (one workgroup = a TH x TW output tile of one crop; per chunk
// of 32 hidden channels: expand GEMM -> fp32 E tile in LDS -> depthwise -> project GEMM accumulate), but the
// two GEMMs run as six v_mfma_f32_16x16x32_bf16 per operand pair on split planes (v = h + m + l exactly, see
// conv_x3_lds_kernel) instead of v_mfma_f32_16x16x4_f32: 16 cycles per 16x16x32 step against 8 x 32 for the
// exact fp32 instruction, 2.7x less matrix time at fp32-level error (tests/test_fp32_gpu.py, fp64 reference).
//
//   X: each wave loads the input pixels of its expand tiles straight from global memory into B-operand
//      registers, split once; X never goes through LDS (ir_f32 kept a fp32 copy there);
//   E = relu6(We[chunk] . X + be), zero outside the image        -> fp32 LDS (the depthwise reads it)
//   D = relu6(dw3x3_S(E) + bd)                                    -> split, bf16 planes in LDS
//   acc += Wp[:, chunk] . D                                       registers for the whole chunk loop
//   y = acc + bp (+ x)
// Weights: the x3w planes the planner packs for these blocks (engine/planner.py split_bf16x3): we bf16
// [hid_pad][3][inp_pad], wp bf16 [oup_pad][3][hid_pad]; wd fp32 [9][hid_pad]; biases fp32.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"
#include "letterbox.h"

namespace arena {

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int ITX_HC = 32;                    // hidden channels per chunk
constexpr int ITX_DPB = 3 * ITX_HC * 2 + 32;  // bytes per D pixel row: [h|m|l][32] bf16 + pad (14 slots)

__host__ __device__ constexpr int itx_ep(int S) { return S == 1 ? ITX_HC : ITX_HC + 4; }  // E pixel pitch

template <int S>
__device__ __forceinline__ int itx_eswz(int pix, int g) {
  const int f = S == 1 ? ((pix ^ (4 * (pix >> 2))) & 7) : 0;
  return (g & ~7) | ((g & 7) ^ f);
}

__device__ __forceinline__ void itx_split8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
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

__device__ __forceinline__ void itx_split4(const float4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
  const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16 th = (bf16)a[i];
    const float r = a[i] - (float)th;
    const bf16 tm = (bf16)r;
    h[i] = th;
    m[i] = tm;
    l[i] = (bf16)(r - (float)tm);
  }
}

__device__ __forceinline__ f32x4 itx_mfma(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                          const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

__device__ __forceinline__ float4 itx_relu6x4(float4 v) {
  return make_float4(relu6f(v.x), relu6f(v.y), relu6f(v.z), relu6f(v.w));
}

}  // namespace

// S: stride; TH x TW: output tile; NTO: oup_pad / 16; KS: inp_pad / 32.
template <int S, int TH, int TW, int NTO, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KS == 1 ? 2 : 1))) void ir_tile_x3_kernel(const IrParams p) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int PIN = PH * PW, MT_IN = (PIN + 15) / 16, ROWS = MT_IN * 16;
  constexpr int POUT = TH * TW, MT_OUT = POUT / 16;
  static_assert(POUT % 16 == 0, "output tile must be a multiple of 16 pixels");
  constexpr int PAIRS = MT_OUT * NTO, PPW = (PAIRS + 3) / 4;
  constexpr int ET = (MT_IN * 2 + 3) / 4;  // expand tiles per wave (pixel tile x hidden half)
  constexpr int EP = itx_ep(S);
  constexpr int INP = KS * 32;
  extern __shared__ __attribute__((aligned(16))) uint8_t itx_lds[];
  float* Es = (float*)itx_lds;                            // [ROWS][EP] fp32
  uint8_t* Ds = itx_lds + ROWS * EP * sizeof(float);      // [POUT][ITX_DPB] bf16 planes
  float* Wd = (float*)(Ds + POUT * ITX_DPB);              // [10][hid_pad]: depthwise taps 0..8, bias

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles = tiles_x * tiles_y;
  const int b = blockIdx.x / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = blockIdx.x - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const float* xb = (const float*)p.x + (size_t)b * p.H * p.W * p.x_cs;
  const bf16* we = (const bf16*)p.we;
  const bf16* wp = (const bf16*)p.wp;
  const float* wd = (const float*)p.wd;
  const int hid_pad = p.hid_pad;

  // ---- this wave's expand tiles: tile tt = wave + 4 i covers halo pixels 16 (tt >> 1) .. +15 and hidden
  // half tt & 1 = wave & 1; the pixels' channels are loaded once, split, and stay in registers
  const int nt_e = wave & 1;
  bf16x8 xh[ET][KS], xm[ET][KS], xl[ET][KS];
  float xin[ET];  // 1: the lane's halo pixel is inside the image (the expanded map is zero-padded)
#pragma unroll
  for (int i = 0; i < ET; ++i) {
    const int tt = wave + 4 * i;
    const int r = (tt >> 1) * 16 + col;
    const int iy = iy0 + r / PW, ix = ix0 + r % PW;
    const bool in = tt < MT_IN * 2 && r < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    xin[i] = in ? 1.f : 0.f;
    const float* src = xb + ((size_t)(in ? iy : 0) * p.W + (in ? ix : 0)) * p.x_cs;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + 8 * kq;
      const bool ok = in && k < p.inp;
      const float4 a = *(const float4*)(src + (ok ? k : 0)), c = *(const float4*)(src + (ok ? k + 4 : 0));
      float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      if (!ok) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      } else if (k + 4 > p.inp) {  // inp % 8 == 4: the upper half of this 8-channel group is padding
#pragma unroll
        for (int j = 4; j < 8; ++j) v[j] = 0.f;
      }
      itx_split8(v, xh[i][ks], xm[i][ks], xl[i][ks]);
    }
  }

  f32x4 acc[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Weights of chunk c + 1 are fetched into registers while chunk c runs (expand: A operand, hidden row h0 +
  // 16 nt_e + col, k 8 kq of each 32-step; project: A operand, output row 16 nt_p + col, hidden k h0 + 8 kq).
  // The prefetch is unconditional (the last chunk re-fetches itself): a conditional one made the wait at the
  // loop head conservative, and the MFMAs then waited for the loads just issued.  The depthwise taps and bias of
  // every chunk are staged in LDS once (Wd [10][hid_pad]): read at the chunk's depthwise they cost an LDS round
  // trip instead of a global one behind the barrier.
  static_assert(NTO == 1 || NTO == 2 || NTO == 4, "a wave's project pairs share one output-channel tile");
  const int nt_p = wave % NTO;
  u32x4 wexp[3 * KS], wnext[3 * KS], wprj[3], wprj_n[3];
  float4 bexp, bnext;
  auto load_expand = [&](int h0, u32x4 (&w)[3 * KS], float4& be) {
    const bf16* row = we + (size_t)(h0 + nt_e * 16 + col) * 3 * INP + 8 * kq;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) w[ks * 3 + pl] = *(const u32x4*)(row + pl * INP + ks * 32);
    be = *(const float4*)((const float*)p.be + h0 + nt_e * 16 + 4 * kq);
  };
  auto load_project = [&](int h0, u32x4 (&w)[3]) {
    const bf16* row = wp + (size_t)(nt_p * 16 + col) * 3 * hid_pad + h0 + 8 * kq;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) w[pl] = *(const u32x4*)(row + pl * hid_pad);
  };
  for (int i = tid; i < 10 * hid_pad / 4; i += 256) {
    const int r = i / (hid_pad / 4), c4 = i - r * (hid_pad / 4);
    const float* src = r < 9 ? wd + (size_t)r * hid_pad : (const float*)p.bd;
    *(float4*)&Wd[r * hid_pad + 4 * c4] = *(const float4*)(src + 4 * c4);
  }
  const int g = tid & 7;  // depthwise channel group (4 channels) of this thread
  load_expand(0, wexp, bexp);
  load_project(0, wprj);

  for (int h0 = 0; h0 < hid_pad; h0 += ITX_HC) {
    const int hn = h0 + ITX_HC < hid_pad ? h0 + ITX_HC : h0;
    load_expand(hn, wnext, bnext);
    load_project(hn, wprj_n);
    // ---- expand: E = relu6(We . X + be) * inside, fp32 into LDS
#pragma unroll
    for (int i = 0; i < ET; ++i) {
      const int tt = wave + 4 * i;
      if (tt >= MT_IN * 2) break;
      f32x4 e = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        e = itx_mfma(__builtin_bit_cast(bf16x8, wexp[ks * 3]), __builtin_bit_cast(bf16x8, wexp[ks * 3 + 1]),
                     __builtin_bit_cast(bf16x8, wexp[ks * 3 + 2]), xh[i][ks], xm[i][ks], xl[i][ks], e);
      const int pix = (tt >> 1) * 16 + col;
      const int hc = nt_e * 16 + 4 * kq;
      // the lane holds hidden channels hc..hc+3 of pixel `pix` (16x16 output layout); its own inside flag
      // belongs to pixel 16 (tt >> 1) + col, the same pixel
      const float m = xin[i];
      const float4 v = make_float4(relu6f(e[0] + bexp.x) * m, relu6f(e[1] + bexp.y) * m,
                                   relu6f(e[2] + bexp.z) * m, relu6f(e[3] + bexp.w) * m);
      *(float4*)&Es[pix * EP + 4 * itx_eswz<S>(pix, hc >> 2)] = v;
    }
    __syncthreads();

    // ---- depthwise 3x3 (stride S) + bias + ReLU6 -> split planes of D
    {
      float4 wk[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) wk[k] = *(const float4*)&Wd[k * hid_pad + h0 + 4 * g];
      const float4 bdw = *(const float4*)&Wd[9 * hid_pad + h0 + 4 * g];
      static_assert(POUT % 32 == 0, "depthwise: whole passes of 32 pixels");
      // all nine taps' LDS reads of a pixel are issued before its FMAs (one address each, computed up front):
      // with the reads interleaved into the FMA chain the compiler reused one register set and waited for
      // every read in turn (nine serialised LDS round trips per pixel)
#pragma unroll 1
      for (int qi = 0; qi < POUT / 32; ++qi) {  // not unrolled: 36 tap addresses would stay live over the chunk loop
        const int q = (tid >> 3) + 32 * qi;
        const int oy = q / TW, ox = q - oy * TW;
        int addr[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int px = (oy * S + t / 3) * PW + ox * S + t % 3;
          addr[t] = px * EP + 4 * itx_eswz<S>(px, g);
        }
        float4 v[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) v[t] = *(const float4*)&Es[addr[t]];
        float4 a = bdw;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float4 w = wk[t];
          a.x = fmaf(v[t].x, w.x, a.x);
          a.y = fmaf(v[t].y, w.y, a.y);
          a.z = fmaf(v[t].z, w.z, a.z);
          a.w = fmaf(v[t].w, w.w, a.w);
        }
        bf16x4 dh, dm, dl;
        itx_split4(itx_relu6x4(a), dh, dm, dl);
        uint8_t* d = Ds + q * ITX_DPB + 8 * g;
        *(bf16x4*)d = dh;
        *(bf16x4*)(d + 64) = dm;
        *(bf16x4*)(d + 128) = dl;
      }
    }
    __syncthreads();

    // ---- project GEMM accumulate (rows = output channels, columns = output pixels)
    {
      const bf16x8 ah = __builtin_bit_cast(bf16x8, wprj[0]), am = __builtin_bit_cast(bf16x8, wprj[1]),
                   al = __builtin_bit_cast(bf16x8, wprj[2]);
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int pr = wave + 4 * j;
        if (pr >= PAIRS) break;
        const int mt = pr / NTO;
        const uint8_t* d = Ds + (mt * 16 + col) * ITX_DPB + 16 * kq;
        acc[j] = itx_mfma(ah, am, al, *(const bf16x8*)d, *(const bf16x8*)(d + 64), *(const bf16x8*)(d + 128), acc[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < 3 * KS; ++k) wexp[k] = wnext[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) wprj[k] = wprj_n[k];
    bexp = bnext;
    // no barrier here: the next chunk's expand writes E, which every wave finished reading before the
    // barrier above, and its depthwise writes D only after the next expand barrier, which every wave reaches
    // after this project
  }

  // ---- epilogue: + bias (+ residual) -> NHWC fp32
  float* yb = (float*)p.y + (size_t)b * p.Ho * p.Wo * p.y_cs;
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int pr = wave + 4 * j;
    if (pr >= PAIRS) break;
    const int mt = pr / NTO, nt = pr - mt * NTO;
    const int q = mt * 16 + col;
    const int oy = oy0 + q / TW, ox = ox0 + q % TW;
    const int co = nt * 16 + 4 * kq;
    if (oy >= p.Ho || ox >= p.Wo || co >= p.oup) continue;
    const float4 bp = *(const float4*)((const float*)p.bp + co);
    float4 v = make_float4(acc[j][0] + bp.x, acc[j][1] + bp.y, acc[j][2] + bp.z, acc[j][3] + bp.w);
    if (p.res) {
      const float4 r = *(const float4*)(xb + ((size_t)oy * p.W + ox) * p.x_cs + co);
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    *(float4*)(yb + ((size_t)oy * p.Wo + ox) * p.y_cs + co) = v;
  }
}


// Classifier front end on the same operand scheme (IrParams.stem with x3w): crop gather into a space-to-depth
// tile of uint8 values (one exact bf16 plane in LDS; the ImageNet normalisation is folded into the weights and
// per-tap constants, see A1), the 2x2 stem conv (32 <- 4 taps x 16 channels) as three MFMAs per K step -> fp32 X
// (+ bias, ReLU6, zero outside the 112 x 112 map), MobileNetV2 block 1 (t = 1: depthwise 32 + ReLU6 on X, project
// 32 -> 16 as x3 MFMAs).  ir_f32.hip's stem mode ran both GEMMs on v_mfma_f32_16x16x4_f32: the stem conv over the
// 1.41x halo alone was ~110 us of matrix time per batch of 32 requests.
// Weights: st_w bf16 [32][3][64] (k = tap * 16 + channel; w / (255 std_c)), st_b fp32 [32 bias][4 taps][32]
// (mean constants), wp bf16 [16][3][32], wd fp32 [9][32], biases fp32 (engine/planner.py ir_block_stem).
__global__ __launch_bounds__(256) void ir_stem_x3_kernel(const IrParams p) {
  constexpr int S = 1, TH = 8, TW = 16;
  constexpr int PH = TH + 2, PW = TW + 2, PIN = PH * PW, MT_IN = (PIN + 15) / 16, ROWS = MT_IN * 16;
  constexpr int POUT = TH * TW, MT_OUT = POUT / 16;
  constexpr int PAIRS = MT_OUT, PPW = (PAIRS + 3) / 4;  // one 16-channel output tile
  constexpr int ET = (MT_IN * 2 + 3) / 4;
  constexpr int XP = 32;                              // X pixel pitch (fp32): the depthwise input
  constexpr int SH = PH + 1, SW = PW + 1, SPB = 96;   // s2d tile: [pixel][h 16 | m 16 | l 16] bf16
  static_assert(SH * SW * SPB <= POUT * ITX_DPB, "s2d tile must fit the D region");
  extern __shared__ __attribute__((aligned(16))) uint8_t itx_lds[];
  float* Xs = (float*)itx_lds;                        // [ROWS][XP] fp32, swizzled 4-channel groups
  uint8_t* Ds = itx_lds + ROWS * XP * sizeof(float);  // [POUT][ITX_DPB] bf16 planes (first: the s2d tile)
  uint8_t* Ss = Ds;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int tiles = tiles_x * tiles_y;
  const int b = blockIdx.x / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = blockIdx.x - b * tiles;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 - 1, ix0 = ox0 - 1;

  // Every weight / constant of the three GEMM phases is requested here, before the gather: fetched at the head of
  // each phase (after its barrier), they were three serial global round trips per workgroup.
  const int nt = wave & 1;  // this wave's 16 stem output channels (A2)
  u32x4 ws[6];
  {
    const bf16* wrow = (const bf16*)p.st_w + (size_t)(nt * 16 + col) * 3 * 64 + 8 * kq;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) ws[ks * 3 + pl] = *(const u32x4*)(wrow + pl * 64 + ks * 32);
  }
  const float4 bb = *(const float4*)(p.st_b + nt * 16 + 4 * kq);
  float4 ct[4];  // per-tap mean constants of this lane's 4 stem channels
#pragma unroll
  for (int tp = 0; tp < 4; ++tp) ct[tp] = *(const float4*)(p.st_b + 32 + tp * 32 + nt * 16 + 4 * kq);
  const int g = tid & 7;  // depthwise channel group (4 channels) of this thread
  float4 wk[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wk[k] = *(const float4*)((const float*)p.wd + (size_t)k * 32 + 4 * g);
  const float4 bdw = *(const float4*)((const float*)p.bd + 4 * g);
  const bf16* wprow = (const bf16*)p.wp + (size_t)col * 3 * 32 + 8 * kq;
  const bf16x8 pah = *(const bf16x8*)wprow, pam = *(const bf16x8*)(wprow + 32), pal = *(const bf16x8*)(wprow + 64);
  const float4 bpv = *(const float4*)((const float*)p.bp + 4 * kq);

  // ---- A1: crop gather -> s2d tile (origin (iy0 - 1, ix0 - 1): the 2x2 stem conv pads top / left by one).
  // The crop resize returns uint8 values k (cv2 INTER_LINEAR, bilinear_rgb), and the normalised input
  // (k / 255 - mean_c) / std_c is affine in k: the planner folds 1 / (255 std_c) into the stem weights and the
  // mean into per-tap constants (st_b[32 + 32 tap + co] = -sum_c w[co][tap][c] mean_c / std_c), so the tile holds
  // k itself, exact in one bf16 plane: three MFMAs per K step instead of six, no normalisation or split
  // arithmetic per pixel.  Outside the crop map the tile is zero and the tap's constant is not added (the
  // normalised input is zero-padded).
  {
    const int S2 = p.st_S >> 1;
    const CropRef cr = p.st_crops[(p.st_ctrl != nullptr ? p.st_ctrl->crop_base : 0) + b];
    const ImageMeta m = p.st_meta[cr.img];
    const int cw = cr.x2 - cr.x1, chh = cr.y2 - cr.y1;
    const bool empty = cw <= 0 || chh <= 0;
    const float sx = empty ? 1.f : (float)((double)cw / (double)p.st_S);
    const float sy = empty ? 1.f : (float)((double)chh / (double)p.st_S);
    const uint8_t* img = p.st_pool + m.offset + ((size_t)cr.y1 * m.w + cr.x1) * 3;
    for (int i = tid; i < SH * SW; i += 256) {
      const int Y = iy0 - 1 + i / SW, X = ix0 - 1 + i % SW;
      float out[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) out[k] = 0.f;
      if ((unsigned)Y < (unsigned)S2 && (unsigned)X < (unsigned)S2 && !empty) {
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int oy = 2 * Y + (pq >> 1), ox = 2 * X + (pq & 1);
          bilinear_rgb(img, m.w, lin_tap(oy, sy, chh), lin_tap(ox, sx, cw), out + pq * 3);
        }
      }
      bf16x8 h0, h1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        h0[k] = (bf16)out[k];
        h1[k] = (bf16)out[k + 8];
      }
      uint8_t* d = Ss + i * SPB;
      *(bf16x8*)d = h0;
      *(bf16x8*)(d + 16) = h1;
    }
  }
  __syncthreads();

  // ---- A2: X = relu6(stem(s2d) + b) over the halo tile (x3 MFMAs, K = 2 steps of 32), zero outside the map
  {
    const int S2 = p.st_S >> 1;
#pragma unroll
    for (int i = 0; i < ET; ++i) {
      const int tt = wave + 4 * i;
      if (tt >= MT_IN * 2) break;
      const int r = (tt >> 1) * 16 + col;
      const int rr = r < PIN ? r : 0;
      const int ry = rr / PW, rx = rr - (rr / PW) * PW;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int tap = ks * 2 + (kq >> 1);
        const uint8_t* sp = Ss + ((ry + (tap >> 1)) * SW + rx + (tap & 1)) * SPB + (kq & 1) * 16;
        const bf16x8 xk = *(const bf16x8*)sp;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ws[ks * 3 + 2]), xk, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ws[ks * 3 + 1]), xk, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ws[ks * 3]), xk, acc, 0, 0, 0);
      }
      // lane (col, kq) holds stem channels 16 nt + 4 kq .. +3 of halo pixel r; add the constants of the taps
      // whose s2d pixel is inside the map
      float4 cs = bb;
#pragma unroll
      for (int tp = 0; tp < 4; ++tp) {
        const int Ys = iy0 - 1 + ry + (tp >> 1), Xs = ix0 - 1 + rx + (tp & 1);
        const float in_t = (unsigned)Ys < (unsigned)S2 && (unsigned)Xs < (unsigned)S2 ? 1.f : 0.f;
        cs.x += in_t * ct[tp].x;
        cs.y += in_t * ct[tp].y;
        cs.z += in_t * ct[tp].z;
        cs.w += in_t * ct[tp].w;
      }
      const int co = nt * 16 + 4 * kq;
      const int iy = iy0 + ry, ix = ix0 + rx;
      const bool in = r < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const float4 v = in ? itx_relu6x4(make_float4(acc[0] + cs.x, acc[1] + cs.y, acc[2] + cs.z, acc[3] + cs.w))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)&Xs[r * XP + 4 * itx_eswz<S>(r, co >> 2)] = v;
    }
  }
  __syncthreads();  // X complete; the s2d tile is dead (its space becomes D)

  // ---- depthwise 3x3 on X (t = 1: X is the hidden map) + bias + ReLU6 -> split planes of D
  {
#pragma unroll 1
    for (int qi = 0; qi < POUT / 32; ++qi) {  // reads issued ahead of the FMAs, as in ir_tile_x3_kernel
      const int q = (tid >> 3) + 32 * qi;
      const int oy = q / TW, ox = q - oy * TW;
      int addr[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int px = (oy + t / 3) * PW + ox + t % 3;
        addr[t] = px * XP + 4 * itx_eswz<S>(px, g);
      }
      float4 v[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) v[t] = *(const float4*)&Xs[addr[t]];
      float4 a = bdw;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 w = wk[t];
        a.x = fmaf(v[t].x, w.x, a.x);
        a.y = fmaf(v[t].y, w.y, a.y);
        a.z = fmaf(v[t].z, w.z, a.z);
        a.w = fmaf(v[t].w, w.w, a.w);
      }
      bf16x4 dh, dm, dl;
      itx_split4(itx_relu6x4(a), dh, dm, dl);
      uint8_t* d = Ds + q * ITX_DPB + 8 * g;
      *(bf16x4*)d = dh;
      *(bf16x4*)(d + 64) = dm;
      *(bf16x4*)(d + 128) = dl;
    }
  }
  __syncthreads();

  // ---- project 32 -> 16 (x3 MFMAs) + bias -> NHWC fp32
  float* yb = (float*)p.y + (size_t)b * p.Ho * p.Wo * p.y_cs;
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int mt = wave + 4 * j;
    if (mt >= PAIRS) break;
    const uint8_t* d = Ds + (mt * 16 + col) * ITX_DPB + 16 * kq;
    const f32x4 acc = itx_mfma(pah, pam, pal, *(const bf16x8*)d, *(const bf16x8*)(d + 64), *(const bf16x8*)(d + 128),
                               f32x4{0.f, 0.f, 0.f, 0.f});
    const int q = mt * 16 + col;
    const int oy = oy0 + q / TW, ox = ox0 + q % TW;
    const int co = 4 * kq;
    if (oy >= p.Ho || ox >= p.Wo || co >= p.oup) continue;
    *(float4*)(yb + ((size_t)oy * p.Wo + ox) * p.y_cs + co) =
        make_float4(acc[0] + bpv.x, acc[1] + bpv.y, acc[2] + bpv.z, acc[3] + bpv.w);
  }
}

namespace {

template <int S, int TH, int TW, int NTO, int KS>
void itx_launch(const IrParams& p, hipStream_t s) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int ROWS = (PH * PW + 15) / 16 * 16;
  constexpr size_t lds0 = (size_t)ROWS * itx_ep(S) * 4 + (size_t)TH * TW * ITX_DPB;
  const size_t lds = lds0 + (size_t)10 * p.hid_pad * 4;  // + the depthwise taps / bias of every chunk
  if (lds > 160 * 1024) throw std::runtime_error("ir_tile_x3: LDS budget exceeded (hid_pad " + std::to_string(p.hid_pad) + ")");
  const int tiles = ((p.Wo + TW - 1) / TW) * ((p.Ho + TH - 1) / TH);
  hipLaunchKernelGGL((ir_tile_x3_kernel<S, TH, TW, NTO, KS>), dim3((unsigned)(p.B * tiles)), dim3(256), lds, s, p);
}

// (S, TH, TW, NTO, KS): stride-1 blocks on 8 x 16 tiles, stride-2 blocks on 4 x 8 tiles (as ir_f32.hip)
#define ITX_CONFIGS(X) \
  X(1, 8, 16, 1, 1)    \
  X(1, 8, 16, 2, 1)    \
  X(1, 8, 16, 4, 1)    \
  X(1, 8, 16, 2, 2)    \
  X(1, 8, 16, 4, 2)    \
  X(2, 4, 8, 1, 1)     \
  X(2, 4, 8, 2, 1)     \
  X(2, 4, 8, 4, 1)     \
  X(2, 4, 8, 4, 2)

}  // namespace

// Shapes this kernel takes (mirrored by engine/validate.py::ir_tile_x3_supported): expanding blocks with
// inp_pad 32 / 64, hid_pad a multiple of 32 and oup_pad 16 / 32 / 64 (stride-2: 16 .. 64, and 64 with inp 64).
bool ir_tile_x3_supported(int stride, int inp_pad, int hid_pad, int oup_pad, int expand) {
  if (!expand || hid_pad % ITX_HC) return false;
#define X(S_, TH_, TW_, NTO_, KS_) \
  if (stride == S_ && oup_pad == NTO_ * 16 && inp_pad == KS_ * 32) return true;
  ITX_CONFIGS(X)
#undef X
  return false;
}

constexpr size_t kStemX3Lds = (size_t)((10 * 18 + 15) / 16 * 16) * 32 * 4 + (size_t)8 * 16 * ITX_DPB;

bool ir_stem_x3(const IrParams& p, hipStream_t s) {
  if (!p.stem || !p.x3w) return false;
  if (p.stride != 1 || p.expand || p.res || p.inp != 32 || p.inp_pad != 32 || p.hid_pad != 32 || p.oup_pad != 16 ||
      p.oup > 16 || p.oup % 4 || p.H != p.W || p.H * 2 != p.st_S || p.Ho != p.H || p.Wo != p.W || p.W < 16 ||
      p.y_cs % 4 || p.st_w == nullptr || p.st_b == nullptr || p.st_crops == nullptr || p.st_meta == nullptr ||
      p.st_pool == nullptr)
    throw std::runtime_error("ir_stem_x3: unsupported geometry (needs MobileNetV2 block 1 at S/2 x S/2)");
  if (p.B <= 0) return true;
  const int tiles = ((p.Wo + 15) / 16) * ((p.Ho + 7) / 8);
  hipLaunchKernelGGL(ir_stem_x3_kernel, dim3((unsigned)(p.B * tiles)), dim3(256), kStemX3Lds, s, p);
  return true;
}

void ir_tile_x3_prepare() {
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_stem_x3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
#define X(S_, TH_, TW_, NTO_, KS_)                                                                       \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_tile_x3_kernel<S_, TH_, TW_, NTO_, KS_>,           \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ITX_CONFIGS(X)
#undef X
}

bool ir_tile_x3(const IrParams& p, hipStream_t s) {
  if (!ir_tile_x3_supported(p.stride, p.inp_pad, p.hid_pad, p.oup_pad, p.expand)) return false;
  if (p.inp % 4 || p.oup % 4 || p.inp > p.inp_pad || p.oup > p.oup_pad || p.x_cs % 4 || p.y_cs % 4)
    throw std::runtime_error("ir_tile_x3: unsupported channel geometry");
  if (p.res && (p.stride != 1 || p.inp != p.oup)) throw std::runtime_error("ir_tile_x3: residual needs s1, inp == oup");
  if (p.Ho != (p.H + 2 - 3) / p.stride + 1 || p.Wo != (p.W + 2 - 3) / p.stride + 1)
    throw std::runtime_error("ir_tile_x3: output size mismatch");
  if (p.B <= 0) return true;
#define X(S_, TH_, TW_, NTO_, KS_)                                                  \
  if (p.stride == S_ && p.oup_pad == NTO_ * 16 && p.inp_pad == KS_ * 32) {          \
    itx_launch<S_, TH_, TW_, NTO_, KS_>(p, s);                                      \
    return true;                                                                    \
  }
  ITX_CONFIGS(X)
#undef X
  return false;
}

}  // namespace arena
