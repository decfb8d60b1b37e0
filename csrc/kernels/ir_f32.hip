// Fused MobileNetV2 inverted residual in exact fp32 (the fp32 counterpart of
// ir_block.hip).  Reference computation (ONNX Runtime fp32 per crop,
// architectures/monolithic/app/inference.py:196 running torchvision's
// mobilenet_v2): Conv1x1+BN+Clip (expand) -> depthwise Conv3x3+BN+Clip ->
// Conv1x1+BN (project) [-> Add].
//
// Unfused, the fp32 expanded tensor of the 112x112 blocks is 112x112x96x4 B =
// 4.8 MB per crop and crosses HBM twice; the profile of the unfused fp32
// program put the >= 28x28 MobileNetV2 blocks at ~1.7 ms per batch of 32
// requests (profiles/r2_fp32_lds_ops.md), almost all memory traffic.  Here one
// workgroup owns a TH x TW output tile of one crop:
//
//   X halo tile ((TH-1)*S+3 x (TW-1)*S+3 pixels, zero outside the image) ... LDS
//   for each chunk of 32 hidden channels:
//     E = relu6(X . We^T + be), zeroed outside the image   v_mfma_f32_16x16x4_f32 -> LDS
//         (the depthwise conv pads the *expanded* map with zeros)
//     D = relu6(dw3x3_S(E) + bd)                            fp32 FMA (VALU)          -> LDS
//     acc += Wp[:, chunk] . D                               v_mfma_f32_16x16x4_f32, registers
//   y = acc + bp (+ x)                                      fp32 NHWC, 16-byte stores
//
// Operand reads use the float4-per-lane k mapping of conv_f32.hip (lane l holds
// k = 4*(l>>4) .. +3 of a 16-deep K chunk, consumed by four MFMAs).
//
// LDS layouts (ds_read_b128 serves 16-lane groups from one 256-B bank row of
// 16 slots of 16 B; MI355X_MICROARCH.md §LDS), measured 38-45 % bank-conflict
// cycles with the previous odd-slot pitches (profiles/r2_fp32_pmc_ops.md):
//   * MFMA operand rows (X for the expand GEMM, D for the project GEMM): lanes
//     read 16 rows x 4 k-groups, conflict-free when the row pitch is 2 (mod 4)
//     slots: K + 8 floats;
//   * the expanded chunk E (and X of a t = 1 block, which the depthwise reads
//     directly): the depthwise reads 8 lanes per pixel, and the expand epilogue
//     writes 16 pixels x 4 groups; 32 floats per pixel with the group index
//     XOR-swizzled by (p ^ 4*(p>>2)) & 7 at stride 1 makes the depthwise reads
//     conflict-free at the cost of a 2-way conflict on the (6x rarer) epilogue
//     writes; at stride 2 the conflict-free layout (48 floats) cost more in
//     occupancy than it saved, so E keeps 36 floats there.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"
#include "letterbox.h"

namespace arena {

namespace {

constexpr int IRF_HC = 32;            // hidden channels per chunk
constexpr int IRF_DP = IRF_HC + 8;    // D row pitch (floats): MFMA operand rows
__host__ __device__ constexpr int irf_ep(int S) { return S == 1 ? IRF_HC : IRF_HC + 4; }  // E pixel pitch
__host__ __device__ constexpr int irf_xp(int inp_pad, bool expand) { return expand ? inp_pad + 8 : inp_pad; }

// swizzled 4-channel group of pixel `pix` in E (and in X of a t = 1 block)
template <int S>
__device__ __forceinline__ int eswz(int pix, int g) {
  const int f = S == 1 ? ((pix ^ (4 * (pix >> 2))) & 7) : 0;
  return (g & ~7) | ((g & 7) ^ f);
}

__device__ __forceinline__ float f4c(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

__device__ __forceinline__ float4 relu6x4(float4 v) {
  return make_float4(relu6f(v.x), relu6f(v.y), relu6f(v.z), relu6f(v.w));
}

}  // namespace

// STEM (classifier front end, t = 1 block 1 only): X is the 2x2 stem conv of the crop-gathered space-to-depth
// tile, computed here (IrParams.stem); the s2d tile and the 112 x 112 x 32 stem map never leave LDS.
template <int S, int TH, int TW, int NTO, bool EXPAND, int KIN, bool STEM = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(S == 2 && KIN == 1 && NTO <= 4 ? 3 : 1))) void ir_f32_kernel(const IrParams p) {
  constexpr int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  constexpr int PIN = PH * PW, MT_IN = (PIN + 15) / 16, ROWS = MT_IN * 16;
  constexpr int POUT = TH * TW, MT_OUT = POUT / 16;
  static_assert(POUT % 16 == 0, "output tile must be a multiple of 16 pixels");
  constexpr int PAIRS = MT_OUT * NTO, PPW = (PAIRS + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) float irf_lds[];
  constexpr int EP = irf_ep(S);
  const int XP = irf_xp(p.inp_pad, EXPAND);
  float* Xs = irf_lds;                                   // [ROWS][XP]
  float* Es = Xs + ROWS * XP;                            // [ROWS][EP] (EXPAND)
  float* Ds = Es + (EXPAND ? ROWS * EP : 0);             // [POUT][IRF_DP]
  float* Ms = Ds + POUT * IRF_DP;                        // [ROWS] 1 inside the image, 0 outside

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
  const float* xb = STEM ? nullptr : (const float*)p.x + (size_t)b * p.H * p.W * p.x_cs;
  const float* we = (const float*)p.we;
  const float* wd = (const float*)p.wd;
  const float* wp = (const float*)p.wp;

  // ---- A: the input halo tile (channels >= inp and pixels outside the image are zero)
  if constexpr (STEM) {
    static_assert(S == 1 && !EXPAND, "the fused stem feeds a stride-1 t = 1 block");
    // A1: crop gather -> s2d tile (SH x SW pixels of 16 fp32, origin (iy0 - 1, ix0 - 1): the 2x2 stem conv
    // pads the s2d map top / left by one), exactly as crop_gather_s2d_kernel<float> computes each pixel
    constexpr int SH = PH + 1, SW = PW + 1, SP = 20;
    static_assert(SH * SW * SP <= POUT * IRF_DP, "s2d tile must fit the D region");
    float* Ss = Ds;
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
      if ((unsigned)Y < (unsigned)S2 && (unsigned)X < (unsigned)S2) {
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int oy = 2 * Y + (pq >> 1), ox = 2 * X + (pq & 1);
          float rgb[3] = {0.f, 0.f, 0.f};
          if (!empty) bilinear_rgb(img, m.w, lin_tap(oy, sy, chh), lin_tap(ox, sx, cw), rgb);
#pragma unroll
          for (int c = 0; c < 3; ++c) out[pq * 3 + c] = (div255<float>(rgb[c]) - p.st_mean[c]) * p.st_inv_std[c];
        }
      }
      float* d = Ss + i * SP;
#pragma unroll
      for (int k = 0; k < 16; k += 4) *(float4*)(d + k) = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
    }
    __syncthreads();
    // A2: X = relu6(stem(s2d) + b) on the halo pixels (exact fp32 MFMA, K = 4 taps x 16), zero outside the map
    for (int pr = wave; pr < MT_IN * 2; pr += 4) {
      const int mt = pr >> 1, nt = pr & 1;
      const int r = mt * 16 + col;
      const int rr = r < PIN ? r : 0;
      const int ry = rr / PW, rx = rr - (rr / PW) * PW;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 bv = *(const float4*)(Ss + ((ry + (t >> 1)) * SW + rx + (t & 1)) * SP + 4 * kq);
        const float4 av = *(const float4*)(p.st_w + (size_t)(nt * 16 + col) * 64 + t * 16 + 4 * kq);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(av, s4), f4c(bv, s4), acc, 0, 0, 0);
      }
      const int co = nt * 16 + 4 * kq;
      const float4 bb = *(const float4*)(p.st_b + co);
      const int iy = iy0 + ry, ix = ix0 + rx;
      const bool in = r < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const float4 v = in ? relu6x4(make_float4(acc[0] + bb.x, acc[1] + bb.y, acc[2] + bb.z, acc[3] + bb.w))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)&Xs[r * XP + 4 * eswz<S>(r, co >> 2)] = v;
    }
  } else {
    const int cg = p.inp_pad >> 2;
    for (int i = tid; i < ROWS * cg; i += 256) {
      const int r = i / cg, g = i - r * cg;
      const int iy = iy0 + r / PW, ix = ix0 + r % PW;
      const bool in = r < PIN && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in && 4 * g < p.inp) v = *(const float4*)(xb + ((size_t)iy * p.W + ix) * p.x_cs + 4 * g);
      *(float4*)&Xs[r * XP + 4 * (EXPAND ? g : eswz<S>(r, g))] = v;
      if (g == 0) Ms[r] = in ? 1.f : 0.f;
    }
  }
  __syncthreads();

  f32x4 acc[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Per-chunk weights live in registers and are fetched one phase ahead of their use (the first
  // version read them from global memory inside each MFMA tile loop and waited on every fetch):
  //   expand weights/bias of chunk h+1 and depthwise taps/bias of chunk h+1 during chunk h's project GEMM,
  //   project weights of chunk h during chunk h's depthwise.
  // A wave's expand tiles all share one hidden-channel half (tt = wave + 4i keeps tt & 1 = wave & 1), so
  // its expand weights are one row per lane; its ET tiles run as interleaved accumulation chains.
  constexpr int KIN_MAX = KIN;                   // inp_pad / 16 (a template parameter: a runtime bound kept
                                                 // every unrolled k-step's registers live)
  constexpr int ET = (MT_IN * 2 + 3) / 4;        // expand tiles per wave
  const int nt_e = wave & 1;
  const int g = tid & 7;                         // depthwise channel group of this thread
  float4 wexp[KIN_MAX], bexp, wk[9], bdw, wprj[PPW][2];
  auto load_expand = [&](int h0) {
#pragma unroll
    for (int kc = 0; kc < KIN_MAX; ++kc)
        wexp[kc] = *(const float4*)(we + (size_t)(h0 + nt_e * 16 + col) * p.inp_pad + 16 * kc + 4 * kq);
    bexp = *(const float4*)((const float*)p.be + h0 + nt_e * 16 + 4 * kq);
  };
  auto load_dw = [&](int h0) {
#pragma unroll
    for (int k = 0; k < 9; ++k) wk[k] = *(const float4*)(wd + (size_t)k * p.hid_pad + h0 + 4 * g);
    bdw = *(const float4*)((const float*)p.bd + h0 + 4 * g);
  };
  auto load_project = [&](int h0) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      // branch-free (a wave past the last pair re-reads a valid row it never uses): a divergent branch here
      // left the wait before the project MFMAs conservative, so they waited for the next chunk's prefetch too
      const int pr = wave + 4 * j < PAIRS ? wave + 4 * j : PAIRS - 1;
      const int nt = pr % NTO;
      const float* wrow = wp + (size_t)(nt * 16 + col) * p.hid_pad + h0 + 4 * kq;
      wprj[j][0] = *(const float4*)wrow;
      wprj[j][1] = *(const float4*)(wrow + 16);
    }
  };
  // Holding the next chunk's 9 depthwise taps across the project GEMM costs 40 VGPRs: at stride 1 (8x8
  // tiles, 3 blocks per CU by LDS) that dropped occupancy and measured slower, so there they load at use.
  constexpr bool PREFETCH_DW = S == 2;
  if constexpr (EXPAND) load_expand(0);
  if constexpr (PREFETCH_DW) load_dw(0);

  for (int h0 = 0; h0 < p.hid_pad; h0 += IRF_HC) {
    const int hn = h0 + IRF_HC < p.hid_pad ? h0 + IRF_HC : h0;  // the last chunk re-fetches itself: no branch
    // ---- B: expand GEMM for this chunk, rows = hidden channel, columns = halo pixel
    const float* E;
    int ep;
    if constexpr (EXPAND) {
      f32x4 e[ET];
#pragma unroll
      for (int i = 0; i < ET; ++i) e[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KIN_MAX; ++kc) {
#pragma unroll
        for (int i = 0; i < ET; ++i) {
          const int tt = wave + 4 * i;
          if (tt >= MT_IN * 2) break;
          const float4 bb = *(const float4*)(Xs + ((tt >> 1) * 16 + col) * XP + 16 * kc + 4 * kq);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(wexp[kc], s4), f4c(bb, s4), e[i], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < ET; ++i) {
        const int tt = wave + 4 * i;
        if (tt >= MT_IN * 2) break;
        const int pix = (tt >> 1) * 16 + col;
        const int hc = nt_e * 16 + 4 * kq;
        const float m = Ms[pix];
        const float4 v = make_float4(relu6f(e[i][0] + bexp.x) * m, relu6f(e[i][1] + bexp.y) * m,
                                     relu6f(e[i][2] + bexp.z) * m, relu6f(e[i][3] + bexp.w) * m);
        *(float4*)&Es[pix * EP + 4 * eswz<S>(pix, hc >> 2)] = v;
      }
      __syncthreads();
      E = Es;
      ep = EP;
    } else {
      E = Xs + h0;  // t = 1 block: the depthwise runs on the input channels themselves
      ep = XP;
    }
    load_project(h0);
    if constexpr (!PREFETCH_DW) load_dw(h0);

    // ---- C: depthwise 3x3 (stride S) + bias + ReLU6 on the chunk; 4 channels per thread item
    static_assert(POUT % 32 == 0, "depthwise: whole passes of 32 pixels");
    // the nine taps' LDS reads are issued before the FMA chain (interleaved, the compiler reused one register
    // set and waited on each read in turn); the pass loop stays rolled so the addresses are not kept live
#pragma unroll 1
    for (int qi = 0; qi < POUT / 32; ++qi) {
      const int q = (tid >> 3) + 32 * qi;
      const int oy = q / TW, ox = q - oy * TW;
      int addr[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int px = (oy * S + t / 3) * PW + ox * S + t % 3;
        addr[t] = px * ep + 4 * eswz<S>(px, g);
      }
      float4 v[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) v[t] = *(const float4*)&E[addr[t]];
      float4 a = bdw;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 w = wk[t];
        a.x = fmaf(v[t].x, w.x, a.x);
        a.y = fmaf(v[t].y, w.y, a.y);
        a.z = fmaf(v[t].z, w.z, a.z);
        a.w = fmaf(v[t].w, w.w, a.w);
      }
      *(float4*)&Ds[q * IRF_DP + 4 * g] = relu6x4(a);
    }
    __syncthreads();
    // next chunk's expand / depthwise weights, in flight during the project GEMM (unconditional: a conditional
    // prefetch made the project's wait for its own weights cover the prefetch as well)
    if constexpr (EXPAND) load_expand(hn);
    if constexpr (PREFETCH_DW) load_dw(hn);

    // ---- D: project GEMM accumulate, rows = output channel, columns = output pixel
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int pr = wave + 4 * j;
        if (pr >= PAIRS) break;
        const int mt = pr / NTO;
        const float4 bb = *(const float4*)(Ds + (mt * 16 + col) * IRF_DP + 16 * kc + 4 * kq);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(wprj[j][kc], s4), f4c(bb, s4), acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
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

// LDS bytes of one workgroup (<= 64 KiB, or an instantiation whose dynamic-LDS limit ir_f32_prepare raised
// before any graph capture)
static size_t irf_lds_bytes(int S, int inp_pad, int expand, int TW = 8) {
  const int TH = S == 1 ? 8 : 4;
  const int PH = (TH - 1) * S + 3, PW = (TW - 1) * S + 3;
  const size_t rows = (size_t)(PH * PW + 15) / 16 * 16;
  return sizeof(float) * (rows * irf_xp(inp_pad, expand) + (expand ? rows * irf_ep(S) : 0) +
                          (size_t)TH * TW * IRF_DP + rows);
}

template <int S, int TH, int TW, int NTO, bool EXPAND, int KIN>
static void irf_launch_k(const IrParams& p, hipStream_t s) {
  const size_t lds = irf_lds_bytes(S, p.inp_pad, EXPAND, TW);
  const int tiles = ((p.Wo + TW - 1) / TW) * ((p.Ho + TH - 1) / TH);
  hipLaunchKernelGGL((ir_f32_kernel<S, TH, TW, NTO, EXPAND, KIN>), dim3((unsigned)(p.B * tiles)), dim3(256), lds, s,
                     p);
}

template <int S, int TH, int TW, int NTO, bool EXPAND>
static void irf_launch(const IrParams& p, hipStream_t s) {
  if constexpr (!EXPAND) {
    irf_launch_k<S, TH, TW, NTO, false, 1>(p, s);
  } else {
    switch (p.inp_pad / 16) {
      case 1: irf_launch_k<S, TH, TW, NTO, true, 1>(p, s); break;
      case 2: irf_launch_k<S, TH, TW, NTO, true, 2>(p, s); break;
      case 3: irf_launch_k<S, TH, TW, NTO, true, 3>(p, s); break;
      default: irf_launch_k<S, TH, TW, NTO, true, 4>(p, s); break;  // inp_pad <= 64 (supported())
    }
  }
}

template <int S, int TH, int TW, bool EXPAND>
static bool irf_nto(const IrParams& p, hipStream_t s) {
  switch (p.oup_pad / 16) {
    case 1: irf_launch<S, TH, TW, 1, EXPAND>(p, s); return true;
    case 2: irf_launch<S, TH, TW, 2, EXPAND>(p, s); return true;
    case 4: irf_launch<S, TH, TW, 4, EXPAND>(p, s); return true;
    case 6: irf_launch<S, TH, TW, 6, EXPAND>(p, s); return true;
    default: return false;
  }
}

// Stride-1 tiles of 8 x 16 output pixels (default; ARENA_IRF_TW=8 restores 8 x 8): the 10 x 18 halo re-expands
// 1.41x the output
// instead of 1.56x for 8 x 8 tiles and each workgroup's fixed cost (staging latency, 3 barriers per hidden
// chunk) is spread over twice the pixels, at 2 instead of 3 workgroups per CU (76 KB LDS with an expansion).
// tools/bench_irc.py, 128 crops: 112x112 t=1 block 167 -> 152 us, 56x56 hid144 228 -> 216, 28x28 hid192 92 -> 76.
static int irf_tw_env() {
  static const int v = [] {
    const char* e = std::getenv("ARENA_IRF_TW");
    return e ? std::atoi(e) : 16;
  }();
  return v;
}
static bool irf_tw16(const IrParams& p) { return irf_tw_env() == 16 && p.Wo >= 16; }

void ir_f32_prepare() {
#define IRF_ATTR(NTO_, KIN_)                                                                                 \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_f32_kernel<1, 8, 16, NTO_, true, KIN_>,               \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define IRF_ATTR_K(NTO_) IRF_ATTR(NTO_, 1) IRF_ATTR(NTO_, 2) IRF_ATTR(NTO_, 3) IRF_ATTR(NTO_, 4)
  IRF_ATTR_K(1) IRF_ATTR_K(2) IRF_ATTR_K(4) IRF_ATTR_K(6)
#undef IRF_ATTR_K
#undef IRF_ATTR
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_f32_kernel<1, 8, 16, 1, false, 1>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_f32_kernel<1, 8, 16, 1, false, 1, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ir_tile_x3_prepare();
}

bool ir_block_f32_supported(int stride, int inp_pad, int hid_pad, int oup_pad, int expand) {
  const int nto = oup_pad / 16;
  return (stride == 1 || stride == 2) && inp_pad % 16 == 0 && inp_pad <= 64 && hid_pad % IRF_HC == 0 &&
         oup_pad % 16 == 0 &&
         (nto == 1 || nto == 2 || nto == 4 || nto == 6) && (expand || hid_pad == inp_pad) &&
         irf_lds_bytes(stride, inp_pad, expand) <= 64 * 1024;
}

// Classifier front end: crop gather + 2x2 s2d stem (16 -> 32, ReLU6) + MobileNetV2 block 1 (t = 1: depthwise
// 32 + ReLU6, project 32 -> 16) in one kernel (IrParams.stem).
static void ir_stem_f32(const IrParams& p, hipStream_t s) {
  if (p.stride != 1 || p.expand || p.res || p.inp != 32 || p.inp_pad != 32 || p.hid_pad != 32 || p.oup_pad != 16 ||
      p.oup > 16 || p.oup % 4 || p.H != p.W || p.H * 2 != p.st_S || p.Ho != p.H || p.Wo != p.W || p.W < 16 ||
      p.y_cs % 4 || p.st_w == nullptr || p.st_b == nullptr || p.st_crops == nullptr || p.st_meta == nullptr ||
      p.st_pool == nullptr)
    throw std::runtime_error("ir_stem_f32: unsupported geometry (needs MobileNetV2 block 1 at S/2 x S/2)");
  if (p.B <= 0) return;
  const size_t lds = irf_lds_bytes(1, 32, 0, 16);
  const int tiles = ((p.Wo + 15) / 16) * ((p.Ho + 7) / 8);
  hipLaunchKernelGGL((ir_f32_kernel<1, 8, 16, 1, false, 1, true>), dim3((unsigned)(p.B * tiles)), dim3(256),
                     lds, s, p);
}

void ir_block_f32(const IrParams& p, hipStream_t s) {
  if (p.stem) {
    if (!ir_stem_x3(p, s)) ir_stem_f32(p, s);  // x3w: the split-plane kernel (ir_tile_x3.hip)
    return;
  }
  if (ir_block_crop_f32(p, s)) return;  // 14x14 / 7x7 maps: whole-map x3 kernel (ir_crop_f32.hip)
  if (p.x_parts > 1 || p.y_parts > 1)
    throw std::runtime_error("ir_block_f32: partial-sum tensors belong to the whole-map 14x14 kernel");
  if (p.x3w) {  // split-plane weights: the tiled x3 kernel (ir_tile_x3.hip)
    if (ir_tile_x3(p, s)) return;
    throw std::runtime_error("ir_block_f32: split-plane weights for a block no x3 kernel takes");
  }
  if (!ir_block_f32_supported(p.stride, p.inp_pad, p.hid_pad, p.oup_pad, p.expand) || p.inp % 4 || p.oup % 4 ||
      p.inp > p.inp_pad || p.oup > p.oup_pad || p.x_cs % 4 || p.y_cs % 4)
    throw std::runtime_error("ir_block_f32: unsupported channel geometry");
  if (p.res && (p.stride != 1 || p.inp != p.oup)) throw std::runtime_error("ir_block_f32: residual needs s1, inp == oup");
  if (p.Ho != (p.H + 2 - 3) / p.stride + 1 || p.Wo != (p.W + 2 - 3) / p.stride + 1)
    throw std::runtime_error("ir_block_f32: output size mismatch");
  if (p.B <= 0) return;
  bool ok;
  if (p.stride == 1 && irf_tw16(p))
    ok = p.expand ? irf_nto<1, 8, 16, true>(p, s) : irf_nto<1, 8, 16, false>(p, s);
  else if (p.stride == 1)
    ok = p.expand ? irf_nto<1, 8, 8, true>(p, s) : irf_nto<1, 8, 8, false>(p, s);
  else
    ok = p.expand ? irf_nto<2, 4, 8, true>(p, s) : irf_nto<2, 4, 8, false>(p, s);
  if (!ok) throw std::runtime_error("ir_block_f32: no kernel for oup_pad " + std::to_string(p.oup_pad));
}

}  // namespace arena
