// Fused MobileNetV2 inverted residual at fp32 accuracy for the 14x14 and 7x7 stages
// (torchvision mobilenet_v2 features[8..17]; the reference runs them as fp32 ONNX per crop,
// architectures/monolithic/app/inference.py:196).
//
// Unfused, each of these ten blocks is three kernels over all crops (1x1 expand GEMM, depthwise, 1x1
// project): 77-134 us per block for 128 crops, 0.99 ms of the 5.18 ms fp32 device time per batch of 32
// requests (profiles/r2_fp32_final_ops.md ops 78-107), with the expanded map crossing the memory system
// twice.  The round-2 whole-map kernel lost to them (profiles/r2_irc_f32_experiment.md: VALU / MFMA ~10,
// 60 % of wave cycles parked at barriers) because the depthwise recomputed its addresses and bounds per
// tap and per chunk and went through an LDS round trip for the project operand.  This version:
//
//   * one workgroup = one half (row band) of one crop, all hidden and all output channels, 8 waves;
//     grid = 2 x crops (256 workgroups for 128 crops: one per CU);
//   * the block input X is loaded ONCE into the expand B-operand registers of the wave that owns its
//     16-pixel tile, already split into three bf16 planes (x = h + m + l exactly to fp32 rounding);
//   * per chunk of HC hidden channels:
//       E = relu6(We[chunk] . X + be)        x3 MFMA 16x16x32 -> fp32 LDS map with a zero border
//       D = relu6(dw3x3_S(E) + bd)           fp32 FMA straight into the project B-operand registers:
//                                            lane (pixel, 8 channels) == the MFMA fragment, no LDS trip,
//                                            tap addresses = one base + constants (the border is the pad)
//       acc += Wp[:, chunk] . D              x3 MFMA, accumulators in registers for the whole loop
//   * chunk weights (pre-split bf16 planes from the host, engine/planner.py::split_bf16x3) are fetched
//     into registers two phases ahead and stored to LDS by all threads: every weight byte leaves L2 once
//     per workgroup; two barriers per chunk.
//   y = acc + bp (+ x, stride 1)                                              fp32 NHWC
//
// Operand mapping of v_mfma_f32_16x16x32_bf16: lane l supplies A[row = l & 15][k = 8 (l >> 4) .. +7]
// and B[k = 8 (l >> 4) .. +7][col = l & 15] and receives D[row = 4 (l >> 4) + r][col = l & 15].  Expand:
// rows = hidden channels (A = We), columns = pixels (B = X).  Project: rows = output channels (A = Wp),
// columns = output pixels (B = D).
//
// LDS bank notes (MI355X_MICROARCH.md §LDS: ds_read_b128 serves 16-lane groups from 16 16-B slots):
//   * weight rows are read 16 rows x 4 k-groups per instruction: row pitch 2 (mod 4) slots;
//   * E is stored as [channel group of 8][pixel][8 fp32] with an odd-slot plane stride: the 16-lane
//     groups of a depthwise read mix k-groups of both parities, which then land on disjoint slot parities.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

constexpr int IRX_THREADS = 512, IRX_WAVES = IRX_THREADS / 64;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int imin(int a, int b) { return a < b ? a : b; }
constexpr int imax(int a, int b) { return a > b ? a : b; }

// 8 fp32 -> three bf16x8 planes with v = h + m + l (round to nearest even at each step)
__device__ __forceinline__ void split8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
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

// a*b to fp32 accuracy from the split planes; smallest terms first (added while the sum is smallest)
__device__ __forceinline__ f32x4 mfma_x3(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

}  // namespace

// input rows the widest of NP bands of NOR rows reads (its E rows without the zero border)
constexpr int band_rows(int HO, int S, int NP, int NOR) {
  int m = 0;
  for (int p = 0; p < NP; ++p) {
    const int oy0 = p * NOR, nor = imin(NOR, HO - oy0);
    if (nor <= 0) continue;
    const int lo = imax(0, oy0 * S - 1), hi = imin(HO * S - 1, (oy0 + nor - 1) * S + 1);
    m = imax(m, hi - lo + 1);
  }
  return m;
}

// HO: output side; S: stride; KS: inp_pad / 32; NOT: oup_pad / 16; HC: hidden channels per chunk; NP: row bands
// (workgroups) per crop.
template <int HO, int S, int KS, int NOT, int HC, int NP = 2>
struct IrxGeom {
  static constexpr int HI = HO * S;                   // input side
  static constexpr int NOR0 = (HO + NP - 1) / NP;     // output rows of a band (the last one may be shorter)
  static constexpr int ER = (NOR0 - 1) * S + 3;       // E rows incl. the zero border
  static constexpr int EW = HI + 2;                   // E columns incl. the zero border
  static constexpr int NEP = ER * EW;                 // E pixels
  static constexpr int NKG = HC / 8;                  // 8-channel groups of a chunk
  static constexpr int EPS = (2 * NEP + 1) * 16;      // bytes per E channel-group plane (odd slot count)
  static constexpr int NX = band_rows(HO, S, NP, NOR0) * HI;  // input pixels of the largest band
  static constexpr int NXT = (NX + 15) / 16;          // expand pixel tiles
  static constexpr int INP = KS * 32;
  static constexpr int NHT = HC / 16;                 // expand hidden tiles per chunk
  static constexpr int EWPT = (NXT <= IRX_WAVES / 2 && NHT % 2 == 0) ? 2 : 1;  // waves sharing an X tile
  static constexpr int HTW = NHT / EWPT;              // expand hidden tiles per wave
  static constexpr int NPT = (NOR0 * HO + 15) / 16;   // project pixel tiles
  static constexpr int NOG = imax(1, IRX_WAVES / NPT);  // output-channel groups (one wave each per tile)
  static constexpr int OTG = (NOT + NOG - 1) / NOG;   // output tiles of 16 per group
  static constexpr int NKS = HC / 32;                 // project K-steps per chunk
  static constexpr int WEB = 6 * INP + 32;            // bytes per We row: [h|m|l][INP] bf16 + pad
  static constexpr int WPB = 6 * HC + 32;             // bytes per Wp row: [h|m|l][HC] bf16 + pad
  static constexpr int E_BYTES = NKG * EPS, WE_BYTES = HC * WEB, WBE_BYTES = HC * 4;
  static constexpr int WP_BYTES = NOT * 16 * WPB, WD_BYTES = 10 * HC * 4;  // WD: 9 taps + bias
  static constexpr int LDS = E_BYTES + WE_BYTES + WBE_BYTES + WP_BYTES + WD_BYTES;
  // 16-byte staging pieces of one chunk
  static constexpr int WE_PPR = 3 * INP / 8, WE_PIECES = HC * WE_PPR + HC / 4;  // + the expand bias
  static constexpr int WP_PPR = 3 * HC / 8, WP_PIECES = NOT * 16 * WP_PPR + 10 * HC / 4;  // + taps, dw bias
  static constexpr int WE_PT = (WE_PIECES + IRX_THREADS - 1) / IRX_THREADS;
  static constexpr int WP_PT = (WP_PIECES + IRX_THREADS - 1) / IRX_THREADS;
};

// Weights (IrParams.x3w = 1, packed by engine/planner.py::split_bf16x3): we bf16 [hid_pad][3][inp_pad] and
// wp bf16 [oup_pad][3][hid_pad] (planes h, m, l of the fp32 weight), wd fp32 [9][hid_pad], biases fp32.
template <int HO, int S, int KS, int NOT, int HC, int NP>
__global__ __launch_bounds__(IRX_THREADS) void ir_x3_kernel(const IrParams p) {
  using G = IrxGeom<HO, S, KS, NOT, HC, NP>;
  constexpr int HI = G::HI, INP = G::INP, EW = G::EW;
  extern __shared__ __align__(16) uint8_t lds[];
  uint8_t* Es = lds;
  uint8_t* WEs = Es + G::E_BYTES;
  float* WBEs = (float*)(WEs + G::WE_BYTES);
  uint8_t* WPs = (uint8_t*)WBEs + G::WBE_BYTES;
  float* WDs = (float*)(WPs + G::WP_BYTES);  // [10][HC]: taps 0..8, bias

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int xparts = p.x_parts > 1 ? p.x_parts : 1, yparts = p.y_parts > 1 ? p.y_parts : 1;
  const int slice = blockIdx.x % yparts, bp_idx = blockIdx.x / yparts;
  const int b = bp_idx / NP, part = bp_idx - (bp_idx / NP) * NP;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int oy0 = part * G::NOR0;
  const int nor = imin(G::NOR0, HO - oy0);
  if (nor <= 0) return;
  const int nout = nor * HO;
  const int iy0 = oy0 * S - 1;                          // image row of E row 0
  const int iy_lo = iy0 < 0 ? 0 : iy0;
  const int iy_hi = imin(HI - 1, (oy0 + nor - 1) * S + 1);
  const int nx = (iy_hi - iy_lo + 1) * HI;
  const float* __restrict__ x = (const float*)p.x;
  const bf16* __restrict__ we = (const bf16*)p.we;
  const bf16* __restrict__ wp = (const bf16*)p.wp;
  const float* __restrict__ wd = (const float*)p.wd;
  const int hid_pad = p.hid_pad, nch_all = hid_pad / HC;
  const int cb = slice * nch_all / yparts, ce = (slice + 1) * nch_all / yparts;  // this slice's hidden chunks

  // ---- chunk weight staging (global -> registers -> LDS); plain unrolled loops, not lambdas: a lambda
  // capturing the staging arrays by reference put them in scratch memory (80-208 B per lane)
  u32x4 rwe[G::WE_PT], rwp[G::WP_PT];  // native vector type: the HIP uint4 struct kept them in scratch
// Every thread loads every piece slot (out-of-range slots re-read a valid address) and the source / destination
// addresses are selects: with per-slot branches the compiler kept the staging arrays in scratch memory.
#define IRX_FETCH_WE(h0_)                                                                   \
  _Pragma("unroll") for (int j = 0; j < G::WE_PT; ++j) {                                   \
    const int e = tid + IRX_THREADS * j;                                                    \
    const int row = e / G::WE_PPR, pc = e - row * G::WE_PPR;                                \
    const bool isw = e < HC * G::WE_PPR;                                                    \
    const int eb = e - HC * G::WE_PPR;                                                      \
    const uint8_t* src = isw ? (const uint8_t*)(we + (size_t)((h0_) + row) * (3 * INP) + pc * 8) \
                             : (const uint8_t*)(p.be + (h0_) + 4 * (eb < HC / 4 ? eb : 0)); \
    rwe[j] = *(const u32x4*)src;                                                            \
  }
#define IRX_STORE_WE()                                                                      \
  _Pragma("unroll") for (int j = 0; j < G::WE_PT; ++j) {                                   \
    const int e = tid + IRX_THREADS * j;                                                    \
    const int row = e / G::WE_PPR, pc = e - row * G::WE_PPR;                                \
    uint8_t* dst = e < HC * G::WE_PPR ? WEs + row * G::WEB + pc * 16                        \
                                      : (uint8_t*)WBEs + 16 * (e - HC * G::WE_PPR);         \
    if (e < G::WE_PIECES) *(u32x4*)dst = rwe[j];                                            \
  }
#define IRX_FETCH_WP(h0_)                                                                   \
  _Pragma("unroll") for (int j = 0; j < G::WP_PT; ++j) {                                   \
    const int e = tid + IRX_THREADS * j;                                                    \
    const int row = e / G::WP_PPR, pc = e - row * G::WP_PPR;                                \
    const int pl = pc / (HC / 8), c8 = pc - pl * (HC / 8);                                  \
    const bool isw = e < NOT * 16 * G::WP_PPR;                                              \
    const int i = isw ? 0 : imin(e - NOT * 16 * G::WP_PPR, 10 * HC / 4 - 1);               \
    const int r = i / (HC / 4), g = i - r * (HC / 4);                                       \
    const float* dsrc = (r < 9 ? wd + (size_t)r * hid_pad : p.bd) + (h0_) + 4 * g;          \
    const uint8_t* src = isw ? (const uint8_t*)(wp + ((size_t)row * 3 + pl) * hid_pad + (h0_) + c8 * 8) \
                             : (const uint8_t*)dsrc;                                        \
    rwp[j] = *(const u32x4*)src;                                                            \
  }
#define IRX_STORE_WP()                                                                      \
  _Pragma("unroll") for (int j = 0; j < G::WP_PT; ++j) {                                   \
    const int e = tid + IRX_THREADS * j;                                                    \
    const int row = e / G::WP_PPR, pc = e - row * G::WP_PPR;                                \
    uint8_t* dst = e < NOT * 16 * G::WP_PPR ? WPs + row * G::WPB + pc * 16                  \
                                            : (uint8_t*)WDs + 16 * (e - NOT * 16 * G::WP_PPR); \
    if (e < G::WP_PIECES) *(u32x4*)dst = rwp[j];                                            \
  }
  IRX_FETCH_WE(cb * HC)
  IRX_FETCH_WP(cb * HC)

  // ---- E: zero everywhere (the border stays zero: it is the depthwise padding)
  for (int i = tid; i < G::E_BYTES / 16; i += IRX_THREADS) ((uint4*)Es)[i] = make_uint4(0u, 0u, 0u, 0u);

  // ---- this wave's expand pixel tile: the block input, split, resident in registers for the whole kernel
  const int xt = wave / G::EWPT, hpart = wave - xt * G::EWPT;
  const bool xw = xt < G::NXT;
  bf16x8 xh[KS], xm[KS], xl[KS];
  int e_off = -1;  // byte offset of this lane's pixel in an E plane (-1: padding pixel)
  {
    const int xp = xt * 16 + col;
    const bool ok = xw && xp < nx;
    const int iy = iy_lo + xp / HI, ix = xp - (xp / HI) * HI;
    const float* src = x + (((size_t)b * HI + (ok ? iy : 0)) * HI + (ok ? ix : 0)) * p.x_cs;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + 8 * kq;
      float v[8];
      const bool kk = ok && k < p.inp;
      float4 a = *(const float4*)(src + (kk ? k : 0)), c = *(const float4*)(src + (kk ? k + 4 : 0));
      for (int j = 1; j < xparts; ++j) {  // partial sums of a hidden-sliced producer, added in order
        const float* sj = src + j * p.inp + (kk ? k : 0);
        const float4 a2 = *(const float4*)sj, c2 = *(const float4*)(sj + 4);
        a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
        c.x += c2.x; c.y += c2.y; c.z += c2.z; c.w += c2.w;
      }
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
      if (!kk) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
      }
      split8(v, xh[ks], xm[ks], xl[ks]);
    }
    if (ok) e_off = ((iy - iy0) * EW + ix + 1) * 32;
  }

  // ---- this wave's depthwise + project unit: (output pixel tile, output-channel group)
  const int upt = wave % G::NPT, uog = wave / G::NPT;
  const bool pw = uog < G::NOG;
  const int ot0 = uog * G::OTG;
  const int q = upt * 16 + col;
  const bool qok = pw && q < nout;
  const int qq = qok ? q : 0;
  const int dw_off = ((qq / HO) * S * EW + (qq - (qq / HO) * HO) * S) * 32;  // tap (0, 0), bytes in a plane
  f32x4 acc[G::OTG];
#pragma unroll
  for (int j = 0; j < G::OTG; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  IRX_STORE_WE()
  IRX_STORE_WP()
  if (ce - cb > 1) {
    IRX_FETCH_WE((cb + 1) * HC)
    IRX_FETCH_WP((cb + 1) * HC)
  }
  __syncthreads();

  for (int c = cb; c < ce; ++c) {
    // ---- expand: E[pix][chunk] = relu6(We[chunk] . X + be) for this wave's hidden tiles
    if (xw) {
#pragma unroll
      for (int i = 0; i < G::HTW; ++i) {
        const int ht = hpart * G::HTW + i;
        f32x4 e = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const uint8_t* ra = WEs + (ht * 16 + col) * G::WEB + (ks * 32 + 8 * kq) * 2;
          e = mfma_x3(*(const bf16x8*)ra, *(const bf16x8*)(ra + INP * 2), *(const bf16x8*)(ra + INP * 4), xh[ks],
                      xm[ks], xl[ks], e);
        }
        if (e_off >= 0) {
          const int ch = ht * 16 + 4 * kq;
          const float4 be = *(const float4*)(WBEs + ch);
          const float4 v = make_float4(relu6f(e[0] + be.x), relu6f(e[1] + be.y), relu6f(e[2] + be.z),
                                       relu6f(e[3] + be.w));
          *(float4*)(Es + (ch >> 3) * G::EPS + e_off + (ch & 7) * 4) = v;
        }
      }
    }
    __syncthreads();  // A: E complete; every wave is past its reads of We / be
    if (c + 1 < ce) {
      IRX_STORE_WE()
      if (c + 2 < ce) {
        IRX_FETCH_WE((c + 2) * HC)
      }
    }

    // ---- depthwise (into the project B operand) + project
    if (pw) {
#pragma unroll
      for (int ks = 0; ks < G::NKS; ++ks) {
        const int kg = ks * 4 + kq;
        const float* wk = WDs + kg * 8;
        float a[8];
        {
          const float4 b0 = *(const float4*)(wk + 9 * HC), b1 = *(const float4*)(wk + 9 * HC + 4);
          a[0] = b0.x; a[1] = b0.y; a[2] = b0.z; a[3] = b0.w; a[4] = b1.x; a[5] = b1.y; a[6] = b1.z; a[7] = b1.w;
        }
        const uint8_t* eb = Es + kg * G::EPS + dw_off;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const uint8_t* ep = eb + ((t / 3) * EW + (t % 3)) * 32;
          const float4 v0 = *(const float4*)ep, v1 = *(const float4*)(ep + 16);
          const float4 w0 = *(const float4*)(wk + t * HC), w1 = *(const float4*)(wk + t * HC + 4);
          a[0] = fmaf(v0.x, w0.x, a[0]);
          a[1] = fmaf(v0.y, w0.y, a[1]);
          a[2] = fmaf(v0.z, w0.z, a[2]);
          a[3] = fmaf(v0.w, w0.w, a[3]);
          a[4] = fmaf(v1.x, w1.x, a[4]);
          a[5] = fmaf(v1.y, w1.y, a[5]);
          a[6] = fmaf(v1.z, w1.z, a[6]);
          a[7] = fmaf(v1.w, w1.w, a[7]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = relu6f(a[i]);
        bf16x8 dh, dm, dl;
        split8(a, dh, dm, dl);
#pragma unroll
        for (int j = 0; j < G::OTG; ++j) {
          const int ot = ot0 + j;
          if (ot >= NOT) break;
          const uint8_t* ra = WPs + (ot * 16 + col) * G::WPB + (ks * 32 + 8 * kq) * 2;
          acc[j] = mfma_x3(*(const bf16x8*)ra, *(const bf16x8*)(ra + HC * 2), *(const bf16x8*)(ra + HC * 4), dh, dm,
                           dl, acc[j]);
        }
      }
    }
    __syncthreads();  // B: every wave is past its reads of E, Wp and the taps
    if (c + 1 < ce) {
      IRX_STORE_WP()
      if (c + 2 < ce) {
        IRX_FETCH_WP((c + 2) * HC)
      }
    }
  }

#undef IRX_FETCH_WE
#undef IRX_STORE_WE
#undef IRX_FETCH_WP
#undef IRX_STORE_WP

  // ---- epilogue: + bp (+ residual, stride 1: the block input at the same pixel) -> NHWC fp32; a hidden slice
  // > 0 writes its bare partial sum at channel offset slice * oup
  if (qok) {
    const int oy = oy0 + q / HO, ox = q - (q / HO) * HO;
    float* yp = (float*)p.y + (((size_t)b * HO + oy) * HO + ox) * p.y_cs + slice * p.oup;
    const float* xr = x + (((size_t)b * HI + oy) * HI + ox) * p.x_cs;
#pragma unroll
    for (int j = 0; j < G::OTG; ++j) {
      const int ot = ot0 + j;
      const int co = ot * 16 + 4 * kq;
      if (ot >= NOT || co >= p.oup) continue;
      float4 v = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
      if (slice == 0) {
        const float4 bp = *(const float4*)(p.bp + co);
        v.x += bp.x;
        v.y += bp.y;
        v.z += bp.z;
        v.w += bp.w;
        if (S == 1 && p.res) {
          float4 r = *(const float4*)(xr + co);
          for (int jp = 1; jp < xparts; ++jp) {  // the block input: its partial sums in the load's order
            const float4 r2 = *(const float4*)(xr + jp * p.inp + co);
            r.x += r2.x; r.y += r2.y; r.z += r2.z; r.w += r2.w;
          }
          v.x += r.x;
          v.y += r.y;
          v.z += r.z;
          v.w += r.w;
        }
      }
      *(float4*)(yp + co) = v;
    }
  }
}

// (HO, S, KS, NOT, HC): the MobileNetV2 14x14 / 7x7 stages at 224
#define ARENA_IRX_CONFIGS(X) \
  X(14, 1, 2, 4, 32)         \
  X(14, 1, 2, 6, 32)         \
  X(14, 1, 3, 6, 32)         \
  X(7, 2, 3, 10, 32)         \
  X(7, 1, 5, 10, 32)         \
  X(7, 1, 5, 20, 32)

// Row bands per crop: 2, or ARENA_IRX_PARTS (3 / 4) for the 14x14 stage — more, shorter bands double the
// workgroups of a launch (one per CU at batch 32 with two; four workgroups per crop at bs 1) at the price of
// recomputing the expand halo rows.
int g_irx_parts = -1;  // -1: ARENA_IRX_PARTS, else auto

// Row bands per crop of the 14x14 kernel.  Auto: two for a full batch (256 workgroups for 128 crops: one per
// CU), four for small crop capacities (bucket 1: 16 crops), where the launch is otherwise a few dozen
// workgroups on 256 CUs — ops 73-78 at bs 1: 233 -> 211 us; at batch 32 four bands cost more than they gain
// (479 -> 571 us; three: 446 us but a lower engine rate), profiles/r4b_irx_parts.md.
// The 7x7 stage: two bands, or one when the hidden channels are sliced over workgroups (the slices already fill
// the chip; one band halves the split weights streamed per output pixel).
int irx_parts(int HO, int S, int crops, int yparts) {
  if (g_irx_parts < 0) {
    const char* e = std::getenv("ARENA_IRX_PARTS");
    g_irx_parts = e != nullptr ? std::atoi(e) : 0;
  }
  int n = g_irx_parts;
  if (n != 2 && n != 3 && n != 4) n = crops <= 32 ? 4 : 2;
  return HO == 14 ? n : (yparts > 1 && S == 1 ? 1 : 2);
}

void set_irx_parts(int n) { g_irx_parts = n; }

// Hidden slices actually used for a planned partial-sum count: all of them for small crop capacities (bucket 1:
// a few dozen workgroups otherwise), at most ARENA_IRX_SLICES_BIG (default 2) for full batches, whose row bands
// already give every CU a workgroup (ops 73-77 at batch 32: 3 slices 367 us, 2 slices 346 us, 1: 382 us;
// profiles/r4c).  Producer and consumer of a partial-sum tensor see the same capacity, so they agree.
int g_irx_big = -1;
void set_irx_slices_big(int n) { g_irx_big = n >= 1 ? n : -1; }
int irx_effective_parts(int planned, int crops) {
  if (planned <= 1) return 1;
  if (g_irx_big < 0) {
    const char* e = std::getenv("ARENA_IRX_SLICES_BIG");
    g_irx_big = e != nullptr ? std::atoi(e) : 2;
    if (g_irx_big < 1) g_irx_big = 1;
  }
  return crops > 32 && planned > g_irx_big ? g_irx_big : planned;
}

void ir_crop_f32_prepare() {
#define X1(HO_, S_, KS_, NOT_, HC_, NP_)                                                                   \
  static_assert(IrxGeom<HO_, S_, KS_, NOT_, HC_, NP_>::LDS <= 160 * 1024, "ir_x3: LDS budget");            \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_x3_kernel<HO_, S_, KS_, NOT_, HC_, NP_>,            \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define X(HO_, S_, KS_, NOT_, HC_) \
  X1(HO_, S_, KS_, NOT_, HC_, 1) X1(HO_, S_, KS_, NOT_, HC_, 2) X1(HO_, S_, KS_, NOT_, HC_, 3) X1(HO_, S_, KS_, NOT_, HC_, 4)
  ARENA_IRX_CONFIGS(X)
#undef X
#undef X1
}

// Shapes this kernel takes (mirrored by engine/validate.py::ir_crop_f32_supported; the planner marks the
// blocks that use it with split-plane weights, IrParams.x3w): an expanding block on a 14x14 (stride 1 or 2)
// or 7x7 (stride 1) input map whose (inp_pad, oup_pad) has a configuration above.
bool ir_block_crop_f32_supported(int H, int stride, int inp_pad, int hid_pad, int oup_pad, int expand) {
  if (!expand || oup_pad % 16) return false;
  const int HO = (H + 2 - 3) / stride + 1;
  if (H != HO * stride) return false;
#define X(HO_, S_, KS_, NOT_, HC_) \
  if (HO == HO_ && stride == S_ && inp_pad == KS_ * 32 && oup_pad == NOT_ * 16 && hid_pad % HC_ == 0) return true;
  ARENA_IRX_CONFIGS(X)
#undef X
  return false;
}

bool ir_block_crop_f32(const IrParams& p, hipStream_t s) {
  if (!p.x3w) return false;  // only blocks planned for an x3 kernel carry split-plane weights
  if (p.H != p.W || p.Ho != p.Wo || !ir_block_crop_f32_supported(p.H, p.stride, p.inp_pad, p.hid_pad, p.oup_pad,
                                                                 p.expand))
    return false;  // the tiled x3 kernel (ir_tile_x3.hip) takes it
  if (p.inp % 8 || p.oup % 4 || p.inp > p.inp_pad || p.oup > p.oup_pad || p.x_cs % 4 || p.y_cs % 4)
    throw std::runtime_error("ir_x3: unsupported channel geometry");
  if (p.res && (p.stride != 1 || p.inp != p.oup)) throw std::runtime_error("ir_x3: residual needs s1, inp == oup");
  if (p.Ho != (p.H + 2 - 3) / p.stride + 1) throw std::runtime_error("ir_x3: output size mismatch");
  if ((p.x_parts > 1 ? p.x_parts : 1) * p.inp > p.x_cs || (p.y_parts > 1 ? p.y_parts : 1) * p.oup > p.y_cs)
    throw std::runtime_error("ir_x3: partial-sum tensor narrower than its planned parts");
  const int xparts = irx_effective_parts(p.x_parts, p.B), yparts = irx_effective_parts(p.y_parts, p.B);
  IrParams q = p;  // the kernel reads the effective counts
  q.x_parts = xparts;
  q.y_parts = yparts;
  if (xparts > 8 || yparts > 8 || yparts > p.hid_pad / 32 || p.x_cs < xparts * p.inp || p.y_cs < yparts * p.oup)
    throw std::runtime_error("ir_x3: unsupported partial-sum geometry (<= 8 parts, <= 1 per hidden chunk)");
  if (p.B <= 0) return true;
  const int np = irx_parts(p.Ho, p.stride, p.B, yparts);
#define X1(HO_, S_, KS_, NOT_, HC_, NP_)                                                                      \
  if (np == NP_) {                                                                                            \
    using G = IrxGeom<HO_, S_, KS_, NOT_, HC_, NP_>;                                                          \
    if (G::NXT * G::EWPT > IRX_WAVES) /* a band's expand tiles must fit the waves */                          \
      throw std::runtime_error("ir_x3: " + std::to_string(NP_) + " row band(s) do not fit this geometry");    \
    hipLaunchKernelGGL((ir_x3_kernel<HO_, S_, KS_, NOT_, HC_, NP_>), dim3((unsigned)(p.B * NP_ * yparts)),    \
                       dim3(IRX_THREADS), G::LDS, s, q);                                                      \
    return true;                                                                                              \
  }
#define X(HO_, S_, KS_, NOT_, HC_)                                                                             \
  if (p.Ho == HO_ && p.stride == S_ && p.inp_pad == KS_ * 32 && p.oup_pad == NOT_ * 16 && p.hid_pad % HC_ == 0) { \
    X1(HO_, S_, KS_, NOT_, HC_, 1) X1(HO_, S_, KS_, NOT_, HC_, 2) X1(HO_, S_, KS_, NOT_, HC_, 3)               \
    X1(HO_, S_, KS_, NOT_, HC_, 4)                                                                            \
  }
  ARENA_IRX_CONFIGS(X)
#undef X
#undef X1
  return false;
}

}  // namespace arena
