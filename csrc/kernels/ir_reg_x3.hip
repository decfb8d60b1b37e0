// Register-resident fused MobileNetV2 inverted residual, fp32-accurate on the bf16 matrix cores (six-product
// triple-bf16 split), for the stride-1 56x56 / 28x28 blocks (torchvision mobilenet_v2 features[3], [5], [6]; the
// reference runs them as fp32 ONNX per crop, /root/reference/architectures/monolithic/app/inference.py:196).
//
// The tiled kernel (ir_tile_x3.hip) moves every hidden chunk through LDS twice: the expanded map E (fp32) for the
// depthwise, whose nine taps re-read each value nine times, and the depthwise output D (split planes) for the
// project GEMM; two barriers per chunk, ~245 KB of LDS traffic per chunk of a 128-pixel tile, 26 % MFMA busy
// (profiles/r4pmc/ops_pmc_hbm.md op 65).  Here nothing but the weights lives in LDS:
//
//   * a wave owns a strip of R output rows x 14 output columns of one crop.  Pixel fragments are 16 consecutive
//     pixels of one row (the 14 columns plus a one-pixel halo each side), so in a 16x16x32 MFMA the fragment's
//     pixels are the N dimension: lane l holds pixel l & 15;
//   * expand E = relu6(We . X + be) runs per halo row on the row's split input (kept in registers for all hidden
//     chunks); the result layout puts hidden channels 4q .. 4q+3 and 16+4q .. 16+4q+3 of pixel l & 15 in lane l
//     (q = l >> 4);
//   * the depthwise 3x3 reads its horizontal neighbours from the adjacent lanes (DPP row_shr:1 / row_shl:1 inside
//     the 16-lane rows, which are exactly the fragment's pixels) and its vertical neighbours from the previous
//     and next rows' E registers (a rolling window of three rows);
//   * D = relu6(dw + bd), split in registers, IS the project MFMA's B operand: the project weights are staged
//     with their hidden columns permuted into the order the lanes hold D (slot 8q + j <-> hidden 4q + j for
//     j < 4, 16 + 4q + j - 4 otherwise), so no value moves between lanes;
//   * acc[r][ot] += Wp . D over the hidden chunks; y = acc + bp (+ x) for the 14 inner columns.
//
// One barrier per workgroup (after the weights are staged); the waves then walk their strips independently.
// Halo cost: the expand runs on R + 2 rows of 16 pixels for R x 14 outputs.
//
// Measured (gfx950, 128 crops, rocprofv3; gpurun_out r5c-r5e, tools/bench_irreg.py): 56x56 hid 160 block 123-148
// us, 28x28 hid 192 56-65 us, against the tiled kernel's 170 / 69 us inside the pipeline (ops 65 / 67-68) — no net
// gain in the pipeline (193.6 us at 56x56, profiles r5b).  The limit is vector issue, not the matrix pipe: one wave
// per SIMD (the strip needs ~440 registers, the overflow sits in AGPRs: ~775 v_accvgpr moves per hidden chunk) and
// ~3000 VALU instructions per 192 MFMAs (the triple-bf16 split of D, the DPP shifts, the depthwise); with every
// phase switched off (ARENA_IR_REG_DBG=7) the strip walk alone still takes 89 us.  Kept behind ARENA_IR_REG=1 (and
// pinned by the fp64 tests) as the starting point of a lower-register variant; the tiled kernel stays the default.
//
// Weights (engine/planner.py, x3w): we bf16 [hid_pad][3][32] (inp_pad 32), wp bf16 [oup_pad][3][hid_pad],
// wd fp32 [9][hid_pad], biases fp32.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int IRR_WEP = 96;
  // bf16 per staged expand row: h | m | l x 32 k

__device__ __forceinline__ void irr_split8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
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

__device__ __forceinline__ f32x4 irr_mfma(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                          const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// value of the lane one pixel to the left (row_shr:1) / right (row_shl:1) inside the 16-lane row; 0 at the row's
// ends (those lanes are halo columns, never stored)
__device__ __forceinline__ float irr_left(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
}
__device__ __forceinline__ float irr_right(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x101, 0xf, 0xf, true));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 irr_relu6x2(f32x2 v) {
  return f32x2{__builtin_amdgcn_fmed3f(v[0], 0.0f, 6.0f), __builtin_amdgcn_fmed3f(v[1], 0.0f, 6.0f)};
}

__host__ __device__ constexpr size_t irr_lds_bytes(int hid_pad, int nto) {
  return (size_t)hid_pad * IRR_WEP * 2 + (size_t)nto * 16 * 3 * hid_pad * 2 + (size_t)11 * hid_pad * 4;
}

}  // namespace

// R: output rows per strip; NTO: oup_pad / 16; WPB: waves per workgroup (each walks its own strips)
template <int R, int NTO, int WPB, bool IRR_SCHED>
__global__ __launch_bounds__(WPB * 64) void ir_reg_x3_kernel(const IrParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t irr_lds[];
  const int hid = p.hid_pad;
  bf16* sWe = (bf16*)irr_lds;                          // [hid][h | m | l][32]
  bf16* sWp = sWe + (size_t)hid * IRR_WEP;             // [NTO * 16][3][hid], hidden columns permuted
  float* sWd = (float*)(sWp + (size_t)NTO * 16 * 3 * hid);  // [9 taps | bd | be][hid]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- stage every weight of the block once
  {
    const u32x4* src = (const u32x4*)p.we;  // [hid][3][32] bf16: 12 pieces of 16 B per row, contiguous
    u32x4* dst = (u32x4*)sWe;
    for (int i = tid; i < hid * 12; i += WPB * 64) dst[i] = src[i];
    // project: 8-byte pieces; dest piece d of a 32-slot chunk holds hidden 4 (d >> 1) + 16 (d & 1) .. + 3
    const uint2* wp2 = (const uint2*)p.wp;  // [oup_pad][3][hid] as 4-bf16 pieces
    uint2* sp2 = (uint2*)sWp;
    const int rowp = 3 * hid / 4;  // pieces per (row, all planes)
    for (int i = tid; i < NTO * 16 * rowp; i += WPB * 64) {
      const int o = i / rowp, r = i - o * rowp;  // r: piece within the row's 3 planes
      const int pl = r / (hid / 4), pc = r - pl * (hid / 4);
      const int chunk = pc >> 3, d = pc & 7;
      const int hsrc = 32 * chunk + 4 * (d >> 1) + 16 * (d & 1);
      sp2[i] = o < p.oup_pad ? wp2[((size_t)o * 3 + pl) * (hid / 4) + hsrc / 4] : make_uint2(0u, 0u);
    }
    const float* wd = (const float*)p.wd;
    for (int i = tid; i < 11 * hid; i += WPB * 64) {
      const int t = i / hid, h = i - t * hid;
      sWd[i] = t < 9 ? wd[(size_t)t * hid + h] : t == 9 ? p.bd[h] : p.be[h];
    }
  }
  __syncthreads();

  const int c = lane & 15, q = lane >> 4;
  const int strips_x = (p.Wo + 13) / 14, strips_y = (p.Ho + R - 1) / R;
  const int per_crop = strips_x * strips_y;
  const int total = live_batch(p.B, p.bdev) * per_crop;
  for (int s = blockIdx.x * WPB + wave; s < total; s += gridDim.x * WPB) {
    const int b = s / per_crop, t = s - (s / per_crop) * per_crop;
    const int sy = t / strips_x, sx = t - (t / strips_x) * strips_x;
    const int y0 = sy * R, x = sx * 14 - 1 + c;  // this lane's pixel column (halo included)
    const bool xin = (unsigned)x < (unsigned)p.W;
    const float* xb = (const float*)p.x + (size_t)b * p.H * p.W * p.x_cs;

    // ---- the strip's input rows y0 - 1 .. y0 + R, channels 8q .. 8q + 7 of this lane's pixel, split once into
    // the expand's B operand (kept for every hidden chunk)
    bf16x8 xh[R + 2], xm[R + 2], xl[R + 2];
    float inside[R + 2];
#pragma unroll
    for (int i = 0; i < R + 2; ++i) {
      const int y = y0 - 1 + i;
      const bool in = xin && (unsigned)y < (unsigned)p.H;
      inside[i] = in ? 1.f : 0.f;
      const int k = 8 * q;
      const float* src = xb + ((size_t)(in ? y : 0) * p.W + (in ? x : 0)) * p.x_cs + (k < p.inp ? k : 0);
      const float4 a = *(const float4*)src, cc = *(const float4*)(src + 4);
      const bool lo = in && k < p.inp, hi = in && k + 4 < p.inp;
      const float v[8] = {lo ? a.x : 0.f, lo ? a.y : 0.f, lo ? a.z : 0.f, lo ? a.w : 0.f,
                          hi ? cc.x : 0.f, hi ? cc.y : 0.f, hi ? cc.z : 0.f, hi ? cc.w : 0.f};
      irr_split8(v, xh[i], xm[i], xl[i]);
    }

    f32x4 acc[R][NTO];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int o = 0; o < NTO; ++o) acc[r][o] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int h0 = 0; h0 < hid; h0 += 32) {
      bf16x8 weh[2], wem[2], wel[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const bf16* r = sWe + (size_t)(h0 + 16 * tt + c) * IRR_WEP + 8 * q;
        weh[tt] = *(const bf16x8*)r;
        wem[tt] = *(const bf16x8*)(r + 32);
        wel[tt] = *(const bf16x8*)(r + 64);
      }
      bf16x8 wph[NTO], wpm[NTO], wpl[NTO];
#pragma unroll
      for (int o = 0; o < NTO; ++o) {
        const bf16* r = sWp + (size_t)(16 * o + c) * 3 * hid + h0 + 8 * q;
        wph[o] = *(const bf16x8*)r;
        wpm[o] = *(const bf16x8*)(r + hid);
        wpl[o] = *(const bf16x8*)(r + 2 * hid);
      }
      // the lane's 8 hidden channels: 4q + j (j < 4) and 16 + 4q + j - 4, as float2 pairs (packed FMA)
      f32x2 wdw[9][4], bdv[4], bev[4];
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float4 w0 = *(const float4*)&sWd[t * hid + h0 + 4 * q];
        const float4 w1 = *(const float4*)&sWd[t * hid + h0 + 16 + 4 * q];
        f32x2* dst = t < 9 ? wdw[t] : t == 9 ? bdv : bev;
        dst[0] = f32x2{w0.x, w0.y};
        dst[1] = f32x2{w0.z, w0.w};
        dst[2] = f32x2{w1.x, w1.y};
        dst[3] = f32x2{w1.z, w1.w};
      }

      // Software pipeline over the rows: iteration r issues the expand of halo row r + 3 (12 MFMAs, needed
      // two iterations later) next to the depthwise of output row r (VALU on rows r .. r + 2, already done) and
      // its project (12 MFMAs), so matrix and vector work of one wave overlap.  E and its left / right
      // neighbours live in a rolling window of four rows.
      f32x2 E[4][4], L[4][4], Rt[4][4];
      const int dbg = p.dbg;
      auto expand = [&](int i) {
        const int sl = i & 3;
        f32x4 e0, e1;
        if (dbg & 1) {  // diagnostic: no expand MFMA
          e0 = f32x4{(float)xh[i][0], (float)xm[i][1], (float)xl[i][2], 0.f};
          e1 = e0;
        } else {
          e0 = irr_mfma(weh[0], wem[0], wel[0], xh[i], xm[i], xl[i], f32x4{0.f, 0.f, 0.f, 0.f});
          e1 = irr_mfma(weh[1], wem[1], wel[1], xh[i], xm[i], xl[i], f32x4{0.f, 0.f, 0.f, 0.f});
        }
        const f32x2 m2 = f32x2{inside[i], inside[i]};
        E[sl][0] = irr_relu6x2(f32x2{e0[0], e0[1]} + bev[0]) * m2;
        E[sl][1] = irr_relu6x2(f32x2{e0[2], e0[3]} + bev[1]) * m2;
        E[sl][2] = irr_relu6x2(f32x2{e1[0], e1[1]} + bev[2]) * m2;
        E[sl][3] = irr_relu6x2(f32x2{e1[2], e1[3]} + bev[3]) * m2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          L[sl][j] = f32x2{irr_left(E[sl][j][0]), irr_left(E[sl][j][1])};
          Rt[sl][j] = f32x2{irr_right(E[sl][j][0]), irr_right(E[sl][j][1])};
        }
      };
      expand(0);
      expand(1);
      expand(2);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r + 3 < R + 2) expand(r + 3);
        f32x2 d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = bdv[j];
        if (dbg & 2) {  // diagnostic: no depthwise (the centre tap only)
#pragma unroll
          for (int j = 0; j < 4; ++j) d[j] = E[(r + 1) & 3][j] + bdv[j];
        } else
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int sl = (r + ky) & 3;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            d[j] = __builtin_elementwise_fma(L[sl][j], wdw[3 * ky][j], d[j]);
            d[j] = __builtin_elementwise_fma(E[sl][j], wdw[3 * ky + 1][j], d[j]);
            d[j] = __builtin_elementwise_fma(Rt[sl][j], wdw[3 * ky + 2][j], d[j]);
          }
        }
        float dv[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x2 v = irr_relu6x2(d[j]);
          dv[2 * j] = v[0];
          dv[2 * j + 1] = v[1];
        }
        bf16x8 dh, dm, dl;
        irr_split8(dv, dh, dm, dl);
        if (dbg & 4) {  // diagnostic: no project MFMA
#pragma unroll
          for (int o = 0; o < NTO; ++o) acc[r][o] += f32x4{(float)dh[o], (float)dm[o], (float)dl[o], 0.f};
        } else {
#pragma unroll
          for (int o = 0; o < NTO; ++o) acc[r][o] = irr_mfma(wph[o], wpm[o], wpl[o], dh, dm, dl, acc[r][o]);
        }
        if constexpr (IRR_SCHED) {
          // interleave: one MFMA, then a few VALU (the depthwise / split of this row)
#pragma unroll
          for (int k = 0; k < 12 + 6 * NTO; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
          }
        }
      }
    }

    // ---- epilogue: the 14 inner columns, + bias (+ residual), NHWC fp32
    if (c >= 1 && c <= 14 && x < p.Wo) {
      float* yb = (float*)p.y + (size_t)b * p.Ho * p.Wo * p.y_cs;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int y = y0 + r;
        if (y >= p.Ho) break;
#pragma unroll
        for (int o = 0; o < NTO; ++o) {
          const int co = 16 * o + 4 * q;
          if (co >= p.oup) continue;
          const float4 bp = *(const float4*)(p.bp + co);
          float4 v = make_float4(acc[r][o][0] + bp.x, acc[r][o][1] + bp.y, acc[r][o][2] + bp.z, acc[r][o][3] + bp.w);
          if (p.res) {
            const float4 rv = *(const float4*)(xb + ((size_t)y * p.W + x) * p.x_cs + co);
            v.x += rv.x;
            v.y += rv.y;
            v.z += rv.z;
            v.w += rv.w;
          }
          *(float4*)(yb + ((size_t)y * p.Wo + x) * p.y_cs + co) = v;
        }
      }
    }
  }
}

namespace {

int irr_rows(int H) {
  static const int forced = [] {
    const char* e = std::getenv("ARENA_IR_REG_ROWS");  // A/B: 4 or 7 rows per strip at every size
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 4 || forced == 7) return forced;
  return H >= 56 ? 7 : 4;
}

template <int R, int NTO, bool SCHED>
void irr_launch(const IrParams& p0, hipStream_t s) {
  static const int dbg_env = [] {
    const char* e = std::getenv("ARENA_IR_REG_DBG");
    return e ? std::atoi(e) : 0;
  }();
  IrParams p = p0;
  p.dbg = dbg_env;
  constexpr int WPB = 4;  // one wave per SIMD: the strip's rows, accumulators and inputs need ~300 VGPRs
  const size_t lds = irr_lds_bytes(p.hid_pad, NTO);
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    ARENA_HIP_CHECK(hipGetDevice(&dev));
    ARENA_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long strips = (long)p.B * ((p.Wo + 13) / 14) * ((p.Ho + R - 1) / R);
  const long wgs = (strips + WPB - 1) / WPB;
  const long grid = wgs < cus ? wgs : cus;  // persistent: one workgroup per CU walks the strips
  hipLaunchKernelGGL((ir_reg_x3_kernel<R, NTO, WPB, SCHED>), dim3((unsigned)grid), dim3(WPB * 64), lds, s, p);
}

int g_irr_on = -1;  // -1: ARENA_IR_REG (default off: see the measurements in the header)

bool irr_enabled() {
  if (g_irr_on < 0) {
    const char* e = std::getenv("ARENA_IR_REG");
    g_irr_on = (e != nullptr && (std::string(e) == "1" || std::string(e) == "on" || std::string(e) == "true")) ? 1 : 0;
  }
  return g_irr_on == 1;
}

}  // namespace

bool ir_reg_x3_supported(int H, int stride, int inp_pad, int hid_pad, int oup_pad, int expand) {
  return stride == 1 && expand && inp_pad == 32 && hid_pad >= 32 && hid_pad % 32 == 0 && (oup_pad == 16 || oup_pad == 32) &&
         H >= 28 && irr_lds_bytes(hid_pad, oup_pad / 16) <= 160 * 1024;
}

bool ir_reg_x3(const IrParams& p, hipStream_t s) {
  if (!irr_enabled() || !p.x3w || p.stem || p.x_parts > 1 || p.y_parts > 1) return false;
  if (!ir_reg_x3_supported(p.H, p.stride, p.inp_pad, p.hid_pad, p.oup_pad, p.expand)) return false;
  if (p.inp % 8 || p.oup % 4 || p.inp > p.inp_pad || p.oup > p.oup_pad || p.x_cs % 4 || p.y_cs % 4 ||
      p.Ho != p.H || p.Wo != p.W || (p.res && p.inp != p.oup))
    throw std::runtime_error("ir_reg_x3: unsupported geometry");
  if (p.B <= 0) return true;
  const int R = irr_rows(p.H);
  static const bool sched = [] {
    const char* e = std::getenv("ARENA_IR_REG_SCHED");  // A/B: MFMA / VALU interleave hints (default on)
    return e == nullptr || std::string(e) != "0";
  }();
#define IRR_GO(R_, NTO_)                                   \
  if (R == R_ && p.oup_pad == NTO_ * 16) {                 \
    if (sched) irr_launch<R_, NTO_, true>(p, s);           \
    else irr_launch<R_, NTO_, false>(p, s);                \
    return true;                                           \
  }
  IRR_GO(7, 2)
  IRR_GO(7, 1)
  IRR_GO(4, 2)
  IRR_GO(4, 1)
#undef IRR_GO
  return false;
}

void set_ir_reg(int v) { g_irr_on = v < 0 ? -1 : (v ? 1 : 0); }

void ir_reg_x3_prepare() {
  const int bytes = 160 * 1024;
#define IRR_ATTR(R_, NTO_, SC_)                                                               \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_reg_x3_kernel<R_, NTO_, 4, SC_>,         \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  IRR_ATTR(7, 2, true) IRR_ATTR(7, 1, true) IRR_ATTR(4, 2, true) IRR_ATTR(4, 1, true)
  IRR_ATTR(7, 2, false) IRR_ATTR(7, 1, false) IRR_ATTR(4, 2, false) IRR_ATTR(4, 1, false)
#undef IRR_ATTR
}

}  // namespace arena
