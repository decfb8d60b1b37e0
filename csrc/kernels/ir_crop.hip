// Whole-crop inverted residual for MobileNetV2's 7x7-output blocks (14 -> 7 stride 2, hid 576, the
// two 7x7 hid-960 residual blocks and the 160 -> 320 block; reference: torchvision mobilenet_v2
// features[14..17], run per crop by architectures/monolithic/app/inference.py:196).
//
// At 7x7 the tile kernels (ir_block.hip) get one output tile per crop and walk 18-30 hidden chunks
// with three workgroup barriers each; unfused, the 7x7x960 expanded map makes two HBM round trips
// through three latency-bound kernels (~50 us per block for 128 crops).  Here one workgroup owns one
// whole crop and its four waves split the HIDDEN channels instead of the pixels:
//
//   X (whole input map, all input channels) ........... LDS, shared, loaded once
//   wave w, for hidden chunks h = w, w+4, ... (32 channels each; no workgroup barrier in the loop):
//     E = relu6(We[h] . X + be)    MFMA 16x16x32 ........ wave-private LDS
//     D = relu6(dw3x3_S(E) + bd)   VALU, 8 ch / lane .... wave-private LDS (49 pixels)
//     acc += Wp[:, h] . D          MFMA, 49 px x oup in AGPR/VGPR accumulators
//   sum of the four waves' partial projections in LDS (fixed wave order), + bp (+ x) -> NHWC bf16
//
// Because the tile is the whole map, the depthwise zero padding is a bounds test on the tap, and no
// expansion is recomputed for a halo.  Weights are read straight from L2 into MFMA operand registers:
// a chunk's expand rows are issued before the previous chunk's depthwise/project so their latency
// hides behind that work (single wave per SIMD).
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace arena {

__device__ __forceinline__ int cswz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}
__device__ __forceinline__ void crop_wave_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have completed
  __builtin_amdgcn_wave_barrier();
}

// RS workgroups per crop split its 7 output rows (RS = 2: rows 0-3 and 4-6; each recomputes the
// expansion of the 1-2 input rows the two halves share, and the grid covers the whole chip).
template <int S, int NSLAB, int MP, int RS>
struct IrCropGeom {
  static constexpr int HI = 7 * S;                       // input map side
  static constexpr int NOR = RS == 1 ? 7 : 4;            // max output rows per workgroup
  static constexpr int IR = RS == 1 ? HI : (S == 1 ? 5 : 8);  // max input rows per workgroup
  static constexpr int PIN = IR * HI, PIN_PAD = (PIN + 15) / 16 * 16;
  static constexpr int NE = PIN_PAD / 16;                // expand N-tiles
  static constexpr int NP = (NOR * 7 + 15) / 16;         // project N-tiles
  static constexpr int X_BYTES = NSLAB * PIN_PAD * 64;
  static constexpr int WAVE_BYTES = PIN_PAD * 64 + NP * 16 * 64;  // E rows + D rows
  static constexpr int R_BYTES = NP * 16 * MP * 16 * 4;           // fp32 [px][oup_pad]
  static constexpr int TAIL = 4 * WAVE_BYTES > R_BYTES ? 4 * WAVE_BYTES : R_BYTES;
  static constexpr int LDS = X_BYTES + TAIL;
};

template <int S, int NSLAB, int MP, int RS>
__global__ __launch_bounds__(256) void ir_crop_kernel(const IrParams p) {
  using G = IrCropGeom<S, NSLAB, MP, RS>;
  constexpr int HI = G::HI, PIN = G::PIN, PIN_PAD = G::PIN_PAD, NE = G::NE, NP = G::NP;
  extern __shared__ __align__(16) uint8_t lds[];
  uint8_t* Xs = lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  uint8_t* Es = lds + G::X_BYTES + wave * G::WAVE_BYTES;
  uint8_t* Ds = Es + PIN_PAD * 64;
  float* R = (float*)(lds + G::X_BYTES);

  // OG = oup_pad / (16 MP) output-channel groups per crop (320-out block: 2); each group recomputes the
  // expansion + depthwise and projects onto its own 16 MP output channels
  const int og_n = p.oup_pad / (MP * 16);
  const int b = blockIdx.x / (RS * og_n), rem = blockIdx.x - b * RS * og_n;
  const int part = rem / og_n, og = rem - part * og_n, oc_base = og * MP * 16;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int oy0 = part * 4, nor = RS == 1 ? 7 : (part ? 3 : 4), nout = nor * 7;
  const int iy_lo = oy0 * S - 1 < 0 ? 0 : oy0 * S - 1;
  const int iy_hi = (oy0 + nor - 1) * S + 2 > HI ? HI : (oy0 + nor - 1) * S + 2;  // exclusive
  const int pin = (iy_hi - iy_lo) * HI;
  const bf16* xb = (const bf16*)p.x + ((size_t)b * HI * HI + (size_t)iy_lo * HI) * p.x_cs;
  const bf16* we = (const bf16*)p.we;
  const bf16* wd = (const bf16*)p.wd;
  const bf16* wp = (const bf16*)p.wp;
  const int nchunks = p.hid_pad >> 5;
  const int cpr = NSLAB * 4;  // 8-channel groups per input pixel

  // expand rows of this wave's first chunk (h0 = 32 * wave)
  uint4 rwe[2][NSLAB];
  auto load_we = [&](int h0) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int sl = 0; sl < NSLAB; ++sl)
        rwe[mt][sl] = *(const uint4*)(we + (size_t)(h0 + mt * 16 + row) * p.inp_pad + sl * 32 + kq * 8);
  };
  if (wave < nchunks) load_we(wave * 32);

  // whole input map -> LDS (zero past inp)
  for (int i = tid; i < PIN_PAD * cpr; i += 256) {
    const int pix = i / cpr, c = i - pix * cpr;
    const bool ok = pix < pin && c * 8 < p.inp;
    const uint4 v = load16_or_zero(xb + (size_t)pix * p.x_cs + c * 8, xb, ok);
    *(uint4*)(Xs + (c >> 2) * PIN_PAD * 64 + cswz(pix, c & 3)) = v;
  }
  __syncthreads();

  f32x4 acc[NP][MP];
#pragma unroll
  for (int n = 0; n < NP; ++n)
#pragma unroll
    for (int m = 0; m < MP; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int dc = lane & 3;  // this lane's 8-channel group in every depthwise item
  for (int h = wave; h < nchunks; h += 4) {
    const int h0 = h * 32;
    // depthwise taps + bias and the projection columns of this chunk: issued now, used after expand
    uint4 wdr[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wdr[t] = *(const uint4*)(wd + (size_t)t * p.hid_pad + h0 + dc * 8);
    const float4 bd0 = *(const float4*)(p.bd + h0 + dc * 8), bd1 = *(const float4*)(p.bd + h0 + dc * 8 + 4);
    uint4 rwp[MP];
#pragma unroll
    for (int m = 0; m < MP; ++m) rwp[m] = *(const uint4*)(wp + (size_t)(oc_base + m * 16 + row) * p.hid_pad + h0 + kq * 8);

    // ---- expand: E[pix][32] = relu6(We[h0..h0+32] . X[pix] + be)
    const float4 be0 = *(const float4*)(p.be + h0 + kq * 4), be1 = *(const float4*)(p.be + h0 + 16 + kq * 4);
    constexpr int EU = NE <= 4 ? 4 : 1;
#pragma unroll EU
    for (int j = 0; j < NE; ++j) {
      f32x4 e0 = {be0.x, be0.y, be0.z, be0.w}, e1 = {be1.x, be1.y, be1.z, be1.w};
#pragma unroll
      for (int sl = 0; sl < NSLAB; ++sl) {
        const bf16x8 bv = *(const bf16x8*)(Xs + sl * PIN_PAD * 64 + cswz(j * 16 + row, kq));
        e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rwe[0][sl]), bv, e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rwe[1][sl]), bv, e1, 0, 0, 0);
      }
      const int pix = j * 16 + row;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int hc = mt * 16 + kq * 4;
        const f32x4 e = mt ? e1 : e0;
        float v[4] = {relu6f(e[0]), relu6f(e[1]), relu6f(e[2]), relu6f(e[3])};
        *(uint2*)(Es + cswz(pix, hc >> 3) + (hc & 7) * 2) = pack4(v);
      }
    }
    // next chunk's expand rows: in flight during this chunk's depthwise + project
    if (h + 4 < nchunks) load_we(h0 + 128);
    crop_wave_sync();

    // ---- depthwise 3x3 stride S over the whole map (zero padding = tap bounds test) -> D[49 (+15 zero)][32]
    // taps (2p, 2p+1) regrouped per channel with v_perm and multiply-added with v_dot2c_f32_bf16
    unsigned wpair[4][8];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const unsigned av[4] = {wdr[2 * pp].x, wdr[2 * pp].y, wdr[2 * pp].z, wdr[2 * pp].w};
      const unsigned cv[4] = {wdr[2 * pp + 1].x, wdr[2 * pp + 1].y, wdr[2 * pp + 1].z, wdr[2 * pp + 1].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        wpair[pp][2 * k] = __builtin_amdgcn_perm(cv[k], av[k], 0x05040100u);
        wpair[pp][2 * k + 1] = __builtin_amdgcn_perm(cv[k], av[k], 0x07060302u);
      }
    }
    float w8[8];
    unpack8(wdr[8], w8);
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int q = it * 16 + (lane >> 2);
      uint4 outv = {0u, 0u, 0u, 0u};
      if (q < nout) {
        const int oy = oy0 + q / 7, ox = q - (q / 7) * 7;
        float a[8] = {bd0.x, bd0.y, bd0.z, bd0.w, bd1.x, bd1.y, bd1.z, bd1.w};
        auto tap = [&](int t) {
          const int iy = oy * S - 1 + t / 3, ix = ox * S - 1 + t % 3;
          const bool ok = (unsigned)iy < (unsigned)HI && (unsigned)ix < (unsigned)HI;
          const uint4 v = *(const uint4*)(Es + cswz(ok ? (iy - iy_lo) * HI + ix : 0, dc));
          return ok ? v : make_uint4(0u, 0u, 0u, 0u);
        };
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const uint4 e0 = tap(2 * pp), e1 = tap(2 * pp + 1);
          const unsigned x0[4] = {e0.x, e0.y, e0.z, e0.w}, x1[4] = {e1.x, e1.y, e1.z, e1.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const unsigned lo = __builtin_amdgcn_perm(x1[k], x0[k], 0x05040100u);
            const unsigned hi = __builtin_amdgcn_perm(x1[k], x0[k], 0x07060302u);
            a[2 * k] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, lo),
                                                       __builtin_bit_cast(bf16x2, wpair[pp][2 * k]), a[2 * k], false);
            a[2 * k + 1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hi),
                                                           __builtin_bit_cast(bf16x2, wpair[pp][2 * k + 1]),
                                                           a[2 * k + 1], false);
          }
        }
        float e8[8];
        unpack8(tap(8), e8);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = relu6f(fmaf(e8[k], w8[k], a[k]));
        outv = pack8(a);
      }
      *(uint4*)(Ds + cswz(q, dc)) = outv;
    }
    crop_wave_sync();

    // ---- project: acc[px tile][oup tile] += Wp[oup][h0..h0+32] . D
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      const bf16x8 bv = *(const bf16x8*)(Ds + cswz(n * 16 + row, kq));
#pragma unroll
      for (int m = 0; m < MP; ++m)
        acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rwp[m]), bv, acc[n][m], 0, 0, 0);
    }
    // E / D are rewritten next iteration by this wave only: its LDS reads above must have returned
    crop_wave_sync();
  }

  // ---- sum the four waves' partial projections in LDS (R aliases the wave scratch), in wave order so
  // the fp32 sum is the same on every run (an ds_add_f32 race would not be bitwise reproducible)
  constexpr int OP = MP * 16;
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int n = 0; n < NP; ++n) {
        const int pix = n * 16 + row;
        if (pix < nout) {
#pragma unroll
          for (int m = 0; m < MP; ++m) {
            float4* r = (float4*)(R + pix * OP + m * 16 + kq * 4);
            float4 v = make_float4(acc[n][m][0], acc[n][m][1], acc[n][m][2], acc[n][m][3]);
            if (w) {
              const float4 o = *r;
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            *r = v;
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- epilogue: + bp (+ residual from the staged input map, stride 1) -> NHWC bf16
  bf16* yb = (bf16*)p.y + ((size_t)b * 49 + oy0 * 7) * p.y_cs;
  const int g4 = (p.oup - oc_base < OP ? p.oup - oc_base : OP) >> 2;
  const int rshift = (oy0 - iy_lo) * 7;  // output pixel -> its input pixel in the staged rows (S == 1)
  for (int i = tid; i < nout * g4; i += 256) {
    const int pix = i / g4, oc = (i - pix * g4) * 4;
    const float4 rv = *(const float4*)(R + pix * OP + oc);
    const float4 bb = *(const float4*)(p.bp + oc_base + oc);
    float v[4] = {rv.x + bb.x, rv.y + bb.y, rv.z + bb.z, rv.w + bb.w};
    if (S == 1 && p.res) {
      float r[4];
      unpack4(*(const uint2*)(Xs + (oc >> 5) * PIN_PAD * 64 + cswz(pix + rshift, (oc & 31) >> 3) + (oc & 7) * 2), r);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += r[k];
    }
    *(uint2*)(yb + (size_t)pix * p.y_cs + oc_base + oc) = pack4(v);
  }
}

template <int S, int NSLAB, int MP, int RS>
static void ir_crop_launch(const IrParams& p, hipStream_t s) {
  using G = IrCropGeom<S, NSLAB, MP, RS>;
  static_assert(G::LDS <= 160 * 1024, "ir_crop: LDS budget");
  if (p.B <= 0) return;
  hipLaunchKernelGGL((ir_crop_kernel<S, NSLAB, MP, RS>), dim3((unsigned)(p.B * RS * (p.oup_pad / (MP * 16)))), dim3(256), G::LDS, s, p);
}

#define ARENA_IR_CROP_CONFIGS(X) \
  X(2, 3, 10)                    \
  X(1, 5, 10)

void ir_crop_prepare() {
#define X(S_, NS_, MP_)                                                                            \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_crop_kernel<S_, NS_, MP_, 1>,               \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));    \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_crop_kernel<S_, NS_, MP_, 2>,               \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ARENA_IR_CROP_CONFIGS(X)
#undef X
}

static bool g_ir_crop = [] {
  const char* e = std::getenv("ARENA_IR_CROP");
  return e ? std::atoi(e) != 0 : true;
}();
void set_ir_crop(bool v) { g_ir_crop = v; }
static int g_ir_crop_split = [] {
  const char* e = std::getenv("ARENA_IR_CROP_SPLIT");
  return e ? (std::atoi(e) == 1 ? 1 : 2) : 2;
}();
void set_ir_crop_split(int v) { g_ir_crop_split = v == 1 ? 1 : 2; }

// Blocks with a 7x7 output map (input 7 at stride 1 or 14 at stride 2), an expansion and 160 or 320
// output channels (320: two workgroups per crop, one per 160-channel group, each over all 7 rows:
// splitting rows as well doubles the recomputed expansion and measured 60 us vs 51 unfused); false = not handled here (the caller falls back to the tile kernels).
bool ir_block_crop(const IrParams& p, hipStream_t s) {
  if (!g_ir_crop || !p.expand || p.Ho != 7 || p.Wo != 7 || p.H != 7 * p.stride || p.W != p.H) return false;
  if (p.oup_pad % 160 || p.oup_pad > 320 || p.oup % 4 || (p.res && (p.stride != 1 || p.oup_pad != 160))) return false;
  const int ns = p.inp_pad / 32;
#define X(S_, NS_, MP_)                                    \
  if (p.stride == S_ && ns == NS_ && p.oup_pad % (MP_ * 16) == 0) { \
    if (g_ir_crop_split == 2 && p.oup_pad == MP_ * 16)     \
      ir_crop_launch<S_, NS_, MP_, 2>(p, s);               \
    else                                                   \
      ir_crop_launch<S_, NS_, MP_, 1>(p, s);               \
    return true;                                           \
  }
  ARENA_IR_CROP_CONFIGS(X)
#undef X
  return false;
}

}  // namespace arena
