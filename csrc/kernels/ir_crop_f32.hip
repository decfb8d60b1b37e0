// Whole-map fused MobileNetV2 inverted residual at fp32 accuracy for the 14x14 and 7x7 stages
// (torchvision mobilenet_v2 features[11..17]; the reference runs them as fp32 ONNX per crop,
// architectures/monolithic/app/inference.py:196).
//
// Unfused, each of these ten blocks is three latency-bound kernels over all crops (1x1 expand GEMM
// with K = 64..160, depthwise, 1x1 project): 85-150 us per block for 128 crops, ~1.07 ms of the fp32
// device time per batch of 32 requests (profiles/r2_fp32_irprefetch_ops.md ops 79-108), the 1x1
// GEMMs at 20-30 % of the fp32 matrix-core rate.  Here one workgroup owns RS = 2 row halves of one
// crop's map (7 of 14 output rows, or 4 / 3 of 7) over OG output-channel groups, the tile spans the
// whole map width (no halo columns, no recomputed expansion except the one or two shared input
// rows), and every GEMM runs on the bf16 matrix cores with the triple-bf16 split of conv_f32.hip
// (v = h + m + l exactly; six partial products, the dropped ones below fp32's own product rounding):
//
//   X (the WG's input rows, all channels) ..... LDS, split into [h | m | l] bf16 planes once
//   (weights arrive pre-split from the host, engine/planner.py::split_bf16x3)
//   for each chunk of 32 hidden channels (2 workgroup barriers per chunk):
//     E = relu6(We[chunk] . X + be)     x3 MFMA 16x16x32 -> fp32 LDS (XOR-swizzled 16-B groups)
//     D = relu6(dw3x3_S(E) + bd)        fp32 FMA, zero padding = tap bounds test -> split planes
//     Wp[:, chunk] -> split planes      (staged alongside the depthwise)
//     acc += Wp[:, chunk] . D           x3 MFMA, accumulators in registers for the whole loop
//   y = acc + bp (+ x from global memory)                      fp32 NHWC
//
// Operand mapping of v_mfma_f32_16x16x32_bf16: lane l supplies A[row = l & 15][k = 8 (l >> 4) .. +7]
// and B[k = 8 (l >> 4) .. +7][col = l & 15] and receives D[row = 4 (l >> 4) + r][col = l & 15]: the
// expand's rows are hidden channels and its columns pixels (a lane ends with 4 consecutive hidden
// channels of one pixel: one float4 into E), the project's rows output channels, columns pixels.
//
// LDS rows that feed ds_read_b128 operand reads (16 rows x 4 k-groups per instruction) have pitches of
// 2 (mod 4) 16-byte slots (conflict-free, MI355X_MICROARCH.md §LDS): X 6 inp + 32 B, D / Wp 224 B.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

__device__ __forceinline__ void split1(float v, bf16& h, bf16& m, bf16& l) {
  h = (bf16)v;
  const float r = v - (float)h;
  m = (bf16)r;
  l = (bf16)(r - (float)m);
}

// 4 fp32 -> three bf16x4 planes at row + {0, PLANE, 2 PLANE} bytes
template <int PLANE>
__device__ __forceinline__ void store_split4(uint8_t* row, const float4& v) {
  bf16x4 h, m, l;
  const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bf16 th, tm, tl;
    split1(f[i], th, tm, tl);
    h[i] = th;
    m[i] = tm;
    l[i] = tl;
  }
  *(bf16x4*)row = h;
  *(bf16x4*)(row + PLANE) = m;
  *(bf16x4*)(row + 2 * PLANE) = l;
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

__device__ __forceinline__ float4 relu6x4(float4 v) {
  return make_float4(relu6f(v.x), relu6f(v.y), relu6f(v.z), relu6f(v.w));
}

constexpr int imin(int a, int b) { return a < b ? a : b; }

}  // namespace

// HO: output side; S: stride; KS: inp_pad / 32; MT: output-channel tiles of 16 per workgroup; RS: row parts.
// 512 threads = 8 waves, two per SIMD.  Every weight of a chunk is fetched from global memory once per
// workgroup and staged in LDS (expand rows and depthwise taps one chunk ahead, single-buffered: each is
// rewritten only in the phase after its last reader's barrier): per-wave register fetches of the expand
// fragments were 4x redundant across the waves sharing a hidden tile and, with per-thread depthwise taps,
// made the vector-memory path the bottleneck (tools/bench_irc.py: 34-143 us per block with every MFMA off).
constexpr int IRC_THREADS = 512, IRC_WAVES = IRC_THREADS / 64;

template <int HO, int S, int KS, int MT, int RS>
struct IrcGeom {
  static constexpr int HI = HO * S;                                  // input side
  static constexpr int NOR = RS == 1 ? HO : (HO + 1) / 2;            // output rows of part 0 (the larger)
  static constexpr int IR = RS == 1 ? HI : imin(HI, (NOR - 1) * S + 2);  // input rows of part 0 (>= part 1)
  static constexpr int PIN_PAD = (IR * HI + 15) / 16 * 16;
  static constexpr int NE = PIN_PAD / 16;                            // expand pixel tiles
  static constexpr int NP = (NOR * HO + 15) / 16;                    // project pixel tiles
  static constexpr int INP = KS * 32;
  static constexpr int XP = 6 * INP + 32;                            // bytes per X / We row: [h|m|l][INP] bf16 + pad
  static constexpr int EP = 128;                                     // bytes per E row: 32 fp32
  static constexpr int DP = 224;                                     // bytes per D / Wp row: [h|m|l][32] bf16 + pad
  static constexpr int X_BYTES = PIN_PAD * XP, E_BYTES = PIN_PAD * EP, D_BYTES = NP * 16 * DP;
  static constexpr int W_BYTES = MT * 16 * DP, WE_BYTES = 32 * XP, WD_BYTES = 10 * 32 * 4;  // WD: 9 taps + bias
  static constexpr int LDS = X_BYTES + E_BYTES + D_BYTES + W_BYTES + WE_BYTES + WD_BYTES;
  static constexpr int PAIRS = MT * NP, PPW = (PAIRS + IRC_WAVES - 1) / IRC_WAVES;  // project tiles (per wave)
  static constexpr int ET = (NE + IRC_WAVES / 2 - 1) / (IRC_WAVES / 2);   // expand pixel tiles per wave
  static constexpr int WPC = (MT * 16 * 12 + IRC_THREADS - 1) / IRC_THREADS;  // Wp 16-B pieces per thread
  static constexpr int WEC = (32 * 3 * INP / 8 + IRC_THREADS - 1) / IRC_THREADS;  // We 16-B pieces per thread
};

// Weights (IrParams.x3w = 1, packed by engine/planner.py::split_bf16x3): we bf16 [hid_pad][3][inp_pad] and
// wp bf16 [oup_pad][3][hid_pad] (planes h, m, l of the fp32 weight), wd fp32 [9][hid_pad], biases fp32.
template <int HO, int S, int KS, int MT, int RS>
__global__ __launch_bounds__(IRC_THREADS) void ir_crop_f32_kernel(const IrParams p) {
  using G = IrcGeom<HO, S, KS, MT, RS>;
  constexpr int HI = G::HI, INP = G::INP, XP = G::XP, NE = G::NE, DP = G::DP;
  extern __shared__ __align__(16) uint8_t lds[];
  uint8_t* Xs = lds;
  uint8_t* Es = Xs + G::X_BYTES;
  uint8_t* Ds = Es + G::E_BYTES;
  uint8_t* Ws = Ds + G::D_BYTES;
  uint8_t* WEs = Ws + G::W_BYTES;
  float* WDs = (float*)(WEs + G::WE_BYTES);  // [10][32]: taps 0..8, bias

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int og_n = p.oup_pad / (MT * 16);
  const int b = blockIdx.x / (RS * og_n), rem = blockIdx.x - b * RS * og_n;
  const int part = rem / og_n, og = rem - part * og_n, oc_base = og * MT * 16;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int oy0 = part * G::NOR;
  const int nor = RS == 1 ? HO : (part ? HO - G::NOR : G::NOR);
  const int nout = nor * HO;
  const int iy_lo = oy0 * S - 1 < 0 ? 0 : oy0 * S - 1;
  const int iy_hi = (oy0 + nor - 1) * S + 2 > HI ? HI : (oy0 + nor - 1) * S + 2;  // exclusive
  const int pin = (iy_hi - iy_lo) * HI;
  const float* xb = (const float*)p.x + ((size_t)b * HI * HI + (size_t)iy_lo * HI) * p.x_cs;
  const bf16* we = (const bf16*)p.we;
  const float* wd = (const float*)p.wd;
  const bf16* wp = (const bf16*)p.wp;
  const int hid_pad = p.hid_pad, nchunks = hid_pad >> 5;

  // chunk weight fetches into registers (global -> VGPR), stored to LDS a phase later
  uint4 wec[G::WEC], wpc[G::WPC];
  float4 wdc;
  auto fetch_we = [&](int h0) {  // piece e = (hidden row, plane, 16-B column) of the chunk's expand rows
#pragma unroll
    for (int j = 0; j < G::WEC; ++j) {
      const int e = tid + IRC_THREADS * j, row = e / (3 * KS * 4), pc = e - row * (3 * KS * 4);
      const bool ok = e < 32 * 3 * KS * 4;
      wec[j] = *(const uint4*)(we + (size_t)(h0 + (ok ? row : 0)) * (3 * INP) + pc * 8);
    }
  };
  auto store_we = [&]() {
#pragma unroll
    for (int j = 0; j < G::WEC; ++j) {
      const int e = tid + IRC_THREADS * j, row = e / (3 * KS * 4), pc = e - row * (3 * KS * 4);
      if (e < 32 * 3 * KS * 4) *(uint4*)(WEs + row * XP + pc * 16) = wec[j];
    }
  };
  auto fetch_wd = [&](int h0) {  // 80 float4: taps 0..8 and the bias, 8 per row
    const int r = tid >> 3, g = tid & 7;
    if (tid < 80) wdc = *(const float4*)((r < 9 ? wd + (size_t)r * hid_pad : p.bd) + h0 + 4 * g);
  };
  auto store_wd = [&]() {
    if (tid < 80) *(float4*)(WDs + tid * 4) = wdc;
  };
  auto fetch_wp = [&](int h0) {  // piece e = (output row, plane, 16-B column) of the chunk's project columns
#pragma unroll
    for (int j = 0; j < G::WPC; ++j) {
      const int e = tid + IRC_THREADS * j, row = e / 12, pc = e - row * 12;
      const bool ok = e < MT * 16 * 12;
      wpc[j] = *(const uint4*)(wp + ((size_t)(oc_base + (ok ? row : 0)) * 3 + (pc >> 2)) * hid_pad + h0 +
                               (pc & 3) * 8);
    }
  };
  auto store_wp = [&]() {
#pragma unroll
    for (int j = 0; j < G::WPC; ++j) {
      const int e = tid + IRC_THREADS * j, row = e / 12, pc = e - row * 12;
      if (e < MT * 16 * 12) *(uint4*)(Ws + row * DP + (pc >> 2) * 64 + (pc & 3) * 16) = wpc[j];
    }
  };
  fetch_we(0);
  fetch_wd(0);

  // ---- X: the workgroup's input rows, split into three bf16 planes (zero past inp and past pin)
  constexpr int CG = INP / 4;
  for (int i = tid; i < G::PIN_PAD * CG; i += IRC_THREADS) {
    const int pix = i / CG, g = i - pix * CG;
    const bool ok = pix < pin && 4 * g < p.inp;
    float4 v = *(const float4*)(ok ? xb + (size_t)pix * p.x_cs + 4 * g : xb);
    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
    store_split4<INP * 2>(Xs + pix * XP + g * 8, v);
  }
  store_we();
  store_wd();

  f32x4 acc[G::PPW];
#pragma unroll
  for (int j = 0; j < G::PPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int mt_e = wave & 1;  // expand: this wave's hidden tile; pixel tiles (wave >> 1) + 4 i
  const int g8 = tid & 7;     // depthwise: this thread's 4-channel group of the chunk
  __syncthreads();

  for (int h = 0; h < nchunks; ++h) {
    const int h0 = h * 32;
    const bool more = h + 1 < nchunks;
    // global fetches for later phases: this chunk's project columns, the next chunk's expand rows / taps
    fetch_wp(h0);
    if (more) {
      fetch_we(h0 + 32);
      fetch_wd(h0 + 32);
    }

    // ---- expand: E[pix][32] = relu6(We[chunk] . X + be) for this wave's hidden tile
    {
      const float4 be = *(const float4*)(p.be + h0 + mt_e * 16 + 4 * kq);
      f32x4 e[G::ET];
#pragma unroll
      for (int i = 0; i < G::ET; ++i) e[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sl = 0; sl < KS; ++sl) {
        const uint8_t* ra = WEs + (mt_e * 16 + col) * XP + sl * 64 + kq * 16;
        const bf16x8 ah = *(const bf16x8*)ra, am = *(const bf16x8*)(ra + INP * 2), al = *(const bf16x8*)(ra + INP * 4);
#pragma unroll
        for (int i = 0; i < G::ET; ++i) {
          const int j = (wave >> 1) + (IRC_WAVES / 2) * i;
          if (j >= NE) break;
          const uint8_t* r = Xs + (j * 16 + col) * XP + sl * 64 + kq * 16;
          const bf16x8 bh = *(const bf16x8*)r, bm = *(const bf16x8*)(r + INP * 2),
                       bl = *(const bf16x8*)(r + INP * 4);
          e[i] = mfma_x3(ah, am, al, bh, bm, bl, e[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < G::ET; ++i) {
        const int j = (wave >> 1) + (IRC_WAVES / 2) * i;
        if (j >= NE) break;
        const int pix = j * 16 + col, grp = mt_e * 4 + kq;
        const float4 v = relu6x4(make_float4(e[i][0] + be.x, e[i][1] + be.y, e[i][2] + be.z, e[i][3] + be.w));
        *(float4*)(Es + pix * G::EP + ((grp ^ (pix & 7)) << 4)) = v;
      }
    }
    __syncthreads();  // E complete; every wave is past its expand reads of WEs

    // ---- depthwise 3x3 (stride S) + bias + ReLU6 -> D planes; Wp(h) and We(h+1) -> LDS
    {
      float4 wk[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wk[t] = *(const float4*)(WDs + t * 32 + 4 * g8);
      const float4 bdw = *(const float4*)(WDs + 9 * 32 + 4 * g8);
      for (int q = tid >> 3; q < nout; q += IRC_THREADS / 8) {
        const int oy = oy0 + q / HO, ox = q - (q / HO) * HO;
        float4 a = bdw;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int iy = oy * S - 1 + ky;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int ix = ox * S - 1 + kx;
            const bool ok = (unsigned)iy < (unsigned)HI && (unsigned)ix < (unsigned)HI;
            const int lp = ok ? (iy - iy_lo) * HI + ix : 0;
            float4 v = *(const float4*)(Es + lp * G::EP + ((g8 ^ (lp & 7)) << 4));
            if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 w = wk[ky * 3 + kx];
            a.x = fmaf(v.x, w.x, a.x);
            a.y = fmaf(v.y, w.y, a.y);
            a.z = fmaf(v.z, w.z, a.z);
            a.w = fmaf(v.w, w.w, a.w);
          }
        }
        store_split4<64>(Ds + q * DP + g8 * 8, relu6x4(a));
      }
    }
    store_wp();
    if (more) store_we();
    __syncthreads();  // D and Wp complete; every wave is past its depthwise reads of WDs

    if (more) store_wd();
    // ---- project: acc[pair] += Wp[oc tile][chunk] . D[pixel tile]
#pragma unroll
    for (int j = 0; j < G::PPW; ++j) {
      const int pr = wave + IRC_WAVES * j;
      if (pr >= G::PAIRS) break;
      const int mt = pr % MT, nt = pr / MT;
      const uint8_t* ra = Ws + (mt * 16 + col) * DP + kq * 16;
      const uint8_t* rb = Ds + (nt * 16 + col) * DP + kq * 16;
      acc[j] = mfma_x3(*(const bf16x8*)ra, *(const bf16x8*)(ra + 64), *(const bf16x8*)(ra + 128),
                       *(const bf16x8*)rb, *(const bf16x8*)(rb + 64), *(const bf16x8*)(rb + 128), acc[j]);
    }
  }

  // ---- epilogue: + bp (+ residual, stride 1: the block input at the same pixel) -> NHWC fp32
  float* yb = (float*)p.y + ((size_t)b * HO * HO + (size_t)oy0 * HO) * p.y_cs;
  const float* xr = (const float*)p.x + ((size_t)b * HI * HI + (size_t)oy0 * HI) * p.x_cs;
#pragma unroll
  for (int j = 0; j < G::PPW; ++j) {
    const int pr = wave + IRC_WAVES * j;
    if (pr >= G::PAIRS) break;
    const int mt = pr % MT, nt = pr / MT;
    const int q = nt * 16 + col, co = oc_base + mt * 16 + 4 * kq;
    if (q >= nout || co >= p.oup) continue;
    const float4 bp = *(const float4*)(p.bp + co);
    float4 v = make_float4(acc[j][0] + bp.x, acc[j][1] + bp.y, acc[j][2] + bp.z, acc[j][3] + bp.w);
    if (S == 1 && p.res) {
      const float4 r = *(const float4*)(xr + (size_t)q * p.x_cs + co);
      v.x += r.x;
      v.y += r.y;
      v.z += r.z;
      v.w += r.w;
    }
    *(float4*)(yb + (size_t)q * p.y_cs + co) = v;
  }
}

// (HO, S, KS, MT): the MobileNetV2 14x14 / 7x7 stages at 224 (RS = 2 row parts per crop)
#define ARENA_IRC_F32_CONFIGS(X) \
  X(14, 1, 2, 4)                 \
  X(14, 1, 2, 6)                 \
  X(14, 1, 3, 6)                 \
  X(7, 2, 3, 10)                 \
  X(7, 1, 5, 10)

void ir_crop_f32_prepare() {
#define X(HO_, S_, KS_, MT_)                                                                                   \
  static_assert(IrcGeom<HO_, S_, KS_, MT_, 2>::LDS <= 160 * 1024, "ir_crop_f32: LDS budget");                  \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)ir_crop_f32_kernel<HO_, S_, KS_, MT_, 2>,                  \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  ARENA_IRC_F32_CONFIGS(X)
#undef X
}

// Shapes this kernel takes (mirrored by engine/validate.py::ir_crop_f32_supported; the planner decides which
// blocks use it and marks them with split-plane weights, IrParams.x3w): an expanding block on a
// 14x14 (stride 1 or 2) or 7x7 (stride 1) input map whose (inp_pad, oup_pad) has a configuration above.
bool ir_block_crop_f32_supported(int H, int stride, int inp_pad, int hid_pad, int oup_pad, int expand) {
  if (!expand || hid_pad % 32 || oup_pad % 16) return false;
  const int HO = (H + 2 - 3) / stride + 1;
  if (H != HO * stride) return false;
#define X(HO_, S_, KS_, MT_) \
  if (HO == HO_ && stride == S_ && inp_pad == KS_ * 32 && oup_pad % (MT_ * 16) == 0 && oup_pad <= 2 * MT_ * 16) \
    return true;
  ARENA_IRC_F32_CONFIGS(X)
#undef X
  return false;
}

bool ir_block_crop_f32(const IrParams& p, hipStream_t s) {
  if (!p.x3w) return false;  // only blocks planned for this kernel carry its split-plane weights
  if (p.H != p.W || p.Ho != p.Wo || !ir_block_crop_f32_supported(p.H, p.stride, p.inp_pad, p.hid_pad, p.oup_pad,
                                                                 p.expand))
    throw std::runtime_error("ir_crop_f32: split-plane weights for a block this kernel does not take");
  if (p.inp % 4 || p.oup % 4 || p.inp > p.inp_pad || p.oup > p.oup_pad || p.x_cs % 4 || p.y_cs % 4)
    throw std::runtime_error("ir_crop_f32: unsupported channel geometry");
  if (p.res && (p.stride != 1 || p.inp != p.oup)) throw std::runtime_error("ir_crop_f32: residual needs s1, inp == oup");
  if (p.Ho != (p.H + 2 - 3) / p.stride + 1) throw std::runtime_error("ir_crop_f32: output size mismatch");
  if (p.B <= 0) return true;
#define X(HO_, S_, KS_, MT_)                                                                              \
  if (p.Ho == HO_ && p.stride == S_ && p.inp_pad == KS_ * 32 && p.oup_pad % (MT_ * 16) == 0) {             \
    using G = IrcGeom<HO_, S_, KS_, MT_, 2>;                                                              \
    const unsigned grid = (unsigned)(p.B * 2 * (p.oup_pad / (MT_ * 16)));                                 \
    hipLaunchKernelGGL((ir_crop_f32_kernel<HO_, S_, KS_, MT_, 2>), dim3(grid),                            \
                       dim3(IRC_THREADS), G::LDS, s, p);                                                  \
    return true;                                                                                          \
  }
  ARENA_IRC_F32_CONFIGS(X)
#undef X
  return false;
}

}  // namespace arena
