// fp32-accurate implicit-GEMM convolution on the 32x32x16 bf16 matrix cores with pre-split weights ("x3g").
//
// The reference runs every detector / classifier conv in ONNX Runtime fp32
// (architectures/monolithic/app/inference.py:158-225).  The earlier fp32-accurate
// kernels (conv_f32.hip: conv_x3_lds / conv_x3_halo, 16x16x32 MFMAs) split both
// operands into three bf16 planes inside the K loop and measured 30-45 % MFMA
// busy: a v_mfma_f32_16x16x32_bf16 leaves 8 of its 16 cycles for vector issue
// (MI355X_MICROARCH.md, cycle constants), so the ~4 VALU instructions per MFMA
// of the split arithmetic and addressing set the pace.  The exact-fp32
// 16x16x4 kernels won many layers back for the same reason.  Here:
//
//   * weights are split once, at plan time (engine/planner.py pack_conv_weight_x3),
//     into [K/32][Cout_pad][h 32 | m 32 | l 32] bf16 and staged by plain copies;
//   * activations are split once per staged element (8 consecutive k per item,
//     v = h + m + l exactly, see conv_x3_lds_kernel) and each staged row feeds
//     BN / 32 MFMA tiles;
//   * the matrix op is v_mfma_f32_32x32x16_bf16: 32 cycles, 24 of them free for
//     vector issue, and half the LDS fragment reads per FLOP of the 16x16 form;
//   * six partial products per operand pair (the dropped am*bl, al*bm, al*bl are
//     below 2^-24 |a||b|), smallest first, fp32 accumulation;
//   * LDS rows of 208 B (13 16-B slots, odd): the fragment reads (lane l: row
//     l & 31, k-half l >> 5) put 16 distinct rows in each ds_read_b128 lane
//     group on 16 distinct slots; the stage is double-buffered (one barrier per
//     32-deep K chunk) and the next chunk's global loads are in flight during
//     the current chunk's MFMAs.
//
// Output tile BM pixels x BN channels per workgroup of 4 waves (WM x WN), each
// wave TM x TN tiles of 32 x 32.  Accumulator lane l holds pixel (l & 31) and
// channels 8g + 4(l >> 5) + {0..3}, g = 0..3: float4 bias / residual / output
// accesses along NHWC channels.
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // not HIP's uint4 struct: arrays of it stay in VGPRs

constexpr int XG_PITCH = 104;  // bf16 per LDS row: 3 planes x 32 k + 8 pad (208 B = 13 slots)

__host__ __device__ constexpr int xg_lds_bytes(int BM, int BN) { return 2 * (BM + BN) * XG_PITCH * 2; }

__device__ __forceinline__ int xg_xcd_remap(int bx, int nx) {
  const int q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
}

__device__ __forceinline__ f32x4 xg_load_f4(const float* p, const float* safe, bool ok) {
  const f32x4 v = *(const f32x4*)(ok ? p : safe);
  return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ u32x4 xg_load_u4(const bf16* p, const bf16* safe, bool ok) {
  const u32x4 v = *(const u32x4*)(ok ? p : safe);
  return ok ? v : u32x4{0u, 0u, 0u, 0u};
}

__device__ __forceinline__ void xg_split8(const f32x4 a, const f32x4 b, bf16x8& h, bf16x8& m, bf16x8& l) {
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
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

__device__ __forceinline__ f32x16 xg_mfma_x3(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                             const bf16x8& bh, const bf16x8& bm, const bf16x8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

}  // namespace

// IL: shape the schedule of each K step (sched_group_barrier) so the next chunk's split arithmetic and LDS stores
// issue between this chunk's MFMAs instead of after them (a wave's vector issue is free for 24 of each
// 32x32x16 MFMA's 32 cycles)
template <int WM, int WN, int TM, int TN, bool IL = false, bool SK = false>
__global__ __launch_bounds__(WM * WN * 64) void conv_x3g_kernel(const ConvParams p) {
  constexpr int NT = WM * WN * 64;  // 4 or 8 waves
  static_assert(WM * WN == 4 || WM * WN == 8, "four or eight waves");
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int AI = BM * 4 / NT;             // activation items (row, 8-k group) per thread
  constexpr int WI = (BN * 12 + NT - 1) / NT;  // 16-B weight pieces per thread (a row is 12 pieces)
  static_assert(BM * 4 % NT == 0, "every thread stages the same number of pixel rows");
  extern __shared__ __attribute__((aligned(16))) bf16 xg_lds[];
  bf16* sA = xg_lds;                     // [2][BM][XG_PITCH] activations
  bf16* sB = xg_lds + 2 * BM * XG_PITCH;  // [2][BN][XG_PITCH] weights

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int HWo = p.Ho * p.Wo;
  const int M = live_batch(p.B, p.bdev) * HWo;
  const int ntn = (p.Cout_pad + BN - 1) / BN;
  // split-K (SK): the grid is splits x tiles, split-major; each split walks its own range of K chunks and stores
  // its raw partial tile into the workspace (x3g_sk_reduce sums them in split order and runs the epilogue)
  const int nsplit = SK ? p.sk_splits : 1;
  const int ntiles = (int)gridDim.x / nsplit;
  const int split = SK ? (int)blockIdx.x / ntiles : 0;
  const int bx = xg_xcd_remap((int)blockIdx.x - split * ntiles, ntiles);
  const int mt = bx / ntn, nt = bx - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= M) return;

  // Operands are read with raw buffer loads: an out-of-range offset (conv padding, pixels past the live batch,
  // channels past Cin) returns zeros without a select per dword, offsets are 32-bit, and the weight offsets
  // are one per-thread constant plus a uniform per-chunk step (host: both tensors < 2 GiB, x3g_supported).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.B * p.H * p.W * p.xs * 4), 0x00020000);
  const int Cin32 = (p.Cin + 31) & ~31;          // each tap's channels padded to whole 32-deep chunks
  const int nk_all = p.KH * p.KW * (Cin32 >> 5);
  const int kc_begin = SK ? split * nk_all / nsplit : 0;
  const int nk = SK ? (split + 1) * nk_all / nsplit - kc_begin : nk_all;  // chunks of this workgroup
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.w3), (short)0, (int)((size_t)nk_all * p.Cout_pad * 192), 0x00020000);
  const int Cin = p.Cin, H = p.H, W = p.W, S = p.stride;
  constexpr int kOob = 0x7fffffff & ~15;  // past every buffer: the load returns zeros

  // per staged item (row, 8-k group): the input pixel of tap (0, 0) and its byte offset — fixed over the K loop
  int a_iy[AI], a_ix[AI], a_off[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int i = tid + NT * j;
    const int m = m0 + (i >> 2);
    if (m < M) {
      const int b = m / HWo, r = m - b * HWo;
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      a_iy[j] = oy * S - p.pad_t;
      a_ix[j] = ox * S - p.pad_l;
      a_off[j] = (((b * H + a_iy[j]) * W + a_ix[j]) * p.xs + 8 * (i & 3)) * 4;
    } else {
      a_iy[j] = -0x40000000;  // never inside the map
      a_ix[j] = 0;
      a_off[j] = 0;
    }
  }
  int w_off[WI];  // byte offset of this thread's 16-B weight pieces within a chunk
#pragma unroll
  for (int j = 0; j < WI; ++j) {
    const int i = tid + NT * j;
    const int row = i / 12, part = i - (i / 12) * 12;
    w_off[j] = i < BN * 12 ? ((n0 + row) * 96 + part * 8) * 2 : kOob;
  }

  // Two register sets: chunk kc + 2's global loads are issued before chunk kc's MFMAs and land in LDS after
  // chunk kc + 1's, so two chunks of matrix work (not one) cover each load's latency.
  f32x4 ra0[AI][2], ra1[AI][2];
  u32x4 rw0[WI], rw1[WI];
  // (ky, kx, c0) of the next chunk to load: chunks are loaded strictly in order, so a running position
  // replaces a division per chunk (the weight layout pads each tap to Cin32: a chunk never straddles two taps)
  int ld_ky = 0, ld_kx = 0, ld_c0 = 0;
  if (SK) {  // the split's first chunk
    const int cpt = Cin32 >> 5, tap = kc_begin / cpt;
    ld_c0 = (kc_begin - tap * cpt) * 32;
    ld_ky = tap / p.KW;
    ld_kx = tap - ld_ky * p.KW;
  }
  auto load = [&](int kc_local, f32x4 (&ra)[AI][2], u32x4 (&rw)[WI]) {
    const int kc = kc_begin + kc_local;  // weight chunk index
    const int ky = ld_ky, kx = ld_kx, c0 = ld_c0;
    ld_c0 += 32;  // advanced with selects, not branches: the K step stays one scheduling region
    const bool wrap = ld_c0 >= Cin32;
    ld_c0 = wrap ? 0 : ld_c0;
    ld_kx += wrap ? 1 : 0;
    const bool wrap2 = ld_kx == p.KW;
    ld_kx = wrap2 ? 0 : ld_kx;
    ld_ky += wrap2 ? 1 : 0;
    const int step = ((ky * W + kx) * p.xs + c0) * 4;  // uniform
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int i = tid + NT * j;
      const int c = c0 + 8 * (i & 3);
      const bool in = (unsigned)(a_iy[j] + ky) < (unsigned)H && (unsigned)(a_ix[j] + kx) < (unsigned)W;
      const int o0 = in && c < Cin ? a_off[j] + step : kOob;
      const int o1 = in && c + 4 < Cin ? a_off[j] + step + 16 : kOob;
      ra[j][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
      ra[j][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
    }
    const int wstep = kc * p.Cout_pad * 192;  // uniform: chunk kc's rows
#pragma unroll
    for (int j = 0; j < WI; ++j) rw[j] = __builtin_amdgcn_raw_buffer_load_b128(wr, w_off[j], wstep, 0);
  };
  auto store = [&](int buf, const f32x4 (&ra)[AI][2], const u32x4 (&rw)[WI]) {
    bf16* a = sA + buf * BM * XG_PITCH;
    bf16* bw = sB + buf * BN * XG_PITCH;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int i = tid + NT * j;
      bf16x8 h, m, l;
      xg_split8(ra[j][0], ra[j][1], h, m, l);
      bf16* d = a + (i >> 2) * XG_PITCH + 8 * (i & 3);
      *(bf16x8*)d = h;
      *(bf16x8*)(d + 32) = m;
      *(bf16x8*)(d + 64) = l;
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int i = tid + NT * j;
      if (BN * 12 % NT == 0 || i < BN * 12) {
        const int row = i / 12, part = i - (i / 12) * 12;
        *(u32x4*)(bw + row * XG_PITCH + part * 8) = rw[j];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int fr = lane & 31, fk = 8 * (lane >> 5);
  auto compute = [&](int buf) {
    const bf16* a = sA + buf * BM * XG_PITCH;
    const bf16* bw = sB + buf * BN * XG_PITCH;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 wh[TN], wmid[TN], wl[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const bf16* r = bw + ((wn * TN + tn) * 32 + fr) * XG_PITCH + ks * 16 + fk;
        wh[tn] = *(const bf16x8*)r;
        wmid[tn] = *(const bf16x8*)(r + 32);
        wl[tn] = *(const bf16x8*)(r + 64);
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const bf16* r = a + ((wm * TM + tm) * 32 + fr) * XG_PITCH + ks * 16 + fk;
        const bf16x8 xh = *(const bf16x8*)r, xm = *(const bf16x8*)(r + 32), xl = *(const bf16x8*)(r + 64);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = xg_mfma_x3(wh[tn], wmid[tn], wl[tn], xh, xm, xl, acc[tm][tn]);
      }
    }
  };

  load(0, ra0, rw0);
  if (nk > 1) load(1, ra1, rw1);
  store(0, ra0, rw0);
  __syncthreads();
  int kc = 0;
  constexpr int NMF = TM * TN * 12;                   // MFMAs per wave per chunk
  constexpr int NVA = (AI * 40 + NMF - 1) / NMF;       // ~split VALU per MFMA slot
  auto shape = [&]() {
    if constexpr (IL) {
#pragma unroll
      for (int i = 0; i < NMF; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, NVA, 0);  // then a few VALU of the split
        if (i % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // and an LDS store
      }
    }
  };
  // Branch-free body (one scheduling region per chunk): loads past the last chunk read zeros (out-of-range
  // buffer offsets) and the buffer they are stored into is not read again.
  for (; kc + 1 < nk; kc += 2) {  // chunk kc in buffer 0, kc + 1 in registers set 1
    load(kc + 2, ra0, rw0);
    compute(0);
    store(1, ra1, rw1);
    shape();
    __syncthreads();
    load(kc + 3, ra1, rw1);
    compute(1);
    store(0, ra0, rw0);
    shape();
    __syncthreads();
  }
  if (kc < nk) compute(0);  // odd chunk count: the last chunk is in buffer 0

  const int kh4 = 4 * (lane >> 5);
  if constexpr (SK) {  // raw partial sums: ws[split][m][Cout_pad]
    const int Mcap = p.B * HWo;
    float* ws = p.sk_ws + (size_t)split * Mcap * p.Cout_pad;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int m = m0 + (wm * TM + tm) * 32 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = n0 + (wn * TN + tn) * 32 + 8 * g + kh4;
          if (c >= p.Cout) continue;
          *(float4*)(ws + (size_t)m * p.Cout_pad + c) =
              make_float4(acc[tm][tn][4 * g], acc[tm][tn][4 * g + 1], acc[tm][tn][4 * g + 2], acc[tm][tn][4 * g + 3]);
        }
    }
    return;
  }

  // ---- epilogue: bias, activation, residual, NHWC fp32 (+ 2x nearest-upsampled copy)
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int m = m0 + (wm * TM + tm) * 32 + fr;
    if (m >= M) continue;
    int b = 0, oy = 0, ox = 0;
    if (p.y2 != nullptr) {
      b = m / HWo;
      const int r = m - b * HWo;
      oy = r / p.Wo;
      ox = r - oy * p.Wo;
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = n0 + (wn * TN + tn) * 32 + 8 * g + kh4;
        if (c >= p.Cout) continue;
        const float4 bias = *(const float4*)(p.bias + c);
        float v[4] = {acc[tm][tn][4 * g] + bias.x, acc[tm][tn][4 * g + 1] + bias.y, acc[tm][tn][4 * g + 2] + bias.z,
                      acc[tm][tn][4 * g + 3] + bias.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
        if (p.res != nullptr) {
          const float4 rv = *(const float4*)((const float*)p.res + (size_t)m * p.rs + c);
          v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
        }
        const float4 o = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)((float*)p.y + (size_t)m * p.ys + c) = o;
        if (p.y2 != nullptr) {
          const int W2 = 2 * p.Wo;
          float* y2 = (float*)p.y2;
          const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
          *(float4*)(y2 + base * p.y2s + c) = o;
          *(float4*)(y2 + (base + 1) * p.y2s + c) = o;
          *(float4*)(y2 + (base + W2) * p.y2s + c) = o;
          *(float4*)(y2 + (base + W2 + 1) * p.y2s + c) = o;
        }
      }
    }
  }
}


// Split-K second pass: out = act(sum_s ws[s] + bias) (+ residual), the x3g epilogue per 4 channels of a pixel.
// The partials are summed in split order, so the result does not depend on which split finished first.
__global__ __launch_bounds__(256) void x3g_sk_reduce_kernel(const ConvParams p) {
  const int HWo = p.Ho * p.Wo;
  const int M = live_batch(p.B, p.bdev) * HWo, Mcap = p.B * HWo;
  const int c4n = p.Cout >> 2;
  const int i = (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (i >= M * c4n) return;
  const int m = i / c4n, c = 4 * (i - m * c4n);
  float4 a = *(const float4*)(p.sk_ws + (size_t)m * p.Cout_pad + c);
  for (int k = 1; k < p.sk_splits; ++k) {
    const float4 v = *(const float4*)(p.sk_ws + ((size_t)k * Mcap + m) * p.Cout_pad + c);
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  const float4 bias = *(const float4*)(p.bias + c);
  float v[4] = {a.x + bias.x, a.y + bias.y, a.z + bias.z, a.w + bias.w};
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
  if (p.res != nullptr) {
    const float4 rv = *(const float4*)((const float*)p.res + (size_t)m * p.rs + c);
    v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
  }
  const float4 o = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)((float*)p.y + (size_t)m * p.ys + c) = o;
  if (p.y2 != nullptr) {
    const int b = m / HWo, r = m - b * HWo, oy = r / p.Wo, ox = r - oy * p.Wo;
    const int W2 = 2 * p.Wo;
    float* y2 = (float*)p.y2;
    const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
    *(float4*)(y2 + base * p.y2s + c) = o;
    *(float4*)(y2 + (base + 1) * p.y2s + c) = o;
    *(float4*)(y2 + (base + W2) * p.y2s + c) = o;
    *(float4*)(y2 + (base + W2 + 1) * p.y2s + c) = o;
  }
}

namespace {

template <int WM, int WN, int TM, int TN, bool IL>
void xg_launch(const ConvParams& p, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const long M = (long)p.B * p.Ho * p.Wo;
  const long tiles = ((M + BM - 1) / BM) * ((p.Cout_pad + BN - 1) / BN);
  hipLaunchKernelGGL((conv_x3g_kernel<WM, WN, TM, TN, IL>), dim3((unsigned)tiles), dim3(WM * WN * 64), xg_lds_bytes(BM, BN), s,
                     p);
}

// split-K: tile variant (XG_VARIANTS id) x splits; a workspace of splits x B x Ho x Wo x Cout_pad fp32 (ConvParams
// sk_ws, per executor slot and lane) holds the partial tiles
template <int WM, int WN, int TM, int TN>
bool xg_launch_sk(const ConvParams& p, hipStream_t s, int splits) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const long M = (long)p.B * p.Ho * p.Wo;
  const int nk = p.KH * p.KW * ((p.Cin + 31) / 32);
  splits = splits < nk ? splits : nk;  // at most one K chunk per split
  if (p.sk_ws == nullptr || splits < 2 || (long)splits * M * p.Cout_pad * 4 > p.sk_ws_bytes || p.Cout_pad % 4)
    return false;
  const long tiles = ((M + BM - 1) / BM) * ((p.Cout_pad + BN - 1) / BN);
  ConvParams q = p;
  q.sk_splits = splits;
  hipLaunchKernelGGL((conv_x3g_kernel<WM, WN, TM, TN, false, true>), dim3((unsigned)(tiles * splits)),
                     dim3(WM * WN * 64), xg_lds_bytes(BM, BN), s, q);
  const long items = M * (p.Cout / 4);
  hipLaunchKernelGGL(x3g_sk_reduce_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, q);
  return true;
}

#define XG_SK_VARIANTS(X) \
  X(0, 2, 2, 1, 1, 2)  /* 64 px x 64 ch */ \
  X(1, 2, 2, 1, 1, 4)  \
  X(2, 2, 2, 1, 1, 8)  \
  X(3, 4, 1, 1, 1, 2)  /* 128 px x 32 ch */ \
  X(4, 4, 1, 1, 1, 4)  \
  X(5, 4, 1, 1, 1, 8)  \
  X(6, 2, 2, 1, 2, 2)  /* 64 px x 128 ch */ \
  X(7, 2, 2, 1, 2, 4)  \
  X(8, 2, 2, 1, 2, 8)

#define XG_VARIANTS(X) \
  X(0, 2, 2, 2, 1)     /* 128 px x  64 ch */ \
  X(1, 2, 2, 2, 2)     /* 128 px x 128 ch */ \
  X(2, 4, 1, 1, 1)     /* 128 px x  32 ch */ \
  X(3, 4, 1, 1, 2)     /* 128 px x  64 ch, one 32-px row per wave */ \
  X(4, 2, 2, 1, 2)     /*  64 px x 128 ch */ \
  X(5, 2, 2, 1, 1)     /*  64 px x  64 ch */ \
  X(6, 2, 4, 2, 1)     /* 128 px x 128 ch, 8 waves */ \
  X(7, 4, 2, 1, 2)     /* 128 px x 128 ch, 8 waves */ \
  X(8, 4, 2, 2, 1)     /* 256 px x  64 ch, 8 waves */ \
  X(9, 4, 2, 1, 1)     /* 128 px x  64 ch, 8 waves */


}  // namespace

bool x3g_supported(const ConvParams& p) {
  const size_t x_bytes = (size_t)p.B * p.H * p.W * p.xs * 4;
  const size_t w_bytes = (size_t)p.KH * p.KW * ((p.Cin + 31) / 32) * p.Cout_pad * 192;
  return p.w3 != nullptr && x_bytes < (1u << 31) - (1u << 20) && w_bytes < (1u << 31) - (1u << 20) && p.Cin % 4 == 0 && p.xs % 4 == 0 && p.Kpad >= p.KH * p.KW * p.Cin &&
         p.Cout % 4 == 0 && p.ys % 4 == 0 &&
         (p.res == nullptr || p.rs % 4 == 0) && (p.y2 == nullptr || p.y2s % 4 == 0) && p.lb_meta == nullptr &&
         p.pw_w == nullptr;
}

bool conv_x3g(const ConvParams& p, hipStream_t s, int v) {
  if (!x3g_supported(p)) return false;
  switch (v) {
#define XG_CASE(V, WM, WN, TM, TN) \
  case V: xg_launch<WM, WN, TM, TN, false>(p, s); return true; \
  case V + 10: xg_launch<WM, WN, TM, TN, true>(p, s); return true;
    XG_VARIANTS(XG_CASE)
#undef XG_CASE
    default: return false;
  }
}

bool conv_x3g_sk(const ConvParams& p, hipStream_t s, int v) {
  if (!x3g_supported(p) || p.Cout % 4) return false;
  switch (v) {
// a shape the workspace cannot hold (a larger crop capacity than the table was tuned with) or with a single K chunk
// runs the same tile unsplit
#define XG_SK_CASE(V, WM, WN, TM, TN, S)                                   \
  case V:                                                                  \
    if (!xg_launch_sk<WM, WN, TM, TN>(p, s, S)) xg_launch<WM, WN, TM, TN, false>(p, s); \
    return true;
    XG_SK_VARIANTS(XG_SK_CASE)
#undef XG_SK_CASE
    default: return false;
  }
}

void x3g_prepare() {
#define XG_ATTR(V, WM, WN, TM, TN)                                                                       \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3g_kernel<WM, WN, TM, TN, false>,                \
                                      hipFuncAttributeMaxDynamicSharedMemorySize,                         \
                                      xg_lds_bytes(WM * TM * 32, WN * TN * 32)));                         \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3g_kernel<WM, WN, TM, TN, true>,                 \
                                      hipFuncAttributeMaxDynamicSharedMemorySize,                         \
                                      xg_lds_bytes(WM * TM * 32, WN * TN * 32)));
  XG_VARIANTS(XG_ATTR)
#undef XG_ATTR
#define XG_SK_ATTR(V, WM, WN, TM, TN, S)                                                                  \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3g_kernel<WM, WN, TM, TN, false, true>,          \
                                      hipFuncAttributeMaxDynamicSharedMemorySize,                         \
                                      xg_lds_bytes(WM * TM * 32, WN * TN * 32)));
  XG_SK_VARIANTS(XG_SK_ATTR)
#undef XG_SK_ATTR
}

}  // namespace arena
