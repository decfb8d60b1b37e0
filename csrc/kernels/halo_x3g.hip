// fp32-accurate 3x3 stride-1 convolution: halo tiles on the 32x32x16 bf16 matrix cores over pre-split
// weights ("x3hg").
//
// The detector's 3x3 stride-1 convs (detect-head cv2/cv3 stacks at 80x80 / 40x40, C3 bottlenecks) ran on
// conv_x3_halo_kernel (conv_f32.hip): 16x16x32 MFMAs, weights split into bf16 planes inside the K loop, two
// barriers per stage and a 32-deep K step.  Its PMC profile (profiles/r3b_pmc_hbm_ops.md, ops 51-58) shows
// 34-42 % MFMA busy, LDS reads at ~3/4 of the MFMA time (every weight fragment feeds 4 MFMAs) and, for the
// 80-channel cls branch, 1.44x padded work (K 80 -> 96, N 80 -> 96).  Here:
//
//   * the weights come pre-split from the plan (engine/planner.py pack_conv_weight_x3, the x3g layout
//     [tap * Cin32 / 32 + c / 32][Cout_pad][h 32 | m 32 | l 32]): a stage's weights are staged by plain
//     16-byte copies, no split arithmetic;
//   * the K step is one tap x 16 input channels (one v_mfma_f32_32x32x16_bf16 deep): Cin 80 is five exact
//     chunks, no zero padding in K;
//   * each staged input halo chunk (16 channels, split once into h | m | l planes on the way into LDS)
//     feeds all nine taps; the weight stage is double-buffered, so there is one barrier per tap (two at a
//     chunk boundary, where the halo is replaced), and the next stage's global loads are in flight during
//     the current stage's MFMAs (the next chunk's halo during all nine taps of the current one; loading two
//     stages ahead measured slower everywhere: the second register set costs occupancy);
//   * 32x32x16 fragments read half the LDS bytes per MAC of the 16x16x32 form, and every wave holds TM
//     pixel fragments: per tap a wave reads TM + TN fragment triples for 6 TM TN MFMAs.
//
// Six partial products per operand pair (am*bm, al*bh, ah*bl, am*bh, ah*bm, ah*bh, smallest first; the
// dropped am*bl, al*bm, al*bl are below 2^-24 |a||b|), fp32 accumulation: the error bound of the other
// fp32-accurate kernels (tests/test_fp32_gpu.py).
//
// Workgroup: WM x WN waves.  Output tile TH x TW pixels of one image x BN channels; a pixel fragment is
// 32 pixels = (32 / TW) rows x TW columns, wave (wm, wn) computes pixel fragments wm*TM .. +TM-1 and
// channel fragments wn*TN .. +TN-1 (32 channels each).  Accumulator lane l holds pixel (l & 31) of its
// fragment and channels 8g + 4(l >> 5) + {0..3}, g = 0..3: float4 bias / residual / output accesses.
// LDS rows (halo pixels and weight rows) are 112 B = 7 16-B slots (odd): 16 consecutive rows of a
// ds_read_b128 lane group land on 16 distinct slots.
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int HG_P = 56;  // bf16 per LDS row: 3 planes x 16 k + 8 pad (112 B)

__host__ __device__ constexpr int hg_th(int TW, int WM, int TM) { return WM * TM * (32 / TW); }
__host__ __device__ constexpr int hg_lds_bytes(int TW, int WM, int WN, int TM, int TN) {
  return ((hg_th(TW, WM, TM) + 2) * (TW + 2) + 2 * WN * TN * 32) * HG_P * 2;
}
__host__ __device__ constexpr int hr_lds_bytes(int TW, int WM, int TM) {  // x3hr: the halo only
  return (hg_th(TW, WM, TM) + 2) * (TW + 2) * HG_P * 2;
}

__device__ __forceinline__ int hg_xcd_remap(int bx, int nx) {
  const int q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
}

__device__ __forceinline__ f32x16 hg_mfma_x3(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                             const bf16x8& bh, const bf16x8& bm, const bf16x8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

}  // namespace

// ---- epilogue shared by the x3hg / x3hr kernels: acc[tm][tn] of wave (wm, wn) for the tile (b, oy0, ox0, n0)
template <int TW, int WM, int WN, int TM, int TN, int PWN>
__device__ __forceinline__ void hg_epilogue(const ConvParams& p, f32x16 (&acc)[TM][TN], int b, int oy0, int ox0,
                                            int n0, int wm, int wn, int lane) {
  constexpr int RF = 32 / TW, BN = WN * TN * 32;
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  const int kh4 = 4 * (lane >> 5);
  if constexpr (PWN > 0) {
    // ---- fused 1x1: out2 = W2 . act(conv + bias) + b2 (+ act2), the 3x3 result is not stored
    constexpr int K2 = BN;
    const bf16* __restrict__ w2 = (const bf16*)p.pw_w;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      bf16x8 bh[2 * TN], bm[2 * TN], bl[2 * TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          float v[8];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int g = 2 * sh + q;
            const int ch = n0 + tn * 32 + 8 * g + kh4;
            const bool ok = ch < p.Cout;
            const float4 bias = ok ? *(const float4*)(p.bias + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) v[4 * q + e] = ok ? apply_act(acc[tm][tn][4 * g + e] + bb[e], p.act) : 0.f;
          }
          const int ks = 2 * tn + sh;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const bf16 th = (bf16)v[e];
            const float r = v[e] - (float)th;
            const bf16 tmid = (bf16)r;
            bh[ks][e] = th;
            bm[ks][e] = tmid;
            bl[ks][e] = (bf16)(r - (float)tmid);
          }
        }
      const int r = (wm * TM + tm) * RF + fr / TW, c = fr % TW;
      const int oy = oy0 + r, ox = ox0 + c;
      const bool live = oy < p.Ho && ox < p.Wo;
      const size_t pix = ((size_t)b * p.Ho + oy) * p.Wo + ox;
#pragma unroll
      for (int t2 = 0; t2 < PWN; ++t2) {
        f32x16 a2;
#pragma unroll
        for (int e = 0; e < 16; ++e) a2[e] = 0.f;
        const bf16* wrow = w2 + (size_t)((t2 * 32 + fr) * 3) * K2 + fk;
#pragma unroll
        for (int ks = 0; ks < 2 * TN; ++ks) {
          const bf16x8 wh = *(const bf16x8*)(wrow + 16 * ks);
          const bf16x8 wmid = *(const bf16x8*)(wrow + K2 + 16 * ks);
          const bf16x8 wl = *(const bf16x8*)(wrow + 2 * K2 + 16 * ks);
          a2 = hg_mfma_x3(wh, wmid, wl, bh[ks], bm[ks], bl[ks], a2);
        }
        if (!live) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ch = t2 * 32 + 8 * g + kh4;
          if (ch >= p.pw_cout) continue;
          const float4 bias = *(const float4*)(p.pw_bias + ch);
          const float4 o = make_float4(apply_act(a2[4 * g] + bias.x, p.pw_act), apply_act(a2[4 * g + 1] + bias.y, p.pw_act),
                                       apply_act(a2[4 * g + 2] + bias.z, p.pw_act), apply_act(a2[4 * g + 3] + bias.w, p.pw_act));
          *(float4*)((float*)p.pw_y + pix * p.pw_ys + ch) = o;
        }
      }
    }
    return;
  }
  // ---- epilogue: bias, activation, residual, NHWC fp32 (+ 2x nearest-upsampled copy)
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = (wm * TM + tm) * RF + fr / TW, c = fr % TW;
    const int oy = oy0 + r, ox = ox0 + c;
    if (oy >= p.Ho || ox >= p.Wo) continue;
    const size_t pix = ((size_t)b * p.Ho + oy) * p.Wo + ox;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = n0 + (wn * TN + tn) * 32 + 8 * g + kh4;
        if (ch >= p.Cout) continue;
        const float4 bias = *(const float4*)(p.bias + ch);
        float v[4] = {acc[tm][tn][4 * g] + bias.x, acc[tm][tn][4 * g + 1] + bias.y, acc[tm][tn][4 * g + 2] + bias.z,
                      acc[tm][tn][4 * g + 3] + bias.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
        if (p.res != nullptr) {
          const float4 rv = *(const float4*)((const float*)p.res + pix * p.rs + ch);
          v[0] += rv.x; v[1] += rv.y; v[2] += rv.z; v[3] += rv.w;
        }
        const float4 o = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)((float*)p.y + pix * p.ys + ch) = o;
        if (p.y2 != nullptr) {
          const int W2 = 2 * p.Wo;
          float* y2 = (float*)p.y2;
          const size_t base = ((size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
          *(float4*)(y2 + base * p.y2s + ch) = o;
          *(float4*)(y2 + (base + 1) * p.y2s + ch) = o;
          *(float4*)(y2 + (base + W2) * p.y2s + ch) = o;
          *(float4*)(y2 + (base + W2 + 1) * p.y2s + ch) = o;
        }
      }
    }
  }
}

// PWN > 0: the Detect head's final 1x1 conv (PWN x 32 >= its output channels) is applied to the activated
// 3x3 result inside the epilogue and only its output is stored (ConvParams.pw_*; WN = 1 and one channel tile,
// so every wave holds all 3x3 channels of its pixels).  The 1x1 contracts over the 3x3 channels in the order
// the accumulators hold them: k-step ks = 2 tn + s, lane half h supplies channels 32 tn + 16 s + 4 h + {0..3}
// and 32 tn + 16 s + 8 + 4 h + {0..3}, so the split 3x3 output feeds the MFMA straight from registers and the
// 1x1 weights are pre-split with their K columns in that order (engine/planner.py pack_pw_weight_x3):
// [PWN * 32 rows][h | m | l][K2 = BN].
template <int TW, int WM, int WN, int TM, int TN, int PWN = 0>
__global__ __launch_bounds__(WM * WN * 64) void conv_x3hg_kernel(const ConvParams p) {
  static_assert(PWN == 0 || WN == 1, "the fused 1x1 needs every 3x3 channel of a pixel in one wave");
  constexpr int NT = WM * WN * 64;
  constexpr int RF = 32 / TW;                         // rows per pixel fragment
  constexpr int TH = WM * TM * RF;                    // tile rows
  constexpr int HC = TW + 2, HPIX = (TH + 2) * HC;    // halo columns, pixels
  constexpr int BN = WN * TN * 32;
  constexpr int XI = (HPIX * 4 + NT - 1) / NT;        // halo float4 items (pixel, 4-channel quarter) per thread
  constexpr int WI = (BN * 6 + NT - 1) / NT;          // 16-B weight pieces per thread per stage (6 per row)
  extern __shared__ __attribute__((aligned(16))) bf16 hg_lds[];
  bf16* sX = hg_lds;                 // [HPIX][HG_P]
  bf16* sW = hg_lds + HPIX * HG_P;   // [2][BN][HG_P]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int ntn = (p.Cout_pad + BN - 1) / BN;
  const int per_img = tiles_x * tiles_y * ntn;
  const int bx = hg_xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / per_img;
  if (b >= live_batch(p.B, p.bdev)) return;
  int t = bx - b * per_img;
  const int nt = t % ntn;  // channel tiles of one pixel tile are neighbours (same XCD: shared halo in L2)
  t /= ntn;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW, n0 = nt * BN;
  const int iy0 = oy0 - p.pad_t, ix0 = ox0 - p.pad_l;
  const int H = p.H, W = p.W, Cin = p.Cin;

  // raw buffer loads: out-of-range offsets (halo outside the map, channels past Cin, weight rows past
  // Cout_pad) read zeros; host: both tensors < 2 GiB (x3hg_supported)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.B * H * W * p.xs * 4), 0x00020000);
  const int cin32 = (Cin + 31) >> 5;  // 32-deep chunks per tap in the x3g weight layout
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.w3), (short)0, (int)((size_t)9 * cin32 * p.Cout_pad * 192), 0x00020000);
  constexpr int kOob = 0x7fffffff & ~15;

  // per halo item: byte offset of its (pixel, quarter) at channel chunk 0, or kOob
  int x_off[XI];
  const size_t img = (size_t)b * H * W;
#pragma unroll
  for (int j = 0; j < XI; ++j) {
    const int i = tid + NT * j;
    const int px = i >> 2, q = i & 3;
    const int hy = px / HC, hx = px - hy * HC;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool in = i < HPIX * 4 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    x_off[j] = in ? (int)(((img + (size_t)iy * W + ix) * p.xs + 4 * q) * 4) : kOob;
  }
  // per weight piece: (row, plane, half) -> byte offset within a 32-deep chunk's row block, or kOob
  int w_off[WI];
#pragma unroll
  for (int j = 0; j < WI; ++j) {
    const int i = tid + NT * j;
    const int row = i / 6, piece = i - (i / 6) * 6;
    const int n = n0 + row;
    w_off[j] = (i < BN * 6 && n < p.Cout_pad) ? (n * 96 + (piece >> 1) * 32 + 8 * (piece & 1)) * 2 : kOob;
  }

  f32x4 rx[XI];
  u32x4 rw[WI];
  auto load_x = [&](int cc) {  // 16 input channels c = 16 cc + 4 q .. + 3 of every halo pixel
#pragma unroll
    for (int j = 0; j < XI; ++j) {
      const int i = tid + NT * j;
      const int c = 16 * cc + 4 * (i & 3);
      const int o = (x_off[j] != kOob && c < Cin) ? x_off[j] + 64 * cc : kOob;
      rx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int j = 0; j < XI; ++j) {
      const int i = tid + NT * j;
      if (HPIX * 4 % NT == 0 || i < HPIX * 4) {
        bf16x4 h, m, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = rx[j][e];
          const bf16 th = (bf16)v;
          const float r = v - (float)th;
          const bf16 tm = (bf16)r;
          h[e] = th;
          m[e] = tm;
          l[e] = (bf16)(r - (float)tm);
        }
        bf16* d = sX + (i >> 2) * HG_P + 4 * (i & 3);
        *(bf16x4*)d = h;
        *(bf16x4*)(d + 16) = m;
        *(bf16x4*)(d + 32) = l;
      }
    }
  };
  auto load_w = [&](int st) {  // stage st = (chunk cc, tap): 16 k of the tap's 32-deep chunk cc / 2
    const int cc = st / 9, tap = st - cc * 9;
    const int step = ((tap * cin32 + (cc >> 1)) * p.Cout_pad * 96 + 16 * (cc & 1)) * 2;  // uniform
#pragma unroll
    for (int j = 0; j < WI; ++j) rw[j] = __builtin_amdgcn_raw_buffer_load_b128(wr, w_off[j], step, 0);
  };
  auto store_w = [&](int buf) {
    bf16* d = sW + buf * BN * HG_P;
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int i = tid + NT * j;
      if (BN * 6 % NT == 0 || i < BN * 6) {
        const int row = i / 6, piece = i - (i / 6) * 6;
        *(u32x4*)(d + row * HG_P + (piece >> 1) * 16 + 8 * (piece & 1)) = rw[j];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  const int fr = lane & 31, fk = 8 * (lane >> 5);
  // halo pixel of this lane's fragment pixel at tap (0, 0), per pixel fragment
  int xpix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = (wm * TM + tm) * RF + fr / TW, c = fr % TW;
    xpix[tm] = r * HC + c;
  }
  auto compute = [&](int buf, int tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ky * HC + kx;
    bf16x8 xh[TM], xm[TM], xl[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const bf16* r = sX + (xpix[tm] + toff) * HG_P + fk;
      xh[tm] = *(const bf16x8*)r;
      xm[tm] = *(const bf16x8*)(r + 16);
      xl[tm] = *(const bf16x8*)(r + 32);
    }
    const bf16* wb = sW + buf * BN * HG_P;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const bf16* r = wb + ((wn * TN + tn) * 32 + fr) * HG_P + fk;
      const bf16x8 wh = *(const bf16x8*)r, wmid = *(const bf16x8*)(r + 16), wl = *(const bf16x8*)(r + 32);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) acc[tm][tn] = hg_mfma_x3(wh, wmid, wl, xh[tm], xm[tm], xl[tm], acc[tm][tn]);
    }
  };

  const int nc = (Cin + 15) >> 4, ns = nc * 9;
  load_x(0);
  load_w(0);
  store_x();
  store_w(0);
  __syncthreads();
  for (int st = 0; st < ns; ++st) {
    const int cc = st / 9, tap = st - cc * 9;
    const bool more = st + 1 < ns;
    if (more) load_w(st + 1);
    if (tap == 0 && cc + 1 < nc) load_x(cc + 1);  // lands during this chunk's nine taps
    compute(st & 1, tap);
    if (more) {
      if (tap == 8) {  // every wave is done with this chunk's halo before it is replaced
        __syncthreads();
        store_x();
      }
      store_w((st + 1) & 1);
      __syncthreads();
    }
  }

  hg_epilogue<TW, WM, WN, TM, TN, PWN>(p, acc, b, oy0, ox0, n0, wm, wn, lane);
}

// x3hr: the x3hg tile with its weights read by every wave straight from global memory (L1 / L2-resident: the
// layer's pre-split planes are 28-83 KB) into fragment registers one tap ahead, instead of through a
// double-buffered LDS stage.  x3hg's per-tap stage ended in a barrier, so every tap waited for the slowest wave's
// weight load and LDS store (round-6 PMC, profiles/r6base/ops_pmc.md: ops 48 / 49 at 42-48 % MFMA busy with
// 32-38 % of wave cycles issue-stalled and 38-45 % parked).  Here the only barriers are the two around the halo
// replacement once per 16-channel chunk, the LDS holds the halo alone (18-36 KB instead of 34-57 KB: more
// workgroups per CU), and the next chunk's halo is loaded in pieces, one per tap after that tap's weight load, so
// waiting for a weight fragment never waits for more than one tap's worth of halo loads (vmcnt counts in order).
// The arithmetic (six partial products per operand pair, 16-deep K steps, fp32 accumulation) and the epilogue are
// x3hg's, so results are bit-identical to it.
template <int TW, int WM, int WN, int TM, int TN, int PWN = 0>
__global__ __launch_bounds__(WM * WN * 64) void conv_x3hr_kernel(const ConvParams p) {
  static_assert(PWN == 0 || WN == 1, "the fused 1x1 needs every 3x3 channel of a pixel in one wave");
  constexpr int NT = WM * WN * 64;
  constexpr int RF = 32 / TW;
  constexpr int TH = WM * TM * RF;
  constexpr int HC = TW + 2, HPIX = (TH + 2) * HC;
  constexpr int BN = WN * TN * 32;
  constexpr int XI = (HPIX * 4 + NT - 1) / NT;        // halo float4 items per thread
  constexpr int XP = (XI + 7) / 8;                    // items issued per tap (the chunk's halo over taps 0..7)
  extern __shared__ __attribute__((aligned(16))) bf16 hg_lds[];
  bf16* sX = hg_lds;  // [HPIX][HG_P]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int tiles_x = (p.Wo + TW - 1) / TW, tiles_y = (p.Ho + TH - 1) / TH;
  const int ntn = (p.Cout_pad + BN - 1) / BN;
  const int per_img = tiles_x * tiles_y * ntn;
  const int bx = hg_xcd_remap(blockIdx.x, gridDim.x);
  const int b = bx / per_img;
  if (b >= live_batch(p.B, p.bdev)) return;
  int t = bx - b * per_img;
  const int nt = t % ntn;
  t /= ntn;
  const int ty = t / tiles_x, tx = t - ty * tiles_x;
  const int oy0 = ty * TH, ox0 = tx * TW, n0 = nt * BN;
  const int iy0 = oy0 - p.pad_t, ix0 = ox0 - p.pad_l;
  const int H = p.H, W = p.W, Cin = p.Cin;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), (short)0, (int)((size_t)p.B * H * W * p.xs * 4), 0x00020000);
  const int cin32 = (Cin + 31) >> 5;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.w3), (short)0, (int)((size_t)9 * cin32 * p.Cout_pad * 192), 0x00020000);
  constexpr int kOob = 0x7fffffff & ~15;

  int x_off[XI];
  const size_t img = (size_t)b * H * W;
#pragma unroll
  for (int j = 0; j < XI; ++j) {
    const int i = tid + NT * j;
    const int px = i >> 2, q = i & 3;
    const int hy = px / HC, hx = px - hy * HC;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool in = i < HPIX * 4 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    x_off[j] = in ? (int)(((img + (size_t)iy * W + ix) * p.xs + 4 * q) * 4) : kOob;
  }
  // this lane's weight rows (A operand: row = output channel fr of fragment tn, k = fk .. fk + 7 of a 16-deep step)
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  int w_off[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + (wn * TN + tn) * 32 + fr;
    w_off[tn] = n < p.Cout_pad ? (n * 96 + fk) * 2 : kOob;
  }

  f32x4 rx[XI];
  auto load_x_piece = [&](int cc, int piece) {  // items piece*XP .. +XP-1 of chunk cc's halo (16 channels)
#pragma unroll
    for (int jj = 0; jj < XP; ++jj) {
      const int j = piece * XP + jj;
      if (j < XI) {
        const int i = tid + NT * j;
        const int c = 16 * cc + 4 * (i & 3);
        const int o = (x_off[j] != kOob && c < Cin) ? x_off[j] + 64 * cc : kOob;
        rx[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o, 0, 0));
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int j = 0; j < XI; ++j) {
      const int i = tid + NT * j;
      if (HPIX * 4 % NT == 0 || i < HPIX * 4) {
        bf16x4 h, m, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = rx[j][e];
          const bf16 th = (bf16)v;
          const float r = v - (float)th;
          const bf16 tm = (bf16)r;
          h[e] = th;
          m[e] = tm;
          l[e] = (bf16)(r - (float)tm);
        }
        bf16* d = sX + (i >> 2) * HG_P + 4 * (i & 3);
        *(bf16x4*)d = h;
        *(bf16x4*)(d + 16) = m;
        *(bf16x4*)(d + 32) = l;
      }
    }
  };
  // stage st = (chunk cc, tap): this lane's three planes of every weight fragment; st == ns (past the end) reads
  // other weights or zeros, never used
  auto load_w = [&](int st, u32x4 (&w)[TN][3]) {
    const int cc = st / 9, tap = st - cc * 9;
    const int step = ((tap * cin32 + (cc >> 1)) * p.Cout_pad * 96 + 16 * (cc & 1)) * 2;  // uniform
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) w[tn][pl] = __builtin_amdgcn_raw_buffer_load_b128(wr, w_off[tn], step + 64 * pl, 0);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  int xpix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int r = (wm * TM + tm) * RF + fr / TW, c = fr % TW;
    xpix[tm] = r * HC + c;
  }
  auto compute = [&](const u32x4 (&w)[TN][3], int tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int toff = ky * HC + kx;
    bf16x8 xh[TM], xm[TM], xl[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const bf16* r = sX + (xpix[tm] + toff) * HG_P + fk;
      xh[tm] = *(const bf16x8*)r;
      xm[tm] = *(const bf16x8*)(r + 16);
      xl[tm] = *(const bf16x8*)(r + 32);
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const bf16x8 wh = __builtin_bit_cast(bf16x8, w[tn][0]), wmid = __builtin_bit_cast(bf16x8, w[tn][1]),
                   wl = __builtin_bit_cast(bf16x8, w[tn][2]);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) acc[tm][tn] = hg_mfma_x3(wh, wmid, wl, xh[tm], xm[tm], xl[tm], acc[tm][tn]);
    }
  };

  const int nc = (Cin + 15) >> 4;
  u32x4 wa[TN][3], wb[TN][3];
#pragma unroll
  for (int piece = 0; piece < 8; ++piece) load_x_piece(0, piece);
  load_w(0, wa);
  store_x();
  __syncthreads();
  // nine taps per chunk, unrolled, the two weight register sets alternating; the loop body is two chunks so the
  // set of each tap is fixed at compile time (9 is odd)
  auto chunk = [&](int cc, u32x4 (&w0)[TN][3], u32x4 (&w1)[TN][3]) {
    const bool more = cc + 1 < nc;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int st = cc * 9 + tap;
      if (tap % 2 == 0) load_w(st + 1, w1);
      else load_w(st + 1, w0);
      if (more && tap < 8) load_x_piece(cc + 1, tap);
      if (tap % 2 == 0) compute(w0, tap);
      else compute(w1, tap);
    }
    if (more) {  // every wave is done with this chunk's halo before it is replaced
      __syncthreads();
      store_x();
      __syncthreads();
    }
  };
  // even chunks run taps 0, 2, .. 8 from wa and leave the next chunk's tap 0 in wb; odd chunks the other way round
  // (one loop, two bodies: a separate odd-count remainder body miscompiled for one tile shape on ROCm 7.2)
  for (int cc = 0; cc < nc; ++cc) {
    if ((cc & 1) == 0) chunk(cc, wa, wb);
    else chunk(cc, wb, wa);
  }

  hg_epilogue<TW, WM, WN, TM, TN, PWN>(p, acc, b, oy0, ox0, n0, wm, wn, lane);
}

namespace {

template <int TW, int WM, int WN, int TM, int TN, int PWN = 0>
void hg_launch(const ConvParams& p, hipStream_t s) {
  constexpr int TH = hg_th(TW, WM, TM), BN = WN * TN * 32;
  const long tiles = (long)p.B * ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * ((p.Cout_pad + BN - 1) / BN);
  hipLaunchKernelGGL((conv_x3hg_kernel<TW, WM, WN, TM, TN, PWN>), dim3((unsigned)tiles), dim3(WM * WN * 64),
                     hg_lds_bytes(TW, WM, WN, TM, TN), s, p);
}

template <int TW, int WM, int WN, int TM, int TN, int PWN = 0>
void hr_launch(const ConvParams& p, hipStream_t s) {
  constexpr int TH = hg_th(TW, WM, TM), BN = WN * TN * 32;
  const long tiles = (long)p.B * ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * ((p.Cout_pad + BN - 1) / BN);
  hipLaunchKernelGGL((conv_x3hr_kernel<TW, WM, WN, TM, TN, PWN>), dim3((unsigned)tiles), dim3(WM * WN * 64),
                     hr_lds_bytes(TW, WM, TM), s, p);
}

// variant v: (TW, WM, WN, TM, TN) -> tile TH x TW pixels x BN channels
#define HG_VARIANTS(X) \
  X(0, 16, 4, 1, 2, 2)  /* 16 x 16 px x  64 ch */ \
  X(1, 16, 4, 1, 1, 2)  /*  8 x 16 px x  64 ch */ \
  X(2, 16, 2, 2, 2, 1)  /*  8 x 16 px x  64 ch, waves split the channels */ \
  X(3, 16, 4, 1, 2, 3)  /* 16 x 16 px x  96 ch */ \
  X(4, 16, 4, 1, 1, 3)  /*  8 x 16 px x  96 ch */ \
  X(5, 16, 4, 1, 2, 5)  /* 16 x 16 px x 160 ch */ \
  X(6, 16, 4, 1, 1, 5)  /*  8 x 16 px x 160 ch */ \
  X(7, 8, 2, 2, 1, 1)   /*  8 x  8 px x  64 ch */ \
  X(8, 8, 4, 1, 1, 2)   /* 16 x  8 px x  64 ch */ \
  X(9, 8, 4, 1, 1, 5)   /* 16 x  8 px x 160 ch */ \
  X(10, 8, 4, 1, 1, 3)  /* 16 x  8 px x  96 ch */ \
  X(11, 16, 8, 1, 1, 5) /* 16 x 16 px x 160 ch, 8 waves */ \
  X(12, 8, 2, 2, 1, 2)  /*  8 x  8 px x 128 ch */ \
  X(13, 8, 2, 1, 1, 5)  /*  8 x  8 px x 160 ch, 2 waves */

// fused-1x1 variants v (kF32X3HGPw + v): (TW, WM, TM, TN, PWN), WN = 1
#define HG_PW_VARIANTS(X) \
  X(0, 16, 4, 1, 2, 2)  /*  8 x 16 px, 64 -> 64 (box branch) */ \
  X(1, 16, 4, 2, 2, 2)  /* 16 x 16 px */ \
  X(2, 16, 4, 1, 3, 3)  /*  8 x 16 px, 80 -> 80 (cls branch) */ \
  X(3, 16, 4, 2, 3, 3)  /* 16 x 16 px */ \
  X(4, 8, 4, 1, 2, 2)   /* 16 x  8 px, 64 -> 64 */ \
  X(5, 8, 4, 1, 3, 3)   /* 16 x  8 px, 80 -> 80 */ \
  X(6, 8, 2, 1, 2, 2)   /*  8 x  8 px, 2 waves: small buckets (kF32X3HGPwSmall) */ \
  X(7, 8, 2, 1, 3, 3)   /*  8 x  8 px, 80 -> 80, 2 waves */

// x3hr variants v (kF32X3HR + v): (TW, WM, WN, TM, TN)
#define HR_VARIANTS(X) \
  X(0, 16, 4, 1, 2, 2)  /* 16 x 16 px x  64 ch */ \
  X(1, 16, 4, 1, 1, 2)  /*  8 x 16 px x  64 ch */ \
  X(2, 16, 4, 1, 2, 3)  /* 16 x 16 px x  96 ch */ \
  X(3, 16, 4, 1, 1, 3)  /*  8 x 16 px x  96 ch */ \
  X(4, 16, 4, 1, 1, 5)  /*  8 x 16 px x 160 ch (the 144-channel head pairs) */ \
  X(5, 16, 8, 1, 1, 5)  /* 16 x 16 px x 160 ch, 8 waves */ \
  X(6, 8, 4, 1, 1, 2)   /* 16 x  8 px x  64 ch */ \
  X(7, 8, 4, 1, 1, 5)   /* 16 x  8 px x 160 ch */ \
  X(8, 16, 2, 2, 2, 1)  /*  8 x 16 px x  64 ch, waves split the channels */ \
  X(9, 8, 4, 1, 1, 3)   /* 16 x  8 px x  96 ch */

// x3hr with the fused Detect-head 1x1 (kF32X3HRPw + v): (TW, WM, TM, TN, PWN), WN = 1
#define HR_PW_VARIANTS(X) \
  X(0, 16, 4, 1, 2, 2)  \
  X(1, 16, 4, 2, 2, 2)  \
  X(2, 16, 4, 1, 3, 3)  \
  X(3, 16, 4, 2, 3, 3)  \
  X(4, 8, 4, 1, 2, 2)   \
  X(5, 8, 4, 1, 3, 3)

}  // namespace

bool x3hg_supported(const ConvParams& p) {
  const size_t x_bytes = (size_t)p.B * p.H * p.W * p.xs * 4;
  const size_t w_bytes = (size_t)9 * ((p.Cin + 31) / 32) * p.Cout_pad * 192;
  return p.w3 != nullptr && p.KH == 3 && p.KW == 3 && p.stride == 1 && p.Cin % 4 == 0 && p.xs % 4 == 0 &&
         x_bytes < (1u << 31) - (1u << 20) && w_bytes < (1u << 31) - (1u << 20) && p.Cout % 4 == 0 &&
         p.ys % 4 == 0 && (p.res == nullptr || p.rs % 4 == 0) && (p.y2 == nullptr || p.y2s % 4 == 0) &&
         p.lb_meta == nullptr && p.pw_w == nullptr;
}

bool x3hg_pw_supported(const ConvParams& p, int bn, int pwn) {
  return p.w3 != nullptr && p.KH == 3 && p.KW == 3 && p.stride == 1 && p.Cin % 4 == 0 && p.xs % 4 == 0 &&
         (size_t)p.B * p.H * p.W * p.xs * 4 < (1u << 31) - (1u << 20) && p.Cout % 4 == 0 && p.Cout_pad <= bn &&
         p.res == nullptr && p.y2 == nullptr && p.lb_meta == nullptr && p.pw_w != nullptr && p.pw_y != nullptr &&
         p.pw_kpad == bn && p.pw_cout % 4 == 0 && p.pw_cout <= 32 * pwn && p.pw_ys % 4 == 0;
}

bool conv_x3hg_pw(const ConvParams& p, hipStream_t s, int v) {
  switch (v) {
#define HG_PW_CASE(V, TW, WM, TM, TN, PWN) \
  case V:                                 \
    if (!x3hg_pw_supported(p, TN * 32, PWN)) return false; \
    hg_launch<TW, WM, 1, TM, TN, PWN>(p, s);                \
    return true;
    HG_PW_VARIANTS(HG_PW_CASE)
#undef HG_PW_CASE
    default: return false;
  }
}

bool conv_x3hg(const ConvParams& p, hipStream_t s, int v) {
  if (!x3hg_supported(p)) return false;
  switch (v) {
#define HG_CASE(V, TW, WM, WN, TM, TN) \
  case V: hg_launch<TW, WM, WN, TM, TN>(p, s); return true;
    HG_VARIANTS(HG_CASE)
#undef HG_CASE
    default: return false;
  }
}

bool conv_x3hr(const ConvParams& p, hipStream_t s, int v) {
  if (!x3hg_supported(p)) return false;
  switch (v) {
#define HR_CASE(V, TW, WM, WN, TM, TN) \
  case V: hr_launch<TW, WM, WN, TM, TN>(p, s); return true;
    HR_VARIANTS(HR_CASE)
#undef HR_CASE
    default: return false;
  }
}

bool conv_x3hr_pw(const ConvParams& p, hipStream_t s, int v) {
  switch (v) {
#define HR_PW_CASE(V, TW, WM, TM, TN, PWN) \
  case V:                                 \
    if (!x3hg_pw_supported(p, TN * 32, PWN)) return false; \
    hr_launch<TW, WM, 1, TM, TN, PWN>(p, s);                \
    return true;
    HR_PW_VARIANTS(HR_PW_CASE)
#undef HR_PW_CASE
    default: return false;
  }
}

void x3hg_prepare() {
#define HG_ATTR(V, TW, WM, WN, TM, TN)                                                            \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3hg_kernel<TW, WM, WN, TM, TN>,           \
                                      hipFuncAttributeMaxDynamicSharedMemorySize,                  \
                                      hg_lds_bytes(TW, WM, WN, TM, TN)));
  HG_VARIANTS(HG_ATTR)
#undef HG_ATTR
#define HG_PW_ATTR(V, TW, WM, TM, TN, PWN)                                                         \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3hg_kernel<TW, WM, 1, TM, TN, PWN>,         \
                                      hipFuncAttributeMaxDynamicSharedMemorySize,                  \
                                      hg_lds_bytes(TW, WM, 1, TM, TN)));
  HG_PW_VARIANTS(HG_PW_ATTR)
#undef HG_PW_ATTR
#define HR_ATTR(V, TW, WM, WN, TM, TN)                                                            \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3hr_kernel<TW, WM, WN, TM, TN>,           \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, hr_lds_bytes(TW, WM, TM)));
  HR_VARIANTS(HR_ATTR)
#undef HR_ATTR
#define HR_PW_ATTR(V, TW, WM, TM, TN, PWN)                                                         \
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_x3hr_kernel<TW, WM, 1, TM, TN, PWN>,         \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, hr_lds_bytes(TW, WM, TM)));
  HR_PW_VARIANTS(HR_PW_ATTR)
#undef HR_PW_ATTR
}

}  // namespace arena
