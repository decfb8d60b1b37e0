// Whole YOLOv5 C3 block in one kernel for the high-resolution levels
// (160x160 with c_ = 16, 80x80 with c_ = 32):
//
//   T  = SiLU(W12 . x + b12)                 cv1 | cv2 (1x1, C1 -> 2c_)
//   repeat NB times (Bottleneck):
//     U  = SiLU(W1 . T[:, :c_] + b1)         1x1 c_ -> c_     (zero outside the image: the 3x3 pads U)
//     Tc = Tc * RES + SiLU(conv3x3(U) + b2)  3x3 c_ -> c_ (+ shortcut)
//   y  = SiLU(W3 . [Tc, T[:, c_:]] + b3)     cv3 (1x1, 2c_ -> 2c_)
//
// Unfused these are 2 + 2*NB launches whose intermediates (T, U) make full
// HBM round trips: at 160x160 with batch 32 each is a 26-52 MB tensor, so
// the block was ~330 MB of traffic for 52 MB in and 52 MB out.  Here one
// workgroup owns an 8x16 output tile and recomputes an NB-pixel halo ring of
// the 1x1 stages (1.4x / 1.9x the 1x1 MACs for NB = 1 / 2) instead; every
// intermediate lives in LDS.  All four stages are MFMA GEMMs over the tile's
// pixels (M) with weights as the A operand (v_mfma_f32_16x16x32_bf16); the
// 3x3 takes its B operand straight from the halo-padded U buffer.
//
// LDS rows are C*2 + 16 bytes: the 16-byte pad staggers consecutive pixels
// across banks, so the 16 lanes of a ds_read_b128 group hit distinct slots.
#include <type_traits>

#include "common.h"
#include "launch.h"

namespace arena {

namespace {

template <int C>
struct Row {
  static constexpr int BYTES = C * 2 + 16;
};

}  // namespace

template <int C1, int CH, int NB, bool RES>
__global__ __launch_bounds__(256) void c3_fused_kernel(const C3Params p) {
  constexpr int TH = 8, TW = 16;
  constexpr int PH = TH + 2 * NB, PW = TW + 2 * NB, NPIX = PH * PW;
  constexpr int C2 = 2 * CH;                      // T channels == output channels
  constexpr int RA = Row<C1>::BYTES, RT = Row<C2>::BYTES, RU = Row<CH>::BYTES;
  constexpr int A_BYTES = NPIX * RA, U_BYTES = NPIX * RU;
  constexpr int AU_BYTES = A_BYTES > U_BYTES ? A_BYTES : U_BYTES;  // U reuses the input tile's space
  constexpr int SL3 = (9 * CH + 31) / 32;          // 3x3 K slabs
  static_assert(C1 % 32 == 0 && (CH == 16 || CH == 32), "C3 geometry");
  __shared__ __align__(16) uint8_t au[AU_BYTES];
  __shared__ __align__(16) uint8_t tb[NPIX * RT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int tiles_x = p.W / TW, tiles = (p.H / TH) * tiles_x;
  const int b = blockIdx.x / tiles;
  if (b >= live_batch(p.B, p.bdev)) return;
  const int t = blockIdx.x - b * tiles;
  const int y0 = (t / tiles_x) * TH, x0 = (t % tiles_x) * TW;
  const bf16* __restrict__ x = (const bf16*)p.x + (size_t)b * p.H * p.W * p.xs;

  // ---- input tile with an NB-pixel halo (zeros outside the image)
  constexpr int CPR1 = C1 / 8;
  for (int i = tid; i < NPIX * CPR1; i += 256) {
    const int pix = i / CPR1, c = i - (i / CPR1) * CPR1;
    const int iy = y0 - NB + pix / PW, ix = x0 - NB + pix % PW;
    const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    *(uint4*)(au + pix * RA + c * 16) = load16_or_zero(x + ((size_t)iy * p.W + ix) * p.xs + c * 8, x, ok);
  }
  __syncthreads();

  // GEMM over the pixels of a sub-rectangle [off, off + rh) x [off, off + rw) of the halo tile:
  // out[pixel][n] = act(sum_k W[n][k] * in[pixel][k] + bias[n]); `emit` stores one lane's 4 channels.
  // (Loading each weight fragment once per wave for all its pixel fragments measured slower: the extra
  // accumulators cost occupancy, and the per-fragment weight reads hit L1.)
  auto region_gemm = [&](int off, int rh, int rw, const uint8_t* in, int rin, int kslabs, const bf16* w, int kpad,
                         const float* bias, auto nfr_tag, auto emit) {
    constexpr int NF = decltype(nfr_tag)::value;
    const int npx = rh * rw, nfrag = (npx + 15) / 16;
    for (int f = wave; f < nfrag; f += 4) {
      const int q = f * 16 + row;  // this lane's pixel (B operand row)
      const int qq = q < npx ? q : npx - 1;
      const int pix = (off + qq / rw) * PW + off + qq % rw;
      f32x4 acc[NF];
#pragma unroll
      for (int n = 0; n < NF; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < kslabs; ++s) {
        const bf16x8 bv = *(const bf16x8*)(in + pix * rin + (s * 32 + kq * 8) * 2);
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          const bf16x8 av = *(const bf16x8*)(w + (size_t)(n * 16 + row) * kpad + s * 32 + kq * 8);
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[n], 0, 0, 0);
        }
      }
      // D layout: lane holds channels n*16 + kq*4 .. +3 of pixel f*16 + row
      const int po = f * 16 + row;
      if (po < npx) {
        const int opix = (off + po / rw) * PW + off + po % rw;
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          const int cb = n * 16 + kq * 4;
          const float4 bb = *(const float4*)(bias + cb);
          float v[4] = {silu(acc[n][0] + bb.x), silu(acc[n][1] + bb.y), silu(acc[n][2] + bb.z), silu(acc[n][3] + bb.w)};
          emit(opix, po, cb, v);
        }
      }
    }
  };
  using NF_T = std::integral_constant<int, C2 / 16>;
  using NF_U = std::integral_constant<int, CH / 16>;

  // ---- T = SiLU(W12 . x + b12) on the whole halo tile
  region_gemm(0, PH, PW, au, RA, C1 / 32, (const bf16*)p.w12, C1, p.b12, NF_T{},
              [&](int opix, int, int cb, float* v) { *(uint2*)(tb + opix * RT + cb * 2) = pack4(v); });
  __syncthreads();

#pragma unroll
  for (int k = 0; k < NB; ++k) {
    // ---- U = SiLU(W1 . T[:, :c_] + b1) on the ring-(NB-k) region; zero outside the image.
    // K is one 32-channel slab of T (for c_ = 16 the weights' k >= 16 columns are zero).
    const int uo = k, uh = PH - 2 * k, uw = PW - 2 * k;
    region_gemm(uo, uh, uw, tb, RT, 1, (const bf16*)p.wb1[k], 32, p.bb1[k], NF_U{},
                [&](int opix, int, int cb, float* v) {
                  const int iy = y0 - NB + opix / PW, ix = x0 - NB + opix % PW;
                  if (!((unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)) v[0] = v[1] = v[2] = v[3] = 0.f;
                  *(uint2*)(au + opix * RU + cb * 2) = pack4(v);
                });
    __syncthreads();
    // ---- Tc = [Tc +] SiLU(conv3x3(U) + b2) on the ring-(NB-k-1) region (in place: a lane reads and
    // writes only its own pixel of T, and every lane reads U, which is not written in this phase)
    {
      const int oo = k + 1, oh = PH - 2 * (k + 1), ow = PW - 2 * (k + 1);
      const int npx = oh * ow, nfrag = (npx + 15) / 16;
      const bf16* w2 = (const bf16*)p.wb2[k];
      constexpr int NF = CH / 16;
      for (int f = wave; f < nfrag; f += 4) {
        const int q = f * 16 + row;
        const int qq = q < npx ? q : npx - 1;
        const int cy = oo + qq / ow, cx = oo + qq % ow;  // centre pixel (halo-tile coordinates)
        f32x4 acc[NF];
#pragma unroll
        for (int n = 0; n < NF; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SL3; ++s) {
          const int k0 = s * 32 + kq * 8;
          int tap = k0 / CH;
          if (tap >= 9) tap = 0;  // zero weight columns of the padded last slab
          const int ci = k0 - (k0 / CH) * CH;
          const int pix = (cy + tap / 3 - 1) * PW + cx + tap % 3 - 1;
          const bf16x8 bv = *(const bf16x8*)(au + pix * RU + ci * 2);
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            const bf16x8 av = *(const bf16x8*)(w2 + (size_t)(n * 16 + row) * (SL3 * 32) + k0);
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[n], 0, 0, 0);
          }
        }
        const int po = f * 16 + row;
        if (po < npx) {
          const int opix = (oo + po / ow) * PW + oo + po % ow;
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            const int cb = n * 16 + kq * 4;
            const float4 bb = *(const float4*)(p.bb2[k] + cb);
            float v[4] = {silu(acc[n][0] + bb.x), silu(acc[n][1] + bb.y), silu(acc[n][2] + bb.z),
                          silu(acc[n][3] + bb.w)};
            uint2* dst = (uint2*)(tb + opix * RT + cb * 2);
            if constexpr (RES) {
              float r[4];
              unpack4(*dst, r);
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] += r[j];
            }
            *dst = pack4(v);
          }
        }
      }
    }
    __syncthreads();
  }

  // ---- y = SiLU(W3 . [Tc, T2] + b3) on the output tile
  bf16* __restrict__ y = (bf16*)p.y + (size_t)b * p.H * p.W * p.ys;
  region_gemm(NB, TH, TW, tb, RT, C2 / 32, (const bf16*)p.w3, C2, p.b3, NF_T{},
              [&](int, int po, int cb, float* v) {
                const int oy = y0 + po / TW, ox = x0 + po % TW;
                *(uint2*)(y + ((size_t)oy * p.W + ox) * p.ys + cb) = pack4(v);
              });
}

template <int C1, int CH, int NB, bool RES>
static void c3_launch(const C3Params& p, hipStream_t s) {
  const long grid = (long)p.B * (p.H / 8) * (p.W / 16);
  if (grid <= 0) return;
  hipLaunchKernelGGL((c3_fused_kernel<C1, CH, NB, RES>), dim3((unsigned)grid), dim3(256), 0, s, p);
}

bool c3_fused_supported(int C1, int CH, int NB, bool res, int H, int W) {
  if (H % 8 != 0 || W % 16 != 0) return false;
  return (C1 == 32 && CH == 16 && NB == 1 && res) || (C1 == 64 && CH == 32 && NB == 2 && res) ||
         (C1 == 128 && CH == 32 && NB == 1 && !res);
}

void c3_fused(const C3Params& p, hipStream_t s) {
  if (!c3_fused_supported(p.C1, p.CH, p.NB, p.res != 0, p.H, p.W))
    throw std::runtime_error("c3_fused: unsupported geometry");
  if (p.xs % 8 != 0 || p.ys % 4 != 0) throw std::runtime_error("c3_fused: pixel strides must be 8 / 4 aligned");
  if (p.C1 == 32) c3_launch<32, 16, 1, true>(p, s);
  else if (p.C1 == 64) c3_launch<64, 32, 2, true>(p, s);
  else c3_launch<128, 32, 1, false>(p, s);
}

}  // namespace arena
