// LDS-pipelined implicit-GEMM convolution (impl 3) for gfx950.
//
// Block tile BM output pixels x BN output channels, 256 threads = 4 waves in a
// WM x WN grid, each wave owning (BM/WM) x (BN/WN) of the tile as
// 16x16x32 bf16 MFMA fragments.  K = (kh, kw, ci) is consumed in stages of BK
// (32 or 64): the im2col rows (NHWC, 16-byte pieces of 8 channels of one tap)
// and the weight rows of stage k+1 are loaded into registers while stage k is
// multiplied out of LDS, then written to the other LDS buffer — one barrier
// per stage.  LDS images are 64-byte rows (32 k) with the 16-byte chunks
// XOR-swizzled by g[(row>>2)&3] (g = {0,2,3,1}) so every ds_read_b128 lane
// group of the fragment read hits 16 distinct bank slots.
//
// Epilogue (same contract as conv_mfma.hip): bias -> activation -> residual ->
// bf16 (or fp32) NHWC store into a channel slice, optional 2x nearest
// upsampled second store.
#include "common.h"
#include "launch.h"

namespace arena {

__device__ __forceinline__ int gswz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}

template <int BM, int BN, int WM, int WN, int BK, bool F32OUT>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const ConvParams p) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int CPR = BK / 8;                       // 16-B chunks per row and stage
  constexpr int BPT = BM * CPR / 256;               // B chunks per thread
  constexpr int APT = (BN * CPR + 255) / 256;       // A chunks per thread
  constexpr int SL = BK / 32;                       // 32-deep slabs per stage
  static_assert(BM * CPR % 256 == 0, "B tile must split evenly");
  __shared__ __align__(16) uint8_t lds[2][SL][(BM + BN) * 64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int wm = wave % WM, wn = wave / WM;

  const int B = live_batch(p.B, p.bdev);
  const int HWo = p.Ho * p.Wo;
  const int M = B * HWo;
  int bx = blockIdx.x;
  {  // XCD-aware bijective remap: neighbouring pixel tiles (shared halo rows) on one L2
    const int nx = gridDim.x, q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
    bx = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int m0 = bx * BM;
  if (m0 >= M) return;
  const int n0 = blockIdx.y * BN;

  const bf16* __restrict__ x = (const bf16*)p.x;
  const bf16* __restrict__ w = (const bf16*)p.w;
  const int Cin = p.Cin, KW = p.KW, taps = p.KH * p.KW;

  // ---- per-thread load assignment (fixed chunk column, BPT rows)
  const int bc = tid % CPR;
  int brow[BPT], biy[BPT], bix[BPT];
  const bf16* bptr[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int r = tid / CPR + j * (256 / CPR);
    brow[j] = r;
    const int m = m0 + r;
    if (m < M) {
      const int b = m / HWo, rem = m - b * HWo;
      const int oy = rem / p.Wo, ox = rem - oy * p.Wo;
      biy[j] = oy * p.stride - p.pad_t;
      bix[j] = ox * p.stride - p.pad_l;
      bptr[j] = x + (size_t)b * p.H * p.W * p.xs;
    } else {
      biy[j] = -(1 << 20);  // never in bounds
      bix[j] = 0;
      bptr[j] = x;
    }
  }
  // (tap, ci) of this thread's chunk at the current stage
  int ci = (bc * 8) % Cin, tap = (bc * 8) / Cin;
  int kh = tap / KW, kw = tap - (tap / KW) * KW;

  uint4 rb[BPT], ra[APT];
  const uint4 zero = {0u, 0u, 0u, 0u};
  auto load_stage = [&](int ks) {
    const bool tv = tap < taps;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int iy = biy[j] + kh, ix = bix[j] + kw;
      const bool ok = tv && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      rb[j] = load16_or_zero(bptr[j] + ((size_t)iy * p.W + ix) * p.xs + ci, x, ok);
    }
#pragma unroll
    for (int j = 0; j < APT; ++j) {
      const int i = tid + j * 256;
      const int n = i / CPR, c = i - n * CPR;
      const int k = ks * BK + c * 8;
      ra[j] = load16_or_zero(w + (size_t)(n0 + n) * p.Kpad + k, w, i < BN * CPR && n0 + n < p.Cout_pad && k < p.Kpad);
    }
    // advance this thread's (tap, ci) by BK
    ci += BK;
    while (ci >= Cin) {
      ci -= Cin;
      ++tap;
      if (++kw == KW) { kw = 0; ++kh; }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int j = 0; j < BPT; ++j)
      *(uint4*)(&lds[buf][bc >> 2][0] + gswz(brow[j], bc & 3)) = rb[j];
#pragma unroll
    for (int j = 0; j < APT; ++j) {
      const int i = tid + j * 256;
      if (i < BN * CPR) {
        const int n = i / CPR, c = i - n * CPR;
        *(uint4*)(&lds[buf][c >> 2][0] + BM * 64 + gswz(n, c & 3)) = ra[j];
      }
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int a = 0; a < FN; ++a)
#pragma unroll
    for (int b = 0; b < FM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = (p.Kpad + BK - 1) / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nks;
    if (more) load_stage(ks + 1);
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      const uint8_t* base = &lds[cur][sl][0];
      bf16x8 bv[FM], av[FN];
#pragma unroll
      for (int f = 0; f < FM; ++f) bv[f] = *(const bf16x8*)(base + gswz(wm * TM + f * 16 + row, kq));
#pragma unroll
      for (int f = 0; f < FN; ++f) av[f] = *(const bf16x8*)(base + BM * 64 + gswz(wn * TN + f * 16 + row, kq));
#pragma unroll
      for (int a = 0; a < FN; ++a)
#pragma unroll
        for (int b = 0; b < FM; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue
#pragma unroll
  for (int a = 0; a < FN; ++a) {
    const int cb = n0 + wn * TN + a * 16 + kq * 4;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int b = 0; b < FM; ++b) {
      const int pix = m0 + wm * TM + b * 16 + row;
      if (pix >= M) continue;
      float v[4] = {acc[a][b][0] + bias.x, acc[a][b][1] + bias.y, acc[a][b][2] + bias.z, acc[a][b][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr) {
        float rv[4];
        unpack4(*(const uint2*)((const bf16*)p.res + (size_t)pix * p.rs + cb), rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      if constexpr (F32OUT) {
        *(float4*)((float*)p.y + (size_t)pix * p.ys + cb) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        const uint2 pk = pack4(v);
        *(uint2*)((bf16*)p.y + (size_t)pix * p.ys + cb) = pk;
        if (p.y2 != nullptr) {
          const int bb = pix / HWo;
          const int r = pix - bb * HWo;
          const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
          const int W2 = 2 * p.Wo;
          bf16* y2 = (bf16*)p.y2;
          const size_t base = ((size_t)(bb * 2 * p.Ho + 2 * oy) * W2 + 2 * ox);
          *(uint2*)(y2 + base * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + 1) * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + W2) * p.y2s + cb) = pk;
          *(uint2*)(y2 + (base + W2 + 1) * p.y2s + cb) = pk;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int BK>
static void igemm_launch(const ConvParams& p, hipStream_t s, long M) {
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((p.Cout_pad + BN - 1) / BN));
  if (p.f32out)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, BK, true>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, BK, false>), grid, dim3(256), 0, s, p);
}

// Tile choice by output-channel count (BN covers Cout_pad where possible) and
// GEMM size (smaller BM when the pixel count would leave CUs idle).
void conv_igemm(const ConvParams& p, hipStream_t s) {
  const long M = (long)p.B * p.Ho * p.Wo;
  const int N = p.Cout_pad;
  const bool deep = p.Kpad >= 64;
  auto enough = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn) >= 512; };
  if (N <= 16) {
    if (deep) igemm_launch<256, 16, 4, 1, 64>(p, s, M);
    else igemm_launch<256, 16, 4, 1, 32>(p, s, M);
  } else if (N <= 32) {
    if (enough(256, 32)) igemm_launch<256, 32, 4, 1, 64>(p, s, M);
    else igemm_launch<128, 32, 4, 1, 64>(p, s, M);
  } else if (N <= 64) {
    if (enough(128, 64)) igemm_launch<128, 64, 2, 2, 64>(p, s, M);
    else igemm_launch<64, 64, 4, 1, 64>(p, s, M);
  } else if (N == 80) {  // Detect class branch (nc = 80): exact 5-fragment width, no padded MFMA column
    if (enough(128, 80)) igemm_launch<128, 80, 4, 1, 64>(p, s, M);
    else igemm_launch<64, 80, 4, 1, 64>(p, s, M);
  } else if (N <= 96) {
    if (enough(128, 96)) igemm_launch<128, 96, 4, 1, 64>(p, s, M);
    else igemm_launch<64, 96, 4, 1, 64>(p, s, M);
  } else if (N == 144) {
    igemm_launch<64, 144, 4, 1, 64>(p, s, M);
  } else {
    if (enough(128, 128)) igemm_launch<128, 128, 2, 2, 64>(p, s, M);
    else igemm_launch<64, 128, 2, 2, 64>(p, s, M);
  }
}

}  // namespace arena
