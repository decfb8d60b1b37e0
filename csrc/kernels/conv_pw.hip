// Pointwise (1x1, stride 1) convolution for gfx950: a memory-bound GEMM
// y[M, N] = act(x[M, K] . W[N, K]^T + b) (+ res), M = batch * H * W pixels.
//
// Counters on the generic kernels showed the 1x1 layers spending their time
// in VALU (per-element index math + epilogue) and in scattered 8-byte stores,
// reaching ~1.2 TB/s.  This kernel is shaped for the HBM stream instead:
//  * every K-step of a wave's pixel fragments is loaded up front (MF x KS
//    independent 16-B loads in flight per lane), with no im2col index math —
//    input pixel = output pixel;
//  * the block's weight slice ([NT*16][KS*32], <= 64 KB) is staged in LDS once
//    (XOR-swizzled 64-B rows, as in conv_igemm.hip) while those loads fly;
//  * the epilogue packs bf16 into a per-wave LDS tile and writes whole pixel
//    rows with 16-B stores (full cache lines instead of 32-B row fragments),
//    including the optional 2x nearest-upsampled copy.
#include "common.h"
#include "launch.h"

namespace arena {

__device__ __forceinline__ int pswz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) * 2)) & 3)) << 4);
}

template <int NT, int KS, int MF>
__global__ __launch_bounds__(256) void conv_pw_kernel(const ConvParams p) {
  constexpr int BNR = NT * 16;                 // weight rows (output channels) of this block
  constexpr int WBYTES = KS * BNR * 64;        // [KS][BNR] 64-B rows
  constexpr int OROW = BNR * 2 + 16;           // output staging row (padded)
  constexpr int OTILE = MF * 16 * OROW;        // per wave
  extern __shared__ __align__(16) uint8_t lds[];
  uint8_t* wl = lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kq = lane >> 4;
  uint8_t* ol = lds + WBYTES + wave * OTILE;

  const int B = live_batch(p.B, p.bdev);
  const int HW = p.Ho * p.Wo;
  const int M = B * HW;
  int bx = blockIdx.x;
  {  // XCD-aware bijective remap
    const int nx = gridDim.x, q = nx / 8, r = nx % 8, x = bx % 8, y = bx / 8;
    bx = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + y;
  }
  const int m0 = bx * (64 * MF);
  if (m0 >= M) return;
  const int n0 = blockIdx.y * BNR;
  const int wpix = m0 + wave * 16 * MF;
  const bf16* __restrict__ x = (const bf16*)p.x;

  // 1. activation fragments for every K-step (independent loads, all in flight)
  uint4 bv[MF][KS];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int pix = wpix + f * 16 + row;
    const bool pv = pix < M;
    const bf16* xp = x + (size_t)(pv ? pix : 0) * p.xs + kq * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + kq * 8;
      bv[f][ks] = load16_or_zero(xp + ks * 32, x, pv && k < p.Cin);
    }
  }
  // 2. weight slice -> LDS
  const bf16* __restrict__ w = (const bf16*)p.w;
  for (int i = tid; i < KS * BNR * 4; i += 256) {
    const int r = i / (KS * 4), rem = i - r * (KS * 4);
    const int ks = rem >> 2, c = rem & 3;
    const uint4 v = load16_or_zero(w + (size_t)(n0 + r) * p.Kpad + ks * 32 + c * 8, w, n0 + r < p.Cout_pad);
    *(uint4*)(wl + ks * BNR * 64 + pswz(r, c)) = v;
  }
  __syncthreads();

  // 3. MFMA
  f32x4 acc[NT][MF];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int f = 0; f < MF; ++f) acc[t][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 a = *(const bf16x8*)(wl + ks * BNR * 64 + pswz(t * 16 + row, kq));
#pragma unroll
      for (int f = 0; f < MF; ++f)
        acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bv[f][ks]), acc[t][f],
                                                            0, 0, 0);
    }
  }

  // 4. epilogue into the wave's LDS tile: [pixel][channel] bf16
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int cl = t * 16 + kq * 4;  // channel within the block slice
    const int cb = n0 + cl;
    if (cb >= p.Cout) continue;
    const float4 bias = *(const float4*)(p.bias + cb);
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int pl = f * 16 + row;
      const int pix = wpix + pl;
      float v[4] = {acc[t][f][0] + bias.x, acc[t][f][1] + bias.y, acc[t][f][2] + bias.z, acc[t][f][3] + bias.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act);
      if (p.res != nullptr && pix < M) {
        float rv[4];
        unpack4(*(const uint2*)((const bf16*)p.res + (size_t)pix * p.rs + cb), rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += rv[r];
      }
      *(uint2*)(ol + pl * OROW + cl * 2) = pack4(v);
    }
  }
  // wave-local tile: no block barrier needed, only the wave's own LDS writes
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();

  // 5. whole-row 16-B stores (+ 2x upsampled copy)
  const int cn = min(BNR, p.Cout - n0);
  const int cpr = cn >> 3;
  bf16* y = (bf16*)p.y;
  for (int i = lane; i < MF * 16 * cpr; i += 64) {
    const int pl = i / cpr, c = i - pl * cpr;
    const int pix = wpix + pl;
    if (pix >= M) continue;
    const uint4 v = *(const uint4*)(ol + pl * OROW + c * 16);
    *(uint4*)(y + (size_t)pix * p.ys + n0 + c * 8) = v;
    if (p.y2 != nullptr) {
      const int b = pix / HW, rr = pix - b * HW;
      const int oy = rr / p.Wo, ox = rr - oy * p.Wo;
      const int W2 = 2 * p.Wo;
      bf16* y2 = (bf16*)p.y2 + n0 + c * 8;
      const size_t base = (size_t)(b * 2 * p.Ho + 2 * oy) * W2 + 2 * ox;
      *(uint4*)(y2 + base * p.y2s) = v;
      *(uint4*)(y2 + (base + 1) * p.y2s) = v;
      *(uint4*)(y2 + (base + W2) * p.y2s) = v;
      *(uint4*)(y2 + (base + W2 + 1) * p.y2s) = v;
    }
  }
}

template <int NT, int KS, int MF>
static void pw_launch(const ConvParams& p, hipStream_t s, long M, int nsplit) {
  constexpr size_t lds = (size_t)KS * NT * 16 * 64 + 4 * (size_t)MF * 16 * (NT * 16 * 2 + 16);
  static_assert(lds <= 160 * 1024, "LDS");
  static bool attr = [] {
    ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)conv_pw_kernel<NT, KS, MF>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    return true;
  }();
  (void)attr;
  dim3 grid((unsigned)((M + 64 * MF - 1) / (64 * MF)), (unsigned)nsplit);
  hipLaunchKernelGGL((conv_pw_kernel<NT, KS, MF>), grid, dim3(256), lds, s, p);
}

// Returns false when the layer is not a supported pointwise shape.
bool conv_pw(const ConvParams& p, hipStream_t s) {
  if (p.KH != 1 || p.KW != 1 || p.stride != 1 || p.pad_t != 0 || p.pad_l != 0 || p.f32out || p.Cout % 8 != 0 ||
      p.Ho != p.H || p.Wo != p.W)
    return false;
  const long M = (long)p.B * p.Ho * p.Wo;
  const int NT = p.Cout_pad / 16, KS = p.Kpad / 32;
#define PW(nt, ks, mf, split)                                                    \
  if (NT == nt * split && KS == ks && (M + 64 * mf - 1) / (64 * mf) >= 512) {    \
    pw_launch<nt, ks, mf>(p, s, M, split);                                       \
    return true;                                                                 \
  }
  // Measured on MI355X (profiles/r1_pw_ops.md): wins for large pixel counts with
  // <= 32 KB weight slices; small maps (20x20, 14x14 crops) and wide/deep weight
  // slices stay on the generic kernels, which amortise weights better.
  PW(1, 1, 4, 1)
  PW(2, 1, 4, 1)
  PW(4, 2, 2, 1)
  PW(4, 4, 2, 1)
  PW(5, 3, 2, 1)
  PW(8, 4, 2, 1)
#undef PW
  return false;
}

}  // namespace arena
