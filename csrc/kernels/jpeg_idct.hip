// Device half of the split JPEG decoder (host half: csrc/runtime/jpeg_decode.h).
//
// A batch of entropy-decoded images (quantized int16 coefficient blocks + one JpegDesc each) becomes packed
// HxWx3 RGB in the staging slot's image pool, where the fused letterbox/stem kernel and the crop gather read
// it — exactly the bytes the host path used to upload after a PIL decode.  Two launches per batch:
//
//   jpeg_idct_kernel    one 8x8 block per 8 lanes: dequantize (row loads of 16 B), islow pass 1 over the
//                       columns and pass 2 over the rows through an LDS transpose, 8 samples (one 8-byte store)
//                       per lane into the component's sample plane.  grid (blocks / 32, images).
//   jpeg_color_kernel   4 horizontally adjacent output pixels per lane: one dword of luma, each chroma sample
//                       loaded once per lane, fancy upsampling (h2v2 / h2v1 / none) + YCbCr->RGB, three 4-byte
//                       stores.  grid (pixels / 1024, images), grid-stride over rows x quads.
//
// The arithmetic is kernels/jpeg_math.h, the same functions the host reference (jpeg_coefs_to_rgb) uses, so
// the result is bit-identical to it and to PIL / libjpeg-turbo (tests/test_jpeg_native_gpu.py).  The work is
// a few MB of traffic per batch of 32 frames: latency, not throughput, is what the layout optimises (every
// lane of a wave does useful work; no divergent per-component loops).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "jpeg_desc.h"
#include "jpeg_math.h"
#include "launch.h"

namespace arena {

namespace {

constexpr int kBlocksPerGroup = 32;  // 8x8 blocks per 256-lane workgroup

// natural index -> zigzag index (the compact payload stores each block's coded coefficients in zigzag order),
// packed for the lanes of a block: byte l of kZigzagCol[k] is the zigzag index of natural (row l, column k).  The
// row is a lane's, so an indexed table would be one divergent memory load per coefficient; as 64-bit literals
// the lookup is a shift of an immediate.
constexpr uint64_t kZigzagCol[8] = {0x2315140a09030200ull, 0x242216130b080401ull, 0x30252117120c0705ull,
                                    0x312f262018110d06ull, 0x39322e271f19100eull, 0x3a38332d281e1a0full,
                                    0x3e3b37342c291d1bull, 0x3f3d3c36352b2a1cull};

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegDesc* __restrict__ descs, uint8_t* __restrict__ pool) {
  __shared__ int32_t ws[kBlocksPerGroup][8][9];  // +1 column: pass-1 column reads hit distinct banks
  const JpegDesc& d = descs[blockIdx.y];
  const int g = threadIdx.x >> 3, l = threadIdx.x & 7;
  const int blk = (int)blockIdx.x * kBlocksPerGroup + g;
  const bool live = blk < d.total_blocks;
  // component of this block: at most 3 ranges
  int c = 0, b = blk;
  const int n0 = d.comp[0].bw * d.comp[0].bh;
  if (d.ncomp > 1 && b >= n0) {
    c = 1;
    b -= n0;
    const int n1 = d.comp[1].bw * d.comp[1].bh;
    if (b >= n1) {
      c = 2;
      b -= n1;
    }
  }
  const JpegCompDesc& cd = d.comp[c];
  // row l of the block: 8 int16 coefficients (16 B) and the matching 8 quantizer steps
  int32_t row[8];
  if (live && d.compact) {
    // compact payload (runtime/jpeg_decode.h jpeg_decode_compact): the block's zigzag mask and first value; the
    // coefficient at natural (l, k) is value popcount(mask below its zigzag bit) when its bit is set
    const uint64_t mask = reinterpret_cast<const uint64_t*>(pool + d.cmask_off)[blk];
    const int32_t v0 = (int32_t)reinterpret_cast<const uint32_t*>(pool + d.cvoff_off)[blk];
    const int16_t* vals = reinterpret_cast<const int16_t*>(pool + d.cval_off);
    const uint4 qv = *reinterpret_cast<const uint4*>(&d.qt[c][l * 8]);
    const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int z = (int)((kZigzagCol[k] >> (8 * l)) & 0xFF);
      const int idx = v0 + __popcll(mask & ((1ull << z) - 1ull));
      int32_t cf = 0;
      if ((mask >> z) & 1ull) cf = (int32_t)vals[idx];  // zero coefficients issue no load
      const int32_t q = (int32_t)((k & 1) ? (qw[k >> 1] >> 16) : (qw[k >> 1] & 0xFFFF));
      row[k] = cf * q;
    }
  } else if (live) {
    const uint4 cv = *reinterpret_cast<const uint4*>(pool + cd.coef_off + (int64_t)b * 128 + l * 16);
    const uint4 qv = *reinterpret_cast<const uint4*>(&d.qt[c][l * 8]);
    const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w}, qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      row[2 * k] = (int32_t)(int16_t)(cw[k] & 0xFFFF) * (int32_t)(qw[k] & 0xFFFF);
      row[2 * k + 1] = (int32_t)(int16_t)(cw[k] >> 16) * (int32_t)(qw[k] >> 16);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) row[k] = 0;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) ws[g][l][k] = row[k];
  __syncthreads();
  // pass 1: column l
  int32_t v[8], o[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = ws[g][r][l];
  jpegm::idct8<int32_t>(v, o, jpegm::kPass1Shift);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) ws[g][r][l] = o[r];
  __syncthreads();
  // pass 2: row l -> 8 samples
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = ws[g][l][k];
  jpegm::idct8<int32_t>(v, o, jpegm::kPass2Shift);
  if (!live) return;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    lo |= (uint32_t)jpegm::idct_sample<int32_t>(o[k]) << (8 * k);
    hi |= (uint32_t)jpegm::idct_sample<int32_t>(o[k + 4]) << (8 * k);
  }
  const int by = b / cd.bw, bx = b - by * cd.bw;
  const int64_t stride = (int64_t)cd.bw * 8;
  uint2* dst = reinterpret_cast<uint2*>(pool + cd.plane_off + (int64_t)(by * 8 + l) * stride + bx * 8);
  *dst = make_uint2(lo, hi);
}

// One lane = 4 horizontally adjacent output pixels x0 .. x0 + 3 (x0 = 4q) of one row.  Their luma is one aligned
// dword of the Y plane (row stride bw * 8, x0 % 4 == 0, planes 8-byte aligned: the IDCT's uint2 stores); with
// 2x horizontal chroma subsampling the four pixels need chroma columns cx0 - 1 .. cx0 + 2 (cx0 = 2q) of each
// chroma row they read, so every chroma sample is loaded once per lane instead of once per pixel and tap.  The
// per-pixel formulas (clamped neighbours, fancy upsampling, fixed-point YCbCr) are exactly chroma_at's of the
// host reference (jpeg_math.h), so the output stays bit-identical.  Rows of a width that is a multiple of 4 store
// 12-byte aligned dword triples; other widths store bytes.
struct ChromaRow {
  int v[4];  // columns max(cx0 - 1, 0), cx0, min(cx0 + 1, cw - 1), min(cx0 + 2, cw - 1)
};

__device__ __forceinline__ ChromaRow chroma_row(const uint8_t* __restrict__ row, int cx0, int cw) {
  ChromaRow r;
  r.v[0] = row[max(cx0 - 1, 0)];
  r.v[1] = row[cx0];
  r.v[2] = row[min(cx0 + 1, cw - 1)];
  r.v[3] = row[min(cx0 + 2, cw - 1)];
  return r;
}

// (cx, nx) of pixel i of the quad as indices into ChromaRow: i = 0 (cx0, cx0 - 1), 1 (cx0, cx0 + 1),
// 2 (cx0 + 1, cx0), 3 (cx0 + 1, cx0 + 2)
__device__ __forceinline__ int quad_c(int i) { return i < 2 ? 1 : 2; }
__device__ __forceinline__ int quad_n(int i) { return i == 0 ? 0 : i == 1 ? 2 : i == 2 ? 1 : 3; }

__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegDesc* __restrict__ descs, uint8_t* __restrict__ pool) {
  const JpegDesc& d = descs[blockIdx.y];
  const int W = d.width, H = d.height, layout = d.layout;
  const int qpr = (W + 3) >> 2;  // quads per row
  const int total = qpr * H;
  const uint8_t* yp = pool + d.comp[0].plane_off;
  const int ys = d.comp[0].bw * 8;
  uint8_t* out_img = pool + d.rgb_off;
  for (int t = (int)blockIdx.x * 256 + (int)threadIdx.x; t < total; t += (int)gridDim.x * 256) {
    const int y = t / qpr, q = t - y * qpr;
    const int x0 = 4 * q;
    const int n = min(4, W - x0);
    const uint32_t yw = *reinterpret_cast<const uint32_t*>(yp + (int64_t)y * ys + x0);
    uint8_t px[12];
    if (layout == JPEG_GRAY) {
#pragma unroll
      for (int i = 0; i < 4; ++i) px[3 * i] = px[3 * i + 1] = px[3 * i + 2] = (uint8_t)(yw >> (8 * i));
    } else {
      int cb[4], cr[4];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const JpegCompDesc& C = d.comp[1 + k];
        const uint8_t* cp = pool + C.plane_off;
        const int cs = C.bw * 8;
        int* dst = k == 0 ? cb : cr;
        if (layout == JPEG_444) {
          const uint32_t w = *reinterpret_cast<const uint32_t*>(cp + (int64_t)y * cs + x0);
#pragma unroll
          for (int i = 0; i < 4; ++i) dst[i] = (int)((w >> (8 * i)) & 0xFF);
        } else if (layout == JPEG_422) {
          const ChromaRow r = chroma_row(cp + (int64_t)y * cs, 2 * q, C.cw);
#pragma unroll
          for (int i = 0; i < 4; ++i) dst[i] = jpegm::fancy_h2v1(r.v[quad_c(i)], r.v[quad_n(i)], i & 1);
        } else {
          const int cy = y >> 1;
          const int ny = (y & 1) ? min(cy + 1, C.ch - 1) : max(cy - 1, 0);
          const ChromaRow a = chroma_row(cp + (int64_t)cy * cs, 2 * q, C.cw);
          const ChromaRow b = chroma_row(cp + (int64_t)ny * cs, 2 * q, C.cw);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            dst[i] = jpegm::fancy_h2v2(a.v[quad_c(i)], a.v[quad_n(i)], b.v[quad_c(i)], b.v[quad_n(i)], i & 1);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) jpegm::ycc_to_rgb((int)((yw >> (8 * i)) & 0xFF), cb[i], cr[i], px + 3 * i);
    }
    uint8_t* out = out_img + ((int64_t)y * W + x0) * 3;
    if (n == 4 && (W & 3) == 0) {
      uint32_t w[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        w[k] = (uint32_t)px[4 * k] | ((uint32_t)px[4 * k + 1] << 8) | ((uint32_t)px[4 * k + 2] << 16) |
               ((uint32_t)px[4 * k + 3] << 24);
      uint32_t* o32 = reinterpret_cast<uint32_t*>(out);
      o32[0] = w[0];
      o32[1] = w[1];
      o32[2] = w[2];
    } else {
      for (int k = 0; k < 3 * n; ++k) out[k] = px[k];
    }
  }
}

}  // namespace

void jpeg_reconstruct(const JpegDesc* d_descs, uint8_t* d_pool, int n_images, int max_blocks, int64_t max_pixels,
                      hipStream_t s) {
  if (n_images <= 0) return;
  const dim3 g1((unsigned)((max_blocks + kBlocksPerGroup - 1) / kBlocksPerGroup), (unsigned)n_images);
  if (max_blocks > 0) hipLaunchKernelGGL(jpeg_idct_kernel, g1, dim3(256), 0, s, d_descs, d_pool);
  // one lane per 4-pixel quad of a row, grid-stride over the image's rows x quads
  const dim3 g2((unsigned)std::max<int64_t>(1, (max_pixels + 1023) / 1024), (unsigned)n_images);
  if (max_pixels > 0) hipLaunchKernelGGL(jpeg_color_kernel, g2, dim3(256), 0, s, d_descs, d_pool);
}

}  // namespace arena
