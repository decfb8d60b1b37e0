// Device half of the split JPEG decoder (host half: csrc/runtime/jpeg_decode.h).
//
// A batch of entropy-decoded images (quantized int16 coefficient blocks + one JpegDesc each) becomes packed
// HxWx3 RGB in the staging slot's image pool, where the fused letterbox/stem kernel and the crop gather read
// it — exactly the bytes the host path used to upload after a PIL decode.  Two launches per batch:
//
//   jpeg_idct_kernel    one 8x8 block per 8 lanes: dequantize (row loads of 16 B), islow pass 1 over the
//                       columns and pass 2 over the rows through an LDS transpose, 8 samples (one 8-byte store)
//                       per lane into the component's sample plane.  grid (blocks / 32, images).
//   jpeg_color_kernel   4 output pixels per lane: fancy chroma upsampling from the planes (h2v2 / h2v1 / none)
//                       + YCbCr->RGB, three 4-byte stores (12 bytes = 4 RGB pixels, aligned).  grid (pixels /
//                       1024, images).
//
// The arithmetic is kernels/jpeg_math.h, the same functions the host reference (jpeg_coefs_to_rgb) uses, so
// the result is bit-identical to it and to PIL / libjpeg-turbo (tests/test_jpeg_native_gpu.py).  The work is
// a few MB of traffic per batch of 32 frames: latency, not throughput, is what the layout optimises (every
// lane of a wave does useful work; no divergent per-component loops).
#include <hip/hip_runtime.h>

#include "jpeg_desc.h"
#include "jpeg_math.h"
#include "launch.h"

namespace arena {

namespace {

constexpr int kBlocksPerGroup = 32;  // 8x8 blocks per 256-lane workgroup

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
  if (live) {
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

__device__ __forceinline__ void chroma_at(const JpegDesc& d, const uint8_t* __restrict__ pool, int x, int y,
                                          int* cb, int* cr) {
  const int layout = d.layout;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const JpegCompDesc& C = d.comp[1 + k];
    const uint8_t* cp = pool + C.plane_off;
    const int64_t cs = (int64_t)C.bw * 8;
    int val;
    if (layout == JPEG_444) {
      val = cp[(int64_t)y * cs + x];
    } else {
      const int cx = x >> 1, xo = x & 1;
      const int nx = xo ? min(cx + 1, C.cw - 1) : max(cx - 1, 0);
      if (layout == JPEG_422) {
        val = jpegm::fancy_h2v1(cp[(int64_t)y * cs + cx], cp[(int64_t)y * cs + nx], xo);
      } else {
        const int cy = y >> 1;
        const int ny = (y & 1) ? min(cy + 1, C.ch - 1) : max(cy - 1, 0);
        val = jpegm::fancy_h2v2(cp[(int64_t)cy * cs + cx], cp[(int64_t)cy * cs + nx], cp[(int64_t)ny * cs + cx],
                                cp[(int64_t)ny * cs + nx], xo);
      }
    }
    if (k == 0) *cb = val;
    else *cr = val;
  }
}

__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegDesc* __restrict__ descs, uint8_t* __restrict__ pool) {
  const JpegDesc& d = descs[blockIdx.y];
  const int W = d.width, H = d.height;
  const int64_t npix = (int64_t)W * H;
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= npix) return;
  const uint8_t* yp = pool + d.comp[0].plane_off;
  const int64_t ys = (int64_t)d.comp[0].bw * 8;
  uint8_t px[12];
  int y = (int)(p0 / W), x = (int)(p0 - (int64_t)y * W);
  const int n = (int)min((int64_t)4, npix - p0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < n) {
      const int yy = yp[(int64_t)y * ys + x];
      if (d.layout == JPEG_GRAY) {
        px[3 * i] = px[3 * i + 1] = px[3 * i + 2] = (uint8_t)yy;
      } else {
        int cb, cr;
        chroma_at(d, pool, x, y, &cb, &cr);
        jpegm::ycc_to_rgb(yy, cb, cr, px + 3 * i);
      }
      if (++x == W) {
        x = 0;
        ++y;
      }
    }
  }
  uint8_t* out = pool + d.rgb_off + p0 * 3;
  if (n == 4) {
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

}  // namespace

void jpeg_reconstruct(const JpegDesc* d_descs, uint8_t* d_pool, int n_images, int max_blocks, int64_t max_pixels,
                      hipStream_t s) {
  if (n_images <= 0) return;
  const dim3 g1((unsigned)((max_blocks + kBlocksPerGroup - 1) / kBlocksPerGroup), (unsigned)n_images);
  if (max_blocks > 0) hipLaunchKernelGGL(jpeg_idct_kernel, g1, dim3(256), 0, s, d_descs, d_pool);
  const dim3 g2((unsigned)((max_pixels + 1023) / 1024), (unsigned)n_images);
  if (max_pixels > 0) hipLaunchKernelGGL(jpeg_color_kernel, g2, dim3(256), 0, s, d_descs, d_pool);
}

}  // namespace arena
