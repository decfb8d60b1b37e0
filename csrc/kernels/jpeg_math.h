// Integer reconstruction arithmetic of a baseline JPEG, shared by the host reference decoder
// (csrc/runtime/jpeg_decode.cpp) and the device kernels (csrc/kernels/jpeg_idct.hip).
//
// The reference decodes uploads with cv2.imdecode / PIL (src/shared/processing/transforms.py:77-110,
// architectures/microservices/classification/app/servicer.py:65-76), both libjpeg(-turbo) with its default
// decompression settings: the accurate integer IDCT (JDCT_ISLOW), "fancy" triangle-filter chroma upsampling and
// the table-driven YCbCr->RGB conversion.  This header reproduces exactly that arithmetic (same fixed-point
// constants, same rounding biases, same edge replication), so a frame reconstructed here is bit-identical to
// PIL's (tests/test_jpeg_native.py pins that on the curated workload).
//
// Attribution: the IDCT below follows the structure and fixed-point constants of libjpeg's jidctint.c (islow), the
// chroma upsampling that of jdsample.c (h2v1 / h2v2 "fancy" upsampling) and the colour conversion that of
// jdcolor.c (ycc_rgb_convert).  Bit-exactness with PIL / libjpeg-turbo requires exactly that arithmetic.  This
// software is based in part on the work of the Independent JPEG Group (see NOTICE at the repository root).
//
// Everything is plain integer math on values the caller supplies; there is no table and no memory access, so
// the same functions run per lane in the HIP kernel and per pixel in the host reference.
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define ARENA_JHD __host__ __device__ __forceinline__
#else
#define ARENA_JHD inline
#endif

namespace arena {
namespace jpegm {

constexpr int kConstBits = 13;
constexpr int kPass1Bits = 2;
// FIX(x) = round(x * 2^13): libjpeg's jidctint.c constants
constexpr int32_t F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433, F_0_765366865 = 6270,
                  F_0_899976223 = 7373, F_1_175875602 = 9633, F_1_501321110 = 12299, F_1_847759065 = 15137,
                  F_1_961570560 = 16069, F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;

// Arithmetic right shift with round-half-up (libjpeg DESCALE).
template <typename T>
ARENA_JHD T descale(T x, int n) {
  return (x + ((T)1 << (n - 1))) >> n;
}

// One 1-D pass of the accurate integer IDCT (jpeg_idct_islow) over in[0..7]; outputs are descaled by `shift`
// (pass 1: kConstBits - kPass1Bits, pass 2: kConstBits + kPass1Bits + 3).  T is the accumulator type: int64_t
// reproduces libjpeg's JLONG exactly for any input, int32_t is exact for every coefficient set a real 8-bit
// image produces (|dequantized coefficient| < 2^15) and is what the GPU uses.
template <typename T>
ARENA_JHD void idct8(const T in[8], T out[8], int shift) {
  // even part: the rotator is sqrt(2) * c(-6)
  T z2 = in[2], z3 = in[6];
  T z1 = (z2 + z3) * F_0_541196100;
  T tmp2 = z1 + z3 * (-F_1_847759065);
  T tmp3 = z1 + z2 * F_0_765366865;
  T tmp0 = (in[0] + in[4]) * ((T)1 << kConstBits);
  T tmp1 = (in[0] - in[4]) * ((T)1 << kConstBits);
  const T tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  // odd part
  tmp0 = in[7];
  tmp1 = in[5];
  tmp2 = in[3];
  tmp3 = in[1];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  T z4 = tmp1 + tmp3;
  const T z5 = (z3 + z4) * F_1_175875602;
  tmp0 = tmp0 * F_0_298631336;
  tmp1 = tmp1 * F_2_053119869;
  tmp2 = tmp2 * F_3_072711026;
  tmp3 = tmp3 * F_1_501321110;
  z1 = z1 * (-F_0_899976223);
  z2 = z2 * (-F_2_562915447);
  z3 = z3 * (-F_1_961570560) + z5;
  z4 = z4 * (-F_0_390180644) + z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  out[0] = descale<T>(tmp10 + tmp3, shift);
  out[7] = descale<T>(tmp10 - tmp3, shift);
  out[1] = descale<T>(tmp11 + tmp2, shift);
  out[6] = descale<T>(tmp11 - tmp2, shift);
  out[2] = descale<T>(tmp12 + tmp1, shift);
  out[5] = descale<T>(tmp12 - tmp1, shift);
  out[3] = descale<T>(tmp13 + tmp0, shift);
  out[4] = descale<T>(tmp13 - tmp0, shift);
}

constexpr int kPass1Shift = kConstBits - kPass1Bits;
constexpr int kPass2Shift = kConstBits + kPass1Bits + 3;

// Pass-2 output -> sample: level shift by 128 and clamp (libjpeg-turbo's SIMD islow saturates; its C table
// agrees for every |x| < 512, i.e. every real image).
template <typename T>
ARENA_JHD uint8_t idct_sample(T x) {
  const T v = x + 128;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// "Fancy" h2v2 upsampling (jdsample.c h2v2_fancy_upsample) of output pixel (x, y): `c00` is the nearest chroma
// sample, `c01` the horizontal neighbour on the output pixel's side, `c10` the vertical neighbour (row above for
// even y, below for odd y), `c11` the diagonal one; neighbours outside the component are the edge sample
// itself (libjpeg replicates the first / last row and column), which reproduces its edge special cases.
ARENA_JHD int fancy_h2v2(int c00, int c01, int c10, int c11, int x_odd) {
  const int this_sum = c00 * 3 + c10;
  const int other_sum = c01 * 3 + c11;
  return (this_sum * 3 + other_sum + (x_odd ? 7 : 8)) >> 4;
}

// h2v1 (4:2:2): jdsample.c h2v1_fancy_upsample; `cn` is the horizontal neighbour on the output pixel's side.
ARENA_JHD int fancy_h2v1(int c, int cn, int x_odd) { return (c * 3 + cn + (x_odd ? 2 : 1)) >> 2; }

// YCbCr -> RGB (jdcolor.c ycc_rgb_convert with its build_ycc_rgb_table entries, SCALEBITS 16).
ARENA_JHD void ycc_to_rgb(int y, int cb, int cr, uint8_t* rgb) {
  const int x_cb = cb - 128, x_cr = cr - 128;
  const int r_off = (91881 * x_cr + 32768) >> 16;                   // FIX(1.40200)
  const int b_off = (116130 * x_cb + 32768) >> 16;                  // FIX(1.77200)
  const int g_off = ((-22554) * x_cb + 32768 + (-46802) * x_cr) >> 16;  // FIX(0.34414), FIX(0.71414)
  const int r = y + r_off, g = y + g_off, b = y + b_off;
  rgb[0] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
  rgb[1] = (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
  rgb[2] = (uint8_t)(b < 0 ? 0 : (b > 255 ? 255 : b));
}

}  // namespace jpegm
}  // namespace arena
