// Letterbox sampling shared by the standalone letterbox kernel (preprocess.hip) and the fp32 stem conv that
// reads the uint8 image directly (conv_f32.hip, impl kF32X3H16 with a letterbox source): both produce the
// space-to-depth(2) pixel through letterbox_s2d_px, so the fused and unfused programs see bitwise the same
// input values.
//
// Reference semantics: src/shared/processing/transforms.py:118-180 (scale = min(T/h, T/w), int-truncated
// new size, floor-centred pad, gray 114, cv2 INTER_LINEAR) and src/shared/processing/yolo_preprocess.py:154-167
// (/255).  INTER_LINEAR geometry: src = (dst + 0.5) * (src_size / dst_size) - 0.5, clamped to the border; the
// interpolated value is rounded to uint8 before normalisation, as cv2 returns a uint8 image.
#pragma once

#include "common.h"
#include "launch.h"

namespace arena {

struct LinTap {
  int i0, i1;
  float f;
};

__device__ __forceinline__ LinTap lin_tap(int d, float scale, int n) {
#pragma clang fp contract(off)  // (d + 0.5) * scale - 0.5 rounded twice, as the host computes it
  float fx = ((float)d + 0.5f) * scale - 0.5f;
  int s0 = (int)floorf(fx);
  float f = fx - (float)s0;
  if (s0 < 0) { s0 = 0; f = 0.f; }
  if (s0 >= n - 1) { s0 = n - 1; f = 0.f; }
  LinTap t;
  t.i0 = s0;
  t.i1 = s0 + 1 < n ? s0 + 1 : n - 1;
  t.f = f;
  return t;
}

__device__ __forceinline__ void bilinear_rgb(const uint8_t* img, int stride_px, LinTap ty, LinTap tx,
                                             float* rgb) {
  // separately rounded multiply and add, as the host resize (numpy) computes them: a fused multiply-add
  // moves values that sit at x.5 to the other side of the uint8 rounding
#pragma clang fp contract(off)
  const uint8_t* r0 = img + (size_t)ty.i0 * stride_px * 3;
  const uint8_t* r1 = img + (size_t)ty.i1 * stride_px * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float a = (float)r0[tx.i0 * 3 + c], b = (float)r0[tx.i1 * 3 + c];
    const float d = (float)r1[tx.i0 * 3 + c], e = (float)r1[tx.i1 * 3 + c];
    const float top = a + (b - a) * tx.f;
    const float bot = d + (e - d) * tx.f;
    float v = top + (bot - top) * ty.f;
    rgb[c] = floorf(v + 0.5f);  // cv2 returns uint8: round to nearest
  }
}

// /255 of a uint8 value: the exact-fp32 pipeline divides as the host preprocessor does; the bf16 pipeline
// multiplies by the reciprocal (the difference is far below its rounding).
template <typename T>
__device__ __forceinline__ float div255(float v) {
  if constexpr (sizeof(T) == 4) return v / 255.0f;
  else return v * (1.0f / 255.0f);
}

// The 12 live channels of letterboxed space-to-depth pixel (Y, X) of image m as uint8 values (exact small
// integers in fp32): out[pq * 3 + c] is colour c of sub-pixel (2Y + pq / 2, 2X + pq % 2) of the T x T
// letterboxed image (cv2 INTER_LINEAR rounded to uint8, gray 114 outside the resized image).
__device__ __forceinline__ void letterbox_s2d_px_u8(const uint8_t* pool, const ImageMeta& m, int Y, int X,
                                                    float* out) {
  const uint8_t* img = pool + m.offset;
  const float sy = (float)((double)m.h / (double)m.new_h);
  const float sx = (float)((double)m.w / (double)m.new_w);
  // unit scale (the image's long side is already T: COCO's 640x480 / 640x427 ...): the bilinear taps have zero
  // weight, so the letterboxed pixel is the source pixel (bitwise the same value) — 3 byte loads instead of 12
  const bool unit = m.new_h == m.h && m.new_w == m.w;
#pragma unroll
  for (int pq = 0; pq < 4; ++pq) {
    const int oy = 2 * Y + (pq >> 1), ox = 2 * X + (pq & 1);
    const int dy = oy - m.pad_h, dx = ox - m.pad_w;
    float rgb[3] = {114.f, 114.f, 114.f};
    if (dy >= 0 && dy < m.new_h && dx >= 0 && dx < m.new_w) {
      if (unit) {
        const uint8_t* px = img + ((size_t)dy * m.w + dx) * 3;
        rgb[0] = (float)px[0];
        rgb[1] = (float)px[1];
        rgb[2] = (float)px[2];
      } else {
        bilinear_rgb(img, m.w, lin_tap(dy, sy, m.h), lin_tap(dx, sx, m.w), rgb);
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) out[pq * 3 + c] = rgb[c];
  }
}

// The same pixel normalised (/255): the letterbox op's output.
template <typename T>
__device__ __forceinline__ void letterbox_s2d_px(const uint8_t* pool, const ImageMeta& m, int Y, int X,
                                                 float* out) {
  letterbox_s2d_px_u8(pool, m, Y, X, out);
#pragma unroll
  for (int c = 0; c < 12; ++c) out[c] = div255<T>(out[c]);
}

}  // namespace arena
