// Device-side description of one entropy-decoded baseline JPEG (the split decoder's hand-off from the host
// Huffman decoder, csrc/runtime/jpeg_decode.h, to the reconstruction kernels, csrc/kernels/jpeg_idct.hip).
// Offsets are bytes from the base of a staging slot's image pool (Executor d_in), so one descriptor array
// describes a whole batch.
#pragma once
#include <cstdint>

namespace arena {

constexpr int kJpegMaxComp = 3;

// Chroma layouts the split decoder reconstructs on the device; anything else goes to the PIL fallback.
enum JpegLayout : int32_t { JPEG_GRAY = 0, JPEG_444 = 1, JPEG_422 = 2, JPEG_420 = 3 };

struct JpegCompDesc {
  int32_t h, v;       // sampling factors
  int32_t bw, bh;     // stored 8x8 blocks per row / block rows (the MCU grid's coverage of this component)
  int32_t cw, ch;     // component size in samples (ceil(width * h / hmax), ceil(height * v / vmax))
  int64_t coef_off;   // int16[bh][bw][64] quantized coefficients, natural order
  int64_t plane_off;  // uint8 reconstructed samples, row stride bw * 8
};

struct JpegDesc {
  int32_t ncomp, layout, width, height;
  int32_t total_blocks;  // sum over components of bw * bh
  int32_t pad_[3];
  int64_t rgb_off;       // packed HxWx3 RGB output (the ImageMeta offset the pipeline reads)
  JpegCompDesc comp[kJpegMaxComp];
  uint16_t qt[kJpegMaxComp][64];  // dequantization table per component, natural order
  // compact payload (runtime/jpeg_decode.h jpeg_decode_compact; comp[].coef_off unused): per block a uint64
  // zigzag mask at cmask_off, a uint32 first-value index at cvoff_off, int16 values in zigzag order at cval_off
  int64_t cmask_off, cvoff_off, cval_off;
  int32_t compact, pad2_;
};
static_assert(sizeof(JpegDesc) == 576, "JpegDesc layout is shared with the kernels");

}  // namespace arena
