// Host half of the split JPEG decoder: marker parsing + baseline Huffman entropy decoding into quantized DCT
// coefficient blocks.  The device half (dequantisation, islow IDCT, fancy chroma upsampling, YCbCr->RGB) runs
// as HIP kernels on the batch (csrc/kernels/jpeg_idct.hip), so the host spends only the entropy decode per
// upload; everything after it is a few microseconds of GPU time per image.
//
// The reference decodes every upload entirely on the CPU (cv2.imdecode, src/shared/processing/transforms.py:
// 77-110; PIL for arm B crops, architectures/microservices/classification/app/servicer.py:65-76).  Here the
// work PIL does in one call is cut where the data is smallest and the arithmetic least parallel: the bit
// serial Huffman stream stays on a host thread, the per-pixel math moves to the GPU.
//
// Scope: baseline / extended-sequential Huffman (SOF0, SOF1), 8-bit samples, one interleaved scan with all
// components, 1 (grayscale) or 3 (YCbCr) components in 4:4:4, 4:2:2 or 4:2:0, restart intervals.  Everything
// else — progressive, arithmetic-coded, 12-bit, CMYK, RGB-coded, multi-scan, other samplings — is reported as
// Unsupported and the caller sends the upload to the PIL fallback (server/decode_pool.py).  The same
// reconstruction arithmetic is available on the host (jpeg_coefs_to_rgb) as the bit-exact reference of the
// kernels and as a host-only decode.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../kernels/jpeg_desc.h"

namespace arena {

struct JpegHuffSpec {
  bool present = false;
  uint8_t bits[17] = {};   // codes per length 1..16
  uint8_t vals[256] = {};  // symbols in code order
};

struct JpegInfo {
  int width = 0, height = 0, ncomp = 0;
  int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
  int layout = -1;
  int restart_interval = 0;
  int comp_id[kJpegMaxComp] = {};
  int tq[kJpegMaxComp] = {}, td[kJpegMaxComp] = {}, ta[kJpegMaxComp] = {};
  JpegCompDesc comp[kJpegMaxComp] = {};  // coef_off: element (int16) offsets into the coefficient buffer
  uint16_t qt[kJpegMaxComp][64] = {};    // per component, natural order
  int64_t coef_count = 0;                // int16 coefficients of all components
  int64_t plane_bytes = 0;               // reconstructed sample planes of all components
  size_t scan_begin = 0;                 // first byte of the entropy-coded segment
  // compact payload (jpeg_decode_compact): its bytes and the byte offsets of its three arrays; -1 = dense int16
  int64_t compact_bytes = -1;
  int64_t cmask_off = 0, cvoff_off = 0, cval_off = 0;
  JpegHuffSpec dc[4], ac[4];
};

enum class JpegStatus : int { Ok = 0, Unsupported = 1, Corrupt = 2 };

// Parse the markers up to the (single) scan.  `max_pixels` > 0 rejects larger frames as Corrupt with an
// "image too large" message (the decode-bomb guard of processing/transforms.py).
JpegStatus jpeg_parse(const uint8_t* data, size_t n, JpegInfo& info, std::string& err, int64_t max_pixels = 0);

// Entropy-decode the scan: info.coef_count int16 quantized coefficients, natural order, one block after the
// other (component c's block (by, bx) at comp[c].coef_off + (by * bw + bx) * 64).  A scan cut short by a
// marker is padded with zero bits (libjpeg's warning, which PIL ignores); a file that simply ends inside the
// scan is Corrupt ("image file is truncated", as PIL raises), like structurally broken streams.
JpegStatus jpeg_decode_coefs(const uint8_t* data, size_t n, const JpegInfo& info, int16_t* coef, std::string& err);

// The same scan into the compact payload the split decoder ships (3-4x fewer bytes than the dense blocks at q90:
// most AC coefficients are zero).  Per 8x8 block, in the dense layout's block order (component 0's blocks row by
// row, then 1, 2): a uint64 mask (bit k: the coefficient at zigzag index k is coded), then per block the uint32
// index of its first value, then the int16 values of every block in zigzag order (16-byte aligned array).  `out`
// holds jpeg_compact_capacity(info) bytes; on success info.compact_bytes / cmask_off / cvoff_off / cval_off
// describe what was written.  Status and error messages as jpeg_decode_coefs.
JpegStatus jpeg_decode_compact(const uint8_t* data, size_t n, JpegInfo& info, uint8_t* out, std::string& err);
int64_t jpeg_total_blocks(const JpegInfo& info);
int64_t jpeg_compact_capacity(const JpegInfo& info);
// bytes of the decoded payload (compact, or dense int16)
int64_t jpeg_payload_bytes(const JpegInfo& info);
// ARENA_JPEG_COMPACT (default 1): the serving paths decode into the compact payload; 0 keeps dense blocks
bool jpeg_compact_enabled();
// compact payload -> dense int16 blocks (host reference paths)
void jpeg_compact_to_dense(const JpegInfo& info, const uint8_t* payload, int16_t* coef);
// the payload as dense blocks: itself when dense, else expanded into `scratch`
const int16_t* jpeg_dense_coefs(const JpegInfo& info, const uint8_t* payload, std::vector<int16_t>& scratch);

// Host reconstruction with the device kernels' exact arithmetic (kernels/jpeg_math.h): packed HxWx3 RGB.
void jpeg_coefs_to_rgb(const JpegInfo& info, const int16_t* coef, uint8_t* rgb);

// The device descriptor of a parsed image, with byte offsets relative to `coef_base` / `plane_base` / `rgb_off`.
JpegDesc jpeg_device_desc(const JpegInfo& info, int64_t coef_base, int64_t plane_base, int64_t rgb_off);

}  // namespace arena
