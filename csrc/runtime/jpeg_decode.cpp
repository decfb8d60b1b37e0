// See jpeg_decode.h.
#include "runtime/jpeg_decode.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../kernels/jpeg_math.h"

namespace arena {

namespace {

// zig-zag index -> natural index, with 16 guard entries so a corrupt run past coefficient 63 stays in the block
// (libjpeg's jpeg_natural_order has the same padding)
constexpr uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// Kraft check of a DHT's code-length counts (JPEG Annex C): the canonical code assigns codes of length l in order,
// so after each length the next code must still fit in l bits.  An over-subscribed table is corrupt data.
bool huff_lengths_valid(const uint8_t* bits) {
  int64_t code = 0;
  for (int l = 1; l <= 16; ++l) {
    code += bits[l];
    if (code > (int64_t(1) << l)) return false;
    code <<= 1;
  }
  return true;
}

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

constexpr int kFastBits = 11;
constexpr int kEobRun = 127;  // ac_fast run of an EOB entry

inline int extend(uint32_t v, int s) { return (int)v - ((v < (1u << (s - 1))) ? (int)((1u << s) - 1) : 0); }

// Decoding tables of one Huffman code (JPEG Annex C / F.2.2.3): an 11-bit lookahead table resolves every code of
// up to 11 bits with one lookup; longer codes walk maxcode / valoff by length.  AC tables also get `ac_fast`:
// when a code and the magnitude bits that follow it fit in the 11-bit lookahead, one lookup yields the run,
// the signed coefficient and the total bit count (most coefficients of a q90 frame).
struct HuffTable {
  uint16_t fast[1 << kFastBits];  // (length << 8) | symbol, 0 = longer than kFastBits
  int32_t ac_fast[1 << kFastBits];  // (value << 16) | (run << 8) | total length, 0 = no shortcut
  int32_t maxcode[18];            // largest code of each length (-1: none); [17] sentinel
  int32_t valoff[17];             // symbol index of the first code of each length minus that code
  uint8_t vals[256];

  bool build(const JpegHuffSpec& s, bool ac) {
    std::memset(fast, 0, sizeof fast);
    std::memset(ac_fast, 0, sizeof ac_fast);
    std::memcpy(vals, s.vals, sizeof vals);
    int32_t code = 0;
    int k = 0;
    for (int l = 1; l <= 16; ++l) {
      const int n = s.bits[l];
      valoff[l] = k - code;
      if (n) {
        for (int i = 0; i < n; ++i, ++k, ++code) {
          // over-subscribed code (too many codes of this or a shorter length): reject it before any table
          // write, as libjpeg's jdhuff.c does; (code << shift) | j would otherwise index past fast / ac_fast
          if (code >= (1 << l) || k >= 256) return false;
          if (l <= kFastBits) {
            const int shift = kFastBits - l;
            const uint8_t sym = s.vals[k];
            const uint16_t e = (uint16_t)((l << 8) | sym);
            for (int j = 0; j < (1 << shift); ++j) {
              const int idx = (code << shift) | j;
              fast[idx] = e;
              const int run = sym >> 4, mag = sym & 15;
              if (ac && mag && l + mag <= kFastBits) {
                const uint32_t bitsv = (uint32_t)(j >> (shift - mag)) & ((1u << mag) - 1);
                const int v = extend(bitsv, mag);
                ac_fast[idx] = (int32_t)((uint32_t)v << 16) | (run << 8) | (l + mag);
              } else if (ac && sym == 0x00) {
                ac_fast[idx] = (kEobRun << 8) | l;  // EOB: the run pushes k past the block
              } else if (ac && sym == 0xF0) {
                ac_fast[idx] = (15 << 8) | l;       // ZRL: 15 zeros + a stored zero = 16 positions
              }
            }
          }
        }
        maxcode[l] = code - 1;
      } else {
        maxcode[l] = -1;
      }
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    return true;
  }
};

// MSB-first bit reader over the entropy-coded segment: removes the 0xFF00 stuffing, stops at a marker and
// then feeds zero bits (libjpeg's behaviour on truncated data).  The fast refill takes up to 7 bytes at once
// when none of them is 0xFF.
struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int bits = 0;
  bool marker = false;
  int64_t pad = 0;         // zero bytes fed because the data ended without a marker
  int64_t zfill = 0;       // zero bytes fed after a marker cut the segment short
  bool truncated = false;  // some of the `pad` bits were consumed (PIL: "image file is truncated")

  __attribute__((always_inline)) inline void refill() {
    if (!marker && end - p >= 8) {
      uint64_t x;
      std::memcpy(&x, p, 8);
      x = __builtin_bswap64(x);
      const int k = (63 - bits) >> 3;  // whole bytes that fit
      const uint64_t keep = ~0ULL << (64 - 8 * k);
      const uint64_t nx = ~x;          // 0xFF bytes -> 0x00
      const uint64_t ff = (nx - 0x0101010101010101ULL) & ~nx & 0x8080808080808080ULL;
      if ((ff & keep) == 0) {
        buf |= (x & keep) >> bits;
        bits += 8 * k;
        p += k;
        return;
      }
    }
    refill_slow();
  }
  void refill_slow() {
    while (bits <= 56) {
      uint32_t b = 0;
      if (marker) ++zfill;
      else if (p >= end) ++pad;
      if (!marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          const uint32_t nb = p + 1 < end ? p[1] : 0xD9;
          if (nb == 0x00) {
            p += 2;
          } else {
            marker = true;  // p stays on the marker
            ++zfill;
            b = 0;
          }
        } else {
          ++p;
        }
      }
      buf |= (uint64_t)b << (56 - bits);
      bits += 8;
    }
  }
  __attribute__((always_inline)) inline void need(int n) {
    if (bits < n) refill();
  }
  __attribute__((always_inline)) inline void skip(int n) {
    buf <<= n;
    bits -= n;
  }
  __attribute__((always_inline)) inline uint32_t get(int n) {  // 1 <= n <= 16, after need()
    const uint32_t v = (uint32_t)(buf >> (64 - n));
    buf <<= n;
    bits -= n;
    return v;
  }
  // one Huffman symbol; needs 16 valid bits
  __attribute__((always_inline)) inline int decode(const HuffTable& t) {
    const uint32_t e = t.fast[buf >> (64 - kFastBits)];
    if (e) {
      skip((int)(e >> 8));
      return (int)(e & 0xFF);
    }
    return decode_slow(t);
  }
  int decode_slow(const HuffTable& t) {
    const uint32_t code16 = (uint32_t)(buf >> 48);
    for (int l = kFastBits + 1; l <= 16; ++l) {
      const int32_t c = (int32_t)(code16 >> (16 - l));
      if (c <= t.maxcode[l]) {
        skip(l);
        return t.vals[(t.valoff[l] + c) & 0xFF];
      }
    }
    // no code matches (corrupt data): libjpeg warns and yields symbol 0; consume 16 bits so the scan advances
    skip(16);
    return 0;
  }
  // Restart marker: drop the bits of the finished interval and step over RSTn (scanning forward if the
  // encoder left padding or the marker is missing, as libjpeg's resync does).
  bool overran() const { return pad * 8 > bits; }
  // libjpeg's insufficient_data: a bit past a marker was consumed; the rest of the segment decodes as zero
  // blocks (uniform grey) instead of reading the zero fill
  bool starved() const { return zfill * 8 > bits; }
  void restart() {
    truncated |= overran();
    pad = 0;
    zfill = 0;
    buf = 0;
    bits = 0;
    marker = false;
    while (p + 1 < end) {
      if (p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7) {
        p += 2;
        return;
      }
      if (p[0] == 0xFF && p[1] != 0x00 && p[1] != 0xFF) return;  // some other marker: leave it for the reader
      ++p;
    }
  }
};

// One 8x8 block: DC difference + AC run/size symbols, coefficients written in natural order.
__attribute__((always_inline)) inline bool decode_block(BitReader& br, const HuffTable& dc, const HuffTable& ac,
                                                        int& pred, int16_t* blk) {
  std::memset(blk, 0, 64 * sizeof(int16_t));
  br.need(32);
  const int s = br.decode(dc);
  if (s) {
    if (s > 15) return false;
    pred += extend(br.get(s), s);
  }
  blk[0] = (int16_t)pred;
  for (int k = 1; k < 64;) {
    br.need(32);  // a code (<= 16 bits) and its magnitude (<= 15 bits)
    const int32_t f = ac.ac_fast[br.buf >> (64 - kFastBits)];
    if (f) {  // one lookup: coefficient, ZRL or EOB
      br.skip(f & 0xFF);
      k += (f >> 8) & 0xFF;
      if (k > 63) break;  // EOB (or a corrupt run past the block)
      blk[kNatural[k]] = (int16_t)(f >> 16);
      ++k;
      continue;
    }
    const int rs = br.decode(ac);
    const int r = rs >> 4, sz = rs & 15;
    if (sz) {
      k += r;
      blk[kNatural[k]] = (int16_t)extend(br.get(sz), sz);
      ++k;
    } else {
      if (r != 15) break;  // EOB
      k += 16;
    }
  }
  return true;
}


// The same block in the compact layout (jpeg_decode.h, jpeg_decode_compact): bit k of *mask set for every coded
// coefficient at zigzag index k, their values appended to vals in zigzag order (the DC always, even when 0).
__attribute__((always_inline)) inline bool decode_block_compact(BitReader& br, const HuffTable& dc, const HuffTable& ac,
                                                                int& pred, uint64_t* mask, int16_t* vals, int64_t& nv) {
  br.need(32);
  const int s = br.decode(dc);
  if (s) {
    if (s > 15) return false;
    pred += extend(br.get(s), s);
  }
  uint64_t m = 1;
  int64_t n = nv;
  vals[n++] = (int16_t)pred;
  for (int k = 1; k < 64;) {
    br.need(32);
    const int32_t f = ac.ac_fast[br.buf >> (64 - kFastBits)];
    if (f) {
      br.skip(f & 0xFF);
      k += (f >> 8) & 0xFF;
      if (k > 63) break;
      m |= 1ull << k;
      vals[n++] = (int16_t)(f >> 16);
      ++k;
      continue;
    }
    const int rs = br.decode(ac);
    const int r = rs >> 4, sz = rs & 15;
    if (sz) {
      k += r;
      const int16_t v = (int16_t)extend(br.get(sz), sz);
      if (k > 63) {  // a corrupt run past the block: the dense decoder's kNatural pad stores it at 63
        if (m >> 63) vals[n - 1] = v;  // zigzag 63 is the last value appended
        else {
          m |= 1ull << 63;
          vals[n++] = v;
        }
      } else {
        m |= 1ull << k;
        vals[n++] = v;
      }
      ++k;
    } else {
      if (r != 15) break;
      k += 16;
    }
  }
  *mask = m;
  nv = n;
  return true;
}

}  // namespace

JpegStatus jpeg_parse(const uint8_t* data, size_t n, JpegInfo& info, std::string& err, int64_t max_pixels) {
  info = JpegInfo{};
  if (n < 4 || data[0] != 0xFF || data[1] != 0xD8) {
    err = "not a JPEG stream";
    return JpegStatus::Unsupported;  // PNG, WebP, ... : the fallback identifies it
  }
  uint16_t qtab[4][64];
  bool qpresent[4] = {false, false, false, false};
  bool saw_sof = false, saw_jfif = false, adobe = false;
  int adobe_transform = -1;
  size_t pos = 2;
  while (true) {
    while (pos < n && data[pos] != 0xFF) ++pos;  // tolerate garbage between markers (libjpeg warns)
    while (pos < n && data[pos] == 0xFF) ++pos;
    if (pos >= n) {
      err = "Failed to decode image: no scan before the end of data";
      return JpegStatus::Corrupt;
    }
    const int m = data[pos++];
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // standalone markers
    if (m == 0xD9) {
      err = "Failed to decode image: end of image before the first scan";
      return JpegStatus::Corrupt;
    }
    if (pos + 2 > n) {
      err = "Failed to decode image: truncated marker";
      return JpegStatus::Corrupt;
    }
    const size_t len = be16(data + pos);
    if (len < 2 || pos + len > n) {
      err = "Failed to decode image: truncated marker segment";
      return JpegStatus::Corrupt;
    }
    const uint8_t* seg = data + pos + 2;
    const size_t sl = len - 2;
    pos += len;
    if (m == 0xC0 || m == 0xC1) {
      if (saw_sof || sl < 6) {
        err = "Failed to decode image: bad SOF";
        return JpegStatus::Corrupt;
      }
      saw_sof = true;
      if (seg[0] != 8) {
        err = "12-bit JPEG";
        return JpegStatus::Unsupported;
      }
      info.height = be16(seg + 1);
      info.width = be16(seg + 3);
      info.ncomp = seg[5];
      if (info.height == 0) {
        err = "height from DNL";
        return JpegStatus::Unsupported;
      }
      if (info.width == 0 || sl < 6 + 3 * (size_t)info.ncomp) {
        err = "Failed to decode image: bad SOF";
        return JpegStatus::Corrupt;
      }
      if (info.ncomp != 1 && info.ncomp != 3) {
        err = "component count";
        return JpegStatus::Unsupported;
      }
      if (max_pixels > 0 && (int64_t)info.width * info.height > max_pixels) {
        err = "Failed to decode image: image too large (" + std::to_string(info.width) + "x" +
              std::to_string(info.height) + " pixels > " + std::to_string(max_pixels) + ")";
        return JpegStatus::Corrupt;
      }
      for (int c = 0; c < info.ncomp; ++c) {
        info.comp_id[c] = seg[6 + 3 * c];
        info.comp[c].h = seg[7 + 3 * c] >> 4;
        info.comp[c].v = seg[7 + 3 * c] & 15;
        info.tq[c] = seg[8 + 3 * c];
        if (info.comp[c].h < 1 || info.comp[c].h > 4 || info.comp[c].v < 1 || info.comp[c].v > 4 || info.tq[c] > 3) {
          err = "Failed to decode image: bad sampling factors";
          return JpegStatus::Corrupt;
        }
      }
    } else if (m == 0xC2 || m == 0xC3 || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) ||
               (m >= 0xCD && m <= 0xCF)) {
      err = "progressive, lossless or arithmetic-coded JPEG";
      return JpegStatus::Unsupported;
    } else if (m == 0xC4) {
      size_t q = 0;
      while (q < sl) {
        const int tc = seg[q] >> 4, th = seg[q] & 15;
        if (tc > 1 || th > 3 || q + 17 > sl) {
          err = "Failed to decode image: bad DHT";
          return JpegStatus::Corrupt;
        }
        JpegHuffSpec& h = tc == 0 ? info.dc[th] : info.ac[th];
        int count = 0;
        h.bits[0] = 0;
        for (int l = 1; l <= 16; ++l) {
          h.bits[l] = seg[q + l];
          count += h.bits[l];
        }
        if (count > 256 || q + 17 + count > sl || !huff_lengths_valid(h.bits)) {
          err = "Failed to decode image: bad DHT";
          return JpegStatus::Corrupt;
        }
        std::memset(h.vals, 0, sizeof h.vals);
        std::memcpy(h.vals, seg + q + 17, count);
        h.present = true;
        q += 17 + count;
      }
    } else if (m == 0xDB) {
      size_t q = 0;
      while (q < sl) {
        const int pq = seg[q] >> 4, tq = seg[q] & 15;
        const size_t need = 1 + (pq ? 128 : 64);
        if (pq > 1 || tq > 3 || q + need > sl) {
          err = "Failed to decode image: bad DQT";
          return JpegStatus::Corrupt;
        }
        for (int k = 0; k < 64; ++k)
          qtab[tq][kNatural[k]] = pq ? be16(seg + q + 1 + 2 * k) : seg[q + 1 + k];
        qpresent[tq] = true;
        q += need;
      }
    } else if (m == 0xDD) {
      if (sl < 2) {
        err = "Failed to decode image: bad DRI";
        return JpegStatus::Corrupt;
      }
      info.restart_interval = be16(seg);
    } else if (m == 0xE0) {
      if (sl >= 5 && std::memcmp(seg, "JFIF\0", 5) == 0) saw_jfif = true;
    } else if (m == 0xEE) {
      if (sl >= 12 && std::memcmp(seg, "Adobe", 5) == 0) {
        adobe = true;
        adobe_transform = seg[11];
      }
    } else if (m == 0xDA) {
      if (!saw_sof) {
        err = "Failed to decode image: scan before frame header";
        return JpegStatus::Corrupt;
      }
      const int ns = sl >= 1 ? seg[0] : 0;
      if (ns != info.ncomp) {
        err = "multi-scan (non-interleaved) JPEG";
        return JpegStatus::Unsupported;
      }
      if (sl < 1 + 2 * (size_t)ns + 3) {
        err = "Failed to decode image: bad SOS";
        return JpegStatus::Corrupt;
      }
      for (int i = 0; i < ns; ++i) {
        const int cs = seg[1 + 2 * i];
        if (cs != info.comp_id[i]) {
          err = "scan component order differs from the frame";
          return JpegStatus::Unsupported;
        }
        info.td[i] = seg[2 + 2 * i] >> 4;
        info.ta[i] = seg[2 + 2 * i] & 15;
        if (info.td[i] > 3 || info.ta[i] > 3 || !info.dc[info.td[i]].present || !info.ac[info.ta[i]].present) {
          err = "Failed to decode image: missing Huffman table";
          return JpegStatus::Corrupt;
        }
      }
      const uint8_t* t = seg + 1 + 2 * ns;
      if (t[0] != 0 || t[1] != 63 || t[2] != 0) {
        err = "Failed to decode image: bad spectral selection for a sequential scan";
        return JpegStatus::Corrupt;
      }
      info.scan_begin = pos;
      break;
    }
    // every other marker (APPn, COM, ...) is skipped by its length
  }
  // colour space as libjpeg guesses it (jdapimin.c default_decompress_parms): only YCbCr is reconstructed here
  if (info.ncomp == 3) {
    if (!saw_jfif && adobe && adobe_transform == 0) {
      err = "RGB-coded JPEG (Adobe transform 0)";
      return JpegStatus::Unsupported;
    }
    if (!saw_jfif && !adobe && info.comp_id[0] == 'R' && info.comp_id[1] == 'G' && info.comp_id[2] == 'B') {
      err = "RGB-coded JPEG";
      return JpegStatus::Unsupported;
    }
  }
  for (int c = 0; c < info.ncomp; ++c) {
    if (!qpresent[info.tq[c]]) {
      err = "Failed to decode image: missing quantization table";
      return JpegStatus::Corrupt;
    }
    std::memcpy(info.qt[c], qtab[info.tq[c]], sizeof info.qt[c]);
    info.hmax = std::max(info.hmax, info.comp[c].h);
    info.vmax = std::max(info.vmax, info.comp[c].v);
  }
  if (info.ncomp == 1) {
    info.layout = JPEG_GRAY;
  } else {
    const JpegCompDesc &y = info.comp[0], &cb = info.comp[1], &cr = info.comp[2];
    if (cb.h != cr.h || cb.v != cr.v || y.h != info.hmax || y.v != info.vmax || y.h % cb.h || y.v % cb.v) {
      err = "chroma sampling";
      return JpegStatus::Unsupported;
    }
    const int rh = y.h / cb.h, rv = y.v / cb.v;
    if (rh == 1 && rv == 1) info.layout = JPEG_444;
    else if (rh == 2 && rv == 1) info.layout = JPEG_422;
    else if (rh == 2 && rv == 2) info.layout = JPEG_420;
    else {
      err = "chroma sampling";
      return JpegStatus::Unsupported;
    }
  }
  info.mcux = (info.width + 8 * info.hmax - 1) / (8 * info.hmax);
  info.mcuy = (info.height + 8 * info.vmax - 1) / (8 * info.vmax);
  int64_t off = 0, planes = 0;
  for (int c = 0; c < info.ncomp; ++c) {
    JpegCompDesc& d = info.comp[c];
    d.cw = (int)(((int64_t)info.width * d.h + info.hmax - 1) / info.hmax);
    d.ch = (int)(((int64_t)info.height * d.v + info.vmax - 1) / info.vmax);
    if (info.ncomp == 1) {  // a single-component scan is not interleaved: one block per MCU
      d.bw = (d.cw + 7) / 8;
      d.bh = (d.ch + 7) / 8;
    } else {
      d.bw = info.mcux * d.h;
      d.bh = info.mcuy * d.v;
    }
    if (info.layout != JPEG_GRAY && info.layout != JPEG_444 && c > 0 && d.cw <= 2) {
      err = "chroma narrower than 3 samples (libjpeg switches to box upsampling)";
      return JpegStatus::Unsupported;
    }
    d.coef_off = off;
    d.plane_off = planes;
    off += (int64_t)d.bw * d.bh * 64;
    planes += (int64_t)d.bw * d.bh * 64;
  }
  info.coef_count = off;
  info.plane_bytes = planes;
  return JpegStatus::Ok;
}

namespace {
// Built decoding tables are ~12 KB each and nearly every upload carries the same few Huffman specs (the
// standard tables of libjpeg encoders), so each decode thread keeps the tables it built last.
struct TableCache {
  struct Entry {
    JpegHuffSpec spec;
    bool ac = false;
    bool valid = false;
    uint64_t used = 0;  // generation (image) that last used the entry: never evicted while that image decodes
    HuffTable table;
  };
  static constexpr int kEntries = 8;  // > the 6 tables one 3-component image can name
  Entry e[kEntries];
  int next = 0;
  uint64_t gen = 0;
  const HuffTable* get(const JpegHuffSpec& s, bool ac) {
    for (Entry& x : e)
      if (x.valid && x.ac == ac && std::memcmp(x.spec.bits, s.bits, sizeof s.bits) == 0 &&
          std::memcmp(x.spec.vals, s.vals, sizeof s.vals) == 0) {
        x.used = gen;
        return &x.table;
      }
    while (e[next].valid && e[next].used == gen) next = (next + 1) % kEntries;
    Entry& x = e[next];
    next = (next + 1) % kEntries;
    x.valid = false;
    if (!x.table.build(s, ac)) return nullptr;
    x.spec = s;
    x.ac = ac;
    x.valid = true;
    x.used = gen;
    return &x.table;
  }
};
}  // namespace

JpegStatus jpeg_decode_coefs(const uint8_t* data, size_t n, const JpegInfo& info, int16_t* coef, std::string& err) {
  thread_local std::unique_ptr<TableCache> cache;
  if (!cache) cache.reset(new TableCache());
  const HuffTable* dcp[kJpegMaxComp] = {};
  const HuffTable* acp[kJpegMaxComp] = {};
  ++cache->gen;
  for (int c = 0; c < info.ncomp; ++c) {
    dcp[c] = cache->get(info.dc[info.td[c]], false);
    acp[c] = dcp[c] ? cache->get(info.ac[info.ta[c]], true) : nullptr;
    if (!dcp[c] || !acp[c]) {
      err = "Failed to decode image: bad Huffman table";
      return JpegStatus::Corrupt;
    }
  }
  BitReader br{data + info.scan_begin, data + n};
  int pred[kJpegMaxComp] = {0, 0, 0};
  const bool single = info.ncomp == 1;
  const int64_t n_mcu = single ? (int64_t)info.comp[0].bw * info.comp[0].bh : (int64_t)info.mcux * info.mcuy;
  const int ri = info.restart_interval;
  int todo = ri;
  bool starved = false;
  for (int64_t m = 0; m < n_mcu; ++m) {
    if (ri) {
      if (todo == 0) {
        br.restart();
        pred[0] = pred[1] = pred[2] = 0;
        todo = ri;
        // a segment that starts right at another marker stays starved (libjpeg process_restart)
        starved = br.p + 1 < br.end && br.p[0] == 0xFF && br.p[1] != 0x00 && !(br.p[1] >= 0xD0 && br.p[1] <= 0xD7)
                      ? starved : false;
      }
      --todo;
    }
    if (starved) {  // insufficient data: zero blocks, predictions untouched (jdhuff.c decode_mcu)
      if (single) {
        std::memset(coef + m * 64, 0, 64 * sizeof(int16_t));
      } else {
        const int my = (int)(m / info.mcux), mx = (int)(m % info.mcux);
        for (int c = 0; c < info.ncomp; ++c) {
          const JpegCompDesc& d = info.comp[c];
          for (int v = 0; v < d.v; ++v)
            std::memset(coef + d.coef_off + (((int64_t)my * d.v + v) * d.bw + (int64_t)mx * d.h) * 64, 0,
                        (size_t)d.h * 64 * sizeof(int16_t));
        }
      }
      continue;
    }
    if (single) {
      if (!decode_block(br, *dcp[0], *acp[0], pred[0], coef + m * 64)) {
        err = "Failed to decode image: bad DC magnitude";
        return JpegStatus::Corrupt;
      }
      starved = br.starved();
      continue;
    }
    const int my = (int)(m / info.mcux), mx = (int)(m % info.mcux);
    for (int c = 0; c < info.ncomp; ++c) {
      const JpegCompDesc& d = info.comp[c];
      for (int v = 0; v < d.v; ++v) {
        int16_t* row = coef + d.coef_off + (((int64_t)my * d.v + v) * d.bw + (int64_t)mx * d.h) * 64;
        for (int h = 0; h < d.h; ++h) {
          if (!decode_block(br, *dcp[c], *acp[c], pred[c], row + h * 64)) {
            err = "Failed to decode image: bad DC magnitude";
            return JpegStatus::Corrupt;
          }
        }
      }
    }
    starved = br.starved();
  }
  if (br.truncated || br.overran()) {
    err = "Failed to decode image: image file is truncated";
    return JpegStatus::Corrupt;
  }
  return JpegStatus::Ok;
}

int64_t jpeg_total_blocks(const JpegInfo& info) {
  int64_t t = 0;
  for (int c = 0; c < info.ncomp; ++c) t += (int64_t)info.comp[c].bw * info.comp[c].bh;
  return t;
}

int64_t jpeg_compact_capacity(const JpegInfo& info) {
  const int64_t tb = jpeg_total_blocks(info);
  return ((tb * 12 + 15) & ~(int64_t)15) + tb * 128;
}

bool jpeg_compact_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("ARENA_JPEG_COMPACT");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

int64_t jpeg_payload_bytes(const JpegInfo& info) { return info.compact_bytes >= 0 ? info.compact_bytes : info.coef_count * 2; }

JpegStatus jpeg_decode_compact(const uint8_t* data, size_t n, JpegInfo& info, uint8_t* out, std::string& err) {
  thread_local std::unique_ptr<TableCache> cache;
  if (!cache) cache.reset(new TableCache());
  const HuffTable* dcp[kJpegMaxComp] = {};
  const HuffTable* acp[kJpegMaxComp] = {};
  ++cache->gen;
  for (int c = 0; c < info.ncomp; ++c) {
    dcp[c] = cache->get(info.dc[info.td[c]], false);
    acp[c] = dcp[c] ? cache->get(info.ac[info.ta[c]], true) : nullptr;
    if (!dcp[c] || !acp[c]) {
      err = "Failed to decode image: bad Huffman table";
      return JpegStatus::Corrupt;
    }
  }
  const int64_t tb = jpeg_total_blocks(info);
  uint64_t* masks = (uint64_t*)out;
  uint32_t* voff = (uint32_t*)(out + tb * 8);
  const int64_t val_at = (tb * 12 + 15) & ~(int64_t)15;
  int16_t* vals = (int16_t*)(out + val_at);
  int64_t nv = 0;
  BitReader br{data + info.scan_begin, data + n};
  int pred[kJpegMaxComp] = {0, 0, 0};
  const bool single = info.ncomp == 1;
  const int64_t n_mcu = single ? (int64_t)info.comp[0].bw * info.comp[0].bh : (int64_t)info.mcux * info.mcuy;
  const int ri = info.restart_interval;
  int todo = ri;
  bool starved = false;
  auto block = [&](int c, int64_t gb) -> bool {
    voff[gb] = (uint32_t)nv;
    if (starved) {  // insufficient data: an all-zero block, predictions untouched (jdhuff.c decode_mcu)
      masks[gb] = 0;
      return true;
    }
    return decode_block_compact(br, *dcp[c], *acp[c], pred[c], masks + gb, vals, nv);
  };
  for (int64_t m = 0; m < n_mcu; ++m) {
    if (ri) {
      if (todo == 0) {
        br.restart();
        pred[0] = pred[1] = pred[2] = 0;
        todo = ri;
        starved = br.p + 1 < br.end && br.p[0] == 0xFF && br.p[1] != 0x00 && !(br.p[1] >= 0xD0 && br.p[1] <= 0xD7)
                      ? starved : false;
      }
      --todo;
    }
    const bool was_starved = starved;
    if (single) {
      if (!block(0, m)) {
        err = "Failed to decode image: bad DC magnitude";
        return JpegStatus::Corrupt;
      }
    } else {
      const int my = (int)(m / info.mcux), mx = (int)(m % info.mcux);
      for (int c = 0; c < info.ncomp; ++c) {
        const JpegCompDesc& d = info.comp[c];
        for (int v = 0; v < d.v; ++v)
          for (int h = 0; h < d.h; ++h) {
            const int64_t gb = d.coef_off / 64 + ((int64_t)my * d.v + v) * d.bw + (int64_t)mx * d.h + h;
            if (!block(c, gb)) {
              err = "Failed to decode image: bad DC magnitude";
              return JpegStatus::Corrupt;
            }
          }
      }
    }
    if (!was_starved) starved = br.starved();
  }
  if (br.truncated || br.overran()) {
    err = "Failed to decode image: image file is truncated";
    return JpegStatus::Corrupt;
  }
  info.compact_bytes = val_at + nv * 2;
  info.cmask_off = 0;
  info.cvoff_off = tb * 8;
  info.cval_off = val_at;
  return JpegStatus::Ok;
}

void jpeg_compact_to_dense(const JpegInfo& info, const uint8_t* payload, int16_t* coef) {
  const int64_t tb = jpeg_total_blocks(info);
  const uint64_t* masks = (const uint64_t*)(payload + info.cmask_off);
  const uint32_t* voff = (const uint32_t*)(payload + info.cvoff_off);
  const int16_t* vals = (const int16_t*)(payload + info.cval_off);
  for (int64_t b = 0; b < tb; ++b) {
    int16_t* blk = coef + b * 64;
    std::memset(blk, 0, 64 * sizeof(int16_t));
    uint64_t m = masks[b];
    int64_t i = voff[b];
    while (m) {
      const int k = __builtin_ctzll(m);
      blk[kNatural[k]] = vals[i++];
      m &= m - 1;
    }
  }
}

const int16_t* jpeg_dense_coefs(const JpegInfo& info, const uint8_t* payload, std::vector<int16_t>& scratch) {
  if (info.compact_bytes < 0) return (const int16_t*)payload;
  scratch.resize((size_t)info.coef_count);
  jpeg_compact_to_dense(info, payload, scratch.data());
  return scratch.data();
}

void jpeg_coefs_to_rgb(const JpegInfo& info, const int16_t* coef, uint8_t* rgb) {
  using namespace jpegm;
  std::vector<uint8_t> planes((size_t)info.plane_bytes);
  for (int c = 0; c < info.ncomp; ++c) {
    const JpegCompDesc& d = info.comp[c];
    const int stride = d.bw * 8;
    for (int by = 0; by < d.bh; ++by) {
      for (int bx = 0; bx < d.bw; ++bx) {
        const int16_t* in = coef + d.coef_off + ((int64_t)by * d.bw + bx) * 64;
        int64_t ws[64];
        for (int col = 0; col < 8; ++col) {
          int64_t v[8], o[8];
          for (int r = 0; r < 8; ++r) v[r] = (int64_t)in[r * 8 + col] * info.qt[c][r * 8 + col];
          idct8<int64_t>(v, o, kPass1Shift);
          for (int r = 0; r < 8; ++r) ws[r * 8 + col] = o[r];
        }
        for (int r = 0; r < 8; ++r) {
          int64_t o[8];
          idct8<int64_t>(ws + r * 8, o, kPass2Shift);
          uint8_t* dst = planes.data() + d.plane_off + (int64_t)(by * 8 + r) * stride + bx * 8;
          for (int k = 0; k < 8; ++k) dst[k] = idct_sample<int64_t>(o[k]);
        }
      }
    }
  }
  const JpegCompDesc& Y = info.comp[0];
  const uint8_t* yp = planes.data() + Y.plane_off;
  const int ys = Y.bw * 8;
  for (int y = 0; y < info.height; ++y) {
    for (int x = 0; x < info.width; ++x) {
      uint8_t* o = rgb + ((int64_t)y * info.width + x) * 3;
      const int yy = yp[(int64_t)y * ys + x];
      if (info.layout == JPEG_GRAY) {
        o[0] = o[1] = o[2] = (uint8_t)yy;
        continue;
      }
      int cc[2];
      for (int k = 0; k < 2; ++k) {
        const JpegCompDesc& C = info.comp[1 + k];
        const uint8_t* cp = planes.data() + C.plane_off;
        const int cs = C.bw * 8;
        if (info.layout == JPEG_444) {
          cc[k] = cp[(int64_t)y * cs + x];
        } else if (info.layout == JPEG_422) {
          const int cx = x >> 1, xo = x & 1;
          const int nx = xo ? std::min(cx + 1, C.cw - 1) : std::max(cx - 1, 0);
          cc[k] = fancy_h2v1(cp[(int64_t)y * cs + cx], cp[(int64_t)y * cs + nx], xo);
        } else {
          const int cx = x >> 1, xo = x & 1, cy = y >> 1;
          const int nx = xo ? std::min(cx + 1, C.cw - 1) : std::max(cx - 1, 0);
          const int ny = (y & 1) ? std::min(cy + 1, C.ch - 1) : std::max(cy - 1, 0);
          cc[k] = fancy_h2v2(cp[(int64_t)cy * cs + cx], cp[(int64_t)cy * cs + nx], cp[(int64_t)ny * cs + cx],
                             cp[(int64_t)ny * cs + nx], xo);
        }
      }
      ycc_to_rgb(yy, cc[0], cc[1], o);
    }
  }
}

JpegDesc jpeg_device_desc(const JpegInfo& info, int64_t coef_base, int64_t plane_base, int64_t rgb_off) {
  JpegDesc d;
  std::memset(&d, 0, sizeof d);
  d.ncomp = info.ncomp;
  d.layout = info.layout;
  d.width = info.width;
  d.height = info.height;
  d.rgb_off = rgb_off;
  int64_t total = 0;
  for (int c = 0; c < info.ncomp; ++c) {
    d.comp[c] = info.comp[c];
    d.comp[c].coef_off = coef_base + info.comp[c].coef_off * 2;
    d.comp[c].plane_off = plane_base + info.comp[c].plane_off;
    total += (int64_t)info.comp[c].bw * info.comp[c].bh;
    std::memcpy(d.qt[c], info.qt[c], sizeof d.qt[c]);
  }
  d.total_blocks = (int32_t)total;
  if (info.compact_bytes >= 0) {  // compact payload at coef_base (jpeg_decode_compact)
    d.compact = 1;
    d.cmask_off = coef_base + info.cmask_off;
    d.cvoff_off = coef_base + info.cvoff_off;
    d.cval_off = coef_base + info.cval_off;
  }
  return d;
}

}  // namespace arena
