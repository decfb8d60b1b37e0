// Host decoder fuzz driver for the split JPEG decoder (csrc/runtime/jpeg_decode.cpp), built host-only under
// AddressSanitizer by tests/test_jpeg_native.py.  Uploads reach this parser straight from untrusted HTTP bodies
// (http_front.cpp decode threads, jpeg_ingest.cpp), so every table built from a segment must stay in bounds.
//
//   jpeg_fuzz <seed.jpg> [iterations]
//
// 1. Over-subscribed DHT code-length counts (too many short codes: bits[1] = 3, or bits[1] = 2 and bits[2] = 1),
//    with the total symbol count kept so the segment still parses: must be rejected as Corrupt.
// 2. Random byte flips / truncations / DHT count rewrites of the seed: any status, no memory error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "runtime/jpeg_decode.h"

using arena::JpegInfo;
using arena::JpegStatus;

namespace {

int compact_mismatches = 0;

// dense decode, and the compact decode (jpeg_decode_compact) of the same bytes: same status, and the compact
// payload expanded equals the dense blocks coefficient for coefficient
JpegStatus run(const std::vector<uint8_t>& d) {
  JpegInfo info;
  std::string err;
  JpegStatus st = arena::jpeg_parse(d.data(), d.size(), info, err, 64 << 20);
  if (st != JpegStatus::Ok) return st;
  std::vector<int16_t> coef((size_t)info.coef_count);
  st = arena::jpeg_decode_coefs(d.data(), d.size(), info, coef.data(), err);
  {
    JpegInfo ci = info;
    std::vector<uint8_t> payload((size_t)arena::jpeg_compact_capacity(ci));
    std::string cerr;
    const JpegStatus cs = arena::jpeg_decode_compact(d.data(), d.size(), ci, payload.data(), cerr);
    if (cs != st) {
      ++compact_mismatches;
    } else if (cs == JpegStatus::Ok) {
      if (ci.compact_bytes > (int64_t)payload.size()) ++compact_mismatches;
      std::vector<int16_t> dense((size_t)ci.coef_count);
      arena::jpeg_compact_to_dense(ci, payload.data(), dense.data());
      if (dense != coef) ++compact_mismatches;
    }
  }
  if (st != JpegStatus::Ok) return st;
  std::vector<uint8_t> rgb((size_t)info.width * info.height * 3);
  arena::jpeg_coefs_to_rgb(info, coef.data(), rgb.data());
  return st;
}

// offsets of the 16 code-length counts of every table in every DHT segment
std::vector<size_t> dht_tables(const std::vector<uint8_t>& d) {
  std::vector<size_t> out;
  size_t p = 2;
  while (p + 4 <= d.size() && d[p] == 0xFF) {
    const int m = d[p + 1];
    const size_t len = ((size_t)d[p + 2] << 8) | d[p + 3];
    if (m == 0xDA) break;
    if (m == 0xC4) {
      size_t q = p + 4;
      while (q + 17 <= p + 2 + len) {
        out.push_back(q + 1);
        int count = 0;
        for (int l = 0; l < 16; ++l) count += d[q + 1 + l];
        q += 17 + count;
      }
    }
    p += 2 + len;
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: jpeg_fuzz seed.jpg [iterations]\n");
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> seed;
  for (int c; (c = std::fgetc(f)) != EOF;) seed.push_back((uint8_t)c);
  std::fclose(f);
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (run(seed) != JpegStatus::Ok) {
    std::fprintf(stderr, "seed does not decode\n");
    return 1;
  }
  const std::vector<size_t> tables = dht_tables(seed);
  if (tables.empty()) {
    std::fprintf(stderr, "no DHT in the seed\n");
    return 1;
  }
  // 1. over-subscribed tables, symbol count unchanged
  int rejected = 0;
  for (size_t t : tables) {
    for (int pattern = 0; pattern < 2; ++pattern) {
      std::vector<uint8_t> d = seed;
      uint8_t* bits = &d[t];  // bits[0] = length 1
      int total = 0;
      for (int l = 0; l < 16; ++l) total += bits[l];
      std::memset(bits, 0, 16);
      int used = 0;
      if (pattern == 0) {
        bits[0] = 3;
        used = 3;
      } else {
        bits[0] = 2;
        bits[1] = 1;
        used = 3;
      }
      if (total < used) continue;
      bits[15] = (uint8_t)(total - used);  // the rest as 16-bit codes
      const JpegStatus st = run(d);
      if (st != JpegStatus::Corrupt) {
        std::fprintf(stderr, "over-subscribed DHT (table at %zu, pattern %d) not rejected: status %d\n", t, pattern,
                     (int)st);
        return 1;
      }
      ++rejected;
    }
  }
  // 2. random mutations
  std::mt19937 rng(1234);
  int counts[3] = {0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> d = seed;
    const int kind = it % 4;
    if (kind == 0) {
      for (int k = 0; k < 8; ++k) d[2 + rng() % (d.size() - 2)] = (uint8_t)rng();
    } else if (kind == 1) {
      d.resize(2 + rng() % (d.size() - 2));
    } else {
      const size_t t = tables[rng() % tables.size()];
      for (int k = 0; k < 3; ++k) d[t + rng() % 16] = (uint8_t)(rng() % 8);
      if (kind == 3) d[2 + rng() % (d.size() - 2)] = (uint8_t)rng();
    }
    counts[(int)run(d)]++;
  }
  if (compact_mismatches) {
    std::printf("jpeg_fuzz: %d compact decodes differ from the dense decode\n", compact_mismatches);
    return 1;
  }
  std::printf("jpeg_fuzz: ok (%d over-subscribed tables rejected; random: %d ok, %d unsupported, %d corrupt; compact "
              "== dense on all)\n",
              rejected, counts[0], counts[1], counts[2]);
  return 0;
}
