// Host entropy-decode throughput of the split JPEG decoder (csrc/runtime/jpeg_decode.cpp): parses each JPEG file
// given on the command line once, then times jpeg_decode_coefs into a reused buffer (the decode threads' steady
// state: pooled output buffers, no page faults).
// build: g++ -O3 -march=native -std=c++17 -Icsrc csrc/tests/jpeg_entropy_bench.cpp csrc/runtime/jpeg_decode.cpp
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "runtime/jpeg_decode.h"

int main(int argc, char** argv) {
  using namespace arena;
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    files.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  if (files.empty()) {
    std::fprintf(stderr, "usage: %s file.jpg...\n", argv[0]);
    return 2;
  }
  std::vector<JpegInfo> infos(files.size());
  std::vector<std::vector<int16_t>> out(files.size());
  for (size_t i = 0; i < files.size(); ++i) {
    std::string err;
    if (jpeg_parse((const uint8_t*)files[i].data(), files[i].size(), infos[i], err) != JpegStatus::Ok) {
      std::fprintf(stderr, "%s: %s\n", argv[i + 1], err.c_str());
      return 1;
    }
    out[i].resize((size_t)infos[i].coef_count);
  }
  // the fastest of `reps` passes over all files: the container's shared CPUs vary by +-15 % between runs
  const int reps = 40;
  double best = 1e30, bytes = 0;
  for (const std::string& f : files) bytes += (double)f.size();
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < files.size(); ++i) {
      std::string err;
      if (jpeg_decode_coefs((const uint8_t*)files[i].data(), files[i].size(), infos[i], out[i].data(), err) !=
          JpegStatus::Ok)
        return 1;
    }
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  std::printf("%.1f us per image, %.1f MB/s of compressed data (%zu files, best of %d passes)\n",
              best / files.size() * 1e6, bytes / best / 1e6, files.size(), reps);
  uint64_t h = 0;
  for (auto& v : out)
    for (int16_t c : v) h = h * 1000003u + (uint16_t)c;
  std::printf("checksum %016llx\n", (unsigned long long)h);
  return 0;
}
