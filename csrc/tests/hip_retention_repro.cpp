// HIP-only reproduction of the host-memory retention of round 5 (profiles/r5_serving/leak/README.md): the serving
// executor's per-upload coefficient DMAs grew the process by ~1.3 KB per upload.  No arena code: pinned buffers, a
// side copy stream, an event hand-off to rotating compute streams, a trivial kernel per batch.
//
//   hip_retention_repro MODE [batches] [uploads per batch] [bytes per upload]
//   MODE  side : one hipMemcpyAsync per upload on a shared side stream, event -> compute stream (round 5's layout)
//         pack : the uploads memcpy'd into one pinned staging buffer per slot, one copy per batch on the side
//                stream (the round-5 fix)
//         same : one copy per upload, issued on the batch's own compute stream (no side stream, no event)
//         pack_same     : pack, the one copy on the batch's compute stream (no side stream, no event)
//         pack_hostwait : pack on the side stream, the host waits for the copy (no cross-stream event wait)
//         pack_sync     : pack, and the side stream synchronized by the host every 64 batches
//         pack_rec      : pack, a fresh event per batch (created and destroyed) instead of the slot's
//
// Prints RSS (/proc/self/statm) every 500 batches and the growth per upload after a 500-batch warm-up.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ void consume(const uint8_t* p, size_t n, unsigned* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n / 4096 && p[i * 4096] == 0xA5) atomicAdd(out, 1u);
}

static double rss_mb() {
  long pages = 0, res = 0;
  FILE* f = std::fopen("/proc/self/statm", "r");
  if (f && std::fscanf(f, "%ld %ld", &pages, &res) != 2) res = 0;
  if (f) std::fclose(f);
  return res * (double)sysconf(_SC_PAGESIZE) / 1e6;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "side";
  const int batches = argc > 2 ? std::atoi(argv[2]) : 6000;
  const int per = argc > 3 ? std::atoi(argv[3]) : 32;
  const size_t bytes = argc > 4 ? (size_t)std::atoll(argv[4]) : (size_t)600 << 10;
  constexpr int kSlots = 4, kStreams = 3, kUploads = 256;  // 4 slots in flight over 3 compute streams
  std::vector<uint8_t*> up(kUploads);  // pooled pinned upload buffers (the decode threads' output)
  for (auto& p : up) { CK(hipHostMalloc(&p, bytes, hipHostMallocDefault)); std::memset(p, 1, bytes); }
  uint8_t *stage[kSlots], *dev[kSlots];
  hipEvent_t copied[kSlots], done[kSlots];
  for (int s = 0; s < kSlots; ++s) {
    CK(hipHostMalloc(&stage[s], bytes * per, hipHostMallocDefault));
    CK(hipMalloc(&dev[s], bytes * per));
    CK(hipEventCreateWithFlags(&copied[s], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&done[s], hipEventDisableTiming));
  }
  hipStream_t copy, comp[kStreams];
  CK(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking));
  for (auto& c : comp) CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  unsigned* hits;
  CK(hipMalloc(&hits, sizeof(unsigned)));
  double rss0 = 0;
  for (int b = 0; b < batches; ++b) {
    const int s = b % kSlots;
    hipStream_t cs = comp[b % kStreams];
    if (b >= kSlots) CK(hipEventSynchronize(done[s]));  // the slot's previous batch completed (collect)
    const bool pack = mode.rfind("pack", 0) == 0;
    const bool on_compute = mode == "same" || mode == "pack_same";
    if (pack) {
      for (int i = 0; i < per; ++i) std::memcpy(stage[s] + i * bytes, up[(b * per + i) % kUploads], bytes);
      CK(hipMemcpyAsync(dev[s], stage[s], bytes * per, hipMemcpyHostToDevice, on_compute ? cs : copy));
    } else {
      for (int i = 0; i < per; ++i)
        CK(hipMemcpyAsync(dev[s] + i * bytes, up[(b * per + i) % kUploads], bytes, hipMemcpyHostToDevice,
                          mode == "same" ? cs : copy));
    }
    if (mode == "pack_hostwait") {
      CK(hipEventRecord(copied[s], copy));
      CK(hipEventSynchronize(copied[s]));
    } else if (mode == "pack_rec") {
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      CK(hipEventRecord(ev, copy));
      CK(hipStreamWaitEvent(cs, ev, 0));
      CK(hipEventDestroy(ev));
    } else if (!on_compute) {
      CK(hipEventRecord(copied[s], copy));
      CK(hipStreamWaitEvent(cs, copied[s], 0));
    }
    if (mode == "pack_sync" && b % 64 == 63) CK(hipStreamSynchronize(copy));
    consume<<<(unsigned)((bytes * per / 4096 + 255) / 256), 256, 0, cs>>>(dev[s], bytes * per, hits);
    CK(hipEventRecord(done[s], cs));
    if (b == 500) rss0 = rss_mb();
    if (b % 500 == 0) std::printf("%s batch %d rss %.1f MB\n", mode.c_str(), b, rss_mb()), std::fflush(stdout);
  }
  CK(hipDeviceSynchronize());
  const double grow = rss_mb() - rss0;
  const double n_up = (double)(batches - 500) * per;
  std::printf("%s: %d batches x %d uploads of %zu B: RSS +%.1f MB after warm-up = %.3f KB per upload\n", mode.c_str(),
              batches, per, bytes, grow, grow * 1e3 / n_up);
  return 0;
}
