// Native pipeline executor: static op program -> per-bucket hipGraphs.
// See executor.h for the design; the op record layouts are documented in
// inference_arena_amd/engine/planner.py (the only producer of programs).
#include "executor.h"
#include "peer.h"

#include <pthread.h>
#include <sys/prctl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <stdexcept>
#include <string>

#include "../kernels/common.h"
#include "../kernels/jpeg_desc.h"
#include "jpeg_decode.h"
#include "trace.h"

namespace arena {

namespace {
float bits_to_float(int64_t v) {
  uint32_t u = (uint32_t)v;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
constexpr size_t kCtrlBytes = 256;
}  // namespace

Executor::Executor(const ExecutorConfig& cfg) : cfg_(cfg) {
  if (cfg_.max_batch <= 0 || cfg_.max_batch > 1024) throw std::runtime_error("Executor: max_batch out of range");
  if (cfg_.cand_cap > 16384) throw std::runtime_error("Executor: cand_cap > 16384");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  prepare_kernels();
  max_B_ = cfg_.max_batch;
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg_.device) == hipSuccess && khz > 0)
      wall_khz_ = (double)khz;
  }
  {
    const char* e = std::getenv("ARENA_DEBUG_SYNC");
    debug_sync_ = e != nullptr ? std::atoi(e) : 0;
    const char* at = std::getenv("ARENA_AUTOTUNE");
    autotune_ = at != nullptr ? std::atoi(at) : 1;
    const char* c = std::getenv("ARENA_COPY_MODE");
    // 0 (default): the input DMA on the shared copy stream, an event hands it to the batch's stream; 2: the DMA on
    // the batch's own stream (no overlap with that stream's previous batch: -0.8 % engine req/s,
    // profiles/r6_serving/leak).  Round 5's modes 1 (host wait) and 3 (per-slot copy streams) measured neutral or
    // worse and are retired (profiles/r5_serving/leak/copy_ab).
    copy_mode_ = c != nullptr && std::atoi(c) == 2 ? 2 : 0;
    const char* cc = std::getenv("ARENA_CONCURRENT");
    concurrent_ = cc != nullptr ? std::atoi(cc) : 1;
    if (debug_sync_) concurrent_ = 0;
    const char* ns = std::getenv("ARENA_SLOTS");
    n_slots_ = concurrent_ ? std::min(kMaxSlots, std::max(2, ns != nullptr ? std::atoi(ns) : 4)) : 2;
    const char* nc = std::getenv("ARENA_CONCURRENCY");
    n_streams_ = concurrent_ ? std::min(n_slots_, std::max(1, nc != nullptr ? std::atoi(nc) : 3)) : 1;
    // staggered launch: 0.25 of the ops is ~22 % of the fp32 program's device time; measured on 1x MI355X
    // (profiles/r6_stagger): engine req/s 9491 -> 10080 with the compact JPEG payload, 9707 -> 10105 dense
    const char* sg = std::getenv("ARENA_STAGGER");
    if (concurrent_ && n_streams_ > 1) {
      std::string spec = sg != nullptr ? sg : "0.25";
      for (size_t a = 0; a < spec.size();) {
        size_t e = spec.find(',', a);
        if (e == std::string::npos) e = spec.size();
        const double f = std::atof(spec.substr(a, e - a).c_str());
        if (f > 0.0 && f < 1.0 && (int)stagger_.size() < kMaxStaggerParts - 1) stagger_.push_back(f);
        a = e + 1;
      }
      std::sort(stagger_.begin(), stagger_.end());
    }
    // the waits apply to full batches only (live images >= ARENA_STAGGER_MIN_BATCH, default 32, or the whole
    // bucket): a device backlog shows as full batches, and below it a wait only adds latency (protocol_r6, 50
    // users: 6.8k req/s with every batch of >= 16 staggered, against 7.6k in round 5)
    const char* sm = std::getenv("ARENA_STAGGER_MIN_BATCH");
    stagger_min_batch_ = sm != nullptr ? std::max(1, std::atoi(sm)) : 32;
  }
  ARENA_HIP_CHECK(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
  ARENA_HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  streams_[0] = compute_;
  for (int i = 1; i < n_streams_; ++i) ARENA_HIP_CHECK(hipStreamCreateWithFlags(&streams_[i], hipStreamNonBlocking));
  for (int s = 0; s < n_slots_; ++s) {
    slots_[s].idx = s;
    slots_[s].stream = streams_[s % n_streams_];
  }
  alloc_slots();
  const int nthreads = std::max(1, cfg_.host_threads);
  for (int t = 0; t < nthreads; ++t) {
    workers_.emplace_back([this]() {
      pthread_setname_np(pthread_self(), "arena-pack");
      uint64_t seen = 0;
      for (;;) {
        std::vector<std::function<void()>>* jobs;
        {
          std::unique_lock<std::mutex> lk(pool_mu_);
          pool_cv_.wait(lk, [&] { return pool_stop_ || pool_gen_ != seen; });
          if (pool_stop_) return;
          seen = pool_gen_;
          jobs = pool_jobs_;
          if (jobs == nullptr) continue;
          ++pool_active_;
        }
        for (;;) {
          const int i = pool_next_.fetch_add(1);
          if (i >= (int)jobs->size()) break;
          (*jobs)[i]();
        }
        std::lock_guard<std::mutex> lk(pool_mu_);
        if (--pool_active_ == 0) pool_done_cv_.notify_all();
      }
    });
  }
}

Executor::~Executor() {
  {
    std::lock_guard<std::mutex> lk(pool_mu_);
    pool_stop_ = true;
  }
  pool_cv_.notify_all();
  for (auto& t : workers_) t.join();
  hipSetDevice(cfg_.device);
  for (int i = 0; i < n_streams_; ++i)
    if (streams_[i]) hipStreamSynchronize(streams_[i]);
  if (copy_) hipStreamSynchronize(copy_);
  for (auto& kv : buckets_) {
    for (int s = 0; s < n_slots_; ++s) destroy_graphs(kv.second, s);
    free_arenas(kv.second);
  }
  for (int i = 1; i < n_streams_; ++i)
    if (streams_[i]) hipStreamDestroy(streams_[i]);
  for (int s = 0; s < n_slots_; ++s) {
    Slot& sl = slots_[s];
    if (sl.d_in) hipFree(sl.d_in);
    if (sl.d_out) hipFree(sl.d_out);
    if (sl.sk_ws) hipFree(sl.sk_ws);
    if (sl.h_in) hipHostFree(sl.h_in);
    if (sl.h_out) hipHostFree(sl.h_out);
  }
  for (uint8_t* p : retired_h_in_) hipHostFree(p);
  retired_h_in_.clear();
  for (int s = 0; s < n_slots_; ++s) {
    Slot& sl = slots_[s];
    if (sl.copied) hipEventDestroy(sl.copied);
    if (sl.started) hipEventDestroy(sl.started);
    if (sl.done) hipEventDestroy(sl.done);
    if (sl.fork_ev) hipEventDestroy(sl.fork_ev);
    for (hipEvent_t& e : sl.phase)
      if (e) hipEventDestroy(e);
    for (int l = 0; l < kMaxLanes; ++l) {
      if (sl.lane_ev[l]) hipEventDestroy(sl.lane_ev[l]);
      if (sl.lane_stream[l]) hipStreamDestroy(sl.lane_stream[l]);
    }
  }
  if (d_weights_) hipFree(d_weights_);
  if (compute_) hipStreamDestroy(compute_);
  if (copy_) hipStreamDestroy(copy_);
}

// ---------------------------------------------------------------- layout
size_t Executor::jpeg_desc_off() const { return kCtrlBytes + align_up(sizeof(ImageMeta) * (size_t)max_B_, 256); }
size_t Executor::in_bytes_meta() const { return jpeg_desc_off() + align_up(sizeof(JpegDesc) * (size_t)max_B_, 256); }
size_t Executor::pool_cap() const {
  return align_up((size_t)cfg_.pool_bytes_per_image * (size_t)std::max(1, cfg_.pool_factor) * max_B_, 256);
}
size_t Executor::in_bytes_total() const { return in_bytes_meta() + pool_cap(); }
size_t Executor::out_off_det() const { return align_up(sizeof(int) * (size_t)max_B_, 256); }
size_t Executor::out_off_topk() const {
  return out_off_det() + align_up(sizeof(Detection) * (size_t)max_B_ * cfg_.max_det, 256);
}
size_t Executor::out_off_raw() const {
  return align_up(out_off_topk() + sizeof(TopkResult) * (size_t)max_B_ * cfg_.max_det, 256);
}
size_t Executor::out_off_xcrops() const { return align_up(out_off_raw() + (size_t)cfg_.raw_out_bytes * max_B_, 256); }
size_t Executor::out_off_stamps() const {
  return align_up(out_off_xcrops() + sizeof(CropRef) * (size_t)max_B_ * cfg_.max_det, 256);
}
size_t Executor::out_bytes_total() const { return out_off_stamps() + 4 * sizeof(uint64_t); }

void Executor::sync_slots() {
  for (int i = 0; i < n_streams_; ++i) ARENA_HIP_CHECK(hipStreamSynchronize(streams_[i]));
}

void Executor::free_arenas(Bucket& bk) {
  for (int s = 0; s < n_slots_; ++s) {
    if (bk.d_arena[s] == nullptr) continue;
    bool first = true;  // free each distinct allocation once (aliased when not concurrent)
    for (int t = 0; t < s; ++t) first &= bk.d_arena[t] != bk.d_arena[s];
    if (first) hipFree(bk.d_arena[s]);
  }
  for (int s = 0; s < kMaxSlots; ++s) bk.d_arena[s] = nullptr;
}

void Executor::alloc_slots() {
  for (int s = 0; s < n_slots_; ++s) {
    Slot& sl = slots_[s];
    // +256 B slack: the fused stem kernels fetch source image rows as aligned dwords, which may
    // run up to 3 bytes past the last image of a full staging pool
    ARENA_HIP_CHECK(hipMalloc(&sl.d_in, in_bytes_total() + 256));
    ARENA_HIP_CHECK(hipMalloc(&sl.d_out, out_bytes_total()));
    // split-K conv workspace (kF32X3GSK), one region per program lane: lanes run concurrently within a slot
    ARENA_HIP_CHECK(hipMalloc(&sl.sk_ws, (size_t)sk_lane_bytes() * (kMaxLanes + 1)));
    // pinned host staging: the meta block plus the host-packed inputs of one full batch at the nominal frame size.
    // Split-decoded JPEGs need only their coefficients staged here (about 2/3 of an RGB frame at 4:2:0), so
    // pool_factor's extra device room needs no host twin; a batch that needs more grows it on demand
    // (ensure_host_staging).
    sl.h_cap = in_bytes_meta() + align_up((size_t)cfg_.pool_bytes_per_image * max_B_, 256);
    ARENA_HIP_CHECK(hipHostMalloc(&sl.h_in, sl.h_cap, hipHostMallocDefault));
    ARENA_HIP_CHECK(hipHostMalloc(&sl.h_out, out_bytes_total(), hipHostMallocDefault));
    ARENA_HIP_CHECK(hipMemset(sl.d_in, 0, in_bytes_total()));
    ARENA_HIP_CHECK(hipMemset(sl.d_out, 0, out_bytes_total()));
    std::memset(sl.h_in, 0, in_bytes_meta());
    ARENA_HIP_CHECK(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
    for (hipEvent_t& e : sl.phase) ARENA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ARENA_HIP_CHECK(hipEventCreate(&sl.started));
    // ARENA_SYNC=blocking: collect() sleeps on the completion interrupt instead of polling the event (HIP's
    // default), which otherwise keeps a core busy per waiting thread for the whole device time of a batch
    static const bool blocking = [] {
      const char* e = std::getenv("ARENA_SYNC");
      return e != nullptr && std::string(e) == "blocking";
    }();
    ARENA_HIP_CHECK(hipEventCreateWithFlags(&sl.done, blocking ? hipEventBlockingSync : hipEventDefault));
  }
}

// Side streams of a slot, created when a lane bucket is captured on it (launch_graph runs lane segments there):
// programs without lanes never create them (no extra queues per process).
void Executor::ensure_lanes(Slot& sl) {
  if (sl.fork_ev != nullptr) return;
  bool lanes = false;
  for (const OpRecord& r : prog_) lanes |= r[kLaneField] > 0;
  if (!lanes) return;
  for (int l = 0; l < kMaxLanes; ++l) {
    ARENA_HIP_CHECK(hipStreamCreateWithFlags(&sl.lane_stream[l], hipStreamNonBlocking));
    ARENA_HIP_CHECK(hipEventCreateWithFlags(&sl.lane_ev[l], hipEventDisableTiming));
  }
  ARENA_HIP_CHECK(hipEventCreateWithFlags(&sl.fork_ev, hipEventDisableTiming));
}

void Executor::set_weights(const void* host, size_t bytes) {
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  if (d_weights_ != nullptr && bytes != weights_bytes_) {
    // captured graphs hold the weight pointer: only a same-size in-place update is allowed
    if (!buckets_.empty()) throw std::runtime_error("set_weights: size change after buckets were captured");
    ARENA_HIP_CHECK(hipFree(d_weights_));
    d_weights_ = nullptr;
  }
  if (d_weights_ == nullptr) ARENA_HIP_CHECK(hipMalloc(&d_weights_, bytes));
  sync_slots();
  ARENA_HIP_CHECK(hipMemcpy(d_weights_, host, bytes, hipMemcpyHostToDevice));
  weights_bytes_ = bytes;
}

void Executor::set_weights_device(const void* dev, size_t bytes) {
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  if (d_weights_ == nullptr || bytes != weights_bytes_)
    throw std::runtime_error("set_weights_device: only a same-size update of uploaded weights is supported");
  sync_slots();
  ARENA_HIP_CHECK(hipMemcpy(d_weights_, dev, bytes, hipMemcpyDeviceToDevice));
}

std::vector<uint8_t> Executor::weights_host() {
  std::vector<uint8_t> out(weights_bytes_);
  if (d_weights_ == nullptr || weights_bytes_ == 0) return out;
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  sync_slots();
  ARENA_HIP_CHECK(hipMemcpy(out.data(), d_weights_, weights_bytes_, hipMemcpyDeviceToHost));
  return out;
}

void Executor::set_program(const int64_t* ops, int n_ops, const int64_t* cls_ops, int n_cls_ops) {
  prog_.resize(n_ops);
  for (int i = 0; i < n_ops; ++i) std::memcpy(prog_[i].data(), ops + (size_t)i * kOpFields, sizeof(OpRecord));
  cls_prog_.resize(n_cls_ops);
  for (int i = 0; i < n_cls_ops; ++i)
    std::memcpy(cls_prog_[i].data(), cls_ops + (size_t)i * kOpFields, sizeof(OpRecord));
  has_topk_ = has_det_ = has_raw_ = has_stamps_ = false;
  for (const auto& r : prog_) {
    has_topk_ |= r[0] == OP_TOPK;
    has_stamps_ |= r[0] == OP_STAMP;
    has_det_ |= r[0] == OP_NMS || r[0] == OP_CROPPLAN;
    for (int f = 1; f < kOpFields; ++f) has_raw_ |= r[f] == BUF_RAWOUT && (r[0] == OP_YOLORAW || r[0] == OP_CONV);
  }
  if (has_raw_ && cfg_.raw_out_bytes <= 0) throw std::runtime_error("program exports raw outputs: raw_out_bytes = 0");
}

int Executor::crop_cap_for(int B) const { return std::max(cfg_.min_crop_cap, B * cfg_.crop_cap_per_image); }

std::vector<int> Executor::buckets() const {
  std::vector<int> r;
  for (auto& kv : buckets_) r.push_back(kv.first);
  return r;
}

uintptr_t Executor::arena_ptr(int B) const {
  auto it = buckets_.find(B);
  return it == buckets_.end() ? 0 : (uintptr_t)it->second.d_arena[0];
}

void Executor::read_arena(int B, int64_t offset, void* dst, size_t bytes) {
  auto it = buckets_.find(B);
  if (it == buckets_.end()) throw std::runtime_error("read_arena: unknown bucket");
  if (offset < 0 || offset + (int64_t)bytes > it->second.info.arena_bytes)
    throw std::runtime_error("read_arena: range outside the arena");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  sync_slots();
  ARENA_HIP_CHECK(hipMemcpy(dst, it->second.d_arena[it->second.last_slot] + offset, bytes, hipMemcpyDeviceToHost));
}

void Executor::add_bucket(int B, const int64_t* offsets, int n_buffers, int64_t arena_bytes,
                          const std::vector<int>* impl) {
  if (B <= 0 || B > max_B_) throw std::runtime_error("add_bucket: B outside (0, max_batch]");
  if (prog_.empty()) throw std::runtime_error("add_bucket: set_program first");
  if (d_weights_ == nullptr) throw std::runtime_error("add_bucket: set_weights first");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  Bucket& bk = buckets_[B];
  bk.info.B = B;
  bk.info.crop_cap = crop_cap_for(B);
  bk.info.offsets.assign(offsets, offsets + n_buffers);
  bk.info.arena_bytes = arena_bytes;
  sync_slots();
  free_arenas(bk);
  const size_t abytes = (size_t)std::max<int64_t>(arena_bytes, 256);
  // Every slot owns its arena, also when the slots are serialised on one stream (ARENA_CONCURRENT=0):
  // collect() of slot s may replay the classifier program for overflow crops after slot s+1's graph has
  // run, and that pass reads slot s's crop plan and activations.
  for (int s = 0; s < n_slots_; ++s) {
    ARENA_HIP_CHECK(hipMalloc(&bk.d_arena[s], abytes));
    ARENA_HIP_CHECK(hipMemset(bk.d_arena[s], 0, abytes));
  }
  bk.impl.assign(prog_.size(), 0);
  if (impl != nullptr) {
    if (impl->size() != prog_.size()) throw std::runtime_error("add_bucket: tuning table does not match the program");
    for (size_t i = 0; i < prog_.size(); ++i) {
      const int v = (*impl)[i];
      const bool f32 = prog_[i][kDtypeField] == 1;
      const bool ok = f32 ? (v >= 0 && v <= 2) || (v >= 10 && v < 10 + kF32Variants) ||
                                (v >= kF32X3 && v < kF32X3 + kF32X3Variants) || v == kF32Halo || v == kF32X3Halo ||
                                v == kF32X3HaloN3 || v == kF32X3HaloN2 || v == kF32Stream || v == kF32StreamN2 ||
                                v == kF32Fc || v == kF32StreamExact || v == kF32X3Halo16 || v == kF32X3Halo16N3 ||
                                v == kF32X3H16 || (v >= kF32X3G && v < kF32X3G + kF32X3GVariants) ||
                                (v >= kF32X3HG && v < kF32X3HG + kF32X3HGVariants) ||
                                (v >= kF32X3HGPw && v < kF32X3HGPw + kF32X3HGPwVariants) ||
                                (v >= kF32X3HGPwSmall && v < kF32X3HGPwSmall + kF32X3HGPwSmallVariants) ||
                                (v >= kF32X3HR && v < kF32X3HR + kF32X3HRVariants) ||
                                (v >= kF32X3HRPw && v < kF32X3HRPw + kF32X3HRPwVariants) ||
                                (v >= kF32X3GSK && v < kF32X3GSK + kF32X3GSKVariants)
                          : v >= 0 && v <= 3;
      if (!ok || (v != 0 && prog_[i][0] != OP_CONV)) throw std::runtime_error("add_bucket: bad tuning entry");
      bk.impl[i] = (int16_t)v;
    }
  } else if (autotune_) {
    autotune(bk);
  }
  for (int s = 0; s < n_slots_; ++s) capture(bk, s);
  if (debug_sync_ || std::getenv("ARENA_DEBUG_ALLOC")) {
    fprintf(stderr, "[arena alloc] bucket %d arena %p..%p (%lld B)\n", B, (void*)bk.d_arena[0],
            (void*)(bk.d_arena[0] + arena_bytes), (long long)arena_bytes);
    for (int s = 0; s < n_slots_; ++s)
      fprintf(stderr, "[arena alloc] slot %d in %p..%p out %p..%p\n", s, (void*)slots_[s].d_in,
              (void*)(slots_[s].d_in + in_bytes_total()), (void*)slots_[s].d_out,
              (void*)(slots_[s].d_out + out_bytes_total()));
    fprintf(stderr, "[arena alloc] weights %p..%p\n", (void*)d_weights_, (void*)(d_weights_ + weights_bytes_));
  }
}

// Per-bucket conv kernel selection: every conv op of the program is timed
// eagerly (bucket capacity, full live counts) with each kernel family — bf16:
// 1 direct MFMA, 2 tiled/LDS (pointwise fast path, 3x3 halo tiles, weight-
// stationary), 3 LDS-pipelined implicit GEMM; fp32: the default policy (0),
// the exact-fp32 LDS implicit-GEMM tile variants that won somewhere in the
// standalone sweep (profiles/r2_fp32_variants.md, impl 10 + v), the 3x3 halo
// kernel (impl 100) and the fp32-accurate triple-bf16-split kernels (impl
// 40 + v, 101) — and the fastest is recorded for the graph capture.  Costs
// ~100-300 ms per bucket; ARENA_AUTOTUNE=0 disables.  Production starts load
// the persisted table instead (engine/tuning.py), so the choice is fixed.
void Executor::autotune(Bucket& bk) {
  Slot& sl = slots_[0];
  Ctrl c{};
  c.n_images = bk.info.B;
  c.n_crops = bk.info.crop_cap;
  ARENA_HIP_CHECK(hipStreamSynchronize(compute_));
  ARENA_HIP_CHECK(hipMemcpy(sl.d_in, &c, sizeof(Ctrl), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  ARENA_HIP_CHECK(hipEventCreate(&e0));
  ARENA_HIP_CHECK(hipEventCreate(&e1));
  static const int kF32Candidates[] = {0,      12,     13,     14,     17,     19,     20,         21,
                                       23,     24,     kF32Halo, kF32X3, kF32X3 + 1, kF32X3 + 4, kF32X3 + 5,
                                       kF32X3 + 6, kF32X3 + 7, kF32X3 + 8, kF32X3Halo, kF32X3HaloN3,
                                       kF32X3HaloN2, kF32Stream, kF32StreamN2, kF32Fc, kF32StreamExact,
                                       kF32X3Halo16, kF32X3Halo16N3, kF32X3H16,
                                       // x3g variants that won a layer in tools/bench_x3g.py (impl 111 + v)
                                       kF32X3G + 5, kF32X3G + 6, kF32X3G + 7, kF32X3G + 9, kF32X3G + 15,
                                       kF32X3G + 16, kF32X3G + 17, kF32X3G + 19,
                                       // x3hg 3x3 stride-1 halo tiles that won a layer in tools/bench_x3g.py
                                       // (halo_x3g.hip; they throw on other convs)
                                       kF32X3HG + 0, kF32X3HG + 1, kF32X3HG + 2, kF32X3HG + 4, kF32X3HG + 6,
                                       kF32X3HG + 7, kF32X3HG + 8, kF32X3HG + 9, kF32X3HG + 10,
                                       // ... with the fused Detect-head 1x1 (the only kernels that take those ops)
                                       kF32X3HGPw + 0, kF32X3HGPw + 1, kF32X3HGPw + 2, kF32X3HGPw + 3,
                                       kF32X3HGPw + 4, kF32X3HGPw + 5, kF32X3HGPwSmall + 0, kF32X3HGPwSmall + 1,
                                       // x3hr: the same tiles with per-wave register weights (halo_x3g.hip)
                                       kF32X3HR + 0, kF32X3HR + 1, kF32X3HR + 2, kF32X3HR + 3, kF32X3HR + 4,
                                       kF32X3HR + 5, kF32X3HR + 6, kF32X3HR + 7, kF32X3HR + 8, kF32X3HR + 9,
                                       kF32X3HRPw + 0, kF32X3HRPw + 1, kF32X3HRPw + 2, kF32X3HRPw + 3,
                                       kF32X3HRPw + 4, kF32X3HRPw + 5,
                                       // split-K x3g (small grids: bucket 1 / 2); skipped where the workspace
                                       // is too small
                                       kF32X3GSK + 0, kF32X3GSK + 1, kF32X3GSK + 2, kF32X3GSK + 3, kF32X3GSK + 4,
                                       kF32X3GSK + 5, kF32X3GSK + 6, kF32X3GSK + 7, kF32X3GSK + 8};
  static const int kBf16Candidates[] = {1, 2, 3};
  for (size_t i = 0; i < prog_.size(); ++i) {
    if (prog_[i][0] != OP_CONV) continue;
    const bool f32 = prog_[i][kDtypeField] == 1;
    if (prog_[i][1] == BUF_POOL) {  // letterbox-source stem: one kernel implements it
      bk.impl[i] = kF32X3H16;
      continue;
    }
    if (!f32 && prog_[i][34] > 0) {  // fused pointwise epilogue: only the v3 halo-tile kernel implements it
      bk.impl[i] = 2;
      continue;
    }
    const int reps = f32 ? 5 : 3;
    std::vector<OpRecord> one(1, prog_[i]);
    float best = 1e30f;
    int best_impl = -1;
    const int* cand = f32 ? kF32Candidates : kBf16Candidates;
    const int n_cand = f32 ? (int)(sizeof(kF32Candidates) / sizeof(int)) : 3;
    for (int ci = 0; ci < n_cand; ++ci) {
      const int impl = cand[ci];
      // warm-up (instruction cache, L2); impl 0 reads bk.impl[i], still 0 here = the default policy.
      // A variant that does not apply to the shape (halo on a non-3x3 conv) throws before launching.
      try {
        enqueue_program(one, bk, sl, compute_, (int)i, impl);
      } catch (const std::runtime_error&) {
        continue;
      }
      ARENA_HIP_CHECK(hipEventRecord(e0, compute_));
      for (int k = 0; k < reps; ++k) enqueue_program(one, bk, sl, compute_, (int)i, impl);
      ARENA_HIP_CHECK(hipEventRecord(e1, compute_));
      ARENA_HIP_CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      ARENA_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (best_impl < 0 || ms < best * 0.97f) {  // a later candidate must win by 3% (stable choices)
        best = ms;
        best_impl = impl;
      }
    }
    bk.impl[i] = (int16_t)std::max(best_impl, 0);
    if (autotune_ > 1)
      fprintf(stderr, "[arena autotune] B=%d op %zu -> impl %d (%.1f us)\n", bk.info.B, i, best_impl,
              best * 1e3f / reps);
  }
  ARENA_HIP_CHECK(hipEventDestroy(e0));
  ARENA_HIP_CHECK(hipEventDestroy(e1));
  ARENA_HIP_CHECK(hipMemset(bk.d_arena[0], 0, std::max<int64_t>(bk.info.arena_bytes, 256)));
}

// Lanes pay off where one batch leaves most CUs idle (small buckets); for full batches the slots already overlap
// batches on the compute streams and side streams only add contention (profiles/r4lanes/).
static int lanes_max_batch() {
  static const int v = [] {
    const char* e = std::getenv("ARENA_LANES_MAX_BATCH");
    return e != nullptr ? std::atoi(e) : 2;
  }();
  return v;
}

bool Executor::lanes_for(const Bucket& bk) const {
  if (bk.info.B > lanes_max_batch()) return false;
  for (const OpRecord& r : prog_)
    if (r[kLaneField] >= 1 && r[kLaneField] <= kMaxLanes) return true;
  return false;
}

// bytes of one lane's split-K workspace (ARENA_SPLITK_WS_MB, default 16): the largest bucket-1 split (the 7x7x960
// -> 320 classifier conv over 16 crops, 8 splits) needs 8 MB
int64_t Executor::sk_lane_bytes() {
  static const int64_t v = [] {
    const char* e = std::getenv("ARENA_SPLITK_WS_MB");
    return (int64_t)std::max(1, e != nullptr ? std::atoi(e) : 16) << 20;
  }();
  return v;
}

void Executor::destroy_graphs(Bucket& bk, int s) {
  if (bk.graph[s]) hipGraphExecDestroy(bk.graph[s]);
  bk.graph[s] = nullptr;
  for (hipGraphExec_t g : bk.parts[s])
    if (g) hipGraphExecDestroy(g);
  bk.parts[s].clear();
  for (auto& sg : bk.segs[s])
    if (sg.g) hipGraphExecDestroy(sg.g);
  bk.segs[s].clear();
}

void Executor::capture(Bucket& bk, int s) {
  Slot& sl = slots_[s];
  hipStream_t st = sl.stream;
  // Validate the program eagerly once (launch errors surface here, not in the graph).
  ARENA_HIP_CHECK(hipStreamSynchronize(st));
  destroy_graphs(bk, s);
  // One capture of ops [a, b) on the slot's stream.  The result D2H copy is issued after the graph launch, not
  // captured: a captured device->pinned-host memcpy node faulted on ROCm 7.0 (torch's runtime) while the same
  // graph without it runs cleanly.
  auto capture_range = [&](size_t a, size_t b) {
    std::vector<OpRecord> part(prog_.begin() + a, prog_.begin() + b);
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    ARENA_HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    try {
      enqueue_program(part, bk, sl, st, (int)a);
    } catch (...) {
      hipStreamEndCapture(st, &g);
      if (g) hipGraphDestroy(g);
      throw;
    }
    ARENA_HIP_CHECK(hipStreamEndCapture(st, &g));
    ARENA_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    ARENA_HIP_CHECK(hipGraphDestroy(g));
    return ge;
  };
  if (!lanes_for(bk)) {
    // buckets of >= 16 are captured in parts (launch_graph decides per batch whether to wait between them)
    std::vector<size_t> cuts{0};
    if (bk.info.B >= 16)
      for (double f : stagger_) {
        const size_t k = (size_t)std::lround(f * (double)prog_.size());
        if (k > cuts.back() && k < prog_.size()) cuts.push_back(k);
      }
    if (cuts.size() > 1) {
      cuts.push_back(prog_.size());
      for (size_t i = 0; i + 1 < cuts.size(); ++i) bk.parts[s].push_back(capture_range(cuts[i], cuts[i + 1]));
    } else {
      bk.graph[s] = capture_range(0, prog_.size());
    }
    return;
  }
  // Lanes: every maximal run of ops with one lane value becomes a linear graph of its own; launch_graph() forks
  // the side streams (ensure_lanes) off the slot's stream at a lane run and joins them at the next lane-0 run.
  ensure_lanes(sl);
  auto lane_of = [&](size_t i) {
    const int64_t l = prog_[i][kLaneField];
    return l >= 1 && l <= kMaxLanes ? (int)l : 0;
  };
  for (size_t a = 0; a < prog_.size();) {
    size_t b = a + 1;
    while (b < prog_.size() && lane_of(b) == lane_of(a)) ++b;
    Bucket::Seg sg;
    sg.lane = lane_of(a);
    sg.g = capture_range(a, b);
    bk.segs[s].push_back(sg);
    a = b;
  }
}

void Executor::launch_graph(Bucket& bk, int s, hipStream_t st, int n_live) {
  if (bk.segs[s].empty()) {
    if (!bk.parts[s].empty()) {
      // and only while the device is saturated: two other batches still in flight
      int others = 0;
      for (int k = 0; k < n_slots_; ++k) others += k != s && slots_[k].busy ? 1 : 0;
      const bool gate = n_live < 0 || (n_live >= std::min(stagger_min_batch_, bk.info.B) && others >= 2);
      // part i (all but the last) after the previously launched batch finished its part i: at most one batch in
      // each gated part at a time, any number in the last (an event already passed, or re-recorded by a later
      // launch of that slot, costs nothing)
      const Slot* prev = gate && last_launched_ >= 0 && last_launched_ != s ? &slots_[last_launched_] : nullptr;
      const size_t np = bk.parts[s].size();
      for (size_t i = 0; i < np; ++i) {
        if (prev && i + 1 < np) ARENA_HIP_CHECK(hipStreamWaitEvent(st, prev->phase[i], 0));
        ARENA_HIP_CHECK(hipGraphLaunch(bk.parts[s][i], st));
        ARENA_HIP_CHECK(hipEventRecord(slots_[s].phase[i], st));
      }
      last_launched_ = s;
      return;
    }
    ARENA_HIP_CHECK(hipGraphLaunch(bk.graph[s], st));
    return;
  }
  Slot& sl = slots_[s];
  bool forked[kMaxLanes] = {};
  bool fork_recorded = false;
  auto join = [&]() {
    for (int l = 0; l < kMaxLanes; ++l)
      if (forked[l]) {
        ARENA_HIP_CHECK(hipEventRecord(sl.lane_ev[l], sl.lane_stream[l]));
        ARENA_HIP_CHECK(hipStreamWaitEvent(st, sl.lane_ev[l], 0));
        forked[l] = false;
      }
    fork_recorded = false;
  };
  for (const Bucket::Seg& sg : bk.segs[s]) {
    if (sg.lane == 0) {
      join();
      ARENA_HIP_CHECK(hipGraphLaunch(sg.g, st));
      continue;
    }
    const int l = sg.lane - 1;
    if (!forked[l]) {
      if (!fork_recorded) {  // everything before the lane region on the slot's stream
        ARENA_HIP_CHECK(hipEventRecord(sl.fork_ev, st));
        fork_recorded = true;
      }
      ARENA_HIP_CHECK(hipStreamWaitEvent(sl.lane_stream[l], sl.fork_ev, 0));
      forked[l] = true;
    }
    ARENA_HIP_CHECK(hipGraphLaunch(sg.g, sl.lane_stream[l]));
  }
  join();
}

uint8_t* Executor::resolve(Bucket& bk, Slot& sl, int64_t buf, int64_t coff, int eb) {
  uint8_t* base = nullptr;
  switch (buf) {
    case BUF_NONE: return nullptr;
    case BUF_CTRL: base = sl.d_in; break;
    case BUF_META: base = sl.d_in + kCtrlBytes; break;
    case BUF_POOL: base = sl.d_in + in_bytes_meta(); break;
    case BUF_DETCOUNT: base = sl.d_out; break;
    case BUF_DET: base = sl.d_out + out_off_det(); break;
    case BUF_TOPK: base = sl.d_out + out_off_topk(); break;
    case BUF_RAWOUT: base = sl.d_out + out_off_raw(); break;
    case BUF_XCROPS: base = sl.d_out + out_off_xcrops(); break;
    default:
      if (buf < 0 || buf >= (int64_t)bk.info.offsets.size())
        throw std::runtime_error("program references unknown buffer " + std::to_string(buf));
      base = bk.d_arena[sl.idx] + bk.info.offsets[buf];
  }
  return base + coff * eb;
}

void Executor::enqueue_program(const std::vector<OpRecord>& prog, Bucket& bk, Slot& sl, hipStream_t s_main,
                               int op_offset, int force_impl) {
  Ctrl* ctrl = (Ctrl*)resolve(bk, sl, BUF_CTRL, 0, 1);
  const ImageMeta* meta = (const ImageMeta*)resolve(bk, sl, BUF_META, 0, 1);
  const uint8_t* pool = resolve(bk, sl, BUF_POOL, 0, 1);
  const int B = bk.info.B, CC = bk.info.crop_cap;
  auto batch = [&](int64_t kind) { return kind == BATCH_CROPS ? CC : B; };
  auto bdev = [&](int64_t kind) -> const int* { return kind == BATCH_CROPS ? &ctrl->n_crops : &ctrl->n_images; };
  const uint8_t* W = d_weights_;

  // Lane ops (kLaneField) run in program order here: the lanes' side streams are driven by launch_graph() over
  // per-lane captured segments, not by forking inside one capture.
  for (size_t oi = 0; oi < prog.size(); ++oi) {
    const OpRecord& r = prog[oi];
    hipStream_t s = s_main;
    // field 47: activation precision of the op (0 bf16, 1 exact fp32; planner.OP_DTYPE_FIELD)
    const bool f32 = r[kDtypeField] == 1;
    const int eb = f32 ? 4 : 2;
    switch (r[0]) {
      case OP_CONV: {
        ConvParams p{};
        const size_t gi = (size_t)op_offset + oi;
        p.impl = force_impl ? force_impl : (gi < bk.impl.size() ? bk.impl[gi] : 0);
        p.x = resolve(bk, sl, r[1], r[2], eb);
        p.xs = (int)r[3];
        p.H = (int)r[4];
        p.W = (int)r[5];
        p.Cin = (int)r[6];
        p.w = W + r[7];
        p.Kpad = (int)r[8];
        p.bias = (const float*)(W + r[9]);
        p.f32out = (int)r[29];
        p.y = resolve(bk, sl, r[10], r[11], p.f32out ? 4 : eb);
        p.ys = (int)r[12];
        p.Ho = (int)r[13];
        p.Wo = (int)r[14];
        p.Cout = (int)r[15];
        p.Cout_pad = (int)r[16];
        p.KH = (int)r[17];
        p.KW = (int)r[18];
        p.stride = (int)r[19];
        p.pad_t = (int)r[20];
        p.pad_l = (int)r[21];
        p.res = resolve(bk, sl, r[22], r[23], eb);
        p.rs = (int)r[24];
        p.y2 = resolve(bk, sl, r[25], r[26], eb);
        p.y2s = (int)r[27];
        p.act = (int)r[28];
        p.B = batch(r[30]);
        p.bdev = bdev(r[30]);
        if (r[41] != 0) p.w3 = W + r[40];  // fp32: pre-split bf16 weight planes for the x3g kernels
        {
          const int64_t ln = r[kLaneField];
          const int li = ln >= 1 && ln <= kMaxLanes ? (int)ln : 0;
          p.sk_ws = (float*)((uint8_t*)sl.sk_ws + (size_t)li * sk_lane_bytes());
          p.sk_ws_bytes = sk_lane_bytes();
        }
        if (r[1] == BUF_POOL) {  // the stem conv samples the letterboxed images itself (fp32 x3-h16 kernel)
          if (!f32 || r[30] != 0) throw std::runtime_error("executor: letterbox-source conv must be fp32 over images");
          p.x = nullptr;
          p.lb_pool = pool;
          p.lb_meta = meta;
          p.impl = kF32X3H16;
        }
        if (r[34] > 0) {  // fused pointwise epilogue (Detect head 3x3 -> 1x1)
          p.pw_w = W + r[31];
          p.pw_kpad = (int)r[32];
          p.pw_bias = (const float*)(W + r[33]);
          p.pw_cout = (int)r[34];
          p.pw_y = resolve(bk, sl, r[36], r[37], eb);
          p.pw_ys = (int)r[38];
          p.pw_act = (int)r[39];
          if (!f32) p.impl = 2;  // bf16: the v3 halo-tile kernel; fp32: the tuned x3hg-pw variant
        }
        if (f32)
          conv2d_f32(p, s);
        else
          conv2d(p, s);
        break;
      }
      case OP_DWCONV: {
        DwParams p{};
        p.x = resolve(bk, sl, r[1], r[2], eb);
        p.xs = (int)r[3];
        p.H = (int)r[4];
        p.W = (int)r[5];
        p.C = (int)r[6];
        p.w = W + r[7];
        p.bias = (const float*)(W + r[8]);
        p.y = resolve(bk, sl, r[9], r[10], eb);
        p.ys = (int)r[11];
        p.Ho = (int)r[12];
        p.Wo = (int)r[13];
        p.stride = (int)r[14];
        p.act = (int)r[15];
        p.B = batch(r[16]);
        p.bdev = bdev(r[16]);
        if (f32)
          dwconv3x3_f32(p, s);
        else
          dwconv3x3(p, s);
        break;
      }
      case OP_IRBLOCK: {
        IrParams p{};
        p.x = resolve(bk, sl, r[1], r[2], eb);
        p.x_cs = (int)r[3];
        p.H = (int)r[4];
        p.W = (int)r[5];
        p.inp = (int)r[6];
        p.inp_pad = (int)r[7];
        p.hid_pad = (int)r[8];
        p.oup = (int)r[9];
        p.oup_pad = (int)r[10];
        p.stride = (int)r[11];
        p.expand = (int)r[12];
        p.res = (int)r[13];
        p.we = W + r[14];
        p.be = (const float*)(W + r[15]);
        p.wd = W + r[16];
        p.bd = (const float*)(W + r[17]);
        p.wp = W + r[18];
        p.bp = (const float*)(W + r[19]);
        p.y = resolve(bk, sl, r[20], r[21], eb);
        p.y_cs = (int)r[22];
        p.Ho = (int)r[23];
        p.Wo = (int)r[24];
        p.B = batch(r[25]);
        p.bdev = bdev(r[25]);
        p.x3w = (int)r[26];
        p.x_parts = (int)r[27];
        p.y_parts = (int)r[28];
        if (!f32 && (p.x_parts > 1 || p.y_parts > 1))
          throw std::runtime_error("executor: partial-sum ir_block tensors are fp32-only");
        p.stem = (int)r[31];
        if (p.stem) {  // fp32 classifier front end: crop gather + stem conv feed the block (ir_f32.hip)
          p.st_pool = pool;
          p.st_meta = meta;
          p.st_crops = (const CropRef*)resolve(bk, sl, r[32], 0, 1);
          p.st_ctrl = ctrl;
          p.st_S = (int)r[33];
          for (int c = 0; c < 3; ++c) {
            p.st_mean[c] = bits_to_float(r[34 + c]);
            p.st_inv_std[c] = bits_to_float(r[37 + c]);
          }
          p.st_w = (const float*)(W + r[40]);
          p.st_b = (const float*)(W + r[41]);
        }
        if (f32)
          ir_block_f32(p, s);
        else
          ir_block(p, s);
        break;
      }
      case OP_SPPF: {
        SppfParams p{};
        p.buf = resolve(bk, sl, r[1], r[2], eb);
        p.xs = (int)r[3];
        p.H = (int)r[4];
        p.W = (int)r[5];
        p.C = (int)r[6];
        p.B = batch(r[7]);
        p.bdev = bdev(r[7]);
        if (f32)
          sppf_pool_f32(p, s);
        else
          sppf_pool(p, s);
        break;
      }
      case OP_LETTERBOX: {
        LetterboxParams p{};
        p.pool = pool;
        p.meta = meta;
        p.ctrl = ctrl;
        p.out = resolve(bk, sl, r[1], 0, eb);
        p.B = B;
        p.T = (int)r[2];
        p.f32 = f32;
        letterbox_s2d(p, s);
        break;
      }
      case OP_STAMP: {
        if (r[1] < 0 || r[1] >= 4) throw std::runtime_error("OP_STAMP: stamp index out of range");
        stamp(sl.d_out + out_off_stamps() + sizeof(uint64_t) * (size_t)r[1], s);
        break;
      }
      case OP_ZERO: {
        uint8_t* ptr = resolve(bk, sl, r[1], 0, 1);
        const size_t bytes = (size_t)r[2] * batch(r[3]);
        zero_fill(ptr, bytes, s);
        break;
      }
      case OP_DECODE: {
        DecodeParams p{};
        for (int l = 0; l < 3; ++l) {
          p.head[l] = resolve(bk, sl, r[1 + 4 * l], r[2 + 4 * l], eb);
          p.xs[l] = (int)r[3 + 4 * l];
          p.hw[l] = (int)r[4 + 4 * l];
          p.stride[l] = (float)r[13 + l];
        }
        p.cand = (Candidate*)resolve(bk, sl, r[16], 0, 1);
        p.cand_count = (int*)resolve(bk, sl, r[17], 0, 1);
        p.conf_thr = bits_to_float(r[18]);
        p.cand_cap = cfg_.cand_cap;
        p.B = B;
        p.ctrl = ctrl;
        p.f32 = f32;
        detect_decode(p, s);
        break;
      }
      case OP_NMS: {
        NmsParams p{};
        p.cand = (const Candidate*)resolve(bk, sl, r[1], 0, 1);
        p.cand_count = (const int*)resolve(bk, sl, r[2], 0, 1);
        p.cand_cap = cfg_.cand_cap;
        p.meta = meta;
        p.B = B;
        p.det = (Detection*)resolve(bk, sl, r[3], 0, 1);
        p.det_count = (int*)resolve(bk, sl, r[4], 0, 1);
        p.max_det = cfg_.max_det;
        p.iou_thr = bits_to_float(r[5]);
        p.ctrl = ctrl;
        nms(p, s);
        break;
      }
      case OP_CROPPLAN: {
        CropPlanParams p{};
        p.det = (Detection*)resolve(bk, sl, r[1], 0, 1);
        p.det_count = (int*)resolve(bk, sl, r[2], 0, 1);
        p.max_det = cfg_.max_det;
        p.meta = meta;
        p.B = B;
        p.crops = (CropRef*)resolve(bk, sl, r[3], 0, 1);
        p.ctrl = ctrl;
        p.crop_cap = CC;
        p.whole = (int)r[4];
        crop_plan(p, s);
        break;
      }
      case OP_CROPGATHER: {
        CropGatherParams p{};
        p.pool = pool;
        p.meta = meta;
        p.crops = (const CropRef*)resolve(bk, sl, r[1], 0, 1);
        p.ctrl = ctrl;
        p.out = resolve(bk, sl, r[2], 0, eb);
        p.f32 = f32;
        p.cap = CC;
        p.S = (int)r[3];
        for (int c = 0; c < 3; ++c) {
          p.mean[c] = bits_to_float(r[4 + c]);
          p.inv_std[c] = bits_to_float(r[7 + c]);
        }
        crop_gather_s2d(p, s);
        break;
      }
      case OP_C3FUSED: {
        C3Params p{};
        p.x = resolve(bk, sl, r[1], r[2], eb);
        p.xs = (int)r[3];
        p.H = (int)r[4];
        p.W = (int)r[5];
        p.C1 = (int)r[6];
        p.CH = (int)r[7];
        p.NB = (int)r[8];
        p.res = (int)r[9];
        p.w12 = W + r[10];
        p.b12 = (const float*)(W + r[11]);
        for (int k = 0; k < 2; ++k) {
          p.wb1[k] = W + r[12 + 4 * k];
          p.bb1[k] = (const float*)(W + r[13 + 4 * k]);
          p.wb2[k] = W + r[14 + 4 * k];
          p.bb2[k] = (const float*)(W + r[15 + 4 * k]);
        }
        p.w3 = W + r[20];
        p.b3 = (const float*)(W + r[21]);
        p.y = resolve(bk, sl, r[22], r[23], eb);
        p.ys = (int)r[24];
        p.B = batch(r[25]);
        p.bdev = bdev(r[25]);
        if (f32)
          c3_x3(p, s);  // fp32-accurate form over pre-split weights (c3_x3.hip)
        else
          c3_fused(p, s);
        break;
      }
      case OP_STEMFUSED: {
        StemFusedParams p{};
        p.src = (int)r[1];
        p.y = resolve(bk, sl, r[2], r[3], eb);
        p.ys = (int)r[4];
        p.S = (int)r[5];
        p.w = W + r[6];
        p.Kpad = (int)r[7];
        p.bias = (const float*)(W + r[8]);
        p.Cout = (int)r[9];
        p.act = (int)r[10];
        p.crops = p.src == 1 ? (const CropRef*)resolve(bk, sl, r[11], 0, 1) : nullptr;
        for (int c = 0; c < 3; ++c) {
          p.mean[c] = bits_to_float(r[12 + c]);
          p.inv_std[c] = bits_to_float(r[15 + c]);
        }
        p.cap = batch(r[18]);
        p.KS = (int)r[19];
        if (r[20]) {  // second conv fused: the destination is its output, the stem output stays in LDS
          p.w2 = W + r[21];
          p.Kpad2 = (int)r[22];
          p.bias2 = (const float*)(W + r[23]);
          p.Cout2 = (int)r[24];
          p.act2 = (int)r[25];
          p.y2 = p.y;
          p.y2s = p.ys;
          p.y = nullptr;
        }
        if (r[26]) {  // first inverted residual fused: the destination is its output
          p.ir_wd = W + r[27];
          p.ir_bd = (const float*)(W + r[28]);
          p.ir_wp = W + r[29];
          p.ir_bp = (const float*)(W + r[30]);
          p.ir_y = p.y;
          p.ir_ys = p.ys;
          p.y = nullptr;
        }
        p.pool = pool;
        p.meta = meta;
        p.ctrl = ctrl;
        if (f32)
          stem_s2_f32(p, s);  // fp32: letterbox + stem + 3x3 s2 conv (the only fp32 stem_fused form)
        else
          stem_fused(p, s);
        break;
      }
      case OP_HEADPOOL: {
        HeadPoolParams p{};
        p.x = resolve(bk, sl, r[1], r[2], eb);
        p.xs = (int)r[3];
        p.HW = (int)r[4];
        p.K = (int)r[5];
        p.w = W + r[6];
        p.Kpad = (int)r[7];
        p.bias = (const float*)(W + r[8]);
        p.N = (int)r[9];
        p.Npad = (int)r[10];
        p.y = resolve(bk, sl, r[11], r[12], eb);
        p.ys = (int)r[13];
        p.act = (int)r[14];
        p.B = batch(r[15]);
        p.bdev = bdev(r[15]);
        if (f32)
          head_pool_f32(p, s);
        else
          head_pool(p, s);
        break;
      }
      case OP_AVGPOOL: {
        AvgPoolParams p{};
        p.x = resolve(bk, sl, r[1], 0, eb);
        p.HW = (int)r[2];
        p.C = (int)r[3];
        p.y = resolve(bk, sl, r[4], 0, eb);
        p.f32 = f32;
        p.B = batch(r[5]);
        p.bdev = bdev(r[5]);
        global_avgpool(p, s);
        break;
      }
      case OP_TOPK: {
        TopkParams p{};
        p.logits = (const float*)resolve(bk, sl, r[1], 0, 4);
        p.N = (int)r[2];
        p.ld = (int)r[3];
        p.out = (TopkResult*)resolve(bk, sl, r[4], 0, 1);
        p.B = CC;
        p.ctrl = ctrl;
        topk_softmax(p, s);
        break;
      }
      case OP_TENSORIN: {
        TensorInParams p{};
        p.pool = pool;
        p.meta = meta;
        p.ctrl = ctrl;
        p.out = resolve(bk, sl, r[1], 0, eb);
        p.B = B;
        p.S = (int)r[2];
        p.f32 = f32;
        tensor_in_s2d(p, s);
        break;
      }
      case OP_YOLORAW: {
        YoloRawParams p{};
        for (int l = 0; l < 3; ++l) {
          p.head[l] = resolve(bk, sl, r[1 + 4 * l], r[2 + 4 * l], eb);
          p.xs[l] = (int)r[3 + 4 * l];
          p.hw[l] = (int)r[4 + 4 * l];
          p.stride[l] = (float)r[13 + l];
        }
        p.B = B;
        p.out = resolve(bk, sl, r[16], 0, 1);
        p.out_stride = (size_t)cfg_.raw_out_bytes;
        p.ctrl = ctrl;
        p.f32 = f32;
        yolo_raw(p, s);
        break;
      }
      default:
        throw std::runtime_error("unknown op type " + std::to_string(r[0]));
    }
    ARENA_HIP_CHECK(hipGetLastError());
  }
}

// ---------------------------------------------------------------- host packing
void Executor::parallel_copy(std::vector<std::function<void()>>& jobs) {
  if (jobs.empty()) return;
  if (jobs.size() == 1 || workers_.empty()) {
    for (auto& j : jobs) j();
    return;
  }
  std::unique_lock<std::mutex> lk(pool_mu_);
  pool_jobs_ = &jobs;
  pool_next_ = 0;
  ++pool_gen_;
  pool_cv_.notify_all();
  lk.unlock();
  // the caller helps; workers that join late find the counter exhausted
  for (;;) {
    const int i = pool_next_.fetch_add(1);
    if (i >= (int)jobs.size()) break;
    jobs[i]();
  }
  lk.lock();
  pool_jobs_ = nullptr;  // no worker can pick this generation up any more
  pool_done_cv_.wait(lk, [&] { return pool_active_ == 0; });
}

int Executor::pick_bucket(int n) const {
  for (auto& kv : buckets_)
    if (kv.first >= n) return kv.first;
  return -1;
}

void Executor::enqueue_results_d2h(Bucket& bk, Slot& sl, int n) {
  size_t d2h = out_off_topk();
  if (has_topk_) d2h += sizeof(TopkResult) * (size_t)bk.info.crop_cap;
  ARENA_HIP_CHECK(hipMemcpyAsync(sl.h_out, sl.d_out, d2h, hipMemcpyDeviceToHost, sl.stream));
  if (has_stamps_)
    ARENA_HIP_CHECK(hipMemcpyAsync(sl.h_out + out_off_stamps(), sl.d_out + out_off_stamps(), 4 * sizeof(uint64_t),
                                   hipMemcpyDeviceToHost, sl.stream));
  if (has_raw_)
    ARENA_HIP_CHECK(hipMemcpyAsync(sl.h_out + out_off_raw(), sl.d_out + out_off_raw(), (size_t)cfg_.raw_out_bytes * n,
                                   hipMemcpyDeviceToHost, sl.stream));
}

int Executor::submit(const std::vector<InputImage>& imgs) {
  trace::Range tr("arena.submit");
  std::lock_guard<std::mutex> lk(mu_);
  const int n = (int)imgs.size();
  if (n <= 0) throw std::runtime_error("submit: empty batch");
  const int B = pick_bucket(n);
  if (B < 0) throw std::runtime_error("submit: batch larger than the largest bucket");
  const int s = next_slot_;
  Slot& sl = slots_[s];
  if (sl.busy) throw std::runtime_error("submit: every staging slot is in flight; collect() first");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  // Batches go round-robin over the compute streams: batch q runs on stream q % n_streams_, behind
  // batch q - n_streams_, so at most n_streams_ graphs execute at once while the staging (pack + H2D)
  // of the next n_slots_ - n_streams_ batches proceeds.
  sl.stream = streams_[seq_++ % n_streams_];
  // The slot's previous graph has been collected; its input copy was consumed.
  // Pool layout of the batch: host-packed inputs (RGB frames, tensors) first, so one H2D of the slot's
  // [ctrl | meta | JPEG descriptors | packed inputs] covers them (the JPEG coefficients packed after them);
  // then per split-decoded JPEG its RGB destination and reconstruction planes.  Everything is validated before the first copy is queued.
  const size_t cap = pool_cap();
  // Split-decoded JPEGs' coefficients are copied on the host into the slot's pinned staging, right after the packed
  // frames, and go to the device in the batch's one DMA.  (Round 5's alternative, one DMA per upload straight from
  // its pooled buffer, made HIP retain ~1.3 KB of host memory per upload: profiles/r5_serving/leak/README.md.)
  {
    // host bytes of the packed (non-JPEG) inputs: grow the slot's pinned staging if this batch needs more (the
    // slot is idle: its previous H2D completed before it was collected)
    size_t need = 0;
    for (int i = 0; i < n; ++i)
      if (imgs[i].jpeg == nullptr)
        need = align_up(need + (imgs[i].bytes > 0 ? (size_t)imgs[i].bytes : (size_t)imgs[i].h * imgs[i].w * 3), 256);
    // the JPEGs' coefficients follow them in the same DMA (layout below)
    for (int i = 0; i < n; ++i)
      if (imgs[i].jpeg != nullptr) need = align_up(need + (size_t)jpeg_payload_bytes(*imgs[i].jpeg), 256);
    if (need > cap) throw std::runtime_error("submit: batch exceeds the staging pool");
    if (in_bytes_meta() + need > sl.h_cap) {
      uint8_t* grown = nullptr;
      const size_t want = in_bytes_meta() + std::max(need, std::min(cap, 2 * (sl.h_cap - in_bytes_meta())));
      ARENA_HIP_CHECK(hipHostMalloc(&grown, want, hipHostMallocDefault));
      std::memcpy(grown, sl.h_in, in_bytes_meta());
      // hipHostFree may synchronise the device, which would stall the other slots' batches: the outgrown buffer
      // is released with the executor (the doubling bounds all retired buffers by the final size)
      retired_h_in_.push_back(sl.h_in);
      ++staging_growths_;
      sl.h_in = grown;
      sl.h_cap = want;
    }
  }
  ImageMeta* meta = (ImageMeta*)(sl.h_in + kCtrlBytes);
  JpegDesc* jdesc = (JpegDesc*)(sl.h_in + jpeg_desc_off());
  uint8_t* pool = sl.h_in + in_bytes_meta();
  size_t off = 0;
  std::vector<std::function<void()>> jobs;
  const int T = cfg_.det_size;
  auto set_meta = [&](int i, const InputImage& im, size_t at) {
    ImageMeta& m = meta[i];
    m.offset = (int64_t)at;
    m.h = im.h;
    m.w = im.w;
    const double sc = std::min((double)T / im.h, (double)T / im.w);
    m.new_w = (int)(im.w * sc);
    m.new_h = (int)(im.h * sc);
    m.pad_w = (T - m.new_w) / 2;
    m.pad_h = (T - m.new_h) / 2;
    m.scale = (float)sc;
  };
  for (int i = 0; i < n; ++i) {
    const InputImage& im = imgs[i];
    if (im.h <= 0 || im.w <= 0) throw std::runtime_error("submit: empty image");
    if (im.jpeg != nullptr) continue;
    const size_t bytes = im.bytes > 0 ? (size_t)im.bytes : (size_t)im.h * im.w * 3;
    if (off + bytes > cap) throw std::runtime_error("submit: batch exceeds the staging pool");
    set_meta(i, im, off);
    // split large images into 1 MiB copy jobs
    const size_t chunk = 1 << 20;
    for (size_t c = 0; c < bytes; c += chunk) {
      const size_t len = std::min(chunk, bytes - c);
      uint8_t* dst = pool + off + c;
      const uint8_t* src = im.data + c;
      jobs.emplace_back([dst, src, len]() { std::memcpy(dst, src, len); });
    }
    off = align_up(off + bytes, 256);
  }
  size_t packed_end = off;
  int nj = 0, max_blocks = 0;
  int64_t max_pix = 0;
  // packed coefficients sit contiguously right after the host-packed inputs, inside the one staging DMA
  std::vector<size_t> coef_at(n, 0);
  {
    for (int i = 0; i < n; ++i) {
      const InputImage& im = imgs[i];
      if (im.jpeg == nullptr) continue;
      const size_t len = (size_t)jpeg_payload_bytes(*im.jpeg);  // compact or dense coefficients
      if (off + len > cap) throw std::runtime_error("submit: batch exceeds the staging pool");
      coef_at[i] = off;
      jobs.emplace_back([dst = pool + off, src = im.data, len]() { std::memcpy(dst, src, len); });
      off = align_up(off + len, 256);
    }
    packed_end = off;
  }
  for (int i = 0; i < n; ++i) {
    const InputImage& im = imgs[i];
    if (im.jpeg == nullptr) continue;
    const JpegInfo& ji = *im.jpeg;
    if (ji.width != im.w || ji.height != im.h) throw std::runtime_error("submit: JPEG geometry mismatch");
    const size_t rgb = off, coef = coef_at[i];
    const size_t planes =
        align_up(rgb + (size_t)im.h * im.w * 3, 256);
    const size_t end = align_up(planes + (size_t)ji.plane_bytes, 256);
    if (end > cap) throw std::runtime_error("submit: batch exceeds the staging pool");
    set_meta(i, im, rgb);
    jdesc[nj] = jpeg_device_desc(ji, (int64_t)coef, (int64_t)planes, (int64_t)rgb);
    max_blocks = std::max(max_blocks, jdesc[nj].total_blocks);
    max_pix = std::max(max_pix, (int64_t)im.h * im.w);
    ++nj;
    off = end;
  }
  {
    trace::Range tp("arena.pack");
    // timing experiments only: ARENA_DEBUG_SKIP_PACK=n reuses the staged pixels after the first n batches
    static const long skip_after = [] {
      const char* e = std::getenv("ARENA_DEBUG_SKIP_PACK");
      return e != nullptr ? std::atol(e) : -1L;
    }();
    if (skip_after < 0 || (long)seq_ <= skip_after) parallel_copy(jobs);
  }
  Ctrl* ctrl = (Ctrl*)sl.h_in;
  std::memset(ctrl, 0, sizeof(Ctrl));
  ctrl->n_images = n;
  ctrl->crop_base = 0;
  sl.in_used = in_bytes_meta() + off;
  hipStream_t cs = copy_mode_ == 2 ? sl.stream : copy_;
  ARENA_HIP_CHECK(hipMemcpyAsync(sl.d_in, sl.h_in, in_bytes_meta() + packed_end, hipMemcpyHostToDevice, cs));
  if (copy_mode_ != 2) {
    ARENA_HIP_CHECK(hipEventRecord(sl.copied, cs));
    ARENA_HIP_CHECK(hipStreamWaitEvent(sl.stream, sl.copied, 0));
  }
  ARENA_HIP_CHECK(hipEventRecord(sl.started, sl.stream));
  // split-decoded JPEGs: dequantize + IDCT + upsample + colour-convert into their RGB slots before the program
  if (nj > 0) {
    trace::Range tj("arena.jpeg_reconstruct");
    jpeg_reconstruct((const JpegDesc*)(sl.d_in + jpeg_desc_off()), sl.d_in + in_bytes_meta(), nj, max_blocks, max_pix,
                     sl.stream);
    ARENA_HIP_CHECK(hipGetLastError());
  }
  // frames exported to another buffer on this device (arm B's IPC ring): device to device, in stream order
  for (int i = 0; i < n; ++i) {
    const InputImage& im = imgs[i];
    if (im.export_dst == nullptr || im.bytes > 0) continue;
    ARENA_HIP_CHECK(hipMemcpyAsync(im.export_dst, sl.d_in + in_bytes_meta() + meta[i].offset, (size_t)im.h * im.w * 3,
                                   hipMemcpyDeviceToDevice, sl.stream));
  }
  if (debug_sync_ >= 3) {
    // 3: whole program as one graph without the D2H node, D2H issued eagerly after it.
    // 4: whole program graph including the D2H node, built fresh.
    Bucket& bk = buckets_.at(B);
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    const size_t d2h = out_off_topk() + sizeof(TopkResult) * (size_t)bk.info.crop_cap;
    ARENA_HIP_CHECK(hipStreamBeginCapture(compute_, hipStreamCaptureModeThreadLocal));
    enqueue_program(prog_, bk, sl, compute_);
    if (debug_sync_ == 4) ARENA_HIP_CHECK(hipMemcpyAsync(sl.h_out, sl.d_out, d2h, hipMemcpyDeviceToHost, compute_));
    ARENA_HIP_CHECK(hipStreamEndCapture(compute_, &g));
    ARENA_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    fprintf(stderr, "[arena debug] launching whole-program graph (mode %d)\n", debug_sync_);
    ARENA_HIP_CHECK(hipGraphLaunch(ge, compute_));
    ARENA_HIP_CHECK(hipStreamSynchronize(compute_));
    fprintf(stderr, "[arena debug] graph done\n");
    if (debug_sync_ == 3) ARENA_HIP_CHECK(hipMemcpyAsync(sl.h_out, sl.d_out, d2h, hipMemcpyDeviceToHost, compute_));
    ARENA_HIP_CHECK(hipStreamSynchronize(compute_));
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  } else if (debug_sync_) {
    // Eager, op-by-op execution with a device sync after every op (ARENA_DEBUG_SYNC=1):
    // a faulting op is reported by index before the context is lost.
    Bucket& bk = buckets_.at(B);
    for (size_t i = 0; i < prog_.size(); ++i) {
      fprintf(stderr, "[arena debug] op %zu type %lld\n", i, (long long)prog_[i][0]);
      fflush(stderr);
      std::vector<OpRecord> one(1, prog_[i]);
      if (debug_sync_ == 2) {  // same op, but through a one-node hipGraph
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        ARENA_HIP_CHECK(hipStreamBeginCapture(compute_, hipStreamCaptureModeThreadLocal));
        enqueue_program(one, bk, sl, compute_);
        ARENA_HIP_CHECK(hipStreamEndCapture(compute_, &g));
        ARENA_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        ARENA_HIP_CHECK(hipGraphLaunch(ge, compute_));
        ARENA_HIP_CHECK(hipStreamSynchronize(compute_));
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
      } else {
        enqueue_program(one, bk, sl, compute_);
      }
      ARENA_HIP_CHECK(hipStreamSynchronize(compute_));
    }
    enqueue_results_d2h(bk, sl, n);
  } else {
    Bucket& bk = buckets_.at(B);
    launch_graph(bk, s, sl.stream, n);
    enqueue_results_d2h(bk, sl, n);
  }
  buckets_.at(B).last_slot = s;
  ARENA_HIP_CHECK(hipEventRecord(sl.done, sl.stream));
  sl.t_submit = std::chrono::steady_clock::now();
  sl.polled = false;
  sl.busy = true;
  sl.bucket = B;
  sl.n_images = n;
  next_slot_ = (next_slot_ + 1) % n_slots_;
  return s;
}

// Completion wait of a slot's batch.  HIP's hipEventSynchronize keeps the waiting thread busy for the whole
// device time of the batch (a core per batcher thread at load; a blocking-sync event did not change that:
// profiles/r5triton2/).  ARENA_SYNC selects:
//   adaptive (default): naps of half the expected remaining time (an estimate per bucket of submit -> observed
//     completion), 20 (ARENA_POLL_US) to 200 us, 1 us timer slack: little CPU while the device works, an early
//     completion seen within one nap, the last stretch polled every 20 us;
//   poll: query + fixed ARENA_POLL_US sleeps (default 50);  spin / blocking: hipEventSynchronize (blocking: the
//     event was created with hipEventBlockingSync).
namespace {
enum SyncMode { kAdaptive, kPoll, kHip };
SyncMode sync_mode() {
  static const SyncMode mode = [] {
    const char* e = std::getenv("ARENA_SYNC");
    const std::string v = e != nullptr ? e : "adaptive";
    return v == "poll" ? kPoll : (v == "spin" || v == "blocking") ? kHip : kAdaptive;
  }();
  return mode;
}
}  // namespace

void Executor::wait_done(Slot& sl) {
  const SyncMode mode = sync_mode();
  if (mode == kHip) {
    ARENA_HIP_CHECK(hipEventSynchronize(sl.done));
    return;
  }
  static const int poll_us = [] {
    const char* u = std::getenv("ARENA_POLL_US");
    return std::max(1, u != nullptr ? std::atoi(u) : (sync_mode() == kPoll ? 50 : 20));
  }();
  thread_local bool slack_set = false;
  if (!slack_set) {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 us: the short sleeps below must not stretch to 50 us
    slack_set = true;
  }
  hipError_t q = hipEventQuery(sl.done);
  if (q != hipErrorNotReady) {
    ARENA_HIP_CHECK(q);
    if (sl.polled) note_done(sl);  // the batcher's completion tests saw it running: a real sample
    return;
  }
  sl.polled = true;
  sl.t_poll = std::chrono::steady_clock::now();
  // Naps toward the expected completion: half the remaining estimate, between ARENA_POLL_US and kMaxNapUs.  A
  // batch that ends earlier than expected is seen within one nap (<= kMaxNapUs late), and the estimate cannot
  // feed on its own oversleeping: a completion seen after a long nap only bounds the true time (note_done).
  constexpr double kMaxNapUs = 200.0;
  while ((q = hipEventQuery(sl.done)) == hipErrorNotReady) {
    double nap = poll_us;
    if (mode == kAdaptive) nap = std::min(kMaxNapUs, std::max((double)poll_us, 0.5 * remaining_us(sl.idx)));
    sl.t_poll = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::microseconds((int64_t)nap));
  }
  ARENA_HIP_CHECK(q);
  note_done(sl);
}

// Completion-time sample of a batch that was seen running (submit -> observed completion), per bucket.  When the
// previous "still running" observation is recent (<= 50 us) the sample is precise and enters an EWMA; after a
// longer gap it is only an upper bound and may lower the estimate, never raise it (otherwise a late wake-up would
// teach the next wait to sleep as long, and the estimate would feed on itself).
void Executor::note_done(Slot& sl) {
  using clk = std::chrono::steady_clock;
  const auto now = clk::now();
  const int B = std::min(std::max(sl.bucket, 0), kMaxEstBuckets - 1);
  const float est = wall_est_us_[B].load(std::memory_order_relaxed);
  const float seen = (float)std::chrono::duration<double, std::micro>(now - sl.t_submit).count();
  const bool precise = std::chrono::duration<double, std::micro>(now - sl.t_poll).count() <= 50.0;
  float upd;
  if (est <= 0.f) upd = seen;
  else if (precise) upd = 0.8f * est + 0.2f * seen;
  else upd = std::min(est, seen);
  wall_est_us_[B].store(upd, std::memory_order_relaxed);
  sl.polled = false;
}

int Executor::ready(int s) {
  if (s < 0 || s >= n_slots_ || sync_mode() == kHip) return -1;  // spin / blocking: the batcher just collects
  Slot& sl = slots_[s];
  if (!sl.busy) return 1;
  const hipError_t q = hipEventQuery(sl.done);
  if (q == hipErrorNotReady) {
    sl.polled = true;
    sl.t_poll = std::chrono::steady_clock::now();
    return 0;
  }
  (void)hipGetLastError();
  if (q == hipSuccess && sl.polled) note_done(sl);
  return 1;  // done, or an error collect() reports
}

double Executor::remaining_us(int s) {
  if (s < 0 || s >= n_slots_) return 0.0;
  const Slot& sl = slots_[s];
  const int B = std::min(std::max(sl.bucket, 0), kMaxEstBuckets - 1);
  const float est = wall_est_us_[B].load(std::memory_order_relaxed);
  if (est <= 0.f) return 0.0;
  return (double)est -
         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - sl.t_submit).count();
}

// The batch's input DMA ran on the shared copy stream and only device streams waited for it (hipStreamWaitEvent).
// Left at that, HIP keeps ~2 KB of live host allocations per batch without bound (profiles/r6_serving/leak:
// +65 B/request of malloc'd bytes in use).  A host synchronisation of the copy stream releases them; a query or a
// synchronize of the copy's event does not (measured, same README).  Every 64 batches the collect synchronizes the
// copy stream: it waits at most for the H2D copies queued behind this batch's, ~0.2 ms per 64 batches.
// ARENA_COPY_RELEASE=0 turns it off.
void Executor::release_copy(Slot& sl) {
  (void)sl;
  static const bool on = [] {
    const char* e = std::getenv("ARENA_COPY_RELEASE");
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (copy_mode_ == 2 || !on) return;
  if (++copy_release_n_ % 64 == 0) ARENA_HIP_CHECK(hipStreamSynchronize(copy_));
}

BatchResult Executor::collect(int s) {
  if (s < 0 || s >= n_slots_) throw std::runtime_error("collect: bad slot");
  Slot& sl = slots_[s];
  if (!sl.busy) throw std::runtime_error("collect: slot not in flight");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  {
    trace::Range tw("arena.collect.wait");
    wait_done(sl);
  }
  release_copy(sl);
  trace::Range tu("arena.collect.unpack");
  BatchResult res;
  res.n_images = sl.n_images;
  res.bucket = sl.bucket;
  float ms = 0.f;
  hipEventElapsedTime(&ms, sl.started, sl.done);
  res.gpu_ms = ms;
  if (has_stamps_) {  // device wall clock at program start, classifier start, program end (OP_STAMP 0 / 1 / 2)
    const uint64_t* st = (const uint64_t*)(sl.h_out + out_off_stamps());
    if (st[1] >= st[0] && st[2] >= st[1] && st[0] != 0) {
      res.det_ms = (double)(st[1] - st[0]) / wall_khz_;
      res.cls_ms = (double)(st[2] - st[1]) / wall_khz_;
    }
  }
  const int n = sl.n_images;
  const int* cnt = (const int*)sl.h_out;
  const Detection* det = (const Detection*)(sl.h_out + out_off_det());
  res.det_count.assign(cnt, cnt + n);
  res.det.assign(det, det + (size_t)n * cfg_.max_det);
  res.crop_offset.resize(n + 1);
  int total = 0;
  for (int i = 0; i < n; ++i) {
    res.crop_offset[i] = total;
    if (has_topk_) total += std::min(cnt[i], cfg_.max_det);
  }
  res.crop_offset[n] = total;
  res.total_crops = total;
  if (has_raw_) res.raw.assign(sl.h_out + out_off_raw(), sl.h_out + out_off_raw() + (size_t)cfg_.raw_out_bytes * n);
  if (!has_det_ && !peer_stage_) res.det_count.assign(n, 0);
  Bucket& bk = buckets_.at(sl.bucket);
  const int CC = bk.info.crop_cap;
  if (has_topk_ && total > CC) {
    // Overflow: classify the remaining crops in extra passes of CC crops.
    std::lock_guard<std::mutex> lk(mu_);
    for (int base = CC; base < total; base += CC) {
      Ctrl c{};
      c.n_images = n;
      c.crop_base = base;
      c.total_crops = total;
      c.n_crops = std::min(CC, total - base);
      // previous pass must have consumed the control block before it is rewritten
      ARENA_HIP_CHECK(hipStreamSynchronize(sl.stream));
      ARENA_HIP_CHECK(hipMemcpy(sl.d_in, &c, sizeof(Ctrl), hipMemcpyHostToDevice));
      enqueue_program(cls_prog_, bk, sl, sl.stream, (int)(prog_.size() - cls_prog_.size()));
    }
    uint8_t* src = sl.d_out + out_off_topk() + sizeof(TopkResult) * (size_t)CC;
    uint8_t* dst = sl.h_out + out_off_topk() + sizeof(TopkResult) * (size_t)CC;
    ARENA_HIP_CHECK(hipMemcpyAsync(dst, src, sizeof(TopkResult) * (size_t)(total - CC), hipMemcpyDeviceToHost,
                                   sl.stream));
    ARENA_HIP_CHECK(hipStreamSynchronize(sl.stream));
  }
  const TopkResult* tk = (const TopkResult*)(sl.h_out + out_off_topk());
  res.topk.assign(tk, tk + total);
  sl.busy = false;
  return res;
}

BatchResult Executor::run(const std::vector<InputImage>& imgs) { return collect(submit(imgs)); }

void Executor::enable_peer(int src, const char* what) {
  if (src < 0 || src == cfg_.device) return;
  if (std::find(peer_enabled_.begin(), peer_enabled_.end(), src) != peer_enabled_.end()) return;
  require_peer_access(cfg_.device, src, what, hip_can_access_peer);  // runtime/peer.h: clear error, no fault
  const hipError_t e = hipDeviceEnablePeerAccess(src, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) ARENA_HIP_CHECK(e);
  (void)hipGetLastError();
  peer_enabled_.push_back(src);
}

int Executor::submit_peer(Executor& src, int src_slot) {
  trace::Range tr("arena.submit_peer");
  if (!peer_stage_) throw std::runtime_error("submit_peer: executor is not a peer stage (set_peer_stage)");
  if (src_slot < 0 || src_slot >= src.n_slots_ || !src.slots_[src_slot].busy)
    throw std::runtime_error("submit_peer: source slot not in flight");
  if (src.max_B_ != max_B_ || src.cfg_.max_det != cfg_.max_det || src.in_bytes_total() != in_bytes_total())
    throw std::runtime_error("submit_peer: source and peer stage need the same max_batch / max_det / staging");
  Slot& ss = src.slots_[src_slot];
  std::lock_guard<std::mutex> lk(mu_);
  const int B = ss.bucket;
  auto it = buckets_.find(B);
  if (it == buckets_.end()) throw std::runtime_error("submit_peer: peer stage lacks bucket " + std::to_string(B));
  const int s = next_slot_;
  Slot& sl = slots_[s];
  if (sl.busy) throw std::runtime_error("submit_peer: every staging slot is in flight; collect() first");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  const int sdev = src.cfg_.device;
  enable_peer(sdev, "submit_peer (split topology)");
  sl.stream = streams_[seq_++ % n_streams_];
  // the detector's graph (and its result copy) finished on the source device
  ARENA_HIP_CHECK(hipStreamWaitEvent(sl.stream, ss.done, 0));
  auto copy = [&](uint8_t* dst, const uint8_t* srcp, size_t n) {
    if (n == 0) return;
    if (sdev == cfg_.device)
      ARENA_HIP_CHECK(hipMemcpyAsync(dst, srcp, n, hipMemcpyDeviceToDevice, sl.stream));
    else
      ARENA_HIP_CHECK(hipMemcpyPeerAsync(dst, cfg_.device, srcp, sdev, n, sl.stream));
  };
  copy(sl.d_in, ss.d_in, ss.in_used);                                                // ctrl, meta, images
  copy(sl.d_out, ss.d_out, out_off_topk());                                          // det counts + dets
  copy(sl.d_out + out_off_xcrops(), ss.d_out + out_off_xcrops(), sizeof(CropRef) * (size_t)max_B_ * cfg_.max_det);
  ARENA_HIP_CHECK(hipEventRecord(sl.started, sl.stream));
  Bucket& bk = it->second;
  launch_graph(bk, s, sl.stream, ss.n_images);
  enqueue_results_d2h(bk, sl, ss.n_images);
  bk.last_slot = s;
  ARENA_HIP_CHECK(hipEventRecord(sl.done, sl.stream));
  sl.t_submit = std::chrono::steady_clock::now();
  sl.polled = false;
  sl.busy = true;
  sl.bucket = B;
  sl.n_images = ss.n_images;
  sl.in_used = ss.in_used;
  next_slot_ = (next_slot_ + 1) % n_slots_;
  return s;
}

int Executor::submit_device(const std::vector<DeviceImage>& imgs, const std::vector<std::vector<Detection>>& dets) {
  trace::Range tr("arena.submit_device");
  if (!peer_stage_) throw std::runtime_error("submit_device: executor is not a second-stage program (set_peer_stage)");
  const int n = (int)imgs.size();
  if (n <= 0 || dets.size() != imgs.size()) throw std::runtime_error("submit_device: one detection list per image");
  std::lock_guard<std::mutex> lk(mu_);
  const int B = pick_bucket(n);
  if (B < 0) throw std::runtime_error("submit_device: batch larger than the largest bucket");
  auto it = buckets_.find(B);
  const int s = next_slot_;
  Slot& sl = slots_[s];
  if (sl.busy) throw std::runtime_error("submit_device: every staging slot is in flight; collect() first");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  sl.stream = streams_[seq_++ % n_streams_];
  // host staging of the small blocks: ctrl + image metadata (d_in), detection counts + detections + crop plan
  // (d_out); h_out is free until this slot's result copy, which the stream orders after these uploads
  Ctrl* ctrl = (Ctrl*)sl.h_in;
  std::memset(sl.h_in, 0, in_bytes_meta());
  ImageMeta* meta = (ImageMeta*)(sl.h_in + kCtrlBytes);
  int* cnt = (int*)sl.h_out;
  Detection* det = (Detection*)(sl.h_out + out_off_det());
  CropRef* crops = (CropRef*)(sl.h_out + out_off_xcrops());
  std::memset(sl.h_out, 0, out_off_topk());
  const size_t cap = pool_cap();
  size_t off = 0;
  int total = 0;
  const int T = cfg_.det_size > 0 ? cfg_.det_size : 640;
  for (int i = 0; i < n; ++i) {
    const DeviceImage& im = imgs[i];
    if (im.h <= 0 || im.w <= 0 || im.ptr == 0) throw std::runtime_error("submit_device: empty image");
    const size_t bytes = (size_t)im.h * im.w * 3;
    if (off + bytes > cap) throw std::runtime_error("submit_device: batch exceeds the staging pool");
    ImageMeta& m = meta[i];
    m.offset = (int64_t)off;
    m.h = im.h;
    m.w = im.w;
    const double sc = std::min((double)T / im.h, (double)T / im.w);
    m.new_w = (int)(im.w * sc);
    m.new_h = (int)(im.h * sc);
    m.pad_w = (T - m.new_w) / 2;
    m.pad_h = (T - m.new_h) / 2;
    m.scale = (float)sc;
    const int k = std::min((int)dets[i].size(), cfg_.max_det);
    cnt[i] = k;
    for (int d = 0; d < k; ++d) {
      const Detection& dd = dets[i][d];
      const float lim = 1e6f;  // casting a non-finite / huge float to int is undefined behaviour
      if (!(std::fabs(dd.x1) < lim && std::fabs(dd.y1) < lim && std::fabs(dd.x2) < lim && std::fabs(dd.y2) < lim))
        throw std::runtime_error("submit_device: box coordinates are not finite or out of range");
      det[(size_t)i * cfg_.max_det + d] = dd;
      CropRef& r = crops[total + d];
      r.img = i;
      r.x1 = std::max(0, (int)dd.x1);
      r.y1 = std::max(0, (int)dd.y1);
      r.x2 = std::min(im.w, (int)dd.x2);
      r.y2 = std::min(im.h, (int)dd.y2);
      r.det = d;
      r.pad_[0] = r.pad_[1] = 0;
    }
    total += k;
    off = align_up(off + bytes, 256);
  }
  if (total > (int)max_B_ * cfg_.max_det) throw std::runtime_error("submit_device: too many crops");
  const int CC = it->second.info.crop_cap;
  ctrl->n_images = n;
  ctrl->crop_base = 0;
  ctrl->total_crops = total;
  ctrl->n_crops = std::min(total, CC);
  ARENA_HIP_CHECK(hipMemcpyAsync(sl.d_in, sl.h_in, in_bytes_meta(), hipMemcpyHostToDevice, sl.stream));
  ARENA_HIP_CHECK(hipMemcpyAsync(sl.d_out, sl.h_out, out_off_topk(), hipMemcpyHostToDevice, sl.stream));
  ARENA_HIP_CHECK(hipMemcpyAsync(sl.d_out + out_off_xcrops(), crops, sizeof(CropRef) * (size_t)std::max(total, 1),
                                 hipMemcpyHostToDevice, sl.stream));
  for (int i = 0; i < n; ++i)
    if (imgs[i].device >= 0 && imgs[i].device != cfg_.device) enable_peer(imgs[i].device, "submit_device");
  for (int i = 0; i < n; ++i) {  // the pixels: device to device, never through the host
    const DeviceImage& im = imgs[i];
    uint8_t* dst = sl.d_in + in_bytes_meta() + meta[i].offset;
    const size_t bytes = (size_t)im.h * im.w * 3;
    if (im.device < 0 || im.device == cfg_.device)
      ARENA_HIP_CHECK(hipMemcpyAsync(dst, (const void*)im.ptr, bytes, hipMemcpyDeviceToDevice, sl.stream));
    else
      ARENA_HIP_CHECK(hipMemcpyPeerAsync(dst, cfg_.device, (const void*)im.ptr, im.device, bytes, sl.stream));
  }
  sl.in_used = in_bytes_meta() + off;
  ARENA_HIP_CHECK(hipEventRecord(sl.started, sl.stream));
  Bucket& bk = it->second;
  launch_graph(bk, s, sl.stream, n);
  enqueue_results_d2h(bk, sl, n);
  bk.last_slot = s;
  ARENA_HIP_CHECK(hipEventRecord(sl.done, sl.stream));
  sl.t_submit = std::chrono::steady_clock::now();
  sl.polled = false;
  sl.busy = true;
  sl.bucket = B;
  sl.n_images = n;
  next_slot_ = (next_slot_ + 1) % n_slots_;
  return s;
}

void Executor::replay(int B, int s, int iters) {
  auto it = buckets_.find(B);
  if (it == buckets_.end()) throw std::runtime_error("replay: unknown bucket");
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  if (s < 0 || s >= n_slots_) throw std::runtime_error("replay: bad slot");
  for (int i = 0; i < iters; ++i) launch_graph(it->second, s, streams_[s % n_streams_]);
}

void Executor::synchronize() {
  ARENA_HIP_CHECK(hipSetDevice(cfg_.device));
  ARENA_HIP_CHECK(hipStreamSynchronize(copy_));
  sync_slots();
}

}  // namespace arena
