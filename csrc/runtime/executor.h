// Native pipeline executor (ONNX Runtime + Triton-instance replacement).
//
// The reference runs each model through an ONNX Runtime CPU session per
// request (src/shared/model/registry.py:184-254; ModelRegistry.get_session)
// and moves every intermediate through host memory.  Here one Executor owns a
// whole GPU-resident two-stage pipeline:
//
//   pinned staging --H2D--> [ctrl | image meta | uint8 image pool]
//     letterbox -> YOLOv5nu convs -> decode -> NMS -> crop plan
//     -> crop gather -> MobileNetV2 convs -> avgpool -> FC -> top-5
//   --D2H--> [det counts | detections | classifications]  (pinned)
//
// The op sequence is a static program produced by the Python planner
// (inference_arena_amd/engine/planner.py): fixed-size int64 records that
// name arena buffers by id.  For every batch bucket the executor resolves the
// records to device pointers once and captures the whole sequence (including
// memsets and the result D2H copy) into a hipGraph; a request batch is then
// one H2D copy on a copy stream + one graph launch on a compute stream.
// Staging slots (pinned + device input/output, activation arena, one graph
// per bucket) outnumber the compute streams: up to ARENA_CONCURRENCY graphs
// execute concurrently on the device while the next batches are packed and
// uploaded into the remaining slots.
#pragma once
#include <chrono>
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../kernels/launch.h"
#include "instance.h"

namespace arena {

constexpr int kOpFields = 48;
constexpr int kDtypeField = 47;  // per-op activation precision: 0 bf16, 1 exact fp32
// Per-op stream lane (planner.OP_LANE_FIELD): 0 = the batch's stream; 1..kMaxLanes = a side stream forked from
// it before the first op of a run of lane ops and joined back at the next lane-0 op (independent branches such
// as the three Detect-head levels run concurrently, inside the captured graph as parallel branches).
constexpr int kLaneField = 46;
constexpr int kMaxLanes = 3;
constexpr int kMaxSlots = 6;
constexpr int kMaxStaggerParts = 5;  // staggered launch: at most 4 split points (executor.cpp launch_graph)
constexpr int kMaxEstBuckets = 257;  // completion-time estimates per bucket size (larger buckets share the last)
using OpRecord = std::array<int64_t, kOpFields>;

enum OpType : int64_t {
  OP_CONV = 1,
  OP_DWCONV = 2,
  OP_SPPF = 3,
  OP_LETTERBOX = 4,
  OP_ZERO = 5,
  OP_DECODE = 6,
  OP_NMS = 7,
  OP_CROPPLAN = 8,
  OP_CROPGATHER = 9,
  OP_AVGPOOL = 10,
  OP_TOPK = 11,
  OP_TENSORIN = 12,
  OP_YOLORAW = 13,
  OP_IRBLOCK = 14,
  OP_STEMFUSED = 15,
  OP_C3FUSED = 16,
  OP_HEADPOOL = 17,
  OP_STAMP = 18,  // 1: stamp index (0 program start, 1 classifier start, 2 end): device wall clock -> results
};

// Reserved buffer ids (the planner's arena buffers are ids >= 0).
enum ReservedBuf : int64_t {
  BUF_NONE = -1,
  BUF_CTRL = -10,
  BUF_META = -11,
  BUF_POOL = -12,
  BUF_DET = -13,
  BUF_DETCOUNT = -14,
  BUF_TOPK = -15,
  BUF_RAWOUT = -16,
  BUF_XCROPS = -17,  // crop plan exported for a second-stage executor (split topology), in the output block
};

// Batch kind of an op: which live count clamps it.
enum BatchKind : int64_t { BATCH_IMAGES = 0, BATCH_CROPS = 1 };

struct ExecutorConfig {
  int device = 0;
  int max_batch = 32;         // largest bucket; sizes the staging slots
  int max_det = 300;          // detections kept per image (reference: unbounded)
  int cand_cap = 8400;        // candidates per image entering NMS (= anchors)
  int crop_cap_per_image = 6; // crops one classification pass holds, per image (overflow -> extra pass)
  int min_crop_cap = 16;
  int64_t pool_bytes_per_image = 640LL * 640 * 3;  // RGB staging bytes per image of a full batch
  // The device image pool of a slot holds pool_factor x that: room for split-decoded JPEGs, whose coefficient
  // blocks (2 B per sample) and reconstruction planes sit next to the RGB frame they turn into (4:2:0 frames
  // need 2.5x, 4:4:4 ones 3x; the batcher closes a batch early when its inputs would not fit).
  int pool_factor = 3;
  int det_size = 640;
  int cls_size = 224;
  int host_threads = 8;
  int64_t raw_out_bytes = 0;  // per-image raw output region (reference tensor contracts)
};

struct BucketInfo {
  int B = 0;
  int crop_cap = 0;
  std::vector<int64_t> offsets;  // arena byte offset per planner buffer id
  int64_t arena_bytes = 0;
};

class Executor : public BatchInstance {
 public:
  explicit Executor(const ExecutorConfig& cfg);
  ~Executor() override;
  Executor(const Executor&) = delete;
  Executor& operator=(const Executor&) = delete;

  void set_weights(const void* host, size_t bytes);
  // Same-size update from device memory of this executor's GPU (e.g. an RCCL broadcast buffer): D2D copy.
  void set_weights_device(const void* dev, size_t bytes);
  // the device weight blob copied back to the host (replica bring-up check: every rank's bytes must hash equal)
  std::vector<uint8_t> weights_host();
  void set_program(const int64_t* ops, int n_ops, const int64_t* cls_ops, int n_cls_ops);
  // `impl` (optional, one entry per program op): conv kernel family per op from a persisted tuning table;
  // when given, the bucket is captured with exactly these choices and no timing runs (deterministic).
  void add_bucket(int B, const int64_t* offsets, int n_buffers, int64_t arena_bytes,
                  const std::vector<int>* impl = nullptr);
  std::vector<int> buckets() const override;
  int crop_cap_for(int B) const;
  const ExecutorConfig& config() const { return cfg_; }
  int max_det() const override { return cfg_.max_det; }
  int64_t raw_out_bytes() const override { return cfg_.raw_out_bytes; }
  int64_t staging_bytes() const override { return (int64_t)pool_cap(); }

  // Asynchronous pipelined API: submit() packs the images into a free staging
  // slot, enqueues H2D + graph and returns the slot id; collect() waits for
  // that slot and returns its results (running overflow classification passes
  // when a batch produced more crops than one pass holds).
  int submit(const std::vector<InputImage>& imgs) override;
  BatchResult collect(int slot) override;
  int ready(int slot) override;
  double remaining_us(int slot) override;
  // Convenience: submit + collect.
  BatchResult run(const std::vector<InputImage>& imgs);

  // Split topology (detection on one GPU, classification on another): enqueue this executor's program on
  // the batch that `src` (a detector + crop-plan program on any device) runs in `src_slot`.  On this
  // executor's stream, after src's slot completes: peer copies (xGMI) of src's staged input block (ctrl
  // with the crop counts, image metadata, the decoded images), its detections and its exported crop
  // plan (BUF_XCROPS), then this program's graph (crop gather + classifier) and the result D2H.  The
  // result of collect() on this executor is the whole request result (detections + classifications).
  int submit_peer(Executor& src, int src_slot);
  // Cross-process device hand-off (arm B, ARENA_CROP_TRANSPORT=device): run this second-stage program (crop
  // gather from the staged images with the exported crop plan -> classifier) on images that already sit in
  // device memory — another process's IPC-shared buffer (IpcBuffer / ipc_open) or any device pointer — with
  // their detections given by the host.  The images are copied device to device into the slot's pool (peer
  // copy when they live on another GPU), the control block, image metadata, detections and the crop plan
  // (the crop_plan_kernel's rules: int-truncated boxes clamped to the image) are staged from the host; the
  // result of collect() is as for submit_peer.
  struct DeviceImage {
    uintptr_t ptr = 0;  // HWC uint8 RGB
    int h = 0, w = 0;
    int device = -1;    // -1: this executor's device
  };
  int submit_device(const std::vector<DeviceImage>& imgs, const std::vector<std::vector<Detection>>& dets);
  // Mark this executor as a second stage (its detections arrive from a peer, see submit_peer).
  void set_peer_stage(bool v) { peer_stage_ = v; }
  bool peer_stage() const { return peer_stage_; }
  int device() const { return cfg_.device; }

  // Run only the captured graph of a bucket on already-staged inputs; used by
  // microbenchmarks to separate host packing from device time.
  void replay(int B, int slot, int iters);
  void synchronize();
  // Staging slots = batches that may be in flight at once (submit() throws when all are busy).
  int num_slots() const override { return n_slots_; }

  // Device pointers for tests / introspection.
  uintptr_t arena_ptr(int B) const;
  // Debug: synchronously copy `bytes` from a bucket's arena at `offset` to host.
  void read_arena(int B, int64_t offset, void* dst, size_t bytes);
  uintptr_t weights_ptr() const { return (uintptr_t)d_weights_; }
  uintptr_t stream() const { return (uintptr_t)compute_; }

 private:
  std::vector<uint8_t*> retired_h_in_;  // outgrown pinned staging, freed with the executor (submit never frees)
  int64_t staging_growths_ = 0;

 public:
  int64_t staging_growths() const { return staging_growths_; }

 private:
  struct Slot {
    // device
    uint8_t* d_in = nullptr;   // ctrl | meta | pool
    uint8_t* d_out = nullptr;  // det_count | det | topk
    float* sk_ws = nullptr;    // split-K conv workspace: (kMaxLanes + 1) x sk_lane_bytes()
    // pinned host
    uint8_t* h_in = nullptr;
    size_t h_cap = 0;  // bytes of h_in (meta + host-packed inputs; grows on demand)
    uint8_t* h_out = nullptr;
    hipEvent_t copied = nullptr, started = nullptr, done = nullptr;
    // staggered launch: phase[i] = the batch finished part i of its program (ARENA_STAGGER)
    hipEvent_t phase[kMaxStaggerParts] = {};
    // Each slot owns an activation arena; its batch runs on one of the
    // executor's compute streams (round-robin by submission), so in-flight
    // batches overlap on the device: the small-grid tail of one batch's layers
    // (20x20 / 7x7 maps leave most of the 256 CUs idle) is filled by another
    // batch's work.  More slots than streams lets the next batches' packing
    // and H2D copies run ahead while the device is busy.
    hipStream_t stream = nullptr;  // stream of the slot's current batch
    hipStream_t lane_stream[kMaxLanes] = {};  // side streams of program lanes (kLaneField)
    hipEvent_t fork_ev = nullptr, lane_ev[kMaxLanes] = {};
    int idx = 0;
    std::chrono::steady_clock::time_point t_submit{};  // host time of the submit (adaptive completion wait)
    bool polled = false;  // a completion test found the batch running (its completion time is a real sample)
    std::chrono::steady_clock::time_point t_poll{};  // last completion test that found it running
    bool busy = false;
    int bucket = 0;
    int n_images = 0;
    size_t in_used = 0;  // staged input bytes (ctrl + meta + images) of the current batch
  };
  struct Bucket {
    BucketInfo info;
    uint8_t* d_arena[kMaxSlots] = {};  // per slot (all aliased when concurrency is off)
    int last_slot = 0;                 // slot whose arena read_arena() inspects
    hipGraphExec_t graph[kMaxSlots] = {};
    // staggered launch (ARENA_STAGGER): the program as consecutive parts split at the stagger points, one graph
    // each (graph[s] unused then)
    std::vector<hipGraphExec_t> parts[kMaxSlots];
    // Lane buckets (program lanes, B <= lanes_max_batch()): the program as contiguous single-lane segments, one
    // graph each; launch_graph() runs lane segments on the slot's side streams between fork / join events.
    // (A single graph with forked branches made HIP's graph launch segfault with GPU_MAX_HW_QUEUES < 4 from the
    // batcher's instance thread: profiles/r5lanes/README.md.)
    struct Seg {
      int lane = 0;
      hipGraphExec_t g = nullptr;
    };
    std::vector<Seg> segs[kMaxSlots];
    std::vector<int16_t> impl;  // per op of prog_: conv kernel family chosen by autotune (0 = default)
  };

  void alloc_slots();
  void ensure_lanes(Slot& sl);
  void sync_slots();
  void free_arenas(Bucket& bk);
  void capture(Bucket& bk, int slot);
  void wait_done(Slot& sl);
  void note_done(Slot& sl);
  void release_copy(Slot& sl);
  static int64_t sk_lane_bytes();
  uint64_t copy_release_n_ = 0;
  void launch_graph(Bucket& bk, int slot, hipStream_t st, int n_live = -1);  // n_live: images of the batch
  void destroy_graphs(Bucket& bk, int slot);
  bool lanes_for(const Bucket& bk) const;
  void enqueue_program(const std::vector<OpRecord>& prog, Bucket& bk, Slot& sl, hipStream_t s,
                       int op_offset = 0, int force_impl = 0);
  void autotune(Bucket& bk);

 public:
  // conv kernel family per program op chosen for bucket B (0 = default / not a conv)
  std::vector<int> conv_choices(int B) const {
    auto it = buckets_.find(B);
    if (it == buckets_.end()) return {};
    return std::vector<int>(it->second.impl.begin(), it->second.impl.end());
  }

 private:
  void enqueue_results_d2h(Bucket& bk, Slot& sl, int n);
  uint8_t* resolve(Bucket& bk, Slot& sl, int64_t buf, int64_t coff_elems, int elem_bytes);
  int pick_bucket(int n) const;
  size_t in_bytes_meta() const;   // ctrl | ImageMeta[max_B] | JpegDesc[max_B]
  size_t jpeg_desc_off() const;
  size_t pool_cap() const;        // image pool bytes of a slot
  size_t in_bytes_total() const;
  size_t out_off_det() const;
  size_t out_off_topk() const;
  size_t out_bytes_total() const;
  size_t out_off_raw() const;
  size_t out_off_xcrops() const;
  size_t out_off_stamps() const;  // 4 x uint64 device wall-clock stamps (OP_STAMP)
  int acquire_slot();
  void parallel_copy(std::vector<std::function<void()>>& jobs);

  ExecutorConfig cfg_;
  int max_B_ = 0;
  hipStream_t compute_ = nullptr, copy_ = nullptr;
  uint8_t* d_weights_ = nullptr;
  size_t weights_bytes_ = 0;
  std::vector<OpRecord> prog_, cls_prog_;
  std::map<int, Bucket> buckets_;
  Slot slots_[kMaxSlots];
  int n_slots_ = 2;
  int next_slot_ = 0;
  hipStream_t streams_[kMaxSlots] = {};  // compute streams (streams_[0] == compute_)
  int n_streams_ = 1;
  uint64_t seq_ = 0;                     // batches submitted
  // Staggered launch (ARENA_STAGGER = "f1[,f2...]", fractions of the program's ops; 0 = off): the program runs as
  // parts split at those ops, and a batch starts part i only once the previously launched batch has finished its
  // part i, so the batches in flight on the compute streams sit at different phases of the program instead of
  // drifting into step (launch_graph)
  std::vector<double> stagger_;  // split points as fractions of the program's ops, ascending
  int stagger_min_batch_ = 32;  // ARENA_STAGGER_MIN_BATCH: batches with fewer live images launch unstaggered
  int last_launched_ = -1;  // slot of the last staggered launch
  bool has_topk_ = false, has_det_ = false, has_raw_ = false, has_stamps_ = false;
  double wall_khz_ = 100000.0;  // wall_clock64 rate (hipDeviceAttributeWallClockRate)
  bool peer_stage_ = false;
  std::vector<int> peer_enabled_;  // devices this executor's device has peer access to
  void enable_peer(int src, const char* what);  // require_peer_access (runtime/peer.h) + hipDeviceEnablePeerAccess
  int copy_mode_ = 0;   // ARENA_COPY_MODE: 0 copy stream + event, 2 copy on the slot's stream
  // ARENA_CONCURRENT: 1 = per-slot streams + arenas (in-flight batches overlap on the device),
  // 0 = two slots serialised on one stream sharing one arena.  ARENA_SLOTS: staging slots when concurrent
  // (default 4), ARENA_CONCURRENCY: compute streams = graphs running at once (default 3).
  int concurrent_ = 1;
  int autotune_ = 1;  // ARENA_AUTOTUNE: 0 off, 1 on, 2 on + report
  int debug_sync_ = 0;  // ARENA_DEBUG_SYNC: 1 eager op-by-op, 2 one graph per op
  std::mutex mu_;
  // host worker pool for packing images into pinned memory
  std::vector<std::thread> workers_;
  std::mutex pool_mu_;
  std::condition_variable pool_cv_, pool_done_cv_;
  std::vector<std::function<void()>>* pool_jobs_ = nullptr;
  std::atomic<int> pool_next_{0};
  std::atomic<float> wall_est_us_[kMaxEstBuckets] = {};  // wait_done(): submit -> completion EWMA per bucket
  int pool_active_ = 0;
  uint64_t pool_gen_ = 0;
  bool pool_stop_ = false;
};

}  // namespace arena
