// Detector tail on the GPU: SPPF pooling (K5), DFL/box decode + class
// threshold compaction (K7), class-aware greedy NMS with un-letterboxing (K8)
// and the crop plan that feeds the classifier (first half of K9).
//
// Reference semantics:
//   decode: ultralytics Detect head exported in the ONNX graph — DFL softmax
//     over 16 bins per side, dist2bbox (ltrb -> xywh) x stride, sigmoid class
//     scores -> [1,84,8400] (experiment.yaml:199-207).
//   threshold + NMS: architectures/monolithic/app/postprocess.py:12-160 —
//     conf = max class score, class = argmax, keep conf >= thr, per-class
//     greedy NMS suppressing IoU > thr (eps 1e-6), output ordered by class id
//     ascending then score descending.
//   un-letterbox + clip: src/shared/processing/transforms.py:183-230.
//   crop box: src/shared/processing/mobilenet_preprocess.py:236-269.
#include <string>
#include <stdexcept>
#include "common.h"
#include "launch.h"

namespace arena {

// ------------------------------------------------------------------ SPPF
// Cascaded 5x5 stride-1 max pools (== 5/9/13 windows, -inf padding) as two
// separable passes through LDS.  One block = one image x 16 channels (two
// 8-channel chunks): the HxW tile is staged once, a horizontal pass writes the
// 5/9/13-wide row maxima, a vertical pass finishes the three windows and
// stores them into the concat slices C, 2C, 3C.  (v1 re-read 169 pixels per
// output from L2 and ran at ~92 us for the YOLO 20x20x128 case.)
constexpr int SPPF_MAX_PIX = 1024;  // H*W per block (YOLO: 20x20 = 400)

__global__ __launch_bounds__(256) void sppf_kernel(const SppfParams p) {
  extern __shared__ __align__(16) uint4 sp[];  // [4][HW][2] 16-B chunks: in, h5, h9, h13
  const int B = live_batch(p.B, p.bdev);
  const int groups = p.C >> 4;
  const int b = blockIdx.x / groups;
  if (b >= B) return;
  const int c0 = (blockIdx.x - b * groups) * 16;
  const int H = p.H, W = p.W, HW = H * W;
  uint4* in = sp;
  uint4* h5 = sp + 2 * HW;
  uint4* h9 = sp + 4 * HW;
  uint4* h13 = sp + 6 * HW;
  bf16* buf = (bf16*)p.buf + (size_t)b * HW * p.xs;
  // all loads issued before the first LDS store: one memory latency, not one per 256 pieces
  constexpr int kIt = (SPPF_MAX_PIX * 2 + 255) / 256;
  uint4 tmp[kIt];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = threadIdx.x + it * 256;
    if (i < HW * 2) tmp[it] = *(const uint4*)(buf + (size_t)(i >> 1) * p.xs + c0 + (i & 1) * 8);
  }
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int i = threadIdx.x + it * 256;
    if (i < HW * 2) in[i] = tmp[it];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HW * 2; i += 256) {
    const int pix = i >> 1, c = i & 1;
    const int y = pix / W, x = pix - y * W;
    float m5[8], m9[8], m13[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m5[k] = m9[k] = m13[k] = -INFINITY;
#pragma unroll
    for (int dx = -6; dx <= 6; ++dx) {
      const int ix = x + dx;
      if ((unsigned)ix >= (unsigned)W) continue;
      float v[8];
      unpack8(in[(y * W + ix) * 2 + c], v);
      const int a = dx < 0 ? -dx : dx;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        m13[k] = fmaxf(m13[k], v[k]);
        if (a <= 4) m9[k] = fmaxf(m9[k], v[k]);
        if (a <= 2) m5[k] = fmaxf(m5[k], v[k]);
      }
    }
    h5[i] = pack8(m5);
    h9[i] = pack8(m9);
    h13[i] = pack8(m13);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HW * 2; i += 256) {
    const int pix = i >> 1, c = i & 1;
    const int y = pix / W, x = pix - y * W;
    float m5[8], m9[8], m13[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m5[k] = m9[k] = m13[k] = -INFINITY;
#pragma unroll
    for (int dy = -6; dy <= 6; ++dy) {
      const int iy = y + dy;
      if ((unsigned)iy >= (unsigned)H) continue;
      const int j = (iy * W + x) * 2 + c;
      const int a = dy < 0 ? -dy : dy;
      float v[8];
      unpack8(h13[j], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) m13[k] = fmaxf(m13[k], v[k]);
      if (a <= 4) {
        unpack8(h9[j], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) m9[k] = fmaxf(m9[k], v[k]);
      }
      if (a <= 2) {
        unpack8(h5[j], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) m5[k] = fmaxf(m5[k], v[k]);
      }
    }
    bf16* o = buf + (size_t)pix * p.xs + c0 + c * 8;
    *(uint4*)(o + p.C) = pack8(m5);
    *(uint4*)(o + 2 * p.C) = pack8(m9);
    *(uint4*)(o + 3 * p.C) = pack8(m13);
  }
}

void sppf_pool(const SppfParams& p, hipStream_t s) {
  if (p.C % 16 != 0 || p.xs < 4 * p.C || p.H * p.W > SPPF_MAX_PIX)
    throw std::runtime_error("sppf_pool: bad geometry (C % 16, xs >= 4C, H*W <= 1024)");
  if (p.B <= 0) return;
  const size_t lds = (size_t)p.H * p.W * 2 * 16 * 4;
  if (lds > 64 * 1024) prepare_kernels();  // raises the dynamic-LDS limit (done before graph capture)
  hipLaunchKernelGGL(sppf_kernel, dim3((unsigned)(p.B * (p.C / 16))), dim3(256), lds, s, p);
}

// ------------------------------------------------------------------ decode
// T = bf16 (default pipeline) or float (exact-fp32 pipeline) head activations.  The fp32 pipeline uses the
// correctly rounded expf (the reference's torch sigmoid / softmax) instead of the v_exp_f32 approximation.
template <typename T>
__device__ __forceinline__ float exp_t(float v) {
  if constexpr (sizeof(T) == 4) return expf(v);
  else return __expf(v);
}

template <typename T>
__global__ __launch_bounds__(256) void decode_kernel(const DecodeParams p) {
  const int n_img = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  const int A0 = p.hw[0] * p.hw[0], A1 = p.hw[1] * p.hw[1], A2 = p.hw[2] * p.hw[2];
  const int A = A0 + A1 + A2;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)n_img * A) return;
  const int b = (int)(tid / A);
  const int a = (int)(tid - (long)b * A);
  int l, r;
  if (a < A0) { l = 0; r = a; } else if (a < A0 + A1) { l = 1; r = a - A0; } else { l = 2; r = a - A0 - A1; }
  const int hw = p.hw[l];
  const T* px = (const T*)p.head[l] + ((size_t)b * hw * hw + r) * p.xs[l];

  // class scores: sigmoid, max + first argmax (ties resolved like np.argmax)
  float best = -1.f;
  int cls = 0;
#pragma unroll
  for (int g = 0; g < 10; ++g) {
    float v[8];
    load8(px + 64 + g * 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sgm = 1.0f / (1.0f + exp_t<T>(-v[i]));
      if (sgm > best) { best = sgm; cls = g * 8 + i; }
    }
  }
  if (!(best >= p.conf_thr)) return;

  float dist[4];
#pragma unroll
  for (int side = 0; side < 4; ++side) {
    float v[16];
    load8(px + side * 16, v);
    load8(px + side * 16 + 8, v + 8);
    float mx = v[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, v[i]);
    float se = 0.f, sw = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = exp_t<T>(v[i] - mx);
      se += e;
      sw += e * (float)i;
    }
    dist[side] = sw / se;
  }
  const int gy = r / hw, gx = r - (r / hw) * hw;
  const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f;
  const float s = p.stride[l];
  const float bx1 = ax - dist[0], by1 = ay - dist[1], bx2 = ax + dist[2], by2 = ay + dist[3];
  const float cx = (bx1 + bx2) * 0.5f * s, cy = (by1 + by2) * 0.5f * s;
  const float w = (bx2 - bx1) * s, h = (by2 - by1) * s;
  const int slot = atomicAdd(&p.cand_count[b], 1);
  if (slot >= p.cand_cap) return;
  Candidate c;
  c.x1 = cx - w * 0.5f;
  c.y1 = cy - h * 0.5f;
  c.x2 = cx + w * 0.5f;
  c.y2 = cy + h * 0.5f;
  c.score = best;
  c.cls = cls;
  c.anchor = a;
  c.pad_ = 0;
  p.cand[(size_t)b * p.cand_cap + slot] = c;
}

void detect_decode(const DecodeParams& p, hipStream_t s) {
  const long A = (long)p.hw[0] * p.hw[0] + (long)p.hw[1] * p.hw[1] + (long)p.hw[2] * p.hw[2];
  const long total = A * p.B;
  if (total <= 0) return;
  if (p.cand_cap > 16384) throw std::runtime_error("detect_decode: cand_cap > 16384");
  if (p.f32)
    hipLaunchKernelGGL(decode_kernel<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(decode_kernel<bf16>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

// ------------------------------------------------------------------ NMS
// One 1024-thread workgroup per image.  Candidates are sorted in LDS by a
// 64-bit key (class asc, score desc, anchor asc) with a bitonic network, then the
// greedy pass walks the sorted list: a suppressed entry costs nothing, a kept
// entry costs one parallel IoU sweep over the rest of its class segment and
// one barrier.
constexpr int NMS_THREADS = 1024;

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(const NmsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int n_img = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  if (b >= n_img) return;
  const int tid = threadIdx.x;
  int n = p.cand_count[b];
  n = n < p.cand_cap ? n : p.cand_cap;
  int P = 2;
  while (P < n) P <<= 1;
  unsigned long long* keys = (unsigned long long*)smem;
  unsigned char* removed = smem + sizeof(unsigned long long) * P;
  const Candidate* cand = p.cand + (size_t)b * p.cand_cap;

  for (int i = tid; i < P; i += NMS_THREADS) {
    unsigned long long k = ~0ull;
    if (i < n) {
      // key = [cls:7][score desc:29][anchor:14][slot:14]: class asc, score desc, ties broken by
      // anchor index (deterministic; atomics make slot order vary), slot recovers the candidate
      const Candidate c = cand[i];
      const unsigned bits = __float_as_uint(c.score);
      unsigned diff = bits <= 0x3F800000u ? 0x3F800000u - bits : 0u;
      diff = diff < (1u << 29) ? diff : (1u << 29) - 1u;
      k = ((unsigned long long)(unsigned)(c.cls & 127) << 57) | ((unsigned long long)diff << 28) |
          ((unsigned long long)(unsigned)(c.anchor & 0x3FFF) << 14) | (unsigned long long)i;
      removed[i] = 0;
    }
    keys[i] = k;
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += NMS_THREADS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], c = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > c) == up) { keys[i] = c; keys[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }

  const ImageMeta m = p.meta[b];
  const float inv = 1.0f / m.scale;
  int kept = 0;
  for (int i = 0; i < n; ++i) {
    if (removed[i]) continue;  // block-uniform: written before the last barrier
    const unsigned long long ki = keys[i];
    const int ci = (int)(ki >> 57);
    const Candidate bi = cand[ki & 0x3FFF];
    if (tid == 0 && kept < p.max_det) {
      Detection d;
      d.x1 = fminf(fmaxf((bi.x1 - (float)m.pad_w) * inv, 0.f), (float)m.w);
      d.y1 = fminf(fmaxf((bi.y1 - (float)m.pad_h) * inv, 0.f), (float)m.h);
      d.x2 = fminf(fmaxf((bi.x2 - (float)m.pad_w) * inv, 0.f), (float)m.w);
      d.y2 = fminf(fmaxf((bi.y2 - (float)m.pad_h) * inv, 0.f), (float)m.h);
      d.conf = bi.score;
      d.cls = bi.cls;
      d.pad_[0] = d.pad_[1] = 0.f;
      p.det[(size_t)b * p.max_det + kept] = d;
    }
    ++kept;
    const float area_i = (bi.x2 - bi.x1) * (bi.y2 - bi.y1);
    for (int j = i + 1 + tid; j < n; j += NMS_THREADS) {
      const unsigned long long kj = keys[j];
      if ((int)(kj >> 57) != ci) break;
      if (removed[j]) continue;
      const Candidate bj = cand[kj & 0x3FFF];
      const float xx1 = fmaxf(bi.x1, bj.x1), yy1 = fmaxf(bi.y1, bj.y1);
      const float xx2 = fminf(bi.x2, bj.x2), yy2 = fminf(bi.y2, bj.y2);
      const float inter = fmaxf(0.f, xx2 - xx1) * fmaxf(0.f, yy2 - yy1);
      const float area_j = (bj.x2 - bj.x1) * (bj.y2 - bj.y1);
      const float iou = inter / (area_i + area_j - inter + 1e-6f);
      if (iou > p.iou_thr) removed[j] = 1;
    }
    __syncthreads();
  }
  if (tid == 0) p.det_count[b] = kept;
}

void prepare_kernels() {
  static bool done = false;
  if (done) return;
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)nms_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
  ir_prepare();
  head_pool_f32_prepare();
  x3_halo_prepare();
  x3g_prepare();
  c3_x3_prepare();
  x3hg_prepare();
  stem_s2_f32_prepare();
  ARENA_HIP_CHECK(hipFuncSetAttribute((const void*)sppf_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
  done = true;
}

void nms(const NmsParams& p, hipStream_t s) {
  if (p.cand_cap > 16384) throw std::runtime_error("nms: cand_cap > 16384");
  int P = 2;
  while (P < p.cand_cap) P <<= 1;
  const size_t lds = (size_t)P * 9;
  if (lds > 160 * 1024) throw std::runtime_error("nms: LDS budget exceeded");
  if (p.B <= 0) return;
  hipLaunchKernelGGL(nms_kernel, dim3(p.B), dim3(NMS_THREADS), lds, s, p);
}

// ------------------------------------------------------------------ crop plan
__global__ __launch_bounds__(256) void crop_plan_kernel(const CropPlanParams p) {
  __shared__ int offs[1024 + 1];
  const int n_img = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  const int tid = threadIdx.x;
  if (p.whole) {
    // classifier-only programs: image b is crop b (its full extent)
    for (int b = tid; b < n_img; b += blockDim.x) {
      const ImageMeta m = p.meta[b];
      Detection d;
      d.x1 = 0.f; d.y1 = 0.f; d.x2 = (float)m.w; d.y2 = (float)m.h;
      d.conf = 1.f; d.cls = -1; d.pad_[0] = d.pad_[1] = 0.f;
      p.det[(size_t)b * p.max_det] = d;
      p.det_count[b] = 1;
      CropRef r;
      r.img = b; r.x1 = 0; r.y1 = 0; r.x2 = m.w; r.y2 = m.h; r.det = 0; r.pad_[0] = r.pad_[1] = 0;
      p.crops[b] = r;
    }
    if (tid == 0) {
      Ctrl* c = p.ctrl;
      c->total_crops = n_img;
      int rem = n_img - c->crop_base;
      rem = rem < 0 ? 0 : rem;
      c->n_crops = rem < p.crop_cap ? rem : p.crop_cap;
    }
    return;
  }
  // Per-image crop offsets: every count is loaded at once, wave 0 scans them in 64-wide chunks
  // (a serial loop over det_count[] paid one global latency per image).
  for (int b = tid; b < n_img; b += blockDim.x) {
    const int k = p.det_count[b];
    offs[b + 1] = k < p.max_det ? k : p.max_det;
  }
  if (tid == 0) offs[0] = 0;
  __syncthreads();
  if (tid < 64) {
    int carry = 0;
    for (int base = 0; base < n_img; base += 64) {
      const int i = base + tid;
      int v = i < n_img ? offs[i + 1] : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (tid >= o) v += u;
      }
      if (i < n_img) offs[i + 1] = v + carry;
      carry += __shfl(v, 63, 64);
    }
    if (tid == 0) {
      Ctrl* c = p.ctrl;
      c->total_crops = carry;
      int rem = carry - c->crop_base;
      rem = rem < 0 ? 0 : rem;
      c->n_crops = rem < p.crop_cap ? rem : p.crop_cap;
    }
  }
  __syncthreads();
  // one crop per thread: image = last b with offs[b] <= i (binary search over the LDS offsets)
  const int total = offs[n_img];
  for (int i = tid; i < total; i += blockDim.x) {
    int lo = 0, hi = n_img - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (offs[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const int b = lo, d = i - offs[lo];
    const ImageMeta m = p.meta[b];
    const Detection det = p.det[(size_t)b * p.max_det + d];
    CropRef r;
    r.img = b;
    r.x1 = max(0, (int)det.x1);
    r.y1 = max(0, (int)det.y1);
    r.x2 = min(m.w, (int)det.x2);
    r.y2 = min(m.h, (int)det.y2);
    r.det = d;
    r.pad_[0] = r.pad_[1] = 0;
    p.crops[i] = r;
  }
}

void crop_plan(const CropPlanParams& p, hipStream_t s) {
  if (p.B > 1024) throw std::runtime_error("crop_plan: batch > 1024");
  hipLaunchKernelGGL(crop_plan_kernel, dim3(1), dim3(256), 0, s, p);
}

}  // namespace arena

namespace arena {

// Raw detector output in the reference's ONNX contract: per image
// [4 + nc, A] fp32 = (cx, cy, w, h) in letterbox pixels followed by the
// sigmoid class scores, for all A = 8400 anchors (experiment.yaml:199-207),
// i.e. what Triton's "yolov5n" model returns to the reference gateway.
template <typename T>
__global__ __launch_bounds__(256) void yolo_raw_kernel(const YoloRawParams p) {
  const int n_img = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  const int A0 = p.hw[0] * p.hw[0], A1 = p.hw[1] * p.hw[1], A2 = p.hw[2] * p.hw[2];
  const int A = A0 + A1 + A2;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)n_img * A) return;
  const int b = (int)(tid / A);
  const int a = (int)(tid - (long)b * A);
  int l, r;
  if (a < A0) { l = 0; r = a; } else if (a < A0 + A1) { l = 1; r = a - A0; } else { l = 2; r = a - A0 - A1; }
  const int hw = p.hw[l];
  const T* px = (const T*)p.head[l] + ((size_t)b * hw * hw + r) * p.xs[l];
  float* out = (float*)((uint8_t*)p.out + (size_t)b * p.out_stride);
  float dist[4];
#pragma unroll
  for (int side = 0; side < 4; ++side) {
    float v[16];
    load8(px + side * 16, v);
    load8(px + side * 16 + 8, v + 8);
    float mx = v[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, v[i]);
    float se = 0.f, sw = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = exp_t<T>(v[i] - mx);
      se += e;
      sw += e * (float)i;
    }
    dist[side] = sw / se;
  }
  const int gy = r / hw, gx = r - (r / hw) * hw;
  const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f, s = p.stride[l];
  const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
  out[0 * A + a] = (x1 + x2) * 0.5f * s;
  out[1 * A + a] = (y1 + y2) * 0.5f * s;
  out[2 * A + a] = (x2 - x1) * s;
  out[3 * A + a] = (y2 - y1) * s;
  for (int g = 0; g < 10; ++g) {
    float v[8];
    load8(px + 64 + g * 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[(size_t)(4 + g * 8 + i) * A + a] = 1.0f / (1.0f + exp_t<T>(-v[i]));
  }
}

void yolo_raw(const YoloRawParams& p, hipStream_t s) {
  const long A = (long)p.hw[0] * p.hw[0] + (long)p.hw[1] * p.hw[1] + (long)p.hw[2] * p.hw[2];
  if (p.out_stride < (size_t)A * 84 * 4) throw std::runtime_error("yolo_raw: output stride too small");
  const long total = A * p.B;
  if (total <= 0) return;
  if (p.f32)
    hipLaunchKernelGGL(yolo_raw_kernel<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(yolo_raw_kernel<bf16>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
}

}  // namespace arena
