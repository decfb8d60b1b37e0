// Device-side preprocessing: letterbox for the detector (K1) and the
// crop-gather + resize + ImageNet normalisation for the classifier (K9).
//
// Reference semantics reproduced here:
//   letterbox: src/shared/processing/transforms.py:118-180 (scale =
//     min(T/h, T/w), new size int-truncated, floor-centred pad, gray 114,
//     cv2 INTER_LINEAR) followed by /255 and HWC->CHW in
//     src/shared/processing/yolo_preprocess.py:154-167.
//   crop: src/shared/processing/mobilenet_preprocess.py:236-269 (int()
//     truncation, clamp, zero-area -> 1x1 black) and :134-160 (direct 224x224
//     INTER_LINEAR resize, (x/255-mean)/std).
// INTER_LINEAR geometry: src = (dst + 0.5) * (src_size / dst_size) - 0.5,
// clamped to the border; the interpolated uint8 value is rounded before
// normalisation, as cv2 returns a uint8 image.
//
// Both kernels emit space-to-depth(2) layouts so that the stride-2 stem convs
// become dense stride-1 convs with 16 (12 live) input channels: YOLO's 6x6/s2
// stem becomes a 3x3/s1 conv, MobileNet's 3x3/s2 stem a 2x2/s1 conv.
#include "common.h"
#include "launch.h"
#include "letterbox.h"

namespace arena {

template <typename T>
__device__ __forceinline__ void store16(T* dst, const float* v) {
  store8(dst, v);
  store8(dst + 8, v + 8);
}

template <typename T>
__global__ __launch_bounds__(256) void letterbox_s2d_kernel(const LetterboxParams p) {
  const int T2 = p.T >> 1;
  const int n_img = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  const long total = (long)n_img * T2 * T2;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int X = (int)(tid % T2);
  const int Y = (int)((tid / T2) % T2);
  const int b = (int)(tid / ((long)T2 * T2));
  float out[16];
  letterbox_s2d_px<T>(p.pool, p.meta[b], Y, X, out);
  out[12] = out[13] = out[14] = out[15] = 0.f;
  store16((T*)p.out + (size_t)tid * 16, out);
}

void letterbox_s2d(const LetterboxParams& p, hipStream_t s) {
  if (p.T % 2 != 0) throw std::runtime_error("letterbox_s2d: T must be even");
  const long total = (long)p.B * (p.T / 2) * (p.T / 2);
  if (total <= 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (p.f32)
    hipLaunchKernelGGL(letterbox_s2d_kernel<float>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(letterbox_s2d_kernel<bf16>, grid, dim3(256), 0, s, p);
}

template <typename T>
__global__ __launch_bounds__(256) void crop_gather_s2d_kernel(const CropGatherParams p) {
  const int S2 = p.S >> 1;
  int n = p.cap;
  if (p.ctrl != nullptr) n = live_batch(p.cap, &p.ctrl->n_crops);
  const long total = (long)n * S2 * S2;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int X = (int)(tid % S2);
  const int Y = (int)((tid / S2) % S2);
  const int i = (int)(tid / ((long)S2 * S2));
  const int base = p.ctrl != nullptr ? p.ctrl->crop_base : 0;
  const CropRef cr = p.crops[base + i];
  const ImageMeta m = p.meta[cr.img];
  const int cw = cr.x2 - cr.x1, ch = cr.y2 - cr.y1;
  float out[16];
  const bool empty = cw <= 0 || ch <= 0;
  const float sx = empty ? 1.f : (float)((double)cw / (double)p.S);
  const float sy = empty ? 1.f : (float)((double)ch / (double)p.S);
  const uint8_t* img = p.pool + m.offset + ((size_t)cr.y1 * m.w + cr.x1) * 3;
#pragma unroll
  for (int pq = 0; pq < 4; ++pq) {
    const int oy = 2 * Y + (pq >> 1), ox = 2 * X + (pq & 1);
    float rgb[3] = {0.f, 0.f, 0.f};
    if (!empty) bilinear_rgb(img, m.w, lin_tap(oy, sy, ch), lin_tap(ox, sx, cw), rgb);
#pragma unroll
    for (int c = 0; c < 3; ++c) out[pq * 3 + c] = (div255<T>(rgb[c]) - p.mean[c]) * p.inv_std[c];
  }
  out[12] = out[13] = out[14] = out[15] = 0.f;
  store16((T*)p.out + (size_t)tid * 16, out);
}

void crop_gather_s2d(const CropGatherParams& p, hipStream_t s) {
  if (p.S % 2 != 0) throw std::runtime_error("crop_gather_s2d: S must be even");
  const long total = (long)p.cap * (p.S / 2) * (p.S / 2);
  if (total <= 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (p.f32)
    hipLaunchKernelGGL(crop_gather_s2d_kernel<float>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(crop_gather_s2d_kernel<bf16>, grid, dim3(256), 0, s, p);
}

}  // namespace arena

namespace arena {

// Reference-contract tensor input (KServe "images" / "input": FP32 NCHW
// [3, S, S], already normalised by the client as in the reference gateway,
// architectures/triton/gateway/app/pipeline.py:131-139) -> space-to-depth
// [S/2, S/2, 16] (bf16 or fp32) for the s2d stem convs.
template <typename T>
__global__ __launch_bounds__(256) void tensor_in_s2d_kernel(const TensorInParams p) {
  const int S2 = p.S >> 1;
  const int n = live_batch(p.B, p.ctrl ? &p.ctrl->n_images : nullptr);
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)n * S2 * S2) return;
  const int X = (int)(tid % S2);
  const int Y = (int)((tid / S2) % S2);
  const int b = (int)(tid / ((long)S2 * S2));
  const float* src = (const float*)(p.pool + p.meta[b].offset);
  const size_t plane = (size_t)p.S * p.S;
  float out[16];
#pragma unroll
  for (int pq = 0; pq < 4; ++pq) {
    const int y = 2 * Y + (pq >> 1), x = 2 * X + (pq & 1);
#pragma unroll
    for (int c = 0; c < 3; ++c) out[pq * 3 + c] = src[c * plane + (size_t)y * p.S + x];
  }
  out[12] = out[13] = out[14] = out[15] = 0.f;
  store16((T*)p.out + (size_t)tid * 16, out);
}

void tensor_in_s2d(const TensorInParams& p, hipStream_t s) {
  if (p.S % 2 != 0) throw std::runtime_error("tensor_in_s2d: S must be even");
  const long total = (long)p.B * (p.S / 2) * (p.S / 2);
  if (total <= 0) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (p.f32)
    hipLaunchKernelGGL(tensor_in_s2d_kernel<float>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(tensor_in_s2d_kernel<bf16>, grid, dim3(256), 0, s, p);
}

}  // namespace arena
