// Shared device-side helpers for the gfx950 (CDNA4) kernels of the arena.
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16; a tensor "view" is (base pointer already
//     offset to its channel slice, pixel stride in elements). Channel counts,
//     slice offsets and pixel strides are multiples of 8, so 16-byte vector
//     loads/stores are always aligned.
//   * batch sizes may be clamped at run time by a device-side counter
//     (`bdev`): the hipGraph of a batch bucket is captured once for the
//     bucket's capacity and the blocks past the live batch exit immediately.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace arena {

enum Act : int { ACT_NONE = 0, ACT_SILU = 1, ACT_RELU6 = 2 };

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// SiLU as v * rcp(1 + exp(-v)): v_exp_f32 + v_rcp_f32 (8-cycle issue each) instead
// of the ~10-instruction IEEE division sequence; error ~1 ulp of fp32, far below
// the bf16 rounding of every stored activation.
__device__ __forceinline__ float silu(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }

// ReLU6 as one v_med3_f32
__device__ __forceinline__ float relu6f(float v) { return __builtin_amdgcn_fmed3f(v, 0.0f, 6.0f); }

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_SILU) return silu(v);
  if (act == ACT_RELU6) return relu6f(v);
  return v;
}

// Unpack / pack 8 bf16 carried in a uint4.
__device__ __forceinline__ void unpack8(uint4 u, float* f) {
  bf16x8 v = __builtin_bit_cast(bf16x8, u);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  return __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ void unpack4(uint2 u, float* f) {
  bf16x4 v = __builtin_bit_cast(bf16x4, u);
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ uint2 pack4(const float* f) {
  bf16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (bf16)f[i];
  return __builtin_bit_cast(uint2, v);
}

// 8 consecutive elements of an NHWC row as fp32, for kernels templated on the
// activation type (bf16 pipeline / exact-fp32 pipeline).
__device__ __forceinline__ void load8(const bf16* p, float* v) { unpack8(*(const uint4*)p, v); }
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(bf16* p, const float* v) { *(uint4*)p = pack8(v); }
__device__ __forceinline__ void store8(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// 16-byte global load that is zero when !ok, without a branch and without
// the "select(ok, global ptr, &local_zero)" pattern the compiler otherwise
// forms for `ok ? *p : zero` — that pattern turns the load into a FLAT load
// and puts a zero vector in scratch memory (measured: 2-3x slower kernels).
// `safe` must be any readable global address (e.g. the tensor base).
__device__ __forceinline__ uint4 load16_or_zero(const void* p, const void* safe, bool ok) {
  const uint4 v = *(const uint4*)(ok ? p : safe);
  return ok ? v : make_uint4(0u, 0u, 0u, 0u);
}

__device__ __forceinline__ int live_batch(int cap, const int* bdev) {
  if (bdev == nullptr) return cap;
  int n = *bdev;
  return n < cap ? (n < 0 ? 0 : n) : cap;
}

// Wave-level reductions (64 lanes).
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace arena

#define ARENA_HIP_CHECK(expr)                                                     \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    }                                                                             \
  } while (0)
