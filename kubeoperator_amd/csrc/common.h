// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of kubeoperator_amd.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; block sizes are multiples of 64;
//   * bf16 tensors are moved as raw 16-bit patterns in 16-byte vectors (8 x bf16 per lane per load),
//     converted to fp32 for math, and rounded back with the hardware v_cvt_pk_bf16_f32 (RNE, NaN-safe);
//   * every launcher is a plain C++ function taking raw device pointers + hipStream_t, so the kernel
//     translation units compile in seconds without PyTorch headers (bindings.cpp adapts tensors).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace kop {

typedef uint16_t bf16_t;  // raw bf16 bit pattern
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

// pack two floats into one dword of two bf16 (lo in bits 0..15), round-to-nearest-even: a vector
// conversion lowers to ONE v_cvt_pk_bf16_f32 (two scalar conversions + an OR would be three instructions)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// 8 x bf16 <-> 8 x f32 for a 16-byte vector
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack2(f[2 * i], f[2 * i + 1]);
  return v;
}

// Wave reductions without the LDS pipe: DPP inside each 16-lane row (lane ^ 1, ^ 2, then the mirrored quad and
// half), v_permlane16_swap / v_permlane32_swap across rows. Every step adds a value to its partner's, so all 64
// lanes end with the same total (a + b == b + a). (A __shfl_xor loop is six ds_bpermute round trips.)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swap16_f32(float v, bool mx) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return mx ? fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1])) : __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float swap32_f32(float v, bool mx) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return mx ? fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1])) : __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1, 0, 3, 2]: lane ^ 1
  v += dpp_f32<0x4E>(v);   // quad_perm [2, 3, 0, 1]: lane ^ 2
  v += dpp_f32<0x141>(v);  // row_half_mirror: the other quad of the 8-lane half
  v += dpp_f32<0x140>(v);  // row_mirror: the other half of the 16-lane row
  return swap32_f32(swap16_f32(v, false), false);
}
// sum over each aligned group of N lanes (N = 2 .. 64), every lane of a group ending with its total
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 2 || N == 4 || N == 8 || N == 16 || N == 32 || N == 64, "power-of-two group");
  v += dpp_f32<0xB1>(v);
  if constexpr (N >= 4) v += dpp_f32<0x4E>(v);
  if constexpr (N >= 8) v += dpp_f32<0x141>(v);
  if constexpr (N >= 16) v += dpp_f32<0x140>(v);
  if constexpr (N >= 32) v = swap16_f32(v, false);
  if constexpr (N >= 64) v = swap32_f32(v, false);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x140>(v));
  return swap32_f32(swap16_f32(v, true), true);
}

// Block-wide sum for blocks of NW waves; `red` must hold NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NW == 1) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  return t;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NW == 1) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Grid size for a memory-bound streaming kernel: enough blocks to fill 256 CUs several times, capped
// (Guideline 11: grid-stride the rest).
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace kop

#define KOP_CHECK_LAUNCH() (void)hipGetLastError()
