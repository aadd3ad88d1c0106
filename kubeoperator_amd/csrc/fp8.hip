// FP8 (OCP E4M3, the gfx950 format) per-tensor quantization for the FP8 GEMM path.
//
// gfx950's matrix cores run FP8 at twice the bf16 rate; hipBLASLt's E4M3 GEMMs reach 2.6-3.3 PF/s at the
// Llama-3-8B projection shapes against 1.2-1.55 PF/s in bf16 (tools/fp8_gemm_probe.py). A GEMM operand is
// quantized with "current scaling": scale = amax(|x|) / 448 (the E4M3 maximum), x8 = rne(x / scale), and the
// GEMM multiplies the dequantization scales back in (torch._scaled_mm scale_a / scale_b).
//
// Two streaming passes: fp8_amax_kernel reduces |x| (one global atomic max per workgroup on the float's bit
// pattern -- non-negative floats order like unsigned integers), then fp8_cast_kernel reads the amax, writes
// the scale and converts 8 values per lane with v_cvt_pk_fp8_f32 (two per instruction) after clamping to
// +-448, storing 8 bytes per lane. The second read of x mostly hits the 256 MB Infinity Cache.
#include "common.h"
#include "kernels.h"

namespace kop {

namespace {
constexpr float kE4M3Max = 448.f;
constexpr int kBlock = 256;
}  // namespace

__global__ void __launch_bounds__(kBlock) fp8_amax_kernel(const bf16_t* __restrict__ x, int64_t n8, int64_t n,
                                                          unsigned* __restrict__ amax) {
  __shared__ float red[kBlock / kWave];
  float m = 0.f;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
  }
  if (blockIdx.x == 0)
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += kBlock) m = fmaxf(m, fabsf(bf2f(x[i])));
  m = block_max<kBlock / kWave>(m, red);
  if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(m));
}

__device__ __forceinline__ uint32_t cvt4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

__global__ void __launch_bounds__(kBlock) fp8_cast_kernel(const bf16_t* __restrict__ x, int64_t n8, int64_t n,
                                                          const unsigned* __restrict__ amax,
                                                          uint8_t* __restrict__ out, float* __restrict__ scale) {
  const float a = __uint_as_float(*amax);
  const float s = (a > 0.f && a < INFINITY) ? a / kE4M3Max : 1.f;
  const float inv = 1.f / s;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale = s;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x2* ov = reinterpret_cast<u32x2*>(out);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf(f[e] * inv, -kE4M3Max), kE4M3Max);
    ov[i] = u32x2{cvt4_fp8(f[0], f[1], f[2], f[3]), cvt4_fp8(f[4], f[5], f[6], f[7])};
  }
  if (blockIdx.x == 0)
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += kBlock) {
      const float v = fminf(fmaxf(bf2f(x[i]) * inv, -kE4M3Max), kE4M3Max);
      out[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
    }
}

int fp8_quantize(const bf16_t* x, int64_t n, uint8_t* out, float* scale, unsigned* amax_ws, hipStream_t stream) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 7)) return -1;
  const int64_t n8 = n / 8;
  const int grid = stream_grid(n8 > 0 ? n8 : 1, kBlock);
  (void)hipMemsetAsync(amax_ws, 0, sizeof(unsigned), stream);
  fp8_amax_kernel<<<grid, kBlock, 0, stream>>>(x, n8, n, amax_ws);
  fp8_cast_kernel<<<grid, kBlock, 0, stream>>>(x, n8, n, amax_ws, out, scale);
  KOP_CHECK_LAUNCH();
  return 0;
}

}  // namespace kop
