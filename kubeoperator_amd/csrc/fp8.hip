// FP8 (OCP E4M3, the gfx950 format) per-tensor quantization for the FP8 GEMM path.
//
// gfx950's matrix cores run FP8 at twice the bf16 rate; hipBLASLt's E4M3 GEMMs reach 2.6-3.3 PF/s at the
// Llama-3-8B projection shapes against 1.2-1.55 PF/s in bf16 (tools/fp8_gemm_probe.py). A GEMM operand is
// quantized with "current scaling": scale = amax(|x|) / 448 (the E4M3 maximum), x8 = rne(x / scale), and the
// GEMM multiplies the dequantization scales back in (torch._scaled_mm scale_a / scale_b).
//
// Two streaming passes: fp8_amax_kernel reduces |x| to one partial maximum per workgroup (at most
// kFp8AmaxBlocks of them: no atomics and no zeroed scratch, so no memset launch per quantization), then
// fp8_cast_kernel reduces the partials in every workgroup, writes the scale and converts 8 values per lane
// with v_cvt_pk_fp8_f32 (two per instruction) after clamping to +-448, storing 8 bytes per lane. The second
// read of x mostly hits the 256 MB Infinity Cache.
#include "common.h"
#include "kernels.h"

namespace kop {

namespace {
constexpr float kE4M3Max = 448.f;
constexpr int kBlock = 256;
}  // namespace

// Partial maxima, one per workgroup (no atomics, no zero-initialised scratch): the cast kernel reduces them.
__global__ void __launch_bounds__(kBlock) fp8_amax_kernel(const bf16_t* __restrict__ x, int64_t n8, int64_t n,
                                                          float* __restrict__ partial) {
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
  if (threadIdx.x == 0) partial[blockIdx.x] = m;
}

// amax over the partial maxima of fp8_amax_kernel (every workgroup reduces the few hundred floats itself)
__device__ __forceinline__ float reduce_partials(const float* __restrict__ partial, int np) {
  __shared__ float red[kBlock / kWave];
  float m = 0.f;
  for (int i = threadIdx.x; i < np; i += kBlock) m = fmaxf(m, partial[i]);
  return block_max<kBlock / kWave>(m, red);
}

__device__ __forceinline__ uint32_t cvt4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

__global__ void __launch_bounds__(kBlock) fp8_cast_kernel(const bf16_t* __restrict__ x, int64_t n8, int64_t n,
                                                          const float* __restrict__ partial, int np,
                                                          uint8_t* __restrict__ out, float* __restrict__ scale) {
  const float a = reduce_partials(partial, np);
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

// Cast with a known dequantization scale (the operand's scale from its earlier quantization): one pass.
__global__ void __launch_bounds__(kBlock) fp8_cast_scaled_kernel(const bf16_t* __restrict__ x, int64_t n8,
                                                                 const float* __restrict__ scale,
                                                                 uint8_t* __restrict__ out) {
  const float inv = 1.f / *scale;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x2* ov = reinterpret_cast<u32x2*>(out);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf(f[e] * inv, -kE4M3Max), kE4M3Max);
    ov[i] = u32x2{cvt4_fp8(f[0], f[1], f[2], f[3]), cvt4_fp8(f[4], f[5], f[6], f[7])};
  }
}

// Transpose + cast with a known scale: out[c][r] = e4m3(in[r][c] / scale). The weight-gradient GEMM
// dW = dY^T X wants both operands K-contiguous (K = tokens); the bf16 path already materialises dY^T and
// X^T (csrc/transpose.hip), and writing them as E4M3 halves those writes. Same tiling as
// transpose_wide_kernel<true>: 64 x 128 tiles through a 65-dword-pitch LDS image, row tiles fastest; each
// lane writes 8 output bytes (8 consecutive rows of one column).
__global__ void __launch_bounds__(256) fp8_transpose_cast_kernel(const bf16_t* __restrict__ in,
                                                                 uint8_t* __restrict__ out, int64_t R, int64_t C,
                                                                 int64_t ldi, int64_t ldo,
                                                                 const float* __restrict__ scale) {
  constexpr int TR = 64, TC = 128, P = 65;
  __shared__ uint32_t lds[TR * P];
  const int t = threadIdx.x;
  const float inv = 1.f / *scale;
  const int64_t tiles_r = (R + TR - 1) / TR;
  const int64_t tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
  const int64_t r0 = tr * TR, c0 = tc * TC;
  const bool full = r0 + TR <= R && c0 + TC <= C;
  u32x4 v[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = p * 16 + (t >> 4), ch = t & 15;
    const int64_t gr = r0 + row, gc = c0 + ch * 8;
    v[p] = u32x4{0u, 0u, 0u, 0u};
    if (full || (gr < R && gc < C)) v[p] = *reinterpret_cast<const u32x4*>(in + gr * ldi + gc);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = p * 16 + (t >> 4), ch = t & 15;
    uint32_t* d = lds + row * P + ch * 4;
    d[0] = v[p][0];
    d[1] = v[p][1];
    d[2] = v[p][2];
    d[3] = v[p][3];
  }
  __syncthreads();
  const int chunk = t & 7;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pair = (t >> 3) + 32 * j;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = lds[(chunk * 8 + i) * P + pair];
    float lo[8], hi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      lo[i] = fminf(fmaxf(__uint_as_float(w[i] << 16) * inv, -kE4M3Max), kE4M3Max);
      hi[i] = fminf(fmaxf(__uint_as_float(w[i] & 0xffff0000u) * inv, -kE4M3Max), kE4M3Max);
    }
    const int64_t oc = c0 + 2 * pair, orr = r0 + chunk * 8;
    if (full || (oc < C && orr < R))
      *reinterpret_cast<u32x2*>(out + oc * ldo + orr) =
          u32x2{cvt4_fp8(lo[0], lo[1], lo[2], lo[3]), cvt4_fp8(lo[4], lo[5], lo[6], lo[7])};
    if (full || (oc + 1 < C && orr < R))
      *reinterpret_cast<u32x2*>(out + (oc + 1) * ldo + orr) =
          u32x2{cvt4_fp8(hi[0], hi[1], hi[2], hi[3]), cvt4_fp8(hi[4], hi[5], hi[6], hi[7])};
  }
}

int fp8_cast_scaled(const bf16_t* x, int64_t n, const float* scale, uint8_t* out, hipStream_t stream) {
  if (n % 8 || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 7)) return -1;
  if (n == 0) return 0;
  fp8_cast_scaled_kernel<<<stream_grid(n / 8, kBlock), kBlock, 0, stream>>>(x, n / 8, scale, out);
  KOP_CHECK_LAUNCH();
  return 0;
}

int fp8_transpose_cast(const bf16_t* in, uint8_t* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                       const float* scale, hipStream_t stream) {
  if (R % 8 || C % 8 || ldi % 8 || ldo % 8) return -1;
  const int64_t n = ((R + 63) / 64) * ((C + 127) / 128);
  if (n == 0) return 0;
  if (n > 0x7fffffff) return -2;
  fp8_transpose_cast_kernel<<<(unsigned)n, 256, 0, stream>>>(in, out, R, C, ldi, ldo, scale);
  KOP_CHECK_LAUNCH();
  return 0;
}

int fp8_quantize(const bf16_t* x, int64_t n, uint8_t* out, float* scale, float* partial_ws, hipStream_t stream) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 7)) return -1;
  const int64_t n8 = n / 8;
  int agrid = stream_grid(n8 > 0 ? n8 : 1, kBlock);
  if (agrid > kFp8AmaxBlocks) agrid = kFp8AmaxBlocks;
  const int grid = stream_grid(n8 > 0 ? n8 : 1, kBlock);
  fp8_amax_kernel<<<agrid, kBlock, 0, stream>>>(x, n8, n, partial_ws);
  fp8_cast_kernel<<<grid, kBlock, 0, stream>>>(x, n8, n, partial_ws, agrid, out, scale);
  KOP_CHECK_LAUNCH();
  return 0;
}

}  // namespace kop
