// Decode projections: y[M, N] = x[M, K] . W[N, K]^T for M <= 8 token rows (gfx950).
// A decode step streams every weight once (16.3 GB per Llama-3-8B step) with almost no reuse, so the op is an
// HBM read at whatever rate the kernel keeps in flight. hipBLASLt's small-M GEMM tiles reach ~3.5 TB/s
// (profiles/r2_decode_llama3_8b_kernel_stats.csv). Here each wave owns R = 4 weight rows and walks K with 16-B
// loads, two 512-element chunks per iteration (8 row loads in flight per lane); the M activation chunks
// come from L2 and feed all 4 rows. fp32 accumulation, one cross-lane reduction per output at the end.
// No LDS, few VGPRs: many waves per SIMD keep enough bytes in flight.
#include "common.h"
#include "kernels.h"

namespace kop {

template <int M>
__global__ void __launch_bounds__(256) gemv_bf16_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                        bf16_t* __restrict__ y, int N, int K, int64_t xs, int64_t ws,
                                                        int64_t ys) {
  constexpr int R = 4;
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (n0 >= N) return;  // wave-uniform
  const bf16_t* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = w + (int64_t)min(n0 + r, N - 1) * ws;
  float acc[M][R];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
  for (int k = lane * 8; k < K; k += 1024) {
    u32x4 wv[2][R];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < R; ++r) wv[h][r] = *reinterpret_cast<const u32x4*>(wr[r] + k + 512 * h);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float xf[8];
        unpack8(*reinterpret_cast<const u32x4*>(x + m * xs + k + 512 * h), xf);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float wf[8];
          unpack8(wv[h][r], wf);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[m][r] = fmaf(xf[e], wf[e], acc[m][r]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc[m][r] = wave_sum(acc[m][r]);
    }
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (n0 + r < N) y[m * ys + n0 + r] = f2bf(acc[m][r]);
  }
}

int gemv_bf16(const bf16_t* x, const bf16_t* w, bf16_t* y, int M, int N, int K, int64_t xs, int64_t ws, int64_t ys,
              hipStream_t stream) {
  // K in whole 1024-element steps (two 16-B chunks per lane per iteration); rows 16-B aligned (checked by the caller)
  if (M < 1 || M > 8 || N < 1 || K < 1024 || K % 1024 != 0 || xs % 8 != 0 || ws % 8 != 0) return 1;
  const dim3 grid((N + 15) / 16);
  switch (M) {
#define KOP_GEMV_CASE(m)                                                                          \
  case m:                                                                                         \
    gemv_bf16_kernel<m><<<grid, 256, 0, stream>>>(x, w, y, N, K, xs, ws, ys);                    \
    break;
    KOP_GEMV_CASE(1) KOP_GEMV_CASE(2) KOP_GEMV_CASE(3) KOP_GEMV_CASE(4)
    KOP_GEMV_CASE(5) KOP_GEMV_CASE(6) KOP_GEMV_CASE(7) KOP_GEMV_CASE(8)
#undef KOP_GEMV_CASE
  }
  return 0;
}

}  // namespace kop
