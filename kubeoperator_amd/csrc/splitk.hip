// Split-K reduction of the weight-gradient GEMM for gfx950: out (+)= sum_s part[s], fp32 partials -> bf16 or fp32
// gradient buffer, rounded once.
//
// Why: dW = dY^T X at GPT-2-small widths is a few dozen 256 x 256 output tiles (768 x 768: 9) reduced over
// T = 32768 token rows, so hipBLASLt's single GEMM keeps most of the 256 CUs idle (0.31-0.69 PF/s). Cutting T
// into s chunks as ONE batched GEMM with fp32 outputs multiplies the tiles by s (proj 768 x 768: 0.124 ms ->
// 0.046 ms for the GEMM at s = 16; profiles/r3_wgrad_splitk_probe.jsonl); this kernel then folds the s partial
// planes into the gradient (and adds the accumulated micro-batches) in one pass instead of a sum + cast + add.
//
// Memory-bound: each thread owns 8 consecutive elements (two 16-B loads per plane, 4 planes in flight), grid-
// strided; the output is read only when accumulating.
#include "common.h"
#include "kernels.h"

namespace kop {

template <bool ACC, bool OUT_F32>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ part, int S, int64_t n8,
                                                            int64_t plane, void* __restrict__ out) {
  const int64_t step = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += step) {
    const f32x4* p = reinterpret_cast<const f32x4*>(part) + 2 * i;
    const int64_t pl4 = plane >> 2;
    f32x4 a = p[0], b = p[1];
    int s = 1;
    for (; s + 3 < S; s += 4) {
      f32x4 a1 = p[s * pl4], b1 = p[s * pl4 + 1];
      f32x4 a2 = p[(s + 1) * pl4], b2 = p[(s + 1) * pl4 + 1];
      f32x4 a3 = p[(s + 2) * pl4], b3 = p[(s + 2) * pl4 + 1];
      f32x4 a4 = p[(s + 3) * pl4], b4 = p[(s + 3) * pl4 + 1];
      a += (a1 + a2) + (a3 + a4);
      b += (b1 + b2) + (b3 + b4);
    }
    for (; s < S; ++s) {
      a += p[s * pl4];
      b += p[s * pl4 + 1];
    }
    if (OUT_F32) {
      f32x4* o = reinterpret_cast<f32x4*>(out) + 2 * i;
      if (ACC) {
        a += o[0];
        b += o[1];
      }
      o[0] = a;
      o[1] = b;
    } else {
      u32x4* o = reinterpret_cast<u32x4*>(out) + i;
      float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      if (ACC) {
        float g[8];
        unpack8(*o, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += g[j];
      }
      *o = pack8(f);
    }
  }
}

int splitk_reduce(const float* part, int S, int64_t n, void* out, bool out_f32, bool accumulate, hipStream_t stream) {
  if (S < 1 || n % 8 != 0 || n <= 0) return -1;
  const int64_t n8 = n / 8;
  int64_t blocks = (n8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  const dim3 g((unsigned)blocks);
  if (out_f32) {
    if (accumulate) splitk_reduce_kernel<true, true><<<g, 256, 0, stream>>>(part, S, n8, n, out);
    else splitk_reduce_kernel<false, true><<<g, 256, 0, stream>>>(part, S, n8, n, out);
  } else {
    if (accumulate) splitk_reduce_kernel<true, false><<<g, 256, 0, stream>>>(part, S, n8, n, out);
    else splitk_reduce_kernel<false, false><<<g, 256, 0, stream>>>(part, S, n8, n, out);
  }
  return 0;
}

}  // namespace kop
