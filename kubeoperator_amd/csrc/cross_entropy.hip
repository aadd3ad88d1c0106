// Fused softmax cross-entropy for gfx950: one pass computes the row log-sum-exp (online max/sum),
// a second pass writes the gradient (softmax - onehot) * scale IN PLACE over the bf16 logits, so the
// [tokens, vocab] probabilities are never materialised in fp32 (V = 128,256 for Llama-3: 2 GB of bf16
// logits per 8k tokens instead of 4 GB fp32 probs + 2 GB grads).
//
// scale is read from device memory (1 / number of non-ignored targets, computed by ce_count_kernel) so
// the whole loss needs no host synchronisation.
#include "common.h"
#include "kernels.h"

namespace kop {

__global__ void ce_count_kernel(const int64_t* __restrict__ tgt, int64_t T, int64_t ignore_index, float* __restrict__ scale,
                                float extra) {
  __shared__ float red[16];
  float c = 0.f;
  for (int64_t i = threadIdx.x; i < T; i += blockDim.x) c += (tgt[i] != ignore_index) ? 1.f : 0.f;
  c = block_sum<16>(c, red);
  if (threadIdx.x == 0) scale[0] = extra / fmaxf(c, 1.f);
}

template <int NT, bool VEC>
__global__ void __launch_bounds__(NT) ce_fwd_kernel(bf16_t* __restrict__ logits, int64_t ld, int V,
                                                    const int64_t* __restrict__ tgt, int64_t ignore_index,
                                                    const float* __restrict__ scale_p, float* __restrict__ loss_rows,
                                                    float* __restrict__ lse_rows, int write_grad) {
  __shared__ float red_m[NT / 64], red_s[NT / 64];
  const int64_t row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int V8 = VEC ? (V >> 3) : 0;
  float m = -INFINITY, s = 0.f;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  for (int c = threadIdx.x; c < V8; c += NT) {
    float f[8];
    unpack8(xv[c], f);
    float cm = f[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) cm = fmaxf(cm, f[i]);
    const float nm = fmaxf(m, cm);
    float add = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) add += __expf(f[i] - nm);
    s = s * __expf(m - nm) + add;
    m = nm;
  }
  for (int i = V8 * 8 + threadIdx.x; i < V; i += NT) {
    const float f = bf2f(x[i]);
    const float nm = fmaxf(m, f);
    s = s * __expf(m - nm) + __expf(f - nm);
    m = nm;
  }
  // merge (m, s) across the wave then the block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if ((threadIdx.x & 63) == 0) {
    red_m[threadIdx.x >> 6] = m;
    red_s[threadIdx.x >> 6] = s;
  }
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) M = fmaxf(M, red_m[i]);
  float Ssum = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) Ssum += red_m[i] == -INFINITY ? 0.f : red_s[i] * __expf(red_m[i] - M);
  const float lse = M + __logf(Ssum);
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  if (threadIdx.x == 0) {
    lse_rows[row] = lse;
    loss_rows[row] = valid ? (lse - bf2f(x[t])) : 0.f;
  }
  if (!write_grad) return;
  __syncthreads();  // everyone has read x[t] above before it is overwritten
  const float sc = valid ? scale_p[0] : 0.f;
  u32x4* xw = reinterpret_cast<u32x4*>(x);
  for (int c = threadIdx.x; c < V8; c += NT) {
    float f[8];
    unpack8(xw[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p = __expf(f[i] - lse);
      f[i] = (p - ((int64_t)(c * 8 + i) == t ? 1.f : 0.f)) * sc;
    }
    xw[c] = pack8(f);
  }
  for (int i = V8 * 8 + threadIdx.x; i < V; i += NT) {
    const float p = __expf(bf2f(x[i]) - lse);
    x[i] = f2bf((p - (i == t ? 1.f : 0.f)) * sc);
  }
}

int cross_entropy_fwd(bf16_t* logits, int64_t ld, int64_t T, int V, const int64_t* tgt, int64_t ignore_index,
                      float* scale, float* loss_rows, float* lse_rows, bool write_grad, float grad_multiplier,
                      hipStream_t stream) {
  ce_count_kernel<<<1, 1024, 0, stream>>>(tgt, T, ignore_index, scale, grad_multiplier);
  const bool vec = (ld % 8 == 0) && (reinterpret_cast<uintptr_t>(logits) % 16 == 0);
  if (vec)
    ce_fwd_kernel<512, true><<<(unsigned)T, 512, 0, stream>>>(logits, ld, V, tgt, ignore_index, scale, loss_rows,
                                                               lse_rows, write_grad ? 1 : 0);
  else
    ce_fwd_kernel<512, false><<<(unsigned)T, 512, 0, stream>>>(logits, ld, V, tgt, ignore_index, scale, loss_rows,
                                                                lse_rows, write_grad ? 1 : 0);
  return 0;
}

}  // namespace kop
