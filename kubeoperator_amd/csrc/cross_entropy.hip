// Fused softmax cross-entropy for gfx950: one pass computes the row log-sum-exp (online max/sum),
// a second pass writes the gradient (softmax - onehot) * scale IN PLACE over the bf16 logits, so the
// [tokens, vocab] probabilities are never materialised in fp32 (V = 128,256 for Llama-3: 2 GB of bf16
// logits per 8k tokens instead of 4 GB fp32 probs + 2 GB grads).
//
// scale is read from device memory (1 / number of non-ignored targets, computed by ce_count_kernel) so
// the whole loss needs no host synchronisation.
#include <cstdlib>

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
  // pass 1 in the log2 domain: max on the raw logits, exp2(fma(f, log2 e, -m log2 e)) -- one FMA + one v_exp_f32 per
  // logit (the __expf form cost a subtract, a multiply and the exponential)
  constexpr float L2E = 1.4426950408889634f;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  for (int c = threadIdx.x; c < V8; c += NT) {
    float f[8];
    unpack8(xv[c], f);
    const float cm = fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])), fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7])));
    const float nm = fmaxf(m, cm);
    const float nb = -nm * L2E;
    float add = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) add += __builtin_amdgcn_exp2f(fmaf(f[i], L2E, nb));
    s = s * __builtin_amdgcn_exp2f((m - nm) * L2E) + add;
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
  const float xt = valid ? bf2f(x[t]) : 0.f;
  if (threadIdx.x == 0) {
    lse_rows[row] = lse;
    loss_rows[row] = valid ? (lse - xt) : 0.f;
  }
  if (!write_grad) return;
  __syncthreads();  // everyone has read x[t] above before it is overwritten
  const float sc = valid ? scale_p[0] : 0.f;
  // pass 2: (softmax - onehot) * scale = exp2(f log2 e - lse log2 e + log2 sc) for every logit (the scale folded into
  // the exponent: one FMA + one exponential + the pack), then the target's own element is rewritten once below
  // instead of an index compare per logit
  // |sc| goes into the exponent, its sign is applied after (a negative grad_multiplier flips every element; the sign
  // branch is uniform, so the common sc > 0 loop carries no extra multiply)
  const float b2 = sc != 0.f ? (__log2f(fabsf(sc)) - lse * L2E) : -INFINITY;
  const float sg = sc < 0.f ? -1.f : 1.f;
  u32x4* xw = reinterpret_cast<u32x4*>(x);
  for (int c = threadIdx.x; c < V8; c += NT) {
    float f[8];
    unpack8(xw[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = __builtin_amdgcn_exp2f(fmaf(f[i], L2E, b2));
    if (sc < 0.f) {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = -f[i];
    }
    xw[c] = pack8(f);
  }
  for (int i = V8 * 8 + threadIdx.x; i < V; i += NT) x[i] = f2bf(sg * __builtin_amdgcn_exp2f(fmaf(bf2f(x[i]), L2E, b2)));
  if (valid) {
    __syncthreads();  // the target's element has been written by its owner above
    if (threadIdx.x == 0) x[t] = f2bf((__expf(xt - lse) - 1.f) * sc);
  }
}

// Register-resident form (vocabularies up to NT * 8 * CPT = 65,536 logits at CPT 16: GPT-2's 50,304; CPT 32 for
// Llama-3's 128,256 spills at 256 VGPRs): every thread loads its CPT 16-byte chunks of the
// row once, keeps them in registers through the max, the sum and the gradient write, so the row is read from HBM
// once (the two-pass kernel above re-reads it, from the MALL at best: 2-3 row images per call). Max and sum are two
// plain block reductions -- no per-chunk online rescale.
template <int NT, int CPT>
__global__ void __launch_bounds__(NT) ce_fwd_reg_kernel(bf16_t* __restrict__ logits, int64_t ld, int V,
                                                        const int64_t* __restrict__ tgt, int64_t ignore_index,
                                                        const float* __restrict__ scale_p,
                                                        float* __restrict__ loss_rows, float* __restrict__ lse_rows,
                                                        int write_grad) {
  constexpr float L2E = 1.4426950408889634f;
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int V8 = V >> 3;
  u32x4* xw = reinterpret_cast<u32x4*>(x);
  u32x4 w[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = threadIdx.x + j * NT;
    w[j] = c < V8 ? xw[c] : u32x4{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};  // bf16 -inf pads
  }
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    float f[8];
    unpack8(w[j], f);
    m = fmaxf(m, fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])), fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7]))));
  }
  m = block_max<NT / 64>(m, red);
  const float nb = -m * L2E;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    float f[8];
    unpack8(w[j], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += __builtin_amdgcn_exp2f(fmaf(f[i], L2E, nb));
  }
  __syncthreads();  // red[] is reused by the second reduction
  s = block_sum<NT / 64>(s, red);
  const float lse = m + __logf(s);
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  const float xt = valid ? bf2f(x[t]) : 0.f;
  if (threadIdx.x == 0) {
    lse_rows[row] = lse;
    loss_rows[row] = valid ? (lse - xt) : 0.f;
  }
  if (!write_grad) return;
  const float sc = valid ? scale_p[0] : 0.f;
  const float b2 = sc != 0.f ? (__log2f(fabsf(sc)) - lse * L2E) : -INFINITY;  // sign applied below (two-pass kernel)
  __syncthreads();  // x[t] read above before any thread overwrites it
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = threadIdx.x + j * NT;
    if (c >= V8) break;
    float f[8];
    unpack8(w[j], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = __builtin_amdgcn_exp2f(fmaf(f[i], L2E, b2));
    if (sc < 0.f) {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = -f[i];
    }
    xw[c] = pack8(f);
  }
  if (valid) {
    __syncthreads();
    if (threadIdx.x == 0) x[t] = f2bf((__expf(xt - lse) - 1.f) * sc);
  }
}

int cross_entropy_fwd(bf16_t* logits, int64_t ld, int64_t T, int V, const int64_t* tgt, int64_t ignore_index,
                      float* scale, float* loss_rows, float* lse_rows, bool write_grad, float grad_multiplier,
                      hipStream_t stream) {
  ce_count_kernel<<<1, 1024, 0, stream>>>(tgt, T, ignore_index, scale, grad_multiplier);
  const bool vec = (ld % 8 == 0) && (reinterpret_cast<uintptr_t>(logits) % 16 == 0);
  static const bool reg = [] {
    const char* e = getenv("KOP_CE_REG");  // 1 (default): register-resident rows where they fit; 0: two passes
    return e == nullptr || atoi(e) != 0;
  }();
  if (vec && reg && V % 8 == 0) {
    const int cpt = ((V / 8) + 511) / 512;
    if (cpt <= 16) {
      ce_fwd_reg_kernel<512, 16><<<(unsigned)T, 512, 0, stream>>>(logits, ld, V, tgt, ignore_index, scale, loss_rows,
                                                                  lse_rows, write_grad ? 1 : 0);
      return 0;
    }
  }
  if (vec)
    ce_fwd_kernel<512, true><<<(unsigned)T, 512, 0, stream>>>(logits, ld, V, tgt, ignore_index, scale, loss_rows,
                                                               lse_rows, write_grad ? 1 : 0);
  else
    ce_fwd_kernel<512, false><<<(unsigned)T, 512, 0, stream>>>(logits, ld, V, tgt, ignore_index, scale, loss_rows,
                                                                lse_rows, write_grad ? 1 : 0);
  return 0;
}

}  // namespace kop
