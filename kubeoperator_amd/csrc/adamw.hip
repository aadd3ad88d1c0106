// Fused AdamW over FLAT parameter storage for gfx950.
//
// The trainer keeps every parameter as a view into one contiguous bf16 buffer, every gradient as a
// view into one contiguous bf16 buffer, and the fp32 master weights / exp_avg / exp_avg_sq as three
// more contiguous fp32 buffers. The optimizer step is therefore ONE streaming launch per weight-decay
// region (no multi-tensor chunk lists, no per-parameter launches): 28 bytes per parameter
// (2 grad + 12 state read, 12 state + 2 param written), 16-byte vector accesses, grid-strided.
// At Llama-3-8B that is ~225 GB per step, i.e. HBM-bound at ~35 ms; with ZeRO-1 each rank runs it
// over its 1/N shard only.
//
// Gradients may be bf16 (default) or fp32 (``--grad-dtype fp32``: micro-batch accumulation and the
// data-parallel reduction in fp32, 30 B/param per step instead of 28).
//
// grad scaling: g_eff = g * gscale * (gscale_dev ? *gscale_dev : 1) -- gscale_dev carries a
// device-computed clip coefficient so gradient clipping needs no host sync.
#include "common.h"
#include "kernels.h"

namespace kop {

// Every byte is touched exactly once per step. Plain (cached) loads and stores: non-temporal ones measured
// 1 % slower on the whole training step (the update overlaps the next forward). The update uses the
// hardware sqrt / reciprocal.
// eight consecutive gradients as fp32 (one 16-byte bf16 load or two 16-byte fp32 loads)
__device__ __forceinline__ void load_grad8(const bf16_t* __restrict__ g, int64_t it, float* f) {
  unpack8(reinterpret_cast<const u32x4*>(g)[it], f);
}
__device__ __forceinline__ void load_grad8(const float* __restrict__ g, int64_t it, float* f) {
  const f32x4 a = reinterpret_cast<const f32x4*>(g)[it * 2], b = reinterpret_cast<const f32x4*>(g)[it * 2 + 1];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = a[i];
    f[i + 4] = b[i];
  }
}

template <typename GT>
__global__ void __launch_bounds__(256) adamw_kernel(bf16_t* __restrict__ p, const GT* __restrict__ g,
                                                    float* __restrict__ master, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t n8, float lr, float b1, float b2,
                                                    float eps, float wd, float inv_bc1, float inv_sqrt_bc2,
                                                    float gscale, const float* __restrict__ gscale_dev) {
  const float gs = gscale * (gscale_dev ? gscale_dev[0] : 1.f);
  const float decay = 1.f - lr * wd;
  const float step = lr * inv_bc1;
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < n8; it += (int64_t)gridDim.x * blockDim.x) {
    f32x4* mp = reinterpret_cast<f32x4*>(master) + it * 2;
    f32x4* mm = reinterpret_cast<f32x4*>(m) + it * 2;
    f32x4* vv = reinterpret_cast<f32x4*>(v) + it * 2;
    float gf[8], w[8], mv[8], vv8[8];
    load_grad8(g, it, gf);
    const f32x4 w0 = mp[0], w1 = mp[1];
    const f32x4 m0 = mm[0], m1 = mm[1];
    const f32x4 v0 = vv[0], v1 = vv[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = w0[i]; w[i + 4] = w1[i];
      mv[i] = m0[i]; mv[i + 4] = m1[i];
      vv8[i] = v0[i]; vv8[i + 4] = v1[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float gi = gf[i] * gs;
      mv[i] = b1 * mv[i] + (1.f - b1) * gi;
      vv8[i] = b2 * vv8[i] + (1.f - b2) * gi * gi;
      const float denom = __builtin_amdgcn_sqrtf(vv8[i]) * inv_sqrt_bc2 + eps;
      w[i] = w[i] * decay - step * mv[i] * __builtin_amdgcn_rcpf(denom);
    }
    mp[0] = f32x4{w[0], w[1], w[2], w[3]};
    mp[1] = f32x4{w[4], w[5], w[6], w[7]};
    mm[0] = f32x4{mv[0], mv[1], mv[2], mv[3]};
    mm[1] = f32x4{mv[4], mv[5], mv[6], mv[7]};
    vv[0] = f32x4{vv8[0], vv8[1], vv8[2], vv8[3]};
    vv[1] = f32x4{vv8[4], vv8[5], vv8[6], vv8[7]};
    reinterpret_cast<u32x4*>(p)[it] = pack8(w);
  }
}

template <typename GT>
static int adamw_launch(bf16_t* p, const GT* g, float* master, float* m, float* v, int64_t n, float lr, float b1,
                        float b2, float eps, float wd, int step, float gscale, const float* gscale_dev,
                        hipStream_t stream) {
  if (n % 8 != 0) return -1;
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  adamw_kernel<GT><<<stream_grid(n / 8, 256), 256, 0, stream>>>(p, g, master, m, v, n / 8, lr, b1, b2, eps, wd,
                                                                (float)(1.0 / bc1), (float)(1.0 / sqrt(bc2)), gscale,
                                                                gscale_dev);
  return 0;
}

int adamw_step(bf16_t* p, const bf16_t* g, float* master, float* m, float* v, int64_t n, float lr, float b1, float b2,
               float eps, float wd, int step, float gscale, const float* gscale_dev, hipStream_t stream) {
  return adamw_launch(p, g, master, m, v, n, lr, b1, b2, eps, wd, step, gscale, gscale_dev, stream);
}

int adamw_step(bf16_t* p, const float* g, float* master, float* m, float* v, int64_t n, float lr, float b1, float b2,
               float eps, float wd, int step, float gscale, const float* gscale_dev, hipStream_t stream) {
  return adamw_launch(p, g, master, m, v, n, lr, b1, b2, eps, wd, step, gscale, gscale_dev, stream);
}

// sum of squares of a bf16 / fp32 buffer, accumulated (atomically, one add per block) into out[0]
template <typename GT>
__global__ void __launch_bounds__(256) sumsq_kernel(const GT* __restrict__ g, int64_t n8, float* __restrict__ out) {
  __shared__ float red[4];
  float a = 0.f;
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < n8; it += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    load_grad8(g, it, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) a += f[i] * f[i];
  }
  a = block_sum<4>(a, red);
  if (threadIdx.x == 0) atomicAdd(out, a);
}

int grad_sumsq(const bf16_t* g, int64_t n, float* out, hipStream_t stream) {
  if (n % 8 != 0) return -1;
  sumsq_kernel<bf16_t><<<stream_grid(n / 8, 256), 256, 0, stream>>>(g, n / 8, out);
  return 0;
}

int grad_sumsq(const float* g, int64_t n, float* out, hipStream_t stream) {
  if (n % 8 != 0) return -1;
  sumsq_kernel<float><<<stream_grid(n / 8, 256), 256, 0, stream>>>(g, n / 8, out);
  return 0;
}

// coef = base * min(1, max_norm / (sqrt(sumsq) + 1e-6)); also stores the norm for logging
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float max_norm, float* __restrict__ coef,
                                 float* __restrict__ norm_out) {
  const float nrm = sqrtf(sumsq[0]);
  norm_out[0] = nrm;
  coef[0] = max_norm > 0.f ? fminf(1.f, max_norm / (nrm + 1e-6f)) : 1.f;
}

int clip_coef(const float* sumsq, float max_norm, float* coef, float* norm_out, hipStream_t stream) {
  clip_coef_kernel<<<1, 1, 0, stream>>>(sumsq, max_norm, coef, norm_out);
  return 0;
}

}  // namespace kop
