// Memory-bound elementwise kernels for gfx950: RoPE (in place on the fused QKV activation), SwiGLU and
// GELU forward/backward. All of them move 16 bytes (8 x bf16) per lane per access (Guideline 13) and
// take cos/sin from a host-precomputed fp32 table instead of evaluating trig per element (Appendix B).
#include "common.h"
#include "kernels.h"

namespace kop {

// ---------------------------------------------------------------------------------------------
// RoPE, rotate-half convention (x_i, x_{i+D/2}) -> (x_i c - x_{i+D/2} s, x_{i+D/2} c + x_i s),
// applied in place to the first `nheads` heads of every token row of a [T, row_stride] activation
// (the Q and K heads of the fused QKV projection; V is untouched). sign = -1 applies the inverse
// rotation, which is the backward pass. Position of token t is pos[t] if given, else t % S.
// Work item = 8 consecutive rotary pairs of one head of one token.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) rope_kernel(bf16_t* __restrict__ x, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, const int* __restrict__ pos,
                                                   int S, int nheads, int D, int64_t row_stride, float sign) {
  // grid: (T, ceil(items_per_token / 256)); item = (head, group of 8 rotary pairs) of token blockIdx.x
  const int half = D >> 1;
  const int per_head = half >> 3;
  const int item = blockIdx.y * blockDim.x + threadIdx.x;
  if (item >= nheads * per_head) return;
  const int64_t t = blockIdx.x;
  const int h = item / per_head, j = item - h * per_head;
  const int p = pos ? pos[t] : (int)(t % S);
  bf16_t* base = x + t * row_stride + (int64_t)h * D + j * 8;
  u32x4* lo = reinterpret_cast<u32x4*>(base);
  u32x4* hi = reinterpret_cast<u32x4*>(base + half);
  const f32x4* cp = reinterpret_cast<const f32x4*>(cos_t + (int64_t)p * half + j * 8);
  const f32x4* sp = reinterpret_cast<const f32x4*>(sin_t + (int64_t)p * half + j * 8);
  const u32x4 lv = *lo, hv = *hi;
  const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
  float a[8], b[8], c[8], sn[8];
  unpack8(lv, a);
  unpack8(hv, b);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    c[i] = c0[i];
    c[i + 4] = c1[i];
    sn[i] = s0[i] * sign;
    sn[i + 4] = s1[i] * sign;
  }
  float o1[8], o2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    o1[i] = a[i] * c[i] - b[i] * sn[i];
    o2[i] = b[i] * c[i] + a[i] * sn[i];
  }
  *lo = pack8(o1);
  *hi = pack8(o2);
}

int rope_inplace(bf16_t* x, const float* cos_t, const float* sin_t, const int* pos, int64_t T, int S, int nheads,
                 int D, int64_t row_stride, bool inverse, hipStream_t stream) {
  if (D % 16 != 0 || row_stride % 8 != 0) return -1;
  if (T == 0) return 0;
  if (T >= (1ll << 31)) return -3;
  const int items = nheads * (D / 16);
  const dim3 grid((unsigned)T, (items + 255) / 256);
  rope_kernel<<<grid, 256, 0, stream>>>(x, cos_t, sin_t, pos, S, nheads, D, row_stride, inverse ? -1.f : 1.f);
  return 0;
}

// ---------------------------------------------------------------------------------------------
// SwiGLU: gu = [gate | up] along the last dim (one fused GEMM output of width 2F).
//   fwd: h = silu(gate) * up                  [T, F]
//   bwd: dgate = dh * up * sig * (1 + gate*(1-sig)),  dup = dh * silu(gate)  -> dgu [T, 2F]
// ---------------------------------------------------------------------------------------------
// grid: (T, ceil(F/8 / 256)): one 16-byte chunk of gate and up per thread, no grid-stride loop and no
// per-item integer division; sigmoid through the hardware reciprocal (v_rcp_f32, 1 ulp)
__device__ __forceinline__ float sigmoidf_fast(float g) { return __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h, int F) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= (F >> 3)) return;
  const int64_t t = blockIdx.x;
  const bf16_t* row = gu + t * 2 * F;
  const u32x4 gv = reinterpret_cast<const u32x4*>(row)[c];
  const u32x4 uv = reinterpret_cast<const u32x4*>(row + F)[c];
  float g[8], u[8], o[8];
  unpack8(gv, g);
  unpack8(uv, u);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = g[i] * sigmoidf_fast(g[i]) * u[i];
  reinterpret_cast<u32x4*>(h + t * F)[c] = pack8(o);
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dh,
                                                         bf16_t* __restrict__ dgu, int F) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= (F >> 3)) return;
  const int64_t t = blockIdx.x;
  const bf16_t* row = gu + t * 2 * F;
  const u32x4 gv = reinterpret_cast<const u32x4*>(row)[c];
  const u32x4 uv = reinterpret_cast<const u32x4*>(row + F)[c];
  const u32x4 dv = reinterpret_cast<const u32x4*>(dh + t * F)[c];
  float g[8], u[8], d[8], dg[8], du[8];
  unpack8(gv, g);
  unpack8(uv, u);
  unpack8(dv, d);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float sg = sigmoidf_fast(g[i]);
    const float silu = g[i] * sg;
    du[i] = d[i] * silu;
    dg[i] = d[i] * u[i] * sg * (1.f + g[i] * (1.f - sg));
  }
  bf16_t* orow = dgu + t * 2 * F;
  reinterpret_cast<u32x4*>(orow)[c] = pack8(dg);
  reinterpret_cast<u32x4*>(orow + F)[c] = pack8(du);
}

int swiglu_fwd(const bf16_t* gu, bf16_t* h, int64_t T, int F, hipStream_t stream) {
  if (F % 8) return -1;
  if (T == 0) return 0;
  if (T >= (1ll << 31)) return -3;
  const dim3 grid((unsigned)T, (F / 8 + 255) / 256);
  swiglu_fwd_kernel<<<grid, 256, 0, stream>>>(gu, h, F);
  return 0;
}
int swiglu_bwd(const bf16_t* gu, const bf16_t* dh, bf16_t* dgu, int64_t T, int F, hipStream_t stream) {
  if (F % 8) return -1;
  if (T == 0) return 0;
  if (T >= (1ll << 31)) return -3;
  const dim3 grid((unsigned)T, (F / 8 + 255) / 256);
  swiglu_bwd_kernel<<<grid, 256, 0, stream>>>(gu, dh, dgu, F);
  return 0;
}

// SwiGLU forward that also writes h^T ([F, T]): the down projection's weight gradient dW = dY^T h then runs
// in the K-contiguous layout from the saved h^T (the row-major h feeds the forward GEMM and is not kept).
// Same tiling as swiglu_bwd_t_kernel.
__global__ void __launch_bounds__(256) swiglu_fwd_t_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h,
                                                           bf16_t* __restrict__ ht, int64_t T, int F, int64_t tiles_r) {
  constexpr int P = 33;
  __shared__ uint32_t lh[64 * P];
  const int t = threadIdx.x;
  const int64_t tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
  const int64_t r0 = tr * 64;
  const int c0 = (int)tc * 64;
  u32x4 gv[2], uv[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int64_t row = r0 + p * 32 + (t >> 3);
    const int col = c0 + (t & 7) * 8;
    gv[p] = *reinterpret_cast<const u32x4*>(gu + row * 2 * F + col);
    uv[p] = *reinterpret_cast<const u32x4*>(gu + row * 2 * F + F + col);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int lrow = p * 32 + (t >> 3), ch = t & 7;
    float g[8], u[8], o[8];
    unpack8(gv[p], g);
    unpack8(uv[p], u);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = g[i] * sigmoidf_fast(g[i]) * u[i];
    const u32x4 po = pack8(o);
    *reinterpret_cast<u32x4*>(h + (r0 + lrow) * F + c0 + ch * 8) = po;
#pragma unroll
    for (int i = 0; i < 4; ++i) lh[lrow * P + ch * 4 + i] = po[i];
  }
  __syncthreads();
  const int chunk = t & 7, pair = t >> 3;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = lh[(chunk * 8 + i) * P + pair];
  u32x4 lo, hi;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
    hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
  }
  const int64_t oc = c0 + 2 * pair, orr = r0 + chunk * 8;
  *reinterpret_cast<u32x4*>(ht + oc * T + orr) = lo;
  *reinterpret_cast<u32x4*>(ht + (oc + 1) * T + orr) = hi;
}

int swiglu_fwd_t(const bf16_t* gu, bf16_t* h, bf16_t* ht, int64_t T, int F, hipStream_t stream) {
  if (F % 64 || T % 64) return -1;
  if (T == 0) return 0;
  const int64_t tiles_r = T / 64, n = tiles_r * (F / 64);
  if (n > 0x7fffffff) return -2;
  swiglu_fwd_t_kernel<<<(unsigned)n, 256, 0, stream>>>(gu, h, ht, T, F, tiles_r);
  return 0;
}

// SwiGLU backward that also writes dgu^T ([2F, T]), the K-contiguous operand of the gate/up weight-gradient
// GEMM: one 64-token x 64-column tile of gate and of up per workgroup, dg / du computed in registers, stored
// row-major and staged through LDS (pitch 33 dwords, conflict-free column reads as in csrc/transpose.hip) for
// the transposed stores. Replaces swiglu_bwd + a separate transpose of dgu (one read + one write of 2*T*F
// bf16 saved). Row tiles fastest in the grid (adjacent transposed output segments).
__global__ void __launch_bounds__(256) swiglu_bwd_t_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dh,
                                                           bf16_t* __restrict__ dgu, bf16_t* __restrict__ dgut,
                                                           int64_t T, int F, int64_t tiles_r) {
  constexpr int P = 33;
  __shared__ uint32_t lg[64 * P], lu[64 * P];
  const int t = threadIdx.x;
  const int64_t tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
  const int64_t r0 = tr * 64;
  const int c0 = (int)tc * 64;
  u32x4 gv[2], uv[2], dv[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int64_t row = r0 + p * 32 + (t >> 3);
    const int col = c0 + (t & 7) * 8;
    gv[p] = *reinterpret_cast<const u32x4*>(gu + row * 2 * F + col);
    uv[p] = *reinterpret_cast<const u32x4*>(gu + row * 2 * F + F + col);
    dv[p] = *reinterpret_cast<const u32x4*>(dh + row * F + col);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int lrow = p * 32 + (t >> 3), ch = t & 7;
    const int64_t row = r0 + lrow;
    const int col = c0 + ch * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(gv[p], g);
    unpack8(uv[p], u);
    unpack8(dv[p], d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sg = sigmoidf_fast(g[i]);
      const float silu = g[i] * sg;
      du[i] = d[i] * silu;
      dg[i] = d[i] * u[i] * sg * (1.f + g[i] * (1.f - sg));
    }
    const u32x4 pg = pack8(dg), pu = pack8(du);
    *reinterpret_cast<u32x4*>(dgu + row * 2 * F + col) = pg;
    *reinterpret_cast<u32x4*>(dgu + row * 2 * F + F + col) = pu;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lg[lrow * P + ch * 4 + i] = pg[i];
      lu[lrow * P + ch * 4 + i] = pu[i];
    }
  }
  __syncthreads();
  const int chunk = t & 7, pair = t >> 3;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const uint32_t* L = half ? lu : lg;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = L[(chunk * 8 + i) * P + pair];
    u32x4 lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
      hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
    }
    const int64_t oc = (int64_t)half * F + c0 + 2 * pair, orr = r0 + chunk * 8;
    *reinterpret_cast<u32x4*>(dgut + oc * T + orr) = lo;
    *reinterpret_cast<u32x4*>(dgut + (oc + 1) * T + orr) = hi;
  }
}

int swiglu_bwd_t(const bf16_t* gu, const bf16_t* dh, bf16_t* dgu, bf16_t* dgut, int64_t T, int F,
                 hipStream_t stream) {
  if (F % 64 || T % 64) return -1;
  if (T == 0) return 0;
  const int64_t tiles_r = T / 64, n = tiles_r * (F / 64);
  if (n > 0x7fffffff) return -2;
  swiglu_bwd_t_kernel<<<(unsigned)n, 256, 0, stream>>>(gu, dh, dgu, dgut, T, F, tiles_r);
  return 0;
}

// ---------------------------------------------------------------------------------------------
// GELU (tanh approximation, GPT-2): y = 0.5 x (1 + tanh(k (x + 0.044715 x^3))), k = sqrt(2/pi)
// ---------------------------------------------------------------------------------------------
// 0.5 (1 + tanh(u)) = sigmoid(2u), so y = x sigmoid(2u) and dy/dx = s + 2 x s (1 - s) u', s = sigmoid(2u): one exp
// and one hardware reciprocal per element (the IEEE division of 1 - 2 / (exp(2u) + 1) cost ~10 VALU ops).
// Streaming: each thread keeps GELU_U independent 16-B loads in flight (grid-stride groups of GELU_U vectors) --
// one load per iteration left the GPT-2 MLP's GELU passes at 4.6-4.7 TB/s.
constexpr int GELU_U = 4;

__device__ __forceinline__ float gelu_s(float a) {
  const float u2 = 1.5957691216f * (a + 0.044715f * a * a * a);  // 2u
  return __builtin_amdgcn_rcpf(1.f + __expf(-u2));
}

__global__ void __launch_bounds__(256) gelu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x4* yv = reinterpret_cast<u32x4*>(y);
  for (int64_t it = blockIdx.x * blockDim.x + threadIdx.x; it < n8; it += GELU_U * stride) {
    u32x4 v[GELU_U];
#pragma unroll
    for (int u = 0; u < GELU_U; ++u)
      if (it + u * stride < n8) v[u] = __builtin_nontemporal_load(xv + it + u * stride);
#pragma unroll
    for (int u = 0; u < GELU_U; ++u) {
      if (it + u * stride >= n8) break;
      float a[8], o[8];
      unpack8(v[u], a);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = a[i] * gelu_s(a[i]);
      yv[it + u * stride] = pack8(o);
    }
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                       bf16_t* __restrict__ dx, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  const u32x4* dv = reinterpret_cast<const u32x4*>(dy);
  u32x4* ov = reinterpret_cast<u32x4*>(dx);
  for (int64_t it = blockIdx.x * blockDim.x + threadIdx.x; it < n8; it += GELU_U * stride) {
    u32x4 xa[GELU_U], da[GELU_U];
#pragma unroll
    for (int u = 0; u < GELU_U; ++u)
      if (it + u * stride < n8) {
        xa[u] = __builtin_nontemporal_load(xv + it + u * stride);
        da[u] = __builtin_nontemporal_load(dv + it + u * stride);
      }
#pragma unroll
    for (int u = 0; u < GELU_U; ++u) {
      if (it + u * stride >= n8) break;
      float a[8], d[8], o[8];
      unpack8(xa[u], a);
      unpack8(da[u], d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float sg = gelu_s(a[i]);
        const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * a[i] * a[i]);
        o[i] = d[i] * (sg + 2.f * a[i] * sg * (1.f - sg) * du);
      }
      ov[it + u * stride] = pack8(o);
    }
  }
}

int gelu_fwd(const bf16_t* x, bf16_t* y, int64_t n, hipStream_t stream) {
  if (n % 8 || n / 8 >= (1ll << 31)) return -1;
  gelu_fwd_kernel<<<stream_grid((n / 8 + GELU_U - 1) / GELU_U, 256), 256, 0, stream>>>(x, y, n / 8);
  return 0;
}
int gelu_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, int64_t n, hipStream_t stream) {
  if (n % 8 || n / 8 >= (1ll << 31)) return -1;
  gelu_bwd_kernel<<<stream_grid((n / 8 + GELU_U - 1) / GELU_U, 256), 256, 0, stream>>>(x, dy, dx, n / 8);
  return 0;
}

}  // namespace kop
