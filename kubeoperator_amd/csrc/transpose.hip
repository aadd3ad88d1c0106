// bf16 2-D transpose for gfx950: out[c][r] = in[r][c].
//
// Why it exists: hipBLASLt's weight-gradient GEMM dW = dY^T X (both operands with the reduction dim T as
// the slow index, "NT") runs at ~1.15 PF/s on MI355X, while the same product with both operands
// K-contiguous ("TN", the forward layout) runs at ~1.55 PF/s (tools/bench_gemm_layouts.py). Materialising
// dY^T and X^T costs one read + one write of each operand: at HBM speed that is far less than the GEMM
// time it saves, but only if the transpose itself streams near bandwidth -- PyTorch's strided copy
// reaches ~1 TB/s, this kernel is built for >4 TB/s.
//
// Default kernel (transpose_wide_kernel<true>): 64 x 128 tiles, row tiles fastest in the grid, so the
// workgroups in flight write adjacent output segments; the column-fastest order leaves every concurrent
// workgroup writing one output column band 16 KB apart (tools/bench_transpose.py, one MI355X:
// 8192 x 28672 178 us = 5.3 TB/s vs 211 us with 64 x 64 tiles; 8192 x 14336 92 vs 110 us; 8192 x 4096
// 22.8 vs 25.1 us; the 64 x 64-tile and column-fastest forms measured there are no longer built).
#include <cstdlib>
#include "common.h"
#include "kernels.h"

namespace kop {


// Wide form: 64 rows x 128 columns per workgroup, 64 B of loads in flight per thread (four 16-B rows)
// instead of 32. LDS pitch 65 dwords; read phase: thread (chunk = t % 8, pair = t / 8 + 32 j) -> dword bank
// (8*chunk + pair + 65 i) mod 64: the 64 lanes of a wave (8 chunks x 8 pairs) hit 64 distinct banks.
template <bool ROWS_FAST>
__global__ void __launch_bounds__(256) transpose_wide_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                                                             int64_t tiles_c) {
  constexpr int TR = 64, TC = 128, P = 65;
  __shared__ uint32_t lds[TR * P];
  const int t = threadIdx.x;
  // ROWS_FAST: consecutive workgroups take consecutive row tiles, so their output segments are adjacent
  const int64_t tiles_r = (R + TR - 1) / TR;
  const int64_t tr = ROWS_FAST ? blockIdx.x % tiles_r : blockIdx.x / tiles_c;
  const int64_t tc = ROWS_FAST ? blockIdx.x / tiles_r : blockIdx.x % tiles_c;
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
    u32x4 lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
      hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
    }
    const int64_t oc = c0 + 2 * pair, orr = r0 + chunk * 8;
    if (full || (oc < C && orr < R)) *reinterpret_cast<u32x4*>(out + oc * ldo + orr) = lo;
    if (full || (oc + 1 < C && orr < R)) *reinterpret_cast<u32x4*>(out + (oc + 1) * ldo + orr) = hi;
  }
}

// RoPE (in place, on the first `rope_cols` columns = the Q and K heads of a fused-QKV row matrix, head_dim 128 / 64)
// fused with the transpose of the WHOLE matrix: the attention backward's dQ|dK|dV leaves the flash kernels
// un-rotated; this applies the inverse rotation (sign = -1) and also writes dQKV^T, the K-contiguous dY operand of
// the QKV weight-gradient GEMM, in the same pass (the separate rope + transpose read dQKV twice more).
// Tiles as transpose_wide_kernel<true> (64 rows x 128 columns = one or two heads); a rotary pair (d, d + D/2) sits
// in lanes t and t ^ (D/16) of one wave: the partner half comes by a lane swap.
template <int D>
__global__ void __launch_bounds__(256) rope_t_kernel(bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                     const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                     int64_t R, int64_t C, int64_t ldx, int64_t ldo, int S,
                                                     int64_t rope_cols, float sign) {
  constexpr int TR = 64, TC = 128, P = 65, HALF = D / 2, PX = HALF / 8;  // PX: lane distance of a rotary pair
  __shared__ uint32_t lds[TR * P];
  const int t = threadIdx.x;
  const int64_t tiles_r = R / TR;
  const int64_t tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
  const int64_t r0 = tr * TR, c0 = tc * TC;
  const int ch = t & 15;
  u32x4 v[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = p * 16 + (t >> 4);
    v[p] = *reinterpret_cast<const u32x4*>(x + (r0 + row) * ldx + c0 + ch * 8);
  }
  if (c0 < rope_cols) {  // block-uniform: a Q or K head
    const bool lo_half = (ch & PX) == 0;
    const int j = (ch & (PX - 1)) * 8;  // rotary pair index of this lane's first column
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = p * 16 + (t >> 4);
      const int pos = (int)((r0 + row) % S);
      u32x4 pv;
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = (uint32_t)__shfl_xor((int)v[p][i], PX, 64);
      const f32x4* cp = reinterpret_cast<const f32x4*>(cos_t + (int64_t)pos * HALF + j);
      const f32x4* sp = reinterpret_cast<const f32x4*>(sin_t + (int64_t)pos * HALF + j);
      const f32x4 c0v = cp[0], c1v = cp[1], s0v = sp[0], s1v = sp[1];
      float mine[8], other[8], o[8];
      unpack8(v[p], mine);
      unpack8(pv, other);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float c = i < 4 ? c0v[i] : c1v[i - 4];
        const float sn = (i < 4 ? s0v[i] : s1v[i - 4]) * sign;
        // (a, b) = (x_d, x_{d+64}) -> (a c - b s, b c + a s)
        o[i] = lo_half ? mine[i] * c - other[i] * sn : mine[i] * c + other[i] * sn;
      }
      v[p] = pack8(o);
      *reinterpret_cast<u32x4*>(x + (r0 + row) * ldx + c0 + ch * 8) = v[p];
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t* d = lds + (p * 16 + (t >> 4)) * P + ch * 4;
    d[0] = v[p][0];
    d[1] = v[p][1];
    d[2] = v[p][2];
    d[3] = v[p][3];
  }
  __syncthreads();
  const int chunk = t & 7;
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int pair = (t >> 3) + 32 * jj;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = lds[(chunk * 8 + i) * P + pair];
    u32x4 lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
      hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
    }
    const int64_t oc = c0 + 2 * pair, orr = r0 + chunk * 8;
    *reinterpret_cast<u32x4*>(out + oc * ldo + orr) = lo;
    *reinterpret_cast<u32x4*>(out + (oc + 1) * ldo + orr) = hi;
  }
}

int rope_transpose(bf16_t* x, bf16_t* out, const float* cos_t, const float* sin_t, int64_t R, int64_t C, int64_t ldx,
                   int64_t ldo, int S, int nheads, int D, bool inverse, hipStream_t stream) {
  if ((D != 128 && D != 64) || R % 64 != 0 || C % 128 != 0 || ldx % 8 != 0 || ldo % 8 != 0 ||
      (int64_t)nheads * D > C || ((int64_t)nheads * D) % 128 != 0)
    return -1;
  const int64_t n = (R / 64) * (C / 128);
  if (n == 0) return 0;
  if (n > 0x7fffffff) return -2;
  const float sign = inverse ? -1.f : 1.f;
  if (D == 128)
    rope_t_kernel<128><<<(unsigned)n, 256, 0, stream>>>(x, out, cos_t, sin_t, R, C, ldx, ldo, S, (int64_t)nheads * D, sign);
  else
    rope_t_kernel<64><<<(unsigned)n, 256, 0, stream>>>(x, out, cos_t, sin_t, R, C, ldx, ldo, S, (int64_t)nheads * D, sign);
  return 0;
}

int transpose2d(const bf16_t* in, bf16_t* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo, hipStream_t stream) {
  if (R % 8 != 0 || C % 8 != 0 || ldi % 8 != 0 || ldo % 8 != 0) return -1;
  const int64_t tiles_r = (R + 63) / 64, tiles_c = (C + 127) / 128;
  const int64_t n = tiles_r * tiles_c;
  if (n == 0) return 0;
  if (n > 0x7fffffff) return -2;
  transpose_wide_kernel<true><<<(unsigned)n, 256, 0, stream>>>(in, out, R, C, ldi, ldo, tiles_c);
  return 0;
}

}  // namespace kop
