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
// 22.8 vs 25.1 us). KOP_TRANSPOSE=square / cols select the older forms.
//
// Square form: one 256-thread workgroup per 64x64 tile. Load: each thread reads 16 B (8 consecutive columns of one
// row), a wave covers 8 rows x 128 B. The tile goes to LDS with a 66-element pitch; the read phase takes
// dword pairs of columns: thread (chunk = t % 8, pair = t / 8) reads rows 8*chunk .. 8*chunk+7 of columns
// 2*pair, 2*pair+1 -> dword bank (8*chunk + 33*i + pair) mod 64, conflict-free for every i -- and writes
// two 16-B output segments; a wave writes 8 output rows x 128 B contiguous.
#include <cstdlib>
#include "common.h"
#include "kernels.h"

namespace kop {

namespace {
constexpr int kTile = 64;
constexpr int kPitchDw = 33;  // (64 + 2) bf16 per LDS row, in dwords
}  // namespace

__global__ void __launch_bounds__(256) transpose_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                        int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                                                        int64_t tiles_c) {
  __shared__ uint32_t lds[kTile * kPitchDw];
  const int t = threadIdx.x;
  const int64_t tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t r0 = tr * kTile, c0 = tc * kTile;
  const bool full = r0 + kTile <= R && c0 + kTile <= C;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = p * 32 + (t >> 3), ch = t & 7;
    const int64_t gr = r0 + row, gc = c0 + ch * 8;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (full || (gr < R && gc < C)) v = *reinterpret_cast<const u32x4*>(in + gr * ldi + gc);
    uint32_t* d = lds + row * kPitchDw + ch * 4;
    d[0] = v[0];
    d[1] = v[1];
    d[2] = v[2];
    d[3] = v[3];
  }
  __syncthreads();
  const int chunk = t & 7, pair = t >> 3;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = lds[(chunk * 8 + i) * kPitchDw + pair];
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

namespace {
int transpose_mode() {
  static const int mode = [] {
    const char* e = getenv("KOP_TRANSPOSE");
    if (e && e[0] == 's') return 0;  // "square": 64x64 tiles
    if (e && e[0] == 'c') return 1;  // "cols": wide tiles, column tiles fastest
    return 2;                        // default: wide tiles, row tiles fastest
  }();
  return mode;
}
}  // namespace

int transpose2d(const bf16_t* in, bf16_t* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo, hipStream_t stream) {
  if (R % 8 != 0 || C % 8 != 0 || ldi % 8 != 0 || ldo % 8 != 0) return -1;
  if (transpose_mode() != 0) {
    const int64_t tiles_r = (R + 63) / 64, tiles_c = (C + 127) / 128;
    const int64_t n = tiles_r * tiles_c;
    if (n == 0) return 0;
    if (n > 0x7fffffff) return -2;
    if (transpose_mode() == 2)
      transpose_wide_kernel<true><<<(unsigned)n, 256, 0, stream>>>(in, out, R, C, ldi, ldo, tiles_c);
    else
      transpose_wide_kernel<false><<<(unsigned)n, 256, 0, stream>>>(in, out, R, C, ldi, ldo, tiles_c);
    return 0;
  }
  const int64_t tiles_r = (R + kTile - 1) / kTile, tiles_c = (C + kTile - 1) / kTile;
  const int64_t n = tiles_r * tiles_c;
  if (n == 0) return 0;
  if (n > 0x7fffffff) return -2;
  transpose_kernel<<<(unsigned)n, 256, 0, stream>>>(in, out, R, C, ldi, ldo, tiles_c);
  return 0;
}

}  // namespace kop
