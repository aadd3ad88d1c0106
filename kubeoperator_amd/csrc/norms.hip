// RMSNorm / LayerNorm forward + backward for gfx950, with the residual add fused in.
//
//   forward :  s = x (+ r)            (the residual stream, written out when r is given)
//              y = norm(s) * w (+ b)  (bf16), rstd (and mean for LayerNorm) saved per row in fp32
//   backward:  ds = dnorm(dy) (+ ds_resid)   -- the residual-stream gradient flows straight through
//              dw (+ db) = sum over rows, two-stage: per-block fp32 partial rows, then a column reduce
//              that writes (or accumulates into) the bf16 gradient buffer slice of the parameter.
//
// Memory-bound: every row is read once as 16-byte vectors (8 bf16 per lane per load, Guideline 13)
// and kept in registers between the statistics pass and the output pass. One 64..256-thread block
// per row, grid-strided.
#include "common.h"
#include "kernels.h"

namespace kop {

template <int NV, bool LN, bool HAS_RES>
__global__ void __launch_bounds__(256) norm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                       const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ y, bf16_t* __restrict__ s_out,
                                                       float* __restrict__ rstd_out, float* __restrict__ mean_out,
                                                       int rows, int H, float eps) {
  __shared__ float red[4];
  const int C = H >> 3;  // 16-byte chunks per row
  const int nw = blockDim.x >> 6;
  float wv[NV][8], bv[NV][8];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = threadIdx.x + v * blockDim.x;
    if (c < C) {
      unpack8(reinterpret_cast<const u32x4*>(w)[c], wv[v]);
      if (LN) unpack8(reinterpret_cast<const u32x4*>(b)[c], bv[v]);
    }
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * H);
    float f[NV][8];
    float acc = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + v * blockDim.x;
      if (c < C) {
        unpack8(xr[c], f[v]);
        if (HAS_RES) {
          float g[8];
          unpack8(reinterpret_cast<const u32x4*>(r + (size_t)row * H)[c], g);
#pragma unroll
          for (int i = 0; i < 8; ++i) f[v][i] += g[i];
          // the residual stream is carried in bf16: normalise exactly what is stored
          u32x4 pk = pack8(f[v]);
          reinterpret_cast<u32x4*>(s_out + (size_t)row * H)[c] = pk;
          unpack8(pk, f[v]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += LN ? f[v][i] : f[v][i] * f[v][i];
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[v][i] = 0.f;
      }
    }
    float mean = 0.f;
    if (LN) {
      float t = wave_sum(acc);
      __syncthreads();
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
      __syncthreads();
      t = 0.f;
      for (int i = 0; i < nw; ++i) t += red[i];
      mean = t / H;
      acc = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = threadIdx.x + v * blockDim.x;
        if (c < C) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float d = f[v][i] - mean;
            acc += d * d;
          }
        }
      }
    }
    float t = wave_sum(acc);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    const float rstd = rsqrtf(t / H + eps);
    if (threadIdx.x == 0) {
      rstd_out[row] = rstd;
      if (LN) mean_out[row] = mean;
    }
    u32x4* yr = reinterpret_cast<u32x4*>(y + (size_t)row * H);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + v * blockDim.x;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (f[v][i] - mean) * rstd * wv[v][i] + (LN ? bv[v][i] : 0.f);
        yr[c] = pack8(o);
      }
    }
  }
}

template <int NV, bool LN, bool HAS_DRES>
__global__ void __launch_bounds__(256) norm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
                                                       const float* __restrict__ mean_in,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int rows, int H) {
  __shared__ float red[8];
  const int C = H >> 3;
  const int nw = blockDim.x >> 6;
  float wv[NV][8], dwa[NV][8], dba[NV][8];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = threadIdx.x + v * blockDim.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) dwa[v][i] = dba[v][i] = 0.f;
    if (c < C) unpack8(reinterpret_cast<const u32x4*>(w)[c], wv[v]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const float rstd = rstd_in[row];
    const float mean = LN ? mean_in[row] : 0.f;
    float xh[NV][8], g[NV][8];
    float a1 = 0.f, a2 = 0.f;  // sum(g*xhat), sum(g)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + v * blockDim.x;
      if (c < C) {
        float d[8];
        unpack8(reinterpret_cast<const u32x4*>(s + (size_t)row * H)[c], xh[v]);
        unpack8(reinterpret_cast<const u32x4*>(dy + (size_t)row * H)[c], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[v][i] = (xh[v][i] - mean) * rstd;
          g[v][i] = d[i] * wv[v][i];
          dwa[v][i] += d[i] * xh[v][i];
          if (LN) dba[v][i] += d[i];
          a1 += g[v][i] * xh[v][i];
          a2 += g[v][i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) xh[v][i] = g[v][i] = 0.f;
      }
    }
    a1 = wave_sum(a1);
    if (LN) a2 = wave_sum(a2);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      red[threadIdx.x >> 6] = a1;
      red[4 + (threadIdx.x >> 6)] = a2;
    }
    __syncthreads();
    a1 = 0.f;
    a2 = 0.f;
    for (int i = 0; i < nw; ++i) {
      a1 += red[i];
      a2 += red[4 + i];
    }
    const float m1 = a1 / H, m2 = a2 / H;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + v * blockDim.x;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (g[v][i] - xh[v][i] * m1 - (LN ? m2 : 0.f));
        if (HAS_DRES) {
          float d2[8];
          unpack8(reinterpret_cast<const u32x4*>(dres + (size_t)row * H)[c], d2);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += d2[i];
        }
        reinterpret_cast<u32x4*>(dx + (size_t)row * H)[c] = pack8(o);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = threadIdx.x + v * blockDim.x;
    if (c < C) {
      f32x4* p = reinterpret_cast<f32x4*>(dw_part + (size_t)blockIdx.x * H + c * 8);
      p[0] = f32x4{dwa[v][0], dwa[v][1], dwa[v][2], dwa[v][3]};
      p[1] = f32x4{dwa[v][4], dwa[v][5], dwa[v][6], dwa[v][7]};
      if (LN) {
        f32x4* q = reinterpret_cast<f32x4*>(db_part + (size_t)blockIdx.x * H + c * 8);
        q[0] = f32x4{dba[v][0], dba[v][1], dba[v][2], dba[v][3]};
        q[1] = f32x4{dba[v][4], dba[v][5], dba[v][6], dba[v][7]};
      }
    }
  }
}

// Column reduce of [nparts, H] fp32 partials into a bf16 gradient (overwrite or accumulate). A block owns a
// 16-column slab (64-byte row pieces) and splits the partial rows over 64 segments, 8 independent sums per
// thread, so each thread has only nparts / 512 dependent L2 round trips. (The earlier 64-column blocks gave
// H / 64 blocks -- 12 at GPT-2's 768 -- with nparts / 128 round trips each: 16 us for 2048 x 768.)
__global__ void __launch_bounds__(1024) col_reduce_kernel(const float* __restrict__ part, int nparts, int H,
                                                          bf16_t* __restrict__ out, int accumulate) {
  constexpr int CW = 16, SEG = 64;
  const int cl = threadIdx.x & (CW - 1);
  const int col = blockIdx.x * CW + cl;
  const int seg = threadIdx.x / CW;
  __shared__ float red[SEG][CW];
  __shared__ float red8[8][CW];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < H) {
    int p = seg;
    for (; p + 7 * SEG < nparts; p += 8 * SEG) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += part[(size_t)(p + i * SEG) * H + col];
    }
    for (int i = 0; p < nparts; p += SEG, i = (i + 1) & 7) acc[i] += part[(size_t)p * H + col];
  }
  red[seg][cl] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (seg < 8) {  // 64 -> 8 segments
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[seg + 8 * i][cl];
    red8[seg][cl] = t;
  }
  __syncthreads();
  if (seg == 0 && col < H) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red8[i][cl];
    if (accumulate) t += bf2f(out[col]);
    out[col] = f2bf(t);
  }
}

static inline int col_reduce_blocks(int H) { return (H + 15) / 16; }

// ---------------------------------------------------------------------------------------------------
// Row-per-wave forward (H a multiple of 512, up to 4096 = Llama-3-8B): a 64-lane wave owns a whole row, each
// lane holds NV = H/512 16-byte chunks (chunk c = lane + 64v, so every v is one contiguous 1 KiB wave
// access), and the row statistics are wave reductions -- no LDS round trip and no __syncthreads per row,
// and 2*NV loads in flight per lane instead of 2. Four rows per 256-thread block. (The backward keeps the
// block-per-row form: a row-per-wave backward holds 8*NV fp32 weight-gradient partials per lane on top of
// the row data and drops to 2 waves per SIMD -- measured slower.)
// ---------------------------------------------------------------------------------------------------
template <int NV, bool LN, bool HAS_RES>
__global__ void __launch_bounds__(256) norm_fwd_wave_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                            const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                            bf16_t* __restrict__ y, bf16_t* __restrict__ s_out,
                                                            float* __restrict__ rstd_out, float* __restrict__ mean_out,
                                                            int rows, int H, float eps) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float inv_h = 1.f / (float)H;
  for (int row = blockIdx.x * 4 + wv; row < rows; row += gridDim.x * 4) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * H);
    u32x4 xv[NV], rv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) xv[v] = xr[lane + 64 * v];
    if (HAS_RES) {
      const u32x4* rr = reinterpret_cast<const u32x4*>(r + (size_t)row * H);
#pragma unroll
      for (int v = 0; v < NV; ++v) rv[v] = rr[lane + 64 * v];
    }
    float f[NV][8];
    float acc = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      unpack8(xv[v], f[v]);
      if (HAS_RES) {
        float g[8];
        unpack8(rv[v], g);
#pragma unroll
        for (int i = 0; i < 8; ++i) f[v][i] += g[i];
        // the residual stream is carried in bf16: normalise exactly what is stored
        const u32x4 pk = pack8(f[v]);
        reinterpret_cast<u32x4*>(s_out + (size_t)row * H)[lane + 64 * v] = pk;
        unpack8(pk, f[v]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += LN ? f[v][i] : f[v][i] * f[v][i];
    }
    float mean = 0.f;
    if (LN) {
      mean = wave_sum(acc) * inv_h;
      acc = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = f[v][i] - mean;
          acc += d * d;
        }
    }
    const float rstd = rsqrtf(wave_sum(acc) * inv_h + eps);
    if (lane == 0) {
      rstd_out[row] = rstd;
      if (LN) mean_out[row] = mean;
    }
    u32x4* yr = reinterpret_cast<u32x4*>(y + (size_t)row * H);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float wf[8], bf[8], o[8];
      unpack8(reinterpret_cast<const u32x4*>(w)[lane + 64 * v], wf);
      if (LN) unpack8(reinterpret_cast<const u32x4*>(b)[lane + 64 * v], bf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (f[v][i] - mean) * rstd * wf[i] + (LN ? bf[i] : 0.f);
      yr[lane + 64 * v] = pack8(o);
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Row-per-wave backward for NARROW rows (H = 256 * NC <= 1024: GPT-2's 768, 512 / 1024 widths). The block-per-
// row kernel above moves only 1.5 KiB per tensor per row at H = 768 between two __syncthreads, so it is
// latency-bound (~1 TB/s, 175 us for 32768 x 768). Here a wave owns a row: each lane holds NC 8-byte chunks
// (4 bf16; chunk c = lane + 64c, one contiguous 512-byte wave access per c), the two row sums are wave
// reductions, and the next row's loads are issued before the current row is computed. The weight-gradient
// partials (12 fp32 per lane at H = 768, 16 at 1024) stay in registers across the rows of the wave and are
// summed over the block's 4 waves in LDS once at the end: one fp32 partial row per block.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ void unpack4(const u32x2 v, float* f) {
  f[0] = __uint_as_float(v[0] << 16);
  f[1] = __uint_as_float(v[0] & 0xffff0000u);
  f[2] = __uint_as_float(v[1] << 16);
  f[3] = __uint_as_float(v[1] & 0xffff0000u);
}

constexpr int kNarrowMaxH = 1024;
constexpr int kNarrowMaxBlocks = 1024;

template <int NC, bool LN, bool HAS_DRES>
__global__ void __launch_bounds__(256) norm_bwd_narrow_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                              const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
                                                              const float* __restrict__ mean_in,
                                                              const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                              float* __restrict__ dw_part, float* __restrict__ db_part,
                                                              int rows, int H) {
  __shared__ f32x4 red[4 * kNarrowMaxH / 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float inv_h = 1.f / (float)H;
  float wf[NC][4], dwa[NC][4], dba[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    unpack4(reinterpret_cast<const u32x2*>(w)[lane + 64 * c], wf[c]);
#pragma unroll
    for (int i = 0; i < 4; ++i) dwa[c][i] = dba[c][i] = 0.f;
  }
  const int stride = gridDim.x * 4;
  int row = blockIdx.x * 4 + wv;
  u32x2 sv[NC], dv[NC], rv[NC];
  if (row < rows) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sv[c] = reinterpret_cast<const u32x2*>(s + (size_t)row * H)[lane + 64 * c];
      dv[c] = reinterpret_cast<const u32x2*>(dy + (size_t)row * H)[lane + 64 * c];
      if (HAS_DRES) rv[c] = reinterpret_cast<const u32x2*>(dres + (size_t)row * H)[lane + 64 * c];
    }
  }
  for (; row < rows; row += stride) {
    u32x2 sc[NC], dc[NC], rc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sc[c] = sv[c];
      dc[c] = dv[c];
      if (HAS_DRES) rc[c] = rv[c];
    }
    const float rstd = rstd_in[row];
    const float mean = LN ? mean_in[row] : 0.f;
    const int nxt = row + stride;
    if (nxt < rows) {  // next row's loads in flight under this row's math
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        sv[c] = reinterpret_cast<const u32x2*>(s + (size_t)nxt * H)[lane + 64 * c];
        dv[c] = reinterpret_cast<const u32x2*>(dy + (size_t)nxt * H)[lane + 64 * c];
        if (HAS_DRES) rv[c] = reinterpret_cast<const u32x2*>(dres + (size_t)nxt * H)[lane + 64 * c];
      }
    }
    float xh[NC][4], g[NC][4];
    float a1 = 0.f, a2 = 0.f;  // sum(g*xhat), sum(g)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float d[4];
      unpack4(sc[c], xh[c]);
      unpack4(dc[c], d);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[c][i] = (xh[c][i] - mean) * rstd;
        g[c][i] = d[i] * wf[c][i];
        dwa[c][i] += d[i] * xh[c][i];
        if (LN) dba[c][i] += d[i];
        a1 += g[c][i] * xh[c][i];
        a2 += g[c][i];
      }
    }
    const float m1 = wave_sum(a1) * inv_h;
    const float m2 = LN ? wave_sum(a2) * inv_h : 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float o[4], r[4];
      if (HAS_DRES) unpack4(rc[c], r);
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = rstd * (g[c][i] - xh[c][i] * m1 - m2) + (HAS_DRES ? r[i] : 0.f);
      reinterpret_cast<u32x2*>(dx + (size_t)row * H)[lane + 64 * c] = u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])};
    }
  }
  // the block's 4 wave partials -> one fp32 partial row (dw, then db)
#pragma unroll
  for (int pass = 0; pass < (LN ? 2 : 1); ++pass) {
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float* a = pass ? dba[c] : dwa[c];
      red[wv * (H >> 2) + lane + 64 * c] = f32x4{a[0], a[1], a[2], a[3]};
    }
    __syncthreads();
    float* out = (pass ? db_part : dw_part) + (size_t)blockIdx.x * H;
    for (int q = threadIdx.x; q < (H >> 2); q += 256) {
      const int h4 = H >> 2;
      reinterpret_cast<f32x4*>(out)[q] = (red[q] + red[h4 + q]) + (red[2 * h4 + q] + red[3 * h4 + q]);
    }
  }
}

static int narrow_nc(int H) {
  if (H % 256 != 0 || H > kNarrowMaxH) return 0;
  return H / 256;
}

// row-per-wave path: H = 512 * NV, NV in {1, 2, 4, 8}
static int wave_nv(int H) {
  if (H % 512 != 0) return 0;
  const int nv = H / 512;
  return (nv == 1 || nv == 2 || nv == 4 || nv == 8) ? nv : 0;
}

static void pick_geom(int H, int& threads, int& nv) {
  const int C = H / 8;
  threads = C >= 256 ? 256 : ((C + 63) / 64) * 64;
  nv = (C + threads - 1) / threads;
}

#define NORM_FWD_DISPATCH(NVv)                                                                              \
  if (nv == NVv) {                                                                                          \
    if (layernorm) {                                                                                        \
      if (r) norm_fwd_kernel<NVv, true, true><<<grid, threads, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
      else norm_fwd_kernel<NVv, true, false><<<grid, threads, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
    } else {                                                                                                \
      if (r) norm_fwd_kernel<NVv, false, true><<<grid, threads, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
      else norm_fwd_kernel<NVv, false, false><<<grid, threads, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
    }                                                                                                       \
    return 0;                                                                                               \
  }

int norm_fwd(const bf16_t* x, const bf16_t* r, const bf16_t* w, const bf16_t* b, bf16_t* y, bf16_t* s_out, float* rstd,
             float* mean, int rows, int H, float eps, bool layernorm, hipStream_t stream) {
  if (H % 8 != 0 || H > 8192) return -1;
  if (const int wn = wave_nv(H)) {
    const int grid = (rows + 3) / 4 < 4096 ? (rows + 3) / 4 : 4096;
#define NORM_FWD_WAVE(NVv)                                                                                  \
    if (wn == NVv) {                                                                                        \
      if (layernorm) {                                                                                      \
        if (r) norm_fwd_wave_kernel<NVv, true, true><<<grid, 256, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
        else norm_fwd_wave_kernel<NVv, true, false><<<grid, 256, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
      } else {                                                                                              \
        if (r) norm_fwd_wave_kernel<NVv, false, true><<<grid, 256, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
        else norm_fwd_wave_kernel<NVv, false, false><<<grid, 256, 0, stream>>>(x, r, w, b, y, s_out, rstd, mean, rows, H, eps); \
      }                                                                                                     \
      return 0;                                                                                             \
    }
    NORM_FWD_WAVE(1)
    NORM_FWD_WAVE(2)
    NORM_FWD_WAVE(4)
    NORM_FWD_WAVE(8)
#undef NORM_FWD_WAVE
  }
  int threads, nv;
  pick_geom(H, threads, nv);
  const int grid = rows < 8192 ? rows : 8192;
  NORM_FWD_DISPATCH(1)
  NORM_FWD_DISPATCH(2)
  NORM_FWD_DISPATCH(3)
  NORM_FWD_DISPATCH(4)
  return -2;
}

#define NORM_BWD_DISPATCH(NVv)                                                                               \
  if (!done && nv == NVv) {                                                                                           \
    if (layernorm) {                                                                                         \
      if (dres) norm_bwd_kernel<NVv, true, true><<<grid, threads, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, part + (size_t)grid * H, rows, H); \
      else norm_bwd_kernel<NVv, true, false><<<grid, threads, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, part + (size_t)grid * H, rows, H); \
    } else {                                                                                                 \
      if (dres) norm_bwd_kernel<NVv, false, true><<<grid, threads, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, nullptr, rows, H); \
      else norm_bwd_kernel<NVv, false, false><<<grid, threads, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, nullptr, rows, H); \
    }                                                                                                        \
    done = true;                                                                                             \
  }

// Blocks of the backward = fp32 weight-gradient partial rows. Narrow rows (GPT-2's 768) need more blocks to
// keep enough rows in flight: 512 blocks x 2 waves was latency-bound at ~1.5 TB/s.
int norm_bwd_partial_rows(int rows, int H) {
  if (narrow_nc(H)) {  // one partial row per 4-row-wave block
    const int g = (rows + 3) / 4;
    return g < kNarrowMaxBlocks ? g : kNarrowMaxBlocks;
  }
  const int cap = H <= 1024 ? 2048 : 512;
  return rows < cap ? rows : cap;
}

int norm_bwd(const bf16_t* dy, const bf16_t* s, const bf16_t* w, const float* rstd, const float* mean,
             const bf16_t* dres, bf16_t* dx, float* part, bf16_t* dw, bf16_t* db, int rows, int H, bool layernorm,
             int accumulate, hipStream_t stream) {
  if (H % 8 != 0 || H > 8192) return -1;
  const int grid = norm_bwd_partial_rows(rows, H);
  bool done = false;
  if (const int nc = narrow_nc(H)) {
#define NORM_BWD_NARROW(NCv)                                                                                 \
    if (!done && nc == NCv) {                                                                                \
      float* dbp = layernorm ? part + (size_t)grid * H : nullptr;                                            \
      if (layernorm) {                                                                                       \
        if (dres) norm_bwd_narrow_kernel<NCv, true, true><<<grid, 256, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, dbp, rows, H); \
        else norm_bwd_narrow_kernel<NCv, true, false><<<grid, 256, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, dbp, rows, H); \
      } else {                                                                                               \
        if (dres) norm_bwd_narrow_kernel<NCv, false, true><<<grid, 256, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, dbp, rows, H); \
        else norm_bwd_narrow_kernel<NCv, false, false><<<grid, 256, 0, stream>>>(dy, s, w, rstd, mean, dres, dx, part, dbp, rows, H); \
      }                                                                                                      \
      done = true;                                                                                           \
    }
    NORM_BWD_NARROW(1)
    NORM_BWD_NARROW(2)
    NORM_BWD_NARROW(3)
    NORM_BWD_NARROW(4)
#undef NORM_BWD_NARROW
  }
  int threads, nv;
  pick_geom(H, threads, nv);
  NORM_BWD_DISPATCH(1)
  NORM_BWD_DISPATCH(2)
  NORM_BWD_DISPATCH(3)
  NORM_BWD_DISPATCH(4)
  if (!done) return -2;
  if (dw == nullptr) return 0;  // partials only: the caller folds them with norm_bwd_reduce (on the side stream)
  return norm_bwd_reduce(part, grid, H, dw, db, layernorm, accumulate, stream);
}

int norm_bwd_reduce(const float* part, int parts, int H, bf16_t* dw, bf16_t* db, bool layernorm, int accumulate,
                    hipStream_t stream) {
  const int cg = col_reduce_blocks(H);
  col_reduce_kernel<<<cg, 1024, 0, stream>>>(part, parts, H, dw, accumulate);
  if (layernorm) col_reduce_kernel<<<cg, 1024, 0, stream>>>(part + (size_t)parts * H, parts, H, db, accumulate);
  return 0;
}

// ---------------------------------------------------------------------------------------------------
// RMSNorm with a TRANSPOSED companion output, for the weight-gradient GEMMs of the projections around it.
//
// dW = dY^T X runs ~1.2x faster on hipBLASLt with both operands K-contiguous, i.e. with X^T and dY^T
// materialised ([H, T] row-major); ops.functional used to make them with separate transpose passes (one
// read + one write of a [T, 4096] bf16 matrix each, 4 per Llama block and micro-batch). Here the norms write
// them while the rows are still in registers:
//   forward : y^T of the normalised activation -- the X operand of the QKV and gate|up weight gradients;
//   backward: dx^T of the residual-stream gradient -- the dY operand of the Wo and W_down weight gradients.
//
// One workgroup = NT = H / 8 threads (thread t owns the 8 columns 8t..8t+7) x RG = 16 rows: the 16 rows of a
// column are in one thread's registers, so each y^T / dx^T row segment (16 tokens = 32 B) is two 16-B stores
// with no LDS round trip. Row statistics: per-thread partials -> LDS [RG][NT] -> each wave sums RG / NW rows.
// The 32-B transposed segments of 4 consecutive row groups form one 128-B line: row groups are dealt so
// that those 4 groups run on the same XCD (blocks b, b+8, b+16, b+24 share one), their partial lines
// merging in that XCD's L2 before write-back.
// ---------------------------------------------------------------------------------------------------
constexpr int kTRG = 16;

__device__ __forceinline__ int64_t t_row_group(bool remap) {
  const int b = blockIdx.x;
  if (!remap) return b;
  return (int64_t)(b >> 5) * 32 + (b & 7) * 4 + ((b >> 3) & 3);
}

// 16 rows x 8 packed bf16 columns (v[r] = row r, columns 8t..8t+7) -> column i's 16 rows as 8 dwords
__device__ __forceinline__ void t_store(const u32x4* v, bf16_t* out_col0, int64_t ldt) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int d = i >> 1;
    u32x4 lo, hi;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a0 = v[2 * k][d], a1 = v[2 * k + 1][d], b0 = v[8 + 2 * k][d], b1 = v[8 + 2 * k + 1][d];
      // selector: even column = low halves of the two rows, odd column = high halves
      lo[k] = (i & 1) ? __builtin_amdgcn_perm(a1, a0, 0x07060302u) : __builtin_amdgcn_perm(a1, a0, 0x05040100u);
      hi[k] = (i & 1) ? __builtin_amdgcn_perm(b1, b0, 0x07060302u) : __builtin_amdgcn_perm(b1, b0, 0x05040100u);
    }
    u32x4* o = reinterpret_cast<u32x4*>(out_col0 + (int64_t)i * ldt);
    o[0] = lo;
    o[1] = hi;
  }
}

// sums RG per-thread partials over the NT threads of the block; returns them in LDS `rs` (scaled by f(row sum))
template <int NT>
__device__ __forceinline__ void t_row_sums(const float* part, float* red, float* rs) {
  constexpr int NW = NT / 64, RPW = kTRG / NW;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
  for (int r = 0; r < kTRG; ++r) red[r * NT + t] = part[r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = wv * RPW + k;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < NW; ++j) v += red[row * NT + lane + 64 * j];
    v = wave_sum(v);
    if (lane == 0) rs[row] = v;
  }
  __syncthreads();
}

template <int NT, bool HAS_RES>
__global__ void __launch_bounds__(NT) rms_fwd_t_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                       const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                       bf16_t* __restrict__ s_out, bf16_t* __restrict__ yt,
                                                       float* __restrict__ rstd_out, int64_t ldt, float eps, int remap) {
  constexpr int H = NT * 8;
  __shared__ float red[kTRG * NT];
  __shared__ float rs[kTRG];
  const int t = threadIdx.x;
  const int64_t r0 = t_row_group(remap) * kTRG;
  u32x4 v[kTRG];
  float ss[kTRG];
#pragma unroll
  for (int k = 0; k < kTRG; ++k) v[k] = reinterpret_cast<const u32x4*>(x + (r0 + k) * H)[t];
  if (HAS_RES) {
    u32x4 rv[kTRG];
#pragma unroll
    for (int k = 0; k < kTRG; ++k) rv[k] = reinterpret_cast<const u32x4*>(r + (r0 + k) * H)[t];
#pragma unroll
    for (int k = 0; k < kTRG; ++k) {
      float f[8], g[8];
      unpack8(v[k], f);
      unpack8(rv[k], g);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] += g[i];
      v[k] = pack8(f);  // the residual stream is carried in bf16: normalise exactly what is stored
      reinterpret_cast<u32x4*>(s_out + (r0 + k) * H)[t] = v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < kTRG; ++k) {
    float f[8];
    unpack8(v[k], f);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += f[i] * f[i];
    ss[k] = a;
  }
  t_row_sums<NT>(ss, red, rs);
#pragma unroll
  for (int k = 0; k < kTRG; ++k) asm volatile("" : "+v"(v[k]));
  float wf[8];
  unpack8(reinterpret_cast<const u32x4*>(w)[t], wf);
#pragma unroll
  for (int k = 0; k < kTRG; ++k) {
    const float rstd = rsqrtf(rs[k] * (1.f / H) + eps);
    if (t == 0) rstd_out[r0 + k] = rstd;
    float f[8];
    unpack8(v[k], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = f[i] * rstd * wf[i];
    v[k] = pack8(f);
    reinterpret_cast<u32x4*>(y + (r0 + k) * H)[t] = v[k];
  }
  t_store(v, yt + (int64_t)(8 * t) * ldt + r0, ldt);
}

// Backward: 4 columns per thread (NT = H / 4), so the 16 held rows of s and dy are 64 VGPRs (8 columns needed
// ~300 with the addresses and spilled at two waves per SIMD).
typedef unsigned int v2u32_t __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x2 pack4(const float* f) { return u32x2{pack2(f[0], f[1]), pack2(f[2], f[3])}; }

template <int NT, bool HAS_DRES>
__global__ void __launch_bounds__(NT) rms_bwd_t_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       bf16_t* __restrict__ dxt, float* __restrict__ dw_part,
                                                       int64_t ldt, int remap) {
  // rows are addressed through buffer descriptors: a scalar row offset + one per-lane VGPR offset (64-bit flat
  // addresses for the 16 rows x 4 tensors cost ~130 VGPRs and spilled)
  constexpr int H = NT * 4;
  __shared__ float red[kTRG * NT];
  __shared__ float rs[kTRG];
  const int t = threadIdx.x;
  const int64_t grp = t_row_group(remap);
  const int64_t r0 = grp * kTRG;
  const int bytes = (int)(ldt * H * 2);
  const auto rs_s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(s), 0, bytes, 0x00020000);
  const auto rs_dy = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(dy), 0, bytes, 0x00020000);
  const auto rs_dx = __builtin_amdgcn_make_buffer_rsrc(dx, 0, bytes, 0x00020000);
  const int vo = t * 8;
  const int row0 = (int)(r0 * H * 2);
  u32x2 sv[kTRG], dv[kTRG];
#pragma unroll
  for (int k = 0; k < kTRG; ++k) {
    sv[k] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_s, vo, row0 + k * H * 2, 0));
    dv[k] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_dy, vo, row0 + k * H * 2, 0));
  }
  float wf[4], dwa[4], a1[kTRG];
  unpack4(reinterpret_cast<const u32x2*>(w)[t], wf);
#pragma unroll
  for (int i = 0; i < 4; ++i) dwa[i] = 0.f;
#pragma unroll
  for (int k = 0; k < kTRG; ++k) {
    const float rstd = rstd_in[r0 + k];
    float xh[4], d[4];
    unpack4(sv[k], xh);
    unpack4(dv[k], d);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xh[i] *= rstd;
      dwa[i] += d[i] * xh[i];
      a += d[i] * wf[i] * xh[i];
    }
    a1[k] = a;
  }
  // the weight-gradient sums are finished BEFORE the reduction (else the compiler sinks them past it and keeps
  // the 16 unpacked rows live), and the rows stay packed across it
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(dwa[i]));
  t_row_sums<NT>(a1, red, rs);
#pragma unroll
  for (int k = 0; k < kTRG; ++k) asm volatile("" : "+v"(sv[k]), "+v"(dv[k]));
  const auto rs_dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(dres), 0, HAS_DRES ? bytes : 0, 0x00020000);
#pragma unroll
  for (int k = 0; k < kTRG; ++k) {
    const float rstd = rstd_in[r0 + k];
    const float m1 = rs[k] * (1.f / H);
    float xh[4], d[4], o[4];
    unpack4(sv[k], xh);
    unpack4(dv[k], d);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = rstd * (d[i] * wf[i] - xh[i] * rstd * m1);
    if (HAS_DRES) {
      float g[4];
      unpack4(__builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_dr, vo, row0 + k * H * 2, 0)), g);
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] += g[i];
    }
    dv[k] = pack4(o);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, dv[k]), rs_dx, vo, row0 + k * H * 2, 0);
  }
  // dx^T: column 4t + i, rows r0 .. r0 + 15 (two 16-B stores)
  const auto rs_dxt = __builtin_amdgcn_make_buffer_rsrc(dxt, 0, bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = i >> 1;
    u32x4 lo, hi;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a0 = dv[2 * k][d], a1v = dv[2 * k + 1][d], b0 = dv[8 + 2 * k][d], b1 = dv[8 + 2 * k + 1][d];
      lo[k] = (i & 1) ? __builtin_amdgcn_perm(a1v, a0, 0x07060302u) : __builtin_amdgcn_perm(a1v, a0, 0x05040100u);
      hi[k] = (i & 1) ? __builtin_amdgcn_perm(b1, b0, 0x07060302u) : __builtin_amdgcn_perm(b1, b0, 0x05040100u);
    }
    const int co = (int)((4 * t + i) * ldt * 2);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, lo), rs_dxt, co, (int)(r0 * 2), 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, hi), rs_dxt, co, (int)(r0 * 2) + 16, 0);
  }
  reinterpret_cast<f32x4*>(dw_part + grp * H)[t] = f32x4{dwa[0], dwa[1], dwa[2], dwa[3]};
}

// the transposed kernels address through 32-bit buffer descriptors / offsets: refuse shapes whose bytes reach 2 GiB
// (out-of-range buffer accesses would silently read 0 / drop stores); callers then take the plain norm kernels
static bool t_shape_ok(int rows, int H) {
  return (H == 2048 || H == 4096) && rows % kTRG == 0 && rows > 0 && (int64_t)rows * H * 2 < ((int64_t)1 << 31);
}
static int t_remap(int rows) { return (rows / kTRG) % 32 == 0 ? 1 : 0; }

int rms_norm_t_parts(int rows, int H) { return t_shape_ok(rows, H) ? rows / kTRG : 0; }

int rms_norm_fwd_t(const bf16_t* x, const bf16_t* r, const bf16_t* w, bf16_t* y, bf16_t* s_out, bf16_t* yt, float* rstd,
                   int rows, int H, float eps, hipStream_t stream) {
  if (!t_shape_ok(rows, H)) return -1;
  const int grid = rows / kTRG, remap = t_remap(rows);
#define RMS_FWD_T(NTv)                                                                                          \
  if (H == NTv * 8) {                                                                                           \
    if (r) rms_fwd_t_kernel<NTv, true><<<grid, NTv, 0, stream>>>(x, r, w, y, s_out, yt, rstd, rows, eps, remap);  \
    else rms_fwd_t_kernel<NTv, false><<<grid, NTv, 0, stream>>>(x, r, w, y, s_out, yt, rstd, rows, eps, remap);   \
    return 0;                                                                                                   \
  }
  RMS_FWD_T(256)
  RMS_FWD_T(512)
#undef RMS_FWD_T
  return -2;
}

int rms_norm_bwd_t(const bf16_t* dy, const bf16_t* s, const bf16_t* w, const float* rstd, const bf16_t* dres,
                   bf16_t* dx, bf16_t* dxt, float* part, bf16_t* dw, int rows, int H, int accumulate,
                   hipStream_t stream) {
  if (!t_shape_ok(rows, H)) return -1;
  const int grid = rows / kTRG, remap = t_remap(rows);
#define RMS_BWD_T(NTv)                                                                                          \
  if (H == NTv * 4) {                                                                                           \
    if (dres) rms_bwd_t_kernel<NTv, true><<<grid, NTv, 0, stream>>>(dy, s, w, rstd, dres, dx, dxt, part, rows, remap); \
    else rms_bwd_t_kernel<NTv, false><<<grid, NTv, 0, stream>>>(dy, s, w, rstd, dres, dx, dxt, part, rows, remap);     \
  }
  RMS_BWD_T(512)
  RMS_BWD_T(1024)
#undef RMS_BWD_T
  col_reduce_kernel<<<col_reduce_blocks(H), 1024, 0, stream>>>(part, grid, H, dw, accumulate);
  return 0;
}

// ---------------------------------------------------------------------------------------------------
// Bias gradient of a linear layer, db[c] (+)= sum_r dy[r, c] (GPT-2's biased projections): stage 1 sums a
// chunk of rows per block into fp32 partials (64 lanes x 16-byte column vectors, 4 row lanes, 4 rows in
// flight per lane), stage 2 is the norm backward's column reduce. Replaces a generic fp32 reduction + cast.
// ---------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) bias_partial_kernel(const bf16_t* __restrict__ dy, int rows, int H,
                                                           int rows_per_part, float* __restrict__ part) {
  const int H8 = H >> 3;
  const int c8 = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_part;
  const int r1 = min(rows, r0 + rows_per_part);
  __shared__ float red[3][64 * 8];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 < H8) {
    const u32x4* p = reinterpret_cast<const u32x4*>(dy) + c8;
    int r = r0 + rl;
    for (; r + 12 < r1; r += 16) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = p[(size_t)(r + 4 * u) * H8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
    }
    for (; r < r1; r += 4) {
      float f[8];
      unpack8(p[(size_t)r * H8], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
  }
  const int lane = threadIdx.x & 63;
  if (rl > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rl - 1][j * 64 + lane] = acc[j];
  }
  __syncthreads();
  if (rl == 0 && c8 < H8) {
    float* o = part + (size_t)blockIdx.y * H + (size_t)c8 * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = acc[j] + red[0][j * 64 + lane] + red[1][j * 64 + lane] + red[2][j * 64 + lane];
  }
}

int bias_grad_parts(int rows, int H) {
  const int gx = (H / 8 + 63) / 64;
  int p = (2048 + gx - 1) / gx;
  const int max_p = (rows + 63) / 64;
  if (p > max_p) p = max_p;
  if (p < 1) p = 1;
  const int per = (rows + p - 1) / p;
  return (rows + per - 1) / per;
}

int bias_grad(const bf16_t* dy, int rows, int H, float* part, bf16_t* db, int accumulate, hipStream_t stream) {
  if (H % 8 != 0 || rows <= 0) return -1;
  const int parts = bias_grad_parts(rows, H);
  const int per = (rows + parts - 1) / parts;
  bias_partial_kernel<<<dim3((H / 8 + 63) / 64, parts), 256, 0, stream>>>(dy, rows, H, per, part);
  col_reduce_kernel<<<col_reduce_blocks(H), 1024, 0, stream>>>(part, parts, H, db, accumulate);
  return 0;
}

}  // namespace kop
