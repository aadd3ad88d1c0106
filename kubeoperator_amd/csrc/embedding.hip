// Embedding weight gradient for gfx950: dW[v] (+)= sum of dy[t] over the tokens t with ids[t] == v.
//
// PyTorch's embedding_dense_backward materialises a dense fp32 [V, H] scratch (zero-filled), sorts, reduces into it
// and casts -- for Llama-3-8B's 128,256 x 4,096 table a 2.1 GB fp32 fill + a 1 GB bf16 fill + a 1 GB copy per micro-
// batch, and ~40 launches (GPT-2-small: the host time of those launches left the compute stream idle ~1 ms per micro-
// batch, profiles/r5_gpt2_host_gap.md). Here the caller sorts the token ids stably (one radix sort) and this kernel
// sums each run of equal ids straight into the gradient buffer: no scratch, touched rows only.
//
// One wave per sorted position; the wave whose position starts a run sums the run's rows IN SORTED ORDER -- token order,
// the sort being stable -- so the result is deterministic. Lanes own 8 columns (one 16-B load per row), the wave sweeps
// the row 512 columns at a time with 8 fp32 accumulators per lane, and writes (or adds into) the bf16 / fp32 output row.
#include "common.h"
#include "kernels.h"

namespace kop {

template <typename OutT>
__device__ __forceinline__ void out_row8(OutT* o, const float* acc, bool accumulate);

template <>
__device__ __forceinline__ void out_row8<bf16_t>(bf16_t* o, const float* acc, bool accumulate) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = acc[i];
  if (accumulate) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(o), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += f[i];
  }
  *reinterpret_cast<u32x4*>(o) = pack8(a);
}

template <>
__device__ __forceinline__ void out_row8<float>(float* o, const float* acc, bool accumulate) {
  f32x4 lo = {acc[0], acc[1], acc[2], acc[3]}, hi = {acc[4], acc[5], acc[6], acc[7]};
  if (accumulate) {
    lo += reinterpret_cast<const f32x4*>(o)[0];
    hi += reinterpret_cast<const f32x4*>(o)[1];
  }
  reinterpret_cast<f32x4*>(o)[0] = lo;
  reinterpret_cast<f32x4*>(o)[1] = hi;
}

template <typename OutT>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int* __restrict__ sid, const int64_t* __restrict__ perm,
                                                        const bf16_t* __restrict__ dy, int64_t ldy,
                                                        OutT* __restrict__ out, int64_t ldo, int T, int H,
                                                        int accumulate) {
  const int lane = threadIdx.x & 63;
  const int pos = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (pos >= T) return;
  const int v = sid[pos];
  if (pos > 0 && sid[pos - 1] == v) return;  // not the start of a run
  // run end: 64 sorted ids per probe
  int end = pos + 1;
  for (;;) {
    const int j = end + lane;
    const bool same = j < T && sid[j] == v;
    const uint64_t m = __ballot(same);
    if (m == ~0ull) {
      end += 64;
      continue;
    }
    end += __builtin_ctzll(~m);  // first lane whose id differs (or past T)
    break;
  }
  OutT* orow = out + (int64_t)v * ldo;
  for (int c0 = 0; c0 < H; c0 += 512) {
    const int c = c0 + 8 * lane;
    if (c >= H) continue;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = pos;
    // 4 rows in flight per lane
    for (; k + 4 <= end; k += 4) {
      u32x4 r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = *reinterpret_cast<const u32x4*>(dy + perm[k + u] * ldy + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(r[u], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += f[i];
      }
    }
    for (; k < end; ++k) {
      float f[8];
      unpack8(*reinterpret_cast<const u32x4*>(dy + perm[k] * ldy + c), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    out_row8<OutT>(orow + c, acc, accumulate != 0);
  }
}

int embedding_bwd(const int* sorted_ids, const int64_t* perm, const bf16_t* dy, int64_t ldy, void* out, bool out_f32,
                  int64_t ldo, int T, int H, bool accumulate, hipStream_t stream) {
  if (H % 8 != 0 || ldy % 8 != 0 || ldo % 8 != 0 || T <= 0) return -1;
  const int grid = (T + 3) / 4;
  if (out_f32)
    embed_bwd_kernel<float><<<grid, 256, 0, stream>>>(sorted_ids, perm, dy, ldy, reinterpret_cast<float*>(out), ldo,
                                                      T, H, accumulate ? 1 : 0);
  else
    embed_bwd_kernel<bf16_t><<<grid, 256, 0, stream>>>(sorted_ids, perm, dy, ldy, reinterpret_cast<bf16_t*>(out), ldo,
                                                       T, H, accumulate ? 1 : 0);
  return 0;
}

}  // namespace kop
