// Stand-alone probe of the RMSNorm-with-transposed-companion forward (csrc/norms.hip rms_fwd_t) at the Llama-3-8B
// shape (T 8192 x H 4096, residual add): the production kernel against variants of its geometry (rows per workgroup,
// columns per thread) and store ablations, plus the plain norm + separate transpose it replaced. Build / run:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I kubeoperator_amd/csrc tools/norm_t_probe.hip -o /tmp/norm_t_probe
//   /tmp/norm_t_probe        (one JSON line per variant: us, TB/s of the bytes the variant must move)
#include <cstdio>
#include <vector>

#include "../kubeoperator_amd/csrc/norms.hip"
#include "../kubeoperator_amd/csrc/transpose.hip"

namespace kop {

template <int CPT>
struct Row {};
template <>
struct Row<8> {
  typedef u32x4 T;
};
template <>
struct Row<4> {
  typedef u32x2 T;
};

template <int CPT>
__device__ __forceinline__ void unpackN(const typename Row<CPT>::T& v, float* f) {
#pragma unroll
  for (int i = 0; i < CPT / 2; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
template <int CPT>
__device__ __forceinline__ typename Row<CPT>::T packN(const float* f) {
  typename Row<CPT>::T v;
#pragma unroll
  for (int i = 0; i < CPT / 2; ++i) v[i] = pack2(f[2 * i], f[2 * i + 1]);
  return v;
}

// generic variant: NT threads x CPT columns (H = NT * CPT), RG rows per workgroup; DO_Y / DO_T: write y / y^T
// REMAP: row groups dealt so that the RG-row segments of one 128-B y^T line share an XCD (blocks b, b+8, ...)
template <int NT, int CPT, int RG, bool DO_Y, bool DO_T, int TMODE = 0>
__global__ void __launch_bounds__(NT) fwdt_var(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                               const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                               bf16_t* __restrict__ s_out, bf16_t* __restrict__ yt,
                                               float* __restrict__ rstd_out, int64_t ldt, float eps) {
  typedef typename Row<CPT>::T RT;
  constexpr int H = NT * CPT, NW = NT / 64, RPW = RG / NW > 0 ? RG / NW : 1;
  constexpr int SEG = 128 / (2 * RG);  // row groups per 128-B y^T line
  // the reduction scratch and (TMODE > 0) the transpose tiles share one array: the tiles are written after the
  // barrier that ends the last read of the scratch
  constexpr int SCR = RG * NT * 4, TILES = TMODE > 0 ? NW * 512 * 32 : 0;
  __shared__ __attribute__((aligned(16))) char smem_[SCR > TILES ? SCR : TILES];
  float* red = reinterpret_cast<float*>(smem_);
  __shared__ float rs[RG];
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  int64_t grp = b;
  if constexpr (SEG > 1) {
    // SEG consecutive groups on blocks b, b+8, ..., b+8(SEG-1)
    grp = (int64_t)(b / (8 * SEG)) * (8 * SEG) + (b & 7) * SEG + ((b >> 3) % SEG);
  }
  const int64_t r0 = grp * RG;
  RT v[RG];
  float ss[RG];
#pragma unroll
  for (int k = 0; k < RG; ++k) v[k] = reinterpret_cast<const RT*>(x + (r0 + k) * H)[t];
  {
    RT rv[RG];
#pragma unroll
    for (int k = 0; k < RG; ++k) rv[k] = reinterpret_cast<const RT*>(r + (r0 + k) * H)[t];
#pragma unroll
    for (int k = 0; k < RG; ++k) {
      float f[CPT], g[CPT];
      unpackN<CPT>(v[k], f);
      unpackN<CPT>(rv[k], g);
#pragma unroll
      for (int i = 0; i < CPT; ++i) f[i] += g[i];
      v[k] = packN<CPT>(f);
      reinterpret_cast<RT*>(s_out + (r0 + k) * H)[t] = v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < RG; ++k) {
    float f[CPT];
    unpackN<CPT>(v[k], f);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) a += f[i] * f[i];
    ss[k] = a;
  }
#pragma unroll
  for (int k = 0; k < RG; ++k) red[k * NT + t] = ss[k];
  __syncthreads();
  {
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int kk = 0; kk < RPW; ++kk) {
      const int row = wv * RPW + kk;
      if (row < RG) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < NW; ++j) s += red[row * NT + lane + 64 * j];
        s = wave_sum(s);
        if (lane == 0) rs[row] = s;
      }
    }
  }
  __syncthreads();
  float wf[CPT];
  unpackN<CPT>(reinterpret_cast<const RT*>(w)[t], wf);
#pragma unroll
  for (int k = 0; k < RG; ++k) {
    const float rstd = rsqrtf(rs[k] * (1.f / H) + eps);
    if (t == 0) rstd_out[r0 + k] = rstd;
    float f[CPT];
    unpackN<CPT>(v[k], f);
#pragma unroll
    for (int i = 0; i < CPT; ++i) f[i] = f[i] * rstd * wf[i];
    v[k] = packN<CPT>(f);
    if constexpr (DO_Y) reinterpret_cast<RT*>(y + (r0 + k) * H)[t] = v[k];
  }
  if constexpr (DO_T && TMODE > 0) {
    // wave-local transpose through LDS (CPT 8, RG 16): the wave's 512 columns x 16 rows as [col][32 B], 16-B chunks
    // XOR-swizzled by the writing lane; read back so consecutive lanes hold consecutive columns
    static_assert(CPT == 8 && RG == 16, "LDS transpose variant: 8 columns x 16 rows per lane");
    const int lane = t & 63, wv = t >> 6;
    char* tb = smem_ + wv * 512 * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int d = i >> 1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u32x4 o;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const uint32_t a0 = v[8 * h + 2 * kk][d], a1 = v[8 * h + 2 * kk + 1][d];
          o[kk] = (i & 1) ? __builtin_amdgcn_perm(a1, a0, 0x07060302u) : __builtin_amdgcn_perm(a1, a0, 0x05040100u);
        }
        *reinterpret_cast<u32x4*>(tb + 256 * lane + 16 * ((2 * i + h) ^ (lane & 15))) = o;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    bf16_t* ytw = yt + (int64_t)(512 * wv) * ldt + r0;
    if constexpr (TMODE == 1) {  // lane l: column 64 i + l, both halves
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 64 * i + lane;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32x4 o = *reinterpret_cast<const u32x4*>(tb + 256 * (c >> 3) + 16 * ((2 * (c & 7) + h) ^ ((c >> 3) & 15)));
          *reinterpret_cast<u32x4*>(ytw + (int64_t)c * ldt + 8 * h) = o;
        }
      }
    } else {  // lanes 2m, 2m + 1: the two halves of column 32 i + m
      const int h = lane & 1, m = lane >> 1;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 32 * i + m;
        const u32x4 o = *reinterpret_cast<const u32x4*>(tb + 256 * (c >> 3) + 16 * ((2 * (c & 7) + h) ^ ((c >> 3) & 15)));
        *reinterpret_cast<u32x4*>(ytw + (int64_t)c * ldt + 8 * h) = o;
      }
    }
  }
  if constexpr (DO_T && TMODE == 0) {
    // column CPT*t + i, rows r0 .. r0 + RG - 1: RG / 8 16-B stores
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int d = i >> 1;
      bf16_t* col = yt + (int64_t)(CPT * t + i) * ldt + r0;
#pragma unroll
      for (int q = 0; q < RG / 8; ++q) {
        u32x4 o;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const uint32_t a0 = v[8 * q + 2 * kk][d], a1 = v[8 * q + 2 * kk + 1][d];
          o[kk] = (i & 1) ? __builtin_amdgcn_perm(a1, a0, 0x07060302u) : __builtin_amdgcn_perm(a1, a0, 0x05040100u);
        }
        reinterpret_cast<u32x4*>(col)[q] = o;
      }
    }
  }
}

}  // namespace kop

using namespace kop;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void fill_rand(bf16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float f = ((h & 0xffff) / 65536.0f - 0.5f) * 4.f;
    p[i] = f2bf(f);
  }
}

int main() {
  const int T = 8192, H = 4096;
  const size_t n = (size_t)T * H, mb = n * 2;
  const int NSET = 4;  // rotating input / output sets: > 256 MB touched between two uses of a buffer
  std::vector<bf16_t*> X(NSET), R(NSET), Y(NSET), S(NSET), YT(NSET);
  for (int i = 0; i < NSET; ++i) {
    CK(hipMalloc(&X[i], mb));
    CK(hipMalloc(&R[i], mb));
    CK(hipMalloc(&Y[i], mb));
    CK(hipMalloc(&S[i], mb));
    CK(hipMalloc(&YT[i], mb));
    fill_rand<<<1024, 256>>>(X[i], n, 17 + i);
    fill_rand<<<1024, 256>>>(R[i], n, 91 + i);
  }
  bf16_t* W;
  float* rstd;
  CK(hipMalloc(&W, H * 2));
  CK(hipMalloc(&rstd, T * 4));
  fill_rand<<<16, 256>>>(W, H, 5);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto&& launch) {
    for (int i = 0; i < 3; ++i) launch(i % NSET);
    (void)hipDeviceSynchronize();
    const int iters = 48;
    (void)hipEventRecord(e0);
    for (int i = 0; i < iters; ++i) launch(i % NSET);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000.0 / iters;
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"TB/s\": %.2f}\n", name, us, bytes / us / 1e6);
    fflush(stdout);
  };
  const double b5 = 5.0 * mb, b4 = 4.0 * mb, b3 = 3.0 * mb;
  timeit("prod rms_fwd_t (RG16, 8 cols/thread, 512 thr)", b5,
         [&](int i) { rms_norm_fwd_t(X[i], R[i], W, Y[i], S[i], YT[i], rstd, T, H, 1e-5f, 0); });
  timeit("plain norm_fwd", b4, [&](int i) { norm_fwd(X[i], R[i], W, nullptr, Y[i], S[i], rstd, nullptr, T, H, 1e-5f, false, 0); });
  timeit("transpose", 2.0 * mb, [&](int i) { transpose2d(Y[i], YT[i], T, H, H, T, 0); });
#define VAR(NAME, BYTES, NT, CPT, RG, DY, DT, ...)                                                                    \
  timeit(NAME, BYTES, [&](int i) {                                                                                  \
    fwdt_var<NT, CPT, RG, DY, DT, ##__VA_ARGS__><<<T / RG, NT>>>(X[i], R[i], W, Y[i], S[i], YT[i], rstd, T, 1e-5f);  \
  })
  VAR("var RG16 cpt8 nt512", b5, 512, 8, 16, true, true);
  VAR("var RG16 cpt8 nt512 no-yT", b4, 512, 8, 16, true, false);
  VAR("var RG16 cpt8 nt512 no-y", b4, 512, 8, 16, false, true);
  VAR("var RG16 cpt8 nt512 s-only", b3, 512, 8, 16, false, false);
  VAR("var RG16 lds-T lane/col", b5, 512, 8, 16, true, true, 1);
  VAR("var RG16 lds-T 2 lanes/col", b5, 512, 8, 16, true, true, 2);
  VAR("var RG16 lds-T lane/col no-y", b4, 512, 8, 16, false, true, 1);
  VAR("var RG16 lds-T 2 lanes/col no-y", b4, 512, 8, 16, false, true, 2);
  CK(hipDeviceSynchronize());
  return 0;
}
