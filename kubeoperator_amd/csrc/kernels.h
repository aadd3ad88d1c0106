// Host-side launcher declarations for every HIP kernel of kubeoperator_amd (gfx950).
// Each returns 0 on success or a negative code for an unsupported shape; all are asynchronous on
// `stream` and capture-safe (no allocation, no synchronisation).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace kop {
typedef uint16_t bf16_t;

// norms.hip
int norm_fwd(const bf16_t* x, const bf16_t* r, const bf16_t* w, const bf16_t* b, bf16_t* y, bf16_t* s_out, float* rstd,
             float* mean, int rows, int H, float eps, bool layernorm, hipStream_t stream);
int norm_bwd_partial_rows(int rows, int H);
// RMSNorm writing the transposed companion ([H, rows]) of its output (forward) / input gradient (backward)
int rms_norm_t_parts(int rows, int H);  // 0: shape not supported
int rms_norm_fwd_t(const bf16_t* x, const bf16_t* r, const bf16_t* w, bf16_t* y, bf16_t* s_out, bf16_t* yt, float* rstd,
                   int rows, int H, float eps, hipStream_t stream);
int rms_norm_bwd_t(const bf16_t* dy, const bf16_t* s, const bf16_t* w, const float* rstd, const bf16_t* dres,
                   bf16_t* dx, bf16_t* dxt, float* part, bf16_t* dw, int rows, int H, int accumulate,
                   hipStream_t stream);
int norm_bwd(const bf16_t* dy, const bf16_t* s, const bf16_t* w, const float* rstd, const float* mean,
             const bf16_t* dres, bf16_t* dx, float* part, bf16_t* dw, bf16_t* db, int rows, int H, bool layernorm,
             int accumulate, hipStream_t stream);  // dw == nullptr: fp32 partials only (norm_bwd_reduce folds them)
int norm_bwd_reduce(const float* part, int parts, int H, bf16_t* dw, bf16_t* db, bool layernorm, int accumulate,
                    hipStream_t stream);
int bias_grad_parts(int rows, int H);
int bias_grad(const bf16_t* dy, int rows, int H, float* part, bf16_t* db, int accumulate, hipStream_t stream);

// elementwise.hip
int rope_inplace(bf16_t* x, const float* cos_t, const float* sin_t, const int* pos, int64_t T, int S, int nheads,
                 int D, int64_t row_stride, bool inverse, hipStream_t stream);
int swiglu_fwd(const bf16_t* gu, bf16_t* h, int64_t T, int F, hipStream_t stream);
int swiglu_bwd(const bf16_t* gu, const bf16_t* dh, bf16_t* dgu, int64_t T, int F, hipStream_t stream);
int swiglu_fwd_t(const bf16_t* gu, bf16_t* h, bf16_t* ht, int64_t T, int F, hipStream_t stream);
int swiglu_bwd_t(const bf16_t* gu, const bf16_t* dh, bf16_t* dgu, bf16_t* dgut, int64_t T, int F, hipStream_t stream);
int gelu_fwd(const bf16_t* x, bf16_t* y, int64_t n, hipStream_t stream);
int gelu_bwd(const bf16_t* x, const bf16_t* dy, bf16_t* dx, int64_t n, hipStream_t stream);

// cross_entropy.hip
int cross_entropy_fwd(bf16_t* logits, int64_t ld, int64_t T, int V, const int64_t* tgt, int64_t ignore_index,
                      float* scale, float* loss_rows, float* lse_rows, bool write_grad, float grad_multiplier,
                      hipStream_t stream);

// adamw.hip
int adamw_step(bf16_t* p, const bf16_t* g, float* master, float* m, float* v, int64_t n, float lr, float b1, float b2,
               float eps, float wd, int step, float gscale, const float* gscale_dev, hipStream_t stream);
int adamw_step(bf16_t* p, const float* g, float* master, float* m, float* v, int64_t n, float lr, float b1, float b2,
               float eps, float wd, int step, float gscale, const float* gscale_dev, hipStream_t stream);
int grad_sumsq(const bf16_t* g, int64_t n, float* out, hipStream_t stream);
int grad_sumsq(const float* g, int64_t n, float* out, hipStream_t stream);
int clip_coef(const float* sumsq, float max_norm, float* coef, float* norm_out, hipStream_t stream);

// transpose.hip
int transpose2d(const bf16_t* in, bf16_t* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo, hipStream_t stream);
// RoPE in place on the first nheads heads (D = 128) + transpose of the whole [R, C] matrix into out [C, R]
int rope_transpose(bf16_t* x, bf16_t* out, const float* cos_t, const float* sin_t, int64_t R, int64_t C, int64_t ldx,
                   int64_t ldo, int S, int nheads, int D, bool inverse, hipStream_t stream);
int splitk_reduce(const float* part, int S, int64_t n, void* out, bool out_f32, bool accumulate, hipStream_t stream);

// fp8.hip: per-tensor OCP E4M3 quantization (current scaling): out = rne(clamp(x / scale)), scale = amax / 448;
// partial_ws: kFp8AmaxBlocks floats of scratch
constexpr int kFp8AmaxBlocks = 512;
int fp8_quantize(const bf16_t* x, int64_t n, uint8_t* out, float* scale, float* partial_ws, hipStream_t stream);
// cast with a known scale; transpose + cast (out[c][r] = e4m3(in[r][c] / scale))
int fp8_cast_scaled(const bf16_t* x, int64_t n, const float* scale, uint8_t* out, hipStream_t stream);
int fp8_transpose_cast(const bf16_t* in, uint8_t* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                       const float* scale, hipStream_t stream);

// flash_attn.hip
int flash_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, bool causal,
                   hipStream_t stream, bf16_t* ot = nullptr);
// 4-wave one-wave-per-SIMD forward (csrc/flash_fwd4.hip); sl2 = scale * log2(e); S % 256 == 0, D 64 / 128
// flash_fwd16.hip: the 8-wave forward on 16x16x32 MFMAs (KOP_FWD_VARIANT=16; D 64 / 128, S % 256 == 0)
int flash_attn_fwd16(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                     int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                     hipStream_t stream, bf16_t* ot);
int flash_attn_fwd4x64(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                       int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                       hipStream_t stream, bf16_t* ot);
size_t flash_attn_bwd_workspace(int B, int S, int Hq, int D);
// dQ algorithm: 10 = from the materialised dS (default), 9 = recompute S/dP (8-wave, staggered),
// 8 = lockstep, <8 = 4-wave.
// v < 0 only queries; returns the previous value. The workspace size depends on it.
int flash_attn_set_dq_variant(int v);
int flash_attn_set_dkdv_cfg(int c);
// heads per workgroup of the one-wave dK/dV kernel: 0 automatic, 1 / 2 / 4 / 8 forced; h < 0 only reads it
int flash_attn_set_dkdv_hpw(int h);
// forward kernel variant: -1 per-head-dim default, 8 / 9 / 10 the 8-wave kernel, < 8 the 4-wave kernel; returns the old
// setting (an argument below -1 only reads it)
int flash_attn_set_fwd_variant(int v);
// one-wave-per-SIMD dK/dV kernel (flash_bwd_w1.hip), D = 128 or 64, S % 256 == 0. ds: the query-major dS that
// fa_bwd_dq_ds_kernel reads (blk_layout: its wave-block form), or nullptr for the store-free build (dQ recomputed);
// qm is kept for the call sites and must be true when ds is set. Returns the number of fp32 dK / dV partials per
// GQA group left in dk_part / dv_part for fa_bwd_finalize_kernel (0: bf16 dK / dV written to dk / dv directly).
int flash_attn_bwd_dkdv64(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                           const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B,
                           int S, int Hq, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                           int64_t dvs, float scale, int causal, bool qm, bool blk_layout, hipStream_t stream);
// dK/dV at D = 64 with two waves per SIMD (flash_bwd_d64.hip), S % 256 == 0; dS in the key-major tiles of
// fa_bwd_dq_ds_kernel<KMAJ>. Returns the fp32 partials per GQA group left for the finalize pass (0: bf16 dK / dV written).
int flash_attn_bwd_dkdv_d64(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                            const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds,
                            int B, int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                            int64_t dvs, float scale, int causal, hipStream_t stream);
// waves per dQ-from-dS workgroup: 4 / 8, 0 automatic (4 at D = 64); v < 0 only reads it
int flash_attn_set_dq_nw(int v);
// workgroup shape of the D = 64 kernel (43 default, 44, 83); v < 0 only reads it
int flash_attn_set_d64_shape(int v);
int flash_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                   const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv, void* workspace, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dos, int64_t dqs,
                   int64_t dks, int64_t dvs, float scale, bool causal, hipStream_t stream);

// embedding.hip: dW[v] (+)= sum of dy[t] over ids[t] == v, from stably sorted int32 ids + the permutation (runs summed
// in token order); out [V, ldo] bf16 or fp32, zeroed by the caller when not accumulating
int embedding_bwd(const int* sorted_ids, const int64_t* perm, const bf16_t* dy, int64_t ldy, void* out, bool out_f32,
                  int64_t ldo, int T, int H, bool accumulate, hipStream_t stream);
// decode_attn.hip: one query token per sequence against a [B, Hkv, Smax, D] KV cache (lens[b] valid keys),
// split-K over 256-key chunks; part_o: B * Hq * nsplit * D floats, part_ml: B * Hq * nsplit * 2 floats
int decode_attn_set_mfma(int on);  // 1: MFMA pass 1 (default), 0: VALU form; < 0: query only
int decode_attn_splits(int max_len);
// gemv.hip: y[M, N] = x[M, K] . W[N, K]^T for M <= 8 decode rows (K a multiple of 1024); 1 = unsupported shape
int gemv_bf16(const bf16_t* x, const bf16_t* w, bf16_t* y, int M, int N, int K, int64_t xs, int64_t ws, int64_t ys,
              hipStream_t stream);
// RoPE at pos[b] on the Q and K heads of each fused QKV row (in place) + K / V rows appended to the caches at pos[b]
int decode_rope_append(bf16_t* qkv, int64_t qs, const float* cos_t, const float* sin_t, const int* pos, bf16_t* kc,
                       bf16_t* vc, int B, int Smax, int Hq, int Hkv, int D, hipStream_t stream);
int decode_attn(const bf16_t* q, int64_t qs, const bf16_t* kc, const bf16_t* vc, const int* lens, bf16_t* o,
                int64_t os, float* part_o, float* part_ml, int B, int Smax, int Hq, int Hkv, int D, int nsplit,
                float scale, hipStream_t stream);
}  // namespace kop
