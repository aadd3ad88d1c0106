// Flash attention forward + backward for gfx950 (CDNA4), bf16 in / fp32 accumulate, causal or full,
// grouped-query (Hq a multiple of Hkv), head_dim 64 or 128. Hand-written on the 32x32x16 bf16 MFMA.
//
// Tensors are addressed in the layout the transformer produces, with no transposes:
//   q/k/v element (b, s, h, d) at ptr + (b*S + s) * stride + h*D + d   (e.g. straight out of the fused
//   QKV projection [T, (Hq + 2 Hkv) D]); o / dq / dk / dv likewise; lse / delta are [B, Hq, S] fp32.
//
// FORWARD (one workgroup = NW waves = 32*NW query rows of one (b, q-head); 64-key K/V tiles)
//   * "swapped" scores: each wave computes S^T = K . Q^T with K as the MFMA A operand (ds_read_b128
//     rows of the XOR-swizzled K tile in LDS) and Q^T as the B operand (Q held in VGPRs for the whole
//     loop), so a lane owns ONE query row and its keys sit in the 16 accumulator registers: the row max
//     is an in-register max plus one cross-half exchange, no LDS round trip.
//   * P stays in registers: the S^T accumulator, packed to bf16, is directly the B operand of
//     O^T = V^T . P^T (the accumulator-as-operand identity); V^T fragments come from the row-major V
//     tile with ds_read_b64_tr_b16 (hardware transpose read).
//   * O^T is accumulated with the query on the lane, so the online-softmax rescale is a per-lane scalar.
//   * K/V tiles are register-staged (global loads for tile i+1 are issued before tile i's MFMAs and
//     written to the other LDS buffer after them: async-STAGE split), double-buffered, one barrier/tile.
//   * causal: waves skip tiles above their diagonal; blocks are issued heaviest-first and remapped so the
//     Hq/Hkv query heads that share a K/V head run on one XCD (L2 reuse of K/V).
// BACKWARD (FA2 structure, one workgroup = NW waves = 32*NW keys of one (b, q-head))
//   * each wave keeps dK^T and dV^T of its 32 keys in accumulator registers while sweeping the query
//     tiles (64 rows) that can see them; S and dP are computed with the KEY on the lane, so their
//     accumulators are directly the B operands of dV^T = dO^T P and dK^T = Q^T dS;
//   * -LSE and -delta are loaded as the initial accumulators of S and dP (p = exp2(c*acc), no subtract);
//   * dS^T goes through LDS once and dQ = dS K is summed over the workgroup's keys on chip, then added
//     to an fp32 dQ accumulator with one no-return float atomic per element per workgroup;
//   * per-q-head dK/dV partials (fp32) are summed over the GQA group and cast to bf16 by a finalize
//     kernel, which also casts dQ.
#include "common.h"
#include "kernels.h"

namespace kop {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

__device__ __forceinline__ bf16x4 lds_tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(p));
}
__device__ __forceinline__ bf16x8 lds_read8(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Byte offset of 16-byte chunk `ch` of row `row` in a swizzled [rows][ROWB bytes] LDS image.
// 256-B rows: chunk ^ (((row&3)<<2)|((row>>2)&3)) serves both ds_read_b128 row reads and
// ds_read_b64_tr_b16 transposed reads (guide T10 image (b)); 128-B rows: chunk ^ ((row>>1)&7).
template <int ROWB>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (ROWB == 256) return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  else return row * 128 + 16 * (ch ^ ((row >> 1) & 7));
}

// bijective XCD-aware remap of the linear block id (guide §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, slot = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// =============================================================================================
// forward
// =============================================================================================
template <int D, int NW>
__global__ void __launch_bounds__(NW * 64) fa_fwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                         const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                         float* __restrict__ lse, int B, int S, int Hq, int Hkv,
                                                         int64_t qs, int64_t ks, int64_t vs, int64_t os,
                                                         float scale_log2, int causal) {
  constexpr int BM = 32 * NW, BN = 64, ROWB = D * 2, CH = D / 8;
  constexpr int TILE = BN * ROWB;                     // bytes of one K or V tile
  constexpr int PT = (BN * CH) / (NW * 64);           // 16-B chunks per thread per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // buffers: K0 V0 K1 V1 (offsets computed, not stored: LDS pointer tables become static initialisers)
#define KBUF(buf) (smem + (buf) * 2 * TILE)
#define VBUF(buf) (smem + (buf) * 2 * TILE + TILE)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = S / BM;
  const int nwork = B * Hq * nqb;
  const int work = xcd_remap(blockIdx.x, nwork);
  const int qb = causal ? (nqb - 1 - work / (B * Hq)) : work / (B * Hq);
  const int rest = work % (B * Hq);
  const int b = rest / Hq, hq = rest % Hq;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;

  // Q^T operand fragments, resident for the whole loop
  bf16x8 qf[D / 16];
  {
    const bf16_t* qp = q + (int64_t)(b * S + q0w + r) * qs + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) oacc[i] = f32x16{0};
  float m = -INFINITY, l = 0.f;

  const int ntiles = causal ? (q0 + BM) / BN : S / BN;
  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  u32x4 kst[PT], vst[PT];
  auto stage_load = [&](int t) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = tid + i * NW * 64, row = c / CH, ch = c % CH;
      kst[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)(t * BN + row) * ks + ch * 8);
      vst[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)(t * BN + row) * vs + ch * 8);
    }
  };
  auto stage_write = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = tid + i * NW * 64, row = c / CH, ch = c % CH;
      *reinterpret_cast<u32x4*>(KBUF(buf) + swz<ROWB>(row, ch)) = kst[i];
      *reinterpret_cast<u32x4*>(VBUF(buf) + swz<ROWB>(row, ch)) = vst[i];
    }
  };

  stage_load(0);
  stage_write(0);
  __syncthreads();

  // transposed-read lane geometry (see header): group g = lane>>4, i = lane&15 -> (q', p')
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;

  for (int it = 0; it < ntiles; ++it) {
    const int buf = it & 1;
    if (it + 1 < ntiles) stage_load(it + 1);
    const int kv0 = it * BN;
    if (!causal || kv0 <= q0w + 31) {
      const char* Kb = KBUF(buf);
      const char* Vb = VBUF(buf);
      f32x16 s0 = f32x16{0}, s1 = f32x16{0};
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const bf16x8 ka = lds_read8(Kb + swz<ROWB>(r, 2 * kk + hh));
        const bf16x8 kb = lds_read8(Kb + swz<ROWB>(32 + r, 2 * kk + hh));
        s0 = mfma32(ka, qf[kk], s0);
        s1 = mfma32(kb, qf[kk], s1);
      }
      if (causal && kv0 + BN - 1 > q0w) {
        const int qi = q0w + r;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = kv0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
          if (key > qi) s0[j] = -INFINITY;
          if (key + 32 > qi) s1[j] = -INFINITY;
        }
      }
      float mx = s0[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s0[j]);
#pragma unroll
      for (int j = 0; j < 16; ++j) mx = fmaxf(mx, s1[j]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx * scale_log2);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s0[j] = __builtin_amdgcn_exp2f(fmaf(s0[j], scale_log2, -mnew));
        s1[j] = __builtin_amdgcn_exp2f(fmaf(s1[j], scale_log2, -mnew));
        ls += s0[j] + s1[j];
      }
      l = l * alpha + ls;
#pragma unroll
      for (int i = 0; i < D / 32; ++i) oacc[i] *= alpha;
      bf16x8 pf[4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const uint32_t a = pack2(s0[8 * s + j], s0[8 * s + j + 1]);
          const uint32_t c = pack2(s1[8 * s + j], s1[8 * s + j + 1]);
          pf[s][j] = (short)(a & 0xffff);
          pf[s][j + 1] = (short)(a >> 16);
          pf[2 + s][j] = (short)(c & 0xffff);
          pf[2 + s][j + 1] = (short)(c >> 16);
        }
      }
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int col = dt * 32 + 16 * tg1 + 4 * tp;
        const int ch = col >> 3, bo = (col & 7) * 2;
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int rowA = (ks4 >> 1) * 32 + 16 * (ks4 & 1) + 4 * hh + tq;
          const bf16x4 va = lds_tr_read(Vb + swz<ROWB>(rowA, ch) + bo);
          const bf16x4 vb = lds_tr_read(Vb + swz<ROWB>(rowA + 8, ch) + bo);
          oacc[dt] = mfma32(cat44(va, vb), pf[ks4], oacc[dt]);
        }
      }
    }
    if (it + 1 < ntiles) stage_write(buf ^ 1);
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / lt;
  if (hh == 0) lse[((int64_t)(b * Hq + hq)) * S + q0w + r] = (m + __log2f(lt)) * 0.69314718056f;
  bf16_t* op = o + (int64_t)(b * S + q0w + r) * os + hq * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u32x2 w;
      w[0] = pack2(oacc[dt][4 * g4] * inv, oacc[dt][4 * g4 + 1] * inv);
      w[1] = pack2(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
      *reinterpret_cast<u32x2*>(op + dt * 32 + 8 * g4 + 4 * hh) = w;
    }
  }
}

// =============================================================================================
// backward
// =============================================================================================

// delta[b, h, s] = sum_d dO * O   (16 lanes per row, 8 elements per lane for D = 128)
template <int D>
__global__ void __launch_bounds__(256) fa_bwd_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                           float* __restrict__ delta, int B, int S, int Hq, int64_t os,
                                                           int64_t dos) {
  constexpr int LPR = D / 8;  // lanes per row
  const int64_t rows = (int64_t)B * S * Hq;
  const int64_t row = (int64_t)blockIdx.x * (256 / LPR) + threadIdx.x / LPR;
  const int c = threadIdx.x % LPR;
  float a = 0.f;
  if (row < rows) {
    const int64_t t = row / Hq;  // token
    const int h = (int)(row % Hq);
    float x[8], y[8];
    unpack8(*reinterpret_cast<const u32x4*>(o + t * os + h * D + c * 8), x);
    unpack8(*reinterpret_cast<const u32x4*>(dout + t * dos + h * D + c * 8), y);
#pragma unroll
    for (int i = 0; i < 8; ++i) a += x[i] * y[i];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
  if (row < rows && c == 0) {
    const int64_t t = row / Hq;
    const int h = (int)(row % Hq);
    const int bb = (int)(t / S), s = (int)(t % S);
    delta[((int64_t)(bb * Hq + h)) * S + s] = a;
  }
}

template <int D, int NW>
__global__ void __launch_bounds__(NW * 64) fa_bwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                         const bf16_t* __restrict__ v, const bf16_t* __restrict__ dout,
                                                         const float* __restrict__ lse, const float* __restrict__ delta,
                                                         float* __restrict__ dq_acc, float* __restrict__ dk_part,
                                                         float* __restrict__ dv_part, int B, int S, int Hq, int Hkv,
                                                         int64_t qs, int64_t ks, int64_t vs, int64_t dos,
                                                         float scale, int causal) {
  constexpr int BN = 32 * NW, BQ = 64, ROWB = D * 2, CH = D / 8;
  constexpr int K_BYTES = BN * ROWB, Q_BYTES = BQ * ROWB, DS_BYTES = BN * BQ * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define Kl (smem)
#define Ql (smem + K_BYTES)
#define Ol (smem + K_BYTES + Q_BYTES)               // dO tile
#define Sl (smem + K_BYTES + 2 * Q_BYTES)           // dS^T tile [BN keys][64 q], 128-B rows

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int nkb = S / BN;
  const int nwork = B * Hq * nkb;
  const int work = xcd_remap(blockIdx.x, nwork);
  // heaviest (earliest keys under a causal mask) first
  const int kb = work / (B * Hq);
  const int rest = work % (B * Hq);
  const int b = rest / Hq, hq = rest % Hq;
  const int kvh = hq / (Hq / Hkv);
  const int k0 = kb * BN, k0w = k0 + 32 * wid;
  const float c2 = scale * 1.4426950408889634f;  // log2(e) * scale
  const float lse_mul = 1.4426950408889634f / c2;   // lse / scale

  // K block -> LDS (rows = keys of this workgroup)
  {
    const bf16_t* kp = k + (int64_t)(b * S + k0) * ks + kvh * D;
    for (int c = tid; c < BN * CH; c += NW * 64) {
      const int row = c / CH, ch = c % CH;
      *reinterpret_cast<u32x4*>(Kl + swz<ROWB>(row, ch)) =
          *reinterpret_cast<const u32x4*>(kp + (int64_t)row * ks + ch * 8);
    }
  }
  // V^T operand fragments of this wave's 32 keys, resident
  bf16x8 vf[D / 16];
  {
    const bf16_t* vp = v + (int64_t)(b * S + k0w + r) * vs + kvh * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) vf[kk] = *reinterpret_cast<const bf16x8*>(vp + 16 * kk);
  }
  f32x16 dkacc[D / 32], dvacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dkacc[i] = dvacc[i] = f32x16{0};

  const float* lse_h = lse + ((int64_t)(b * Hq + hq)) * S;
  const float* del_h = delta + ((int64_t)(b * Hq + hq)) * S;
  const bf16_t* qbase = q + (int64_t)(b * S) * qs + hq * D;
  const bf16_t* dobase = dout + (int64_t)(b * S) * dos + hq * D;
  const int qt0 = causal ? k0 / BQ : 0;
  const int nqt = S / BQ;
  constexpr int PT = (BQ * CH) / (NW * 64);

  for (int qt = qt0; qt < nqt; ++qt) {
    const int q0 = qt * BQ;
    __syncthreads();  // previous tile's readers are done with Q/dO/dS
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = tid + i * NW * 64, row = c / CH, ch = c % CH;
      const u32x4 a = *reinterpret_cast<const u32x4*>(qbase + (int64_t)(q0 + row) * qs + ch * 8);
      const u32x4 d = *reinterpret_cast<const u32x4*>(dobase + (int64_t)(q0 + row) * dos + ch * 8);
      *reinterpret_cast<u32x4*>(Ql + swz<ROWB>(row, ch)) = a;
      *reinterpret_cast<u32x4*>(Ol + swz<ROWB>(row, ch)) = d;
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qs0 = q0 + 32 * sub;
      u32x2 dsw[4];
      if (causal && qs0 + 31 < k0w) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) dsw[g4] = u32x2{0u, 0u};
      } else {
        // initial accumulators: -lse/scale and -delta for the 16 query rows this lane holds
        f32x16 sacc, dpacc;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 lv = *reinterpret_cast<const f32x4*>(lse_h + qs0 + 8 * g4 + 4 * hh);
          const f32x4 dv = *reinterpret_cast<const f32x4*>(del_h + qs0 + 8 * g4 + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sacc[4 * g4 + e] = -lv[e] * lse_mul;
            dpacc[4 * g4 + e] = -dv[e];
          }
        }
#pragma unroll
        for (int kk = 0; kk < D / 16; ++kk) {
          const bf16x8 qa = lds_read8(Ql + swz<ROWB>(32 * sub + r, 2 * kk + hh));
          const bf16x8 kbf = lds_read8(Kl + swz<ROWB>(32 * wid + r, 2 * kk + hh));
          const bf16x8 oa = lds_read8(Ol + swz<ROWB>(32 * sub + r, 2 * kk + hh));
          sacc = mfma32(qa, kbf, sacc);
          dpacc = mfma32(oa, vf[kk], dpacc);
        }
        // P and dS (key on the lane: key = k0w + r; query row from the register index)
        const int key = k0w + r;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int qi = qs0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
          float p = __builtin_amdgcn_exp2f(sacc[j] * c2);
          if (causal && key > qi) p = 0.f;
          sacc[j] = p;
          dpacc[j] = p * dpacc[j];
        }
        bf16x8 pb[2], sb[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const uint32_t a = pack2(sacc[8 * s + j], sacc[8 * s + j + 1]);
            const uint32_t c = pack2(dpacc[8 * s + j], dpacc[8 * s + j + 1]);
            pb[s][j] = (short)(a & 0xffff);
            pb[s][j + 1] = (short)(a >> 16);
            sb[s][j] = (short)(c & 0xffff);
            sb[s][j + 1] = (short)(c >> 16);
          }
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          dsw[g4][0] = pack2(dpacc[4 * g4], dpacc[4 * g4 + 1]);
          dsw[g4][1] = pack2(dpacc[4 * g4 + 2], dpacc[4 * g4 + 3]);
        }
        // dV^T += dO^T P,  dK^T += Q^T dS   (transposed reads of the dO / Q tiles)
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const int col = dt * 32 + 16 * tg1 + 4 * tp;
          const int ch = col >> 3, bo = (col & 7) * 2;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int rowA = 32 * sub + 16 * s + 4 * hh + tq;
            const bf16x8 oa = cat44(lds_tr_read(Ol + swz<ROWB>(rowA, ch) + bo), lds_tr_read(Ol + swz<ROWB>(rowA + 8, ch) + bo));
            const bf16x8 qa = cat44(lds_tr_read(Ql + swz<ROWB>(rowA, ch) + bo), lds_tr_read(Ql + swz<ROWB>(rowA + 8, ch) + bo));
            dvacc[dt] = mfma32(oa, pb[s], dvacc[dt]);
            dkacc[dt] = mfma32(qa, sb[s], dkacc[dt]);
          }
        }
      }
      // dS^T -> LDS: row = this lane's key (32*wid + r), 4 consecutive queries per 8-byte store
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int qcol = 32 * sub + 8 * g4 + 4 * hh;
        *reinterpret_cast<u32x2*>(Sl + swz<128>(32 * wid + r, qcol >> 3) + (qcol & 7) * 2) = dsw[g4];
      }
    }
    __syncthreads();
    // dQ[64 q][D] partial = dS [64 q][BN keys] . K [BN][D]; 32x32 output tiles split over the waves
    constexpr int NT = 2 * (D / 32);
#pragma unroll
    for (int u = 0; u < (NT + NW - 1) / NW; ++u) {
      const int ti = wid + u * NW;
      if (ti < NT) {
        const int qi = ti / (D / 32), dti = ti % (D / 32);
        f32x16 acc = f32x16{0};
        const int qcol = 32 * qi + 16 * tg1 + 4 * tp;  // dS^T columns (queries) for the A transposed read
        const int dcol = 32 * dti + 16 * tg1 + 4 * tp;  // K columns (d) for the B transposed read
#pragma unroll 4
        for (int kk = 0; kk < BN / 16; ++kk) {
          const int krow = 16 * kk + 8 * hh + tq;
          const bf16x8 a = cat44(lds_tr_read(Sl + swz<128>(krow, qcol >> 3) + (qcol & 7) * 2),
                                 lds_tr_read(Sl + swz<128>(krow + 4, qcol >> 3) + (qcol & 7) * 2));
          const bf16x8 bb = cat44(lds_tr_read(Kl + swz<ROWB>(krow, dcol >> 3) + (dcol & 7) * 2),
                                  lds_tr_read(Kl + swz<ROWB>(krow + 4, dcol >> 3) + (dcol & 7) * 2));
          acc = mfma32(a, bb, acc);
        }
        float* dqp = dq_acc + (int64_t)(b * S + q0 + 32 * qi) * Hq * D + hq * D + 32 * dti + r;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int row = (j & 3) + 8 * (j >> 2) + 4 * hh;
          atomicAdd(dqp + (int64_t)row * Hq * D, acc[j] * scale);
        }
      }
    }
  }
  // dK, dV partials of this q-head: lane holds dK^T[d][key = k0w + r]
  float* dkp = dk_part + (int64_t)(b * S + k0w + r) * Hq * D + hq * D;
  float* dvp = dv_part + (int64_t)(b * S + k0w + r) * Hq * D + hq * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = dt * 32 + 8 * g4 + 4 * hh;
      *reinterpret_cast<f32x4*>(dkp + d) = f32x4{dkacc[dt][4 * g4] * scale, dkacc[dt][4 * g4 + 1] * scale,
                                                 dkacc[dt][4 * g4 + 2] * scale, dkacc[dt][4 * g4 + 3] * scale};
      *reinterpret_cast<f32x4*>(dvp + d) =
          f32x4{dvacc[dt][4 * g4], dvacc[dt][4 * g4 + 1], dvacc[dt][4 * g4 + 2], dvacc[dt][4 * g4 + 3]};
    }
  }
}

// dq = bf16(dq_acc); dk/dv = bf16(sum over the GQA group of the per-q-head partials)
template <int D>
__global__ void __launch_bounds__(256) fa_bwd_finalize_kernel(const float* __restrict__ dq_acc,
                                                              const float* __restrict__ dk_part,
                                                              const float* __restrict__ dv_part, bf16_t* __restrict__ dq,
                                                              bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int64_t T,
                                                              int Hq, int Hkv, int64_t dqs, int64_t dks, int64_t dvs) {
  const int grp = Hq / Hkv;
  const int64_t nq = T * Hq * (D / 8), nk = T * Hkv * (D / 8);
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < nq + nk; it += (int64_t)gridDim.x * blockDim.x) {
    if (it < nq) {
      const int64_t t = it / (Hq * (D / 8));
      const int rem = (int)(it % (Hq * (D / 8)));
      const f32x4* src = reinterpret_cast<const f32x4*>(dq_acc + t * Hq * D + rem * 8);
      const f32x4 a = src[0], c = src[1];
      const float f[8] = {a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
      *reinterpret_cast<u32x4*>(dq + t * dqs + rem * 8) = pack8(f);
    } else {
      const int64_t j = it - nq;
      const int64_t t = j / (Hkv * (D / 8));
      const int rem = (int)(j % (Hkv * (D / 8)));
      const int h = rem / (D / 8), c8 = rem % (D / 8);
      float fk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int g = 0; g < grp; ++g) {
        const int64_t off = t * Hq * D + (int64_t)(h * grp + g) * D + c8 * 8;
        const f32x4* pk = reinterpret_cast<const f32x4*>(dk_part + off);
        const f32x4* pv = reinterpret_cast<const f32x4*>(dv_part + off);
        const f32x4 k0 = pk[0], k1 = pk[1], v0 = pv[0], v1 = pv[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          fk[e] += k0[e];
          fk[e + 4] += k1[e];
          fv[e] += v0[e];
          fv[e + 4] += v1[e];
        }
      }
      *reinterpret_cast<u32x4*>(dk + t * dks + h * D + c8 * 8) = pack8(fk);
      *reinterpret_cast<u32x4*>(dv + t * dvs + h * D + c8 * 8) = pack8(fv);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
constexpr int kFwdWaves = 4;
constexpr int kBwdWaves = 4;

int flash_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, bool causal,
                   hipStream_t stream) {
  constexpr int NW = kFwdWaves;
  if (S % (32 * NW) != 0 || Hq % Hkv != 0) return -1;
  if (qs % 8 || ks % 8 || vs % 8 || os % 8) return -2;
  const int grid = B * Hq * (S / (32 * NW));
  const float sl2 = scale * 1.4426950408889634f;
  if (D == 128) {
    const size_t lds = 4 * 64 * 256;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fa_fwd_kernel<128, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    fa_fwd_kernel<128, NW><<<grid, NW * 64, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal);
  } else if (D == 64) {
    const size_t lds = 4 * 64 * 128;
    fa_fwd_kernel<64, NW><<<grid, NW * 64, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal);
  } else {
    return -3;
  }
  return 0;
}

size_t flash_attn_bwd_workspace(int B, int S, int Hq, int D) {
  // dq_acc + dk_part + dv_part (fp32, [B*S, Hq, D] each) + delta [B, Hq, S]
  return (size_t)B * S * Hq * D * 4 * 3 + (size_t)B * Hq * S * 4;
}

int flash_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                   const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv, void* workspace, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dos, int64_t dqs,
                   int64_t dks, int64_t dvs, float scale, bool causal, hipStream_t stream) {
  constexpr int NW = kBwdWaves;
  if (S % (32 * NW) != 0 || S % 64 != 0 || Hq % Hkv != 0) return -1;
  const int64_t T = (int64_t)B * S;
  float* dq_acc = reinterpret_cast<float*>(workspace);
  float* dk_part = dq_acc + T * Hq * D;
  float* dv_part = dk_part + T * Hq * D;
  float* delta = dv_part + T * Hq * D;
  (void)hipMemsetAsync(dq_acc, 0, (size_t)T * Hq * D * 4, stream);
  const int rows_per_block = 256 / (D / 8);
  const int dgrid = (int)((T * Hq + rows_per_block - 1) / rows_per_block);
  const int grid = B * Hq * (S / (32 * NW));
  if (D == 128) {
    fa_bwd_delta_kernel<128><<<dgrid, 256, 0, stream>>>(o, dout, delta, B, S, Hq, os, dos);
    const size_t lds = (32 * NW) * 256 + 2 * 64 * 256 + (32 * NW) * 64 * 2;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fa_bwd_kernel<128, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    fa_bwd_kernel<128, NW><<<grid, NW * 64, lds, stream>>>(q, k, v, dout, lse, delta, dq_acc, dk_part, dv_part, B, S,
                                                            Hq, Hkv, qs, ks, vs, dos, scale, causal);
    fa_bwd_finalize_kernel<128><<<2048, 256, 0, stream>>>(dq_acc, dk_part, dv_part, dq, dk, dv, T, Hq, Hkv, dqs, dks,
                                                          dvs);
  } else if (D == 64) {
    fa_bwd_delta_kernel<64><<<dgrid, 256, 0, stream>>>(o, dout, delta, B, S, Hq, os, dos);
    const size_t lds = (32 * NW) * 128 + 2 * 64 * 128 + (32 * NW) * 64 * 2;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fa_bwd_kernel<64, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    fa_bwd_kernel<64, NW><<<grid, NW * 64, lds, stream>>>(q, k, v, dout, lse, delta, dq_acc, dk_part, dv_part, B, S,
                                                           Hq, Hkv, qs, ks, vs, dos, scale, causal);
    fa_bwd_finalize_kernel<64><<<2048, 256, 0, stream>>>(dq_acc, dk_part, dv_part, dq, dk, dv, T, Hq, Hkv, dqs, dks,
                                                         dvs);
  } else {
    return -3;
  }
  return 0;
}

}  // namespace kop
