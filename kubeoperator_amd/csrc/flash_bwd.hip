// Flash attention BACKWARD for gfx950 (CDNA4 / MI355X), bf16 in / fp32 accumulate, causal or full, GQA,
// head_dim 64 or 128, on the 32x32x16 bf16 MFMA. Same tensor addressing as flash_fwd.hip.
//
// Why two main kernels and no dQ atomics: on MI355X float atomics execute at the memory side at
// ~1.3 TB/s chip-wide (MI355X_MICROARCH.md "Global float atomics"). The one-kernel FA2 form adds a dQ
// partial per (key block, query tile): at Llama-3-8B shape (S 8192, 32 heads, 128-key blocks) that is
// 4.3 GB of atomic bytes per layer -> a 3.3 ms floor, more than all the MFMA work. Recomputing S and dP
// in a second sweep costs 2 extra MFMA products instead, at full MFMA rate and with no cross-workgroup
// traffic, so:
//
//   fa_bwd_delta_kernel : delta = rowsum(dO * O)                                   [B, Hq, S] fp32
//   fa_bwd_dkdv_kernel  : one workgroup = 4 waves = 128 keys of one (b, q-head); sweeps the query
//       tiles (64 rows) that see them. Key on the lane: S = Q.K^T and dP = dO.V^T with K^T / V^T
//       operand fragments resident in VGPRs, -LSE/scale and -delta loaded as the initial accumulators
//       (p = exp2(c*acc), no subtraction); their accumulators are directly the B operands of
//       dV^T += dO^T.P and dK^T += Q^T.dS (transposed reads of the Q / dO tiles). Q, dO, LSE, delta
//       tiles arrive by LDS-DMA into a 2-deep ring behind counted vmcnt + raw barriers.
//       Writes per-q-head fp32 dK/dV partials (summed over the GQA group by the finalize kernel).
//   fa_bwd_dq_kernel    : one workgroup = 4 waves = 128 queries of one (b, q-head); sweeps the key
//       tiles (64 keys) like the forward pass. Query on the lane: S^T = K.Q^T and dP^T = V.dO^T with
//       Q^T / dO^T resident, per-lane scalar LSE and delta, dS^T = P^T (dP^T - delta) packed to bf16
//       is directly the B operand of dQ^T += K^T.dS^T (K^T by transposed reads of the K tile).
//       dQ is written once, in bf16, straight into the strided dQKV gradient.
//   fa_bwd_finalize_kernel : dK, dV = bf16(sum over the GQA group of the per-q-head partials).
//
// Default since the dS variant (KOP_DQ_VARIANT 10): the dK/dV kernel also stores its bf16 dS tiles
// ([B, Hq, S, S], ~1 TB/s of extra writes it hides under its MFMA work) and fa_bwd_dq_ds_kernel computes
// dQ = scale * dS.K from them -- one MFMA product plus an HBM stream instead of three products; at
// Llama-3-8B shape the backward drops from 3.31 to 2.89 ms (profiles/r1_attn_dq10_bench.log). The
// buffer is capped at 16 GiB; longer sequences fall back to the recompute kernels.
#include "attn_common.h"
#include "kernels.h"

namespace kop {

// delta[b, h, s] = sum_d dO * O
// and the dK/dV kernel's accumulator initialisers: nlse = -lse / scale (S = Q.K^T starts there, so
// p = exp2(c * acc)) and ndelta = -delta (dP starts there) -- no negate / scale VALU per stage.
// A workgroup owns DROWS consecutive positions s of ONE (b, h): the three [B, Hq, S] fp32 outputs and the lse input
// are contiguous runs (the token-major order before wrote and read them 4 bytes at a time at a stride of S * 4),
// each lane group of D/8 lanes reads one 16-byte chunk of its row, and every lane has all of its rows' loads in
// flight before the first reduction.
constexpr int kDeltaRows = 64;
template <int D>
__global__ void __launch_bounds__(256) fa_bwd_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse, float* __restrict__ delta,
                                                           float* __restrict__ nlse, float* __restrict__ ndelta,
                                                           float lse_mul, int B, int S, int Hq, int64_t os,
                                                           int64_t dos) {
  constexpr int LPR = D / 8;              // lanes per row
  constexpr int RPI = 256 / LPR;          // rows per pass of the block
  constexpr int NP = kDeltaRows / RPI;    // passes
  const int nsb = (S + kDeltaRows - 1) / kDeltaRows;
  const int bh = blockIdx.x / nsb, s0 = (blockIdx.x % nsb) * kDeltaRows;
  const int bb = bh / Hq, h = bh % Hq;
  const int c = threadIdx.x % LPR, r = threadIdx.x / LPR;
  u32x4 xo[NP], xd[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int s = s0 + p * RPI + r;
    if (s < S) {
      const int64_t t = (int64_t)bb * S + s;
      xo[p] = *reinterpret_cast<const u32x4*>(o + t * os + h * D + c * 8);
      xd[p] = *reinterpret_cast<const u32x4*>(dout + t * dos + h * D + c * 8);
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int s = s0 + p * RPI + r;
    float x[8], y[8], a = 0.f;
    if (s < S) {
      unpack8(xo[p], x);
      unpack8(xd[p], y);
#pragma unroll
      for (int i = 0; i < 8; ++i) a += x[i] * y[i];
    }
    a = group_sum<LPR>(a);  // DPP inside the row's lane group (a __shfl_xor loop was ds_bpermute round trips)
    if (s < S && c == 0) {
      const int64_t i = (int64_t)bh * S + s;
      delta[i] = a;
      ndelta[i] = -a;
      nlse[i] = -lse[i] * lse_mul;
    }
  }
}

template <int D>
static void launch_delta(const bf16_t* o, const bf16_t* dout, const float* lse, float* delta, float* nlse, float* ndelta,
                         float lse_mul, int B, int S, int Hq, int64_t os, int64_t dos, hipStream_t stream) {
  static_assert(kDeltaRows % (256 / (D / 8)) == 0, "whole passes");
  const int nsb = (S + kDeltaRows - 1) / kDeltaRows;
  fa_bwd_delta_kernel<D><<<B * Hq * nsb, 256, 0, stream>>>(o, dout, lse, delta, nlse, ndelta, lse_mul, B, S, Hq, os, dos);
}

// =============================================================================================
// dK / dV
// =============================================================================================
// slot of key (k & 15) inside its 16-key group in the dS buffer: keys {0-3, 8-11, 4-7, 12-15} so lane half hh
// of the dQ kernel reads the 8 keys {4hh..4hh+3, 8+4hh..8+4hh+3} of its MFMA B fragment as one 16-B chunk
__device__ __forceinline__ int ds_slot(int key) {
  return (key & ~15) | (key & 3) | ((key & 4) << 1) | ((key & 8) >> 1);
}

// DIRECT (no GQA, Hq == Hkv): the workgroup's sums are already the final dK / dV, written as bf16 straight
// into dk_part / dv_part reinterpreted as the bf16 outputs (row strides dks / dvs), with no finalize pass.
// NW waves x 32 keys per workgroup; NSTAGE-deep ring of query stages (prefetch distance NSTAGE - 1).
// NW = 4: two workgroups per CU; NW = 8: one 512-thread workgroup per CU (each staged Q/dO tile then serves
// 256 keys, and the LDS left over holds a 3-deep ring).
template <int D, int NW, bool WDS = false, bool DIRECT = false, int NSTAGE = 2>
__global__ void __launch_bounds__(NW * 64, (NW >= 8 ? 1 : 2)) fa_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ nlse, const float* __restrict__ ndelta,
    float* __restrict__ dk_part, float* __restrict__ dv_part, bf16_t* __restrict__ ds, int B, int S, int Hq,
    int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, float scale, int causal, int64_t dks = 0,
    int64_t dvs = 0) {
  // LDS: the workgroup's K block (BN rows, read as the S = Q.K^T B operand) + a 2-deep ring of 32-query
  // stages {Q, dO, lse/delta}; 66 KiB at D = 128 so two workgroups share a CU (V^T stays in VGPRs).
  constexpr int BN = 32 * NW, BQ = 32, ROWB = D * 2;
  constexpr int KB = BN * ROWB;                  // K block bytes
  constexpr int QT = BQ * ROWB;                  // bytes of one Q (or dO) stage
  constexpr int STAGE = 2 * QT + 1024;           // Q, dO, {lse[32], delta[32]} piece
  constexpr int MYP = (2 * QT / 1024) / NW;      // Q/dO DMA pieces per wave per stage
  static_assert(MYP * NW * 1024 == 2 * QT, "stage must split evenly over the waves");
  static_assert(NSTAGE == 2 || NSTAGE == 3, "2- or 3-deep stage ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const Kl = smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int nkb = S / BN;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nkb);
  const int kb = aw.rank;  // heaviest key blocks (earliest keys under a causal mask) first
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int k0 = kb * BN, k0w = k0 + 32 * wid;
  const float c2 = scale * 1.4426950408889634f;

  const float* lse_h = nlse + ((int64_t)(b * Hq + hq)) * S;
  const float* del_h = ndelta + ((int64_t)(b * Hq + hq)) * S;
  const bf16_t* qbase = q + (int64_t)(b * S) * qs + hq * D;
  const bf16_t* dobase = dout + (int64_t)(b * S) * dos + hq * D;
  // first query tile that sees any key of this workgroup; the waves of later keys skip leading tiles
  const int qt0 = causal ? k0 / BQ : 0;
  const int nqt = S / BQ;

  auto issue = [&](int qt, int stage) {
    char* base = smem + KB + stage * STAGE;
    const int q0 = qt * BQ;
    dma_tile_a<ROWB, NW, BQ>(base, qbase + (int64_t)q0 * qs, qs, wid, lane);
    dma_tile_a<ROWB, NW, BQ>(base + QT, dobase + (int64_t)q0 * dos, dos, wid, lane);
    if (wid == 0) {
      // lanes 0-7: lse[q0..q0+31], lanes 8-15: delta[...]; lanes 16-63 repeat into the unused tail
      const int l = lane & 15;
      const float* src = (l < 8 ? lse_h + q0 + 4 * l : del_h + q0 + 4 * (l - 8));
      glds16(src, base + 2 * QT);
    }
  };

  // K block of the workgroup -> LDS (counted with the first stage)
  dma_tile_a<ROWB, NW, BN>(Kl, k + (int64_t)(b * S + k0) * ks + kvh * D, ks, wid, lane);
  issue(qt0, 0);
  if constexpr (NSTAGE == 3) {
    if (qt0 + 1 < nqt) issue(qt0 + 1, 1);
  }
  // lane bases of the sub-tiled images (swza): row reads of rows r (+32*i) at chunk 2kk+hh, transposed
  // reads of rows R0 + 4hh + tq
  constexpr int RB = ROWB * 8;
  const int rb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int rb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  const int tb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int tb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);
  auto raddr = [&](const char* base, int kk) {
    return base + ((kk & 1) ? rb_lane1 : rb_lane0) + 512 * (kk >> 1);
  };
  // V^T operand fragments of this wave's 32 keys (B operand of dP = dO.V^T; key = k0w + r), resident
  bf16x8 vf[D / 16];
  {
    const bf16_t* vp = v + (int64_t)(b * S + k0w + r) * vs + kvh * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) vf[kk] = *reinterpret_cast<const bf16x8*>(vp + 16 * kk);
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(vf[kk]));
  }
  f32x16 dkacc[D / 32], dvacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dkacc[i] = dvacc[i] = f32x16{0};

  // one barrier per stage: it publishes stage qt AND proves every wave is done with stage qt-1, whose slot
  // the DMA of stage qt+1 then refills (prefetch distance: one stage of compute)
  // the previous stage's dS stores are this wave's 16 youngest vector-memory ops: they may stay in flight
  // across the barrier (only this stage's DMA, issued before them, must have landed)
  bool stored = false;
  // the causal mask is needed only in the workgroup's diagonal region (its first BN/BQ = NW query stages):
  // the stage body is instantiated twice -- masked for those stages, mask-free for the rest -- so the 32
  // compare/select VALU per stage (~1 per MFMA in this VALU-issue-bound loop) leave the steady state
  // (two loops, not a branch in one body: a branch merged the live ranges and spilled)
  auto body = [&](int qt, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int stage = (qt - qt0) % NSTAGE;
    if constexpr (NSTAGE == 2) {
      if (WDS && stored) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // in flight, oldest first: ..., DMA(qt), [stores(qt-2)], DMA(qt+1), [stores(qt-1)]: wait until only
      // DMA(qt+1) and the previous stage's stores may remain (everything older, DMA(qt) included, landed)
      const bool nxt = qt + 1 < nqt;
      const bool st = WDS && stored;
      if (!nxt) {
        if (st) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (wid == 0) {  // wave 0 also issues the lse / delta piece
        if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MYP + 1 + 16) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MYP + 1) : "memory");
      } else {
        if (st) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MYP + 16) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MYP) : "memory");
      }
    }
    stored = false;
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (qt + NSTAGE - 1 < nqt) issue(qt + NSTAGE - 1, (qt + NSTAGE - 1 - qt0) % NSTAGE);
    const char* Ql = smem + KB + stage * STAGE;
    const char* Ol = Ql + QT;
    const float* LD = reinterpret_cast<const float*>(Ql + 2 * QT);
    const int qs0 = qt * BQ;
    if (!causal || qs0 + 31 >= k0w) {  // else every query of the tile precedes every key of the wave
      f32x16 sacc, dpacc;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int qr = 8 * g4 + 4 * hh;
        const f32x4 lv = *reinterpret_cast<const f32x4*>(LD + qr);
        const f32x4 dv = *reinterpret_cast<const f32x4*>(LD + 32 + qr);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sacc[4 * g4 + e] = lv[e];
          dpacc[4 * g4 + e] = dv[e];
        }
      }
      (void)raddr;
      {
        // per k-step one group of 3 row reads (Q row r, K row 32*wid + r, dO row r), two in flight
        const uint32_t qb0 = lds_addr(Ql) + rb_lane0, qb1 = lds_addr(Ql) + rb_lane1;
        const uint32_t ob0 = lds_addr(Ol) + rb_lane0, ob1 = lds_addr(Ol) + rb_lane1;
        const uint32_t kw0 = lds_addr(Kl) + rb_lane0 + RB * 4 * wid, kw1 = lds_addr(Kl) + rb_lane1 + RB * 4 * wid;
        auto grp = [&](auto kc, bf16x8* dst) {
          constexpr int kk = decltype(kc)::value;
          dst[0] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? qb1 : qb0);
          dst[1] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? kw1 : kw0);
          dst[2] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? ob1 : ob0);
        };
        constexpr int NK = D / 16;
        bf16x8 ga[3], gb[3];
        grp(std::integral_constant<int, 0>{}, ga);
        grp(std::integral_constant<int, 1>{}, gb);
        static_for<NK>([&](auto kc) {
          constexpr int kk = decltype(kc)::value;
          bf16x8* cur = (kk & 1) ? gb : ga;
          if constexpr (kk + 1 < NK) wait_rows3<3>(cur);
          else wait_rows3<0>(cur);
          sacc = mfma32(cur[0], cur[1], sacc);
          dpacc = mfma32(cur[2], vf[kk], dpacc);
          if constexpr (kk + 2 < NK) grp(std::integral_constant<int, kk + 2>{}, cur);
        });
      }
      const int key = k0w + r;
      // key > query  <=>  kd > (j & 3) + 8 * (j >> 2): one subtraction, then compares with constants
      const int kd = key - qs0 - 4 * hh;
      (void)kd;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float p = __builtin_amdgcn_exp2f(sacc[j] * c2);
        if constexpr (MASK) {
          if (kd > (j & 3) + 8 * (j >> 2)) p = 0.f;
        }
        sacc[j] = p;
        dpacc[j] = p * dpacc[j];
      }
      const bf16x8 pb[2] = {pack_acc8(sacc, 0), pack_acc8(sacc, 1)};
      const bf16x8 sb[2] = {pack_acc8(dpacc, 0), pack_acc8(dpacc, 1)};
      if constexpr (WDS) {
        // unscaled bf16 dS -> ds[b, hq, q, slot(key)]: per store the 32 keys of a row half-wave are 64
        // contiguous bytes (the same rounding dK uses below);
        // issued before the dK/dV products so their latency hides under them
        // wave-uniform row pointer (SGPRs) + one 32-bit lane offset: no per-store 64-bit address VGPRs
        // saddr stores: 64-bit row pointer in SGPRs (SALU adds), 32-bit lane byte offset in one VGPR; the
        // loop-top vmcnt(0) retires them (hipcc does not see these stores)
        const uint32_t loff = 2u * (uint32_t)(4 * hh * S + ds_slot(key));
        const uint64_t row0 = (uint64_t)(uintptr_t)(ds + ((int64_t)(b * Hq + hq) * S + qs0) * S);
        const u32x4 w0 = __builtin_bit_cast(u32x4, sb[0]), w1 = __builtin_bit_cast(u32x4, sb[1]);
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          const uint32_t w = (j < 8) ? w0[j >> 1] : w1[(j - 8) >> 1];
          const uint64_t ra = row0 + (uint64_t)(2 * ((j & 3) + 8 * (j >> 2))) * (uint64_t)S;
          const uint64_t rb = ra + 2ull * (uint64_t)S;
          asm volatile("global_store_short %0, %1, %2" ::"v"(loff), "v"(w), "s"(ra) : "memory");
          asm volatile("global_store_short_d16_hi %0, %1, %2" ::"v"(loff), "v"(w), "s"(rb) : "memory");
        }
        stored = true;
      }
      // transposed dO / Q reads: rows 16s + 4hh + tq (+8) are tb_lane[(row0>>3)&1] + RB*(row0>>3), column
      // block dt is +512*dt (sub-tiled image, all immediates)
      const uint32_t o0 = lds_addr(Ol) + tb_lane0, o1 = lds_addr(Ol) + tb_lane1;
      const uint32_t q0a = lds_addr(Ql) + tb_lane0, q1a = lds_addr(Ql) + tb_lane1;
      static_for<D / 32>([&](auto dtc) {
        constexpr int dt = decltype(dtc)::value;
        bf16x4 t[8];
        static_for<2>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          t[4 * s + 0] = lds_tr_read_off<RB * 2 * s + 512 * dt>(o0);
          t[4 * s + 1] = lds_tr_read_off<RB * (2 * s + 1) + 512 * dt>(o1);
          t[4 * s + 2] = lds_tr_read_off<RB * 2 * s + 512 * dt>(q0a);
          t[4 * s + 3] = lds_tr_read_off<RB * (2 * s + 1) + 512 * dt>(q1a);
        });
        wait_tr<8, 0>(t);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dvacc[dt] = mfma32(cat44(t[4 * s], t[4 * s + 1]), pb[s], dvacc[dt]);
          dkacc[dt] = mfma32(cat44(t[4 * s + 2], t[4 * s + 3]), sb[s], dkacc[dt]);
        }
      });
    }
    asm volatile("" ::: "memory");
  };
  int qt = qt0;
  if (causal) {
    const int qd = qt0 + NW < nqt ? qt0 + NW : nqt;
    for (; qt < qd; ++qt) body(qt, std::true_type{});
  }
  for (; qt < nqt; ++qt) body(qt, std::false_type{});
  if constexpr (DIRECT) {
    bf16_t* dkb = reinterpret_cast<bf16_t*>(dk_part) + (int64_t)(b * S + k0w + r) * dks + hq * D;
    bf16_t* dvb = reinterpret_cast<bf16_t*>(dv_part) + (int64_t)(b * S + k0w + r) * dvs + hq * D;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * hh;
        *reinterpret_cast<u32x2*>(dkb + d) =
            u32x2{pack2(dkacc[dt][4 * g4] * scale, dkacc[dt][4 * g4 + 1] * scale),
                  pack2(dkacc[dt][4 * g4 + 2] * scale, dkacc[dt][4 * g4 + 3] * scale)};
        *reinterpret_cast<u32x2*>(dvb + d) =
            u32x2{pack2(dvacc[dt][4 * g4], dvacc[dt][4 * g4 + 1]), pack2(dvacc[dt][4 * g4 + 2], dvacc[dt][4 * g4 + 3])};
      }
    }
    return;
  }
  // per-q-head partials: lane holds dK^T[d][key = k0w + r]
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

// =============================================================================================
// dQ
// =============================================================================================
template <int D, int NW>
__global__ void __launch_bounds__(NW * 64, 2) fa_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dq, int B, int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos,
    int64_t dqs, float scale, int causal) {
  constexpr int BM = 32 * NW, BN = 64, ROWB = D * 2;
  constexpr int TILE = BN * ROWB;
  constexpr int PPW = (TILE / 1024) / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(buf) (smem + (buf) * 2 * TILE)
#define VBUF(buf) (smem + (buf) * 2 * TILE + TILE)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;
  const float c2 = scale * 1.4426950408889634f;

  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  auto issue = [&](int t, int buf) {
    dma_tile<ROWB, NW, BN>(KBUF(buf), kbase + (int64_t)(t * BN) * ks, ks, wid, lane);
    dma_tile<ROWB, NW, BN>(VBUF(buf), vbase + (int64_t)(t * BN) * vs, vs, wid, lane);
  };
  issue(0, 0);

  const int qi = q0w + r;
  bf16x8 qf[D / 16], of[D / 16];
  float lse2, dl;
  {
    const bf16_t* qp = q + (int64_t)(b * S + qi) * qs + hq * D + 8 * hh;
    const bf16_t* op = dout + (int64_t)(b * S + qi) * dos + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) {
      qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
      of[kk] = *reinterpret_cast<const bf16x8*>(op + 16 * kk);
    }
    lse2 = lse[((int64_t)(b * Hq + hq)) * S + qi] * 1.4426950408889634f;
    dl = delta[((int64_t)(b * Hq + hq)) * S + qi];
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(qf[kk]), "+v"(of[kk]));
    asm volatile("" : "+v"(lse2), "+v"(dl));
  }
  f32x16 dqacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dqacc[i] = f32x16{0};

  for (int it = 0; it < ntiles; ++it) {
    const int buf = it & 1;
    if (it + 1 < ntiles) {
      issue(it + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int kv0 = it * BN;
    if (!causal || kv0 <= q0w + 31) {
      const char* Kb = KBUF(buf);
      const char* Vb = VBUF(buf);
      f32x16 s0 = f32x16{0}, s1 = f32x16{0}, p0 = f32x16{0}, p1 = f32x16{0};
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        const bf16x8 ka = lds_read8(Kb + swz<ROWB>(r, 2 * kk + hh));
        const bf16x8 kb = lds_read8(Kb + swz<ROWB>(32 + r, 2 * kk + hh));
        const bf16x8 va = lds_read8(Vb + swz<ROWB>(r, 2 * kk + hh));
        const bf16x8 vb = lds_read8(Vb + swz<ROWB>(32 + r, 2 * kk + hh));
        s0 = mfma32(ka, qf[kk], s0);
        s1 = mfma32(kb, qf[kk], s1);
        p0 = mfma32(va, of[kk], p0);
        p1 = mfma32(vb, of[kk], p1);
      }
      const bool diag = causal && kv0 + BN - 1 > q0w;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int key = kv0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
        float pa = __builtin_amdgcn_exp2f(fmaf(s0[j], c2, -lse2));
        float pb = __builtin_amdgcn_exp2f(fmaf(s1[j], c2, -lse2));
        if (diag && key > qi) pa = 0.f;
        if (diag && key + 32 > qi) pb = 0.f;
        s0[j] = pa * (p0[j] - dl);
        s1[j] = pb * (p1[j] - dl);
      }
      bf16x8 sf[4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const uint32_t a = pack2(s0[8 * s + j], s0[8 * s + j + 1]);
          const uint32_t c = pack2(s1[8 * s + j], s1[8 * s + j + 1]);
          sf[s][j] = (short)(a & 0xffff);
          sf[s][j + 1] = (short)(a >> 16);
          sf[2 + s][j] = (short)(c & 0xffff);
          sf[2 + s][j + 1] = (short)(c >> 16);
        }
      }
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int col = dt * 32 + 16 * tg1 + 4 * tp;
        const int ch = col >> 3, bo = (col & 7) * 2;
        bf16x4 t[8];
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int rowA = (ks4 >> 1) * 32 + 16 * (ks4 & 1) + 4 * hh + tq;
          t[2 * ks4] = lds_tr_read_asm(Kb + swz<ROWB>(rowA, ch) + bo);
          t[2 * ks4 + 1] = lds_tr_read_asm(Kb + swz<ROWB>(rowA + 8, ch) + bo);
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                       "+v"(t[7]));
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) dqacc[dt] = mfma32(cat44(t[2 * ks4], t[2 * ks4 + 1]), sf[ks4], dqacc[dt]);
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#undef KBUF
#undef VBUF
  bf16_t* dp = dq + (int64_t)(b * S + qi) * dqs + hq * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u32x2 w;
      w[0] = pack2(dqacc[dt][4 * g4] * scale, dqacc[dt][4 * g4 + 1] * scale);
      w[1] = pack2(dqacc[dt][4 * g4 + 2] * scale, dqacc[dt][4 * g4 + 3] * scale);
      *reinterpret_cast<u32x2*>(dp + dt * 32 + 8 * g4 + 4 * hh) = w;
    }
  }
}

// 8-wave dQ: 512 threads = 256 query rows of one (b, q-head), same K/V tile stream and staggered halves as
// fa_fwd8_kernel (flash_fwd.hip): waves 4-7 run half a tile behind (dS + dQ MFMAs of tile t-1, then the
// S^T / dP^T MFMAs of tile t, carried across the barrier), 4-slot LDS ring, one barrier per tile.
template <int D, bool STAGGER>
__global__ void __launch_bounds__(512, 1) fa_bwd_dq8_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dq, int B, int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos,
    int64_t dqs, float scale, int causal) {
  constexpr int NW = 8, BM = 256, BN = 64, ROWB = D * 2;
  constexpr int TILE = BN * ROWB;
  constexpr int NSLOT = STAGGER ? 4 : 3;
  constexpr int PPW = (TILE / 1024) / NW;
  static_assert(PPW >= 1 && PPW * NW * 1024 == TILE, "tile must split evenly over the waves");
  constexpr int DT = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(sl) (smem + (sl) * 2 * TILE)
#define VBUF(sl) (smem + (sl) * 2 * TILE + TILE)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const bool late = STAGGER && wid >= 4;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;
  const float c2 = scale * 1.4426950408889634f;

  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  auto issue = [&](int t) {
    dma_tile_a<ROWB, NW, BN>(KBUF(t % NSLOT), kbase + (int64_t)(t * BN) * ks, ks, wid, lane);
    dma_tile_a<ROWB, NW, BN>(VBUF(t % NSLOT), vbase + (int64_t)(t * BN) * vs, vs, wid, lane);
  };
  issue(0);
  if (ntiles > 1) issue(1);

  const int qi = q0w + r;
  bf16x8 qf[D / 16], of[D / 16];
  float lse2, dl;
  {
    const bf16_t* qp = q + (int64_t)(b * S + qi) * qs + hq * D + 8 * hh;
    const bf16_t* op = dout + (int64_t)(b * S + qi) * dos + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) {
      qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
      of[kk] = *reinterpret_cast<const bf16x8*>(op + 16 * kk);
    }
    lse2 = lse[((int64_t)(b * Hq + hq)) * S + qi] * 1.4426950408889634f;
    dl = delta[((int64_t)(b * Hq + hq)) * S + qi];
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(qf[kk]), "+v"(of[kk]));
    asm volatile("" : "+v"(lse2), "+v"(dl));
  }
  f32x16 dqacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dqacc[i] = f32x16{0};
  if (wid >= 4) __builtin_amdgcn_s_setprio(1);

  // lane bases of the sub-tiled image (swza), as in fa_fwd8_kernel: rows r / r+32 at chunk 2kk+hh, and
  // the transposed reads of rows R0 + 4hh + tq
  constexpr int RB = ROWB * 8;
  const int rb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int rb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  const int tb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int tb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);
  auto raddr = [&](const char* base, int kk, int half) {
    return base + ((kk & 1) ? rb_lane1 : rb_lane0) + RB * 4 * half + 512 * (kk >> 1);
  };
  // S^T = K.Q^T and dP^T = V.dO^T for the 64 keys of tile t
  auto scores = [&](int t, f32x16& s0, f32x16& s1, f32x16& p0, f32x16& p1) {
    const char* Kb = KBUF(t % NSLOT);
    const char* Vb = VBUF(t % NSLOT);
    s0 = s1 = p0 = p1 = f32x16{0};
    (void)raddr;
    // per k-step one group of 4 row reads (K rows r, r+32; V rows r, r+32), two groups in flight
    const uint32_t kb0 = lds_addr(Kb) + rb_lane0, kb1 = lds_addr(Kb) + rb_lane1;
    const uint32_t vb0 = lds_addr(Vb) + rb_lane0, vb1 = lds_addr(Vb) + rb_lane1;
    auto grp = [&](auto kc, bf16x8* dst) {
      constexpr int kk = decltype(kc)::value;
      dst[0] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? kb1 : kb0);
      dst[1] = lds_read8_off<RB * 4 + 512 * (kk >> 1)>((kk & 1) ? kb1 : kb0);
      dst[2] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? vb1 : vb0);
      dst[3] = lds_read8_off<RB * 4 + 512 * (kk >> 1)>((kk & 1) ? vb1 : vb0);
    };
    constexpr int NK = D / 16;
    bf16x8 ga[4], gb[4];
    grp(std::integral_constant<int, 0>{}, ga);
    grp(std::integral_constant<int, 1>{}, gb);
    static_for<NK>([&](auto kc) {
      constexpr int kk = decltype(kc)::value;
      bf16x8* cur = (kk & 1) ? gb : ga;
      if constexpr (kk + 1 < NK) wait_rows4<4>(cur);
      else wait_rows4<0>(cur);
      s0 = mfma32(cur[0], qf[kk], s0);
      s1 = mfma32(cur[1], qf[kk], s1);
      p0 = mfma32(cur[2], of[kk], p0);
      p1 = mfma32(cur[3], of[kk], p1);
      if constexpr (kk + 2 < NK) grp(std::integral_constant<int, kk + 2>{}, cur);
    });
  };
  // K^T fragments of key group ks4 for every output block dt (independent dQ accumulators per MFMA)
  constexpr int NR = 2 * DT;
  auto kread = [&](const char* Kb, auto ks4c, bf16x4* t) {
    constexpr int ks4 = decltype(ks4c)::value;
    constexpr int R0 = (ks4 >> 1) * 32 + 16 * (ks4 & 1);
    const uint32_t b0 = lds_addr(Kb) + tb_lane0, b1 = lds_addr(Kb) + tb_lane1;
    static_for<DT>([&](auto dtc) {
      constexpr int dt = decltype(dtc)::value;
      t[2 * dt] = lds_tr_read_off<RB * (R0 >> 3) + 512 * dt>(((R0 >> 3) & 1) ? b1 : b0);
      t[2 * dt + 1] = lds_tr_read_off<RB * ((R0 + 8) >> 3) + 512 * dt>((((R0 + 8) >> 3) & 1) ? b1 : b0);
    });
  };
  // dS^T = P^T (dP^T - delta) and dQ^T += K^T . dS^T
  auto grad = [&](int t, f32x16& s0, f32x16& s1, f32x16& p0, f32x16& p1) {
    const char* Kb = KBUF(t % NSLOT);
    bf16x4 ta[NR];
    kread(Kb, std::integral_constant<int, 0>{}, ta);  // flies under the dS VALU work
    const int kv0 = t * BN;
    const bool diag = causal && kv0 + BN - 1 > q0w;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int key = kv0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
      float pa = __builtin_amdgcn_exp2f(fmaf(s0[j], c2, -lse2));
      float pb = __builtin_amdgcn_exp2f(fmaf(s1[j], c2, -lse2));
      if (diag && key > qi) pa = 0.f;
      if (diag && key + 32 > qi) pb = 0.f;
      s0[j] = pa * (p0[j] - dl);
      s1[j] = pb * (p1[j] - dl);
    }
    const bf16x8 sf[4] = {pack_acc8(s0, 0), pack_acc8(s0, 1), pack_acc8(s1, 0), pack_acc8(s1, 1)};
    static_for<4>([&](auto ks4c) {
      constexpr int ks4 = decltype(ks4c)::value;
      if constexpr (ks4 > 0) kread(Kb, ks4c, ta);
      wait_tr<NR, 0>(ta);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) dqacc[dt] = mfma32(cat44(ta[2 * dt], ta[2 * dt + 1]), sf[ks4], dqacc[dt]);
    });
  };

  const int nloop = ntiles + (STAGGER ? 1 : 0);
  auto top = [&](int it) {
    if (it < ntiles) {
      if (it + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < ntiles) issue(it + 2);
  };
  if (late) {
    f32x16 s0, s1, p0, p1;
    bool pending = false;
    for (int it = 0; it < nloop; ++it) {
      top(it);
      if (pending) grad(it - 1, s0, s1, p0, p1);
      pending = it < ntiles && (!causal || it * BN <= q0w + 31);
      if (pending) scores(it, s0, s1, p0, p1);
      asm volatile("" ::: "memory");
    }
  } else {
    for (int it = 0; it < nloop; ++it) {
      top(it);
      if (it < ntiles && (!causal || it * BN <= q0w + 31)) {
        f32x16 s0, s1, p0, p1;
        scores(it, s0, s1, p0, p1);
        grad(it, s0, s1, p0, p1);
      }
      asm volatile("" ::: "memory");
    }
  }
#undef KBUF
#undef VBUF
  bf16_t* dp = dq + (int64_t)(b * S + qi) * dqs + hq * D;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u32x2 w;
      w[0] = pack2(dqacc[dt][4 * g4] * scale, dqacc[dt][4 * g4 + 1] * scale);
      w[1] = pack2(dqacc[dt][4 * g4 + 2] * scale, dqacc[dt][4 * g4 + 3] * scale);
      *reinterpret_cast<u32x2*>(dp + dt * 32 + 8 * g4 + 4 * hh) = w;
    }
  }
}

// dQ from the materialised dS (KOP_DQ_VARIANT 10): dQ = scale * dS . K with dS written by the dK/dV kernel,
// so neither S nor dP is recomputed (the recompute dQ kernels above redo 2 of their 3 MFMA products).
// One workgroup = 8 waves = 256 query rows of HP q-heads sharing a KV head, 64-key tiles: the K tile (read transposed, as
// the forward reads V) and the [256 x 64] dS tile both arrive by LDS-DMA into a 3-slot ring; per 16-key
// group a lane's B fragment dS^T is one ds_read_b128 of its row (keys are stored in MFMA order, ds_slot),
// and dQ^T += K^T . dS^T accumulates in DT independent chains. The dS stream (half of B*Hq*S*S bf16 under
// a causal mask) makes this kernel HBM-bound, ~3x cheaper than recomputing.
// BLK: dS in the wave-block layout of fa_bwd_dkdv64_kernel ([B, Hq, S/32, S/64, 32 queries, 64 slots]); the
// tile's dS rows of one head and 32-query stage are then one contiguous 4-KB block.
// KMAJ: dS in the tiles of fa_bwd_dkdv64_kernel<QM = false, BLK> ([B, Hq, S/64, S/32] x 4 KB: block 2c + s holds, for
// key 32c + r, queries 16s + 4hh + 0..3 and 16s + 8 + 4hh + 0..3 as the two 8-B halves of chunk 32hh + (r ^ 4hh ^ 8s)):
// each wave's 32 query rows of a 64-key tile
// are one such tile, copied lane-linear into LDS and read with ds_read_b64_tr_b16 -- lane 4q + p of a 16-lane group
// names key row q (4 consecutive elements = 4 queries); the XOR spreads one 32-lane half's 32 reads over all 64 banks.
// The two transposed reads of a k-step take keys R0 + 4hh + 0..3 and R0 + 8 + 4hh + 0..3, the K^T operand's k order.
// NW: waves per workgroup (32 query rows each). 8: one 512-thread workgroup per CU; 4: two 256-thread workgroups per
// CU (at D = 64 a 3-slot ring is 72 KB), so one workgroup's ramp-up / drain overlaps the other's stream.
template <int D, int HP, bool BLK = false, bool NTL = false, bool KMAJ = false, int NW = 8>
__global__ void __launch_bounds__(NW * 64, 1) fa_bwd_dq_ds_kernel(const bf16_t* __restrict__ ds,
                                                                  const bf16_t* __restrict__ k, bf16_t* __restrict__ dq,
                                                                  int B, int S, int Hq, int Hkv, int64_t ks, int64_t dqs,
                                                                  float scale, int causal) {
  // HP q-heads of one GQA group per workgroup (RH = 32 NW / HP query rows each) share every K tile: the
  // kernel streams dS, so K re-reads from L2/MALL are the traffic worth cutting
  constexpr int BM = 32 * NW, RH = BM / HP, WPH = NW / HP, BN = 64, ROWB = D * 2, NSLOT = 3;
  static_assert(NW % HP == 0, "every wave within one head");
  constexpr int KT = BN * ROWB, DST = BM * BN * 2, SLOT = KT + DST;
  constexpr int PPW = (KT / 1024) / NW + (DST / 1024) / NW;  // DMA pieces per wave per tile
  static_assert((KT / 1024) % NW == 0 && (DST / 1024) % NW == 0, "tiles must split evenly over the waves");
  static_assert(RH % 32 == 0, "each wave owns 32 rows of one head");
  constexpr int DT = D / 32, NR = 2 * DT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int ngrp = Hq / HP, nqb = S / RH;
  const AttnWork aw = attn_work(blockIdx.x, B, ngrp, (Hq / Hkv) / HP, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hg = aw.unit;
  const int kvh = (hg * HP) / (Hq / Hkv);
  const int hq = hg * HP + wid / WPH;  // this wave's head
  const int q0 = qb * RH, q0w = q0 + 32 * (wid % WPH);
  const int ntiles = causal ? (q0 + RH + BN - 1) / BN : S / BN;
  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  // dS tile: rows 0..255 of the image = HP heads x RH rows; an 8-row DMA piece never straddles heads
  const int lrow = (lane & 31) >> 2, lhi = lane >> 5, lslot = lane & 3;
  auto issue = [&](int t) {
    char* sl = smem + (t % NSLOT) * SLOT;
    dma_tile_a<ROWB, NW, BN>(sl, kbase + (int64_t)(t * BN) * ks, ks, wid, lane);
#pragma unroll
    for (int i = 0; i < (DST / 1024) / NW; ++i) {
      const int piece = wid + i * NW;
      if constexpr (KMAJ) {  // piece = 1 KB of image tile piece / 4 (= rows 32 * tile ..), lane-linear
        const int tile = piece >> 2, sub = piece & 3;
        const bf16_t* src = ds + (((int64_t)(b * Hq + hg * HP + (32 * tile) / RH) * (S / 64) + t) * (S / 32) +
                                  (q0 + (32 * tile) % RH) / 32) * 2048 + sub * 512 + lane * 8;
        if constexpr (NTL) glds16_nt(src, sl + KT + piece * 1024);
        else glds16(src, sl + KT + piece * 1024);
        continue;
      }
      const int row = 8 * piece + lrow;
      const int ch = 4 * lhi + (lslot ^ ((row >> 2) & 3));
      const int qrow = q0 + row % RH;
      const bf16_t* src =
          BLK ? ds + (((int64_t)(b * Hq + hg * HP + row / RH) * (S / 32) + qrow / 32) * (S / 64) + t) * 2048 +
                    (qrow % 32) * 64 + ch * 8
              : ds + ((int64_t)(b * Hq + hg * HP + row / RH) * S + qrow) * S + t * BN + ch * 8;
      if constexpr (NTL) glds16_nt(src, sl + KT + piece * 1024);  // dS: read once, by this CU only
      else glds16(src, sl + KT + piece * 1024);
    }
  };
  issue(0);
  if (ntiles > 1) issue(1);

  constexpr int RB = ROWB * 8;
  // K^T transposed reads (as the forward's V^T): rows R0 + 4hh + tq (+8) at column block dt
  const int kb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int kb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);
  // dS row reads of image row 32*wid + r at chunk 2*ks4 + hh in the sub-tiled [256][128 B] image
  const int ds_lane0 = 4096 * wid + 1024 * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int ds_lane1 = 4096 * wid + 1024 * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  // KMAJ transposed reads: lane 4q + p of its 16-lane group names key R0 + 4hh + q (+8 for the second read), queries
  // 16 tg1 + 4p .. +3, i.e. query half s = tg1, storing lane half p & 1, 8-B half p >> 1 of its chunk; R0 = 16 ks4 adds
  // 2048 (ks4 >> 1) + 256 (ks4 & 1) bytes
  const int kr1 = 4 * hh + tq, kr2 = kr1 + 8, ksh = tp & 1;
  const int dk_lane = 4096 * wid + 1024 * tg1 + 16 * (32 * ksh + (kr1 ^ (4 * ksh) ^ (8 * tg1))) + 8 * (tp >> 1);
  const int dk_lane2 = 4096 * wid + 1024 * tg1 + 16 * (32 * ksh + (kr2 ^ (4 * ksh) ^ (8 * tg1))) + 8 * (tp >> 1);
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = f32x16{0};
  const int qi = q0w + r;

  for (int it = 0; it < ntiles; ++it) {
    if (it + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < ntiles) issue(it + 2);
    const int kv0 = it * BN;
    if (!causal || kv0 <= q0w + 31) {
      const char* sl = smem + (it % NSLOT) * SLOT;
      const uint32_t kb0 = lds_addr(sl) + kb_lane0, kb1 = lds_addr(sl) + kb_lane1;
      const uint32_t db0 = lds_addr(sl + KT) + ds_lane0, db1 = lds_addr(sl + KT) + ds_lane1;
      bf16x8 f[4];
      const uint32_t dk0 = lds_addr(sl + KT) + dk_lane, dk1 = lds_addr(sl + KT) + dk_lane2;
      (void)dk0;
      (void)dk1;
      static_for<4>([&](auto ks4c) {
        constexpr int ks4 = decltype(ks4c)::value;
        if constexpr (KMAJ)
          f[ks4] = cat44(lds_tr_read_off<2048 * (ks4 >> 1) + 256 * (ks4 & 1)>(dk0),
                         lds_tr_read_off<2048 * (ks4 >> 1) + 256 * (ks4 & 1)>(dk1));
        else
          f[ks4] = lds_read8_off<512 * (ks4 >> 1)>((ks4 & 1) ? db1 : db0);
      });
      const bool diag = causal && kv0 + BN - 1 > q0w;
      static_for<4>([&](auto ks4c) {
        constexpr int ks4 = decltype(ks4c)::value;
        constexpr int R0 = 16 * ks4;
        bf16x4 t[NR];
        static_for<DT>([&](auto dtc) {
          constexpr int dt = decltype(dtc)::value;
          t[2 * dt] = lds_tr_read_off<RB * (R0 >> 3) + 512 * dt>(((R0 >> 3) & 1) ? kb1 : kb0);
          t[2 * dt + 1] = lds_tr_read_off<RB * ((R0 + 8) >> 3) + 512 * dt>((((R0 + 8) >> 3) & 1) ? kb1 : kb0);
        });
        wait_tr<NR, 0>(t);
        bf16x8 fb = f[ks4];
        if (diag) {  // keys past the query: zero (the dK/dV kernel never wrote fully masked 32x32 blocks)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int key = kv0 + R0 + 4 * hh + (e & 3) + 8 * (e >> 2);
            if (key > qi) fb[e] = 0;
          }
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) acc[dt] = mfma32(cat44(t[2 * dt], t[2 * dt + 1]), fb, acc[dt]);
      });
    }
    asm volatile("" ::: "memory");
  }
  bf16_t* dp = dq + (int64_t)(b * S + qi) * dqs + hq * D;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u32x2 w;
      w[0] = pack2(acc[dt][4 * g4] * scale, acc[dt][4 * g4 + 1] * scale);
      w[1] = pack2(acc[dt][4 * g4 + 2] * scale, acc[dt][4 * g4 + 3] * scale);
      *reinterpret_cast<u32x2*>(dp + dt * 32 + 8 * g4 + 4 * hh) = w;
    }
  }
}

// dS is read exactly once, by one CU: load it non-temporally (default; KOP_DQ_NT=0 for the cached policy). The
// K tiles every query block of the GQA group re-reads then keep their L2 lines: causal backward 1.813 / 1.826 ms vs
// 1.886 / 1.874 ms cached, same box alternating (profiles/r4_dq_nt_ab.jsonl)
static bool dq_nt() {
  static const bool on = [] {
    const char* e = getenv("KOP_DQ_NT");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

template <int D, int HP, bool BLK, bool NTL, bool KMAJ = false, int NW = 8>
static void launch_dq_ds_nt(const bf16_t* ds, const bf16_t* k, bf16_t* dq, int B, int S, int Hq, int Hkv, int64_t ks,
                            int64_t dqs, float scale, bool causal, hipStream_t stream) {
  const size_t lds = 3 * (64 * (D * 2) + 32 * NW * 64 * 2);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_bwd_dq_ds_kernel<D, HP, BLK, NTL, KMAJ, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  fa_bwd_dq_ds_kernel<D, HP, BLK, NTL, KMAJ, NW><<<B * (Hq / HP) * (S / (32 * NW / HP)), NW * 64, lds, stream>>>(
      ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal);
}

// waves per dQ workgroup: KOP_DQ_NW (4 / 8; 0 = automatic: 4 for a causal D = 64 backward with at most 4 heads per
// workgroup, else 8). GPT-2 shape causal backward 0.338 / 0.339 ms with 4 vs 0.342 / 0.342 with 8, non-causal 2-3 %
// slower with 4; at D = 128 a 4-wave workgroup's ring leaves no room for a second one per CU: the Llama-3-8B shape
// runs 1.80 vs 1.65 ms (profiles/r6_dq_nw_bchunk_gpt2_ab.jsonl, profiles/r6_dq_nw_llama_ab.jsonl)
static int g_dq_nw = -1;
int flash_attn_set_dq_nw(int v) {
  if (g_dq_nw < 0) {
    const char* e = getenv("KOP_DQ_NW");
    g_dq_nw = e ? atoi(e) : 0;
  }
  const int old = g_dq_nw;
  if (v >= 0) g_dq_nw = v;
  return old;
}

template <int D, int HP, bool BLK = false, bool KMAJ = false>
static void launch_dq_ds(const bf16_t* ds, const bf16_t* k, bf16_t* dq, int B, int S, int Hq, int Hkv, int64_t ks,
                         int64_t dqs, float scale, bool causal, hipStream_t stream) {
  const int req = flash_attn_set_dq_nw(-1);
  const bool nw4 = HP <= 4 && S % 128 == 0 && (req == 4 || (req == 0 && D == 64 && causal));
  if constexpr (HP <= 4) {
    if (nw4) {
      if (dq_nt()) launch_dq_ds_nt<D, HP, BLK, true, KMAJ, 4>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
      else launch_dq_ds_nt<D, HP, BLK, false, KMAJ, 4>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
      return;
    }
  }
  (void)nw4;
  if (dq_nt()) launch_dq_ds_nt<D, HP, BLK, true, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
  else launch_dq_ds_nt<D, HP, BLK, false, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
}

// dk/dv = bf16(sum of the NP per-group partials): partial p of KV head h at slot h * grp + p of [T, Hq, D]
// (NP = grp when every q-head wrote its own; fewer when the dK/dV kernel swept several heads per workgroup)
template <int D>
__global__ void __launch_bounds__(256) fa_bwd_finalize_kernel(const float* __restrict__ dk_part,
                                                              const float* __restrict__ dv_part, bf16_t* __restrict__ dk,
                                                              bf16_t* __restrict__ dv, int64_t T, int Hq, int Hkv,
                                                              int64_t dks, int64_t dvs, int np) {
  const int grp = Hq / Hkv;
  const int64_t nk = T * Hkv * (D / 8);
  for (int64_t it = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; it < nk; it += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = it / (Hkv * (D / 8));
    const int rem = (int)(it % (Hkv * (D / 8)));
    const int h = rem / (D / 8), c8 = rem % (D / 8);
    float fk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < np; ++g) {
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

// ---------------------------------------------------------------------------------------------
constexpr int kBwdWaves = 4;

static int g_dq_variant = -1;  // -1: read KOP_DQ_VARIANT on first use
static int dq_variant() {
  if (g_dq_variant < 0) {
    const char* e = getenv("KOP_DQ_VARIANT");
    g_dq_variant = e ? atoi(e) : 10;
  }
  return g_dq_variant;
}
int flash_attn_set_dq_variant(int v) {
  const int old = dq_variant();
  if (v >= 0) g_dq_variant = v;
  return old;
}
constexpr size_t kMaxDsBytes = (size_t)16 << 30;  // dS buffer cap; above it dQ recomputes (variant 9)
static size_t ds_bytes(int B, int S, int Hq) { return (size_t)B * Hq * S * S * 2; }
static bool use_ds(int B, int S, int Hq) {
  return dq_variant() == 10 && S % 256 == 0 && ds_bytes(B, S, Hq) <= kMaxDsBytes;
}

size_t flash_attn_bwd_workspace(int B, int S, int Hq, int D) {
  // dk_part + dv_part (fp32, [B*S, Hq, D] each) + delta, nlse, ndelta ([B, Hq, S] each)
  // (+ dS [B, Hq, S, S] bf16 for variant 10)
  return (size_t)B * S * Hq * D * 4 * 2 + (size_t)B * Hq * S * 4 * 3 + (use_ds(B, S, Hq) ? ds_bytes(B, S, Hq) : 0);
}

// dK/dV kernel with the dS stores (variant 10): workgroup shape W waves x 32 keys, NS-deep stage ring
template <int D, int W, int NS>
static void launch_dkdv_ds(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                           const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds,
                           int B, int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                           int64_t dvs, float scale, int causal, hipStream_t stream) {
  const size_t lds = 32 * W * (D * 2) + NS * (2 * 32 * (D * 2) + 1024);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<D, W, true, false, NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<D, W, true, true, NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const dim3 grid(B * Hq * (S / (32 * W)));
  if (Hq == Hkv)  // no GQA: bf16 dK / dV straight from the kernel
    fa_bwd_dkdv_kernel<D, W, true, true, NS><<<grid, W * 64, lds, stream>>>(
        q, k, v, dout, nlse, ndelta, reinterpret_cast<float*>(dk), reinterpret_cast<float*>(dv), ds, B, S, Hq, Hkv,
        qs, ks, vs, dos, scale, causal, dks, dvs);
  else
    fa_bwd_dkdv_kernel<D, W, true, false, NS><<<grid, W * 64, lds, stream>>>(
        q, k, v, dout, nlse, ndelta, dk_part, dv_part, ds, B, S, Hq, Hkv, qs, ks, vs, dos, scale, causal);
}

// dQ from the materialised dS with HP q-heads of a GQA group per workgroup (HP the largest power of two <= 8
// dividing the group)
template <int D, bool BLK, bool KMAJ = false>
static void launch_dq_ds_hp(int hp, const bf16_t* ds, const bf16_t* k, bf16_t* dq, int B, int S, int Hq, int Hkv,
                            int64_t ks, int64_t dqs, float scale, bool causal, hipStream_t stream) {
  if (hp == 8) launch_dq_ds<D, 8, BLK, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
  else if (hp == 4) launch_dq_ds<D, 4, BLK, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
  else if (hp == 2) launch_dq_ds<D, 2, BLK, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
  else launch_dq_ds<D, 1, BLK, KMAJ>(ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
}

static int g_dkdv_cfg = -1;  // -1: read KOP_DKDV_CFG on first use
static int dkdv_cfg() {
  if (g_dkdv_cfg < 0) {
    // 67 (default): one wave per SIMD, 64 keys per wave, key-major dS tiles stored from registers (D = 128); 64: the
    // same with the LDS-staged wave-block dS; 66: LDS-staged row-major dS; 42: two waves per SIMD, 32 keys per wave, 4-wave
    // workgroups (every D); 68: the D = 64 two-waves-per-SIMD kernel of flash_bwd_d64.hip. 67 vs 64: causal backward 1.731 / 1.721 ms vs
    // 1.778 / 1.790 ms at the Llama-3-8B shape, same box (profiles/r4_dkdv_kmaj_ab.jsonl)
    const char* e = getenv("KOP_DKDV_CFG");
    g_dkdv_cfg = e ? atoi(e) : 67;
  }
  return g_dkdv_cfg;
}
int flash_attn_set_dkdv_cfg(int c) {
  const int old = dkdv_cfg();
  if (c >= 0) g_dkdv_cfg = c;
  return old;
}

template <int D>
static void launch_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                       const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv, void* workspace, int B, int S, int Hq,
                       int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dos, int64_t dqs, int64_t dks,
                       int64_t dvs, float scale, bool causal, hipStream_t stream) {
  constexpr int NW = kBwdWaves;
  const int64_t T = (int64_t)B * S;
  float* dk_part = reinterpret_cast<float*>(workspace);
  float* dv_part = dk_part + T * Hq * D;
  float* delta = dv_part + T * Hq * D;
  float* nlse = delta + T * Hq;
  float* ndelta = nlse + T * Hq;
  launch_delta<D>(o, dout, lse, delta, nlse, ndelta, 1.f / scale, B, S, Hq, os, dos, stream);
  const size_t lds_kv = 32 * NW * (D * 2) + 2 * (2 * 32 * (D * 2) + 1024);
  const size_t lds_q = 4 * 64 * (D * 2);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<D, NW, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_kv);
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<D, NW, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_kv);
    (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv_kernel<D, NW, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_kv);
    (void)hipFuncSetAttribute((const void*)fa_bwd_dq_kernel<D, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_q);
    attr = true;
  }
  const int variant = dq_variant();
  if (use_ds(B, S, Hq)) {
    bf16_t* ds = reinterpret_cast<bf16_t*>(ndelta + T * Hq);
    const bool direct = Hq == Hkv;
    const int cfg = dkdv_cfg();
    const int cflag = causal ? 1 : 0;
    const int grp = Hq / Hkv;  // heads per dQ workgroup: largest power of two dividing the GQA group, <= 8
    static const int hp_env = [] {  // KOP_DQ_HP: force the dQ kernel's heads per workgroup (A/B)
      const char* e = getenv("KOP_DQ_HP");
      return e ? atoi(e) : 0;
    }();
    const int hp = (hp_env > 0 && grp % hp_env == 0 && hp_env <= 8) ? hp_env
                   : (grp % 8 == 0) ? 8 : (grp % 4 == 0) ? 4 : (grp % 2 == 0) ? 2 : 1;
    // one wave per SIMD (flash_bwd_w1.hip): query-major dS staged through LDS into whole-line stores, in the
    // wave-block layout (cfg 64; 640 = the same at D = 64, opt-in) or plain rows (66); cfg 67 / 670: key-major tiles
    // stored straight from the accumulators (no LDS staging), read back transposed by the dQ kernel
    // (at D = 64 the one-wave kernel is opt-in as 670 since round 6: the default 67 runs flash_bwd_d64.hip there;
    // the one-wave kernel had beaten the older 4-wave cfg 42 kernel 0.372 vs 0.402 ms: profiles/r4_gpt2_kmaj_d64_ab.jsonl)
    const bool kmaj = (D == 128 && cfg == 67) || (D == 64 && cfg == 670);
    const bool one_wave = S % 256 == 0 && ((D == 128 && (cfg == 64 || cfg == 66 || cfg == 67)) ||
                                           (D == 64 && (cfg == 640 || cfg == 670)));
    const bool blk = one_wave && cfg != 66;
    bool done = false;
    int np = direct ? 0 : Hq / Hkv;  // fp32 partials per GQA group left for the finalize pass
    // cfg 68 (and the default 67 at D = 64): the D = 64 dK/dV kernel with two waves per SIMD (flash_bwd_d64.hip),
    // key-major dS tiles. GPT-2-small shape causal backward 0.335-0.345 ms vs 0.373-0.387 with the one-wave kernel
    // (cfg 670), step +0.5-0.9 % (profiles/r6_gpt2_dkdv68_step_ab.jsonl)
    const bool w2 = D == 64 && (cfg == 68 || cfg == 67) && S % 256 == 0;
    if (w2) {
      np = flash_attn_bwd_dkdv_d64(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs,
                                   dos, dks, dvs, scale, cflag, stream);
      done = true;
    } else if (one_wave) {
      np = flash_attn_bwd_dkdv64(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, D, qs, ks, vs,
                                 dos, dks, dvs, scale, cflag, !kmaj, blk, stream);
      done = true;
    }
    if (!done)
      launch_dkdv_ds<D, NW, 2>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs,
                               dos, dks, dvs, scale, cflag, stream);
    if ((one_wave && kmaj) || w2) launch_dq_ds_hp<D, false, true>(hp, ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
    else if (blk) launch_dq_ds_hp<D, true>(hp, ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
    else launch_dq_ds_hp<D, false>(hp, ds, k, dq, B, S, Hq, Hkv, ks, dqs, scale, causal, stream);
    if (np > 0) fa_bwd_finalize_kernel<D><<<2048, 256, 0, stream>>>(dk_part, dv_part, dk, dv, T, Hq, Hkv, dks, dvs, np);
    return;
  }
  int np = Hq / Hkv;
  if (D == 128 && (dkdv_cfg() == 64 || dkdv_cfg() == 67) && S % 256 == 0) {
    // the one-wave dK/dV kernel without dS stores; dQ recomputes S and dP below. It writes bf16 dK / dV itself
    // when Hq == Hkv, so the finalize pass is then skipped.
    np = flash_attn_bwd_dkdv64(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, nullptr, B, S, Hq, Hkv, D, qs, ks,
                               vs, dos, dks, dvs, scale, causal ? 1 : 0, false, false, stream);
  } else {
    fa_bwd_dkdv_kernel<D, NW, false><<<B * Hq * (S / (32 * NW)), NW * 64, lds_kv, stream>>>(
        q, k, v, dout, nlse, ndelta, dk_part, dv_part, nullptr, B, S, Hq, Hkv, qs, ks, vs, dos, scale, causal);
  }
  if (S % 256 == 0 && variant >= 8) {
    const bool stg = variant != 8;
    const size_t lds8 = (stg ? 4 : 3) * 2 * 64 * (D * 2);
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)fa_bwd_dq8_kernel<D, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(4 * 2 * 64 * (D * 2)));
      (void)hipFuncSetAttribute((const void*)fa_bwd_dq8_kernel<D, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(3 * 2 * 64 * (D * 2)));
      attr8 = true;
    }
    if (stg)
      fa_bwd_dq8_kernel<D, true><<<B * Hq * (S / 256), 512, lds8, stream>>>(q, k, v, dout, lse, delta, dq, B, S, Hq,
                                                                            Hkv, qs, ks, vs, dos, dqs, scale, causal);
    else
      fa_bwd_dq8_kernel<D, false><<<B * Hq * (S / 256), 512, lds8, stream>>>(q, k, v, dout, lse, delta, dq, B, S, Hq,
                                                                             Hkv, qs, ks, vs, dos, dqs, scale, causal);
  } else {
    fa_bwd_dq_kernel<D, NW><<<B * Hq * (S / (32 * NW)), NW * 64, lds_q, stream>>>(
        q, k, v, dout, lse, delta, dq, B, S, Hq, Hkv, qs, ks, vs, dos, dqs, scale, causal);
  }
  if (np > 0) fa_bwd_finalize_kernel<D><<<2048, 256, 0, stream>>>(dk_part, dv_part, dk, dv, T, Hq, Hkv, dks, dvs, np);
}

int flash_attn_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                   const float* lse, bf16_t* dq, bf16_t* dk, bf16_t* dv, void* workspace, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, int64_t dos, int64_t dqs,
                   int64_t dks, int64_t dvs, float scale, bool causal, hipStream_t stream) {
  if (S % (32 * kBwdWaves) != 0 || S % 64 != 0 || Hq % Hkv != 0) return -1;
  if (D == 128)
    launch_bwd<128>(q, k, v, o, dout, lse, dq, dk, dv, workspace, B, S, Hq, Hkv, qs, ks, vs, os, dos, dqs, dks, dvs,
                    scale, causal, stream);
  else if (D == 64)
    launch_bwd<64>(q, k, v, o, dout, lse, dq, dk, dv, workspace, B, S, Hq, Hkv, qs, ks, vs, os, dos, dqs, dks, dvs,
                   scale, causal, stream);
  else
    return -3;
  return 0;
}

}  // namespace kop
