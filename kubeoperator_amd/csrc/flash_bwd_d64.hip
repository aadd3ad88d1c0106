// Flash attention BACKWARD, dK / dV stage at head_dim 64 with TWO waves per SIMD (gfx950 / MI355X).
//
// Why a D = 64 kernel of its own: the one-wave-per-SIMD kernel (flash_bwd_w1.hip, the D = 128 default) pays
// about the same cycles per 32-query stage at D = 64 as at D = 128 -- half the MFMAs, but the same exponentials,
// dS stores, LDS latencies and stage barrier, none of which a single wave per SIMD can hide behind another wave's
// matrix work (profiles/r5_experiments.md "GPT-2 shape (D = 64) backward"). At D = 64 the register budget
// allows more: a wave of 32 keys needs 64 accumulators (dK^T, dV^T: 32 keys x 64 columns each) plus 32 registers
// of resident K / V fragments, so two waves fit on every SIMD (256 registers each) and the softmax VALU of one
// wave issues beside the other wave's MFMAs.
//
// A workgroup of NW waves owns 32 NW keys of one (batch, q-head); wave w owns keys k0 + 32w .. +31. The default
// shape is 4 waves (two workgroups per CU, each with its own barriers); 8 waves (one per CU) measured 2 % slower.
// Per 32-query stage and wave (all products on v_mfma_f32_32x32x16_bf16, key on the lane):
//   S  = Q.K^T  - lse/scale   (4 MFMAs; A = Q rows from LDS, B = K^T fragments resident in VGPRs)
//   dP = dO.V^T - delta       (4 MFMAs; A = dO rows from LDS, B = V^T fragments resident)
//   P = exp2(c * S), dS = P * dP, both packed to bf16 straight from the accumulators
//   dV^T += dO^T.P, dK^T += Q^T.dS  (4 + 4 MFMAs; A = transposed reads of the staged dO / Q tiles)
//   dS -> the key-major tiles fa_bwd_dq_ds_kernel<KMAJ> reads (two 16-B non-temporal stores per lane)
// The stage ring (Q, dO, -lse/scale, -delta of 32 queries; 3 slots, LDS-DMA, one barrier per stage) is swept
// from the last query stage down, so every workgroup of a head reads the same stage at about the same time
// (its lines are then still in the XCD's L2). Under a causal mask a wave computes the stages above its diagonal
// unmasked, its one diagonal stage masked, and only joins the barriers / DMA of the stages below.
// What bounds it (timing ablations, profiles/r6_experiments.md): the dS write stream and the stage ring -- removing
// every MFMA saves 24 us of ~190 at the GPT-2 bench shape, removing the dS stores 50 us.
#include <cstdlib>

#include "attn_common.h"
#include "kernels.h"

namespace kop {

// NW waves per workgroup (BN = 32 NW keys), NS-slot stage ring (prefetch distance NS - 1).
// DIAG (timing ablations, WRONG results; instantiated only in the -DKOP_ABLATIONS probe build): 1 no dS stores,
// 2 no exponentials, 4 no stage barrier, 16 no dV / dK products, 32 no S / dP products.
template <bool DIRECT, int NW, int NS, int DIAG = 0>
__global__ void __launch_bounds__(NW * 64, 2) fa_bwd_dkdv_d64_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ nlse, const float* __restrict__ ndelta,
    float* __restrict__ dk_part, float* __restrict__ dv_part, bf16_t* __restrict__ dst, int B, int S, int Hq, int Hkv,
    int64_t qs, int64_t ks, int64_t vs, int64_t dos, float scale, int causal, int64_t dks, int64_t dvs) {
  constexpr int D = 64, BN = 32 * NW, BQ = 32, ROWB = 2 * D;
  constexpr int QT = BQ * ROWB, STAGE = 2 * QT + 1024, RB = ROWB * 8, NK = D / 16, DT = D / 32;
  constexpr int PPW = (2 * QT / 1024) / NW;  // 1-KB DMA pieces of the Q / dO tiles per wave per stage
  static_assert(PPW * NW * 1024 == 2 * QT && NS >= 3 && NS <= 4, "stage pieces split evenly; 3- or 4-slot ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int grp = Hq / Hkv, nkb = S / BN;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, grp, nkb);
  const int kb = aw.rank;  // heaviest key blocks (earliest keys under a causal mask) first
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / grp;
  const float c2 = scale * 1.4426950408889634f;
  {
    const int k0 = kb * BN, k0w = k0 + 32 * wid;
    const int nqt = S / BQ;
    const int qt0 = causal ? k0 / BQ : 0;        // the workgroup's lowest stage
    const int qdiag = causal ? k0w / BQ : -1;    // this wave's diagonal stage (keys == queries of the stage)
    const int tot = nqt - qt0;                   // stages swept by every wave (barriers / DMA)

    // resident K^T / V^T fragments of the wave's 32 keys (B operands of S and dP): key k0w + r, columns 16kk + 8hh ..
    bf16x8 kf[NK], vf[NK];
    {
      const bf16_t* kp = k + (int64_t)(b * S + k0w + r) * ks + kvh * D + 8 * hh;
      const bf16_t* vp = v + (int64_t)(b * S + k0w + r) * vs + kvh * D + 8 * hh;
  #pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        kf[kk] = *reinterpret_cast<const bf16x8*>(kp + 16 * kk);
        vf[kk] = *reinterpret_cast<const bf16x8*>(vp + 16 * kk);
      }
  #pragma unroll
      for (int kk = 0; kk < NK; ++kk) asm volatile("" : "+v"(kf[kk]), "+v"(vf[kk]));
    }

    // DMA cursor: stage i of the sweep is query stage nqt - 1 - i. The 8 1-KB pieces of a stage's Q and dO tiles go
    // round the waves (piece p = wid + NW j: Q rows 8p.. for p < 4, dO rows 8(p - 4).. after), wave 0 also brings the
    // 256 B of -lse/scale and -delta.
    const int lrow = (lane & 31) >> 2, lhi = lane >> 5, lslot = lane & 3;
    const bf16_t* isrc[PPW];
    int64_t ioff[PPW], istep[PPW];
  #pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = wid + NW * j, pw = pc & 3;
      const bool qpiece = pc < 4;
      isrc[j] = qpiece ? q + (int64_t)(b * S + (nqt - 1) * BQ) * qs + hq * D
                    : dout + (int64_t)(b * S + (nqt - 1) * BQ) * dos + hq * D;
      const int64_t stride = qpiece ? qs : dos;
      const int prow = 8 * pw + lrow;  // the row of the stage tile this lane's 16 B come from
      ioff[j] = (int64_t)prow * stride + 8 * (4 * lhi + (lslot ^ ((prow >> 2) & 3)));
      istep[j] = (int64_t)BQ * stride;
    }
    const float* il = (((lane & 15) < 8) ? nlse + 4 * (lane & 15) : ndelta + 4 * ((lane & 15) - 8)) +
                      (int64_t)(b * Hq + hq) * S + (nqt - 1) * BQ;
    const int pcount = PPW + (wid == 0 ? 1 : 0);  // DMA instructions this wave issues per stage
    int isq = 0, islot = 0;
    auto issue_next = [&]() {
      char* base = smem + islot * STAGE;
  #pragma unroll
      for (int j = 0; j < PPW; ++j) {
        glds16(isrc[j] + ioff[j], base + 1024 * (wid + NW * j));
        isrc[j] -= istep[j];
      }
      if (wid == 0) glds16(il, base + 2 * QT);
      il -= BQ;
      ++isq;
      islot = islot == NS - 1 ? 0 : islot + 1;
    };
    asm volatile("" ::: "memory");
  #pragma unroll
    for (int i = 0; i < NS - 1; ++i)
      if (isq < tot) issue_next();

    // lane bases of the sub-tiled stage images (swza): row reads of row r at chunk 2kk + hh (+512 per 32 columns),
    // transposed reads of rows 4hh + tq (+8, +16, +24) at column block dt (+512 dt)
    const int rb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
    const int rb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
    const int tb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
    const int tb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);

    // dS tiles [B, Hq, S/64, S/32] x 4 KB: the wave is key half c = wid & 1 of its 64-key tile; lane (r, hh) stores
    // its packed quad s at chunk 32hh + (r ^ 4hh ^ 8s) of block s (fa_bwd_dq_ds_kernel<KMAJ> reads them back)
    const uint64_t dsrow = (uint64_t)(uintptr_t)(dst + (((int64_t)(b * Hq + hq) * (S / 64) + k0w / 64) * (S / 32)) * 2048) +
                           2048ull * (uint64_t)(wid & 1);
    const uint32_t kto0 = 16u * (uint32_t)(32 * hh + (r ^ (4 * hh))), kto1 = 1024u + 16u * (uint32_t)(32 * hh + (r ^ (4 * hh) ^ 8));

    f32x16 dk[DT], dv[DT];
  #pragma unroll
    for (int i = 0; i < DT; ++i) dk[i] = dv[i] = f32x16{0};

    // dS stores issued in the previous NS - 1 stages (st[0] the latest) and the ring cursor of the computed stage
    int st[3] = {0, 0, 0};
    int cslot = 0, cur = 0;
    // top of stage i: its DMA has landed (younger: the stores of stages i-NS+1 .. i-1 and the DMAs of stages
    // i+1 .. i+NS-2, interleaved), every wave is past stage i-1 (whose slot the DMA of stage i+NS-1 then refills).
    // The steady state (every younger stage stored, every younger DMA issued) takes a constant count; the sweep's
    // head, tail and the waves below their diagonal go through vm_wait_le's compare tree
    auto top = [&]() -> int {
      int younger = 0;
  #pragma unroll
      for (int i = 0; i < NS - 1; ++i) younger += st[i];
      const int ahead = tot - 1 - cur < NS - 2 ? tot - 1 - cur : NS - 2;
      younger += ahead * pcount;
      constexpr int FULL = 2 * (NS - 1) + (NS - 2) * PPW;
      if (younger == FULL + (NS - 2) * (wid == 0 ? 1 : 0)) {
        if (wid == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FULL + NS - 2) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FULL) : "memory");
      } else {
        vm_wait_le(younger);
      }
      ++cur;
  #pragma unroll
      for (int i = NS - 2; i > 0; --i) st[i] = st[i - 1];
      st[0] = 0;
      const int slot = cslot;
      cslot = cslot == NS - 1 ? 0 : cslot + 1;
      if constexpr (!(DIAG & 4)) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (isq < tot) issue_next();
      return slot;
    };

    auto stage = [&](int qt, int slot, auto mask_c) {
      constexpr bool MASK = decltype(mask_c)::value;
      const char* Ql = smem + slot * STAGE;
      const char* Ol = Ql + QT;
      const uint32_t qb0 = lds_addr(Ql) + rb_lane0, qb1 = lds_addr(Ql) + rb_lane1;
      const uint32_t ob0 = lds_addr(Ol) + rb_lane0, ob1 = lds_addr(Ol) + rb_lane1;
      // -lse/scale (bytes 0..127) and -delta (128..255): accumulator row j is query (j&3) + 8(j>>2) + 4hh
      const uint32_t ldb = lds_addr(Ql + 2 * QT) + 16 * hh;
      f32x4 lq[4], ld[4];
      bf16x8 qf[NK], of[NK];
      static_for<4>([&](auto g) { lq[decltype(g)::value] = lds_read16f_off<32 * decltype(g)::value>(ldb); });
      static_for<NK>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        qf[kk] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? qb1 : qb0);
      });
      static_for<4>([&](auto g) { ld[decltype(g)::value] = lds_read16f_off<128 + 32 * decltype(g)::value>(ldb); });
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(lq[0]), "+v"(lq[1]), "+v"(lq[2]), "+v"(lq[3]));
      f32x16 s = cat4f(lq);
      // S chain; the dO row reads go out as the Q rows retire
      static_for<NK>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(qf[kk]) : "n"(NK - 1 - kk + 4 + kk));
        f32x16& acc = s;
        const bf16x8 a = qf[kk], b = kf[kk];
        if constexpr (!(DIAG & 32)) acc = mfma32(a, b, acc);
        else asm volatile("" : "+v"(acc) : "v"(a), "v"(b));
        of[kk] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? ob1 : ob0);
      });
      asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(ld[0]), "+v"(ld[1]), "+v"(ld[2]), "+v"(ld[3]) : "n"(NK));
      f32x16 dp = cat4f(ld);
      static_for<NK>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(of[kk]) : "n"(NK - 1 - kk));
        f32x16& acc = dp;
        const bf16x8 a = of[kk], b = vf[kk];
        if constexpr (!(DIAG & 32)) acc = mfma32(a, b, acc);
        else asm volatile("" : "+v"(acc) : "v"(a), "v"(b));
      });
      // the transposed reads of the dV product (dO^T) and of the first dK column block (Q^T) fly under the
      // exponentials (at most 12 LDS reads in flight)
      const uint32_t o0 = lds_addr(Ol) + tb_lane0, o1 = lds_addr(Ol) + tb_lane1;
      const uint32_t qa0 = lds_addr(Ql) + tb_lane0, qa1 = lds_addr(Ql) + tb_lane1;
      bf16x4 to[DT][4], tqv[DT][4];
      auto trr = [&](uint32_t b0, uint32_t b1, auto dtc, bf16x4* t) {
        constexpr int dt = decltype(dtc)::value;
        t[0] = lds_tr_read_off<512 * dt>(b0);
        t[1] = lds_tr_read_off<RB + 512 * dt>(b1);
        t[2] = lds_tr_read_off<RB * 2 + 512 * dt>(b0);
        t[3] = lds_tr_read_off<RB * 3 + 512 * dt>(b1);
      };
      static_for<DT>([&](auto dtc) { trr(o0, o1, dtc, to[decltype(dtc)::value]); });
      trr(qa0, qa1, std::integral_constant<int, 0>{}, tqv[0]);
      // P = exp2(c * S) (diagonal stage: keys past the query masked), packed as the B operand of dV^T += dO^T.P
      const int kd = r - 4 * hh;  // key - query + ((j&3) + 8(j>>2)) on the diagonal stage (qs0 == k0w)
      (void)kd;
  #pragma unroll
      for (int j = 0; j < 16; ++j) {
        float p = (DIAG & 2) ? s[j] * c2 : __builtin_amdgcn_exp2f(s[j] * c2);
        if constexpr (MASK) {
          if (kd > (j & 3) + 8 * (j >> 2)) p = 0.f;
        }
        s[j] = p;
      }
      const bf16x8 pb[2] = {pack_acc8(s, 0), pack_acc8(s, 1)};
      // dV^T += dO^T . P
      static_for<DT>([&](auto dtc) {
        constexpr int dt = decltype(dtc)::value;
        wait_tr<4, 4 * (DT - 1 - dt) + 4>(to[dt]);  // younger: the later dO^T block, the first Q^T block
        f32x16& acc = dv[dt];
        const bf16x8 a0 = cat44(to[dt][0], to[dt][1]), a1 = cat44(to[dt][2], to[dt][3]), b0 = pb[0], b1 = pb[1];
        if constexpr (!(DIAG & 16)) {
          acc = mfma32(a0, b0, acc);
          acc = mfma32(a1, b1, acc);
        } else {
          asm volatile("" : "+v"(acc) : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
        }
      });
      static_for<DT - 1>([&](auto dtc) {
        trr(qa0, qa1, std::integral_constant<int, decltype(dtc)::value + 1>{}, tqv[decltype(dtc)::value + 1]);
      });
      // dS = P * (dP - delta), bf16, stored key-major and packed as the B operand of dK^T += Q^T . dS
  #pragma unroll
      for (int j = 0; j < 16; ++j) dp[j] *= s[j];
      const bf16x8 sb[2] = {pack_acc8(dp, 0), pack_acc8(dp, 1)};
      {
        const uint64_t row = dsrow + 4096ull * (uint64_t)qt;
        const u32x4 w0 = __builtin_bit_cast(u32x4, sb[0]), w1 = __builtin_bit_cast(u32x4, sb[1]);
        if constexpr (!(DIAG & 1)) {
          asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" ::"v"(kto0), "v"(w0), "s"(row) : "memory");
          asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" ::"v"(kto1), "v"(w1), "s"(row) : "memory");
          st[0] = 2;
        } else {
          asm volatile("" ::"v"(w0), "v"(w1), "s"(row));
        }
      }
      static_for<DT>([&](auto dtc) {
        constexpr int dt = decltype(dtc)::value;
        wait_tr<4, 4 * (DT - 1 - dt)>(tqv[dt]);  // younger: the later Q^T blocks
        f32x16& acc = dk[dt];
        const bf16x8 a0 = cat44(tqv[dt][0], tqv[dt][1]), a1 = cat44(tqv[dt][2], tqv[dt][3]), b0 = sb[0], b1 = sb[1];
        if constexpr (!(DIAG & 16)) {
          acc = mfma32(a0, b0, acc);
          acc = mfma32(a1, b1, acc);
        } else {
          asm volatile("" : "+v"(acc) : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
        }
      });
      asm volatile("" ::: "memory");
    };

    int qt = nqt - 1;
    for (; qt > qdiag && qt >= qt0; --qt) stage(qt, top(), std::false_type{});
    if (causal) {
      stage(qt, top(), std::true_type{});  // qt == qdiag
      for (--qt; qt >= qt0; --qt) (void)top();
    }

    auto out = [&](int key) {
      if constexpr (DIRECT) {
        bf16_t* dkb = reinterpret_cast<bf16_t*>(dk_part) + (int64_t)(b * S + key) * dks + kvh * D;
        bf16_t* dvb = reinterpret_cast<bf16_t*>(dv_part) + (int64_t)(b * S + key) * dvs + kvh * D;
  #pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
  #pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int d = dt * 32 + 8 * g4 + 4 * hh;
            *reinterpret_cast<u32x2*>(dkb + d) =
                u32x2{pack2(dk[dt][4 * g4] * scale, dk[dt][4 * g4 + 1] * scale),
                      pack2(dk[dt][4 * g4 + 2] * scale, dk[dt][4 * g4 + 3] * scale)};
            *reinterpret_cast<u32x2*>(dvb + d) =
                u32x2{pack2(dv[dt][4 * g4], dv[dt][4 * g4 + 1]), pack2(dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3])};
          }
        }
      } else {  // per-q-head fp32 partial, slot hq of [T, Hq, D] (the finalize pass sums the GQA group)
        float* dkp = dk_part + (int64_t)(b * S + key) * Hq * D + hq * D;
        float* dvp = dv_part + (int64_t)(b * S + key) * Hq * D + hq * D;
  #pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
  #pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int d = dt * 32 + 8 * g4 + 4 * hh;
            *reinterpret_cast<f32x4*>(dkp + d) = f32x4{dk[dt][4 * g4] * scale, dk[dt][4 * g4 + 1] * scale,
                                                       dk[dt][4 * g4 + 2] * scale, dk[dt][4 * g4 + 3] * scale};
            *reinterpret_cast<f32x4*>(dvp + d) = f32x4{dv[dt][4 * g4], dv[dt][4 * g4 + 1], dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]};
          }
        }
      }
    };
    out(k0w + r);
  }
}

template <int NW, int NS, int DIAG = 0>
static int launch_d64(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                      const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B, int S,
                      int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks, int64_t dvs,
                      float scale, int causal, hipStream_t stream) {
  constexpr size_t lds = NS * (2 * 32 * 128 + 1024);
  const dim3 grid(B * Hq * (S / (32 * NW)));
  if (Hq == Hkv) {
    fa_bwd_dkdv_d64_kernel<true, NW, NS, DIAG><<<grid, NW * 64, lds, stream>>>(
        q, k, v, dout, nlse, ndelta, reinterpret_cast<float*>(dk), reinterpret_cast<float*>(dv), ds, B, S, Hq, Hkv, qs,
        ks, vs, dos, scale, causal, dks, dvs);
    return 0;
  }
  fa_bwd_dkdv_d64_kernel<false, NW, NS, DIAG><<<grid, NW * 64, lds, stream>>>(
      q, k, v, dout, nlse, ndelta, dk_part, dv_part, ds, B, S, Hq, Hkv, qs, ks, vs, dos, scale, causal, 0, 0);
  return Hq / Hkv;
}

// workgroup shape (KOP_D64_SHAPE, A/B): 43 (default) 4 waves x 32 keys (two workgroups per CU, each with its own
// barriers), 3-slot ring; 44 the same with 4 slots; 83 8 waves (one workgroup per CU), 3 slots. GPT-2 shape causal
// backward 0.335 / 0.338 ms (43) vs 0.343 / 0.345 (44) and 0.343 / 0.347 (83), same box alternating. (Key-block
// pairs per workgroup with a head's workgroups adjacent in one XCD measured 0.347: removed, profiles/r6_experiments.md.)
static int g_d64_shape = -1;  // -1: read KOP_D64_SHAPE on first use
int flash_attn_set_d64_shape(int v) {
  if (g_d64_shape < 0) {
    const char* e = getenv("KOP_D64_SHAPE");
    g_d64_shape = e ? atoi(e) : 43;
  }
  const int old = g_d64_shape;
  if (v >= 0) g_d64_shape = v;
  return old;
}

int flash_attn_bwd_dkdv_d64(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                            const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds,
                            int B, int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                            int64_t dvs, float scale, int causal, hipStream_t stream) {
  if (S % 256 != 0 || Hq % Hkv != 0 || ds == nullptr) return -1;
  const int shape = flash_attn_set_d64_shape(-1);
#ifdef KOP_ABLATIONS
  static const int diag = [] {
    const char* e = getenv("KOP_D64_DIAG");
    return e ? atoi(e) : 0;
  }();
#define KOP_D64_DIAG_CASE(DG)                                                                                        \
  case DG:                                                                                                         \
    return launch_d64<4, 3, DG>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, \
                                dos, dks, dvs, scale, causal, stream);
  switch (diag) {
    KOP_D64_DIAG_CASE(1) KOP_D64_DIAG_CASE(2) KOP_D64_DIAG_CASE(3) KOP_D64_DIAG_CASE(4) KOP_D64_DIAG_CASE(16)
    KOP_D64_DIAG_CASE(32) KOP_D64_DIAG_CASE(48) KOP_D64_DIAG_CASE(7) KOP_D64_DIAG_CASE(55)
    default: break;
  }
#undef KOP_D64_DIAG_CASE
#endif
  if (shape == 83)
    return launch_d64<8, 3>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, dos,
                            dks, dvs, scale, causal, stream);
  if (shape == 44)
    return launch_d64<4, 4>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, dos,
                            dks, dvs, scale, causal, stream);
  return launch_d64<4, 3>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, dos,
                          dks, dvs, scale, causal, stream);
}

}  // namespace kop
