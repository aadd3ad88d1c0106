// Flash attention FORWARD for gfx950 (CDNA4 / MI355X): bf16 in, fp32 accumulate, causal or full, GQA,
// head_dim 64 or 128, on the 32x32x16 bf16 MFMA.
//
// q/k/v/o element (b, s, h, d) at ptr + (b*S + s) * stride + h*D + d (the fused-QKV activation's column
// views, no transposes); lse [B, Hq, S] fp32 = natural-log sum of exp(scale * q.k).
//
// Structure (one workgroup = NW waves = 32*NW query rows of one (b, q-head); 64-key K/V tiles):
//   * K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction) into a 2-deep
//     ring: no staging registers, the DMA of tile i+1 flies during tile i's MFMAs behind a COUNTED
//     vmcnt and raw s_barrier (a __syncthreads would drain it). The XOR-swizzled LDS image is produced
//     by permuting each lane's SOURCE address (the DMA destination is lane-linear), so row reads
//     (ds_read_b128) and transposed reads (ds_read_b64_tr_b16) of the image are conflict-free.
//   * swapped scores S^T = K . Q^T: K is the MFMA A operand (LDS row reads, prefetched one k-step
//     ahead), Q^T the B operand held in VGPRs for the whole sweep; each lane owns one query row, its 32
//     keys are in accumulator registers -> row max = in-register max + one half-wave exchange.
//   * P never leaves registers: the S^T accumulator packed to bf16 is directly the B operand of
//     O^T = V^T . P^T (accumulator-as-operand identity); V^T fragments come from tr_b16 reads of the
//     row-major V image. O^T has the query on the lane, so softmax rescales are per-lane scalars.
//   * lazy rescale: O and l are rescaled only when a tile raises some row's max by more than 2^8
//     (wave-uniform branch); otherwise p = exp2(s - m_ref) <= 256, exact in fp32 and fine in bf16.
//   * causal: waves skip tiles above their diagonal; blocks are issued heaviest-first and remapped so
//     the query heads sharing one K/V head run on one XCD (shared L2).
//   * __launch_bounds__(256, 2): <= 256 VGPRs so two workgroups (8 waves) share a CU and one wave's
//     softmax VALU work overlaps the other's MFMAs.
#include "attn_common.h"
#include "kernels.h"

#ifndef KOP_FWD8_KDEPTH
#define KOP_FWD8_KDEPTH 2
#endif

namespace kop {

template <int D, int NW>
__global__ void __launch_bounds__(NW * 64, 2) fa_fwd_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                            const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                            float* __restrict__ lse, int B, int S, int Hq, int Hkv,
                                                            int64_t qs, int64_t ks, int64_t vs, int64_t os,
                                                            float scale_log2, int causal) {
  constexpr int BM = 32 * NW, BN = 64, ROWB = D * 2;
  constexpr int TILE = BN * ROWB;          // bytes of one K or V tile
  constexpr int SLOTS = ROWB / 16;         // 16-B slots per row
  constexpr int RPP = 1024 / ROWB;         // rows per 1-KiB DMA piece
  constexpr int PPW = (TILE / 1024) / NW;  // DMA pieces per wave per tile (each of K and V)
  static_assert(PPW * NW * 1024 == TILE, "tile must split evenly over the waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(buf) (smem + (buf) * 2 * TILE)
#define VBUF(buf) (smem + (buf) * 2 * TILE + TILE)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;

  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  // DMA lane geometry: lane -> (row within piece, slot); the slot's chunk is pre-swizzled in the source
  const int prow = lane / SLOTS, pslot = lane % SLOTS;
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = wid * PPW + i;
      const int row = piece * RPP + prow;
      const int ch = pslot ^ swz_xor<ROWB>(row);
      glds16(kbase + (int64_t)(t * BN + row) * ks + ch * 8, KBUF(buf) + piece * 1024);
      glds16(vbase + (int64_t)(t * BN + row) * vs + ch * 8, VBUF(buf) + piece * 1024);
    }
  };

  issue(0, 0);

  // Q^T operand fragments, resident for the whole sweep
  bf16x8 qf[D / 16];
  {
    const bf16_t* qp = q + (int64_t)(b * S + q0w + r) * qs + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
    // retire the Q loads HERE: a register still pending inside the loop would make hipcc emit
    // vmcnt(0) at its first use every iteration, draining the in-flight K/V DMA
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(qf[kk]));
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) oacc[i] = f32x16{0};
  float m = -INFINITY, l = 0.f;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;

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
      f32x16 s0 = f32x16{0}, s1 = f32x16{0};
      bf16x8 ka = lds_read8(Kb + swz<ROWB>(r, hh));
      bf16x8 kb = lds_read8(Kb + swz<ROWB>(32 + r, hh));
#pragma unroll
      for (int kk = 0; kk < D / 16; ++kk) {
        bf16x8 na, nb;
        if (kk + 1 < D / 16) {
          na = lds_read8(Kb + swz<ROWB>(r, 2 * (kk + 1) + hh));
          nb = lds_read8(Kb + swz<ROWB>(32 + r, 2 * (kk + 1) + hh));
        }
        s0 = mfma32(ka, qf[kk], s0);
        s1 = mfma32(kb, qf[kk], s1);
        if (kk + 1 < D / 16) {
          ka = na;
          kb = nb;
        }
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
      float mx = fmaxf(s0[0], s1[0]);
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, fmaxf(s0[j], s1[j]));
      mx = xor32_max(mx);
      const float mt = mx * scale_log2;
      if (__any(mt > m + 8.f)) {
        const float mnew = fmaxf(m, mt);
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        m = mnew;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < D / 32; ++i) oacc[i] *= alpha;
      }
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s0[j] = __builtin_amdgcn_exp2f(fmaf(s0[j], scale_log2, -m));
        s1[j] = __builtin_amdgcn_exp2f(fmaf(s1[j], scale_log2, -m));
        ls += s0[j] + s1[j];
      }
      l += ls;
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
        bf16x4 t[8];
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int rowA = (ks4 >> 1) * 32 + 16 * (ks4 & 1) + 4 * hh + tq;
          t[2 * ks4] = lds_tr_read_asm(Vb + swz<ROWB>(rowA, ch) + bo);
          t[2 * ks4 + 1] = lds_tr_read_asm(Vb + swz<ROWB>(rowA + 8, ch) + bo);
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),
                       "+v"(t[7]));
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) oacc[dt] = mfma32(cat44(t[2 * ks4], t[2 * ks4 + 1]), pf[ks4], oacc[dt]);
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with buf before iteration it+1 refills it
  }
#undef KBUF
#undef VBUF

  const float lt = xor32_sum(l);
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

// ------------------------------------------------------------------------------------------------------
// 8-wave forward: one 512-thread workgroup = 256 query rows (8 waves x 32) of one (b, q-head), so every
// K/V tile fetched into LDS serves twice the query rows of the 4-wave kernel, and the two waves sharing a
// SIMD (w and w+4) belong to ONE workgroup, where their phases can be arranged:
//   * STAGGER: waves 4-7 run half a tile behind -- in the interval of tile t they do softmax + P.V of tile
//     t-1 and then Q.K^T of tile t (keeping S^T in registers across the barrier), while waves 0-3 do
//     Q.K^T, softmax and P.V of tile t. Each SIMD then pairs one wave's MFMA phase with the other's VALU
//     (softmax) phase instead of running both in lockstep (guide: MI355X_MICROARCH "Two waves per SIMD",
//     item 9). The ring has 4 slots so the late half can still read V(t-1) while t+2 is being fetched.
//   * one barrier per tile (the ring is deep enough that a slot is refilled only after every wave has
//     passed the barrier that follows its last read);
//   * V^T fragments for the next 32-column block are read (ds_read_b64_tr_b16) while the current block's
//     MFMAs run, retired by counted lgkmcnt waits; the first block's reads fly under the softmax.
template <int D, bool STAGGER, bool PK>
__global__ void __launch_bounds__(512, 1) fa_fwd8_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                         const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                         float* __restrict__ lse, int B, int S, int Hq, int Hkv,
                                                         int64_t qs, int64_t ks, int64_t vs, int64_t os,
                                                         float scale_log2, int causal, bf16_t* __restrict__ ot) {
  constexpr int NW = 8, BM = 256, BN = 64, ROWB = D * 2;
  constexpr int TILE = BN * ROWB;
  constexpr int NSLOT = STAGGER ? 4 : 3;
  constexpr int SLOTS = ROWB / 16, RPP = 1024 / ROWB;
  constexpr int PPW = (TILE / 1024) / NW;  // DMA pieces per wave per tile, each of K and V
  static_assert(PPW >= 1 && PPW * NW * 1024 == TILE, "tile must split evenly over the waves");
  constexpr int DT = D / 32;                // 32-column output blocks
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(sl) (smem + (sl) * 2 * TILE)
#define VBUF(sl) (smem + (sl) * 2 * TILE + TILE)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const bool late = STAGGER && wid >= 4;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;

  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  (void)SLOTS;
  (void)RPP;
  auto issue = [&](int t) {
    const int sl = t % NSLOT;
    dma_tile_a<ROWB, NW, BN>(KBUF(sl), kbase + (int64_t)(t * BN) * ks, ks, wid, lane);
    dma_tile_a<ROWB, NW, BN>(VBUF(sl), vbase + (int64_t)(t * BN) * vs, vs, wid, lane);
  };
  issue(0);
  if (ntiles > 1) issue(1);

  bf16x8 qf[D / 16];
  {
    const bf16_t* qp = q + (int64_t)(b * S + q0w + r) * qs + hq * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
#pragma unroll
    for (int kk = 0; kk < D / 16; ++kk) asm volatile("" : "+v"(qf[kk]));
  }
  f32x16 oacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) oacc[i] = f32x16{0};
  float m = -INFINITY, l = 0.f;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  if (wid >= 4) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half (T5)

  // S^T = K . Q^T for the 64 keys of tile t (two 32-key accumulators), causal mask applied
  // lane base offsets of the sub-tiled image (swza): K rows r / r+32 at chunk 2kk+hh are
  // kb_lane[kk&1] + RB*4*(row>=32) + 512*(kk>>1); V^T tr-reads of rows R0 + 4hh + tq (R0 % 8 == 0) at
  // column block dt are vb_lane[(R0>>3)&1] + RB*(R0>>3) + 512*dt (RB = 8 rows of the image)
  constexpr int RB = ROWB * 8;
  const int kb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int kb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  const int vb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int vb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);
  auto kaddr = [&](const char* Kb, int kk, int half) {
    return Kb + ((kk & 1) ? kb_lane1 : kb_lane0) + RB * 4 * half + 512 * (kk >> 1);
  };
  (void)kaddr;
  // K row fragments in groups of 4 reads (k-steps 2g, 2g+1 x rows r, r+32), two groups in flight, each
  // retired by a counted lgkmcnt right before its MFMAs
  constexpr int NG = D / 32;
  auto kgroup = [&](uint32_t k0, uint32_t k1, auto gc, bf16x8* dst) {
    constexpr int g = decltype(gc)::value;
    static_for<2>([&](auto jc) {
      constexpr int kk = 2 * g + decltype(jc)::value;
      dst[2 * decltype(jc)::value] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? k1 : k0);
      dst[2 * decltype(jc)::value + 1] = lds_read8_off<RB * 4 + 512 * (kk >> 1)>((kk & 1) ? k1 : k0);
    });
  };
  auto qk = [&](int t, f32x16& s0, f32x16& s1) {
    const char* Kb = KBUF(t % NSLOT);
    const uint32_t k0 = lds_addr(Kb) + kb_lane0, k1 = lds_addr(Kb) + kb_lane1;
    s0 = f32x16{0};
    s1 = f32x16{0};
    // K row groups KG deep (KOP_FWD8_KDEPTH; 2 = the round-4 form)
    constexpr int KG = KOP_FWD8_KDEPTH < NG ? KOP_FWD8_KDEPTH : NG;
    bf16x8 gk[KG][4];
    static_for<KG>([&](auto i) { kgroup(k0, k1, i, gk[decltype(i)::value]); });
    static_for<NG>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      bf16x8* cur = gk[g % KG];
      constexpr int younger = 4 * (NG - 1 - g < KG - 1 ? NG - 1 - g : KG - 1);
      wait_rows4<younger>(cur);
      s0 = mfma32(cur[0], qf[2 * g], s0);
      s1 = mfma32(cur[1], qf[2 * g], s1);
      s0 = mfma32(cur[2], qf[2 * g + 1], s0);
      s1 = mfma32(cur[3], qf[2 * g + 1], s1);
      if constexpr (g + KG < NG) kgroup(k0, k1, std::integral_constant<int, g + KG>{}, cur);
    });
    const int kv0 = t * BN;
    if (causal && kv0 + BN - 1 > q0w) {
      const int qi = q0w + r;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int key = kv0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
        if (key > qi) s0[j] = -INFINITY;
        if (key + 32 > qi) s1[j] = -INFINITY;
      }
    }
  };
  // V^T fragments of key group ks4 (16 keys) for every 32-column output block dt (NR = 2*DT transposed
  // reads, each a lane base + immediate); consecutive P.V MFMAs go to DT independent accumulators
  constexpr int NR = 2 * DT;
  auto vread = [&](const char* Vb, auto ks4c, bf16x4* t) {
    constexpr int ks4 = decltype(ks4c)::value;
    constexpr int R0 = (ks4 >> 1) * 32 + 16 * (ks4 & 1);  // rows R0 + 4hh + tq and R0 + 8 + ...
    const uint32_t b0 = lds_addr(Vb) + vb_lane0, b1 = lds_addr(Vb) + vb_lane1;
    static_for<DT>([&](auto dtc) {
      constexpr int dt = decltype(dtc)::value;
      t[2 * dt] = lds_tr_read_off<RB * (R0 >> 3) + 512 * dt>(((R0 >> 3) & 1) ? b1 : b0);
      t[2 * dt + 1] = lds_tr_read_off<RB * ((R0 + 8) >> 3) + 512 * dt>((((R0 + 8) >> 3) & 1) ? b1 : b0);
    });
  };
  // online softmax of tile t's scores and O^T += V^T . P^T
  auto softmax_pv = [&](int t, f32x16& s0, f32x16& s1, auto db_tag) {
    constexpr bool DB = decltype(db_tag)::value;  // double-buffered V^T reads (needs 16 more VGPRs)
    const char* Vb = VBUF(t % NSLOT);
    bf16x4 ta[NR], tb[DB ? NR : 1];
    vread(Vb, std::integral_constant<int, 0>{}, ta);  // flies under the softmax
    float mx = max32(s0, s1);
    mx = xor32_max(mx);
    const float mt = mx * scale_log2;
    if (__any(mt > m + 8.f)) {
      const float mnew = fmaxf(m, mt);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i) oacc[i] *= alpha;
    }
    if constexpr (PK) {
      fma_pk16(s0, scale_log2, -m);
      fma_pk16(s1, scale_log2, -m);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s0[j] = __builtin_amdgcn_exp2f(s0[j]);
        s1[j] = __builtin_amdgcn_exp2f(s1[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s0[j] = __builtin_amdgcn_exp2f(fmaf(s0[j], scale_log2, -m));
        s1[j] = __builtin_amdgcn_exp2f(fmaf(s1[j], scale_log2, -m));
      }
    }
    l += sum32(s0, s1);
    const bf16x8 pf[4] = {pack_acc8(s0, 0), pack_acc8(s0, 1), pack_acc8(s1, 0), pack_acc8(s1, 1)};
    static_for<4>([&](auto ks4c) {
      constexpr int ks4 = decltype(ks4c)::value;
      bf16x4* cur = (DB && (ks4 & 1)) ? tb : ta;
      bf16x4* nxt = (DB && (ks4 & 1)) ? ta : tb;
      if constexpr (!DB) {
        if constexpr (ks4 > 0) vread(Vb, ks4c, cur);
        wait_tr<NR, 0>(cur);
      } else if constexpr (ks4 + 1 < 4) {
        vread(Vb, std::integral_constant<int, ks4 + 1>{}, nxt);
        wait_tr<NR, NR>(cur);
      } else {
        wait_tr<NR, 0>(cur);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt] = mfma32(cat44(cur[2 * dt], cur[2 * dt + 1]), pf[ks4], oacc[dt]);
    });
  };

  const int nloop = ntiles + (STAGGER ? 1 : 0);
  // every wave executes the same number of barriers; the two halves run separate loops so each loop's
  // live ranges are allocated on their own (one merged body spills)
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
    f32x16 sp0, sp1;  // scores of the pending tile, carried across the barrier
    bool pending = false;
    for (int it = 0; it < nloop; ++it) {
      top(it);
      if (pending) softmax_pv(it - 1, sp0, sp1, std::false_type{});
      pending = it < ntiles && (!causal || it * BN <= q0w + 31);
      if (pending) qk(it, sp0, sp1);
      asm volatile("" ::: "memory");
    }
  } else {
    for (int it = 0; it < nloop; ++it) {
      top(it);
      if (it < ntiles && (!causal || it * BN <= q0w + 31)) {
        f32x16 s0, s1;
        qk(it, s0, s1);
        softmax_pv(it, s0, s1, std::true_type{});
      }
      asm volatile("" ::: "memory");
    }
  }
#undef KBUF
#undef VBUF

  const float lt = xor32_sum(l);
  const float inv = 1.f / lt;
  if (hh == 0) lse[((int64_t)(b * Hq + hq)) * S + q0w + r] = (m + __log2f(lt)) * 0.69314718056f;
  if (ot != nullptr) {
    // O^T [Hq*D, B*S] as well: the K-contiguous X operand of the Wo weight-gradient GEMM. Lane r holds one
    // token of every column it owns, so a column's 32 tokens of the wave are one 64-B segment (the two waves of
    // a 128-B line are in this workgroup and merge in L2); rounded exactly like O.
    const int64_t T = (int64_t)B * S;
    bf16_t* otp = ot + (int64_t)(hq * D + 4 * hh) * T + (int64_t)b * S + q0w + r;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) otp[(int64_t)(dt * 32 + 8 * g + i) * T] = f2bf(oacc[dt][4 * g + i] * inv);
  }
  // widened store tail (guide T21): lane r holds columns 8g..8g+3 of row r, lane r+32 columns 8g+4..8g+7; one
  // v_permlane32_swap per dword of a (g, g+1) pair leaves lane r with columns 16p..16p+7 and lane r+32 with
  // 16p+8..16p+15, so each lane writes 16 B per pair: 8 dwordx4 stores instead of 16 dwordx2
  bf16_t* op = o + (int64_t)(b * S + q0w + r) * os + hq * D + 8 * hh;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int g0 = 2 * pr, g1 = 2 * pr + 1;
      const uint32_t a0 = pack2(oacc[dt][4 * g0] * inv, oacc[dt][4 * g0 + 1] * inv);
      const uint32_t a1 = pack2(oacc[dt][4 * g0 + 2] * inv, oacc[dt][4 * g0 + 3] * inv);
      const uint32_t b0 = pack2(oacc[dt][4 * g1] * inv, oacc[dt][4 * g1 + 1] * inv);
      const uint32_t b1 = pack2(oacc[dt][4 * g1 + 2] * inv, oacc[dt][4 * g1 + 3] * inv);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      *reinterpret_cast<u32x4*>(op + dt * 32 + 16 * pr) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
  }
}

template <int D, bool STAGGER, bool PK = false>
static void launch_fwd8(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S,
                        int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                        hipStream_t stream, bf16_t* ot) {
  const size_t lds = (STAGGER ? 4 : 3) * 2 * 64 * (D * 2);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_fwd8_kernel<D, STAGGER, PK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  const int grid = B * Hq * (S / 256);
  fa_fwd8_kernel<D, STAGGER, PK><<<grid, 512, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal,
                                                             ot);
}

constexpr int kFwdWaves = 4;

template <int D>
static void launch_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                       int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                       hipStream_t stream) {
  constexpr int NW = kFwdWaves;
  const size_t lds = 4 * 64 * (D * 2);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_fwd_kernel<D, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int grid = B * Hq * (S / (32 * NW));
  fa_fwd_kernel<D, NW><<<grid, NW * 64, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal);
}

static int g_fwd_variant = -2;  // -2: read KOP_FWD_VARIANT on first use; -1: per-head-dim default
int flash_attn_set_fwd_variant(int v) {
  if (g_fwd_variant == -2) {
    const char* e = getenv("KOP_FWD_VARIANT");
    g_fwd_variant = e ? atoi(e) : -1;
  }
  const int old = g_fwd_variant;
  if (v >= -1) g_fwd_variant = v;
  return old;
}

int flash_attn_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                   int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float scale, bool causal,
                   hipStream_t stream, bf16_t* ot) {
  if (S % (32 * kFwdWaves) != 0 || Hq % Hkv != 0) return -1;
  if (qs % 8 || ks % 8 || vs % 8 || os % 8) return -2;
  const float sl2 = scale * 1.4426950408889634f;
  // KOP_FWD_VARIANT: 8 lockstep 8-wave kernel (scalar-FMA softmax), 10 the same with packed FMAs, 9 staggered halves,
  // 16 the 8-wave structure on 16x16x32 MFMAs, < 8 the 4-wave kernel. Defaults per head dim from same-box probes:
  // D = 128 -> 8 (2-3 % over 10, profiles/r3_fwd_variant_probe.jsonl; 3-4 % over 16, whose 16-cycle MFMAs hold
  // the VALU issue half the time instead of a quarter, profiles/r5_fwd16_vdepth_ab.jsonl); D = 64 -> 16 (7 % over the
  // 4-wave kernel causal, 11 % over 8 non-causal at the GPT-2 shape; S % 256 == 0, else the 4-wave kernel).
  const int env_variant = flash_attn_set_fwd_variant(-3);  // current setting (-3 changes nothing)
  int variant = env_variant >= 0 ? env_variant : (D == 64) ? 16 : 8;
  if (ot != nullptr && variant < 8) variant = 8;  // O^T comes only from the 8-wave kernels
  // 12: the 4-wave one-wave-per-SIMD kernel, 64 rows per wave, hand-scheduled double pipeline (csrc/flash_fwd4.hip;
  // D = 128). An 8-wave double pipeline (QK of tile t+1 beside the softmax of tile t, 2 waves per SIMD) ran 15 %
  // slower and spilled: profiles/r5_experiments.md
  // 16: the 8-wave structure on 16x16x32 MFMAs (csrc/flash_fwd16.hip)
  if (S % 256 == 0 && variant == 16 && (D == 64 || D == 128))
    return flash_attn_fwd16(q, k, v, o, lse, B, S, Hq, Hkv, D, qs, ks, vs, os, sl2, causal, stream, ot);
  if (S % 256 == 0 && variant == 12 && D == 128) {
    return flash_attn_fwd4x64(q, k, v, o, lse, B, S, Hq, Hkv, D, qs, ks, vs, os, sl2, causal, stream, ot);
  }
  if (S % 256 == 0 && variant >= 8) {
    if (D == 128) {
      if (variant == 9) launch_fwd8<128, true>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
      else if (variant == 10) launch_fwd8<128, false, true>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
      else launch_fwd8<128, false>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
    } else if (D == 64) {
      if (variant == 9) launch_fwd8<64, true>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
      else if (variant == 10) launch_fwd8<64, false, true>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
      else launch_fwd8<64, false>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
    } else return -3;
    return 0;
  }
  if (ot != nullptr) return -4;  // O^T only from the 8-wave kernel
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream);
  else return -3;
  return 0;
}

}  // namespace kop
