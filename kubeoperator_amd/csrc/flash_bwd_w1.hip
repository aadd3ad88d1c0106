// Flash attention BACKWARD, dK / dV stage with one wave per SIMD (gfx950 / MI355X), D = 128.
// Built with -mllvm -amdgpu-mfma-vgpr-form=true (ops/_build.py FILE_FLAGS): the S / dP MFMAs are VGPR-form
// builtins (their results feed the softmax VALU directly, hipcc pads those hazards), while the dK^T / dV^T
// chains are inline-asm MFMAs on "+a" operands -- 256 accumulators pinned in the AGPR half of the 512-register
// file. (Left to its heuristic, hipcc put every MFMA in AGPR form: 320 AGPRs of demand for 256, ~600
// v_accvgpr moves per stage.) Wait states the asm needs: 2 after a VALU write of an A / B operand (the s_nop 1
// opening each statement); 18 after the last MFMA before the accumulators are read (the epilogue nop statement).
#include "attn_common.h"
#include "kernels.h"

namespace kop {


// QM staging write: lane r holds key r (of the block at byte offset BLK), queries 16S + {0-3, 8-11} (+4 for hh = 1);
// one permlane32_swap per dword pairs the halves into queries 16S + 8hh .. +7 (16 B) -> one ds_write_b128
template <int S16, int BLK>
__device__ __forceinline__ void stage_w(const u32x4& w, uint32_t base, std::integral_constant<int, BLK>) {
  const auto a = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
  const auto c = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
  const u32x4 o = {a[0], c[0], a[1], c[1]};
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(base), "v"(o), "n"(BLK));
}
// QM store instruction I: 8 slot-ordered keys (two transposed reads) of one query row -> 16 B
template <int I, bool NT = false>
__device__ __forceinline__ void stage_st(const bf16x4* x, uint64_t base, uint32_t off) {
  const u32x4 o = __builtin_bit_cast(u32x4, cat44(x[0], x[1]));
  if constexpr (NT)
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 nt\n\ts_nop 1" ::"v"(off), "v"(o), "s"(base), "n"(32 * I)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3\n\ts_nop 1" ::"v"(off), "v"(o), "s"(base), "n"(32 * I)
                 : "memory");
}

#ifndef KOP_DKDV_SDEPTH
#define KOP_DKDV_SDEPTH 4  // S-phase row-read depth in k-steps (3: the round-4 form)
#endif
#ifndef KOP_DKDV_PDEPTH
#define KOP_DKDV_PDEPTH 3  // dP-phase dO row-read depth in k-steps (4 measured equal: r5_experiments.md)
#endif
#ifndef KOP_DKDV_TDEPTH
#define KOP_DKDV_TDEPTH 3  // transposed-read ring of the dV / dK phases: TDEPTH - 1 steps ahead (2 in round 4; 4 measured equal)
#endif

// acc += a . b on the 32x32x16 bf16 MFMA with the accumulator in AGPRs (a dependent chain needs no wait states)
__device__ __forceinline__ void mfma32_agpr(f32x16& acc, bf16x8 a, bf16x8 b) {
  asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// =============================================================================================
// dK / dV, one wave per SIMD (KOP_DKDV_CFG 64, the default at D = 128)
// =============================================================================================
// The 2-waves-per-SIMD kernel (flash_bwd.hip fa_bwd_dkdv_kernel) gives each wave 32 keys, so every staged Q / dO tile is re-read from LDS
// per 32 keys (40 KB of LDS reads per wave per 32 MFMAs: the LDS array, not the matrix pipe, paced it --
// profiles/r3_attn_pmc_summary.txt) and it stored dS as 2-byte scatters (16 stores + 64 SALU address adds per
// stage). Here one 256-thread workgroup holds a CU alone (__launch_bounds__(256, 1): 512 registers per wave)
// and each wave owns 64 keys:
//   * dK^T / dV^T for 64 keys x 128 columns are 256 fp32 accumulators: the AGPR half of the register file;
//     V^T fragments of the 64 keys stay resident in VGPRs; every Q / dO fragment read from LDS feeds two
//     MFMAs (48 KB of LDS reads per 64 MFMAs);
//   * -lse / scale and -delta of the stage's 32 queries are the C operands of the first S and dP MFMAs
//     (shared by both 32-key blocks: no accumulator-initialisation moves), so p = exp2(c * acc), dS = p * acc;
//   * per stage: S (16 MFMAs) | dP (16) beside the exponentials | dV (16) beside dS | dK (16) -- each VALU
//     phase has an independent MFMA phase to hide under;
//   * dS is stored TRANSPOSED ([B, Hq, key, query], unscaled bf16): the accumulator holds one key per lane and
//     4-query runs per register quad, so one v_permlane32_swap per dword pairs the two lane halves into
//     8-query (16 B) runs -- 4 dwordx4 stores per wave per stage instead of 32 two-byte stores.
// Stage ring: Q / dO / {-lse/scale, -delta} of 32 queries, NS deep, behind counted vmcnt + raw barriers.

// DIAG bit 1: no dS stores -- the build the recompute-dQ path (KOP_DQ_VARIANT 9) launches. Timing ablations
// (KOP_DKDV64_DIAG, wrong results): 2 no exponentials, 4 no stage DMA, 8 no stage barrier, 32 no DMA wait; 16
// non-temporal dS stores (correct, slower).
// QM: dS in the query-major layout of fa_bwd_dkdv_kernel ([B, Hq, query, slot(key)]), staged through LDS so each
// wave writes whole 128-B lines (its 64 keys are one line of every query row). (QM = false, a transposed layout
// stored straight from the accumulators, measured slower and is no longer launched: profiles/r3_experiments.md.)
// BLK (with QM): wave-block dS layout [B, Hq, S/32, S/64, 32 queries, 64 slots]: a wave's stage tile is one contiguous
// 4 KB block (its workgroup's stage: 16 KB), instead of 32 rows of 128 B spread 2*S bytes apart.
// KT (QM = false with BLK): dS tiles of [B, Hq, S/64, S/32] stored straight from the accumulators -- no LDS staging
// (its ds_write_b128s are the slow LDS path) and no lane exchange: lane (r, hh)'s packed register quad s holds key r
// (+32 c for key block c), queries 16 s + 4 hh + 0..3 and 16 s + 8 + 4 hh + 0..3 (two 8-B runs); a wave's stage tile is
// 4 KB = four 1-KB blocks (c, s), and the lane stores the quad as-is at chunk 32 hh + (r ^ 4 hh ^ 8 s) of block 2 c + s
// (a v_permlane32_swap pairing into 8-query runs first cost 8 cross-lane ops per stage). Every store
// instruction then writes one whole 1-KB block, each 16-lane quarter two whole 128-B lines (a plain [64 keys][32
// queries] tile had each quarter write 16 B into 16 rows: 4 stores per stage then cost 14 % of the kernel). The XOR
// keeps the dQ kernel's ds_read_b64_tr_b16 reads of the tile conflict-free (fa_bwd_dq_ds_kernel<KMAJ>).
// REV: sweep the query stages from the last one down to the workgroup's diagonal. Every workgroup of a head then
// reads the same Q / dO stage at the same time (forward order starts workgroup kb 8*kb stages later, so a stage is
// re-read ~16 us apart -- long enough for the dS write stream to evict it from the XCD's 4 MB L2).
// HPW: query heads of one GQA group swept by the workgroup one after the other, accumulating into the same dK^T /
// dV^T registers (their keys and values are shared). HPW == the group size (DIRECT) writes bf16 dK / dV outright;
// otherwise the workgroup writes one fp32 partial per HPW heads (slot kvh * grp + part of [T, Hq, D]) and
// fa_bwd_finalize_kernel sums grp / HPW partials.
template <int D, bool DIRECT, int NS, bool QM, int DIAG = 0, bool BLK = false, bool REV = false, int HPW = 1>
__global__ void __launch_bounds__(256, 1) fa_bwd_dkdv64_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ nlse, const float* __restrict__ ndelta,
    float* __restrict__ dk_part, float* __restrict__ dv_part, bf16_t* __restrict__ dst, int B, int S, int Hq, int Hkv,
    int64_t qs, int64_t ks, int64_t vs, int64_t dos, float scale, int causal, int64_t dks, int64_t dvs) {
  constexpr int NW = 4, KW = 64, BN = NW * KW, BQ = 32, ROWB = D * 2;
  constexpr int KB = BN * ROWB, QT = BQ * ROWB, STAGE = 2 * QT + 1024;
  constexpr int MYP = (2 * QT / 1024) / NW;  // Q / dO DMA pieces per wave per stage
  static_assert(MYP * NW * 1024 == 2 * QT, "stage must split evenly over the waves");
  constexpr int DT = D / 32, NK = D / 16, RB = ROWB * 8;
  static_assert(NS == 3, "the vmcnt bookkeeping below tracks the stores of the two previous stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const Kl = smem;  // K image of the workgroup's 256 keys: only the second 32-key block of each wave is read

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int nkb = S / BN, grp = Hq / Hkv;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq / HPW, grp / HPW, nkb);
  const int kb = aw.rank;  // heaviest key blocks (earliest keys under a causal mask) first
  const int b = aw.b, hq0 = aw.unit * HPW;
  const int kvh = hq0 / grp;
  const int k0 = kb * BN, k0w = k0 + KW * wid;
  const float c2 = scale * 1.4426950408889634f;
  const int qt0 = causal ? k0 / BQ : 0;
  const int nqt = S / BQ;
  // the sweep: HPW heads x nst query stages in sequence (sq = head * nst + position in the order below). The DMA
  // issue runs NS - 1 stages ahead through a cursor advanced one stage at a time: the Q / dO / lse-delta source
  // pointers step by +-BQ rows (and jump to the next head's first stage at the end of a head), the ring slot is a
  // counter -- no integer multiply or division on the scalar unit per stage (the per-stage address products and
  // `% NS` were ~70 serial instructions in front of every stage's first MFMA)
  const int nst = nqt - qt0, tot = HPW * nst;
  const int qfirst = REV ? nqt - 1 : qt0;
  constexpr int QSTEP = REV ? -BQ : BQ;
  int iqt = qfirst, isq = 0, islot = 0;
  const bf16_t* iq = q + (int64_t)(b * S + qfirst * BQ) * qs + hq0 * D;
  const bf16_t* io = dout + (int64_t)(b * S + qfirst * BQ) * dos + hq0 * D;
  const int64_t iq_step = (int64_t)QSTEP * qs, io_step = (int64_t)QSTEP * dos;
  const int64_t iq_wrap = D - (int64_t)nst * iq_step, io_wrap = D - (int64_t)nst * io_step;
  // lse / delta rows of the stage: lane l < 8 reads -lse/scale floats 4l.., lanes 8..15 -delta floats 4(l-8)..
  const float* il = (((lane & 15) < 8) ? nlse + 4 * (lane & 15) : ndelta + 4 * ((lane & 15) - 8)) +
                    ((int64_t)(b * Hq + hq0)) * S + qfirst * BQ;
  const int64_t il_wrap = S - (int64_t)nst * QSTEP;
  dma_tile_a<ROWB, NW, BN>(Kl, k + (int64_t)(b * S + k0) * ks + kvh * D, ks, wid, lane);
  auto issue_next = [&]() {
    char* base = smem + KB + islot * STAGE;
    dma_tile_a<ROWB, NW, BQ>(base, iq, qs, wid, lane);
    dma_tile_a<ROWB, NW, BQ>(base + QT, io, dos, wid, lane);
    if (wid == 0) glds16(il, base + 2 * QT);
    iqt += REV ? -1 : 1;
    iq += iq_step;
    io += io_step;
    il += QSTEP;
    if (REV ? iqt < qt0 : iqt >= nqt) {
      iqt = qfirst;
      iq += iq_wrap;
      io += io_wrap;
      il += il_wrap;
    }
    ++isq;
    islot = islot == NS - 1 ? 0 : islot + 1;
  };
  issue_next();
#pragma unroll
  for (int i = 1; i < NS - 1; ++i)
    if (isq < tot) issue_next();

  const int rb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int rb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  const int tb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int tb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);

  // V^T fragments (B operand of dP = dO.V^T) of the wave's 64 keys and the K^T fragments (B operand of S = Q.K^T)
  // of its first 32 keys (key = k0w + 32*c + r, columns 16kk + 8hh ..), resident for the whole sweep; the second
  // key block's K rows still come from the LDS image. (Every stage used to re-read all 64 keys' K rows from LDS: 16
  // of the ~56 KB a wave read per stage, with the stage LDS-bandwidth bound -- dropping the 8 KB of dS staging
  // traffic alone saved 14 %. All 64 keys resident spilled at 512 registers and ran 11 % slower: r4_experiments.md.)
  bf16x8 vf0[NK], vf1[NK], kf0[NK];
  {
    const bf16_t* vp = v + (int64_t)(b * S + k0w + r) * vs + kvh * D + 8 * hh;
    const bf16_t* kp = k + (int64_t)(b * S + k0w + r) * ks + kvh * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      vf0[kk] = *reinterpret_cast<const bf16x8*>(vp + 16 * kk);
      vf1[kk] = *reinterpret_cast<const bf16x8*>(vp + 32 * vs + 16 * kk);
      kf0[kk] = *reinterpret_cast<const bf16x8*>(kp + 16 * kk);
    }
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) asm volatile("" : "+v"(vf0[kk]), "+v"(vf1[kk]), "+v"(kf0[kk]));
  }
  f32x16 dk0[DT], dk1[DT], dv0[DT], dv1[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dk0[i] = dk1[i] = dv0[i] = dv1[i] = f32x16{0};

  const int pcount = MYP + (wid == 0 ? 1 : 0);  // DMA ops this wave issues per stage
  int st1 = 0, st2 = 0;                           // dS stores issued in the previous / second-previous stage
  // dS^T rows of the wave's keys: row pointer in SGPRs (per head), lane offset (key r, queries 16s + 8hh) in one VGPR
  constexpr bool KT = !QM && BLK;
  auto dsrow_of = [&](int hq) {
    return KT ? (uint64_t)(uintptr_t)(dst + (((int64_t)(b * Hq + hq) * (S / 64) + k0w / 64) * (S / 32)) * 2048)
              : (uint64_t)(uintptr_t)(dst + ((int64_t)(b * Hq + hq) * S + k0w) * S);
  };
  const uint32_t dsoff = 2u * (uint32_t)(r * S + 8 * hh);
  // KT: byte offset of lane (r, hh)'s 16-B chunk in block (c, s): the s = 0 / s = 1 forms (c adds 2048 B)
  const uint32_t kto0 = 16u * (uint32_t)(32 * hh + (r ^ (4 * hh))), kto1 = 1024u + 16u * (uint32_t)(32 * hh + (r ^ (4 * hh) ^ 8));
  // QM staging image of the wave's stage tile: [64 keys][32 queries] bf16, 64-B rows, 16-B chunks XOR-swizzled
  // by (key >> 1) & 3. Writes: lane (key r of block c, queries 16s + 8hh ..) -> chunk 2s + hh. Transposed reads:
  // lane group G = lane >> 4 reads keys 16i + 4(G >> 1) + {0-3} and +8 (slot order) for queries 16(G & 1) + (lane & 15)
  // in store instruction i; the store puts those 8 keys (16 B) at dS[query][k0w + 16i + 8(G >> 1)].
  char* const stg = smem + KB + NS * STAGE + wid * 4096;
  const int xw = (r >> 1) & 3;
  const uint32_t stw0 = lds_addr(stg) + 64 * r + 16 * (hh ^ xw), stw1 = lds_addr(stg) + 64 * r + 16 * ((2 + hh) ^ xw);
  const int sg = lane >> 4, si = lane & 15, sq = si >> 2, sp = si & 3;
  const int skey = 4 * (sg >> 1) + sq;
  const uint32_t str = lds_addr(stg) + 64 * skey + 16 * ((2 * (sg & 1) + (sp >> 1)) ^ ((skey >> 1) & 3)) + 8 * (sp & 1);
  auto dsq_of = [&](int hq) {
    return BLK ? (uint64_t)(uintptr_t)(dst + ((int64_t)(b * Hq + hq) * (S / 32) * (S / 64) + k0w / 64) * 2048)
               : (uint64_t)(uintptr_t)(dst + ((int64_t)(b * Hq + hq) * S) * S + k0w);
  };
  const uint32_t sqoff = BLK ? 2u * (uint32_t)((16 * (sg & 1) + si) * 64 + 8 * (sg >> 1))
                             : 2u * (uint32_t)((16 * (sg & 1) + si) * S + 8 * (sg >> 1));
  (void)stw0; (void)stw1; (void)str; (void)sqoff;

  int cslot = 0;  // ring slot of the stage being computed (sq % NS)
  auto body = [&](int sq, int qt, uint64_t dsrow, uint64_t dsq, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    (void)dsrow; (void)dsq;
    // DMA(sq) is older than: stores(sq-2), DMA(sq+NS-2), stores(sq-1) (and the other DMAs still in flight). In the
    // steady state that is 8 + MYP (+1 on wave 0, whose lse/delta piece the constant wait then also retires: a
    // stricter wait, still correct); a runtime count goes through vm_wait_le's compare tree (~45 scalar
    // instructions and 16 branches), so only the sweep's first stages and its tail take it
    if constexpr (!(DIAG & 36)) {
      static_assert(NS == 3 && 8 + MYP <= 15, "constant steady-state wait");
      const int younger = st1 + st2 + ((sq + 1 < tot) ? pcount : 0);
      if (younger >= 8 + MYP) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + MYP) : "memory");
      else vm_wait_le(younger);
    }
    st2 = st1;
    st1 = 0;
    const int slot = cslot;
    cslot = cslot == NS - 1 ? 0 : cslot + 1;
    if constexpr (!(DIAG & 8)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (!(DIAG & 4)) {
      if (isq < tot) issue_next();  // the cursor is at stage sq + NS - 1
    }
    const int qs0 = qt * BQ;
    if (causal && qs0 + BQ - 1 < k0w) return;  // every query of the stage precedes every key of the wave
    const char* Ql = smem + KB + slot * STAGE;
    const char* Ol = Ql + QT;
    // Every LDS read below is an inline-asm read retired by a counted lgkmcnt, and every step ends in
    // sched_barrier(0): left to itself hipcc sank the MFMAs below later reads, which serialised them (one wave
    // per SIMD has no partner wave to hide that). Prefetch distance: 3 steps for row reads, 1 step (the 4 MFMAs
    // of a step, 128 cycles) for transposed reads.
    const uint32_t qb0 = lds_addr(Ql) + rb_lane0, qb1 = lds_addr(Ql) + rb_lane1;
    const uint32_t ob0 = lds_addr(Ol) + rb_lane0, ob1 = lds_addr(Ol) + rb_lane1;
    const uint32_t kw0 = lds_addr(Kl) + rb_lane0 + RB * 8 * wid + RB * 4, kw1 = lds_addr(Kl) + rb_lane1 + RB * 8 * wid + RB * 4;
    const uint32_t o0 = lds_addr(Ol) + tb_lane0, o1 = lds_addr(Ol) + tb_lane1;
    const uint32_t qa0 = lds_addr(Ql) + tb_lane0, qa1 = lds_addr(Ql) + tb_lane1;
    // -lse/scale (bytes 0..127) and -delta (128..255) of the stage's queries; accumulator row j is query
    // (j&3) + 8(j>>2) + 4hh, i.e. floats 8g + 4hh .. +3 for register quad g
    const uint32_t ldb = lds_addr(Ql + 2 * QT) + 16 * hh;
    auto grp = [&](auto kc, bf16x8* d2) {  // S-phase row reads of k-step kk: the Q row, the second key block's K row
      constexpr int kk = decltype(kc)::value;
      d2[0] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? qb1 : qb0);
      d2[1] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? kw1 : kw0);
    };
    auto dor = [&](auto kc) {  // dP-phase row read of k-step kk: dO row
      constexpr int kk = decltype(kc)::value;
      return lds_read8_off<512 * (kk >> 1)>((kk & 1) ? ob1 : ob0);
    };
    auto trr = [&](uint32_t b0, uint32_t b1, auto dtc, bf16x4* t) {  // transposed reads of column block dt
      constexpr int dt = decltype(dtc)::value;
      t[0] = lds_tr_read_off<512 * dt>(b0);
      t[1] = lds_tr_read_off<RB + 512 * dt>(b1);
      t[2] = lds_tr_read_off<RB * 2 + 512 * dt>(b0);
      t[3] = lds_tr_read_off<RB * 3 + 512 * dt>(b1);
    };
    using I = std::integral_constant<int, 0>;
    (void)I{};
    // ---- S = Q.K^T (16 MFMAs); the -lse/scale C operand is shared by both key blocks
    f32x4 lq[4];
    static_for<4>([&](auto g) { lq[decltype(g)::value] = lds_read16f_off<32 * decltype(g)::value>(ldb); });
    // S-phase row groups, KS deep (KOP_DKDV_SDEPTH 3 / 4): group kk lands in buffer kk % KS and is read KS steps
    // (2 KS MFMAs) ahead of its MFMAs
    constexpr int KS = KOP_DKDV_SDEPTH;
    bf16x8 gq[KS][2];
    static_for<KS>([&](auto i) { grp(i, gq[decltype(i)::value]); });
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(lq[0]), "+v"(lq[1]), "+v"(lq[2]), "+v"(lq[3]) : "n"(2 * KS));
    const f32x16 cl = cat4f(lq);
    f32x16 s0, s1;
    constexpr int PD = KOP_DKDV_PDEPTH, TD = KOP_DKDV_TDEPTH;
    bf16x8 dof[PD];
    f32x4 ld[4];
    static_for<NK>([&](auto kc) {
      constexpr int kk = decltype(kc)::value;
      bf16x8* cur = gq[kk % KS];
      // younger than group kk: the next KS - 1 groups, and from step NK-2 on the dP phase's 4 + PD early reads
      constexpr int younger = 2 * (NK - 1 - kk < KS - 1 ? NK - 1 - kk : KS - 1) + (kk > NK - 3 ? 4 + PD : 0);
      asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(cur[0]), "+v"(cur[1]) : "n"(younger));
      s0 = mfma32(cur[0], kf0[kk], kk == 0 ? cl : s0);
      s1 = mfma32(cur[0], cur[1], kk == 0 ? cl : s1);
      if constexpr (kk + KS < NK) grp(std::integral_constant<int, kk + KS>{}, cur);
      if constexpr (kk == NK - 3) {  // the dP phase's first reads fly under the last S MFMAs
        static_for<4>([&](auto g) { ld[decltype(g)::value] = lds_read16f_off<128 + 32 * decltype(g)::value>(ldb); });
        static_for<PD>([&](auto i) { dof[decltype(i)::value] = dor(i); });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    // ---- dP = dO.V^T (16 MFMAs) beside p = exp2(c * acc) and its bf16 packing (2 score pairs per block per step)
    const int kd = k0w + r - qs0 - 4 * hh;  // key - query + ((j&3) + 8(j>>2)) for register j of block 0
    (void)kd;
    f32x16 p0, p1;
    u32x4 pw0[2], pw1[2];
    // transposed-read jobs j = 0..2DT-1 of the dV (dO^T block j) and dK (Q^T block j - DT) phases, in buffers
    // tr3[j % 3], each issued two steps (8 MFMAs, ~256 cycles) before its MFMAs: with one step (one 128-cycle MFMA
    // step) of prefetch the waits sat in the LDS latency
    bf16x4 tr3[TD][4];
    auto job = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < DT) trr(o0, o1, std::integral_constant<int, j>{}, tr3[j % TD]);
      else trr(qa0, qa1, std::integral_constant<int, j - DT>{}, tr3[j % TD]);
    };
    static_for<NK>([&](auto kc) {
      constexpr int kk = decltype(kc)::value;
      bf16x8& cur = dof[kk % PD];
      // younger than dO row kk: the next PD - 1 rows, and from step NK-2 on the dV phase's early transposed reads
      constexpr int younger = (NK - 1 - kk < PD - 1 ? NK - 1 - kk : PD - 1) + (kk > NK - 3 ? 4 * (TD - 1) : 0);
      if constexpr (kk == 0) {
        asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(ld[0]), "+v"(ld[1]), "+v"(ld[2]), "+v"(ld[3]) : "n"(younger + 1));
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(cur) : "n"(younger));
      } else {
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(cur) : "n"(younger));
      }
      if constexpr (kk == 0) {
        const f32x16 cd = cat4f(ld);
        p0 = mfma32(cur, vf0[kk], cd);
        p1 = mfma32(cur, vf1[kk], cd);
      } else {
        p0 = mfma32(cur, vf0[kk], p0);
        p1 = mfma32(cur, vf1[kk], p1);
      }
      if constexpr (kk + PD < NK) cur = dor(std::integral_constant<int, kk + PD>{});
      if constexpr (kk == NK - 3) static_for<(TD - 1 < 2 * DT ? TD - 1 : 2 * DT)>([&](auto jc) { job(jc); });
      // this step's slice of the 16 scores per block: EP = 16 / NK elements (2 at D = 128, 4 at D = 64)
      constexpr int EP = 16 / NK;
#pragma unroll
      for (int e = 0; e < EP; ++e) {
        const int j = EP * kk + e;
        float a = (DIAG & 2) ? s0[j] * c2 : __builtin_amdgcn_exp2f(s0[j] * c2);
        float c = (DIAG & 2) ? s1[j] * c2 : __builtin_amdgcn_exp2f(s1[j] * c2);
        if constexpr (MASK) {
          if (kd > (j & 3) + 8 * (j >> 2)) a = 0.f;
          if (kd + 32 > (j & 3) + 8 * (j >> 2)) c = 0.f;
        }
        s0[j] = a;
        s1[j] = c;
      }
#pragma unroll
      for (int pi = EP * kk / 2; pi < EP * (kk + 1) / 2; ++pi) {
        pw0[pi >> 2][pi & 3] = pack2(s0[2 * pi], s0[2 * pi + 1]);
        pw1[pi >> 2][pi & 3] = pack2(s1[2 * pi], s1[2 * pi + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    const bf16x8 pb0[2] = {__builtin_bit_cast(bf16x8, pw0[0]), __builtin_bit_cast(bf16x8, pw0[1])};
    const bf16x8 pb1[2] = {__builtin_bit_cast(bf16x8, pw1[0]), __builtin_bit_cast(bf16x8, pw1[1])};
    // ---- dV^T += dO^T.P (16 MFMAs; each transposed fragment feeds both key blocks) beside dS = p * (dP - delta),
    // its packing and the transposed dS stores
    u32x4 sw0[2], sw1[2];
    // KT: the stage's tile (4 KB) and its second key block (keys 32..63: + 32 rows of 64 B)
    // DIAG 256 (timing ablation, wrong dQ): every stage's KT stores go to the wave's first tile (same 4 KB)
    const uint64_t row0 = KT ? dsrow + ((DIAG & 256) ? 0ull : 4096ull * (uint64_t)qt) : dsrow + 2ull * (uint64_t)qs0;
    const uint64_t row1 = KT ? row0 + 2048ull : row0 + 2ull * 32ull * (uint64_t)S;
    auto st = [](const u32x4& w, uint64_t row, int s, uint32_t off) {  // the row-major transposed layout (QM = false)
      // lane r holds key r, queries 16s + {0-3, 8-11} (+4 for hh = 1); one permlane32_swap per dword pairs the
      // halves into queries 16s + 8hh .. +7: 16 B per lane
      const auto a = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
      const auto c = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
      const u32x4 o = {a[0], c[0], a[1], c[1]};
      const uint64_t rs = row + 32ull * (uint64_t)s;
      asm volatile("global_store_dwordx4 %0, %1, %2\n\ts_nop 1" ::"v"(off), "v"(o), "s"(rs) : "memory");
    };
    // KT: the packed quad as-is (see the layout note), non-temporally (nt): dS is read back once, by the dQ kernel, and
    // left to the default policy its 2.15 GB stream pushed the Q / dO / K lines the stages re-read out of each XCD's L2
    // -- causal backward 1.659 / 1.668 ms vs 1.718 / 1.720 plain, sc1 1.697 / 1.690 (same box; on the LDS-staged layout
    // both policies had measured slower: r4_experiments.md). DIAG 64 / 128: sc1 / plain (A/B)
    auto st_kt = [](const u32x4& w, uint64_t row, uint32_t off) {
      if constexpr (DIAG & 64)
        asm volatile("global_store_dwordx4 %0, %1, %2 sc1\n\ts_nop 1" ::"v"(off), "v"(w), "s"(row) : "memory");
      else if constexpr (!(DIAG & 128))
        asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" ::"v"(off), "v"(w), "s"(row) : "memory");
      else
        asm volatile("global_store_dwordx4 %0, %1, %2\n\ts_nop 1" ::"v"(off), "v"(w), "s"(row) : "memory");
    };
    static_for<DT>([&](auto dtc) {
      constexpr int dt = decltype(dtc)::value;
      bf16x4* t = tr3[dt % TD];
      wait_tr<4, 4 * (TD - 2)>(t);  // jobs dt + 1 .. dt + TD - 2 may still fly
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        mfma32_agpr(dv0[dt], cat44(t[2 * s], t[2 * s + 1]), pb0[s]);
        mfma32_agpr(dv1[dt], cat44(t[2 * s], t[2 * s + 1]), pb1[s]);
      }
      // into job dt - 1's buffer (its MFMAs issued a step ago). Only real jobs: an asm read into registers nothing
      // reads afterwards lets hipcc hand them to other values while the LDS data is still on its way (seen at D = 64,
      // 2 DT = 4 jobs, with TDEPTH 4: wrong dS)
      if constexpr (dt + TD - 1 < 2 * DT) job(std::integral_constant<int, dt + TD - 1>{});
      // this step's slice of dS = p * (dP - delta): ED = 16 / DT elements (4 at D = 128, 8 at D = 64); query half
      // hs (elements 8hs .. 8hs+7) is complete -- and stored -- at the step that finishes its element 8hs + 7
      constexpr int ED = 16 / DT;
#pragma unroll
      for (int e = 0; e < ED; ++e) {
        const int j = ED * dt + e;
        p0[j] *= s0[j];
        p1[j] *= s1[j];
      }
#pragma unroll
      for (int pi = ED * dt / 2; pi < ED * (dt + 1) / 2; ++pi) {
        sw0[pi >> 2][pi & 3] = pack2(p0[2 * pi], p0[2 * pi + 1]);
        sw1[pi >> 2][pi & 3] = pack2(p1[2 * pi], p1[2 * pi + 1]);
      }
      static_for<2>([&](auto hc) {
        constexpr int hs = decltype(hc)::value;
        constexpr bool done_here = (ED * (dt + 1) > 8 * hs + 7) && (ED * dt <= 8 * hs + 7);
        if constexpr (done_here && (DIAG & 1)) asm volatile("" ::"v"(sw0[hs]), "v"(sw1[hs]));
        if constexpr (done_here && !(DIAG & 1)) {
          if constexpr (QM) {
            stage_w<hs>(sw0[hs], hs ? stw1 : stw0, std::integral_constant<int, 0>{});
            stage_w<hs>(sw1[hs], hs ? stw1 : stw0, std::integral_constant<int, 2048>{});
          } else {
            if constexpr (KT) {
              // stored in the dK phase below, one per step behind its MFMAs
            } else {
              st(sw0[hs], row0, hs, dsoff);
              st(sw1[hs], row1, hs, dsoff);
            }
          }
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    st1 = (DIAG & 1) ? 0 : 4;
    const bf16x8 sb0[2] = {__builtin_bit_cast(bf16x8, sw0[0]), __builtin_bit_cast(bf16x8, sw0[1])};
    const bf16x8 sb1[2] = {__builtin_bit_cast(bf16x8, sw1[0]), __builtin_bit_cast(bf16x8, sw1[1])};
    // ---- dK^T += Q^T.dS; QM: the staged dS tile goes out as whole lines in 4 store instructions, SPI = 4 / DT per
    // step (each two transposed reads, stored one step later)
    const uint64_t dsq0 = BLK ? dsq + 4096ull * (uint64_t)qt * (uint64_t)(S / 64) : dsq + 2ull * (uint64_t)qs0 * (uint64_t)S;
    constexpr int SPI = 4 / DT;
    static_assert(SPI * DT == 4 && (SPI == 1 || SPI == 2), "4 staged store instructions over the dK steps");
    bf16x4 xa[2 * SPI], xb[2 * SPI];
    auto xwait = [&](bf16x4* t, bf16x4* x) {
      if constexpr (SPI == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(x[0]), "+v"(x[1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
    };
    static_for<DT>([&](auto dtc) {
      constexpr int dt = decltype(dtc)::value;
      bf16x4* t = tr3[(DT + dt) % TD];  // job DT + dt
      bf16x4* xc = (dt & 1) ? xb : xa;
      bf16x4* xp = (dt & 1) ? xa : xb;
      if constexpr (QM && !(DIAG & 1)) {
        xwait(t, xp);
        if constexpr (dt > 0)
          static_for<SPI>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            stage_st<(dt - 1) * SPI + u, (DIAG & 16) != 0>(xp + 2 * u, dsq0, sqoff);
          });
      } else {
        // jobs DT + dt + 1 .. min(2 DT - 1, DT + dt + TD - 2) may still fly
        constexpr int yj = (2 * DT - 1 - (DT + dt)) < (TD - 2) ? (2 * DT - 1 - (DT + dt)) : (TD - 2);
        wait_tr<4, 4 * yj>(t);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        mfma32_agpr(dk0[dt], cat44(t[2 * s], t[2 * s + 1]), sb0[s]);
        mfma32_agpr(dk1[dt], cat44(t[2 * s], t[2 * s + 1]), sb1[s]);
      }
      if constexpr (DT + dt + TD - 1 < 2 * DT) job(std::integral_constant<int, DT + dt + TD - 1>{});
      if constexpr (KT && !(DIAG & 1)) {
        // the 4 dS stores spread over the dK steps (each blocks its wave while the CU's store path takes its 1 KB;
        // bunched 2 + 2 in the dV phase they were exposed): store u = (key block u & 1, query half u >> 1)
        static_for<4 / DT>([&](auto uc) {
          constexpr int u = dt * (4 / DT) + decltype(uc)::value, c = u & 1, hs = u >> 1;
          st_kt(c ? sw1[hs] : sw0[hs], c ? row1 : row0, hs ? kto1 : kto0);
        });
      }
      if constexpr (QM && !(DIAG & 1))
        static_for<SPI>([&](auto uc) {
          constexpr int u = decltype(uc)::value, I = dt * SPI + u;
          xc[2 * u] = lds_tr_read_off<1024 * I>(str);
          xc[2 * u + 1] = lds_tr_read_off<1024 * I + 512>(str);
        });
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (QM && !(DIAG & 1)) {
      bf16x4* xl = ((DT - 1) & 1) ? xb : xa;
      if constexpr (SPI == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xl[0]), "+v"(xl[1]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xl[0]), "+v"(xl[1]), "+v"(xl[2]), "+v"(xl[3]));
      static_for<SPI>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        stage_st<(DT - 1) * SPI + u, (DIAG & 16) != 0>(xl + 2 * u, dsq0, sqoff);
      });
    }
    asm volatile("" ::: "memory");
  };
  // the causal mask is needed only in the BN / BQ stages nearest the diagonal (qt < qd)
  const int qd = causal ? (qt0 + BN / BQ < nqt ? qt0 + BN / BQ : nqt) : qt0;
  // per head: two loops (unmasked / masked stages) -- one loop with a branch between the two body instantiations
  // made hipcc spill ~500 VGPRs
  for (int hi = 0; hi < HPW; ++hi) {
    const int s0 = hi * nst;
    const uint64_t dr = dsrow_of(hq0 + hi), dq = dsq_of(hq0 + hi);
    if constexpr (REV) {
      for (int qt = nqt - 1; qt >= qd; --qt) body(s0 + (nqt - 1 - qt), qt, dr, dq, std::false_type{});
      for (int qt = qd - 1; qt >= qt0; --qt) body(s0 + (nqt - 1 - qt), qt, dr, dq, std::true_type{});
    } else {
      int qt = qt0;
      for (; qt < qd; ++qt) body(s0 + (qt - qt0), qt, dr, dq, std::true_type{});
      for (; qt < nqt; ++qt) body(s0 + (qt - qt0), qt, dr, dq, std::false_type{});
    }
  }
  // the accumulators leave the AGPRs through compiler v_accvgpr_read: 18 wait states after the last 16-pass MFMA
  // that wrote them (hipcc pads nothing after an asm MFMA)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(dk0[0]), "+a"(dk0[1]), "+a"(dk0[2]), "+a"(dk0[3]), "+a"(dk1[0]), "+a"(dk1[1]), "+a"(dk1[2]),
                 "+a"(dk1[3]), "+a"(dv0[0]), "+a"(dv0[1]), "+a"(dv0[2]), "+a"(dv0[3]), "+a"(dv1[0]), "+a"(dv1[1]),
                 "+a"(dv1[2]), "+a"(dv1[3]));

  auto out = [&](const f32x16* dka, const f32x16* dva, int key) {
    if constexpr (DIRECT) {
      bf16_t* dkb = reinterpret_cast<bf16_t*>(dk_part) + (int64_t)(b * S + key) * dks + kvh * D;
      bf16_t* dvb = reinterpret_cast<bf16_t*>(dv_part) + (int64_t)(b * S + key) * dvs + kvh * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = dt * 32 + 8 * g4 + 4 * hh;
          *reinterpret_cast<u32x2*>(dkb + d) =
              u32x2{pack2(dka[dt][4 * g4] * scale, dka[dt][4 * g4 + 1] * scale),
                    pack2(dka[dt][4 * g4 + 2] * scale, dka[dt][4 * g4 + 3] * scale)};
          *reinterpret_cast<u32x2*>(dvb + d) =
              u32x2{pack2(dva[dt][4 * g4], dva[dt][4 * g4 + 1]), pack2(dva[dt][4 * g4 + 2], dva[dt][4 * g4 + 3])};
        }
      }
    } else {
      const int slot = kvh * grp + (hq0 % grp) / HPW;  // this workgroup's partial of the group
      float* dkp = dk_part + (int64_t)(b * S + key) * Hq * D + slot * D;
      float* dvp = dv_part + (int64_t)(b * S + key) * Hq * D + slot * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = dt * 32 + 8 * g4 + 4 * hh;
          *reinterpret_cast<f32x4*>(dkp + d) = f32x4{dka[dt][4 * g4] * scale, dka[dt][4 * g4 + 1] * scale,
                                                     dka[dt][4 * g4 + 2] * scale, dka[dt][4 * g4 + 3] * scale};
          *reinterpret_cast<f32x4*>(dvp + d) =
              f32x4{dva[dt][4 * g4], dva[dt][4 * g4 + 1], dva[dt][4 * g4 + 2], dva[dt][4 * g4 + 3]};
        }
      }
    }
  };
  out(dk0, dv0, k0w + r);
  out(dk1, dv1, k0w + 32 + r);
}

// heads per workgroup: the largest power of two dividing the GQA group that still leaves >= 2 workgroups per CU under
// a causal mask (the causal key blocks differ 32x in work; fewer, longer workgroups would end on a few heavy ones), >= 1
// without one (equal work per workgroup: fewer partials win -- Llama-3-8B shape non-causal 2.862 / 2.861 ms with HPW 4
// vs 2.899 / 2.940 with 2, causal 2.14 vs 1.65 ms: profiles/r4_dkdv_hpw_recheck.jsonl).
// KOP_DKDV_HPW / flash_attn_set_dkdv_hpw override it (1 / 2 / 4 / 8; 0 automatic).
static int g_hpw = -1;  // -1: read KOP_DKDV_HPW on first use; 0: automatic; 1 / 2 / 4 / 8: forced
int flash_attn_set_dkdv_hpw(int h) {
  if (g_hpw < 0) {
    const char* e = getenv("KOP_DKDV_HPW");
    g_hpw = e ? atoi(e) : 0;
  }
  const int old = g_hpw;
  if (h >= 0) g_hpw = h;
  return old;
}
static int pick_hpw(int B, int S, int Hq, int Hkv, bool causal) {
  const int env = flash_attn_set_dkdv_hpw(-1);
  const int grp = Hq / Hkv;
  if (env > 0) return (grp % env == 0 && env <= 8) ? env : 1;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  int h = 1;
  const int64_t min_wg = (causal ? 2 : 1) * (int64_t)cus;
  while (h * 2 <= 8 && grp % (h * 2) == 0 && (int64_t)B * (Hq / (h * 2)) * (S / 256) >= min_wg) h *= 2;
  return h;
}

template <int D>
static int dkdv64_launch(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                         const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B,
                         int S, int Hq, int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                         int64_t dvs, float scale, int causal, bool qm, bool blk_layout, hipStream_t stream) {
  constexpr int NS = 3;
  const size_t lds = 256 * (D * 2) + NS * (2 * 32 * (D * 2) + 1024) + 4 * 4096;
  const int grp = Hq / Hkv;
#ifdef KOP_ABLATIONS
  // timing ablations of the stage (DIAG bits above; WRONG dK / dV / dS except 16 / 64 / 128): compiled only into the
  // probe build of tools/ (-DKOP_ABLATIONS), never into the shipped extension
  static const int diag = [] {
    const char* e = getenv("KOP_DKDV64_DIAG");
    return e ? atoi(e) : 0;
  }();
#endif
  // one instantiation per (DIRECT, QM, DIAG, BLK, REV, HPW) actually launched; the dynamic-LDS attribute is set on
  // first use. Returns the number of partials per GQA group the finalize pass must sum (0: dK / dV written).
#define KOP_LAUNCH(DIR, QMV, DG, BL) KOP_LAUNCH_R(DIR, QMV, DG, BL, true, 1)
#define KOP_LAUNCH_R(DIR, QMV, DG, BL, RV, HP)                                                                         \
  do {                                                                                                             \
    static bool attr = false;                                                                                      \
    if (!attr) {                                                                                                   \
      (void)hipFuncSetAttribute((const void*)fa_bwd_dkdv64_kernel<D, DIR, NS, QMV, DG, BL, RV, HP>,                 \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
      attr = true;                                                                                                 \
    }                                                                                                              \
    const dim3 grid(B * (Hq / HP) * (S / 256));                                                                    \
    if (DIR)                                                                                                       \
      fa_bwd_dkdv64_kernel<D, DIR, NS, QMV, DG, BL, RV, HP><<<grid, 256, lds, stream>>>(                             \
          q, k, v, dout, nlse, ndelta, reinterpret_cast<float*>(dk), reinterpret_cast<float*>(dv), ds, B, S, Hq, Hkv, \
          qs, ks, vs, dos, scale, causal, dks, dvs);                                                               \
    else                                                                                                           \
      fa_bwd_dkdv64_kernel<D, DIR, NS, QMV, DG, BL, RV, HP><<<grid, 256, lds, stream>>>(                             \
          q, k, v, dout, nlse, ndelta, dk_part, dv_part, ds, B, S, Hq, Hkv, qs, ks, vs, dos, scale, causal, 0, 0);  \
    return (DIR) ? 0 : grp / (HP);                                                                                 \
  } while (0)
#ifdef KOP_ABLATIONS
  if (diag != 0 && Hq != Hkv && qm && ds != nullptr) {
    switch (diag) {
      case 1: KOP_LAUNCH(false, true, 1, false);
      case 2: KOP_LAUNCH(false, true, 2, false);
      case 4: KOP_LAUNCH(false, true, 4, false);
      case 8: KOP_LAUNCH(false, true, 8, false);
      case 16: KOP_LAUNCH(false, true, 16, false);
      case 32: KOP_LAUNCH(false, true, 32, false);
      case 48: KOP_LAUNCH(false, true, 48, false);
      default: break;
    }
  }
#endif
  if (ds == nullptr) {  // no dS at all (dQ recomputes it): the store-free build
    if (Hq == Hkv) KOP_LAUNCH(true, true, 1, false);
    else KOP_LAUNCH(false, true, 1, false);
  }
  if (Hq == Hkv) {
#ifdef KOP_ABLATIONS
    if (diag != 0 && blk_layout && !qm) {  // timing ablations of the KT build (wrong results except 0)
      switch (diag) {
        case 1: KOP_LAUNCH(true, false, 1, true);
        case 2: KOP_LAUNCH(true, false, 2, true);
        case 4: KOP_LAUNCH(true, false, 4, true);
        case 8: KOP_LAUNCH(true, false, 8, true);
        case 12: KOP_LAUNCH(true, false, 12, true);
        case 3: KOP_LAUNCH(true, false, 3, true);
        default: break;
      }
    }
#endif
    if (blk_layout && !qm) KOP_LAUNCH(true, false, 0, true);  // KT tiles
    if (blk_layout) KOP_LAUNCH(true, true, 0, true);
    else KOP_LAUNCH(true, true, 0, false);
  }
  const int hpw = pick_hpw(B, S, Hq, Hkv, causal != 0);
  if (blk_layout && !qm) {  // KT tiles: dS stored straight from the accumulators
#ifdef KOP_ABLATIONS
    if (diag == 1 && hpw == 2 && grp != 2) KOP_LAUNCH_R(false, false, 1, true, true, 2);  // ablation: no dS stores
    if (diag == 64 && hpw == 2 && grp != 2) KOP_LAUNCH_R(false, false, 64, true, true, 2);  // sc1 dS stores
    if (diag == 128 && hpw == 2 && grp != 2) KOP_LAUNCH_R(false, false, 128, true, true, 2);  // plain dS stores
    if (diag == 256 && hpw == 2 && grp != 2) KOP_LAUNCH_R(false, false, 256, true, true, 2);  // stores to one tile
#endif
    switch (hpw) {
      case 2: if (grp == 2) KOP_LAUNCH_R(true, false, 0, true, true, 2); else KOP_LAUNCH_R(false, false, 0, true, true, 2);
      case 4: if (grp == 4) KOP_LAUNCH_R(true, false, 0, true, true, 4); else KOP_LAUNCH_R(false, false, 0, true, true, 4);
      case 8: if (grp == 8) KOP_LAUNCH_R(true, false, 0, true, true, 8); else KOP_LAUNCH_R(false, false, 0, true, true, 8);
      default: KOP_LAUNCH(false, false, 0, true);
    }
  }
  if (blk_layout) {
    switch (hpw) {
      case 2: if (grp == 2) KOP_LAUNCH_R(true, true, 0, true, true, 2); else KOP_LAUNCH_R(false, true, 0, true, true, 2);
      case 4: if (grp == 4) KOP_LAUNCH_R(true, true, 0, true, true, 4); else KOP_LAUNCH_R(false, true, 0, true, true, 4);
      case 8: if (grp == 8) KOP_LAUNCH_R(true, true, 0, true, true, 8); else KOP_LAUNCH_R(false, true, 0, true, true, 8);
      default: KOP_LAUNCH(false, true, 0, true);
    }
  }
  KOP_LAUNCH(false, true, 0, false);
#undef KOP_LAUNCH
#undef KOP_LAUNCH_R
}

int flash_attn_bwd_dkdv64(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout, const float* nlse,
                          const float* ndelta, float* dk_part, float* dv_part, bf16_t* dk, bf16_t* dv, bf16_t* ds, int B,
                          int S, int Hq, int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t dos, int64_t dks,
                          int64_t dvs, float scale, int causal, bool qm, bool blk_layout, hipStream_t stream) {
  if (D == 128)
    return dkdv64_launch<128>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, dos,
                              dks, dvs, scale, causal, qm, blk_layout, stream);
  return dkdv64_launch<64>(q, k, v, dout, nlse, ndelta, dk_part, dv_part, dk, dv, ds, B, S, Hq, Hkv, qs, ks, vs, dos, dks,
                           dvs, scale, causal, qm, blk_layout, stream);
}

}  // namespace kop
