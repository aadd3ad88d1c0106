// Flash attention FORWARD, 4 waves per workgroup and ONE wave per SIMD (gfx950 / MI355X), D = 128, with the main loop
// scheduled by hand.
//
// Why: the 8-wave kernel (flash_fwd.hip) pairs two waves per SIMD that run the same phase in lockstep, so its MFMA
// pipe idles while both do softmax (~0.52 MFMA utilisation, profiles/r4_attn_pmc_summary_normalized.txt). Here each
// wave owns 64 query rows (two 32-row blocks) and the whole 512-entry register file, and keeps its own matrix pipe
// busy: the QK^T MFMAs of key tile t+1 and the P.V MFMAs of tile t form one 64-MFMA block per tile whose gaps carry
// tile t's softmax (guide T15 double pipeline; cdna_hip_programming.md '4-wave, one-wave-per-SIMD structure').
// Every K row fragment and V^T fragment read from LDS feeds two MFMAs (both row blocks).
//
// Register ownership (the compiler cannot be trusted with it: left alone it moved the accumulators between AGPRs and
// VGPRs ~200 times per tile and spilled Q, see profiles/r5_experiments.md):
//   * a[64:191]  O^T accumulators, 8 tiles of 32x32 fp32 (row block rb, 32-column block dt at a[64 + 16 (4 rb + dt)]),
//                written only by inline-asm MFMAs, read back by inline-asm v_accvgpr_read;
//   * a[192:255] Q^T fragments (row block rb, k-step kk at a[192 + 4 (8 rb + kk)]), loaded straight from global
//                memory into AGPRs, the B operand of every S MFMA;
//   * a[0:63]    left to hipcc (it parks VGPRs there under pressure; the build test checks it stays below a64);
//   * VGPRs      (hipcc's) S^T score tiles of t and t+1, K / V^T fragments, P^T operands, softmax state.
// The asm MFMAs are hazard-padded by hand (hipcc pads nothing around inline asm): 2 wait states (s_nop 1) before each
// P.V MFMA whose P operand a VALU has just written; 18 before any access to O after its last MFMA (o_fence); VALU
// reads of an S tile happen >= 8 MFMA slots after its last MFMA (schedule) or behind an 18-state fence (s_fence).
// tools/isa_mfma_hazards.py checks the built code (VALU write -> MFMA source within 2 states).
//
// Schedule of one tile (64 slots = one MFMA each + fillers, pinned by sched_barrier):
//   slots  0-31  S^T(t+1) = K(t+1) . Q^T   K row fragments 2 groups ahead; LDS-DMA of tile t+2 every 3 slots;
//                                          exponentials / row sums / bf16 packs of S(t) (1-2 per slot)
//   slots 32-63  O^T += V^T(t) . P^T(t)    V^T fragments one 16-key group ahead; the rest of S(t)'s
//                                          exponentials (needed by the last two key groups), then S(t+1)'s row max
//   after        the rescale decision for t+1 (lazy, 2^8; rare O rescale through v_accvgpr read / write)
// The diagonal tile (causal mask) and the last tile take an unscheduled path.
// Layout, DMA ring (3 slots), work order and O / O^T / lse outputs as the 8-wave kernel.
#include "attn_common.h"
#include "kernels.h"

#ifndef KOP_FWD4_PVNOP
#define KOP_FWD4_PVNOP 0  // 1: s_nop 1 before every P.V MFMA (not only where the schedule needs it)
#endif
#ifndef KOP_FWD4_SBG
#define KOP_FWD4_SBG 1  // slots per sched_barrier group (1: every slot pinned)
#endif

namespace kop {

namespace fwd4 {

#ifndef KOP_FWD4_RING
#define KOP_FWD4_RING 3  // LDS ring slots: 3 = DMA two tiles ahead, 4 = three (measured equal: r5_experiments.md)
#endif
constexpr int D = 128, NW = 4, BM = 256, BN = 64, ROWB = 2 * D, TILE = BN * ROWB, NSLOT = KOP_FWD4_RING;
constexpr int AHEAD = NSLOT - 1;  // tiles the LDS-DMA runs ahead of the tile being consumed
constexpr int PPW = (TILE / 1024) / NW;  // LDS-DMA pieces per wave per tile, each of K and V
constexpr int DT = D / 32, NR = 2 * DT, NK = D / 16, NG = D / 32;
constexpr int RB = ROWB * 8;
static_assert(PPW == 4 && NG == 4 && DT == 4, "schedule tables assume D = 128");

// the asm-owned AGPRs sit at the TOP of the file (a[64:255]): hipcc allocates its own AGPRs (VGPR spill space)
// from a0 upward, and tests/test_kernel_resources.py fails the build if it ever reaches a64
constexpr int ABASE = 64;
constexpr int OB(int rb, int dt) { return ABASE + 16 * (DT * rb + dt); }
constexpr int QB(int rb, int kk) { return ABASE + 16 * 2 * DT + 4 * (NK * rb + kk); }
static_assert(QB(1, NK - 1) + 3 == 255, "O and Q fill a[64:255]");

// ---- schedule tables (slot = one MFMA) ----
// the 64 exponentials of tile t: element e -> (rb, h, j); order = the P^T operand deadlines
constexpr int e_rb(int e) { return e < 16 ? 0 : e < 32 ? 1 : ((e - 32) / 8) & 1; }
constexpr int e_h(int e) { return e < 32 ? 0 : 1; }
constexpr int e_j(int e) { return e < 32 ? (e & 15) : (e < 48 ? (e & 7) : 8 + (e & 7)); }
// slots 0..55: one per slot in the QK half (it also carries the LDS-DMA), 1-2 per slot in the P.V half
constexpr int e_slot(int e) { return e < 24 ? e : 24 + (e - 24) * 32 / 40; }
// In-order issue stalls on a dependent operand, so each element is software-pipelined over the slots (an MFMA's
// 32 cycles between stages): v_fma (argument) at e_slot - 2, v_exp at e_slot - 1, the row-sum add at e_slot + 1;
// slot -1 is the preamble before the first MFMA
constexpr int fma_slot(int e) { return e_slot(e) - 2 < -1 ? -1 : e_slot(e) - 2; }
constexpr int exp_slot(int e) { return e_slot(e) - 1 < -1 ? -1 : e_slot(e) - 1; }
constexpr int add_slot(int e) { return e_slot(e) + 1; }
// P^T operand pf[rb][k] (k = 2h + j/8) is complete after its 8th exponential: pack it two slots after that
constexpr bool e_last(int e) { return (e & 7) == 7; }
constexpr int pack_slot(int e) { return exp_slot(e) + 2; }
// row-max ops of S(t+1) (16 v_max3 per row block, the two blocks' chains interleaved) in slots 40..61, the
// cross-half finish in 62
constexpr int x_slot(int x) { return 40 + x * 22 / 32; }

}  // namespace fwd4

using namespace fwd4;

// ---- inline-asm primitives on fixed AGPRs ----
template <int Q>
__device__ __forceinline__ void s_mfma0(f32x16& s, const bf16x8& kf) {  // s = K . Q^T (chain start)
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, a[%2:%3], 0" : "=&v"(s) : "v"(kf), "n"(Q), "n"(Q + 3));
}
template <int Q>
__device__ __forceinline__ void s_mfma(f32x16& s, const bf16x8& kf) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, a[%2:%3], %0" : "+v"(s) : "v"(kf), "n"(Q), "n"(Q + 3));
}
// NOP: 2 wait states first, for a P^T operand packed by the instruction just before (the schedule says where;
// tools/isa_mfma_hazards.py checks the built code)
template <int O, bool NOP = true>
__device__ __forceinline__ void o_mfma(const bf16x8& vf, const bf16x8& pf) {  // O^T += V^T . P^T
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%2:%3], %0, %1, a[%2:%3]" ::"v"(vf), "v"(pf), "n"(O),
                 "n"(O + 15));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%2:%3], %0, %1, a[%2:%3]" ::"v"(vf), "v"(pf), "n"(O), "n"(O + 15));
}
__device__ __forceinline__ void o_fence() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }
template <int O>
__device__ __forceinline__ void o_scale4(float al) {  // a[O..O+3] *= al
  float t0, t1, t2, t3;
  asm volatile(
      "v_accvgpr_read_b32 %0, a[%5]\n\tv_accvgpr_read_b32 %1, a[%6]\n\tv_accvgpr_read_b32 %2, a[%7]\n\t"
      "v_accvgpr_read_b32 %3, a[%8]\n\tv_mul_f32 %0, %0, %4\n\tv_mul_f32 %1, %1, %4\n\tv_mul_f32 %2, %2, %4\n\t"
      "v_mul_f32 %3, %3, %4\n\tv_accvgpr_write_b32 a[%5], %0\n\tv_accvgpr_write_b32 a[%6], %1\n\t"
      "v_accvgpr_write_b32 a[%7], %2\n\tv_accvgpr_write_b32 a[%8], %3"
      : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
      : "v"(al), "n"(O), "n"(O + 1), "n"(O + 2), "n"(O + 3));
}
template <int O>
__device__ __forceinline__ float o_read(std::integral_constant<int, O>) {
  float x;
  asm volatile("v_accvgpr_read_b32 %0, a[%1]" : "=v"(x) : "n"(O));
  return x;
}
template <int Q>
__device__ __forceinline__ void q_load(const bf16_t* p) {  // counted by the caller's vmcnt
  asm volatile("global_load_dwordx4 a[%1:%2], %0, off" ::"v"(p), "n"(Q), "n"(Q + 3) : "memory");
}

#define KOP_A8(n) "a" #n "0", "a" #n "1", "a" #n "2", "a" #n "3", "a" #n "4", "a" #n "5", "a" #n "6", "a" #n "7", \
                  "a" #n "8", "a" #n "9"
// claims a64..a255 for the kernel descriptor (the asm above names them literally)
__device__ __forceinline__ void claim_agprs() {
  asm volatile("" ::: "a64", "a65", "a66", "a67", "a68", "a69", KOP_A8(7), KOP_A8(8), KOP_A8(9), KOP_A8(10), KOP_A8(11),
               KOP_A8(12), KOP_A8(13), KOP_A8(14), KOP_A8(15), KOP_A8(16), KOP_A8(17), KOP_A8(18), KOP_A8(19),
               KOP_A8(20), KOP_A8(21), KOP_A8(22), KOP_A8(23), KOP_A8(24), "a250", "a251", "a252", "a253", "a254",
               "a255");
}
#undef KOP_A8

// f32 ops of the fillers are plain C++: this file is built with -fno-slp-vectorize (no v_pk_*_f32 beside MFMAs, an
// anti-lever: MI355X_MICROARCH.md 'price of one filler') and -fno-honor-nans (fmaxf -> v_max3_f32 with no
// canonicalising v_max of each asm-produced score); inline-asm VALU would cost an s_nop after every statement
__device__ __forceinline__ float max3n(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

#ifdef KOP_FWD4_STAMP
// per-segment cycle stamps (tools/fwd4_probe.hip): s_memtime at points with no LDS read outstanding
__device__ unsigned long long g_fwd4_stamp[12];
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define KOP_STAMP(var) const unsigned long long var = stamp_now()
#else
#define KOP_STAMP(var)
#endif

__device__ __forceinline__ float half_swap_max(float x) {  // max over lanes l and l ^ 32
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

__global__ void __launch_bounds__(256, 1) fa_fwd4x64_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                            const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                            float* __restrict__ lse, int B, int S, int Hq, int Hkv,
                                                            int64_t qs, int64_t ks, int64_t vs, int64_t os,
                                                            float scale_log2, int causal, bf16_t* __restrict__ ot) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(sl) (smem + (sl) * 2 * TILE)
#define VBUF(sl) (smem + (sl) * 2 * TILE + TILE)
  claim_agprs();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 64;  // this wave's rows: q0w + 32 rb + r
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;
  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;

  // Q^T fragments into a[128:191] first, then tiles 0 and 1: the prologue's vmcnt(2 PPW) covers Q and tile 0
  static_for<2>([&](auto rbc) {
    constexpr int rb = decltype(rbc)::value;
    const bf16_t* qp = q + (int64_t)(b * S + q0w + 32 * rb + r) * qs + hq * D + 8 * hh;
    static_for<NK>([&](auto kc) { q_load<QB(rb, decltype(kc)::value)>(qp + 16 * decltype(kc)::value); });
  });
  // one LDS-DMA piece (i < PPW: K, else V) of tile t, the per-piece form of dma_tile_a
  const int lrow = (lane & 31) >> 2, lhi = lane >> 5, lslot = lane & 3;
  // LDS-DMA piece i of tile t (i < PPW: K, else V): piece pc = wid + NW i covers rows 16 i + row0 of the tile, and
  // every piece of a wave reads the same lane chunk, so the source is a wave-uniform row base (SGPRs) plus one
  // loop-invariant lane byte offset (the saddr form: no per-piece 64-bit VALU address arithmetic)
  static_assert(ROWB / 128 == 2 && NW == 4, "piece geometry");
  const int row0 = 8 * (wid >> 1) + lrow;
  const int ch0 = 4 * (2 * (wid & 1) + lhi) + (lslot ^ ((row0 >> 2) & 3));
  const uint32_t loff_k = (uint32_t)((row0 * ks + ch0 * 8) * 2), loff_v = (uint32_t)((row0 * vs + ch0 * 8) * 2);
  auto piece_src = [&](int t, int i) {
    const bool isv = i >= PPW;
    const int ii = isv ? i - PPW : i;
    return isv ? reinterpret_cast<const char*>(vbase + (int64_t)(t * BN + 16 * ii) * vs) + loff_v
               : reinterpret_cast<const char*>(kbase + (int64_t)(t * BN + 16 * ii) * ks) + loff_k;
  };
  auto piece_dst = [&](int sl, int i) {
    const bool isv = i >= PPW;
    const int pc = wid + (isv ? i - PPW : i) * NW;
    return (isv ? VBUF(sl) : KBUF(sl)) + pc * 1024;
  };
  auto piece_at = [&](int t, int sl, int i) { glds16(piece_src(t, i), piece_dst(sl, i)); };
  auto piece = [&](int t, int i) { piece_at(t, t % NSLOT, i); };
  auto issue = [&](int t) {
    for (int i = 0; i < 2 * PPW; ++i) piece(t, i);
  };
  static_assert(AHEAD <= 4, "S % 256 == 0 gives ntiles >= 4");
  for (int t = 0; t < AHEAD; ++t) issue(t);
  static_for<16 * 2 * DT>([&](auto ic) {
    asm volatile("v_accvgpr_write_b32 a[%0], 0" ::"n"(ABASE + decltype(ic)::value));
  });

  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg1 = (lane >> 4) & 1;
  const int kb_lane0 = RB * (r >> 3) + 64 * (r & 7) + 16 * (hh ^ ((r >> 2) & 3));
  const int kb_lane1 = RB * (r >> 3) + 64 * (r & 7) + 16 * ((2 + hh) ^ ((r >> 2) & 3));
  const int vb_lane0 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ hh) + 8 * (tp & 1);
  const int vb_lane1 = 64 * (4 * hh + tq) + 16 * ((2 * tg1 + (tp >> 1)) ^ (2 + hh)) + 8 * (tp & 1);

  // K group g (k-steps 2g, 2g+1 x key halves): dst[2 j + h]
  auto kgroup = [&](uint32_t k0, uint32_t k1, auto gc, bf16x8* dst) {
    constexpr int g = decltype(gc)::value;
    static_for<2>([&](auto jc) {
      constexpr int kk = 2 * g + decltype(jc)::value;
      dst[2 * decltype(jc)::value] = lds_read8_off<512 * (kk >> 1)>((kk & 1) ? k1 : k0);
      dst[2 * decltype(jc)::value + 1] = lds_read8_off<RB * 4 + 512 * (kk >> 1)>((kk & 1) ? k1 : k0);
    });
  };
  // V^T fragment pair i (0 .. NR-1) of 16-key group ks4
  auto vread1 = [&](uint32_t b0, uint32_t b1, auto ks4c, auto ic) -> bf16x4 {
    constexpr int ks4 = decltype(ks4c)::value, i = decltype(ic)::value, dt = i / 2;
    constexpr int R0 = (ks4 >> 1) * 32 + 16 * (ks4 & 1) + 8 * (i & 1);
    return lds_tr_read_off<RB * (R0 >> 3) + 512 * dt>(((R0 >> 3) & 1) ? b1 : b0);
  };
  // S^T of tile t, MFMAs in order (no fillers); all K fragments read up front (no read into a register an
  // in-flight asm MFMA may still be reading)
  auto qk_plain = [&](int t, f32x16 (&s)[2][2]) {
    const char* Kb = KBUF(t % NSLOT);
    const uint32_t k0 = lds_addr(Kb) + kb_lane0, k1 = lds_addr(Kb) + kb_lane1;
    bf16x8 kf[NG][4];
    static_for<NG>([&](auto gc) { kgroup(k0, k1, gc, kf[decltype(gc)::value]); });
    static_for<NG>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      wait_rows4<4 * (NG - 1 - g)>(kf[g]);
      static_for<8>([&](auto wc) {
        constexpr int w = decltype(wc)::value, kk = 2 * g + w / 4, rb = (w / 2) & 1, h = w & 1;
        if constexpr (kk == 0) s_mfma0<QB(rb, 0)>(s[rb][h], kf[g][2 * (w / 4) + h]);
        else s_mfma<QB(rb, kk)>(s[rb][h], kf[g][2 * (w / 4) + h]);
      });
    });
  };
  auto s_fence = [&](f32x16 (&sx)[2][2]) {  // 18 wait states, and hipcc's reads of S below this point
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(sx[0][0]), "+v"(sx[0][1]), "+v"(sx[1][0]), "+v"(sx[1][1]));
  };
  auto mask = [&](int t, f32x16 (&s)[2][2]) {
    const int kv0 = t * BN;
    if (causal && kv0 + BN - 1 > q0w) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int d = kv0 + 4 * hh - (q0w + 32 * rb + r);  // key - query of register 0
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int cj = (j & 3) + 8 * (j >> 2);
          if (d + cj > 0) s[rb][0][j] = -INFINITY;
          if (d + cj + 32 > 0) s[rb][1][j] = -INFINITY;
        }
      }
    }
  };
  // rescale decision at a new tile's row maxima (scaled), one wave-uniform branch for both row blocks
  auto decide = [&](float mt0, float mt1) {
    if (__any(mt0 > m[0] + 8.f || mt1 > m[1] + 8.f)) {
      o_fence();
      const float mt[2] = {mt0, mt1};
      static_for<2>([&](auto rbc) {
        constexpr int rb = decltype(rbc)::value;
        const float mnew = fmaxf(m[rb], mt[rb]);
        const float alpha = __builtin_amdgcn_exp2f(m[rb] - mnew);
        m[rb] = mnew;
        l[rb] *= alpha;
        static_for<4 * DT>([&](auto ic) { o_scale4<OB(rb, 0) + 4 * decltype(ic)::value>(alpha); });
      });
    }
  };
  auto rowmax = [&](const f32x16 (&s)[2][2], int rb) { return half_swap_max(max32(s[rb][0], s[rb][1])) * scale_log2; };
  // exponentials + row sums + P^T packs of S(t), then O^T += V^T . P^T (no fillers)
  auto softmax_pv_plain = [&](int t, f32x16 (&s)[2][2]) {
    bf16x8 pf[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s[rb][0][j] = __builtin_amdgcn_exp2f(fmaf(s[rb][0][j], scale_log2, -m[rb]));
        s[rb][1][j] = __builtin_amdgcn_exp2f(fmaf(s[rb][1][j], scale_log2, -m[rb]));
      }
      l[rb] += sum32(s[rb][0], s[rb][1]);
      pf[rb][0] = pack_acc8(s[rb][0], 0);
      pf[rb][1] = pack_acc8(s[rb][0], 1);
      pf[rb][2] = pack_acc8(s[rb][1], 0);
      pf[rb][3] = pack_acc8(s[rb][1], 1);
    }
    const char* Vb = VBUF(t % NSLOT);
    const uint32_t b0 = lds_addr(Vb) + vb_lane0, b1 = lds_addr(Vb) + vb_lane1;
    static_for<4>([&](auto ks4c) {
      bf16x4 tv[NR];
      static_for<NR>([&](auto ic) { tv[decltype(ic)::value] = vread1(b0, b1, ks4c, ic); });
      wait_tr<NR, 0>(tv);
      static_for<8>([&](auto wc) {
        constexpr int w = decltype(wc)::value, dt = w / 2, rb = w & 1;
        o_mfma<OB(rb, dt)>(cat44(tv[2 * dt], tv[2 * dt + 1]), pf[rb][decltype(ks4c)::value]);
      });
    });
  };
  auto act = [&](int t) { return t < ntiles && (!causal || t * BN <= q0w + 63); };
  auto diag = [&](int t) { return causal && t * BN + BN - 1 > q0w; };

#ifdef KOP_FWD4_STAMP
  unsigned long long st_seg[4] = {0, 0, 0, 0};  // preamble, QK half, PV half, decide (per scheduled tile, summed)
#endif
  // ---- the scheduled tile: S(t+1) MFMAs + softmax of S(t) + P(t).V MFMAs + row max of S(t+1) ----
  auto sched = [&](int t, f32x16 (&cs)[2][2], f32x16 (&ns)[2][2]) {
    const char* Kb = KBUF((t + 1) % NSLOT);
    const uint32_t k0 = lds_addr(Kb) + kb_lane0, k1 = lds_addr(Kb) + kb_lane1;
    const char* Vb = VBUF(t % NSLOT);
    const uint32_t b0 = lds_addr(Vb) + vb_lane0, b1 = lds_addr(Vb) + vb_lane1;
    bf16x8 kbuf[2][4];
    bf16x4 vbuf[2][NR];
    bf16x8 pf[2][4];
    float lsum[2] = {0.f, 0.f};
    const char* dsrc = nullptr;
#ifdef KOP_FWD4_STAMP
    const unsigned long long sp0 = stamp_now();
    unsigned long long sp1 = 0, sp2 = 0;
#endif
    float mx[2];
    const float nm0 = -m[0], nm1 = -m[1];
    const int t2src = t + AHEAD < ntiles ? t + AHEAD : ntiles - 1, t2slot = (t + AHEAD) % NSLOT;
    // the softmax of S(t) and the row max of S(t+1) placed in slot s (-1: preamble)
    auto fillers = [&](auto sc) {
      constexpr int s = decltype(sc)::value;
      static_for<64>([&](auto ec) {
        constexpr int e = decltype(ec)::value, rb = e_rb(e), h = e_h(e), j = e_j(e);
        if constexpr (fma_slot(e) == s) cs[rb][h][j] = fmaf(cs[rb][h][j], scale_log2, rb ? nm1 : nm0);
        if constexpr (exp_slot(e) == s) cs[rb][h][j] = __builtin_amdgcn_exp2f(cs[rb][h][j]);
        if constexpr (add_slot(e) == s) lsum[rb] += cs[rb][h][j];
        if constexpr (e_last(e) && pack_slot(e) == s) pf[rb][2 * h + j / 8] = pack_acc8(cs[rb][h], j / 8);
      });
      if constexpr (s >= 40) {
        static_for<32>([&](auto xc) {
          constexpr int x = decltype(xc)::value, rb = x & 1, j = x >> 1;
          if constexpr (x_slot(x) == s) {
            if constexpr (j == 0) mx[rb] = max3n(ns[rb][0][0], ns[rb][1][0], ns[rb][0][1]);
            else if constexpr (j == 1) mx[rb] = max3n(mx[rb], ns[rb][1][1], ns[rb][0][2]);
            else if constexpr (j < 15) mx[rb] = max3n(mx[rb], ns[rb][1][j], ns[rb][0][j + 1]);
            else mx[rb] = fmaxf(mx[rb], ns[rb][1][15]);
          }
        });
      }
    };
    kgroup(k0, k1, std::integral_constant<int, 0>{}, kbuf[0]);
    kgroup(k0, k1, std::integral_constant<int, 1>{}, kbuf[1]);
    fillers(std::integral_constant<int, -1>{});
    __builtin_amdgcn_sched_barrier(0);
    static_for<64>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      // ---- the slot's MFMA ----
      if constexpr (s < 32) {
        constexpr int g = s / 8, w = s % 8, kk = 2 * g + w / 4, rb = (w / 2) & 1, h = w & 1;
        if constexpr (w == 0) {  // group g landed (group 1 / the first V^T reads may still be in flight)
          if constexpr (g == 0 || g == 3) wait_rows4<4>(kbuf[g & 1]);
          else wait_rows4<0>(kbuf[g & 1]);
        }
#ifdef KOP_FWD4_STAMP
        if constexpr (s == 0) sp1 = stamp_now();
#endif
        if constexpr (kk == 0) s_mfma0<QB(rb, 0)>(ns[rb][h], kbuf[g & 1][2 * (w / 4) + h]);
        else s_mfma<QB(rb, kk)>(ns[rb][h], kbuf[g & 1][2 * (w / 4) + h]);
        // group g+2 into group g's buffer, one MFMA after group g's last read of it (slot 8(g+1))
        if constexpr (w == 0 && g >= 1 && g + 1 < NG) kgroup(k0, k1, std::integral_constant<int, g + 1>{}, kbuf[(g + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        constexpr int ks4 = (s - 32) / 8, w = (s - 32) % 8, dt = w / 2, rb = w & 1;
        if constexpr (w == 0) wait_tr<NR, 0>(vbuf[ks4 & 1]);
#ifdef KOP_FWD4_STAMP
        if constexpr (s == 32) sp2 = stamp_now();
#endif
        // pf[rb][ks4] was packed >= 1 slot (>= 1 MFMA) earlier except pf[1][3] (pack_slot 56, first use 57)
        o_mfma<OB(rb, dt), KOP_FWD4_PVNOP || (ks4 == 3 && rb == 1 && dt == 0)>(
            cat44(vbuf[ks4 & 1][2 * dt], vbuf[ks4 & 1][2 * dt + 1]), pf[rb][ks4]);
      }
      __builtin_amdgcn_sched_barrier(0);  // the MFMA opens its slot: its issue separates the slots' fillers
      // ---- fillers ----
      // V^T fragments: group 0 in slots 28-31 (two per slot), group ks4+1 during group ks4 (one per slot)
      if constexpr (s >= 20 && s < 28) {
        vbuf[0][s - 20] = vread1(b0, b1, std::integral_constant<int, 0>{}, std::integral_constant<int, s - 20>{});
      }
      if constexpr (s >= 32 && s < 56 && (s - 32) % 8 < 4) {
        constexpr int ks4 = (s - 32) / 8;
        static_for<2>([&](auto ic) {
          constexpr int i = 2 * ((s - 32) % 8) + decltype(ic)::value;
          vbuf[(ks4 + 1) & 1][i] = vread1(b0, b1, std::integral_constant<int, ks4 + 1>{}, std::integral_constant<int, i>{});
        });
      }
      // LDS-DMA of tile t+AHEAD: 8 pieces in slots 2, 5, ..., 23. Branch-free: past the last tile the last tile
      // is fetched again into a dead slot (tile t-1's), the loop's exit drains it
      // (address one slot ahead: the DMA would otherwise wait on its own address arithmetic)
      if constexpr (s >= 1 && s <= 22 && (s - 1) % 3 == 0) dsrc = piece_src(t2src, (s - 1) / 3);
      if constexpr (s >= 2 && s <= 23 && (s - 2) % 3 == 0) glds16(dsrc, piece_dst(t2slot, (s - 2) / 3));
      fillers(sc);
      if constexpr (s == 62) {
        mx[0] = half_swap_max(mx[0]) * scale_log2;
        mx[1] = half_swap_max(mx[1]) * scale_log2;
      }
      if constexpr ((s + 1) % KOP_FWD4_SBG == 0) __builtin_amdgcn_sched_barrier(0);
    });
    l[0] += lsum[0];
    l[1] += lsum[1];
#ifdef KOP_FWD4_STAMP
    const unsigned long long sp3 = stamp_now();
#endif
    decide(mx[0], mx[1]);
#ifdef KOP_FWD4_STAMP
    const unsigned long long sp4 = stamp_now();
    st_seg[0] += sp1 - sp0;
    st_seg[1] += sp2 - sp1;
    st_seg[2] += sp3 - sp2;
    st_seg[3] += sp4 - sp3;
#endif
  };

  f32x16 sa[2][2], sb[2][2];
  // Q and tile 0 landed, tiles 1 .. AHEAD-1 in flight
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW * (AHEAD - 1)) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (act(0)) {
    qk_plain(0, sa);
    s_fence(sa);
    mask(0, sa);
    decide(rowmax(sa, 0), rowmax(sa, 1));
  }
#ifdef KOP_FWD4_STAMP
  unsigned long long st_wait = 0, st_sched = 0, st_plain = 0, n_sched = 0, n_plain = 0;
  KOP_STAMP(t_begin);
#endif
  auto step = [&](int it, f32x16 (&cs)[2][2], f32x16 (&ns)[2][2]) {
    KOP_STAMP(t0);
    // K(it+1) is read this trip: its DMA landed, the AHEAD-2 later tiles' may still fly (every trip issues exactly
    // one tile's pieces, clamped past the end, so the count holds)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW * (AHEAD - 2)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    KOP_STAMP(t1);
#ifdef KOP_FWD4_STAMP
    st_wait += t1 - t0;
#endif
    if (act(it + 1) && !diag(it + 1)) {
      sched(it, cs, ns);
#ifdef KOP_FWD4_STAMP
      st_sched += stamp_now() - t1;
      ++n_sched;
#endif
    } else {
#ifdef KOP_FWD4_STAMP
      ++n_plain;
#endif
      for (int i = 0; i < 2 * PPW; ++i)
        piece_at(it + AHEAD < ntiles ? it + AHEAD : ntiles - 1, (it + AHEAD) % NSLOT, i);
      if (act(it + 1)) {
        qk_plain(it + 1, ns);
        softmax_pv_plain(it, cs);
        s_fence(ns);
        mask(it + 1, ns);
        decide(rowmax(ns, 0), rowmax(ns, 1));
      } else if (act(it)) {
        softmax_pv_plain(it, cs);
      }
#ifdef KOP_FWD4_STAMP
      st_plain += stamp_now() - t1;
#endif
    }
    asm volatile("" ::: "memory");
  };
#ifndef KOP_FWD4_UNROLL
  // one tile per trip; the score tiles swap names through a copy
  for (int it = 0; it < ntiles; ++it) {
    step(it, sa, sb);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      sa[rb][0] = sb[rb][0];
      sa[rb][1] = sb[rb][1];
    }
  }
#else
  // two tiles per trip, the score tiles alternating roles (no copies)
  int it = 0;
  for (; it + 1 < ntiles; it += 2) {
    step(it, sa, sb);
    step(it + 1, sb, sa);
  }
  if (it < ntiles) step(it, sa, sb);
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped DMA past the last tile
#undef KBUF
#undef VBUF
#ifdef KOP_FWD4_STAMP
  KOP_STAMP(t_loop);
#endif

  o_fence();
  const int64_t T = (int64_t)B * S;
  static_for<2>([&](auto rbc) {
    constexpr int rb = decltype(rbc)::value;
    const int row = q0w + 32 * rb + r;
    const float lt = l[rb] + __shfl_xor(l[rb], 32, 64);
    const float inv = 1.f / lt;
    if (hh == 0) lse[((int64_t)(b * Hq + hq)) * S + row] = (m[rb] + __log2f(lt)) * 0.69314718056f;
    bf16_t* op = o + (int64_t)(b * S + row) * os + hq * D + 8 * hh;
    bf16_t* otp = ot ? ot + (int64_t)(hq * D + 4 * hh) * T + (int64_t)b * S + row : nullptr;
    static_for<DT>([&](auto dtc) {
      constexpr int dt = decltype(dtc)::value;
      float x[16];
      static_for<16>([&](auto ic) {
        x[decltype(ic)::value] = o_read(std::integral_constant<int, OB(rb, dt) + decltype(ic)::value>{}) * inv;
      });
      if (otp != nullptr) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) otp[(int64_t)(dt * 32 + 8 * g + i) * T] = f2bf(x[4 * g + i]);
      }
      // widened store tail (guide T21), as the 8-wave kernel
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int g0 = 2 * pr, g1 = 2 * pr + 1;
        const uint32_t a0 = pack2(x[4 * g0], x[4 * g0 + 1]), a1 = pack2(x[4 * g0 + 2], x[4 * g0 + 3]);
        const uint32_t c0 = pack2(x[4 * g1], x[4 * g1 + 1]), c1 = pack2(x[4 * g1 + 2], x[4 * g1 + 3]);
        const auto s0 = __builtin_amdgcn_permlane32_swap(a0, c0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(a1, c1, false, false);
        *reinterpret_cast<u32x4*>(op + dt * 32 + 16 * pr) = u32x4{s0[0], s1[0], s0[1], s1[1]};
      }
    });
  });
#ifdef KOP_FWD4_STAMP
  KOP_STAMP(t_end);
  if (lane == 0) {
    atomicAdd(&g_fwd4_stamp[0], st_wait);
    atomicAdd(&g_fwd4_stamp[1], st_sched);
    atomicAdd(&g_fwd4_stamp[2], st_plain);
    atomicAdd(&g_fwd4_stamp[3], n_sched);
    atomicAdd(&g_fwd4_stamp[4], n_plain);
    atomicAdd(&g_fwd4_stamp[5], t_loop - t_begin);
    atomicAdd(&g_fwd4_stamp[6], t_end - t_loop);
    atomicAdd(&g_fwd4_stamp[7], 1ull);
    for (int i = 0; i < 4; ++i) atomicAdd(&g_fwd4_stamp[8 + i], st_seg[i]);
  }
#endif
}

int flash_attn_fwd4x64(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                       int Hkv, int Dh, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                       hipStream_t stream, bf16_t* ot) {
  if (S % BM != 0 || Hq % Hkv != 0 || Dh != D) return -1;
  const size_t lds = NSLOT * 2 * TILE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_fwd4x64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int grid = B * Hq * (S / BM);
  fa_fwd4x64_kernel<<<grid, 256, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, ot);
  return 0;
}

}  // namespace kop
