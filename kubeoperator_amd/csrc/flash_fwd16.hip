// Flash attention FORWARD on 16x16x32 MFMAs (gfx950 / MI355X), KOP_FWD_VARIANT=16, D = 64 / 128.
//
// Same workgroup shape and K/V pipeline as the 8-wave kernel (flash_fwd.hip fa_fwd8_kernel: 8 waves x 32 query rows,
// 64-key tiles by LDS-DMA through a 3-slot ring, one barrier per tile), with both products on
// v_mfma_f32_16x16x32_bf16 instead of 32x32x16. Under the power cap the smaller MFMA shape delivers more FLOP/s
// per watt (MI355X_MICROARCH.md: ~1.15x in sustained bf16 loops on random data), and the attention kernels run
// power-held at 1.8-2.0 GHz (profiles/r5_attn_pmc_summary_normalized.txt). Layouts (16x16x32: lane l holds
// A[row l&15][k 8(l>>4)..+7], B[k 8(l>>4)..+7][col l&15], C[row 4(l>>4)+r][col l&15]):
//   * S^T [16 keys x 16 queries] = K . Q^T per key block b (4 per tile) and query block qq (2 per wave): the
//     16 K rows of block b are keys 32(b>>1) + 8(i>>2) + 4(b&1) + (i&3), so a lane's S^T values of blocks 2c and
//     2c+1 are its query's keys 32c + 8(l>>4) .. +7 -- the P^T operand of the P.V product for key block c, packed
//     in place (no lane exchange);
//   * O^T [16 dims x 16 queries] += V^T . P^T per dim block e: V^T by ds_read_b64_tr_b16 from the V image;
//   * a query's softmax state lives in the 4 lanes {col, col+16, col+32, col+48}: the row max is two shuffles,
//     the row sum stays per lane until the epilogue; the O^T accumulator of a query is in the same lanes, so
//     the rescale is lane-local.
// K and V images: [64 rows][ROWB] with each row's 16-B chunks XOR-permuted by the row (the DMA source chunk is
// permuted, the destination stays lane-linear) so a K row read (16 rows, one chunk) and a V transposed read
// (8 rows x 2 chunks per 32-lane half) hit 64 distinct banks.
#include <cstdlib>

#include "attn_common.h"
#include "kernels.h"

namespace kop {
namespace fwd16 {

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int ROWB>
__device__ __forceinline__ int kx(int r) {  // K image chunk XOR: rows 8a + 4bb + c, a, c in 0..3 -> 16 slots
  if constexpr (ROWB == 256) return (r & 3) | (((r >> 3) & 3) << 2);
  else return ((r >> 1) & 1) | (((r >> 3) & 3) << 1);
}
template <int ROWB>
__device__ __forceinline__ int vx(int r) {  // V image chunk XOR (even): rows 8g + 4h + q of a 32-lane half
  if constexpr (ROWB == 256) return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
  else return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}
// LDS-DMA of a [ROWS][ROWB] image, 1-KiB pieces over NW waves, lane l of piece p -> row RPP p + l / SLOTS, slot
// l % SLOTS, holding source chunk slot ^ X(row)
template <int ROWB, int NW, int ROWS, bool ISK>
__device__ __forceinline__ void dma_img(char* lds, const bf16_t* src, int64_t rs, int wid, int lane) {
  constexpr int SLOTS = ROWB / 16, RPP = 1024 / ROWB, PIECES = ROWS * ROWB / 1024;
  static_assert(PIECES % NW == 0, "tile pieces must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < PIECES / NW; ++i) {
    const int piece = wid + i * NW;
    const int row = RPP * piece + lane / SLOTS, slot = lane % SLOTS;
    const int ch = slot ^ (ISK ? kx<ROWB>(row) : vx<ROWB>(row));
    glds16(src + (int64_t)row * rs + ch * 8, lds + piece * 1024);
  }
}
template <int CNT>
__device__ __forceinline__ void wait_k4(bf16x8* t) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(CNT));
}

}  // namespace fwd16

// VD: V^T dim blocks read ahead of the P.V MFMAs (KOP_FWD16_VD, A/B)
template <int D, int VD0>
__global__ void __launch_bounds__(512, 1) fa_fwd16_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                          const bf16_t* __restrict__ v, bf16_t* __restrict__ o,
                                                          float* __restrict__ lse, int B, int S, int Hq, int Hkv,
                                                          int64_t qs, int64_t ks, int64_t vs, int64_t os,
                                                          float scale_log2, int causal, bf16_t* __restrict__ ot) {
  using namespace fwd16;
  constexpr int NW = 8, BM = 256, BN = 64, ROWB = D * 2, TILE = BN * ROWB, NSLOT = 3;
  constexpr int NS = D / 32;  // k-steps of S (32 dims each)
  constexpr int NE = D / 16;  // 16-dim output blocks
  constexpr int PPW = (TILE / 1024) / NW;
  static_assert(PPW >= 1, "tile must give every wave a DMA piece");
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define KBUF(sl) (smem + (sl) * 2 * TILE)
#define VBUF(sl) (smem + (sl) * 2 * TILE + TILE)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int nqb = S / BM;
  const AttnWork aw = attn_work(blockIdx.x, B, Hq, Hq / Hkv, nqb);
  const int qb = causal ? (nqb - 1 - aw.rank) : aw.rank;
  const int b = aw.b, hq = aw.unit;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int ntiles = causal ? (q0 + BM) / BN : S / BN;
  const bf16_t* kbase = k + (int64_t)(b * S) * ks + kvh * D;
  const bf16_t* vbase = v + (int64_t)(b * S) * vs + kvh * D;
  auto issue = [&](int t) {
    const int sl = t % NSLOT;
    dma_img<ROWB, NW, BN, true>(KBUF(sl), kbase + (int64_t)(t * BN) * ks, ks, wid, lane);
    dma_img<ROWB, NW, BN, false>(VBUF(sl), vbase + (int64_t)(t * BN) * vs, vs, wid, lane);
  };
  issue(0);
  if (ntiles > 1) issue(1);

  // Q^T B operand: query q0w + 16 qq + col, dims 32 s + 8 g
  bf16x8 qf[2][NS];
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) {
    const bf16_t* qp = q + (int64_t)(b * S + q0w + 16 * qq + col) * qs + hq * D + 8 * g;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[qq][s] = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
  }
#pragma unroll
  for (int qq = 0; qq < 2; ++qq)
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(qf[qq][s]));
  f32x4 oacc[2][NE];
#pragma unroll
  for (int qq = 0; qq < 2; ++qq)
#pragma unroll
    for (int e = 0; e < NE; ++e) oacc[qq][e] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  // K row read of k-step s, key block b2: row 32(b2>>1) + 4(b2&1) + krow, logical chunk 4s + g
  const int krow = 8 * (col >> 2) + (col & 3);
  const int kxl = kx<ROWB>(krow);  // the XOR of every row this lane reads (rows differ in bits 2 and 5 only)
  int koff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = krow * ROWB + 16 * ((4 * s + g) ^ kxl);
  // V^T transposed read of dim block e, key block c, half h: row 32c + 8g + 4h + tq, logical chunk 2e + (tp>>1)
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const int vrow = 8 * g + tq;
  const int vxl = vx<ROWB>(vrow) >> 1;
  int voff[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) voff[e] = vrow * ROWB + 16 * (2 * (e ^ vxl) + (tp >> 1)) + 8 * (tp & 1);

  auto tile = [&](int t) {
    const uint32_t kb = lds_addr(KBUF(t % NSLOT)), vb = lds_addr(VBUF(t % NSLOT));
    // ---- S^T: sc[qq][b2], two k-steps of K fragments in flight
    f32x4 sc[2][4];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq)
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2) sc[qq][b2] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 kf[2][4];
    auto kread = [&](auto sc_, bf16x8* dst) {
      constexpr int s = decltype(sc_)::value;
      const uint32_t a = kb + koff[s];
      dst[0] = lds_read8_off<0>(a);
      dst[1] = lds_read8_off<4 * ROWB>(a);
      dst[2] = lds_read8_off<32 * ROWB>(a);
      dst[3] = lds_read8_off<36 * ROWB>(a);
    };
    kread(std::integral_constant<int, 0>{}, kf[0]);
    if constexpr (NS > 1) kread(std::integral_constant<int, 1>{}, kf[1]);
    static_for<NS>([&](auto sc_) {
      constexpr int s = decltype(sc_)::value;
      bf16x8* cur = kf[s & 1];
      if constexpr (s + 1 < NS) wait_k4<4>(cur);
      else wait_k4<0>(cur);
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2)
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) sc[qq][b2] = mfma16(cur[b2], qf[qq][s], sc[qq][b2]);
      if constexpr (s + 2 < NS) kread(std::integral_constant<int, s + 2>{}, cur);
    });
    const int kv0 = t * BN;
    if (causal && kv0 + BN - 1 > q0w) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int qi = q0w + 16 * qq + col;
#pragma unroll
        for (int b2 = 0; b2 < 4; ++b2)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kv0 + 32 * (b2 >> 1) + 8 * g + 4 * (b2 & 1) + r > qi) sc[qq][b2][r] = -INFINITY;
      }
    }
    // ---- online softmax per query block (one rescale test for both); P^T operands of key blocks c = 0, 1
    float mt[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      float mx = max3f(sc[qq][0][0], sc[qq][0][1], sc[qq][0][2]);
      mx = max3f(mx, sc[qq][0][3], sc[qq][1][0]);
      mx = max3f(mx, sc[qq][1][1], sc[qq][1][2]);
      mx = max3f(mx, sc[qq][1][3], sc[qq][2][0]);
      mx = max3f(mx, sc[qq][2][1], sc[qq][2][2]);
      mx = max3f(mx, sc[qq][2][3], sc[qq][3][0]);
      mx = max3f(mx, sc[qq][3][1], sc[qq][3][2]);
      mx = fmaxf(mx, sc[qq][3][3]);
      mt[qq] = xor32_max(xor16_max(mx)) * scale_log2;
    }
    if (__any(mt[0] > m[0] + 8.f || mt[1] > m[1] + 8.f)) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const float mnew = fmaxf(m[qq], mt[qq]);
        const float alpha = __builtin_amdgcn_exp2f(m[qq] - mnew);
        m[qq] = mnew;
        l[qq] *= alpha;
#pragma unroll
        for (int e = 0; e < NE; ++e) oacc[qq][e] *= alpha;
      }
    }
    bf16x8 pf[2][2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      float ls = 0.f;
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sc[qq][b2][r] = __builtin_amdgcn_exp2f(fmaf(sc[qq][b2][r], scale_log2, -m[qq]));
          ls += sc[qq][b2][r];
        }
      l[qq] += ls;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const u32x4 w = {pack2(sc[qq][2 * c][0], sc[qq][2 * c][1]), pack2(sc[qq][2 * c][2], sc[qq][2 * c][3]),
                         pack2(sc[qq][2 * c + 1][0], sc[qq][2 * c + 1][1]),
                         pack2(sc[qq][2 * c + 1][2], sc[qq][2 * c + 1][3])};
        pf[qq][c] = __builtin_bit_cast(bf16x8, w);
      }
    }
    // ---- O^T += V^T . P^T: per dim block e the 4 transposed reads of key blocks 0 / 1, VD blocks in flight ahead
    constexpr int VD = VD0 < NE ? VD0 : NE;
    bf16x4 tr[VD + 1][4];
    auto vread = [&](auto ec, bf16x4* dst) {
      constexpr int e = decltype(ec)::value;
      const uint32_t a = vb + voff[e];
      dst[0] = lds_tr_read_off<0>(a);
      dst[1] = lds_tr_read_off<4 * ROWB>(a);
      dst[2] = lds_tr_read_off<32 * ROWB>(a);
      dst[3] = lds_tr_read_off<36 * ROWB>(a);
    };
    static_for<VD>([&](auto ec) { vread(ec, tr[decltype(ec)::value]); });
    static_for<NE>([&](auto ec) {
      constexpr int e = decltype(ec)::value;
      bf16x4* cur = tr[e % (VD + 1)];
      if constexpr (e + VD < NE) vread(std::integral_constant<int, e + VD>{}, tr[(e + VD) % (VD + 1)]);
      constexpr int younger = 4 * ((NE - 1 - e) < VD ? (NE - 1 - e) : VD);
      wait_tr<4, younger>(cur);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16x8 vf = cat44(cur[2 * c], cur[2 * c + 1]);
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) oacc[qq][e] = mfma16(vf, pf[qq][c], oacc[qq][e]);
      }
    });
  };

  for (int it = 0; it < ntiles; ++it) {
    if (it + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + 2 < ntiles) issue(it + 2);
    if (!causal || it * BN <= q0w + 31) tile(it);
    asm volatile("" ::: "memory");
  }
#undef KBUF
#undef VBUF

  const int64_t T = (int64_t)B * S;
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) {
    const float lt = xor32_sum(xor16_sum(l[qq]));
    const float inv = 1.f / lt;
    const int qi = q0w + 16 * qq + col;
    if (g == 0) lse[((int64_t)(b * Hq + hq)) * S + qi] = (m[qq] + __log2f(lt)) * 0.69314718056f;
    bf16_t* op = o + (int64_t)(b * S + qi) * os + hq * D + 4 * g;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const f32x4 a = oacc[qq][e] * inv;
      *reinterpret_cast<u32x2*>(op + 16 * e) = u32x2{pack2(a[0], a[1]), pack2(a[2], a[3])};
      if (ot != nullptr) {
        // O^T [Hq*D, B*S]: dims 16e + 4g + r of token qi (16 consecutive tokens per store = 32 B)
        bf16_t* otp = ot + (int64_t)(hq * D + 16 * e + 4 * g) * T + (int64_t)b * S + qi;
#pragma unroll
        for (int r = 0; r < 4; ++r) otp[(int64_t)r * T] = f2bf(a[r]);
      }
    }
  }
}

template <int D, int VD>
static void launch_fwd16(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                         int Hkv, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                         hipStream_t stream, bf16_t* ot) {
  constexpr size_t lds = 3 * 2 * 64 * (D * 2);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fa_fwd16_kernel<D, VD>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  fa_fwd16_kernel<D, VD><<<B * Hq * (S / 256), 512, lds, stream>>>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2,
                                                                  causal ? 1 : 0, ot);
}

int flash_attn_fwd16(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                     int Hkv, int D, int64_t qs, int64_t ks, int64_t vs, int64_t os, float sl2, bool causal,
                     hipStream_t stream, bf16_t* ot) {
  if (S % 256 != 0 || Hq % Hkv != 0 || (D != 64 && D != 128)) return -1;
  // V^T read-ahead depth 2 (depths 1-3 measured within 1 % of each other: profiles/r5_fwd16_vdepth_ab.jsonl)
  if (D == 128) launch_fwd16<128, 2>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
  else launch_fwd16<64, 2>(q, k, v, o, lse, B, S, Hq, Hkv, qs, ks, vs, os, sl2, causal, stream, ot);
  return 0;
}

}  // namespace kop
