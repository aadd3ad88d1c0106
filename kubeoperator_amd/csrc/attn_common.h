// Shared device helpers of the flash-attention kernels (gfx950): MFMA wrapper, LDS row / transposed reads,
// the swizzled LDS tile image, LDS-DMA issue and the XCD-aware block remap.
#pragma once
#include <type_traits>
#include <utility>

#include "common.h"

namespace kop {
// compile-time loop: f(std::integral_constant<int, i>{}) for i = 0 .. N-1 (indices usable as template args)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

__device__ __forceinline__ bf16x4 lds_tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(p));
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)(p));
}
// Transposed read hidden from hipcc's memory model: the builtin form makes hipcc drain every in-flight
// LDS-DMA (vmcnt(0)) before it. The caller retires these with lds_wait_tr() before the first consumer.
__device__ __forceinline__ bf16x4 lds_tr_read_asm(const char* p) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr(p)));
  return r;
}
__device__ __forceinline__ bf16x8 lds_read8(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
// Transposed read at a lane base address (VGPR) + compile-time byte offset (the instruction's offset field).
template <int OFF>
__device__ __forceinline__ bf16x4 lds_tr_read_off(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
// Row read (ds_read_b128) at a lane base + immediate, hidden from hipcc's scheduler like the transposed
// reads: hipcc would otherwise fold a prefetch chain into one register quad and wait on every read.
template <int OFF>
__device__ __forceinline__ bf16x8 lds_read8_off(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
template <int CNT>
__device__ __forceinline__ void wait_rows4(bf16x8* t) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(CNT));
}
template <int CNT>
__device__ __forceinline__ void wait_rows3(bf16x8* t) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]) : "n"(CNT));
}
// Retire transposed reads: wait until at most CNT LDS ops are outstanding and tell hipcc the NR fragments
// in t[] are written at that point (they come from inline-asm reads it cannot track).
template <int NR, int CNT>
__device__ __forceinline__ void wait_tr(bf16x4* t) {
  static_assert(NR == 4 || NR == 8, "4 or 8 fragments");
  if constexpr (NR == 8)
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7])
                 : "n"(CNT));
  else
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : "n"(CNT));
}
__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// v_max3_f32 without hipcc's canonicalising v_max on each MFMA result (fmaxf would emit 3 instructions)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float d;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// max / sum over lanes l and l ^ 16 (16-lane rows 0 <-> 1, 2 <-> 3) and l ^ 32 (halves) with v_permlane16/32_swap:
// a register exchange, where __shfl_xor is a ds_bpermute round trip through the LDS pipe (on a softmax's critical
// path: profiles/r5_experiments.md, the 16x16x32 forward)
__device__ __forceinline__ float xor16_max(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float xor16_sum(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
// max over the 32 scores of two accumulators: 16 v_max3
__device__ __forceinline__ float max32(const f32x16& a, const f32x16& b) {
  float m = max3f(a[0], b[0], a[1]);
#pragma unroll
  for (int j = 1; j < 16; ++j) m = max3f(m, a[j], b[j]);
  return m;
}
// sum of the 32 values of two accumulators with packed adds (v_pk_add_f32: two lanes' worth per issue)
__device__ __forceinline__ float sum32(const f32x16& a, const f32x16& b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f2{a[2 * i], a[2 * i + 1]} + f2{b[2 * i], b[2 * i + 1]};
#pragma unroll
  for (int i = 4; i < 8; ++i)
    acc[i & 3] += f2{a[2 * i], a[2 * i + 1]} + f2{b[2 * i], b[2 * i + 1]};
  const f2 s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  return s[0] + s[1];
}
// s = s * c + b over one accumulator with packed FMAs (v_pk_fma_f32: two values per issue, half the VALU
// slots of 16 v_fma_f32 in the softmax's exponent argument)
__device__ __forceinline__ void fma_pk16(f32x16& s, float c, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 c2 = {c, c}, b2 = {b, b};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f2 t = __builtin_elementwise_fma(f2{s[2 * i], s[2 * i + 1]}, c2, b2);
    s[2 * i] = t[0];
    s[2 * i + 1] = t[1];
  }
}
// accumulator registers 8h .. 8h+7 -> one bf16x8 MFMA operand (4 v_cvt_pk_bf16_f32, no sub-word moves)
__device__ __forceinline__ bf16x8 pack_acc8(const f32x16& s, int h) {
  const u32x4 w = {pack2(s[8 * h], s[8 * h + 1]), pack2(s[8 * h + 2], s[8 * h + 3]), pack2(s[8 * h + 4], s[8 * h + 5]),
                   pack2(s[8 * h + 6], s[8 * h + 7])};
  return __builtin_bit_cast(bf16x8, w);
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Byte offset of 16-byte chunk `ch` of row `row` in a swizzled [rows][ROWB bytes] LDS image.
// 256-B rows: chunk ^ (((row&3)<<2)|((row>>2)&3)) serves both ds_read_b128 row reads and
// ds_read_b64_tr_b16 transposed reads (guide T10 image (b)); 128-B rows: chunk ^ ((row>>1)&7).
template <int ROWB>
__device__ __forceinline__ int swz_xor(int row) {
  if constexpr (ROWB == 256) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (row >> 1) & 7;
}
template <int ROWB>
__device__ __forceinline__ int swz(int row, int ch) {
  return row * ROWB + 16 * (ch ^ swz_xor<ROWB>(row));
}

// One 16-B-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at lds_uniform + 16*l.
__device__ __forceinline__ void glds16(const void* g, char* lds_uniform) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_uniform, 16, 0, 0);
}
// The same with the non-temporal policy (cache-policy bits = 2, nt): for bytes one CU reads exactly once
// (MI355X_MICROARCH.md 'nt-weights': no L2 allocation, so the re-read operands keep their lines)
__device__ __forceinline__ void glds16_nt(const void* g, char* lds_uniform) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_uniform, 16, 0, 2);
}

// Fill a swizzled [rows][ROWB] LDS image of `rows` rows by LDS-DMA: pieces of 1 KiB are spread over the
// NW waves of the block; each lane's SOURCE chunk is permuted so the lane-linear destination is the
// swizzled image (guide §5.4 rule 21). Issues (rows*ROWB/1024)/NW DMA instructions per wave.
template <int ROWB, int NW, int ROWS>
__device__ __forceinline__ void dma_tile(char* lds, const bf16_t* src, int64_t row_stride, int wid, int lane) {
  constexpr int SLOTS = ROWB / 16, RPP = 1024 / ROWB;
  constexpr int PIECES = ROWS * ROWB / 1024;
  static_assert(PIECES % NW == 0, "tile pieces must split evenly over the waves");
  const int prow = lane / SLOTS, pslot = lane % SLOTS;
#pragma unroll
  for (int i = 0; i < PIECES / NW; ++i) {
    const int piece = wid + i * NW;
    const int row = piece * RPP + prow;
    const int ch = pslot ^ swz_xor<ROWB>(row);
    glds16(src + (int64_t)row * row_stride + ch * 8, lds + piece * 1024);
  }
}

// Sub-tiled image (guide T10 image (a)): 8-row x 64-byte subtiles of 512 B, XOR-swizzled inside, so
// ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads are both conflict-free AND every read of a
// 32x32x16 operand is one of TWO lane base addresses plus a compile-time immediate (no per-read VALU).
template <int ROWB>
__device__ __forceinline__ int swza(int row, int ch) {
  return (ROWB * 8) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// LDS-DMA fill of a sub-tiled [ROWS][ROWB] image: 1-KiB pieces over NW waves; lane l of piece p lands at
// byte 1024p + 16l, so its SOURCE (row, chunk) is the one the image puts there.
template <int ROWB, int NW, int ROWS>
__device__ __forceinline__ void dma_tile_a(char* lds, const bf16_t* src, int64_t row_stride, int wid, int lane) {
  constexpr int PIECES = ROWS * ROWB / 1024, PPB = ROWB / 128;  // pieces per 8-row block
  static_assert(PIECES % NW == 0, "tile pieces must split evenly over the waves");
  const int lrow = (lane & 31) >> 2, lhi = lane >> 5, lslot = lane & 3;
#pragma unroll
  for (int i = 0; i < PIECES / NW; ++i) {
    const int piece = wid + i * NW;
    const int row = 8 * (piece / PPB) + lrow;
    const int ch = 4 * (2 * (piece % PPB) + lhi) + (lslot ^ ((row >> 2) & 3));
    glds16(src + (int64_t)row * row_stride + ch * 8, lds + piece * 1024);
  }
}

// Work order of the attention kernels: bid -> (batch, head unit, block rank), rank 0 = the HEAVIEST block
// under a causal mask (the kernels map rank to their query / key block). Workgroups are dispatched to the
// 8 XCDs round-robin in bid order (bid & 7), so the order must balance the XCDs as well as the CUs:
//   * when the L2-sharing groups (UG consecutive head units reading one K/V head) split evenly over the
//     XCDs, XCD x runs groups x, x+8, ... -- every XCD gets the same mix of block sizes, its heads share
//     their K/V in its L2, and inside the XCD the blocks go heaviest-first (list scheduling ~ LPT);
//   * otherwise plain bid order, rank-major: consecutive (heavy) blocks land on different XCDs.
// (A contiguous-chunk XCD remap of a rank-major order put all of the heaviest blocks on XCD 0: causal
// attention ran at ~58 % of the non-causal rate, profiles/r2_attn_causal_balance.jsonl.)
struct AttnWork {
  int b, unit, rank;
};
__device__ __forceinline__ AttnWork attn_work(int bid, int B, int NU, int UG, int nblk) {
  (void)nblk;
  UG = UG < 1 ? 1 : UG;
  const int G = (NU % UG == 0) ? B * (NU / UG) : 0;
  if (G > 0 && (G & 7) == 0) {
    const int xcd = bid & 7, s = bid >> 3;
    const int per = (G >> 3) * UG;  // head units per XCD
    const int rank = s / per, rem = s % per;
    const int g = (rem / UG) * 8 + xcd;
    const int gpb = NU / UG;  // groups per batch entry
    return {g / gpb, (g % gpb) * UG + rem % UG, rank};
  }
  const int rank = bid / (B * NU), rem = bid % (B * NU);
  return {rem / NU, rem % NU, rank};
}

// 16-byte LDS read (4 floats) at a lane base + immediate, retired by the caller's counted lgkmcnt
template <int OFF>
__device__ __forceinline__ f32x4 lds_read16f_off(uint32_t base) {
  f32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
__device__ __forceinline__ f32x16 cat4f(const f32x4* q) {
  return f32x16{q[0][0], q[0][1], q[0][2], q[0][3], q[1][0], q[1][1], q[1][2], q[1][3],
                q[2][0], q[2][1], q[2][2], q[2][3], q[3][0], q[3][1], q[3][2], q[3][3]};
}

#define KOP_VM_CASE(n) \
  case n:              \
    asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); \
    break;
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (0..15)
__device__ __forceinline__ void vm_wait_le(int n) {
  switch (n) {
    KOP_VM_CASE(0) KOP_VM_CASE(1) KOP_VM_CASE(2) KOP_VM_CASE(3) KOP_VM_CASE(4) KOP_VM_CASE(5) KOP_VM_CASE(6)
    KOP_VM_CASE(7) KOP_VM_CASE(8) KOP_VM_CASE(9) KOP_VM_CASE(10) KOP_VM_CASE(11) KOP_VM_CASE(12) KOP_VM_CASE(13)
    KOP_VM_CASE(14)
    default:
      asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  }
}
#undef KOP_VM_CASE

}  // namespace kop
