// Decode attention for gfx950 (serving): one new query token per sequence against its KV cache, GQA, split-K
// ("flash decoding") so a batch of a few sequences still fills the 256 CUs.
//
//   q      [B, Hq * D]           bf16 rows (row stride qs: the Q columns of the fused QKV projection)
//   cache  K, V [B, Hkv, Smax, D] bf16, keys [0, len[b]) valid: a (sequence, KV head) owns one contiguous
//          [Smax, D] slab, so a workgroup's 256-key chunk is one contiguous 64 KiB stream per tensor
//   o      [B, Hq * D]           bf16
//
// Memory-bound: every step streams the whole live cache (Llama-3-8B, 8k context: 4 MiB of K+V per sequence
// and layer), so the kernels are built around coalesced 16-byte loads and reuse of each K/V row by all
// G = Hq / Hkv query heads of its group.
//
// Pass 1: grid (splits, B * Hkv), 256 threads. A workgroup owns CH = 128 keys of one (sequence, KV head).
// Default: decode_attn_mfma_kernel (both products on 16x16x32 MFMAs, G heads as padded columns; below). The VALU
// form (KOP_DECODE_ATTN=valu):
//   thread t = (key group kg = t / 16, segment sg = t % 16): the 16 threads of a key group read one 256-byte
//   K row (D = 128) as 16 x 16 B -- a wave loads 4 whole rows per instruction -- and each keeps G partial dot
//   products of its 8 dims, summed over the 16 lanes with 4 butterfly shuffles. Scores (already scaled by
//   log2 e / sqrt(D)) go to LDS; the workgroup's max / sum of exp2 per head come from a block reduction;
//   P . V runs with the same (key group, segment) mapping on the V rows (every K and V load of a thread is
//   issued up front); the key groups' [G x D] partial sums are added with butterflies inside each wave, then
//   over the 4 waves in LDS. Output per split: unnormalised acc [G, D], running max m and sum l (fp32).
// Pass 2: grid B * Hq, one wave: o = sum_s acc_s 2^(m_s - M) / sum_s l_s 2^(m_s - M).
#include "attn_common.h"
#include <cstdlib>
#include <string>
#include "kernels.h"

namespace kop {

namespace {
constexpr int kThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1e30f;
}  // namespace

// CH keys per workgroup (one split): 256 (16 K + 16 V row segments in flight per thread, ~180 VGPRs, two
// workgroups per CU) or 128 (8 + 8, more workgroups per CU to overlap one's softmax with another's loads)
template <int D, int G, int CH>
__global__ void __launch_bounds__(kThreads) decode_attn_split_kernel(
    const bf16_t* __restrict__ q, int64_t qs, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ lens, int Smax, int Hkv, float scale_log2, float* __restrict__ part_o,
    float* __restrict__ part_ml, int nsplit) {
  constexpr int SEGS = D / 8;         // 16-byte segments per row (16 at D = 128, 8 at D = 64)
  constexpr int KG = kThreads / SEGS; // key groups (16 / 32)
  constexpr int KPT = CH / KG;        // keys per thread (16 / 8 at CH 256)
  __shared__ float s_p[G][CH];        // scores, then probabilities
  __shared__ float s_red[G][kThreads / 64];
  __shared__ f32x4 s_acc[kThreads / 64][G][D / 4];
  const int split = blockIdx.x;
  const int b = blockIdx.y / Hkv, kvh = blockIdx.y % Hkv;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int kg = t / SEGS, sg = t % SEGS;
  const int len = min(lens[b], Smax);  // never read past the cache, whatever the caller's lengths
  const int k0 = split * CH;
  constexpr int64_t rs = D;  // cache row stride (elements) between consecutive keys of one KV head
  const bf16_t* kbase = kc + ((int64_t)b * Hkv + kvh) * Smax * D + sg * 8;
  const bf16_t* vbase = vc + ((int64_t)b * Hkv + kvh) * Smax * D + sg * 8;
  float* po = part_o + (((int64_t)b * Hkv + kvh) * G * nsplit) * D;  // [G][nsplit][D] for this (b, kvh)
  float* pml = part_ml + (((int64_t)b * Hkv + kvh) * G * nsplit) * 2;
  if (k0 >= len) {  // split past the sequence: an empty partial
    if (t < G) {
      pml[(t * nsplit + split) * 2] = kNegBig;
      pml[(t * nsplit + split) * 2 + 1] = 0.f;
    }
    for (int i = t; i < G * D; i += kThreads) po[((i / D) * nsplit + split) * D + i % D] = 0.f;
    return;
  }
  // this thread's 8 query dims of each head of the group, pre-scaled
  float qv[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    unpack8(*reinterpret_cast<const u32x4*>(q + (int64_t)b * qs + (int64_t)(kvh * G + h) * D + sg * 8), qv[h]);
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[h][i] *= scale_log2;
  }
  // ---- every K and V row segment of this thread in flight at once (V is consumed after the softmax)
  u32x4 kr[KPT], vr[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int key = k0 + kg + KG * j;
    kr[j] = key < len ? *reinterpret_cast<const u32x4*>(kbase + (int64_t)key * rs) : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int key = k0 + kg + KG * j;
    vr[j] = key < len ? *reinterpret_cast<const u32x4*>(vbase + (int64_t)key * rs) : u32x4{0u, 0u, 0u, 0u};
  }
  // ---- scores: key k0 + kg + KG * j
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    float kf[8];
    unpack8(kr[j], kf);
    float d[G];
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) a += qv[h][i] * kf[i];
      d[h] = a;
    }
#pragma unroll
    for (int o = SEGS / 2; o > 0; o >>= 1)
#pragma unroll
      for (int h = 0; h < G; ++h) d[h] += __shfl_xor(d[h], o, 64);
    const int kl = kg + KG * j;
    if (sg < G) {  // lane sg of the key group stores head sg's score (all lanes hold every head's sum)
      float v = 0.f;
#pragma unroll
      for (int h = 0; h < G; ++h) v = (h == sg) ? d[h] : v;
      s_p[sg][kl] = (k0 + kl < len) ? v : kNegBig;
    }
  }
  __syncthreads();
  // ---- per-head max and sum over the CH keys (thread t covers key t of every head; CH <= 256 threads)
  float m[G], l[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float mv = wave_max(t < CH ? s_p[h][t] : kNegBig);
    if (lane == 0) s_red[h][wv] = mv;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float mm = s_red[h][0];
#pragma unroll
    for (int w = 1; w < kThreads / 64; ++w) mm = fmaxf(mm, s_red[h][w]);
    m[h] = mm;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float s = t < CH ? s_p[h][t] : kNegBig;
    const float p = s <= 0.5f * kNegBig ? 0.f : exp2f(s - m[h]);
    if (t < CH) s_p[h][t] = p;
    const float sv = wave_sum(p);
    if (lane == 0) s_red[h][wv] = sv;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float ss = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) ss += s_red[h][w];
    l[h] = ss;
  }
  // ---- P . V with the score mapping: this thread's 8 dims of keys kg + KG * j
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    float vf[8];
    unpack8(vr[j], vf);
    const int kl = kg + KG * j;
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float p = s_p[h][kl];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] += p * vf[i];
    }
  }
  // the wave's 64 / SEGS key groups summed with butterflies (same segment = lanes SEGS apart), then the 4 waves in LDS
#pragma unroll
  for (int o = SEGS; o < 64; o <<= 1)
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] += __shfl_xor(acc[h][i], o, 64);
  if (lane < SEGS) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      s_acc[wv][h][2 * sg] = f32x4{acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
      s_acc[wv][h][2 * sg + 1] = f32x4{acc[h][4], acc[h][5], acc[h][6], acc[h][7]};
    }
  }
  __syncthreads();
  // ---- write the split's partials
  for (int i = t; i < G * D / 4; i += kThreads) {
    const int h = i / (D / 4), c = i % (D / 4);
    f32x4 s = s_acc[0][h][c];
#pragma unroll
    for (int w = 1; w < kThreads / 64; ++w) s += s_acc[w][h][c];
    reinterpret_cast<f32x4*>(po + ((int64_t)h * nsplit + split) * D)[c] = s;
  }
  if (t < G) {  // register arrays are not indexed by a runtime value (that would go through scratch)
    float mt = 0.f, lt = 0.f;
#pragma unroll
    for (int h = 0; h < G; ++h) {
      mt = (h == t) ? m[h] : mt;
      lt = (h == t) ? l[h] : lt;
    }
    pml[(t * nsplit + split) * 2] = mt;
    pml[(t * nsplit + split) * 2 + 1] = lt;
  }
}

// ---------------------------------------------------------------------------------------------------------
// Pass 1 on the matrix cores (default; KOP_DECODE_ATTN=valu selects the kernel above). The VALU form spends
// its time on the per-key 16-lane butterflies of the scores and on the P . V FMAs, not on HBM: 3.9 TB/s at
// batch 64 x 2k context (profiles/r5_experiments.md). Here each of the 4 waves owns 32 of the workgroup's 128
// keys and both products are v_mfma_f32_16x16x32_bf16 with the G query heads as 16 padded columns:
//   * S^T [16 keys x 16 heads] = K . Q^T: the A operand (lane l: key row, 8 dims) is one 16-byte load straight
//     from the cache row; the 16 key rows of block b are keys 8(i >> 2) + 4b + (i & 3), so that lane l ends up
//     holding its head (l & 15)'s scores of keys 8(l >> 4) .. +7 -- exactly the B operand P^T of the P . V
//     product, with no lane exchange;
//   * O^T [16 dims x 16 heads] += V^T . P^T: V^T comes from an LDS image of the wave's 32 V rows (LDS-DMA,
//     lane-linear, each lane's source chunk XOR-permuted by the row so the ds_read_b64_tr_b16 transposed reads
//     of a 32-lane half hit 64 distinct banks);
//   * the softmax over the wave's 32 keys is lane-local plus two shuffles; the 4 waves' (m, l, O) meet in LDS
//     once, and the split's partial goes out in the VALU kernel's format (same pass 2).
// ---------------------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int OFF>
__device__ __forceinline__ bf16x4 dec_tr_read(uint32_t base) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
// XOR of a V row's 16-byte chunk slots in the LDS image (row r = 8g + 4h + q of the wave's 32 keys): spreads the
// 8 rows a 32-lane half reads per transposed read over distinct chunk slots
template <int ROWB>
__device__ __forceinline__ int dec_vx(int r) {
  if constexpr (ROWB == 256) return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
  else return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}

template <int D, int G>
__global__ void __launch_bounds__(kThreads) decode_attn_mfma_kernel(
    const bf16_t* __restrict__ q, int64_t qs, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ lens, int Smax, int Hkv, float scale_log2, float* __restrict__ part_o,
    float* __restrict__ part_ml, int nsplit) {
  static_assert(D == 64 || D == 128, "head dim");
  static_assert(G >= 1 && G <= 8, "heads per KV group");
  constexpr int CH = 128, KW = 32, ROWB = D * 2, NS = D / 32, NC = D / 16, VPW = KW * ROWB / 1024;
  constexpr int NWV = kThreads / 64;
  // V images of the 4 waves (KW rows each); after the products the same bytes hold the waves' O^T partials
  __shared__ __attribute__((aligned(16))) char s_v[NWV * KW * ROWB];
  __shared__ float s_ml[NWV][G][2];
  static_assert(NWV * G * D * 4 <= NWV * KW * ROWB, "partials fit the V images");
  const int split = blockIdx.x;
  const int b = blockIdx.y / Hkv, kvh = blockIdx.y % Hkv;
  const int t = threadIdx.x, lane = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int len = min(lens[b], Smax);
  const int k0 = split * CH;
  float* po = part_o + (((int64_t)b * Hkv + kvh) * G * nsplit) * D;
  float* pml = part_ml + (((int64_t)b * Hkv + kvh) * G * nsplit) * 2;
  if (k0 >= len) {  // split past the sequence: an empty partial
    if (t < G) {
      pml[(t * nsplit + split) * 2] = kNegBig;
      pml[(t * nsplit + split) * 2 + 1] = 0.f;
    }
    for (int i = t; i < G * D; i += kThreads) po[((i / D) * nsplit + split) * D + i % D] = 0.f;
    return;
  }
  const int kb = k0 + KW * wv;  // the wave's first key
  const bool live = kb < len;   // wave-uniform
  const int col = lane & 15, g = lane >> 4;
  const bf16_t* kbase = kc + ((int64_t)b * Hkv + kvh) * Smax * D;
  const bf16_t* vbase = vc + ((int64_t)b * Hkv + kvh) * Smax * D;
  char* const vimg = s_v + wv * (KW * ROWB);
  float m = kNegBig, l = 0.f;
  f32x4 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (live) {
    // Q^T B operand: head `col` (zero past G), dims 32s + 8g .. +7
    bf16x8 qf[NS];
    const bf16_t* qrow = q + (int64_t)b * qs + (int64_t)(kvh * G + (col < G ? col : 0)) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 32 * s);
      if (col >= G) qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    // K A operand of block bb: key row kb + 8(col >> 2) + 4bb + (col & 3) (clamped: masked below), dims 32s + 8g
    bf16x8 kf[2][NS];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int key = min(kb + 8 * (col >> 2) + 4 * bb + (col & 3), len - 1);
      const bf16_t* kr = kbase + (int64_t)key * D + 8 * g;
#pragma unroll
      for (int s = 0; s < NS; ++s) kf[bb][s] = *reinterpret_cast<const bf16x8*>(kr + 32 * s);
    }
    // V rows -> LDS image: piece i covers rows RPP i .. (1 KiB); lane -> (row, chunk slot), source chunk = slot ^ x
    {
      constexpr int SLOTS = ROWB / 16, RPP = 1024 / ROWB;
#pragma unroll
      for (int i = 0; i < VPW; ++i) {
        const int r = RPP * i + lane / SLOTS, slot = lane % SLOTS;
        const int key = min(kb + r, len - 1);
        glds16(vbase + (int64_t)key * D + 8 * (slot ^ dec_vx<ROWB>(r)), vimg + 1024 * i);
      }
    }
    // S^T: lane holds head `col`, keys kb + 8g + 4bb + j in sc[bb][j]
    f32x4 sc[2];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      sc[bb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) sc[bb] = mfma16(kf[bb][s], qf[s], sc[bb]);
    }
    float p[8];
    float mx = kNegBig;
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kb + 8 * g + 4 * bb + j;
        p[4 * bb + j] = key < len ? sc[bb][j] * scale_log2 : kNegBig;
        mx = fmaxf(mx, p[4 * bb + j]);
      }
    mx = xor32_max(xor16_max(mx));
    m = mx;  // key kb is valid, so m is finite
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p[j] = exp2f(p[j] - m);
      ls += p[j];
    }
    ls = xor32_sum(xor16_sum(ls));
    l = ls;
    const u32x4 pw = {pack2(p[0], p[1]), pack2(p[2], p[3]), pack2(p[4], p[5]), pack2(p[6], p[7])};
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pw);
    // V^T A operand of dim block c: two transposed reads (rows 8g + 4h + q, chunk 2c + (p >> 1) of the image)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tq = (lane >> 2) & 3, tp = lane & 3;
    const int x = dec_vx<ROWB>(8 * g + tq) >> 1;  // the same for h = 0 / 1
    const uint32_t vb = lds_addr(vimg) + (8 * g + tq) * ROWB + 8 * (tp & 1);
#pragma unroll
    for (int c0 = 0; c0 < NC; c0 += 4) {
      bf16x4 tr[8];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t a = vb + 16 * ((2 * (c0 + c) + (tp >> 1)) ^ (2 * x));
        tr[2 * c] = dec_tr_read<0>(a);
        tr[2 * c + 1] = dec_tr_read<4 * ROWB>(a);
      }
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(tr[0]), "+v"(tr[1]), "+v"(tr[2]), "+v"(tr[3]), "+v"(tr[4]), "+v"(tr[5]), "+v"(tr[6]),
                     "+v"(tr[7]));
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c0 + c] = mfma16(cat44(tr[2 * c], tr[2 * c + 1]), pf, acc[c0 + c]);
    }
  }
  // ---- the 4 waves' (m, l, O^T) -> one partial of the split
  __syncthreads();  // every wave is done with its V image
  float* so = reinterpret_cast<float*>(s_v);  // [wave][head][D]
  if (col < G) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) so[(wv * G + col) * D + 16 * c + 4 * g + r] = acc[c][r];
    if (g == 0) {
      s_ml[wv][col][0] = m;
      s_ml[wv][col][1] = l;
    }
  }
  __syncthreads();
  for (int i = t; i < G * D; i += kThreads) {
    const int h = i / D, d = i % D;
    float M = kNegBig;
#pragma unroll
    for (int w = 0; w < NWV; ++w) M = fmaxf(M, s_ml[w][h][0]);
    float o = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float wt = s_ml[w][h][1] > 0.f ? exp2f(s_ml[w][h][0] - M) : 0.f;
      o += so[(w * G + h) * D + d] * wt;
      L += s_ml[w][h][1] * wt;
    }
    po[((int64_t)h * nsplit + split) * D + d] = o;
    if (d == 0) {
      pml[(h * nsplit + split) * 2] = M;
      pml[(h * nsplit + split) * 2 + 1] = L;
    }
  }
}

// one wave per (sequence, query head): the split maxima / sums are reduced across the lanes, then every lane
// (D / 64 dims) folds the splits eight at a time -- eight independent partial loads in flight instead of a chain
// of dependent ones per split (13 -> ~5 us per layer at batch 64 x 2k context)
template <int D>
__global__ void __launch_bounds__(64) decode_attn_combine_kernel(const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml, int Hq,
                                                                 int nsplit, bf16_t* __restrict__ o, int64_t os) {
  // blockIdx.x = b * Hq + h; partials of head h live at (b, kvh, g) = row b * Hq + h in [B, Hkv, G] order
  constexpr int DPT = D / 64;
  const int bh = blockIdx.x, t = threadIdx.x;
  const float* ml = part_ml + (int64_t)bh * nsplit * 2;
  const float* po = part_o + (int64_t)bh * nsplit * D + DPT * t;
  float mloc = kNegBig;
  for (int s = t; s < nsplit; s += 64) mloc = fmaxf(mloc, ml[2 * s]);
  const float M = wave_max(mloc);
  float lloc = 0.f;
  for (int s = t; s < nsplit; s += 64) lloc += ml[2 * s + 1] > 0.f ? ml[2 * s + 1] * exp2f(ml[2 * s] - M) : 0.f;
  const float L = wave_sum(lloc);
  float a[DPT];
#pragma unroll
  for (int d = 0; d < DPT; ++d) a[d] = 0.f;
  int s = 0;
  for (; s + 8 <= nsplit; s += 8) {
    float mv[8], lv[8], pv[8][DPT];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mv[i] = ml[2 * (s + i)];
      lv[i] = ml[2 * (s + i) + 1];
#pragma unroll
      for (int d = 0; d < DPT; ++d) pv[i][d] = po[(int64_t)(s + i) * D + d];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float w = lv[i] > 0.f ? exp2f(mv[i] - M) : 0.f;
#pragma unroll
      for (int d = 0; d < DPT; ++d) a[d] += pv[i][d] * w;
    }
  }
  for (; s < nsplit; ++s) {
    const float w = ml[2 * s + 1] > 0.f ? exp2f(ml[2 * s] - M) : 0.f;
#pragma unroll
    for (int d = 0; d < DPT; ++d) a[d] += po[(int64_t)s * D + d] * w;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int b = bh / Hq, h = bh % Hq;
  bf16_t* op = o + (int64_t)b * os + (int64_t)h * D + DPT * t;
  if constexpr (DPT == 2) *reinterpret_cast<uint32_t*>(op) = pack2(a[0] * inv, a[1] * inv);
  else op[0] = f2bf(a[0] * inv);
}

static constexpr int chunk_keys() { return 128; }  // keys per pass-1 workgroup (256 measured -2 % at batch 128)

// ---------------------------------------------------------------------------------------------------------
// Decode-step append: RoPE at each sequence's position on its new Q and K heads (in place in the fused QKV row)
// and the rotated K row + the V row written into the cache at that position -- one launch per layer instead of
// a RoPE kernel and two scatter copies. grid (B, ceil(items / 256)); items per token: (Hq + Hkv) heads x D/16
// rotary chunks (8 pairs each), then Hkv x D/8 16-byte V chunks.
// ---------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) decode_rope_append_kernel(bf16_t* __restrict__ qkv, int64_t qs,
                                                                 const float* __restrict__ cos_t,
                                                                 const float* __restrict__ sin_t,
                                                                 const int* __restrict__ pos, bf16_t* __restrict__ kc,
                                                                 bf16_t* __restrict__ vc, int Smax, int Hq, int Hkv,
                                                                 int D) {
  const int b = blockIdx.x;
  const int item = blockIdx.y * blockDim.x + threadIdx.x;
  const int half = D >> 1, per_head = half >> 3;
  const int n_rot = (Hq + Hkv) * per_head, n_v = Hkv * (D >> 3);
  if (item >= n_rot + n_v) return;
  const int p = min(max(pos[b], 0), Smax - 1);
  bf16_t* row = qkv + (int64_t)b * qs;
  if (item < n_rot) {
    const int h = item / per_head, j = item - h * per_head;
    bf16_t* base = row + (int64_t)h * D + j * 8;
    const f32x4* cp = reinterpret_cast<const f32x4*>(cos_t + (int64_t)p * half + j * 8);
    const f32x4* sp = reinterpret_cast<const f32x4*>(sin_t + (int64_t)p * half + j * 8);
    float a[8], c[8], o1[8], o2[8], bb[8], sn[8];
    unpack8(*reinterpret_cast<const u32x4*>(base), a);
    unpack8(*reinterpret_cast<const u32x4*>(base + half), bb);
    const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      c[i] = c0[i];
      c[i + 4] = c1[i];
      sn[i] = s0[i];
      sn[i + 4] = s1[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o1[i] = a[i] * c[i] - bb[i] * sn[i];
      o2[i] = bb[i] * c[i] + a[i] * sn[i];
    }
    const u32x4 lo = pack8(o1), hi = pack8(o2);
    *reinterpret_cast<u32x4*>(base) = lo;
    *reinterpret_cast<u32x4*>(base + half) = hi;
    if (h >= Hq) {  // a K head: its rotated row goes to the cache
      bf16_t* dst = kc + (((int64_t)b * Hkv + (h - Hq)) * Smax + p) * D + j * 8;
      *reinterpret_cast<u32x4*>(dst) = lo;
      *reinterpret_cast<u32x4*>(dst + half) = hi;
    }
  } else {
    const int v = item - n_rot, vh = v / (D >> 3), ch = v - vh * (D >> 3);
    const u32x4 val = *reinterpret_cast<const u32x4*>(row + (int64_t)(Hq + Hkv + vh) * D + ch * 8);
    *reinterpret_cast<u32x4*>(vc + (((int64_t)b * Hkv + vh) * Smax + p) * D + ch * 8) = val;
  }
}

int decode_rope_append(bf16_t* qkv, int64_t qs, const float* cos_t, const float* sin_t, const int* pos, bf16_t* kc,
                       bf16_t* vc, int B, int Smax, int Hq, int Hkv, int D, hipStream_t stream) {
  if (D % 16 != 0 || qs % 8 != 0) return -1;
  const int items = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  decode_rope_append_kernel<<<dim3(B, (items + 255) / 256), 256, 0, stream>>>(qkv, qs, cos_t, sin_t, pos, kc, vc, Smax,
                                                                              Hq, Hkv, D);
  return 0;
}

int decode_attn_splits(int max_len) { return (max_len + chunk_keys() - 1) / chunk_keys(); }

static int g_decode_mfma = -1;  // -1: read KOP_DECODE_ATTN (mfma, the default, | valu) on first use
static bool decode_mfma() {
  if (g_decode_mfma < 0) {
    const char* e = getenv("KOP_DECODE_ATTN");
    g_decode_mfma = (e && std::string(e) == "valu") ? 0 : 1;
  }
  return g_decode_mfma != 0;
}
int decode_attn_set_mfma(int on) {
  const int old = decode_mfma() ? 1 : 0;
  if (on >= 0) g_decode_mfma = on ? 1 : 0;
  return old;
}

template <int D, int G>
static void launch_split(const bf16_t* q, int64_t qs, const bf16_t* kc, const bf16_t* vc, const int* lens, int B,
                         int Smax, int Hkv, float sl2, float* po, float* pml, int nsplit, hipStream_t stream) {
  if (decode_mfma())
    decode_attn_mfma_kernel<D, G><<<dim3(nsplit, B * Hkv), kThreads, 0, stream>>>(q, qs, kc, vc, lens, Smax, Hkv, sl2,
                                                                                 po, pml, nsplit);
  else
    decode_attn_split_kernel<D, G, 128><<<dim3(nsplit, B * Hkv), kThreads, 0, stream>>>(q, qs, kc, vc, lens, Smax, Hkv,
                                                                                       sl2, po, pml, nsplit);
}

int decode_attn(const bf16_t* q, int64_t qs, const bf16_t* kc, const bf16_t* vc, const int* lens, bf16_t* o,
                int64_t os, float* part_o, float* part_ml, int B, int Smax, int Hq, int Hkv, int D, int nsplit,
                float scale, hipStream_t stream) {
  const int ch = chunk_keys();
  if (Hq % Hkv != 0 || nsplit < 1 || nsplit * ch > Smax + ch - 1 || qs % 8 != 0 || os % 2 != 0) return -1;
  const int G = Hq / Hkv;
  const float sl2 = scale * kLog2e;
#define DEC_CASE(DV, GV)                                                                                     \
  if (D == DV && G == GV) {                                                                                  \
    launch_split<DV, GV>(q, qs, kc, vc, lens, B, Smax, Hkv, sl2, part_o, part_ml, nsplit, stream);           \
    decode_attn_combine_kernel<DV><<<B * Hq, 64, 0, stream>>>(part_o, part_ml, Hq, nsplit, o, os);       \
    return 0;                                                                                                \
  }
  DEC_CASE(128, 1)
  DEC_CASE(128, 2)
  DEC_CASE(128, 4)
  DEC_CASE(128, 8)
  DEC_CASE(64, 1)
  DEC_CASE(64, 2)
  DEC_CASE(64, 4)
  DEC_CASE(64, 8)
#undef DEC_CASE
  return -2;
}

}  // namespace kop
