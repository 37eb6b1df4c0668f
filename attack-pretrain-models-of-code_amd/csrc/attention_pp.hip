// attention_pp.hip — the fused attention of the split-precision modes over packed bf16 planes.
//
// attn_x3_kernel's algorithm (128 queries of one (sequence, head) per workgroup, the query on the
// lane, online softmax in the exp2 domain, optional bit-packed data-flow mask), fed by the QKV
// GEMM's packed-plane output (gemm_planes.hip PK_EPI_BIAS_PACKED: per 32 columns a block
// [hi 32 | lo 32] for NP = 2, plain bf16 for NP = 1) instead of f32:
//   * Q is read once as planes; its softmax scale log2(e)/8 is folded into Wq and bq at engine
//     creation, so the kernel converts and scales nothing;
//   * a key's 64 d of K (or V) are one contiguous 128·NP-byte run of its token row, so a 32-key
//     tile moves global -> LDS by LDS-DMA (global_load_lds_dwordx4, 4 key rows of 256 B per wave
//     instruction for NP = 2) into a double-buffered stage, with no register staging and no
//     hi/lo split in the loop;
//   * the DMA picks each lane's source chunk so that LDS position c of key row r holds logical
//     chunk c ^ swizzle(r): K rows (read by ds_read_b128, one key row per lane) XOR by the row's
//     low bits, V rows (read by ds_read_b64_tr_b16 in 4-key blocks) by (r & 3) << 2, both
//     conflict-free for their reads;
//   * S^T = K·Q^T and O^T += V^T·P^T on v_mfma_f32_32x32x16_bf16, 3 products per term pair for
//     NP = 2 (x_hi·y_hi + x_hi·y_lo + x_lo·y_hi), P split into hi/lo from the S accumulator.
#include <cfloat>
#include <type_traits>

#include "common.h"

// m0 is written only by dma16 below; nothing else in this kernel reads it
#pragma clang diagnostic ignored "-Winline-asm"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int QPB = 128, KT = 32, OSTRIDE = 65;
constexpr int QKV_COLS = 3 * AE_HIDDEN;

// One LDS-DMA wave instruction: 64 lanes x 16 B from per-lane global addresses into
// lds_base + 16 * lane (SALU write of m0 -> LDS-DMA needs one wait state).
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(gsrc), "s"(lds_base)
      : "memory", "m0");
}
// The same with a uniform 64-bit base in SGPRs and a per-lane 32-bit byte offset (saddr form):
// advancing a tile is two scalar adds instead of per-lane 64-bit address arithmetic.
__device__ __forceinline__ void dma16s(uint32_t voff, const void* sbase, uint32_t lds_base) {
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, %1"
      :
      : "v"(voff), "s"(sbase), "s"(lds_base)
      : "memory", "m0");
}

// One 4-B-per-lane LDS-DMA (saddr form): lane l's dword lands at lds_base + 4 * l
__device__ __forceinline__ void dma4s(uint32_t voff, const void* sbase, uint32_t lds_base) {
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %0, %1"
      :
      : "v"(voff), "s"(sbase), "s"(lds_base)
      : "memory", "m0");
}

template <int NP>
struct PPL {
  static constexpr int RB = 128 * NP;             // bytes of one key's 64 d (NP planes)
  static constexpr int CR = RB / 16;              // 16-B chunks per key row
  static constexpr int TILE = KT * RB;            // K (or V) tile
  static constexpr int STAGE = 2 * TILE;          // K then V
  static constexpr int ROWS_PER_DMA = 1024 / RB;  // key rows per wave DMA instruction
  static constexpr int DMA_PER_WAVE = KT / ROWS_PER_DMA / 4;  // per matrix, 4 waves
  static constexpr int LDS =
      (2 * STAGE > 4 * 32 * OSTRIDE * 4) ? 2 * STAGE : 4 * 32 * OSTRIDE * 4;
};

// logical 16-B chunk of (plane p, d) in a key row: block d / 32 holds [hi 32 | lo 32] (NP = 2)
template <int NP>
__device__ __forceinline__ int chunk_of(int p, int d) {
  return (d >> 5) * 4 * NP + 4 * p + ((d & 31) >> 3);
}
template <int NP>
__device__ __forceinline__ int kpos(int r, int x) {
  return x ^ (r & (PPL<NP>::CR - 1));
}
template <int NP>
__device__ __forceinline__ int vpos(int r, int x) {
  return NP == 2 ? x ^ ((r & 3) << 2) : x ^ (((r >> 1) & 1) << 2);
}
}  // namespace

// PIPE 1: software-pipelined loop — the S MFMAs of key tile kt + 1 issue in the same scheduling
// region as the exp / P-split VALU of tile kt (independent streams the SIMD co-issues), K and V in
// separate 2-slot rings (K two tiles ahead, V one).
// PIPE 4 (production): PIPE 1 with the O rescale unconditional, so no branch splits the region
// and tile kt's exp / P split really sits beside tile kt+1's S MFMAs, interleaved by
// sched_group_barrier (K reads, then one MFMA per five vector instructions).
// PIPE 2: PIPE 4 with fewer vector instructions per tile and nothing between the two streams:
// the O rescale is unconditional (no branch splits the region, so the exp / split really sits
// beside the next tile's S MFMAs, interleaved by sched_group_barrier), the tile max by 3-input
// max, and the exp / P split on packed f32 pairs with P's hi plane the TRUNCATED bf16 of p (its
// upper 16 bits, one shift-or per pair) and lo = bf16(p - hi), exact to 2^-16 of p as the
// rounded split.
template <int NP, bool HAS_MASK, bool PLANES, int PIPE>
__global__ __launch_bounds__(256, (PIPE == 5 || (PIPE >= 60 && PIPE != 64 && !(HAS_MASK && NP == 2))) ? 3 : 2) void attn_pp_kernel(const unsigned short* __restrict__ qkvp,
                                                         float* __restrict__ out,
                                                         unsigned short* __restrict__ op,
                                                         const int* __restrict__ cu,
                                                         const int* __restrict__ q_rows,
                                                         const uint32_t* __restrict__ mask,
                                                         int mask_L) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  // PIPE 66: PIPE 6 with saddr DMA (per-lane offsets computed once, tiles advanced on the scalar
  // unit) and the cross-half row max by v_permlane32_swap instead of an LDS permute.  PIPE 61-65:
  // timing diagnostics of 66 (results WRONG; tools/attn_bench.py only): 1 = no exp / P split
  // (P = bf16(S)), 2 = no tile max (fixed reference max 0), 3 = no barriers in the loop, 4 = no
  // PV MFMAs (no V reads), 5 = no S MFMAs after the prologue (no K reads)
  // PIPE 67: 66 with the tile max as a 3-level tree of v_max3 (depth 3 instead of a chain of 8);
  // PIPE 68: 67 with the exp / split on packed f32 pairs (experiments)
  constexpr int PB = PIPE >= 60 ? 6 : PIPE;
  constexpr int DG = (PIPE >= 61 && PIPE <= 65) ? PIPE - 60 : 0;
  constexpr bool FAST = PIPE >= 60;
  constexpr bool TREE = PIPE == 67 || PIPE == 68, PKX = PIPE == 68;
  static_assert(!(HAS_MASK && PB == 6 && !FAST),
                "PIPE 6 has no mask path (its loop keeps no ordinary global load, so its mask "
                "launches run PIPE 4); PIPE 66 moves the mask words by LDS-DMA");
  // PIPE 66 with a mask: the tile's mask words (one per query) ride the K / V DMA stream into a
  // 3-slot LDS ring of 4 waves x 256 B (lanes 32-63 duplicate lanes 0-31), so the loop still has
  // no compiler-visible global load and every wait stays a counted vmcnt
  constexpr int MASK_RING = (HAS_MASK && PB == 6) ? 3 * 4 * 256 : 0;
  // PIPE 6: three K and three V slots (the O staging of the epilogue fits inside)
  constexpr int LDS_BYTES =
      PB == 6 ? (6 * P::TILE > 4 * 32 * 66 * 4 ? 6 * P::TILE : 4 * 32 * 66 * 4) + MASK_RING : P::LDS;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QPB >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  constexpr size_t LDR = (size_t)NP * QKV_COLS;  // elements of one packed token row

  // Q fragments (pre-scaled): step s covers d = 16s + 8 lh .. +8 (B operand: B[k=d][j=q])
  const int q = qb * QPB + wave * 32 + li;
  const int qr = q < nq ? q : nq - 1;
  bf16x8 qh[4], ql[4];
  {
    const unsigned short* qp = qkvp + (size_t)(start + qr) * LDR + (size_t)head * 64 * NP;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * lh;
      const int off = (d >> 5) * 32 * NP + (d & 31);
      qh[s] = *reinterpret_cast<const bf16x8*>(qp + off);
      if (TERMS == 3) ql[s] = *reinterpret_cast<const bf16x8*>(qp + off + 32);
    }
  }

  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  const int dr = lane / P::CR, dc = lane % P::CR;
  // DMA of one matrix (K: moff 0 into slot kslot, V: moff 2·AE_HIDDEN) of key tile kt
  auto issue1 = [&](int kt, int moff, uint32_t dst, bool vimg) {
#pragma unroll
    for (int j = 0; j < P::DMA_PER_WAVE; ++j) {
      const int i = wave * P::DMA_PER_WAVE + j;
      const int r = i * P::ROWS_PER_DMA + dr;
      int key = kt * KT + r;
      key = key < len ? key : len - 1;
      const unsigned short* row = qkvp + (size_t)(start + key) * LDR;
      dma16(row + (size_t)(moff + head * 64) * NP + (vimg ? vpos<NP>(r, dc) : kpos<NP>(r, dc)) * 8,
            dst + i * 1024);
    }
  };

  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;
  const uint32_t* mrow = nullptr;
  if (HAS_MASK) mrow = mask + ((size_t)seq * mask_L + qr) * (mask_L / 32);

  // S^T = K Q^T over a K image (4 k-steps of 16 d); lane li reads key row li
  auto s_mfma = [&](const unsigned char* stk, floatx16& s) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * lh;
      const unsigned char* kr = stk + li * P::RB;
      const bf16x8 kh =
          *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(0, d0)) * 16);
      if (TERMS == 3) {
        const bf16x8 kl =
            *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(1, d0)) * 16);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[ks], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[ks], s, 0, 0, 0);
      }
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[ks], s, 0, 0, 0);
    }
  };
  // mask + running max of tile kt (lane = query); returns the new max
  auto tile_max = [&](int kt, floatx16& s) {
    uint32_t mbits = 0xffffffffu;
    if (HAS_MASK) mbits = mrow[kt];
    float mt = -INFINITY;
    if (!HAS_MASK && (kt + 1) * KT <= len) {  // full tile, no mask: no per-key select
#pragma unroll
      for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s[r], s[r + 1]));
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = mfma32_row(r, lh);
        // absent keys (beyond the sequence) are -inf; keys the mask excludes score the most
        // negative finite float, as HF's additive finfo(f32).min mask does: a query row that
        // excludes every key then attends all of them uniformly (GraphCodeBERT truncated nodes)
        const bool in = kt * KT + kk < len;
        s[r] = !in ? -INFINITY : (((mbits >> kk) & 1u) ? s[r] : -FLT_MAX);
        mt = fmaxf(mt, s[r]);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    return fmaxf(m_run, mt);  // finite: key kt·KT is present in every tile
  };
  // P = exp2(S - m) (in place), its row sum, and the bf16 hi / lo split of P^T for the PV MFMAs
  auto exp_split = [&](floatx16& s, float m_new, bf16x8 (&ph)[2], bf16x8 (&pl)[2]) {
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(s[r] - m_new);  // exp2(-inf) = 0
      psum += p;
      const __bf16 h = (__bf16)p;
      ph[r >> 3][r & 7] = h;
      pl[r >> 3][r & 7] = (__bf16)(p - (float)h);
    }
    return psum;
  };
  // PIPE 2's exp / split: packed pairs, truncated hi (see above)
  auto exp_split2 = [&](floatx16& s, float m_new, bf16x8 (&ph)[2], bf16x8 (&pl)[2]) {
    floatx2 acc2 = {0.f, 0.f};
    const floatx2 mm = {m_new, m_new};
    u32x4 hw[2], lw[2];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const floatx2 d = floatx2{s[2 * q], s[2 * q + 1]} - mm;
      // (scalar copies: __builtin_bit_cast of an ext_vector ELEMENT reads element 0 — a clang
      // lowering hazard this loop hit, every pair's second hi plane was its first's)
      const float px = __builtin_amdgcn_exp2f(d.x), py = __builtin_amdgcn_exp2f(d.y);
      acc2 += floatx2{px, py};
      const uint32_t b0 = __builtin_bit_cast(uint32_t, px) & 0xffff0000u;
      const uint32_t b1 = __builtin_bit_cast(uint32_t, py) & 0xffff0000u;
      const float lx = px - __builtin_bit_cast(float, b0);
      const float ly = py - __builtin_bit_cast(float, b1);
      hw[q >> 2][q & 3] = (b0 >> 16) | b1;  // [hi(p.x) | hi(p.y) << 16]
      const bf16x2 l2 = {(__bf16)lx, (__bf16)ly};
      lw[q >> 2][q & 3] = __builtin_bit_cast(uint32_t, l2);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      ph[t] = __builtin_bit_cast(bf16x8, hw[t]);
      pl[t] = __builtin_bit_cast(bf16x8, lw[t]);
    }
    return acc2.x + acc2.y;
  };
  // exp_split on packed f32 pairs with the same rounded hi / lo planes (only the row sum's
  // association differs: two interleaved partial sums)
  auto exp_split_pk = [&](floatx16& s, float m_new, bf16x8 (&ph)[2], bf16x8 (&pl)[2]) {
    floatx2 acc2 = {0.f, 0.f};
    const floatx2 mm = {m_new, m_new};
    u32x4 hw[2], lw[2];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const floatx2 d = floatx2{s[2 * q], s[2 * q + 1]} - mm;
      const float px = __builtin_amdgcn_exp2f(d.x), py = __builtin_amdgcn_exp2f(d.y);
      const floatx2 pp = {px, py};
      acc2 += pp;
      const bf16x2 h2 = {(__bf16)px, (__bf16)py};
      const uint32_t hb = __builtin_bit_cast(uint32_t, h2);
      const floatx2 hf = {__builtin_bit_cast(float, hb << 16), __builtin_bit_cast(float, hb & 0xffff0000u)};
      const floatx2 l = pp - hf;
      const float lx = l.x, ly = l.y;
      const bf16x2 l2 = {(__bf16)lx, (__bf16)ly};
      hw[q >> 2][q & 3] = hb;
      lw[q >> 2][q & 3] = __builtin_bit_cast(uint32_t, l2);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      ph[t] = __builtin_bit_cast(bf16x8, hw[t]);
      pl[t] = __builtin_bit_cast(bf16x8, lw[t]);
    }
    return acc2.x + acc2.y;
  };
  // O^T += V^T P^T (2 k-steps of 16 keys, 2 d-tiles).  P^T straight from the S accumulator:
  // registers 8t..8t+7 of lane half h hold keys 16t + 4h + {0..3} and 16t + 8 + 4h + {0..3};
  // the V^T operand takes the same keys through the transposed read
  auto pv_mfma = [&](const unsigned char* stv, const bf16x8 (&ph)[2], const bf16x8 (&pl)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k0 = 16 * t + 4 * lh;
      // lane 16g + 4q + p addresses key row k0 + q (and k0 + 8 + q), d columns
      // 32 dt + 16 (g & 1) + 4p; it receives d = 32 dt + (lane & 31) of those 4 keys
      const int kq = k0 + ((lane >> 2) & 3);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const int cb = (col & 7) * 2;
        const unsigned char* va = stv + kq * P::RB + cb;
        const unsigned char* vb = stv + (kq + 8) * P::RB + cb;
        bf16x8 vh, vl;
        {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(0, col)) * 16));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(0, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = b[e]; }
        }
        if (TERMS == 3) {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(1, col)) * 16));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(1, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vl[e] = a[e]; vl[4 + e] = b[e]; }
        }
        floatx16& o = dt == 0 ? o0 : o1;
        if (TERMS == 3) {
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph[t], o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl[t], o, 0, 0, 0);
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph[t], o, 0, 0, 0);
      }
    }
  };
  auto rescale = [&](float alpha) {
    if (__any(alpha != 1.f)) {  // alpha == 1 exactly when no row max moved: skipping is exact
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
  };

  const int nkt = (len + KT - 1) / KT;
  if constexpr (PB == 6) {
    // 3-slot rings: K_j in slot j % 3, V_j in slot 3 + j % 3.  Iteration kt issues V_{kt+2} and
    // K_{kt+3} and, at its end, waits only for what iteration kt+1 reads (V_{kt+1}, K_{kt+2},
    // issued one iteration earlier): a counted vmcnt leaves this iteration's DMA in flight across
    // the raw s_barrier, so every transfer has two tiles of compute to land in.
    auto kslot = [&](int j) { return (uint32_t)(j * P::TILE); };        // prologue tiles 0..2
    auto vslot = [&](int j) { return (uint32_t)((3 + j) * P::TILE); };
    auto wait_vm = [](int n) {  // n = DMA instructions allowed to stay outstanding
      if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (HAS_MASK && n == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (HAS_MASK && n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (HAS_MASK && n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (HAS_MASK && n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto barrier = []() {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (DG != 3) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    constexpr int DM = P::DMA_PER_WAVE;  // DMA instructions per wave per matrix tile
    // FAST: byte offsets of this lane's DMA chunks from the sequence's first token row (K and V,
    // one per DMA instruction), fixed for the whole loop; a full tile kt adds kt·KT rows to the
    // scalar base; the last, partial tile clamps its key rows the per-lane way (issue1)
    uint32_t voff[2][FAST ? DM : 1];
    const unsigned char* sbase =
        reinterpret_cast<const unsigned char*>(qkvp + (size_t)start * LDR);
    if constexpr (FAST) {
#pragma unroll
      for (int j = 0; j < DM; ++j) {
        const int r = (wave * DM + j) * P::ROWS_PER_DMA + dr;
        voff[0][j] = 2u * ((uint32_t)r * (uint32_t)LDR + (AE_HIDDEN + head * 64) * NP + kpos<NP>(r, dc) * 8);
        voff[1][j] = 2u * ((uint32_t)r * (uint32_t)LDR + (2 * AE_HIDDEN + head * 64) * NP + vpos<NP>(r, dc) * 8);
      }
    }
    auto issue = [&](int kt, bool isv, uint32_t dst) {
      if constexpr (FAST) {
        const unsigned char* sb = sbase + (size_t)kt * KT * LDR * 2;
        if ((kt + 1) * KT <= len) {
#pragma unroll
          for (int j = 0; j < DM; ++j) dma16s(voff[isv][j], sb, dst + (wave * DM + j) * 1024);
        } else {  // key rows past the sequence re-read its last row (finite, masked to -inf)
          const int last = len - 1 - kt * KT;
#pragma unroll
          for (int j = 0; j < DM; ++j) {
            const int over = (wave * DM + j) * P::ROWS_PER_DMA + dr - last;
            const uint32_t v = voff[isv][j] - (over > 0 ? (uint32_t)over * (uint32_t)(LDR * 2) : 0u);
            dma16s(v, sb, dst + (wave * DM + j) * 1024);
          }
        }
      } else {
        issue1(kt, isv ? 2 * AE_HIDDEN : AE_HIDDEN, dst, isv);
      }
    };
    // mask words of tile j: query qr's word j, from the sequence's first mask row (scalar base)
    constexpr int MW = HAS_MASK ? 1 : 0;  // DMA instructions per tile for the mask
    constexpr uint32_t MASK_OFF = 6 * P::TILE > 4 * 32 * 66 * 4 ? 6 * P::TILE : 4 * 32 * 66 * 4;
    const uint32_t* mbase = HAS_MASK ? mask + (size_t)seq * mask_L * (mask_L / 32) : nullptr;
    const uint32_t moff = HAS_MASK ? (uint32_t)qr * (uint32_t)(mask_L / 32) * 4u : 0u;
    auto issue_m = [&](int j) {
      if constexpr (HAS_MASK)
        dma4s(moff, mbase + j, lds0 + MASK_OFF + (uint32_t)((j % 3) * 1024 + wave * 256));
    };
    // prologue: K0 V0 M0 K1 V1 M1 K2 (as many as exist; M = mask words, masked launches only)
    issue(0, false, lds0 + kslot(0));
    issue(0, true, lds0 + vslot(0));
    issue_m(0);
    int after_k0 = DM + MW, after_k1 = 0;
    if (nkt > 1) {
      issue(1, false, lds0 + kslot(1));
      issue(1, true, lds0 + vslot(1));
      issue_m(1);
      after_k0 += 2 * DM + MW;
      after_k1 = DM + MW;
    }
    if (nkt > 2) {
      issue(2, false, lds0 + kslot(2));
      after_k0 += DM;
      after_k1 += DM;
    }
    wait_vm(after_k0);  // K0 landed
    barrier();
    floatx16 sA, sB;  // S of the current / next tile, alternating by tile parity
    s_mfma(lds + kslot(0), sA);
    if constexpr (DG == 5) sB = sA;
    wait_vm(after_k1);  // V0, M0 (and K1) landed
    barrier();  // every wave has read K0 (its slot takes K3) and sees V0, M0, K1
    // one tile; R = kt % 6 fixes the slots (R % 3) and the S buffers (R % 2) at compile time, so
    // every LDS address of the body is a constant offset from a per-lane base
    auto body = [&](auto rc, int kt, floatx16& s_cur, floatx16& s_next) {
      constexpr int R = decltype(rc)::value;
      constexpr uint32_t KS_NEXT = ((R + 1) % 3) * P::TILE, VS_CUR = (3 + R % 3) * P::TILE;
      constexpr uint32_t VS_ISS = (3 + (R + 2) % 3) * P::TILE, KS_ISS = (R % 3) * P::TILE;
      int n_iss = 0;
      if (kt + 2 < nkt) {
        issue_m(kt + 2);
        issue(kt + 2, true, lds0 + VS_ISS);
        n_iss += DM + MW;
      }
      if (kt + 3 < nkt) {
        issue(kt + 3, false, lds0 + KS_ISS);
        n_iss += DM;
      }
      // deferred rescale (cdna_hip_programming.md T13): keep the running max unless some row's
      // tile max exceeds it by more than 8 (log2 domain), so P <= 2^8 and the O rescale runs only
      // on the tiles that move a max by that much — the same softmax with another reference max
      float m_new = 0.f, alpha = 1.f;
      bool grow = false;
      if constexpr (DG != 2) {
        float mt = -INFINITY;
        if (!HAS_MASK && (kt + 1) * KT <= len) {
          if constexpr (TREE) {
            float a[6];
#pragma unroll
            for (int r = 0; r < 5; ++r) a[r] = fmaxf(s_cur[3 * r], fmaxf(s_cur[3 * r + 1], s_cur[3 * r + 2]));
            a[5] = s_cur[15];
            mt = fmaxf(fmaxf(a[0], fmaxf(a[1], a[2])), fmaxf(a[3], fmaxf(a[4], a[5])));
          } else {
#pragma unroll
            for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s_cur[r], s_cur[r + 1]));
          }
        } else {
          uint32_t mb = 0xffffffffu;
          if constexpr (HAS_MASK)
            mb = *reinterpret_cast<const uint32_t*>(lds + MASK_OFF + (R % 3) * 1024 + wave * 256 + 4 * li);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kk = mfma32_row(r, lh);
            // absent keys -inf; keys the mask excludes the most negative finite float (HF's
            // additive finfo.min mask), as tile_max
            const bool in = kt * KT + kk < len;
            s_cur[r] = !in ? -INFINITY : (((mb >> kk) & 1u) ? s_cur[r] : -FLT_MAX);
            mt = fmaxf(mt, s_cur[r]);
          }
        }
        if constexpr (FAST) {
          // lanes l and l ^ 32 hold the two halves of a query's keys: swap the halves on the VALU
          const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, mt),
                                                          __builtin_bit_cast(uint32_t, mt), false, false);
          mt = fmaxf(__builtin_bit_cast(float, (uint32_t)sw[0]), __builtin_bit_cast(float, (uint32_t)sw[1]));
        } else {
          mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        }
        grow = __any(mt > m_run + 8.f);
        m_new = grow ? fmaxf(m_run, mt) : m_run;
        alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 1 when m_new == m_run; 0 from -inf
      }
      bf16x8 ph[2], pl[2];
      __builtin_amdgcn_sched_barrier(0);
      float psum;
      if constexpr (DG == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) ph[r >> 3][r & 7] = (__bf16)s_cur[r];
        pl[0] = ph[0];
        pl[1] = ph[1];
        psum = s_cur[0];
      } else {
        psum = PKX ? exp_split_pk(s_cur, m_new, ph, pl) : exp_split(s_cur, m_new, ph, pl);
      }
      if constexpr (DG != 5) s_mfma(lds + KS_NEXT, s_next);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      l_run = l_run * alpha + psum;
      m_run = m_new;
      if (grow) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      }
      if constexpr (DG == 4) {
#pragma unroll
        for (int r = 0; r < 8; ++r) { o0[r] += (float)ph[0][r]; o1[r] += (float)pl[1][r]; }
      } else {
        pv_mfma(lds + VS_CUR, ph, pl);
      }
      wait_vm(n_iss);  // V_{kt+1}, K_{kt+2} landed; this iteration's DMA stays in flight
      barrier();
    };
    for (int kt = 0; kt < nkt; kt += 6) {
      body(std::integral_constant<int, 0>(), kt, sA, sB);
      if (kt + 1 >= nkt) break;
      body(std::integral_constant<int, 1>(), kt + 1, sB, sA);
      if (kt + 2 >= nkt) break;
      body(std::integral_constant<int, 2>(), kt + 2, sA, sB);
      if (kt + 3 >= nkt) break;
      body(std::integral_constant<int, 3>(), kt + 3, sB, sA);
      if (kt + 4 >= nkt) break;
      body(std::integral_constant<int, 4>(), kt + 4, sA, sB);
      if (kt + 5 >= nkt) break;
      body(std::integral_constant<int, 5>(), kt + 5, sB, sA);
    }
  } else if (PIPE == 0) {
    // stage b = [K | V] of one tile, two stages
    issue1(0, AE_HIDDEN, lds0, false);
    issue1(0, 2 * AE_HIDDEN, lds0 + P::TILE, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      // the other stage was last read in iteration kt - 1, before its closing barrier
      if (kt + 1 < nkt) {
        issue1(kt + 1, AE_HIDDEN, lds0 + (cur ^ 1) * P::STAGE, false);
        issue1(kt + 1, 2 * AE_HIDDEN, lds0 + (cur ^ 1) * P::STAGE + P::TILE, true);
      }
      const unsigned char* stk = lds + cur * P::STAGE;
      floatx16 s;
      s_mfma(stk, s);
      const float m_new = tile_max(kt, s);
      const float alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
      bf16x8 ph[2], pl[2];
      const float psum = exp_split(s, m_new, ph, pl);
      l_run = l_run * alpha + psum;
      m_run = m_new;
      rescale(alpha);
      pv_mfma(stk + P::TILE, ph, pl);
      // tile kt + 1 landed (this wave's DMA), and every wave is done reading stage cur
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // K ring (slots 0, 1) then V ring (slots 2, 3): K_j in slot j & 1, V_j in slot 2 + (j & 1)
    auto kslot = [&](int j) { return (uint32_t)((j & 1) * P::TILE); };
    auto vslot = [&](int j) { return (uint32_t)((2 + (j & 1)) * P::TILE); };
    issue1(0, AE_HIDDEN, lds0 + kslot(0), false);
    issue1(0, 2 * AE_HIDDEN, lds0 + vslot(0), true);
    if (nkt > 1) issue1(1, AE_HIDDEN, lds0 + kslot(1), false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    floatx16 s_cur;
    s_mfma(lds + kslot(0), s_cur);
    __syncthreads();  // every wave has read K_0 before K_2 lands in its slot
    for (int kt = 0; kt < nkt; ++kt) {
      // V_{kt+1} into V_{kt-1}'s slot and K_{kt+2} into K_kt's slot: both last read in
      // iteration kt - 1 (or the prologue), before its closing barrier
      if (kt + 1 < nkt) issue1(kt + 1, 2 * AE_HIDDEN, lds0 + vslot(kt + 1), true);
      if (kt + 2 < nkt) issue1(kt + 2, AE_HIDDEN, lds0 + kslot(kt + 2), false);
      const float m_new = tile_max(kt, s_cur);
      const float alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
      bf16x8 ph[2], pl[2];
      floatx16 s_next;
      // one scheduling region: tile kt's exp / split on the VALU, tile kt + 1's S on the MFMA
      // (the last iteration's S of a tile past the end reads a stale slot and is discarded;
      // unconditional so the region has no branch)
      float psum;
      if constexpr (PIPE >= 2) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PIPE >= 4) psum = exp_split(s_cur, m_new, ph, pl);
        else psum = exp_split2(s_cur, m_new, ph, pl);
        s_mfma(lds + kslot(kt + 1), s_next);
        if constexpr (PIPE != 3) {
          // the K fragment reads first, then one S MFMA per few vector instructions
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
          for (int i = 0; i < 12; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      } else {
        psum = exp_split(s_cur, m_new, ph, pl);
        s_mfma(lds + kslot(kt + 1), s_next);
      }
      l_run = l_run * alpha + psum;
      m_run = m_new;
      if constexpr (PIPE >= 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      } else {
        rescale(alpha);
      }
      pv_mfma(lds + vslot(kt), ph, pl);
      s_cur = s_next;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if constexpr (PB == 6) {
    // O through LDS (rows of 66 floats: 8-B aligned, 2-way on the column writes), then 16-B
    // stores of whole output chunks: 8 (planes) or 8 (f32) store instructions per wave instead of
    // one 2-B store per row and plane
    constexpr int S6 = 66;
    float* os6 = reinterpret_cast<float*>(lds) + wave * 32 * S6;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = mfma32_row(r, lh);
      os6[li * S6 + d] = o0[r] * inv;
      os6[li * S6 + 32 + d] = o1[r] * inv;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own rows: no barrier
    constexpr int CPR = PLANES ? 8 * NP : 16;             // 16-B chunks per output row
    constexpr int RPI = 64 / CPR;                         // rows per store instruction
    const int c = lane % CPR;
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int rr = it * RPI + lane / CPR;
      const int qq = qb * QPB + wave * 32 + rr;
      const float* src = os6 + rr * S6;
      if (PLANES) {
        // chunk c: block c / (4 NP), plane (c / 4) % NP, d = 32 block + 8 (c % 4) .. + 7
        const int d0 = 32 * (c / (4 * NP)) + 8 * (c % 4);
        const bool lo_plane = NP == 2 && ((c >> 2) & 1);
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const floatx2 v = *reinterpret_cast<const floatx2*>(src + d0 + 2 * e);
          const __bf16 hx = (__bf16)v.x, hy = (__bf16)v.y;
          bf16x2 pr;
          if (lo_plane) pr = bf16x2{(__bf16)(v.x - (float)hx), (__bf16)(v.y - (float)hy)};
          else pr = bf16x2{hx, hy};
          w[e] = __builtin_bit_cast(uint32_t, pr);
        }
        if (qq < nq) {
          unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + head * 64 * NP + c * 8;
          *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
        }
      } else {
        const floatx2 a = *reinterpret_cast<const floatx2*>(src + 4 * c);
        const floatx2 b = *reinterpret_cast<const floatx2*>(src + 4 * c + 2);
        if (qq < nq)
          *reinterpret_cast<floatx4*>(out + (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + 4 * c) =
              floatx4{a.x, a.y, b.x, b.y};
      }
    }
    return;
  }
  float* os = reinterpret_cast<float*>(lds) + wave * 32 * OSTRIDE;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = mfma32_row(r, lh);
    os[li * OSTRIDE + d] = o0[r] * inv;
    os[li * OSTRIDE + 32 + d] = o1[r] * inv;
  }
  __syncthreads();
  for (int rr = 0; rr < 32; ++rr) {
    const int qq = qb * QPB + wave * 32 + rr;
    if (qq < nq) {
      const float v = os[rr * OSTRIDE + lane];
      if (PLANES) {  // packed planes of the O-projection operand (gemm_planes.hip layout)
        const int c = head * AE_HEAD_DIM + lane;
        unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + (c >> 5) * 32 * NP + (c & 31);
        const unsigned short h = f2bf(v);
        dst[0] = h;
        if (NP == 2) dst[32] = f2bf(v - __builtin_bit_cast(float, (uint32_t)h << 16));
      } else {
        out[(size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + lane] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// attn_pp8_kernel (variant 7): the same attention as attn_pp_kernel on 8 waves that share each
// SIMD in a fixed ping-pong (MI355X_MICROARCH.md "Two waves per SIMD";
// cdna_hip_programming.md T16).  Both 4-wave groups own the same 128 queries (wave w and w + 4
// share a SIMD and a 32-query slice) but split the KEYS: group g takes key tiles g, g + 2, g + 4,
// ... from its own 4-slot K and V rings, and the two partial softmaxes (m, l, O) are merged at the
// end (flash-decoding inside the workgroup).  A group's work alternates two segment kinds:
//   V(i): softmax of S(i) -> P(i) (deferred rescale as PIPE 6), the O rescale, the LDS reads of
//         the next C segment's operands (K(i+1), V(i)) and the DMA of K(i+3), V(i+3);
//   C(i): MFMAs only — S(i+1) = K(i+1)·Q^T and O += V(i)^T·P(i)^T — then the counted vmcnt that
//         lands K(i+2), V(i+1);
// group 1 runs one segment behind group 0, and an s_barrier separates segments, so on every SIMD
// one wave feeds the matrix pipe while its partner runs the softmax VALU and the LDS traffic.
// Measured SLOWER than PIPE 6 (B=64 x L=512, same box: 286.8 vs 173.3 us,
// profiles/r3q_attn_pp7_ab.jsonl), correct (tests/test_kernels_gpu.py variant 7): a V segment
// (softmax VALU + 24 LDS reads + 4 LDS-DMA issues) runs about twice a C segment's 24 MFMAs, so
// the matrix pipe idles at every barrier, and with one workgroup per CU each workgroup's
// prologue (Q, first tiles) and merge / store epilogue are no longer hidden by a co-resident
// one.  Kept as an experiment (ae_bench_attention_pp variant 7), not used by the engine.
template <int NP, bool PLANES>
__global__ __launch_bounds__(512, 1) void attn_pp8_kernel(const unsigned short* __restrict__ qkvp,
                                                          float* __restrict__ out,
                                                          unsigned short* __restrict__ op,
                                                          const int* __restrict__ cu,
                                                          const int* __restrict__ q_rows) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  constexpr int NSL = 4;                      // ring slots per matrix per group
  constexpr int GRING = 2 * NSL * P::TILE;    // a group's K then V slots
  constexpr int MERGE_BYTES = 4 * 34 * 64 * 4;  // group 1's (O, m, l) per lane, after the loop
  constexpr int STAGE_BYTES = 4 * 32 * 66 * 4;  // group 0's context staging, after the merge
  constexpr int MERGE_OFF = GRING > STAGE_BYTES ? GRING : (STAGE_BYTES + 1023) / 1024 * 1024;
  constexpr int LDS_BYTES = 2 * GRING > MERGE_OFF + MERGE_BYTES ? 2 * GRING : MERGE_OFF + MERGE_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QPB >= nq) return;  // the whole workgroup: no barrier is skipped by part of it

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, gw = wave & 3;
  const int li = lane & 31, lh = lane >> 5;
  constexpr size_t LDR = (size_t)NP * QKV_COLS;

  const int q = qb * QPB + gw * 32 + li;
  const int qr = q < nq ? q : nq - 1;
  bf16x8 qh[4], ql[4];
  {
    const unsigned short* qp = qkvp + (size_t)(start + qr) * LDR + (size_t)head * 64 * NP;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * lh;
      const int off = (d >> 5) * 32 * NP + (d & 31);
      qh[s] = *reinterpret_cast<const bf16x8*>(qp + off);
      if (TERMS == 3) ql[s] = *reinterpret_cast<const bf16x8*>(qp + off + 32);
    }
  }

  const int nkt = (len + KT - 1) / KT;
  const int n = (nkt - grp + 1) >> 1;  // this group's key tiles: t = 2 i + grp, i < n
  const int nA = (nkt + 1) >> 1;       // group 0's count (>= group 1's)
  const uint32_t ring = (uint32_t)(uintptr_t)lds + grp * GRING;
  const unsigned char* gl = lds + grp * GRING;
  constexpr int DM = P::DMA_PER_WAVE;
  const int dr = lane / P::CR, dc = lane % P::CR;
  // DMA of this group's i-th K (moff = AE_HIDDEN) or V (2 AE_HIDDEN) tile into its slot
  auto issue = [&](int i, bool is_v) {
    const int t = 2 * i + grp;
    const uint32_t dst = ring + ((is_v ? NSL : 0) + (i & (NSL - 1))) * P::TILE;
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      const int pi = gw * DM + j;
      const int r = pi * P::ROWS_PER_DMA + dr;
      int key = t * KT + r;
      key = key < len ? key : len - 1;
      const unsigned short* row = qkvp + (size_t)(start + key) * LDR;
      const int moff = is_v ? 2 * AE_HIDDEN : AE_HIDDEN;
      dma16(row + (size_t)(moff + head * 64) * NP + (is_v ? vpos<NP>(r, dc) : kpos<NP>(r, dc)) * 8,
            dst + pi * 1024);
    }
  };
  auto wait_vm = [](int k) {  // k = DMA instructions allowed to stay outstanding
    if (k >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (k >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (k >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (k >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (k >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // operand fragments of the next C segment (read in the V segment before it)
  bf16x8 kfh[4], kfl[4];       // K(i+1): per 16-d step, hi / lo planes of this lane's key row
  bf16x8 vfh[2][2], vfl[2][2];  // V(i): [key step t][d tile]
  auto read_k = [&](int i) {
    const unsigned char* kr = gl + (i & (NSL - 1)) * P::TILE + li * P::RB;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * lh;
      kfh[ks] = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(0, d0)) * 16);
      if (TERMS == 3)
        kfl[ks] = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(1, d0)) * 16);
    }
  };
  auto read_v = [&](int i) {
    const unsigned char* stv = gl + (NSL + (i & (NSL - 1))) * P::TILE;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kq = 16 * t + 4 * lh + ((lane >> 2) & 3);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const int cb = (col & 7) * 2;
        const unsigned char* va = stv + kq * P::RB + cb;
        const unsigned char* vb = stv + (kq + 8) * P::RB + cb;
        const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(0, col)) * 16));
        const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(0, col)) * 16));
#pragma unroll
        for (int e = 0; e < 4; ++e) { vfh[t][dt][e] = a[e]; vfh[t][dt][4 + e] = b[e]; }
        if (TERMS == 3) {
          const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(1, col)) * 16));
          const bf16x4 d = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(1, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vfl[t][dt][e] = c[e]; vfl[t][dt][4 + e] = d[e]; }
        }
      }
    }
  };

  floatx16 s, o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;
  bf16x8 ph[2], pl[2];

  // C(i): S(i+1) (if it exists) and O += V(i)^T P(i)^T (i >= 0); then land K(i+2), V(i+1)
  auto seg_c = [&](int i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + 1 < n) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (TERMS == 3) {
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfl[ks], qh[ks], s, 0, 0, 0);
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ks], ql[ks], s, 0, 0, 0);
        }
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ks], qh[ks], s, 0, 0, 0);
      }
    }
    if (i >= 0 && i < n) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          floatx16& o = dt == 0 ? o0 : o1;
          if (TERMS == 3) {
            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfl[t][dt], ph[t], o, 0, 0, 0);
            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfh[t][dt], pl[t], o, 0, 0, 0);
          }
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfh[t][dt], ph[t], o, 0, 0, 0);
        }
    }
    // DMA issue order K0 V0 K1 V1 ...: after K(i+2) come V(i+2), K(i+3), V(i+3)
    if (i + 2 < n) wait_vm(DM * (1 + (i + 3 < n ? 2 : 0)));
    else wait_vm(0);
  };
  // V(i): softmax of S(i), O rescale, the next C segment's operand reads, DMA of tile i+3
  auto seg_v = [&](int i) {
    if (i < 0 || i >= n) return;
    const int t = 2 * i + grp;
    float mt = -INFINITY;
    if ((t + 1) * KT <= len) {
#pragma unroll
      for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s[r], s[r + 1]));
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool in = t * KT + mfma32_row(r, lh) < len;
        s[r] = in ? s[r] : -INFINITY;
        mt = fmaxf(mt, s[r]);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const bool grow = __any(mt > m_run + 8.f);
    const float m_new = grow ? fmaxf(m_run, mt) : m_run;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(s[r] - m_new);
      psum += p;
      const __bf16 h = (__bf16)p;
      ph[r >> 3][r & 7] = h;
      pl[r >> 3][r & 7] = (__bf16)(p - (float)h);
    }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (grow) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    if (i + 1 < n) read_k(i + 1);
    read_v(i);
    if (i + 3 < n) {
      issue(i + 3, false);
      issue(i + 3, true);
    }
  };

  // prologue: K0 V0 K1 V1 K2 V2 of this group (as many as exist); K0 landed -> its fragments
  int issued = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < n) {
      issue(i, false);
      issue(i, true);
      issued += 2;
    }
  wait_vm(n > 0 ? DM * (issued - 1) : 0);
  // Q through an empty asm: its uses in the loop then depend on the asm, not on the loads, so
  // hipcc places its wait for them here (once, with the prologue DMA) instead of inside every
  // C segment, where it drained the tile DMA in flight (measured: 296 vs 175 us)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    asm volatile("" : "+v"(qh[k]));
    if (TERMS == 3) asm volatile("" : "+v"(ql[k]));
  }
  barrier();
  if (n > 0) read_k(0);
  // C(-1) lands K(1) (and V(0)); the segment loop's barriers make them visible to the group

  // both groups run the same loop [C(j-1) | V(j)], a barrier after each segment; group 1 first
  // passes one extra barrier (and group 0 one after the loop), so it runs one segment behind:
  // group 0's C segments meet group 1's V segments and vice versa
  if (grp == 1) barrier();
  for (int j = 0; j <= nA; ++j) {
    seg_c(j - 1);
    barrier();
    seg_v(j);
    barrier();
  }
  if (grp == 0) barrier();

  // merge: group 1 publishes (O, m, l) per lane, group 0 combines and writes the context
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  float* mg = reinterpret_cast<float*>(lds + MERGE_OFF) + gw * 34 * 64;
  if (grp == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      mg[r * 64 + lane] = o0[r];
      mg[(16 + r) * 64 + lane] = o1[r];
    }
    mg[32 * 64 + lane] = m_run;
    mg[33 * 64 + lane] = l_tot;
  }
  barrier();
  if (grp == 1) return;
  const float mb = mg[32 * 64 + lane], lb = mg[33 * 64 + lane];
  const float mm = fmaxf(m_run, mb);
  // -inf - -inf cannot occur: group 0 always has a tile, so m_run is finite
  const float fa = __builtin_amdgcn_exp2f(m_run - mm), fb = __builtin_amdgcn_exp2f(mb - mm);
  const float lt = l_tot * fa + lb * fb;
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  const float ca = fa * inv, cbf = fb * inv;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    o0[r] = o0[r] * ca + mg[r * 64 + lane] * cbf;
    o1[r] = o1[r] * ca + mg[(16 + r) * 64 + lane] * cbf;
  }
  // context through LDS (PIPE 6's epilogue; the staging area is group 0's ring, nothing reads
  // it any more), 16-B stores of whole output chunks
  constexpr int S6 = 66;
  float* os6 = reinterpret_cast<float*>(lds) + gw * 32 * S6;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = mfma32_row(r, lh);
    os6[li * S6 + d] = o0[r];
    os6[li * S6 + 32 + d] = o1[r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int CPR = PLANES ? 8 * NP : 16;
  constexpr int RPI = 64 / CPR;
  const int c = lane % CPR;
#pragma unroll
  for (int it = 0; it < 32 / RPI; ++it) {
    const int rr = it * RPI + lane / CPR;
    const int qq = qb * QPB + gw * 32 + rr;
    const float* src = os6 + rr * S6;
    if (PLANES) {
      const int d0 = 32 * (c / (4 * NP)) + 8 * (c % 4);
      const bool lo_plane = NP == 2 && ((c >> 2) & 1);
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const floatx2 v = *reinterpret_cast<const floatx2*>(src + d0 + 2 * e);
        const __bf16 hx = (__bf16)v.x, hy = (__bf16)v.y;
        bf16x2 pr;
        if (lo_plane) pr = bf16x2{(__bf16)(v.x - (float)hx), (__bf16)(v.y - (float)hy)};
        else pr = bf16x2{hx, hy};
        w[e] = __builtin_bit_cast(uint32_t, pr);
      }
      if (qq < nq) {
        unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + head * 64 * NP + c * 8;
        *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
      }
    } else {
      const floatx2 a = *reinterpret_cast<const floatx2*>(src + 4 * c);
      const floatx2 b = *reinterpret_cast<const floatx2*>(src + 4 * c + 2);
      if (qq < nq)
        *reinterpret_cast<floatx4*>(out + (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + 4 * c) =
            floatx4{a.x, a.y, b.x, b.y};
    }
  }
}

// ------------------------------------------------------------------------------------------
// attn_pw64_kernel (variant 8): one wave per SIMD, 64 queries per wave (two 32-query blocks),
// 4 waves = 256 queries per workgroup, one workgroup per CU (cdna_hip_programming.md's
// "pwg4x64" structure): each K fragment read from LDS serves both query blocks' S MFMAs and each
// V fragment both blocks' PV MFMAs (half the LDS reads per query), and a wave's 48 MFMAs per key
// tile are independent chains of two blocks whose issue gaps take the other block's softmax VALU
// — latency is hidden inside the wave instead of by a second, uncoordinated wave on the SIMD.
// Rings, waits and the deferred rescale are PIPE 6's; registers: up to 512 per wave.
// Measured SLOWER than PIPE 6 (B=64 x L=512, same box: 273.0 vs 175.1 us,
// profiles/r3r_attn_pw64_ab.jsonl), correct (tests/test_kernels_gpu.py variant 8): the body needs
// 355 registers, 160 AGPR <-> VGPR moves per tile come with them, and a lone wave per SIMD
// exposes every dependency the interleave cannot cover.  Kept as an experiment (variant 8).
template <int NP, bool PLANES>
__global__ __launch_bounds__(256, 1) void attn_pw64_kernel(const unsigned short* __restrict__ qkvp,
                                                           float* __restrict__ out,
                                                           unsigned short* __restrict__ op,
                                                           const int* __restrict__ cu,
                                                           const int* __restrict__ q_rows) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  constexpr int QW = 256;  // queries per workgroup
  constexpr int LDS_BYTES = 6 * P::TILE > 4 * 32 * 66 * 4 ? 6 * P::TILE : 4 * 32 * 66 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QW >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  constexpr size_t LDR = (size_t)NP * QKV_COLS;

  // Q fragments of the two blocks (b = 0, 1: queries qb*256 + wave*64 + 32 b + li)
  bf16x8 qh[2][4], ql[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int q = qb * QW + wave * 64 + 32 * b + li;
    const int qr = q < nq ? q : nq - 1;
    const unsigned short* qp = qkvp + (size_t)(start + qr) * LDR + (size_t)head * 64 * NP;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * lh;
      const int off = (d >> 5) * 32 * NP + (d & 31);
      qh[b][s] = *reinterpret_cast<const bf16x8*>(qp + off);
      if (TERMS == 3) ql[b][s] = *reinterpret_cast<const bf16x8*>(qp + off + 32);
    }
  }

  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  const int dr = lane / P::CR, dc = lane % P::CR;
  auto issue1 = [&](int kt, int moff, uint32_t dst, bool vimg) {
#pragma unroll
    for (int j = 0; j < P::DMA_PER_WAVE; ++j) {
      const int i = wave * P::DMA_PER_WAVE + j;
      const int r = i * P::ROWS_PER_DMA + dr;
      int key = kt * KT + r;
      key = key < len ? key : len - 1;
      const unsigned short* row = qkvp + (size_t)(start + key) * LDR;
      dma16(row + (size_t)(moff + head * 64) * NP + (vimg ? vpos<NP>(r, dc) : kpos<NP>(r, dc)) * 8,
            dst + i * 1024);
    }
  };
  auto wait_vm = [](int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int DM = P::DMA_PER_WAVE;

  floatx16 o[2][2];  // [block][d tile]
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) { o[b][0][r] = 0.f; o[b][1][r] = 0.f; }
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  // S^T of both blocks from one read of the K fragments
  auto s_mfma = [&](const unsigned char* stk, floatx16 (&s)[2]) {
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[b][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * lh;
      const unsigned char* kr = stk + li * P::RB;
      const bf16x8 kh = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(0, d0)) * 16);
      bf16x8 kl;
      if (TERMS == 3) kl = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(li, chunk_of<NP>(1, d0)) * 16);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (TERMS == 3) {
          s[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[b][ks], s[b], 0, 0, 0);
          s[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[b][ks], s[b], 0, 0, 0);
        }
        s[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[b][ks], s[b], 0, 0, 0);
      }
    }
  };
  // O^T += V^T P^T for both blocks from one read of each V fragment
  auto pv_mfma = [&](const unsigned char* stv, const bf16x8 (&ph)[2][2], const bf16x8 (&pl)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kq = 16 * t + 4 * lh + ((lane >> 2) & 3);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const int cb = (col & 7) * 2;
        const unsigned char* va = stv + kq * P::RB + cb;
        const unsigned char* vb = stv + (kq + 8) * P::RB + cb;
        bf16x8 vh, vl;
        {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(0, col)) * 16));
          const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(0, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = c[e]; }
        }
        if (TERMS == 3) {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(1, col)) * 16));
          const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(1, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vl[e] = a[e]; vl[4 + e] = c[e]; }
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (TERMS == 3) {
            o[b][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph[b][t], o[b][dt], 0, 0, 0);
            o[b][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl[b][t], o[b][dt], 0, 0, 0);
          }
          o[b][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph[b][t], o[b][dt], 0, 0, 0);
        }
      }
    }
  };

  const int nkt = (len + KT - 1) / KT;
  auto kslot = [&](int j) { return (uint32_t)(j * P::TILE); };
  auto vslot = [&](int j) { return (uint32_t)((3 + j) * P::TILE); };
  int groups = 2;
  issue1(0, AE_HIDDEN, lds0 + kslot(0), false);
  issue1(0, 2 * AE_HIDDEN, lds0 + vslot(0), true);
  if (nkt > 1) {
    issue1(1, AE_HIDDEN, lds0 + kslot(1), false);
    issue1(1, 2 * AE_HIDDEN, lds0 + vslot(1), true);
    groups += 2;
  }
  if (nkt > 2) {
    issue1(2, AE_HIDDEN, lds0 + kslot(2), false);
    ++groups;
  }
  wait_vm(DM * (groups - 1));
  // Q through an empty asm: hipcc waits for its loads here once, not inside the loop
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      asm volatile("" : "+v"(qh[b][k]));
      if (TERMS == 3) asm volatile("" : "+v"(ql[b][k]));
    }
  barrier();
  floatx16 sA[2], sB[2];
  s_mfma(lds + kslot(0), sA);
  wait_vm(nkt > 1 ? DM * (groups - 3) : 0);
  barrier();

  auto body = [&](auto rc, int kt, floatx16 (&s_cur)[2], floatx16 (&s_next)[2]) {
    constexpr int R = decltype(rc)::value;
    constexpr uint32_t KS_NEXT = ((R + 1) % 3) * P::TILE, VS_CUR = (3 + R % 3) * P::TILE;
    constexpr uint32_t VS_ISS = (3 + (R + 2) % 3) * P::TILE, KS_ISS = (R % 3) * P::TILE;
    int n_iss = 0;
    if (kt + 2 < nkt) {
      issue1(kt + 2, 2 * AE_HIDDEN, lds0 + VS_ISS, true);
      n_iss += DM;
    }
    if (kt + 3 < nkt) {
      issue1(kt + 3, AE_HIDDEN, lds0 + KS_ISS, false);
      n_iss += DM;
    }
    const bool full = (kt + 1) * KT <= len;
    float m_new[2], alpha[2];
    bool grow[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float mt = -INFINITY;
      if (full) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s_cur[b][r], s_cur[b][r + 1]));
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool in = kt * KT + mfma32_row(r, lh) < len;
          s_cur[b][r] = in ? s_cur[b][r] : -INFINITY;
          mt = fmaxf(mt, s_cur[b][r]);
        }
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      grow[b] = __any(mt > m_run[b] + 8.f);
      m_new[b] = grow[b] ? fmaxf(m_run[b], mt) : m_run[b];
      alpha[b] = __builtin_amdgcn_exp2f(m_run[b] - m_new[b]);
    }
    bf16x8 ph[2][2], pl[2][2];
    float psum[2] = {0.f, 0.f};
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(s_cur[b][r] - m_new[b]);
        psum[b] += p;
        const __bf16 h = (__bf16)p;
        ph[b][r >> 3][r & 7] = h;
        pl[b][r >> 3][r & 7] = (__bf16)(p - (float)h);
      }
    s_mfma(lds + KS_NEXT, s_next);
    // K fragment reads first, then one S MFMA per ~7 vector instructions
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      l_run[b] = l_run[b] * alpha[b] + psum[b];
      m_run[b] = m_new[b];
    }
    if (grow[0] || grow[1]) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) { o[b][0][r] *= alpha[b]; o[b][1][r] *= alpha[b]; }
    }
    pv_mfma(lds + VS_CUR, ph, pl);
    wait_vm(n_iss);
    barrier();
  };
  for (int kt = 0; kt < nkt; kt += 6) {
    body(std::integral_constant<int, 0>(), kt, sA, sB);
    if (kt + 1 >= nkt) break;
    body(std::integral_constant<int, 1>(), kt + 1, sB, sA);
    if (kt + 2 >= nkt) break;
    body(std::integral_constant<int, 2>(), kt + 2, sA, sB);
    if (kt + 3 >= nkt) break;
    body(std::integral_constant<int, 3>(), kt + 3, sB, sA);
    if (kt + 4 >= nkt) break;
    body(std::integral_constant<int, 4>(), kt + 4, sA, sB);
    if (kt + 5 >= nkt) break;
    body(std::integral_constant<int, 5>(), kt + 5, sB, sA);
  }

  // context: per block through the wave's LDS rows (66 floats), 16-B stores of whole chunks
  constexpr int S6 = 66;
  float* os6 = reinterpret_cast<float*>(lds) + wave * 32 * S6;
  constexpr int CPR = PLANES ? 8 * NP : 16;
  constexpr int RPI = 64 / CPR;
  const int c = lane % CPR;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float l_tot = l_run[b] + __shfl_xor(l_run[b], 32, 64);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = mfma32_row(r, lh);
      os6[li * S6 + d] = o[b][0][r] * inv;
      os6[li * S6 + 32 + d] = o[b][1][r] * inv;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int rr = it * RPI + lane / CPR;
      const int qq = qb * QW + wave * 64 + 32 * b + rr;
      const float* src = os6 + rr * S6;
      if (PLANES) {
        const int d0 = 32 * (c / (4 * NP)) + 8 * (c % 4);
        const bool lo_plane = NP == 2 && ((c >> 2) & 1);
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const floatx2 v = *reinterpret_cast<const floatx2*>(src + d0 + 2 * e);
          const __bf16 hx = (__bf16)v.x, hy = (__bf16)v.y;
          bf16x2 pr;
          if (lo_plane) pr = bf16x2{(__bf16)(v.x - (float)hx), (__bf16)(v.y - (float)hy)};
          else pr = bf16x2{hx, hy};
          w[e] = __builtin_bit_cast(uint32_t, pr);
        }
        if (qq < nq) {
          unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + head * 64 * NP + c * 8;
          *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
        }
      } else {
        const floatx2 a = *reinterpret_cast<const floatx2*>(src + 4 * c);
        const floatx2 b2 = *reinterpret_cast<const floatx2*>(src + 4 * c + 2);
        if (qq < nq)
          *reinterpret_cast<floatx4*>(out + (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + 4 * c) =
              floatx4{a.x, a.y, b2.x, b2.y};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // block 0's rows read before block 1's land
  }
}

// ------------------------------------------------------------------------------------------
// attn_kt64_kernel (variant 9): PIPE 6 with 64-key tiles — the per-tile fixed work (row-max
// exchange, rescale decision, DMA issue, counted wait, barrier) is paid once per 64 keys, and the
// S of a tile is two independent 12-MFMA chains.  K and V tiles of 64 keys (16 KiB each for
// NP = 2) in 2-slot rings: iteration kt issues V(kt+1) and K(kt+2) and waits for them at its end.
// Measured and not kept: correct (tests/test_kernels_gpu.py variant 9) but 217.1 vs 186.2 µs
// full-length, 136.3 vs 126.6 µs ragged against PIPE 6 (profiles/r3x_attn_kt64_ab.log): the
// per-key VALU falls only ~3 % and the 2-slot rings prefetch one tile less deep.
template <int NP, bool PLANES>
__global__ __launch_bounds__(256, 2) void attn_kt64_kernel(const unsigned short* __restrict__ qkvp,
                                                           float* __restrict__ out,
                                                           unsigned short* __restrict__ op,
                                                           const int* __restrict__ cu,
                                                           const int* __restrict__ q_rows) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  constexpr int KT2 = 64;
  constexpr int TILE2 = KT2 * P::RB;  // one 64-key K (or V) tile
  constexpr int DM = KT2 / P::ROWS_PER_DMA / 4;  // DMA instructions per wave per matrix tile
  constexpr int LDS_BYTES = 4 * TILE2 > 4 * 32 * 66 * 4 ? 4 * TILE2 : 4 * 32 * 66 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QPB >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  constexpr size_t LDR = (size_t)NP * QKV_COLS;

  const int q = qb * QPB + wave * 32 + li;
  const int qr = q < nq ? q : nq - 1;
  bf16x8 qh[4], ql[4];
  {
    const unsigned short* qp = qkvp + (size_t)(start + qr) * LDR + (size_t)head * 64 * NP;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * lh;
      const int off = (d >> 5) * 32 * NP + (d & 31);
      qh[s] = *reinterpret_cast<const bf16x8*>(qp + off);
      if (TERMS == 3) ql[s] = *reinterpret_cast<const bf16x8*>(qp + off + 32);
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  const int dr = lane / P::CR, dc = lane % P::CR;
  // DMA of a 64-key K (moff AE_HIDDEN) or V (2 AE_HIDDEN) tile; row r of the tile keeps the
  // 32-key tiles' swizzles (they depend on r's low bits only)
  auto issue = [&](int kt, int moff, uint32_t dst, bool vimg) {
#pragma unroll
    for (int j = 0; j < DM; ++j) {
      const int i = wave * DM + j;
      const int r = i * P::ROWS_PER_DMA + dr;
      int key = kt * KT2 + r;
      key = key < len ? key : len - 1;
      const unsigned short* row = qkvp + (size_t)(start + key) * LDR;
      dma16(row + (size_t)(moff + head * 64) * NP + (vimg ? vpos<NP>(r, dc) : kpos<NP>(r, dc)) * 8,
            dst + i * 1024);
    }
  };
  auto wait_vm = [](int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;

  // S^T of both 32-key halves of a 64-key K image
  auto s_mfma = [&](const unsigned char* stk, floatx16 (&s)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[h][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int d0 = 16 * ks + 8 * lh;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = 32 * h + li;
        const unsigned char* kr = stk + row * P::RB;
        const bf16x8 kh = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(row, chunk_of<NP>(0, d0)) * 16);
        if (TERMS == 3) {
          const bf16x8 kl =
              *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(row, chunk_of<NP>(1, d0)) * 16);
          s[h] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[ks], s[h], 0, 0, 0);
          s[h] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[ks], s[h], 0, 0, 0);
        }
        s[h] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[ks], s[h], 0, 0, 0);
      }
    }
  };
  // O^T += V^T P^T over 64 keys (4 k-steps of 16)
  auto pv_mfma = [&](const unsigned char* stv, const bf16x8 (&ph)[4], const bf16x8 (&pl)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kq = 16 * t + 4 * lh + ((lane >> 2) & 3);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const int cb = (col & 7) * 2;
        const unsigned char* va = stv + kq * P::RB + cb;
        const unsigned char* vb = stv + (kq + 8) * P::RB + cb;
        bf16x8 vh, vl;
        {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(0, col)) * 16));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(0, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = b[e]; }
        }
        if (TERMS == 3) {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(1, col)) * 16));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(1, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vl[e] = a[e]; vl[4 + e] = b[e]; }
        }
        floatx16& o = dt == 0 ? o0 : o1;
        if (TERMS == 3) {
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph[t], o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl[t], o, 0, 0, 0);
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph[t], o, 0, 0, 0);
      }
    }
  };

  const int nkt = (len + KT2 - 1) / KT2;
  // prologue: K0, V0, K1 (slots: K_j in j & 1, V_j in 2 + (j & 1))
  issue(0, AE_HIDDEN, lds0, false);
  issue(0, 2 * AE_HIDDEN, lds0 + 2 * TILE2, true);
  if (nkt > 1) issue(1, AE_HIDDEN, lds0 + TILE2, false);
  wait_vm(nkt > 1 ? 2 * DM : DM);  // K0 landed
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // Q through an empty asm: hipcc waits for it here, once
    asm volatile("" : "+v"(qh[k]));
    if (TERMS == 3) asm volatile("" : "+v"(ql[k]));
  }
  barrier();
  floatx16 sA[2], sB[2];
  s_mfma(lds, sA);
  wait_vm(0);  // V0, K1 landed
  barrier();  // every wave has read K0 (its slot takes K2) and sees V0, K1

  auto body = [&](auto rc, int kt, floatx16 (&s_cur)[2], floatx16 (&s_next)[2]) {
    constexpr int R = decltype(rc)::value;  // kt & 1
    constexpr uint32_t KS_NEXT = (1 - R) * TILE2, VS_CUR = (2 + R) * TILE2;
    constexpr uint32_t VS_ISS = (2 + (1 - R)) * TILE2, KS_ISS = R * TILE2;
    int n_iss = 0;
    if (kt + 1 < nkt) {
      issue(kt + 1, 2 * AE_HIDDEN, lds0 + VS_ISS, true);  // V(kt+1) into V(kt-1)'s slot
      n_iss += DM;
    }
    if (kt + 2 < nkt) {
      issue(kt + 2, AE_HIDDEN, lds0 + KS_ISS, false);  // K(kt+2) into K(kt)'s slot
      n_iss += DM;
    }
    float mt = -INFINITY;
    if ((kt + 1) * KT2 <= len) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s_cur[h][r], s_cur[h][r + 1]));
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool in = kt * KT2 + 32 * h + mfma32_row(r, lh) < len;
          s_cur[h][r] = in ? s_cur[h][r] : -INFINITY;
          mt = fmaxf(mt, s_cur[h][r]);
        }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const bool grow = __any(mt > m_run + 8.f);
    const float m_new = grow ? fmaxf(m_run, mt) : m_run;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    bf16x8 ph[4], pl[4];
    float psum = 0.f;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(s_cur[h][r] - m_new);
        psum += p;
        const __bf16 hv = (__bf16)p;
        ph[2 * h + (r >> 3)][r & 7] = hv;
        pl[2 * h + (r >> 3)][r & 7] = (__bf16)(p - (float)hv);
      }
    s_mfma(lds + KS_NEXT, s_next);  // unconditional: the last tile's reads a stale slot, unused
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (grow) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }
    pv_mfma(lds + VS_CUR, ph, pl);
    (void)n_iss;
    wait_vm(0);  // V(kt+1), K(kt+2): iteration kt+1 reads both
    barrier();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    body(std::integral_constant<int, 0>(), kt, sA, sB);
    if (kt + 1 >= nkt) break;
    body(std::integral_constant<int, 1>(), kt + 1, sB, sA);
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  constexpr int S6 = 66;
  float* os6 = reinterpret_cast<float*>(lds) + wave * 32 * S6;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = mfma32_row(r, lh);
    os6[li * S6 + d] = o0[r] * inv;
    os6[li * S6 + 32 + d] = o1[r] * inv;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int CPR = PLANES ? 8 * NP : 16;
  constexpr int RPI = 64 / CPR;
  const int c = lane % CPR;
#pragma unroll
  for (int it = 0; it < 32 / RPI; ++it) {
    const int rr = it * RPI + lane / CPR;
    const int qq = qb * QPB + wave * 32 + rr;
    const float* src = os6 + rr * S6;
    if (PLANES) {
      const int d0 = 32 * (c / (4 * NP)) + 8 * (c % 4);
      const bool lo_plane = NP == 2 && ((c >> 2) & 1);
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const floatx2 v = *reinterpret_cast<const floatx2*>(src + d0 + 2 * e);
        const __bf16 hx = (__bf16)v.x, hy = (__bf16)v.y;
        bf16x2 pr;
        if (lo_plane) pr = bf16x2{(__bf16)(v.x - (float)hx), (__bf16)(v.y - (float)hy)};
        else pr = bf16x2{hx, hy};
        w[e] = __builtin_bit_cast(uint32_t, pr);
      }
      if (qq < nq) {
        unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + head * 64 * NP + c * 8;
        *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
      }
    } else {
      const floatx2 a = *reinterpret_cast<const floatx2*>(src + 4 * c);
      const floatx2 b = *reinterpret_cast<const floatx2*>(src + 4 * c + 2);
      if (qq < nq)
        *reinterpret_cast<floatx4*>(out + (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + 4 * c) =
            floatx4{a.x, a.y, b.x, b.y};
    }
  }
}

// qkvp: packed planes [T][np·2304] with Q pre-scaled by log2(e)/8; context to op (packed planes)
// or out (f32 [T, 768]).  q_rows / max_q: the CLS-only launch of the last layer.
namespace {
template <int PIPE>
hipError_t app_launch(const unsigned short* qkvp, float* out, unsigned short* op, const int* cu,
                      const int* q_rows, int max_q, int n, int heads, const uint32_t* mask,
                      int mask_L, int np, hipStream_t stream) {
  if (n <= 0 || max_q <= 0) return hipSuccess;
  if (np != 1 && np != 2) return hipErrorInvalidValue;
  dim3 grid((max_q + QPB - 1) / QPB, heads, n), block(256);
#define APP_LAUNCH(N, M, PL)                                                                 \
  hipLaunchKernelGGL((attn_pp_kernel<N, M, PL, M ? (PIPE >= 60 ? 66 : PIPE >= 6 ? 4 : PIPE) : (PIPE >= 60 ? PIPE : PIPE >= 7 ? 6 : PIPE)>), grid, block, 0,      \
                     stream, qkvp, out, op, cu,                                                 \
                     q_rows, mask, mask_L)
#define APP_MP(N)                                                      \
  if (op) {                                                            \
    if (mask) APP_LAUNCH(N, true, true); else APP_LAUNCH(N, false, true);   \
  } else {                                                             \
    if (mask) APP_LAUNCH(N, true, false); else APP_LAUNCH(N, false, false); \
  }
  if (PIPE == 9 && !mask) {  // 64-key tiles (no mask path: masks run PIPE 4)
    if (np == 2) {
      if (op) hipLaunchKernelGGL((attn_kt64_kernel<2, true>), grid, block, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_kt64_kernel<2, false>), grid, block, 0, stream, qkvp, out, op, cu, q_rows);
    } else {
      if (op) hipLaunchKernelGGL((attn_kt64_kernel<1, true>), grid, block, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_kt64_kernel<1, false>), grid, block, 0, stream, qkvp, out, op, cu, q_rows);
    }
    return hipGetLastError();
  }
  if (PIPE == 8 && !mask) {  // 4 waves x 64 queries (no mask path: masks run PIPE 4)
    dim3 grid8((max_q + 255) / 256, heads, n);
    if (np == 2) {
      if (op) hipLaunchKernelGGL((attn_pw64_kernel<2, true>), grid8, block, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_pw64_kernel<2, false>), grid8, block, 0, stream, qkvp, out, op, cu, q_rows);
    } else {
      if (op) hipLaunchKernelGGL((attn_pw64_kernel<1, true>), grid8, block, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_pw64_kernel<1, false>), grid8, block, 0, stream, qkvp, out, op, cu, q_rows);
    }
    return hipGetLastError();
  }
  if (PIPE == 7 && !mask) {  // the 8-wave ping-pong kernel (no mask path: masks run PIPE 4)
    dim3 block8(512);
    if (np == 2) {
      if (op) hipLaunchKernelGGL((attn_pp8_kernel<2, true>), grid, block8, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_pp8_kernel<2, false>), grid, block8, 0, stream, qkvp, out, op, cu, q_rows);
    } else {
      if (op) hipLaunchKernelGGL((attn_pp8_kernel<1, true>), grid, block8, 0, stream, qkvp, out, op, cu, q_rows);
      else hipLaunchKernelGGL((attn_pp8_kernel<1, false>), grid, block8, 0, stream, qkvp, out, op, cu, q_rows);
    }
    return hipGetLastError();
  }
  if (np == 2) {
    APP_MP(2)
  } else {
    APP_MP(1)
  }
#undef APP_MP
#undef APP_LAUNCH
  return hipGetLastError();
}
// production loop: PIPE 66 = PIPE 6 with saddr DMA and the permlane row max, at three
// workgroups per CU (168 registers): packed-plane output (the engine's launch), B=64 x L=512, same
// box, interleaved rounds: pp6 192.3 / pp66 172.2 us median, ragged 138.6 / 123.5
// (profiles/r3y_attn_diag_ab.jsonl; again 207.7 / 178.3 and 130.6 / 125.3 on another box,
// profiles/r3z_attn_spec_ab.jsonl).  Before it PIPE 6 over PIPE 4 (pp4 198.3 / pp6 190.8 us,
// profiles/r3n_attn_ab.jsonl) and PIPE 4 over 1 (197.0 / 192.6, ragged 129.1 / 126.5,
// profiles/r3i_attn_ab.jsonl); the masked launches keep PIPE 4.  PIPE 2-3 (packed split) and 5 (3
// workgroups per CU of PIPE 4) measured no better than 4.  Measured and not kept: the tile's P
// computed against the running max before the tile max is known (recomputed when the max
// moves; bit-identical) 190.7 vs 178.3 us, and that on packed pairs 191.6
// (profiles/r3z_attn_spec_ab.jsonl).  PIPE 61-65 timing diagnostics of 66 (r3y): without the
// exp / split 160.5 us, without the tile max 161.5, without barriers 176.1, without the next
// tile's S MFMAs 151.7 of 172.2 — no single stage bounds the loop.  PIPE 67 (66 with the tile max
// as a depth-3 tree of v_max3, bit-identical): 178.0 vs 181.5 us, ragged 121.2 vs 122.8
// (profiles/r3an_attn_tree_max_ab.jsonl) — production; the masked launches run 66 (their max
// takes the per-key select path).  PIPE 68 (67 with the exp / split on packed pairs): 193.1 vs
// 184.5 (profiles/r3am_attn_ab.jsonl), and the row sum in two interleaved partial sums (a shorter
// add chain) 188.5 / 188.2 vs 187.3 / 188.7 (profiles/r3ao_attn_psum2_ab.jsonl), and other
// interleaves of the next S MFMAs with the exp / split (8 or 3 vector instructions per MFMA, or
// the compiler's own order: 181.2 / 181.6 / 183.7 vs 179.8 / 179.5 us,
// profiles/r3as_attn_interleave_ab.jsonl): not kept.
constexpr int APP_PIPE = 67;
}  // namespace

extern "C" hipError_t ae_launch_attention_pp(const unsigned short* qkvp, float* out,
                                             unsigned short* op, const int* cu, const int* q_rows,
                                             int max_q, int n, int heads, const uint32_t* mask,
                                             int mask_L, int np, hipStream_t stream) {
  return app_launch<APP_PIPE>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np,
                              stream);
}

// Kernel experiments (tools/attn_bench.py, tests): variant 0 = two-stage loop, 1 = pipelined,
// 2 = pipelined with the packed / branch-free tile (PIPE 2 above), 3 = 2 without the
// interleave hints, 4 = the previous production loop (rounded split, branch-free rescale,
// interleave hints), 5 = 4 at three workgroups per CU, 6 = the round-3 loop (3-slot rings,
// deferred rescale), 7 = attn_pp8_kernel (8-wave ping-pong, keys split over two groups), 8 =
// attn_pw64_kernel, 9 = attn_kt64_kernel, 61-65 = timing diagnostics of 66 (WRONG results), 66 =
// saddr DMA + permlane max, 67 = the production loop (66 + tree max), 68 = 67 on packed pairs.
// (An XCD-aware workgroup order — the q-blocks of one (sequence, head) on one XCD — measured 2-3 %
// slower, profiles/r2i_attn_pp_ab.jsonl: the K/V re-reads are Infinity-Cache hits, not the bound.)
extern "C" hipError_t ae_bench_attention_pp(const unsigned short* qkvp, float* out,
                                            unsigned short* op, const int* cu, const int* q_rows,
                                            int max_q, int n, int heads, const uint32_t* mask,
                                            int mask_L, int np, int variant, hipStream_t stream) {
  switch (variant) {  // PIPE 6 diagnostics / the saddr + permlane form (see attn_pp_kernel)
    case 61: return app_launch<61>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 62: return app_launch<62>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 63: return app_launch<63>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 64: return app_launch<64>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 65: return app_launch<65>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 66: return app_launch<66>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 67: return app_launch<67>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 68: return app_launch<68>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    default: break;
  }
  if (variant == 9)
    return app_launch<9>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 8)
    return app_launch<8>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 7)
    return app_launch<7>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 6)
    return app_launch<6>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 5)
    return app_launch<5>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 4)
    return app_launch<4>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 3)
    return app_launch<3>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 2)
    return app_launch<2>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 1)
    return app_launch<1>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  if (variant == 0)
    return app_launch<0>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
  return hipErrorInvalidValue;
}
