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

// max without the canonicalising v_max x, x that fmaxf (llvm.maxnum, IEEE mode) puts in front of
// every MFMA result it reads: IEEE maximum (v_maximum3_f32 on gfx950).  Scores are finite or
// -inf (absent keys), never NaN, so the two agree on every value the loop sees.
__device__ __forceinline__ float max_nc(float a, float b) { return __builtin_elementwise_maximum(a, b); }

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
template <int N>
__device__ __forceinline__ void wait_vm_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
}  // namespace

// PIPE 4: software-pipelined loop — the S MFMAs of key tile kt + 1 issue in the same scheduling
// region as the exp / P-split VALU of tile kt (independent streams the SIMD co-issues), K and V in
// separate 2-slot rings (K two tiles ahead, V one), the O rescale unconditional (no branch splits
// the region), interleaved by sched_group_barrier (K reads, then one MFMA per five vector
// instructions).  Kept only as the mask path of the PIPE 6 reference (bench variant 6).
// PIPE 6 / 66 / 67: below (67 is the production loop).
template <int NP, bool HAS_MASK, bool PLANES, int PIPE>
__global__ __launch_bounds__(256, (PIPE >= 60 && !(HAS_MASK && NP == 2)) ? 3 : 2) void attn_pp_kernel(const unsigned short* __restrict__ qkvp,
                                                         float* __restrict__ out,
                                                         unsigned short* __restrict__ op,
                                                         const int* __restrict__ cu,
                                                         const int* __restrict__ q_rows,
                                                         const uint32_t* __restrict__ mask,
                                                         int mask_L) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  // PIPE 66: PIPE 6 with saddr DMA (per-lane offsets computed once, tiles advanced on the scalar
  // unit) and the cross-half row max by v_permlane32_swap instead of an LDS permute.
  // PIPE 67: 66 with the tile max as a 3-level tree of v_max3 (depth 3 instead of a chain of 8).
  static_assert(PIPE == 4 || PIPE == 6 || PIPE == 66 || PIPE == 67 || PIPE == 72 || PIPE == 74,
                "loop variants 4, 6, 66, 67, 72, 74");
  constexpr int PB = PIPE >= 60 ? 6 : PIPE;
  constexpr bool FAST = PIPE >= 60;
  constexpr bool TREE = PIPE == 67 || PIPE == 72 || PIPE == 74;
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
      psum = r == 0 ? p : psum + p;  // p >= +0: the same sum without the leading 0 + p
      const __bf16 h = (__bf16)p;
      ph[r >> 3][r & 7] = h;
      pl[r >> 3][r & 7] = (__bf16)(p - (float)h);
    }
    return psum;
  };
  // PIPE 72: tile kt's exp / split and tile kt+1's S MFMAs in one hand-ordered stream — per
  // 16-d step: that step's K fragments, its 3 MFMAs, then a quarter of the exp / split (4 of the
  // lane's 16 scores) — so one wave feeds both pipes instead of relying on another wave's phase
  auto exp_s_fused = [&](floatx16& s, float m_new, bf16x8 (&ph)[2], bf16x8 (&pl)[2],
                         const unsigned char* stk, floatx16& sn) {
    float psum = 0.f;
    const unsigned char* kr = stk + li * P::RB;
    // the swizzled chunk offsets from an opaque row index: recomputed per tile (2 VALU per read)
    // rather than held in 8 loop-invariant registers
    int kli = li;
    asm volatile("" : "+v"(kli));
    bf16x8 kh[2], kl[2];
    auto kread = [&](int ks, int b) {
      const int d0 = 16 * ks + 8 * lh;
      kh[b] = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(kli, chunk_of<NP>(0, d0)) * 16);
      if (TERMS == 3)
        kl[b] = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(kli, chunk_of<NP>(1, d0)) * 16);
    };
    kread(0, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int b = ks & 1;
      if (ks + 1 < 4) kread(ks + 1, b ^ 1);
      if (TERMS == 3) {
        sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[b], qh[ks], ks == 0 ? floatx16{} : sn, 0, 0, 0);
        sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[b], ql[ks], sn, 0, 0, 0);
        sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[b], qh[ks], sn, 0, 0, 0);
      } else {
        sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[b], qh[ks], ks == 0 ? floatx16{} : sn, 0, 0, 0);
      }
#pragma unroll
      for (int r = 4 * ks; r < 4 * ks + 4; ++r) {
        const float pr = __builtin_amdgcn_exp2f(s[r] - m_new);
        psum += pr;
        const __bf16 h = (__bf16)pr;
        ph[r >> 3][r & 7] = h;
        pl[r >> 3][r & 7] = (__bf16)(pr - (float)h);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return psum;
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
      __builtin_amdgcn_s_barrier();
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
      {
        float mt = -INFINITY;
        if (!HAS_MASK && (kt + 1) * KT <= len) {
          if constexpr (TREE) {
            float a[6];
#pragma unroll
            for (int r = 0; r < 5; ++r) a[r] = max_nc(s_cur[3 * r], max_nc(s_cur[3 * r + 1], s_cur[3 * r + 2]));
            a[5] = s_cur[15];
            mt = max_nc(max_nc(a[0], max_nc(a[1], a[2])), max_nc(a[3], max_nc(a[4], a[5])));
          } else {
#pragma unroll
            for (int r = 0; r < 16; r += 2) mt = fmaxf(mt, fmaxf(s_cur[r], s_cur[r + 1]));
          }
        } else {
          uint32_t mb = 0xffffffffu;
          if constexpr (HAS_MASK)
            mb = *reinterpret_cast<const uint32_t*>(lds + MASK_OFF + (R % 3) * 1024 + wave * 256 + 4 * li);
          // PIPE 74 (masked launches): a full tile whose mask words are all ones for every query
          // of the wave (GraphCodeBERT's code rows over code keys) takes the tree max with no
          // per-key select — the same scores, so the same bits
          if (PIPE == 74 && (kt + 1) * KT <= len && __all(mb == 0xffffffffu)) {
            float a[6];
#pragma unroll
            for (int r = 0; r < 5; ++r) a[r] = max_nc(s_cur[3 * r], max_nc(s_cur[3 * r + 1], s_cur[3 * r + 2]));
            a[5] = s_cur[15];
            mt = max_nc(max_nc(a[0], max_nc(a[1], a[2])), max_nc(a[3], max_nc(a[4], a[5])));
          } else {
            // the lane half's 4-key offset taken out once per tile, so every per-key bit position
            // and bound below is a compile-time constant (no 16 per-lane shift amounts held
            // across the loop)
            const uint32_t mbh = mb >> (4 * lh);
            const int lim = len - kt * KT - 4 * lh;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int k0 = mfma32_row(r, 0);
              // absent keys -inf; keys the mask excludes the most negative finite float (HF's
              // additive finfo.min mask), as tile_max
              const bool in = k0 < lim;
              s_cur[r] = !in ? -INFINITY : (((mbh >> k0) & 1u) ? s_cur[r] : -FLT_MAX);
              mt = max_nc(mt, s_cur[r]);
            }
          }
        }
        if constexpr (FAST) {
          // lanes l and l ^ 32 hold the two halves of a query's keys: swap the halves on the VALU
          const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, mt),
                                                          __builtin_bit_cast(uint32_t, mt), false, false);
          mt = max_nc(__builtin_bit_cast(float, (uint32_t)sw[0]), __builtin_bit_cast(float, (uint32_t)sw[1]));
        } else {
          mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        }
        grow = __any(mt > m_run + 8.f);
        m_new = grow ? max_nc(m_run, mt) : m_run;
        alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 1 when m_new == m_run; 0 from -inf
      }
      // PIPE 72: the rare O rescale BEFORE the region, so no branch separates tile kt's exp /
      // split from tile kt+1's S MFMAs and this tile's PV (in PIPE 67 the compiler sinks the exp /
      // split past the rescale branch, leaving the 12 S MFMAs back to back and the VALU chained
      // into the PV MFMAs that consume it; that reorder alone, round-4 loop 69, measured 225.8 vs
      // 184.9 us, and at two workgroups per CU, loop 70, 190.9: profiles/r4g_attn_ab.jsonl)
      if (PIPE == 72 && grow) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      }
      bf16x8 ph[2], pl[2];
      __builtin_amdgcn_sched_barrier(0);
      float psum;
      if constexpr (PIPE == 72) {
        psum = exp_s_fused(s_cur, m_new, ph, pl, lds + KS_NEXT, s_next);
      } else {
        psum = exp_split(s_cur, m_new, ph, pl);
        s_mfma(lds + KS_NEXT, s_next);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      l_run = l_run * alpha + psum;
      m_run = m_new;
      if (PIPE != 72 && grow) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
      }
      pv_mfma(lds + VS_CUR, ph, pl);
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
      __builtin_amdgcn_sched_barrier(0);
      const float psum = exp_split(s_cur, m_new, ph, pl);
      s_mfma(lds + kslot(kt + 1), s_next);
      // the K fragment reads first, then one S MFMA per few vector instructions
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      l_run = l_run * alpha + psum;
      m_run = m_new;
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
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

// PIPE 80: two 32-query blocks per wave (64 queries: block A = the 4-wave loops' wave 2w, block B
// = wave 2w + 1), two waves per workgroup (the same 128-query blocks), four workgroups per CU, so
// two waves per SIMD within 256 registers.  One wave's instruction stream interleaves the blocks:
// S_A, then S_B under block A's row max / exp / split, then PV_A under block B's, then PV_B — the
// K and V fragments each serve both blocks (half the LDS reads per MFMA), and every block's
// arithmetic is PIPE 6's (same MFMA order, tile max, deferred rescale, exp / split and row sum),
// so the context is bit-identical.  K and V in 2-slot rings (tile kt + 2 issued once every wave
// has finished tile kt), 32 KiB per workgroup.  No mask path (masked launches run PIPE 66).
template <int NP, bool PLANES, int NW, bool QLDS, int NS, int DIAG = 0, bool KH = false>
__global__ __launch_bounds__(64 * NW, 2) void attn_pq_kernel(const unsigned short* __restrict__ qkvp,
                                                          float* __restrict__ out,
                                                          unsigned short* __restrict__ op,
                                                          const int* __restrict__ cu,
                                                          const int* __restrict__ q_rows) {
  using P = PPL<NP>;
  constexpr int TERMS = NP == 2 ? 3 : 1;
  constexpr int QB = 64 * NW;                        // queries per workgroup
  constexpr int DM = KT / P::ROWS_PER_DMA / NW;      // DMA instructions per wave per matrix tile
  // QLDS: the Q lo-plane fragments in LDS (1 KiB per wave, block and 16-d step, lane-major) instead
  // of 32 registers, past the K / V rings
  constexpr bool QL = QLDS && TERMS == 3;
  constexpr int QOFF = 2 * NS * P::TILE;  // NS K slots, then NS V slots
  constexpr int RING_Q = QOFF + (QL ? NW * 8 * 1024 : 0);
  constexpr int LDS_BYTES = RING_Q > NW * 32 * 66 * 4 ? RING_Q : NW * 32 * 66 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QB >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  constexpr size_t LDR = (size_t)NP * QKV_COLS;

  // Q fragments of both blocks (pre-scaled; B operand: B[k = d][j = q])
  bf16x8 qh[2][4], ql[2][QL ? 1 : 4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int q = qb * QB + wave * 64 + b * 32 + li;
    const int qr = q < nq ? q : nq - 1;
    const unsigned short* qp = qkvp + (size_t)(start + qr) * LDR + (size_t)head * 64 * NP;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int d = 16 * s + 8 * lh;
      const int off = (d >> 5) * 32 * NP + (d & 31);
      qh[b][s] = *reinterpret_cast<const bf16x8*>(qp + off);
      if constexpr (QL) {
        *reinterpret_cast<bf16x8*>(lds + QOFF + ((wave * 2 + b) * 4 + s) * 1024 + lane * 16) =
            *reinterpret_cast<const bf16x8*>(qp + off + 32);
      } else if (TERMS == 3) {
        ql[b][s] = *reinterpret_cast<const bf16x8*>(qp + off + 32);
      }
    }
  }

  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
  const int dr = lane / P::CR, dc = lane % P::CR;
  // K_j in slot j & 1, V_j in slot 2 + (j & 1)
  // per-lane byte offset of DMA instruction j's chunk from the tile's first token row (K: isv 0),
  // recomputed per issue (outside the MFMA regions) rather than held in 2·DM registers
  auto voff = [&](int isv, int j) {
    const int r = (wave * DM + j) * P::ROWS_PER_DMA + dr;
    return 2u * ((uint32_t)r * (uint32_t)LDR + ((1 + isv) * AE_HIDDEN + head * 64) * NP +
                 (isv ? vpos<NP>(r, dc) : kpos<NP>(r, dc)) * 8);
  };
  const unsigned char* sbase = reinterpret_cast<const unsigned char*>(qkvp + (size_t)start * LDR);
  auto issue = [&](int kt, int isv) {
    const unsigned char* sb = sbase + (size_t)kt * KT * LDR * 2;
    const uint32_t dst = lds0 + (uint32_t)((isv * NS + kt % NS) * P::TILE);
    if ((kt + 1) * KT <= len) {
#pragma unroll
      for (int j = 0; j < DM; ++j) dma16s(voff(isv, j), sb, dst + (wave * DM + j) * 1024);
    } else {  // key rows past the sequence re-read its last row (finite, masked to -inf)
      const int last = len - 1 - kt * KT;
#pragma unroll
      for (int j = 0; j < DM; ++j) {
        const int over = (wave * DM + j) * P::ROWS_PER_DMA + dr - last;
        const uint32_t v = voff(isv, j) - (over > 0 ? (uint32_t)over * (uint32_t)(LDR * 2) : 0u);
        dma16s(v, sb, dst + (wave * DM + j) * 1024);
      }
    }
  };
  auto barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // wait until at most nt tiles (2·DM DMA instructions each) of this wave are in flight
  auto wait_tiles = [](int nt) {
    if (nt >= 2) wait_vm_n<4 * DM>();
    else if (nt == 1) wait_vm_n<2 * DM>();
    else wait_vm_n<0>();
  };

  floatx16 o[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) { o[b][0][r] = 0.f; o[b][1][r] = 0.f; }
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  // O_b^T += V^T P_b^T for key step t, d tile dt (PIPE 6's order: t outer, dt inner)
  auto pv_step = [&](const unsigned char* stv, int ln, int b, int t, int dt, const bf16x8 (&ph)[2],
                     const bf16x8 (&pl)[2]) {
    {
      const int k0 = 16 * t + 4 * (ln >> 5);
      const int kq = k0 + ((ln >> 2) & 3);
      {
        const int col = dt * 32 + 16 * ((ln >> 4) & 1) + 4 * (ln & 3);
        const int cb = (col & 7) * 2;
        const unsigned char* va = stv + kq * P::RB + cb;
        const unsigned char* vb = stv + (kq + 8) * P::RB + cb;
        bf16x8 vh, vl;
        if (DIAG == 1) {
          asm volatile("" : "=v"(vh), "=v"(vl));
        } else {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(0, col)) * 16));
          const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(0, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = c[e]; }
        }
        if (TERMS == 3 && DIAG != 1) {
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(va + vpos<NP>(kq, chunk_of<NP>(1, col)) * 16));
          const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(vb + vpos<NP>(kq + 8, chunk_of<NP>(1, col)) * 16));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vl[e] = a[e]; vl[4 + e] = c[e]; }
        }
        floatx16& oo = o[b][dt];
        if (TERMS == 3) {
          oo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph[t], oo, 0, 0, 0);
          oo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl[t], oo, 0, 0, 0);
        }
        oo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph[t], oo, 0, 0, 0);
      }
    }
  };
  // block b's tile max (absent keys -inf), deferred-rescale decision, P = exp2(S - m) split into
  // bf16 hi / lo, and the row sum — PIPE 67's arithmetic; the O rescale is left to the caller
  // block b's tile max (absent keys -inf) and the deferred-rescale decision (PIPE 67's
  // arithmetic): the reference max m_new and alpha = exp2(m_run - m_new)
  auto tile_max = [&](auto fc, int kt, int b, floatx16& s, float& m_new, float& alpha, bool& grow) {
    float mt = -INFINITY;
    if constexpr (decltype(fc)::value) {  // full tile (compile-time: no branch in the region)
      float a[6];
#pragma unroll
      for (int r = 0; r < 5; ++r) a[r] = max_nc(s[3 * r], max_nc(s[3 * r + 1], s[3 * r + 2]));
      a[5] = s[15];
      mt = max_nc(max_nc(a[0], max_nc(a[1], a[2])), max_nc(a[3], max_nc(a[4], a[5])));
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool in = kt * KT + mfma32_row(r, lh) < len;
        s[r] = in ? s[r] : -INFINITY;
        mt = max_nc(mt, s[r]);
      }
    }
    const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, mt),
                                                    __builtin_bit_cast(uint32_t, mt), false, false);
    mt = max_nc(__builtin_bit_cast(float, (uint32_t)sw[0]), __builtin_bit_cast(float, (uint32_t)sw[1]));
    grow = __any(mt > m_run[b] + 8.f);
    // m_new = grow ? max(m_run, mt) : m_run as a bit select on the uniform grow mask: a select on
    // a wave-uniform condition becomes a branch, which would end the scheduling region here
    const uint32_t gm = 0u - (uint32_t)grow;
    m_new = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, max_nc(m_run[b], mt)) & gm) |
                                          (__builtin_bit_cast(uint32_t, m_run[b]) & ~gm));
    alpha = __builtin_amdgcn_exp2f(m_run[b] - m_new);
  };
  // P = exp2(S - m_new) for scores r0 .. r1 - 1, split into bf16 hi / lo, summed in r order
  auto exp_split = [&](const floatx16& s, float m_new, int r0, int r1, bf16x8 (&ph)[2],
                       bf16x8 (&pl)[2], float& psum) {
    if constexpr (DIAG == 3) {  // timing diagnostic: S's bits as P, no exp / split
      if (r0 == 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ph[h] = __builtin_bit_cast(bf16x8, floatx4{s[8 * h], s[8 * h + 1], s[8 * h + 2], s[8 * h + 3]});
          pl[h] = __builtin_bit_cast(bf16x8, floatx4{s[8 * h + 4], s[8 * h + 5], s[8 * h + 6], s[8 * h + 7]});
        }
        psum = s[0];
      }
      return;
    }
#pragma unroll
    for (int r = r0; r < r1; ++r) {
      const float p = __builtin_amdgcn_exp2f(s[r] - m_new);
      psum = r == 0 ? p : psum + p;
      const __bf16 h = (__bf16)p;
      ph[r >> 3][r & 7] = h;
      pl[r >> 3][r & 7] = (__bf16)(p - (float)h);
    }
  };
  // the 16-d K fragments of step ks (lane li: key row li)
  auto kread = [&](const unsigned char* stk, int ln, int ks, bf16x8& kh, bf16x8& kl) {
    if constexpr (DIAG == 1) {  // timing diagnostic: opaque register values, no LDS read
      asm volatile("" : "=v"(kh), "=v"(kl));
      return;
    }
    const int kli = ln & 31;
    const unsigned char* kr = stk + kli * P::RB;
    const int d0 = 16 * ks + 8 * (ln >> 5);
    kh = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(kli, chunk_of<NP>(0, d0)) * 16);
    if (TERMS == 3) kl = *reinterpret_cast<const bf16x8*>(kr + kpos<NP>(kli, chunk_of<NP>(1, d0)) * 16);
  };
  auto s_step = [&](int b, int ks, const bf16x8& kh, const bf16x8& kl, floatx16& s) {
    if (TERMS == 3) {
      bf16x8 qlf;
      if (DIAG == 1 && QL) asm volatile("" : "=v"(qlf));
      else qlf = QL ? *reinterpret_cast<const bf16x8*>(lds + QOFF + ((wave * 2 + b) * 4 + ks) * 1024 + lane * 16)
                            : ql[b][QL ? 0 : ks];
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[b][ks], ks == 0 ? floatx16{} : s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qlf, s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[b][ks], s, 0, 0, 0);
    } else {
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[b][ks], ks == 0 ? floatx16{} : s, 0, 0, 0);
    }
  };
  // scores of block A's softmax chunk c (c = 1..3 after the tile max in chunk 0)
  constexpr int CH[5] = {0, 0, 6, 11, 16};

  const int nkt = (len + KT - 1) / KT;
  // prologue: tiles 0 .. NS-1 (as many as exist); tile 0 waited for
#pragma unroll
  for (int j = 0; j < NS; ++j)
    if (j < nkt) {
      issue(j, 0);
      issue(j, 1);
    }
  wait_tiles(min(nkt, NS) - 1);
  barrier();
  auto body = [&](auto rc, auto fc, int kt) {
    constexpr int R = decltype(rc)::value;
    const unsigned char* stk = lds + R * P::TILE;
    const unsigned char* stv = lds + (NS + R) * P::TILE;
    floatx16 sa, sb;
    bf16x8 pha[2], pla[2], phb[2], plb[2];
    bf16x8 kh[2], kl[2];
    float ma, mb, aa, ab, psa = 0.f, psb = 0.f;
    bool ga, gb;
    // the lane index through an opaque copy: the swizzled LDS addresses are recomputed per tile
    // (a few VALU) instead of held in loop-invariant registers the two blocks' state needs
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // S_A (matrix pipe only; the other wave on the SIMD fills the VALU).  KH: the tile's K
    // fragments read once into 32 registers for both blocks, else read again for S_B
    bf16x8 kall[KH ? 4 : 1][2];
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (KH) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) kread(stk, ln, ks, kall[ks][0], kall[ks][1]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s_step(0, ks, kall[ks][0], kall[ks][1], sa);
    } else {
      kread(stk, ln, 0, kh[0], kl[0]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (ks + 1 < 4) kread(stk, ln, ks + 1, kh[(ks + 1) & 1], kl[(ks + 1) & 1]);
        s_step(0, ks, kh[ks & 1], kl[ks & 1], sa);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // S_B under block A's tile max (step 0) and exp / split (steps 1-3), fenced per step
    if (!KH) kread(stk, ln, 0, kh[0], kl[0]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (!KH && ks + 1 < 4) kread(stk, ln, ks + 1, kh[(ks + 1) & 1], kl[(ks + 1) & 1]);
      if constexpr (KH) s_step(1, ks, kall[ks][0], kall[ks][1], sb);
      else s_step(1, ks, kh[ks & 1], kl[ks & 1], sb);
      if (ks == 0) tile_max(fc, kt, 0, sa, ma, aa, ga);
      else exp_split(sa, ma, CH[ks], CH[ks + 1], pha, pla, psa);
      __builtin_amdgcn_sched_barrier(0);
    }
    // pin block A's P fragments before the rescale branch: without a use here the compiler sinks
    // the whole exp / split past it, out of the region it shares with S_B's MFMAs
    asm volatile("" ::"v"(pha[0]), "v"(pha[1]), "v"(pla[0]), "v"(pla[1]), "v"(psa));
    l_run[0] = l_run[0] * aa + psa;
    m_run[0] = ma;
    if (ga) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o[0][0][r] *= aa; o[0][1][r] *= aa; }
    }
    __builtin_amdgcn_sched_barrier(0);
    // PV_A under block B's tile max and exp / split, fenced per (key step, d tile)
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      pv_step(stv, ln, 0, st >> 1, st & 1, pha, pla);
      if (st == 0) tile_max(fc, kt, 1, sb, mb, ab, gb);
      else exp_split(sb, mb, CH[st], CH[st + 1], phb, plb, psb);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" ::"v"(phb[0]), "v"(phb[1]), "v"(plb[0]), "v"(plb[1]), "v"(psb));
    l_run[1] = l_run[1] * ab + psb;
    m_run[1] = mb;
    if (gb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o[1][0][r] *= ab; o[1][1][r] *= ab; }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int st = 0; st < 4; ++st) pv_step(stv, ln, 1, st >> 1, st & 1, phb, plb);
    // tile kt + 1 landed (tiles kt + 2 .. kt + NS - 1 stay in flight); every wave is done with
    // slot R: tile kt + NS into it
    if (DIAG != 2 && DIAG != 4) {
      wait_tiles(min(nkt - 1, kt + NS - 1) - kt - 1);
      barrier();
    }
    if (DIAG != 4 && kt + NS < nkt) {
      issue(kt + NS, 0);
      issue(kt + NS, 1);
    }
  };
  // the last tile, when partial, runs the per-key select form of the tile max
  const int nfull = len / KT;
  using T0 = std::integral_constant<int, 0>;
  using T1 = std::integral_constant<int, 1>;
  using T2 = std::integral_constant<int, NS == 3 ? 2 : 0>;
  using FULL = std::true_type;
  using PART = std::false_type;
  for (int kt = 0; kt < nkt; kt += NS) {
    if (kt < nfull) body(T0(), FULL(), kt);
    else body(T0(), PART(), kt);
    if (kt + 1 >= nkt) break;
    if (kt + 1 < nfull) body(T1(), FULL(), kt + 1);
    else body(T1(), PART(), kt + 1);
    if constexpr (NS == 3) {
      if (kt + 2 >= nkt) break;
      if (kt + 2 < nfull) body(T2(), FULL(), kt + 2);
      else body(T2(), PART(), kt + 2);
    }
  }

  // epilogue: each block's O through the wave's LDS rows (66 floats), then 16-B stores
  constexpr int S6 = 66;
  float* os6 = reinterpret_cast<float*>(lds) + wave * 32 * S6;
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own rows: no barrier
    constexpr int CPR = PLANES ? 8 * NP : 16;
    constexpr int RPI = 64 / CPR;
    const int c = lane % CPR;
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int rr = it * RPI + lane / CPR;
      const int qq = qb * QB + wave * 64 + b * 32 + rr;
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
        const floatx2 e = *reinterpret_cast<const floatx2*>(src + 4 * c + 2);
        if (qq < nq)
          *reinterpret_cast<floatx4*>(out + (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + 4 * c) =
              floatx4{a.x, a.y, e.x, e.y};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // block A's rows read before B's land
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
  hipLaunchKernelGGL((attn_pp_kernel<N, M, PL, M ? (PIPE == 72 ? 72 : PIPE == 74 ? 74 : PIPE >= 60 ? 66 : 4) : (PIPE == 74 ? 67 : PIPE)>), grid, block, 0, \
                     stream, qkvp, out, op, cu,                                                 \
                     q_rows, mask, mask_L)
#define APP_MP(N)                                                      \
  if (op) {                                                            \
    if (mask) APP_LAUNCH(N, true, true); else APP_LAUNCH(N, false, true);   \
  } else {                                                             \
    if (mask) APP_LAUNCH(N, true, false); else APP_LAUNCH(N, false, false); \
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
#ifdef AE_TOOLS
// PIPE 80 (attn_pq_kernel): 4-wave workgroups of 256 queries, no mask
template <int NSL, int DIAG = 0, bool KH = false>
hipError_t apq_launch(const unsigned short* qkvp, float* out, unsigned short* op, const int* cu,
                      const int* q_rows, int max_q, int n, int heads, int np, hipStream_t stream) {
  if (n <= 0 || max_q <= 0) return hipSuccess;
  if (np != 1 && np != 2) return hipErrorInvalidValue;
  constexpr int NW = 4;
  dim3 grid((max_q + 64 * NW - 1) / (64 * NW), heads, n), block(64 * NW);
#define APQ(N, PL) hipLaunchKernelGGL((attn_pq_kernel<N, PL, NW, true, NSL, DIAG, KH>), grid, block, 0, stream, qkvp, out, op, cu, q_rows)
  if (np == 2) {
    if (op) APQ(2, true); else APQ(2, false);
  } else {
    if (op) APQ(1, true); else APQ(1, false);
  }
#undef APQ
  return hipGetLastError();
}
#endif  // AE_TOOLS
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
// profiles/r3as_attn_interleave_ab.jsonl): not kept.  Round 4: loop 73 — masked launches
// skipping key tiles no query of the wave attends (bit-identical to 66 when every row of the
// wave attends some key) — measured 347 vs 324 us on GraphCodeBERT-shaped masks and 352 vs 325
// on random ones at B=64 x L=640 (the if / else around the tile's work costs 38 registers and
// the schedule more than the skipped tiles return; tools/attn_bench.py --mask --mask-gcb): removed.
// Round 6: PIPE 74 = 67 for unmasked launches; masked launches run 66 with a fast path for full
// tiles whose mask words are all ones across the wave (the tree max, no per-key select) —
// bit-identical to 66 (test_attention_pp_masked_fast_path_bit_identical) and 3-5 % faster on
// GraphCodeBERT-shaped masks at B = 64 x L = 640 (302-306 vs 314-318 us; ragged 161.9 vs 174.0),
// neutral on random masks (226.4 vs 226.9), profiles/r6v_*, r6w_*.
constexpr int APP_PIPE = 74;
}  // namespace

extern "C" hipError_t ae_launch_attention_pp(const unsigned short* qkvp, float* out,
                                             unsigned short* op, const int* cu, const int* q_rows,
                                             int max_q, int n, int heads, const uint32_t* mask,
                                             int mask_L, int np, hipStream_t stream) {
  return app_launch<APP_PIPE>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np,
                              stream);
}

#ifdef AE_TOOLS
// Tools library only (-DAE_TOOLS, lib/libalert_engine_tools.so).
// Kernel experiments (tools/attn_bench.py, tests): 67 = the production loop, 66 = the same
// without the tree row max, 6 = the round-3 loop both restructure bit-identically (its mask
// launches run PIPE 4).  Earlier loops (0-5), the 8-wave ping-pong (7), 4 waves x 64 queries (8),
// 64-key tiles (9), the packed-pair exp (68) and the timing diagnostics 61-65 (results WRONG)
// were measured and removed (git history before round 4; numbers in DESIGN.md §3).
// (An XCD-aware workgroup order — the q-blocks of one (sequence, head) on one XCD — measured 2-3 %
// slower, profiles/r2i_attn_pp_ab.jsonl: the K/V re-reads are Infinity-Cache hits, not the bound.)
extern "C" hipError_t ae_bench_attention_pp(const unsigned short* qkvp, float* out,
                                            unsigned short* op, const int* cu, const int* q_rows,
                                            int max_q, int n, int heads, const uint32_t* mask,
                                            int mask_L, int np, int variant, hipStream_t stream) {
  switch (variant) {
    case 6: return app_launch<6>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 66: return app_launch<66>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 67: return app_launch<67>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 72: return app_launch<72>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 74: return app_launch<74>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream);
    case 80: return mask ? app_launch<67>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream)
                         : apq_launch<2>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    case 81: return mask ? app_launch<67>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream)
                         : apq_launch<3>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    // timing diagnostics of 81 (results WRONG): 82 no LDS fragment reads, 83 no end-of-tile wait /
    // barrier, 84 no exp / split, 85 no DMA after the prologue and no waits
    case 82: return apq_launch<3, 1>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    case 83: return apq_launch<3, 2>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    case 84: return apq_launch<3, 3>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    case 85: return apq_launch<3, 4>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    case 86: return mask ? app_launch<67>(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, stream)
                         : apq_launch<3, 0, true>(qkvp, out, op, cu, q_rows, max_q, n, heads, np, stream);
    default: break;
  }
  return hipErrorInvalidValue;
}
#endif  // AE_TOOLS
