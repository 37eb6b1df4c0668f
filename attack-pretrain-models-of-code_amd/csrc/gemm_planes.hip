// gemm_planes.hip — packed bf16-plane MFMA GEMM of the split-precision encoder
// (AE_PREC_BF16 / AE_PREC_F32X3).
//
// Operands arrive already split into bf16: the weights at engine creation (W = W_hi + W_lo), the
// activations by the kernel that produced them (the embedding LayerNorm, attention, the GEMM
// epilogues), so the
// main loop moves and multiplies nothing but bf16.  Packed layout ("NP planes per 128-B block"):
//   NP = 2 (f32x3): row = K/32 blocks of 128 B, block b = [hi of k 32b..32b+31 | lo of the same]
//   NP = 1 (bf16):  row = K bf16 (the hi plane)
// so one K-tile of a row is always one full 128-B cache line.  With NP = 2 every product is
//     a·w ≈ a_hi·w_hi + a_hi·w_lo + a_lo·w_hi          (3 bf16 MFMAs, f32 accumulate)
// from ONE load of the four planes.
//
// Two kernels, chosen per shape by ae_launch_gemm_packed: gemm_pp_kernel (256 x 256 tiles, every
// epilogue) and gemm_pp192_kernel (256 x 192 tiles for the N = 768 GEMMs: f32 epilogues and the
// residual + row-statistics epilogue of the folded LayerNorm).  Both:
//   * operands reach LDS by LDS-DMA (global_load_lds_dwordx4, one wave instruction = 8 rows x
//     128 B, lane-linear image); the 16-B chunk of row r is XOR-swizzled by (r >> 1) & 7 on the
//     SOURCE address, so fragment ds_read_b128s of 16 rows hit 16 different bank slots
//   * DMA issued from inline asm with hand-counted vmcnt (the compiler's wait-count pass would
//     otherwise drain it before every fragment read); raw s_barrier; XCD-aware tile order
//   * epilogues: +bias -> f32, +bias+residual -> f32, +bias -> tanh -> f32, +bias -> GELU -> packed
//     bf16 planes (the FFN2 operand), +bias -> packed planes (QKV), and the folded-LayerNorm pair:
//     the QKV / FFN1 GEMMs over the PRE-LayerNorm rows with the row's (mean, rstd) applied in the
//     epilogue (FoldArgs), the O-projection / FFN2 writing f32 + planes + per-tile row statistics
//     (StatArgs) — no LayerNorm pass over the rows and no exchange between workgroups
// The round-1 kernel (gemm_pk_kernel, one wave group, 2-3 stage ring), the role-split persistent
// kernel (gemm_pprs_kernel) and the two-workgroups-per-CU kernel (gemm_w2.hip) were measured
// slower and removed (git history before round 4; DESIGN.md §3 keeps their numbers).
#include <type_traits>

#include "common.h"


// m0 is written only by dma16 below; nothing else in these kernels reads it
#pragma clang diagnostic ignored "-Winline-asm"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// PK_EPI_BIAS_PACKED: +bias -> packed planes (the QKV output feeding attention_pp.hip); only the
// ping-pong 256 x 256 kernel has it
// PK_EPI_BIAS_FOLD / PK_EPI_GELU_FOLD: PK_EPI_BIAS_PACKED / PK_EPI_GELU_PACKED whose A operand is
// the PRE-LayerNorm row v of the previous residual add, with the LayerNorm folded into the GEMM
// (the QKV and FFN1 GEMMs of the encoder; see FoldArgs)
// PK_EPI_RES_STATS: +bias +residual -> f32 + packed planes + per-tile row statistics;
// PK_EPI_RES_STATS_LN: the same with the residual a pre-LayerNorm row, normalised on the fly
// (see StatArgs; 256 x 192 kernel only).  (Round 4's PK_EPI_RES_LN = 5 — residual + LayerNorm
// inside the O-projection / FFN2 epilogue, the 4 column tiles of a row block exchanging row
// statistics as co-resident workgroups — was replaced by the folded form in round 5: DESIGN.md §3.)
enum { PK_EPI_BIAS = 0, PK_EPI_GELU_PACKED = 1, PK_EPI_RES = 2, PK_EPI_TANH = 3, PK_EPI_BIAS_PACKED = 4,
       PK_EPI_GELU_FOLD = 6, PK_EPI_BIAS_FOLD = 7, PK_EPI_RES_STATS = 8, PK_EPI_RES_STATS_LN = 9 };

// (mean, M2) of a row segment: M2 = sum of squared deviations from the segment mean
struct RowStat {
  float mean, m2;
};

// LayerNorm folded into the following GEMM.  With x = LN(v) = (v - mean) * rstd * g + b,
//   x·W^T + bias = rstd * (v·W'^T - mean * s) + bias'
// where W' = W with column k scaled by g[k], s[n] = sum_k W'[n][k] and bias' = bias + W·b (all
// prepared at engine creation), so the GEMM multiplies the pre-LayerNorm rows v directly and the
// epilogue applies the row's (mean, rstd) — merged from the 4 per-tile statistics the producing
// PK_EPI_RES_STATS epilogue wrote.  No LayerNorm pass over the rows.
//
// Plane shift: the producer splits v - kappa into the planes (kappa = its bias plus the LayerNorm
// shift b of its residual: the per-column constant part of v, StatArgs::shift), so the split's
// rounding scales with |v - kappa| — the row's spread — and not with a common row offset or a
// per-column outlier constant.  The consumer starts its accumulators at kc[n] = sum_k kappa[k] ·
// W'[n][k] (W' as its planes hold it; FoldArgs::kc), so acc = v·W'^T still.
struct FoldArgs {
  const float* s;          // [N]
  const uint64_t* stats;   // [M rows][4] RowStat of the 4 192-column tiles of each row
  float eps;
  const float* kc;         // [N] or null: the accumulator start (plane shift of the A rows)
};

// (mean, rstd) of a 768-wide row from its 4 tile statistics (n = 192 each), merged as (0,1),
// (2,3), then the halves — the order every consumer uses, so every kernel gets the same bits
__device__ __forceinline__ void row_norm(const uint64_t* st, float eps, float& mean, float& rstd) {
  RowStat p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = __builtin_bit_cast(RowStat, st[q]);
  const float d01 = p[0].mean - p[1].mean, d23 = p[2].mean - p[3].mean;
  const float m01 = (p[0].mean + p[1].mean) * 0.5f, m23 = (p[2].mean + p[3].mean) * 0.5f;
  const float q01 = (p[0].m2 + p[1].m2) + 96.f * d01 * d01;
  const float q23 = (p[2].m2 + p[3].m2) + 96.f * d23 * d23;
  const float d = m01 - m23;
  mean = (m01 + m23) * 0.5f;
  const float var = ((q01 + q23) + 192.f * d * d) * (1.f / 768.f);
  rstd = rsqrtf(var + eps);
}

// Arguments of the PK_EPI_RES_STATS(_LN) epilogue (gemm_pp192_kernel).
struct StatArgs {
  const float* gamma;      // _LN: the residual's LayerNorm gain / shift
  const float* beta;
  float eps;
  __bf16* xp;              // packed planes of v - shift ([M][NP * N])
  uint64_t* stats;         // [M][4] RowStat of each output row over each 192-column tile
  const uint64_t* rstats;  // _LN: the residual's own tile statistics
  const float* shift;      // [N] or null: kappa, subtracted from v before the plane split
};

namespace {
constexpr int PK_ROWB = 128;

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

}  // namespace

// keeps a value live in a diagnostic build whose consumer was cut out (rule 17)
__device__ __forceinline__ void keep_f32(float x) { asm volatile("" ::"v"(x)); }

// 16-B chunk swizzle of row r of an epilogue staging region (gemm_pp_kernel): rows r and r + 16
// land on different banks
__device__ __forceinline__ int pk_swz(int r) { return (r & 15) ^ (((r >> 4) & 1) << 3); }

// element offset of (row, col) in a packed [rows][NP*ld] matrix, plane p
__device__ __forceinline__ size_t pk_index(int row, int col, int ld, int np, int p) {
  return (size_t)row * np * ld + (size_t)(col >> 5) * 32 * np + 32 * p + (col & 31);
}

// ------------------------------------------------------------------------------------------
// Ping-pong 256 x 256 packed GEMM (gemm_pp_kernel).
//
// The main loop is built so that a SIMD's matrix pipe is fed by one wave while its other wave
// moves data:
//   * 8 waves = two groups of four (wave w sits on SIMD w % 4, so each SIMD holds one wave of
//     each group); group g owns rows 128 g .. 128 g + 127 of the tile, wave (g, wn) a 128 x 64
//     block.  Group 1 executes one extra s_barrier before the loop, so between any two barriers
//     one group runs MFMAs while the other reads fragments and issues DMA (and vice versa).
//   * a 128-B K-tile (NP 2: 32 k of hi | lo; NP 1: 64 k) is consumed in four phases, one
//     64 x 32 quadrant of the wave's block each: (m-half 0, n-half 0) reading A(mh 0) and
//     W(nh 0); (0, 1) reading W(nh 1); (1, 1) reading A(mh 1); (1, 0) reading nothing.
//   * two 64-KiB LDS stages (K-tiles kt and kt+1).  K-tile kt+2 goes into kt's stage one
//     quarter per phase (2 DMA pieces per wave each, issued between the wave's own MFMAs of the
//     phase, where their issue cost hides), every quarter >= 2 phases after its last
//     LDS read: A(mh 0) at phase 2 and W(nh 0) at phase 3 of kt, W(nh 1) at phase 0 and A(mh 1)
//     at phase 1 of kt+1.  Each quarter is waited for (counted vmcnt(6), never 0 in steady
//     state) one phase before the phase that reads it, so a barrier separates every issuer's
//     wait from the read — what the staggered groups need.  (A deeper ring — 10 quarter slots
//     in 160 KiB, quarters DMA'd 8 phases ahead — measured 3-7 % slower: DMA latency is not
//     what bounds this loop; nor do two phases per K-tile (half the barriers) help.)
//   * measured (tools/gemm_bench.py, DIAG 7 = the same MFMAs with no barrier, read or DMA):
//     the matrix pipe alone sustains ~1.86 GHz-equivalent under this load (spec peak assumes
//     2.4 GHz); the full main loop runs at 84-87 % of that MFMA-only time.
//   * the MFMA computes the transposed product D^T = W·A^T, so lane l holds 4 consecutive
//     output columns of output row l % 32 per register quad.  The epilogue writes them (after
//     bias / GELU / plane split) into the free LDS as the output's own byte image, one 64-row
//     half of the wave's block at a time, then copies whole 256-B row segments out with 16-B
//     lanes (+ residual / tanh on the coalesced side).
namespace {
template <int N>
__device__ __forceinline__ void pp_wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
}  // namespace

// DIAG (timing experiments only, through ae_bench_gemm_packed; results WRONG): 1 = no DMA after
// the prologue, 2 = no MFMAs, 3 = no fragment reads after K-tile 0, 4 = no epilogue, 5 = no
// vmcnt waits in the loop, 6 = MFMAs + barriers only (no DMA / reads / waits after K-tile 0),
// 7 = MFMAs only (6 without barriers); 8 = plain (not non-temporal) epilogue stores, results
// exact; 9 (PP_PERSIST) = the production kernel on a persistent grid, results exact (measured
// FFN1 392.5 -> 397.9 us, QKV 295.8 -> 291.1 us, profiles/r3q_gemm_persistent_ab.jsonl: workgroup
// turnover is not what the epilogue costs, so the production grid stays one workgroup per
// tile).  Production instantiations have DIAG = 0.
template <int NP, int EPI, int DIAG>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ R, float* __restrict__ C, __bf16* __restrict__ Cp, int M, int N,
    int K, int group_m, FoldArgs fold) {
  extern __shared__ __attribute__((aligned(16))) unsigned char pk_smem[];
  constexpr int BM = 256, BN = 256, ROWB = PK_ROWB;
  constexpr int A_BYTES = BM * ROWB, STAGE = (BM + BN) * ROWB;  // 64 KiB per K-tile
  constexpr int KB = 64 / NP;                                     // k per K-tile
  constexpr int NS = KB / 16;                                     // 16-deep MFMA steps
  constexpr int T = NP == 2 ? 3 : 1;                              // MFMAs per product

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  constexpr bool FOLD_EPI = EPI == PK_EPI_GELU_FOLD || EPI == PK_EPI_BIAS_FOLD;
  // persistent when the grid is smaller than the tile count (pp_launch): workgroup w takes the
  // virtual blocks w, w + grid, ... — the same tiles, XCD and order as one block per tile — so a
  // CU goes from one tile's epilogue straight into the next tile's prologue, with no workgroup
  // retire / dispatch between them
  for (int vb = blockIdx.x; vb < tiles_m * tiles_n; vb += gridDim.x) {
  const int t = xcd_remap(vb, tiles_m * tiles_n);
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm0 = first_m + (t - g * per_group) % gsize, tn0 = (t - g * per_group) / gsize;
  const int m0 = tm0 * BM, n0 = tn0 * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // group = wm
  const int li = lane & 31, lh = lane >> 5;
  const size_t lda = (size_t)NP * K;

  // ---- DMA pieces (8 rows x 128 B each): per K-tile every wave issues 8, as 4 quarters:
  // [0,1] A(mh 0) rows {0..63, 128..191}, [2,3] W(nh 0) rows {64 q + 0..31},
  // [4,5] W(nh 1) rows {64 q + 32..63}, [6,7] A(mh 1) rows {64..127, 192..255}
  const char* src[8];
  uint32_t dst[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int pidx = 2 * wave + (j & 1);  // 0..15 within the quarter
    const bool is_a = j < 2 || j >= 6;
    const int r0 = is_a ? (pidx >> 3) * 128 + (pidx & 7) * 8 + (j >= 6 ? 64 : 0)
                        : (pidx >> 2) * 64 + (pidx & 3) * 8 + (j >= 4 ? 32 : 0);
    const int r = r0 + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    if (is_a) {
      const int gr = m0 + r < M ? m0 + r : M - 1;
      src[j] = reinterpret_cast<const char*>(A + gr * lda) + 16 * cs;
      dst[j] = r0 * ROWB;
    } else {
      const int gr = n0 + r < N ? n0 + r : N - 1;
      src[j] = reinterpret_cast<const char*>(W + gr * lda) + 16 * cs;
      dst[j] = A_BYTES + r0 * ROWB;
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)pk_smem;
  const int nk = K / KB;
  auto issue = [&](int q, int kt) {  // quarter q (pieces 2q, 2q+1) of K-tile kt
    dma16(src[2 * q] + (size_t)kt * ROWB, lds0 + (kt & 1) * STAGE + dst[2 * q]);
    dma16(src[2 * q + 1] + (size_t)kt * ROWB, lds0 + (kt & 1) * STAGE + dst[2 * q + 1]);
  };


  floatx16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int sw = (li >> 1) & 7;  // fragment rows are 32-aligned + li
  const int a_row = (wm * 128 + li) * ROWB;
  const int w_row = A_BYTES + (wn * 64 + li) * ROWB;
  bf16x8 fa[2][NS][NP];   // A fragments of the current m-half: [tm in half][step][plane]
  bf16x8 fw[2][NS][NP];   // W fragments: [n-half][step][plane]

  auto read_a = [&](const unsigned char* st, int mh, int kt) {
    if ((DIAG == 3 || DIAG == 6 || DIAG == 7) && kt > 0) return;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          fa[tt][s][p] = *reinterpret_cast<const bf16x8*>(
              st + a_row + (2 * mh + tt) * 32 * ROWB + 16 * ((4 * p + 2 * s + lh) ^ sw));
  };
  auto read_w = [&](const unsigned char* st, int nh, int kt) {
    if ((DIAG == 3 || DIAG == 6 || DIAG == 7) && kt > 0) return;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        fw[nh][s][p] = *reinterpret_cast<const bf16x8*>(
            st + w_row + nh * 32 * ROWB + 16 * ((4 * p + 2 * s + lh) ^ sw));
  };
  // a quadrant's MFMAs; DMA quarter q of K-tile kd (if dma) rides in the MFMA issue gaps —
  // one piece after each third of the MFMAs — instead of in the load section (measured: the
  // glds issue cost then hides behind the matrix pipe; in the load section it serialises)
  auto mfma_quad = [&](int mh, int nh, auto qc, bool dma, int kd) {
    constexpr int q = decltype(qc)::value;
    constexpr int NM = NS * 2 * T;  // MFMAs of the quadrant
    if (DIAG == 2) {
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          asm volatile("" ::"v"(fw[nh][s][p]));
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) asm volatile("" ::"v"(fa[tt][s][p]));
        }
      if (dma) issue(q, kd);
      return;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int s = i / (2 * T), tt = (i / T) % 2, term = i % T;
      floatx16& c = acc[2 * mh + tt][nh];
      const bf16x8& x = (T == 3 && term == 1) ? fw[nh][s][NP - 1] : fw[nh][s][0];
      const bf16x8& y = (T == 3 && term == 0) ? fa[tt][s][NP - 1] : fa[tt][s][0];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
      if (DIAG != 1 && DIAG != 6 && DIAG != 7 && dma && (i == NM / 3 - 1 || i == 2 * NM / 3 - 1)) {
        const int j = 2 * q + (i == NM / 3 - 1 ? 0 : 1);
        __builtin_amdgcn_sched_barrier(0);
        dma16(src[j] + (size_t)kd * ROWB, lds0 + (kd & 1) * STAGE + dst[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // end of a load section: the fragment reads retire before the MFMAs that use them
  auto sync_compute = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    if (DIAG != 7) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_load = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    if (DIAG != 7) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // folded LayerNorm: the epilogue's side data — bias' and s of the tile's 256 columns (2 KiB)
  // and the 4 tile statistics of its 256 rows (8 KiB) — moved into LDS past the stages by
  // LDS-DMA ahead of the prologue (waves 0-4, two 1-KiB pieces each).  They are older than every
  // K-tile piece, so the counted waits below cover them; the epilogue reads them at LDS latency.
  constexpr uint32_t SIDE = 2 * STAGE;  // byte offset of [bias' 256 | s 256] then [256 rows][4] u64
  if constexpr (FOLD_EPI) {
    if (wave == 0) {
      const int c = min(n0 + 4 * lane, N - 4);
      dma16(bias + c, lds0 + SIDE);
      dma16(fold.s + c, lds0 + SIDE + 1024);
    } else if (wave <= 4) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r0 = (wave - 1) * 64 + h * 32;  // first tile row of the piece; 2 lanes per row
        dma16(fold.stats + (size_t)min(m0 + r0 + (lane >> 1), M - 1) * 4 + 2 * (lane & 1),
              lds0 + SIDE + 2048 + (uint32_t)(r0 * 32));
      }
    } else if (wave == 5 && fold.kc) {  // the accumulator start kc of the tile's 256 columns
      dma16(fold.kc + min(n0 + 4 * lane, N - 4), lds0 + SIDE + 10240);
    }
  }
  // prologue: K-tile 0 whole and K-tile 1's first two quarters (the loop issues the rest)
  if (nk > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) issue(q, 0);
  }
  if (nk > 1) {
    issue(0, 1);
    issue(1, 1);
    pp_wait_vm<8>();  // K-tile 0's A(mh 0) + W(nh 0) landed (this wave's pieces)
  } else {
    pp_wait_vm<0>();
  }
  if (DIAG == 1 || DIAG == 6 || DIAG == 7) pp_wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  if constexpr (FOLD_EPI) {
    // plane shift (FoldArgs): the accumulators start at kc of their columns (side data, landed
    // with this wave's first wait — older than every K-tile piece — and visible past the barrier)
    if (fold.kc) {
      const float* const kcl = reinterpret_cast<const float*>(pk_smem + SIDE + 10240);
#pragma unroll
      for (int tn = 0; tn < 2; ++tn)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const floatx4 k4 = *reinterpret_cast<const floatx4*>(kcl + wn * 64 + tn * 32 + 8 * j + 4 * lh);
#pragma unroll
          for (int tm = 0; tm < 4; ++tm)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[tm][tn][4 * j + i] = k4[i];
        }
    }
  }
  if (wm == 1) sync_load();  // group 1 runs one phase behind

  auto wait6 = [&](bool full) {
    if (DIAG == 5 || DIAG == 1 || DIAG == 6 || DIAG == 7) return;
    if (full) pp_wait_vm<6>();
    else pp_wait_vm<0>();
  };
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = pk_smem + (kt & 1) * STAGE;
    const bool next1 = kt + 1 < nk, next2 = kt + 2 < nk;
    // phase 0: quadrant (0, 0); wait for W(nh 1) of kt; W(nh 1) of kt+1 into its stage
    wait6(next1);
    read_a(st, 0, kt);
    read_w(st, 0, kt);
    sync_compute();
    mfma_quad(0, 0, std::integral_constant<int, 2>(), next1, kt + 1);
    sync_load();
    // phase 1: quadrant (0, 1); wait for A(mh 1) of kt; A(mh 1) of kt+1 into its stage
    wait6(next1);
    read_w(st, 1, kt);
    sync_compute();
    mfma_quad(0, 1, std::integral_constant<int, 3>(), next1, kt + 1);
    sync_load();
    // phase 2: quadrant (1, 1); A(mh 0) of kt+2 into kt's stage
    read_a(st, 1, kt);
    sync_compute();
    mfma_quad(1, 1, std::integral_constant<int, 0>(), next2, kt + 2);
    sync_load();
    // phase 3: quadrant (1, 0); wait for A(mh 0) + W(nh 0) of kt+1; W(nh 0) of kt+2
    wait6(next2);
    sync_compute();
    mfma_quad(1, 0, std::integral_constant<int, 1>(), next2, kt + 2);
    sync_load();
  }
  if (DIAG != 0 && DIAG != 8 && DIAG != 9) pp_wait_vm<0>();
  if (wm == 0) sync_load();
  if (DIAG == 7) __builtin_amdgcn_s_barrier();  // same barrier count in both groups; every LDS read and DMA done
  if (DIAG == 4) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) keep_f32(acc[a][b][r]);
    continue;
  }

  // ---- epilogue.  acc[tm][tn] register 4 j + i of lane l = output row wm*128 + tm*32 + (l & 31),
  // column wn*64 + tn*32 + 8 j + 4 (l >> 5) + i.  Per 64-row half (tm pair), the wave writes its
  // 64 x 64 block into its own 16-KiB LDS region in the output's byte image — f32 rows of 256 B,
  // or packed rows (NP 2: two 128-B [hi 32 | lo 32] blocks; NP 1: 128 B of hi) — with the 16-B
  // chunk index XOR-ed by pk_swz(row), then stores it with 16-B lanes, whole row segments per
  // instruction.  A 256-B row is one sweep of the 64 LDS banks, so the 32 rows a store
  // instruction writes (lanes 0-31) would meet rows r and r + 16 on the same banks under a plain
  // (row & 15) swizzle: pk_swz also flips chunk bit 3 for rows 16-31 (the round-3 counters put
  // exactly 2048 conflict cycles on every 256 x 256 tile, profiles/r3ap_pmc_sq.json).
  constexpr bool FOLD = EPI == PK_EPI_GELU_FOLD || EPI == PK_EPI_BIAS_FOLD;
  constexpr bool GELU = EPI == PK_EPI_GELU_PACKED || EPI == PK_EPI_GELU_FOLD;
  constexpr bool PACKED = GELU || FOLD || EPI == PK_EPI_BIAS_PACKED;
  constexpr int RB = PACKED ? 64 * 2 * NP : 256;  // bytes of a row segment
  constexpr int CPR = RB / 16;                                       // 16-B chunks per row
  unsigned char* reg = pk_smem + wave * 16384;
  const int cb0 = n0 + wn * 64;
  // folded LayerNorm: (mean, rstd) of this lane's 4 rows (rows past M read row M - 1; not
  // stored), all 16 statistics loads issued together — one memory latency per tile, not four
  // (from the side data the prologue moved into LDS: bias' / s of the tile's columns, the tile
  // rows' statistics; rows past M carry row M - 1's, never stored)
  float fneg[4] = {0.f, 0.f, 0.f, 0.f}, frs[4] = {1.f, 1.f, 1.f, 1.f};
  const float* const colt = reinterpret_cast<const float*>(pk_smem + SIDE);
  if constexpr (FOLD) {
    const uint64_t* lst = reinterpret_cast<const uint64_t*>(pk_smem + SIDE + 2048);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mu;
      row_norm(lst + (wm * 128 + r * 32 + li) * 4, fold.eps, mu, frs[r]);
      fneg[r] = -mu;
    }
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      // folded form: this column block's bias' / s quads read from LDS once for both row passes
      floatx4 fbv[4], fsv[4];
      if constexpr (FOLD) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cc = tn * 32 + 8 * j + 4 * lh;
          const int col = cb0 + cc < N ? cb0 + cc : N - 4;
          fbv[j] = *reinterpret_cast<const floatx4*>(colt + (col - n0));
          fsv[j] = *reinterpret_cast<const floatx4*>(colt + 256 + (col - n0));
        }
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int lr = tt * 32 + li;  // row within the half
        if constexpr (PACKED) {
          // lane half lh holds columns 8 j + 4 lh .. + 3 (4 bf16 = 8 B per plane) of every j; a
          // v_permlane32_swap per register pair (j, j + 1) hands each half the other's 8 B, so
          // the low half writes whole 16-B chunks j = 0, 2 and the high half j = 1, 3: 16-B
          // writes whose 16-lane groups hit 16 distinct chunk slots (8-B writes put 32 lanes on
          // 16 slots: 2048 bank-conflict cycles per tile, profiles/r4g_pmc_lds.json)
          const floatx16& c = acc[2 * half + tt][tn];
          uint32_t hw[4][2], lw[4][2];
          gelu_f2 y[8];  // pair i/2 of register quad j: y[2 j + i / 2]
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cc = tn * 32 + 8 * j + 4 * lh;  // column within the wave's 64
            const int col = cb0 + cc < N ? cb0 + cc : N - 4;
            const floatx4 bv = FOLD ? fbv[j] : *reinterpret_cast<const floatx4*>(bias + col);
            if constexpr (FOLD) {  // rstd * (acc - mean * s) + bias'
              const floatx4 sv = fsv[j];
#pragma unroll
              for (int i = 0; i < 4; i += 2)
                y[2 * j + i / 2] = __builtin_elementwise_fma(
                    __builtin_elementwise_fma(gelu_f2{sv[i], sv[i + 1]}, gelu_f2(fneg[2 * half + tt]),
                                              gelu_f2{c[4 * j + i], c[4 * j + i + 1]}),
                    gelu_f2(frs[2 * half + tt]), gelu_f2{bv[i], bv[i + 1]});
            } else {
#pragma unroll
              for (int i = 0; i < 4; i += 2)
                y[2 * j + i / 2] = gelu_f2{c[4 * j + i], c[4 * j + i + 1]} + gelu_f2{bv[i], bv[i + 1]};
            }
          }
          if constexpr (GELU) gelu_exp2_pairs(y);
#pragma unroll
          for (int k = 0; k < 8; ++k) split_pair(y[k], hw[k >> 1][k & 1], lw[k >> 1][k & 1]);
#pragma unroll
          for (int jp = 0; jp < 4; jp += 2) {
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const auto sh = __builtin_amdgcn_permlane32_swap(hw[jp][w], hw[jp + 1][w], false, false);
              hw[jp][w] = sh[0];
              hw[jp + 1][w] = sh[1];
              if (NP == 2) {
                const auto sl = __builtin_amdgcn_permlane32_swap(lw[jp][w], lw[jp + 1][w], false, false);
                lw[jp][w] = sl[0];
                lw[jp + 1][w] = sl[1];
              }
            }
            // this half's chunk: columns 8 (jp + lh) .. + 7 of block tn
            const int hb = tn * 64 * NP + 16 * (jp + lh);
            const int ch = ((hb >> 4) ^ pk_swz(lr)) & (CPR - 1);
            *reinterpret_cast<uint4*>(reg + lr * RB + ch * 16) =
                uint4{hw[jp][0], hw[jp][1], hw[jp + 1][0], hw[jp + 1][1]};
            if (NP == 2) {
              const int cl = (((hb + 64) >> 4) ^ pk_swz(lr)) & (CPR - 1);
              *reinterpret_cast<uint4*>(reg + lr * RB + cl * 16) =
                  uint4{lw[jp][0], lw[jp][1], lw[jp + 1][0], lw[jp + 1][1]};
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const floatx16& c = acc[2 * half + tt][tn];
            const int cc = tn * 32 + 8 * j + 4 * lh;  // column within the wave's 64
            floatx4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = c[4 * j + i];
            const int ch = (cc >> 2) ^ pk_swz(lr);
            *reinterpret_cast<floatx4*>(reg + lr * RB + ch * 16) = v;
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own region: no barrier
    constexpr int RPI = 64 / CPR;  // rows per store instruction
    // a lane keeps its 16-B column chunk c for the whole half and moves down RPI rows per store:
    // 32-bit element offsets from the half's uniform base row, one multiply per lane instead of a
    // 64-bit row x stride product per store (three quarter-rate integer ops each)
    const int lr0 = lane / CPR, c = lane % CPR;
    const int rbase = m0 + wm * 128 + half * 64;
    const uint32_t ldc = (uint32_t)(PACKED ? NP * N : N);  // elements per output row
    uint32_t off0 = (uint32_t)lr0 * ldc + (PACKED ? c * 8 : 4 * c);
    asm("" : "+v"(off0));  // opaque: keeps the per-store offset an add (no re-derived multiply)
    // 16 B of the packed row: column block (c*16 / (64 NP)), all within the wave's 64 columns
    const int col = PACKED ? cb0 + (c * 16) / (2 * NP) : cb0 + 4 * c;
    floatx4 bv = {0.f, 0.f, 0.f, 0.f};
    if (!PACKED && col < N) bv = *reinterpret_cast<const floatx4*>(bias + col);
#pragma unroll
    for (int k = 0; k < 64 / RPI; ++k) {
      const int lr = k * RPI + lr0;
      const bool ok = rbase + lr < M;
      const uint4 v = *reinterpret_cast<const uint4*>(reg + lr * RB + ((c ^ pk_swz(lr)) & (CPR - 1)) * 16);
      const uint32_t o = off0 + (uint32_t)(k * RPI) * ldc;
      if (PACKED) {
        if (ok && col < N) {
          __bf16* dstp = Cp + (size_t)rbase * NP * N + (size_t)(cb0 >> 5) * 32 * NP + o;
          if (DIAG != 8)
            __builtin_nontemporal_store(__builtin_bit_cast(floatx4, v), reinterpret_cast<floatx4*>(dstp));
          else
            *reinterpret_cast<uint4*>(dstp) = v;
        }
      } else {
        if (ok && col < N) {
          floatx4 f = __builtin_bit_cast(floatx4, v) + bv;
          if (EPI == PK_EPI_TANH)
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = tanhf(f[i]);
          float* dst = C + (size_t)rbase * N + cb0 + o;
          if (EPI == PK_EPI_RES) f += *reinterpret_cast<const floatx4*>(R + (size_t)rbase * N + cb0 + o);
          if (DIAG != 8)
            __builtin_nontemporal_store(f, reinterpret_cast<floatx4*>(dst));
          else
            *reinterpret_cast<floatx4*>(dst) = f;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // region reads done before it is rewritten
  }
  // every wave's staging reads done before the next tile's prologue DMA rewrites the stages
  // (raw barrier: the epilogue's stores stay in flight)
  if constexpr (DIAG != 9) break;  // one tile per workgroup: no loop-carried state
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  }  // tile loop
}

// ------------------------------------------------------------------------------------------
// Ping-pong 256 x 192 packed GEMM (gemm_pp192_kernel): the N = 768 GEMMs (O-projection, FFN2)
// tile as 128 x 4 = 512 tiles = 2 full rounds on 256 CUs instead of 384 256^2 tiles (1.5 rounds,
// the second half idle).  gemm_pp_kernel's structure with a 64 x 96 block per wave: group g
// (rows 128 g ..) holds 4 waves as 2 (m) x 2 (n); a K-tile is consumed in three phases, one
// 64 x 32 column block (tn) each — phase 0 reads A (both 32-row blocks) and W(tn 0), phases 1
// and 2 read W(tn 1), W(tn 2).  Two 56-KiB stages; K-tile kt+2's A + W(tn 0) go into kt's stage
// at phase 2 of kt (their last read was phase 0), W(tn 1) and W(tn 2) of kt+1 at phases 0 and 1
// of kt (>= 2 phases after their last read); each waited one phase before it is read.  f32
// epilogues only (bias / +residual / tanh), staged through LDS in 32-row passes with 400-B
// padded rows (conflict-free), stored as whole 384-B row segments.
template <int NP, int EPI, bool NT = false>
__global__ __launch_bounds__(512, 1) void gemm_pp192_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ W, const float* __restrict__ bias,
    const float* R, float* C, int M, int N, int K, int group_m, StatArgs ln) {
  extern __shared__ __attribute__((aligned(16))) unsigned char pk_smem[];
  constexpr int BM = 256, BN = 192, ROWB = PK_ROWB;
  constexpr int A_BYTES = BM * ROWB, STAGE = (BM + BN) * ROWB;  // 56 KiB per K-tile
  constexpr int KB = 64 / NP, NS = KB / 16, T = NP == 2 ? 3 : 1;

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm0 = first_m + (t - g * per_group) % gsize, tn0 = (t - g * per_group) / gsize;
  const int m0 = tm0 * BM, n0 = tn0 * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, sm = (wave >> 1) & 1, sn = wave & 1;  // group, sub-row, sub-column
  const int li = lane & 31, lh = lane >> 5;
  const size_t lda = (size_t)NP * K;

  // ---- DMA pieces (8 rows x 128 B) per wave per K-tile: [0..3] A rows 32 wave + 8 u, [4..6]
  // W(tn) rows 96 (wave >> 2) + 32 tn + 8 (wave & 3) (the 64 W rows of column block tn)
  const char* src[7];
  uint32_t dst[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const bool is_a = j < 4;
    const int r0 = is_a ? 32 * wave + 8 * j : 96 * (wave >> 2) + 32 * (j - 4) + 8 * (wave & 3);
    const int r = r0 + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    if (is_a) {
      const int gr = m0 + r < M ? m0 + r : M - 1;
      src[j] = reinterpret_cast<const char*>(A + gr * lda) + 16 * cs;
      dst[j] = r0 * ROWB;
    } else {
      const int gr = n0 + r < N ? n0 + r : N - 1;
      src[j] = reinterpret_cast<const char*>(W + gr * lda) + 16 * cs;
      dst[j] = A_BYTES + r0 * ROWB;
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)pk_smem;
  const int nk = K / KB;
  auto issue = [&](int j, int kt) {
    dma16(src[j] + (size_t)kt * ROWB, lds0 + (kt & 1) * STAGE + dst[j]);
  };

  floatx16 acc[2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int sw = (li >> 1) & 7;
  const int a_row = (wm * 128 + sm * 64 + li) * ROWB;
  const int w_row = A_BYTES + (sn * 96 + li) * ROWB;
  bf16x8 fa[2][NS][NP], fw[3][NS][NP];
  auto read_a = [&](const unsigned char* st) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          fa[tt][s][p] = *reinterpret_cast<const bf16x8*>(
              st + a_row + tt * 32 * ROWB + 16 * ((4 * p + 2 * s + lh) ^ sw));
  };
  auto read_w = [&](const unsigned char* st, int tn) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        fw[tn][s][p] = *reinterpret_cast<const bf16x8*>(
            st + w_row + tn * 32 * ROWB + 16 * ((4 * p + 2 * s + lh) ^ sw));
  };
  // column block tn's MFMAs; DMA pieces j0 .. j0 + nj - 1 of K-tile kd ride in the issue gaps
  auto mfma_col = [&](int tn, auto j0c, auto njc, bool dma, int kd) {
    constexpr int J0 = decltype(j0c)::value, NJ = decltype(njc)::value;
    constexpr int NM = NS * 2 * T;
    constexpr int EVERY = NJ > 0 ? NM / (NJ + 1) : NM + 1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int s = i / (2 * T), tt = (i / T) % 2, term = i % T;
      floatx16& c = acc[tt][tn];
      const bf16x8& x = (T == 3 && term == 1) ? fw[tn][s][NP - 1] : fw[tn][s][0];
      const bf16x8& y = (T == 3 && term == 0) ? fa[tt][s][NP - 1] : fa[tt][s][0];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
      if (dma && i % EVERY == EVERY - 1 && i / EVERY < NJ) {
        const int j = J0 + i / EVERY;
        __builtin_amdgcn_sched_barrier(0);
        dma16(src[j] + (size_t)kd * ROWB, lds0 + (kd & 1) * STAGE + dst[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_compute = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_load = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // PK_EPI_RES_STATS(_LN): the epilogue's side data — bias (gamma, beta) of the tile's 192
  // columns (1 KiB each) and, for _LN, the residual rows' tile statistics (8 KiB) — moved into LDS
  // past the stages by LDS-DMA ahead of the prologue (older than every K-tile piece, so the
  // counted waits below cover them)
  constexpr bool STATS_EPI = EPI == PK_EPI_RES_STATS || EPI == PK_EPI_RES_STATS_LN;
  constexpr uint32_t SIDE = 2 * STAGE;  // [bias | gamma | beta] (1 KiB each), [256 rows][4] u64
  if constexpr (STATS_EPI) {
    if (wave == 0) {
      const int c = n0 + 4 * min(lane, 47);
      dma16(bias + c, lds0 + SIDE);
      if constexpr (EPI == PK_EPI_RES_STATS_LN) {
        dma16(ln.gamma + c, lds0 + SIDE + 1024);
        dma16(ln.beta + c, lds0 + SIDE + 2048);
      }
    } else if (EPI == PK_EPI_RES_STATS_LN && wave <= 4) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r0 = (wave - 1) * 64 + h * 32;  // first tile row of the piece; 2 lanes per row
        dma16(ln.rstats + (size_t)min(m0 + r0 + (lane >> 1), M - 1) * 4 + 2 * (lane & 1),
              lds0 + SIDE + 3072 + (uint32_t)(r0 * 32));
      }
    } else if (wave == 5 && ln.shift) {  // the plane shift kappa of the tile's 192 columns
      dma16(ln.shift + n0 + 4 * min(lane, 47), lds0 + SIDE + 11264);
    }
  }
  // prologue: K-tile 0 whole, K-tile 1's A + W(tn 0) (its W(tn 1), W(tn 2): phases 0, 1 of kt 0)
  if (nk > 0) {
#pragma unroll
    for (int j = 0; j < 7; ++j) issue(j, 0);
  }
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < 5; ++j) issue(j, 1);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // K-tile 0's A + W(tn 0)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wm == 1) sync_load();  // group 1 runs one phase behind

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = pk_smem + (kt & 1) * STAGE;
    const bool next1 = kt + 1 < nk, next2 = kt + 2 < nk;
    // phase 0: reads A, W(tn 0); waits for W(tn 1) of kt; W(tn 1) of kt+1 into its stage
    if (next1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    read_a(st);
    read_w(st, 0);
    sync_compute();
    mfma_col(0, std::integral_constant<int, 5>(), std::integral_constant<int, 1>(), next1,
             kt + 1);
    sync_load();
    // phase 1: reads W(tn 1); waits for W(tn 2) of kt; W(tn 2) of kt+1 into its stage
    if (next1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    read_w(st, 1);
    sync_compute();
    mfma_col(1, std::integral_constant<int, 6>(), std::integral_constant<int, 1>(), next1,
             kt + 1);
    sync_load();
    // phase 2: reads W(tn 2); waits for A + W(tn 0) of kt+1; A + W(tn 0) of kt+2 into kt's stage
    if (next1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    read_w(st, 2);
    sync_compute();
    mfma_col(2, std::integral_constant<int, 0>(), std::integral_constant<int, 5>(), next2,
             kt + 2);
    sync_load();
  }
  if (wm == 0) sync_load();  // same barrier count in both groups; every LDS read and DMA done

  if constexpr (EPI == PK_EPI_RES_STATS || EPI == PK_EPI_RES_STATS_LN) {
    // ---- v = (acc + bias) + residual as f32 and packed planes, plus this tile's (mean, M2) of
    // every row: the producing half of the folded LayerNorm (FoldArgs) — the O-projection / FFN2
    // of every encoder layer.  The layer input x = LN(v_prev) is never stored: in the _LN form
    // the residual rows are the previous pre-LayerNorm rows v_prev, normalised here with their
    // own statistics (rowops.hip layernorm_kernel's formula); otherwise the residual is used as
    // it is (layer 0: the embedding LayerNorm's output).  acc[tm][tn] register 4 j + i of lane l
    // = row wm*128 + sm*64 + tm*32 + (l & 31), column sn*96 + tn*32 + 8 j + 4 (l >> 5) + i of
    // the tile (the transposed MFMA product).  R may alias C: every element is read before this
    // workgroup writes it, and no other workgroup touches this tile.
    const int cb0 = n0 + sn * 96;
    const int rb0 = m0 + wm * 128 + sm * 64 + li;  // + 32 tm
    constexpr int RS = 400;
    unsigned char* reg = pk_smem + wave * 32 * RS;
    const int prow0 = m0 + wm * 128 + sm * 64;
    constexpr bool rnorm = EPI == PK_EPI_RES_STATS_LN;
    // the residual rows' (mean, rstd) for both passes and the tile's bias (gamma, beta) columns,
    // all from the side data the prologue moved into LDS (rows past M carry row M - 1's)
    const float* const colt = reinterpret_cast<const float*>(pk_smem + SIDE);
    float rmu[2] = {0.f, 0.f}, rrs[2] = {1.f, 1.f};
    if constexpr (rnorm) {
      const uint64_t* rst = reinterpret_cast<const uint64_t*>(pk_smem + SIDE + 3072);
#pragma unroll
      for (int tm = 0; tm < 2; ++tm)
        row_norm(rst + (rb0 - m0 + 32 * tm) * 4, ln.eps, rmu[tm], rrs[tm]);
    }
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const int idx = k * 64 + lane, lr = idx / 24, c = idx % 24;
        const int row = prow0 + tm * 32 + lr;
        const floatx4 f = row < M ? *reinterpret_cast<const floatx4*>(R + (size_t)row * N + cb0 + 4 * c)
                                  : floatx4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<floatx4*>(reg + lr * RS + c * 16) = f;
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int tn = 0; tn < 3; ++tn)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tc = sn * 96 + tn * 32 + 8 * j + 4 * lh;  // column within the tile
          const floatx4 bv = *reinterpret_cast<const floatx4*>(colt + tc);
          floatx4 rv = *reinterpret_cast<const floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16);
          if constexpr (rnorm) {
            const floatx4 gg = *reinterpret_cast<const floatx4*>(colt + 256 + tc);
            const floatx4 bb = *reinterpret_cast<const floatx4*>(colt + 512 + tc);
#pragma unroll
            for (int i = 0; i < 4; ++i) rv[i] = (rv[i] - rmu[tm]) * rrs[tm] * gg[i] + bb[i];
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[tm][tn][4 * j + i] = (acc[tm][tn][4 * j + i] + bv[i]) + rv[i];
            // computed here, not sunk to the statistics below (which would keep every loaded
            // column vector live until then and spill)
            asm volatile("" : "+v"(acc[tm][tn][4 * j + i]));
          }
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next pass rewrites
    }
    // per row over the wave's 96 columns (the lane halves hold 48 each), then the two waves of a
    // row (sn = 0, 1) merged through LDS in sn order
    float mean96[2], m2_96[2];
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
      float sum = 0.f;
#pragma unroll
      for (int tn = 0; tn < 3; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += acc[tm][tn][r];
      sum += __shfl_xor(sum, 32, 64);
      const float mu = sum * (1.f / 96.f);
      float q = 0.f;
#pragma unroll
      for (int tn = 0; tn < 3; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[tm][tn][r] - mu;
          q += d * d;
        }
      q += __shfl_xor(q, 32, 64);
      mean96[tm] = mu;
      m2_96[tm] = q;
    }
    RowStat* lst = reinterpret_cast<RowStat*>(pk_smem + 8 * 32 * RS);
    if (lh == 0) {
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) lst[(wave * 2 + tm) * 32 + li] = RowStat{mean96[tm], m2_96[tm]};
    }
    __syncthreads();
    if (sn == 0 && lh == 0) {
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        const RowStat o = lst[((wave ^ 1) * 2 + tm) * 32 + li];
        const float d = mean96[tm] - o.mean;
        const RowStat t{(mean96[tm] + o.mean) * 0.5f, (m2_96[tm] + o.m2) + 48.f * d * d};
        if (rb0 + 32 * tm < M) ln.stats[(size_t)(rb0 + 32 * tm) * 4 + tn0] = __builtin_bit_cast(uint64_t, t);
      }
    }
    // v through the wave's LDS region again: x-style whole row segments (two 16-B f32 stores and
    // one 16-B store per plane for 8 consecutive columns of a row per lane)
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
      for (int tn = 0; tn < 3; ++tn)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          floatx4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = acc[tm][tn][4 * j + i];
          *reinterpret_cast<floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16) = o;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int kk = k % 3, g = k / 3;
        const int idx = kk * 64 + lane, lr = idx / 12 + 16 * g, c8 = idx % 12;
        const int row = prow0 + tm * 32 + lr;
        const floatx4 o0 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32);
        const floatx4 o1 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32 + 16);
        if (row < M) {
          const int col = cb0 + 8 * c8;
          float* const vrow = C + (size_t)prow0 * N + (uint32_t)(lr + tm * 32) * (uint32_t)N;
          *reinterpret_cast<floatx4*>(vrow + col) = o0;
          *reinterpret_cast<floatx4*>(vrow + col + 4) = o1;
          uint32_t h[4], l[4];  // column pairs as packed bf16 conversions (split_pair)
          floatx4 p0 = o0, p1 = o1;  // the planes hold v - kappa (the plane shift, FoldArgs)
          if (ln.shift) {
            const float* const kap = reinterpret_cast<const float*>(pk_smem + SIDE + 11264);
            p0 -= *reinterpret_cast<const floatx4*>(kap + (col - n0));
            p1 -= *reinterpret_cast<const floatx4*>(kap + (col - n0) + 4);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            split_pair(i < 2 ? gelu_f2{p0[2 * i], p0[2 * i + 1]} : gelu_f2{p1[2 * i - 4], p1[2 * i - 3]},
                       h[i], l[i]);
          unsigned short* dst = reinterpret_cast<unsigned short*>(ln.xp) + (size_t)prow0 * NP * N +
                                (uint32_t)(lr + tm * 32) * (uint32_t)(NP * N) +
                                (uint32_t)((col >> 5) * 32 * NP + (col & 31));
          *reinterpret_cast<uint4*>(dst) = uint4{h[0], h[1], h[2], h[3]};
          if (NP == 2) *reinterpret_cast<uint4*>(dst + 32) = uint4{l[0], l[1], l[2], l[3]};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }

  if constexpr (EPI == PK_EPI_BIAS_PACKED) {
    // ---- +bias -> packed planes (the QKV GEMM of the half-batch streams: N = 2304 = 12 x 192
    // tiles = 3 full rounds of 256 CUs where 256-wide tiles take 2.25).  C is the packed output
    // [M][NP * N] here.  Per 32-row pass the wave's 32 x 96 block (+ bias) goes to its LDS region
    // (400-B rows), then every lane takes 8 consecutive columns of a row: one 16-B store per
    // plane (the mode-0 LayerNorm store pattern without the f32 copy).  Requires N % 192 == 0.
    constexpr int RS = 400;
    unsigned char* reg = pk_smem + wave * 32 * RS;
    const int cb0 = n0 + sn * 96;
    const int prow0 = m0 + wm * 128 + sm * 64;
    unsigned short* const cp = reinterpret_cast<unsigned short*>(C);
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
      for (int tn = 0; tn < 3; ++tn)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const floatx4 bv = *reinterpret_cast<const floatx4*>(bias + cb0 + tn * 32 + 8 * j + 4 * lh);
          floatx4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[tm][tn][4 * j + i] + bv[i];
          *reinterpret_cast<floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16) = v;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int kk = k % 3, g = k / 3;
        const int idx = kk * 64 + lane, lr = idx / 12 + 16 * g, c8 = idx % 12;
        const int row = prow0 + tm * 32 + lr;
        const floatx4 o0 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32);
        const floatx4 o1 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32 + 16);
        if (row < M) {
          const int col = cb0 + 8 * c8;
          uint32_t h[4], l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float a = i < 2 ? o0[2 * i] : o1[2 * i - 4], b = i < 2 ? o0[2 * i + 1] : o1[2 * i - 3];
            const uint32_t ha = f2bf(a), hb = f2bf(b);
            h[i] = ha | (hb << 16);
            l[i] = (uint32_t)f2bf(a - __builtin_bit_cast(float, ha << 16)) |
                   ((uint32_t)f2bf(b - __builtin_bit_cast(float, hb << 16)) << 16);
          }
          unsigned short* dst = cp + (size_t)prow0 * NP * N + (uint32_t)(lr + tm * 32) * (uint32_t)(NP * N) +
                                (uint32_t)((col >> 5) * 32 * NP + (col & 31));
          *reinterpret_cast<uint4*>(dst) = uint4{h[0], h[1], h[2], h[3]};
          if (NP == 2) *reinterpret_cast<uint4*>(dst + 32) = uint4{l[0], l[1], l[2], l[3]};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }

  // ---- epilogue: per 32-row pass (tm), the wave's 32 x 96 f32 block goes to its LDS region
  // (rows of 400 B: 384 + 16 pad, so 16 lanes of different rows hit 16 different bank slots),
  // then whole 384-B row segments go out with 16-B lanes (+ bias, tanh / residual)
  constexpr int RS = 400;
  unsigned char* reg = pk_smem + wave * 32 * RS;
  const int cb0 = n0 + sn * 96;
  // store round k = 3 g + kk covers chunks 64 k + lane of the pass's 32 x 24 = round kk's chunks
  // 8 g rows further down: the three rounds' (row, column) and 32-bit offsets from the wave's
  // first row are computed once, every other round adds a uniform 8 g rows
  const int rbase = m0 + wm * 128 + sm * 64;
  int lrk[3], ck[3];
  uint32_t offk[3];
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    const int idx = kk * 64 + lane;
    lrk[kk] = idx / 24;
    ck[kk] = idx % 24;
    offk[kk] = (uint32_t)lrk[kk] * (uint32_t)N + 4 * ck[kk];
    asm("" : "+v"(offk[kk]));  // opaque: keeps the per-store offset an add
  }
  float* const cbase = C + (size_t)rbase * N + cb0;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        floatx4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[tm][tn][4 * j + i];
        *reinterpret_cast<floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16) = v;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int kk = k % 3, g = k / 3;
      const int lr = lrk[kk] + 8 * g, c = ck[kk];
      const int row = rbase + tm * 32 + lr;
      const int col = cb0 + 4 * c;
      floatx4 f = *reinterpret_cast<const floatx4*>(reg + lr * RS + c * 16);
      if (row < M && col < N) {
        const uint32_t o = offk[kk] + (uint32_t)(tm * 32 + 8 * g) * (uint32_t)N;
        f += *reinterpret_cast<const floatx4*>(bias + col);
        if (EPI == PK_EPI_TANH)
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] = tanhf(f[i]);
        if (EPI == PK_EPI_RES) f += *reinterpret_cast<const floatx4*>(R + (size_t)rbase * N + cb0 + o);
        if (NT)
          __builtin_nontemporal_store(f, reinterpret_cast<floatx4*>(cbase + o));
        else
          *reinterpret_cast<floatx4*>(cbase + o) = f;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

namespace {
int cu_count();
// ------------------------------------------------------------------------------------------
// Two-per-CU 128 x 192 packed GEMM (gemm_p2_kernel): the N = 768 GEMMs (O-projection, FFN2) with
// the residual + statistics epilogue of the folded LayerNorm (PK_EPI_RES_STATS(_LN)), built so that
// TWO workgroups share a CU and one's epilogue — HBM-bound: the residual rows in, v and its planes
// out, 590 KB per 256 x 192 tile of gemm_pp192_kernel — runs under the other's MFMAs, which one
// workgroup per CU cannot do.  4 waves (2 x 2 blocks of 64 x 96, gemm_pp192_kernel's wave block
// and epilogue), 80 KiB of LDS: two 40-KiB stages of a 32-k K-tile (A 128 rows + W 192 rows) and
// nothing else — the epilogue's side data (bias, gamma / beta, the plane shift, the residual rows'
// statistics: 8 KiB) is moved by LDS-DMA into the tail of the stage that frees up first during the
// last two K-tiles, and the staging regions fill the stages once the loop is done.  No ping-pong
// between wave groups: per K-tile every wave waits for its own pieces, a barrier, its fragment
// reads, a barrier (the stage is free), then its 36 MFMAs with K-tile kt+2's 10 DMA pieces in
// their issue gaps; the co-resident workgroup fills the matrix pipe while this one waits.
// V = 1: the fragment reads pipelined against the MFMAs — all 20 issued, the MFMAs of column block
// 0 after the A and W(0) reads (the compiler's partial lgkmcnt), block 1 after W(1), then the
// stage-free barrier and block 2 with K-tile kt+2's DMA pieces.
template <int NP, int EPI, int V = 0>
__global__ __launch_bounds__(256, 2) void gemm_p2_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ W, const float* __restrict__ bias,
    const float* R, float* C, int M, int N, int K, int group_m, StatArgs ln, FoldArgs fold) {
  extern __shared__ __attribute__((aligned(16))) unsigned char pk_smem[];
  constexpr bool FOLD = EPI == PK_EPI_GELU_FOLD || EPI == PK_EPI_BIAS_FOLD;
  static_assert(EPI == PK_EPI_RES_STATS || EPI == PK_EPI_RES_STATS_LN || FOLD,
                "statistics or folded-LayerNorm epilogues only");
  constexpr int BM = 128, BN = 192, ROWB = PK_ROWB;
  constexpr int A_BYTES = BM * ROWB, STAGE = (BM + BN) * ROWB;  // 40 KiB per K-tile
  constexpr int KB = 64 / NP, NS = KB / 16, T = NP == 2 ? 3 : 1;
  constexpr int NPC = 10;  // DMA pieces per wave per K-tile: 4 of A (rows 32 w ..), 6 of W (48 w ..)

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm0 = first_m + (t - g * per_group) % gsize, tn0 = (t - g * per_group) / gsize;
  const int m0 = tm0 * BM, n0 = tn0 * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sm = wave >> 1, sn = wave & 1;  // sub-row (64 rows), sub-column (96 columns)
  const int li = lane & 31, lh = lane >> 5;
  const size_t lda = (size_t)NP * K;

  const char* src[NPC];
  uint32_t dst[NPC];
#pragma unroll
  for (int j = 0; j < NPC; ++j) {
    const bool is_a = j < 4;
    const int r0 = is_a ? 32 * wave + 8 * j : 48 * wave + 8 * (j - 4);
    const int r = r0 + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    if (is_a) {
      const int gr = m0 + r < M ? m0 + r : M - 1;
      src[j] = reinterpret_cast<const char*>(A + gr * lda) + 16 * cs;
      dst[j] = r0 * ROWB;
    } else {
      const int gr = n0 + r < N ? n0 + r : N - 1;
      src[j] = reinterpret_cast<const char*>(W + gr * lda) + 16 * cs;
      dst[j] = A_BYTES + r0 * ROWB;
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)pk_smem;
  const int nk = K / KB;
  auto issue = [&](int j, int kt) {
    dma16(src[j] + (size_t)kt * ROWB, lds0 + (kt & 1) * STAGE + dst[j]);
  };
  // the epilogue's side data: into the tail of the stage that frees up first at the end of the
  // loop (K-tile nk - 2's; with one K-tile, the unused second stage)
  const int side_stage = nk >= 2 ? ((nk - 2) & 1) : 1;
  const uint32_t SIDE = side_stage * STAGE + STAGE - 8192;  // bias | gamma | beta | shift | rstats
  constexpr bool rnorm = EPI == PK_EPI_RES_STATS_LN;
  auto issue_side = [&]() {
    if constexpr (FOLD) {  // bias' | s | kc | the tile rows' statistics (FoldArgs)
      if (wave == 0) {
        dma16(bias + n0 + 4 * min(lane, 47), lds0 + SIDE);
      } else if (wave == 1) {
        dma16(fold.s + n0 + 4 * min(lane, 47), lds0 + SIDE + 1024);
      } else if (wave == 2) {
        if (fold.kc) dma16(fold.kc + n0 + 4 * min(lane, 47), lds0 + SIDE + 2048);
      } else {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int r0 = h * 32;
          dma16(fold.stats + (size_t)min(m0 + r0 + (lane >> 1), M - 1) * 4 + 2 * (lane & 1),
                lds0 + SIDE + 4096 + (uint32_t)(r0 * 32));
        }
      }
      return;
    }
    if (wave == 0) {
      dma16(bias + n0 + 4 * min(lane, 47), lds0 + SIDE);
    } else if (wave == 1) {
      if (rnorm) {
        dma16(ln.gamma + n0 + 4 * min(lane, 47), lds0 + SIDE + 1024);
        dma16(ln.beta + n0 + 4 * min(lane, 47), lds0 + SIDE + 2048);
      }
    } else if (wave == 2) {
      if (ln.shift) dma16(ln.shift + n0 + 4 * min(lane, 47), lds0 + SIDE + 3072);
    } else if (rnorm) {
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int r0 = h * 32;  // first tile row of the piece; 2 lanes per row
        dma16(ln.rstats + (size_t)min(m0 + r0 + (lane >> 1), M - 1) * 4 + 2 * (lane & 1),
              lds0 + SIDE + 4096 + (uint32_t)(r0 * 32));
      }
    }
  };

  floatx16 acc[2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int sw = (li >> 1) & 7;
  const int a_row = (sm * 64 + li) * ROWB;
  const int w_row = A_BYTES + (sn * 96 + li) * ROWB;
  bf16x8 fa[2][NS][NP], fw[3][NS][NP];

  if (nk > 0) {
#pragma unroll
    for (int j = 0; j < NPC; ++j) issue(j, 0);
  }
  if (nk > 1) {
#pragma unroll
    for (int j = 0; j < NPC; ++j) issue(j, 1);
  } else {
    issue_side();
  }

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = pk_smem + (kt & 1) * STAGE;
    // this wave's pieces of K-tile kt (K-tile kt + 1's may still be in flight), then everyone's
    if (kt + 1 < nk) wait_vm<NPC>();
    else wait_vm<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          fa[tt][s2][p] = *reinterpret_cast<const bf16x8*>(
              st + a_row + tt * 32 * ROWB + 16 * ((4 * p + 2 * s2 + lh) ^ sw));
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          fw[tn][s2][p] = *reinterpret_cast<const bf16x8*>(
              st + w_row + tn * 32 * ROWB + 16 * ((4 * p + 2 * s2 + lh) ^ sw));
    const bool dma = kt + 2 < nk;
    constexpr int NM = NS * 2 * T;  // MFMAs per column block
    auto mfma_block = [&](int tn, bool with_dma) {
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        const int s2 = i / (2 * T), tt = (i / T) % 2, term = i % T;
        floatx16& c = acc[tt][tn];
        const bf16x8& x = (T == 3 && term == 1) ? fw[tn][s2][NP - 1] : fw[tn][s2][0];
        const bf16x8& y = (T == 3 && term == 0) ? fa[tt][s2][NP - 1] : fa[tt][s2][0];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
        if (with_dma) {
          // K-tile kt + 2's pieces in the MFMA issue gaps: 10 over the MFMAs that follow the
          // stage-free barrier (V 0: all 3 x NM of them, V 1: block 2's NM)
          constexpr int SPAN = V == 0 ? 3 * NM : NM;
          constexpr int EVERY = SPAN / NPC > 0 ? SPAN / NPC : 1;
          const int gi = (V == 0 ? tn * NM : 0) + i;
          if (dma && gi % EVERY == EVERY - 1 && gi / EVERY < NPC) {
            __builtin_amdgcn_sched_barrier(0);
            issue(gi / EVERY, kt + 2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if (with_dma && V == 1 && dma && NM / (NM / NPC > 0 ? NM / NPC : 1) < NPC) {
        // fewer MFMAs than pieces: the rest after the block
#pragma unroll
        for (int j = NM / (NM / NPC > 0 ? NM / NPC : 1); j < NPC; ++j) issue(j, kt + 2);
      }
    };
    if constexpr (V == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // every wave holds its fragments: stage kt & 1 is free
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 == nk) issue_side();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int tn = 0; tn < 3; ++tn) mfma_block(tn, true);
      __builtin_amdgcn_s_setprio(0);
    } else {
      __builtin_amdgcn_s_setprio(1);
      mfma_block(0, false);
      mfma_block(1, false);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // every wave holds its fragments: stage kt & 1 is free
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 == nk) issue_side();
      __builtin_amdgcn_s_setprio(1);
      mfma_block(2, true);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // every wave is past its last fragment reads (the loop's second barrier); the side data landed
  // with each issuer's final vmcnt(0) before the last K-tile's first barrier
  if constexpr (FOLD) {
    // ---- folded LayerNorm (gemm_pp_kernel's PK_EPI_*_FOLD for a 128 x 192 tile): y = rstd ·
    // ((acc + kc) − mean · s) + bias', GELU'd for FFN1, staged per 32-row half in the wave's LDS
    // rows and stored as packed planes with 16-B lanes.  kc (the plane shift's accumulator start)
    // is added here rather than preloaded: it lands with the epilogue's side data.
    constexpr int RS = 400;
    unsigned char* reg = pk_smem + (wave < 3 ? (side_stage ^ 1) * STAGE + wave * 32 * RS
                                             : side_stage * STAGE);
    const float* const colt = reinterpret_cast<const float*>(pk_smem + SIDE);
    const uint64_t* const fst = reinterpret_cast<const uint64_t*>(pk_smem + SIDE + 4096);
    const int cb0 = n0 + sn * 96, prow0 = m0 + sm * 64;
    const bool has_kc = fold.kc != nullptr;
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
      float mu, rs;
      row_norm(fst + (sm * 64 + tm * 32 + li) * 4, fold.eps, mu, rs);
#pragma unroll
      for (int tn = 0; tn < 3; ++tn) {
        gelu_f2 y[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tc = sn * 96 + tn * 32 + 8 * j + 4 * lh;  // column within the tile
          const floatx4 bv = *reinterpret_cast<const floatx4*>(colt + tc);
          const floatx4 sv = *reinterpret_cast<const floatx4*>(colt + 256 + tc);
          floatx4 kv = {0.f, 0.f, 0.f, 0.f};
          if (has_kc) kv = *reinterpret_cast<const floatx4*>(colt + 512 + tc);
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const gelu_f2 a = gelu_f2{acc[tm][tn][4 * j + i], acc[tm][tn][4 * j + i + 1]} +
                              gelu_f2{kv[i], kv[i + 1]};
            y[2 * j + i / 2] = __builtin_elementwise_fma(
                __builtin_elementwise_fma(gelu_f2{sv[i], sv[i + 1]}, gelu_f2(-mu), a), gelu_f2(rs),
                gelu_f2{bv[i], bv[i + 1]});
          }
        }
        if constexpr (EPI == PK_EPI_GELU_FOLD) gelu_exp2_pairs(y);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16) =
              floatx4{y[2 * j].x, y[2 * j].y, y[2 * j + 1].x, y[2 * j + 1].y};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own rows: no barrier
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int kk = k % 3, g2 = k / 3;
        const int idx = kk * 64 + lane, lr = idx / 12 + 16 * g2, c8 = idx % 12;
        const int row = prow0 + tm * 32 + lr;
        const floatx4 o0 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32);
        const floatx4 o1 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32 + 16);
        if (row < M) {
          const int col = cb0 + 8 * c8;
          uint32_t h[4], l[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            split_pair(i < 2 ? gelu_f2{o0[2 * i], o0[2 * i + 1]} : gelu_f2{o1[2 * i - 4], o1[2 * i - 3]},
                       h[i], l[i]);
          unsigned short* dstp = reinterpret_cast<unsigned short*>(ln.xp) + (size_t)prow0 * NP * N +
                                 (uint32_t)(lr + tm * 32) * (uint32_t)(NP * N) +
                                 (uint32_t)((col >> 5) * 32 * NP + (col & 31));
          *reinterpret_cast<uint4*>(dstp) = uint4{h[0], h[1], h[2], h[3]};
          if (NP == 2) *reinterpret_cast<uint4*>(dstp + 32) = uint4{l[0], l[1], l[2], l[3]};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next half lands
    }
    return;
  }

  // ---- v = (acc + bias) + residual as f32 and packed planes of v - shift, plus this tile's
  // (mean, M2) of every row (gemm_pp192_kernel's epilogue for a 128-row tile; see there).
  // acc[tm][tn] register 4 j + i of lane l = row sm*64 + tm*32 + (l & 31), column sn*96 + tn*32 +
  // 8 j + 4 (l >> 5) + i of the tile.  R may alias C (no other workgroup touches this tile).
  const int cb0 = n0 + sn * 96;
  const int rb0 = m0 + sm * 64 + li;  // + 32 tm
  constexpr int RS = 400;
  // staging: waves 0-2 in the other stage, wave 3 at the head of the side stage; the row
  // statistics exchange after it
  unsigned char* reg = pk_smem + (wave < 3 ? (side_stage ^ 1) * STAGE + wave * 32 * RS
                                           : side_stage * STAGE);
  RowStat* lst = reinterpret_cast<RowStat*>(pk_smem + side_stage * STAGE + 32 * RS);
  const int prow0 = m0 + sm * 64;
  const float* const colt = reinterpret_cast<const float*>(pk_smem + SIDE);
  float rmu[2] = {0.f, 0.f}, rrs[2] = {1.f, 1.f};
  if constexpr (rnorm) {
    const uint64_t* rst = reinterpret_cast<const uint64_t*>(pk_smem + SIDE + 4096);
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) row_norm(rst + (rb0 - m0 + 32 * tm) * 4, ln.eps, rmu[tm], rrs[tm]);
  }
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int idx = k * 64 + lane, lr = idx / 24, c = idx % 24;
      const int row = prow0 + tm * 32 + lr;
      const floatx4 f = row < M ? *reinterpret_cast<const floatx4*>(R + (size_t)row * N + cb0 + 4 * c)
                                : floatx4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<floatx4*>(reg + lr * RS + c * 16) = f;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int tc = sn * 96 + tn * 32 + 8 * j + 4 * lh;  // column within the tile
        const floatx4 bv = *reinterpret_cast<const floatx4*>(colt + tc);
        floatx4 rv = *reinterpret_cast<const floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16);
        if constexpr (rnorm) {
          const floatx4 gg = *reinterpret_cast<const floatx4*>(colt + 256 + tc);
          const floatx4 bb = *reinterpret_cast<const floatx4*>(colt + 512 + tc);
#pragma unroll
          for (int i = 0; i < 4; ++i) rv[i] = (rv[i] - rmu[tm]) * rrs[tm] * gg[i] + bb[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[tm][tn][4 * j + i] = (acc[tm][tn][4 * j + i] + bv[i]) + rv[i];
          asm volatile("" : "+v"(acc[tm][tn][4 * j + i]));
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  float mean96[2], m2_96[2];
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
    float sum = 0.f;
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += acc[tm][tn][r];
    sum += __shfl_xor(sum, 32, 64);
    const float mu = sum * (1.f / 96.f);
    float q = 0.f;
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = acc[tm][tn][r] - mu;
        q += d * d;
      }
    q += __shfl_xor(q, 32, 64);
    mean96[tm] = mu;
    m2_96[tm] = q;
  }
  if (lh == 0) {
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) lst[(wave * 2 + tm) * 32 + li] = RowStat{mean96[tm], m2_96[tm]};
  }
  __syncthreads();
  if (sn == 0 && lh == 0) {
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
      const RowStat o = lst[((wave ^ 1) * 2 + tm) * 32 + li];
      const float d = mean96[tm] - o.mean;
      const RowStat t2{(mean96[tm] + o.mean) * 0.5f, (m2_96[tm] + o.m2) + 48.f * d * d};
      if (rb0 + 32 * tm < M) ln.stats[(size_t)(rb0 + 32 * tm) * 4 + tn0] = __builtin_bit_cast(uint64_t, t2);
    }
  }
#pragma unroll
  for (int tm = 0; tm < 2; ++tm) {
#pragma unroll
    for (int tn = 0; tn < 3; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        floatx4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = acc[tm][tn][4 * j + i];
        *reinterpret_cast<floatx4*>(reg + li * RS + (tn * 8 + 2 * j + lh) * 16) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int kk = k % 3, g2 = k / 3;
      const int idx = kk * 64 + lane, lr = idx / 12 + 16 * g2, c8 = idx % 12;
      const int row = prow0 + tm * 32 + lr;
      const floatx4 o0 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32);
      const floatx4 o1 = *reinterpret_cast<const floatx4*>(reg + lr * RS + c8 * 32 + 16);
      if (row < M) {
        const int col = cb0 + 8 * c8;
        float* const vrow = C + (size_t)prow0 * N + (uint32_t)(lr + tm * 32) * (uint32_t)N;
        *reinterpret_cast<floatx4*>(vrow + col) = o0;
        *reinterpret_cast<floatx4*>(vrow + col + 4) = o1;
        uint32_t h[4], l[4];
        floatx4 p0 = o0, p1 = o1;  // the planes hold v - kappa (the plane shift, FoldArgs)
        if (ln.shift) {
          const float* const kap = colt + 768;  // SIDE + 3072
          p0 -= *reinterpret_cast<const floatx4*>(kap + (col - n0));
          p1 -= *reinterpret_cast<const floatx4*>(kap + (col - n0) + 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          split_pair(i < 2 ? gelu_f2{p0[2 * i], p0[2 * i + 1]} : gelu_f2{p1[2 * i - 4], p1[2 * i - 3]},
                     h[i], l[i]);
        unsigned short* dstp = reinterpret_cast<unsigned short*>(ln.xp) + (size_t)prow0 * NP * N +
                               (uint32_t)(lr + tm * 32) * (uint32_t)(NP * N) +
                               (uint32_t)((col >> 5) * 32 * NP + (col & 31));
        *reinterpret_cast<uint4*>(dstp) = uint4{h[0], h[1], h[2], h[3]};
        if (NP == 2) *reinterpret_cast<uint4*>(dstp + 32) = uint4{l[0], l[1], l[2], l[3]};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// DIAG value of the persistent launch (exact results): one workgroup per CU looping over tiles
constexpr int PP_PERSIST = 9;

template <int NP, int EPI, int DIAG>
hipError_t pp_launch(const __bf16* A, const __bf16* W, const float* bias, const float* R, float* C,
                     __bf16* Cp, int M, int N, int K, int group_m, hipStream_t st,
                     FoldArgs fold = FoldArgs{}) {
  // 128 KiB (+ 11 KiB of side data for the folded epilogues: bias' / s columns, row statistics,
  // the accumulator start kc)
  constexpr int lds = 2 * (256 + 256) * PK_ROWB +
                      (EPI == PK_EPI_GELU_FOLD || EPI == PK_EPI_BIAS_FOLD ? 11264 : 0);
  if (hipError_t e = ensure_dynamic_lds((const void*)gemm_pp_kernel<NP, EPI, DIAG>, lds); e != hipSuccess)
    return e;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  // persistent grid (one workgroup per CU looping over the tiles) or one workgroup per tile
  const int grid = DIAG == PP_PERSIST ? std::min(tiles, cu_count()) : tiles;
  hipLaunchKernelGGL((gemm_pp_kernel<NP, EPI, DIAG>), dim3(grid), dim3(512), lds, st, A, W, bias,
                     R, C, Cp, M, N, K, group_m, fold);
  return hipGetLastError();
}

template <int NP, int DIAG>
hipError_t pp_epi(int epi, const __bf16* A, const __bf16* W, const float* bias, const float* R,
                  float* C, __bf16* Cp, int M, int N, int K, int group_m, hipStream_t st) {
  if constexpr (DIAG != 0 && DIAG != PP_PERSIST) {  // diagnostic builds: split-bf16, bias / GELU only
    if (NP != 2 || (epi != PK_EPI_BIAS && epi != PK_EPI_GELU_PACKED)) return hipErrorInvalidValue;
    if (epi == PK_EPI_BIAS)
      return pp_launch<2, PK_EPI_BIAS, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    return pp_launch<2, PK_EPI_GELU_PACKED, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
  } else {
    switch (epi) {
      case PK_EPI_BIAS:
        return pp_launch<NP, PK_EPI_BIAS, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
      case PK_EPI_GELU_PACKED:
        return pp_launch<NP, PK_EPI_GELU_PACKED, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
      case PK_EPI_BIAS_PACKED:
        return pp_launch<NP, PK_EPI_BIAS_PACKED, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
      case PK_EPI_RES:
        return pp_launch<NP, PK_EPI_RES, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
      default: return pp_launch<NP, PK_EPI_TANH, DIAG>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    }
  }
}

template <int NP, int EPI, bool NT = false>
hipError_t pp192_launch(const __bf16* A, const __bf16* W, const float* bias, const float* R,
                        float* C, int M, int N, int K, int group_m, hipStream_t st,
                        StatArgs ln = StatArgs{}) {
  // 112 KiB (+ 12 KiB of side data for the residual + statistics epilogues: bias, gamma, beta,
  // the residual rows' statistics, the plane shift)
  constexpr int lds = 2 * (256 + 192) * PK_ROWB +
                      (EPI == PK_EPI_RES_STATS || EPI == PK_EPI_RES_STATS_LN ? 12288 : 0);
  if (hipError_t e = ensure_dynamic_lds((const void*)gemm_pp192_kernel<NP, EPI, NT>, lds); e != hipSuccess)
    return e;
  const int tiles_m = (M + 255) / 256;
  const int tiles = tiles_m * ((N + 191) / 192);
  hipLaunchKernelGGL((gemm_pp192_kernel<NP, EPI, NT>), dim3(tiles), dim3(512), lds, st, A, W, bias, R,
                     C, M, N, K, group_m, ln);
  return hipGetLastError();
}

template <int NP, int EPI, int V = 0>
hipError_t p2_launch(const __bf16* A, const __bf16* W, const float* bias, const float* R, float* C,
                     int M, int N, int K, int group_m, hipStream_t st, StatArgs ln,
                     FoldArgs fold = FoldArgs{}) {
  constexpr int lds = 2 * (128 + 192) * PK_ROWB;  // 80 KiB: two workgroups per CU
  if (hipError_t e = ensure_dynamic_lds((const void*)gemm_p2_kernel<NP, EPI, V>, lds); e != hipSuccess)
    return e;
  const int tiles = ((M + 127) / 128) * ((N + 191) / 192);
  hipLaunchKernelGGL((gemm_p2_kernel<NP, EPI, V>), dim3(tiles), dim3(256), lds, st, A, W, bias, R,
                     C, M, N, K, group_m, ln, fold);
  return hipGetLastError();
}

// f32 epilogues only (bias, +residual, tanh); N % 32 == 0
hipError_t pp192_dispatch(const unsigned short* A, const unsigned short* W, const float* bias,
                          const float* R, float* C, unsigned short* Cp, int M, int N, int K,
                          int epi, int np, int group_m, hipStream_t st, bool nt = false) {
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  if (epi == PK_EPI_GELU_PACKED) return hipErrorInvalidValue;
  if (epi == PK_EPI_BIAS_PACKED) {  // packed planes into Cp (passed as the kernel's C)
    if (N % 192 != 0 || !Cp || nt) return hipErrorInvalidValue;
    float* cp = reinterpret_cast<float*>(Cp);
    if (np == 2) return pp192_launch<2, PK_EPI_BIAS_PACKED>(a, w, bias, R, cp, M, N, K, group_m, st);
    return pp192_launch<1, PK_EPI_BIAS_PACKED>(a, w, bias, R, cp, M, N, K, group_m, st);
  }
  if (nt) {  // timing variant (ae_bench_gemm_packed diag 8): non-temporal stores
#ifdef AE_TOOLS
    if (np != 2 || (epi != PK_EPI_RES && epi != PK_EPI_BIAS)) return hipErrorInvalidValue;
    if (epi == PK_EPI_BIAS) return pp192_launch<2, PK_EPI_BIAS, true>(a, w, bias, R, C, M, N, K, group_m, st);
    return pp192_launch<2, PK_EPI_RES, true>(a, w, bias, R, C, M, N, K, group_m, st);
#else
    return hipErrorInvalidValue;
#endif
  }
  if (np == 2) {
    if (epi == PK_EPI_BIAS) return pp192_launch<2, PK_EPI_BIAS>(a, w, bias, R, C, M, N, K, group_m, st);
    if (epi == PK_EPI_RES) return pp192_launch<2, PK_EPI_RES>(a, w, bias, R, C, M, N, K, group_m, st);
    return pp192_launch<2, PK_EPI_TANH>(a, w, bias, R, C, M, N, K, group_m, st);
  }
  if (epi == PK_EPI_BIAS) return pp192_launch<1, PK_EPI_BIAS>(a, w, bias, R, C, M, N, K, group_m, st);
  if (epi == PK_EPI_RES) return pp192_launch<1, PK_EPI_RES>(a, w, bias, R, C, M, N, K, group_m, st);
  return pp192_launch<1, PK_EPI_TANH>(a, w, bias, R, C, M, N, K, group_m, st);
}

template <int DIAG>
hipError_t pp_dispatch(const unsigned short* A, const unsigned short* W, const float* bias,
                       const float* R, float* C, unsigned short* Cp, int M, int N, int K, int epi,
                       int np, int group_m, hipStream_t st) {
  auto bf = [](const unsigned short* p) { return reinterpret_cast<const __bf16*>(p); };
  __bf16* cp = reinterpret_cast<__bf16*>(Cp);
  if (np == 2) return pp_epi<2, DIAG>(epi, bf(A), bf(W), bias, R, C, cp, M, N, K, group_m, st);
  return pp_epi<1, DIAG>(epi, bf(A), bf(W), bias, R, C, cp, M, N, K, group_m, st);
}
}  // namespace

namespace {
constexpr int PK_GROUP_M = 4;  // grouped tile order: 4 > 8 > 16 > 32 M-tiles by A/B (round 1);
                               // re-swept on the ping-pong kernel (profiles/r3at_gemm_group_m_ab.jsonl)

bool pk_shape_ok(int M, int N, int K, int np) {
  return K % 64 == 0 && N % 32 == 0 && (np == 1 || np == 2) && N > 0 && M >= 0;
}
}  // namespace

namespace {
int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// tile width of the ping-pong GEMM for an M x N output (see ae_launch_gemm_packed)
// packed192: the 256 x 192 kernel may take the packed-plane (QKV) epilogue too
int pp_choose(int M, int N, int epi, bool packed192 = false) {
  if (epi == PK_EPI_GELU_PACKED) return 256;
  if (epi == PK_EPI_BIAS_PACKED && (N % 192 != 0 || !packed192)) return 256;
  const long tm = (M + 255) / 256, cus = cu_count();
  const long r256 = (tm * ((N + 255) / 256) + cus - 1) / cus;
  const long r192 = (tm * ((N + 191) / 192) + cus - 1) / cus;
  return 0.89 * (double)r192 < (double)r256 ? 192 : 256;
}
}  // namespace

// C = A·W^T (+epilogue) over packed bf16 planes.  A: [M][np*K], W: [N][np*K] packed (see top);
// f32 output C [M][N] or packed output planes Cp [M][np*N] (GELU epilogue).  np: 2 = split-bf16
// (f32-class), 1 = plain bf16.  Requires K % 64 == 0 and N % 32 == 0.
extern "C" hipError_t ae_launch_gemm_packed(const unsigned short* A, const unsigned short* W,
                                            const float* bias, const float* R, float* C,
                                            unsigned short* Cp, int M, int N, int K, int epi,
                                            int np, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!pk_shape_ok(M, N, K, np)) return hipErrorInvalidValue;
  // the ping-pong kernels for every encoder GEMM: 256 x 192 or 256 x 256 tiles, whichever
  // finishes first by rounds of CU-count tiles x per-tile time (tools/gemm_bench.py: a 256 x 192
  // round takes 0.89 of a 256 x 256 round; the 192 kernel has f32 epilogues only)
  return pp_choose(M, N, epi) == 192
             ? pp192_dispatch(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st)
             : pp_dispatch<0>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
}



// The folded-LayerNorm pair (FoldArgs).  Cp = packed planes of
//   gelu = 0: rstd * (A·W'^T - mean * s) + bias'          (the QKV GEMM of layers >= 1)
//   gelu = 1: GELU(rstd * (A·W'^T - mean * s) + bias')    (FFN1)
// A: the packed planes of the pre-LayerNorm rows v (of v - kappa under the plane shift, when kc =
// kappa·W'^T is given: the accumulators start at kc); stats: v's [M][4] tile statistics.
extern "C" hipError_t ae_launch_gemm_packed_fold(const unsigned short* A, const unsigned short* W,
                                                 const float* bias, const float* s,
                                                 const uint64_t* stats, float eps,
                                                 unsigned short* Cp, int M, int N, int K, int gelu,
                                                 int np, const float* kc, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!pk_shape_ok(M, N, K, np) || !bias || !s || !stats || !Cp) return hipErrorInvalidValue;
  const FoldArgs fold{s, stats, eps, kc};
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  __bf16* cp = reinterpret_cast<__bf16*>(Cp);
  if (np == 2)
    return gelu ? pp_launch<2, PK_EPI_GELU_FOLD, 0>(a, w, bias, nullptr, nullptr, cp, M, N, K, PK_GROUP_M, st, fold)
                : pp_launch<2, PK_EPI_BIAS_FOLD, 0>(a, w, bias, nullptr, nullptr, cp, M, N, K, PK_GROUP_M, st, fold);
  return gelu ? pp_launch<1, PK_EPI_GELU_FOLD, 0>(a, w, bias, nullptr, nullptr, cp, M, N, K, PK_GROUP_M, st, fold)
              : pp_launch<1, PK_EPI_BIAS_FOLD, 0>(a, w, bias, nullptr, nullptr, cp, M, N, K, PK_GROUP_M, st, fold);
}

// LayerNorm of M pre-LayerNorm rows v from their [M][4] tile statistics (row_norm's merge order)
// with the expression the PK_EPI_RES_STATS_LN residual uses, so the last full layer's output x (the
// CLS path, MLM head and encode outputs) carries the same bits as every folded consumer's view of
// the same rows.  One wave per row.
__global__ __launch_bounds__(256) void layernorm_stats_kernel(const float* __restrict__ v,
                                                              const uint64_t* __restrict__ stats,
                                                              const float* __restrict__ g,
                                                              const float* __restrict__ b,
                                                              float eps, int M,
                                                              float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  float mu, rs;
  row_norm(stats + (size_t)row * 4, eps, mu, rs);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    const floatx4 x = *reinterpret_cast<const floatx4*>(v + (size_t)row * 768 + col);
    const floatx4 gg = *reinterpret_cast<const floatx4*>(g + col);
    const floatx4 bb = *reinterpret_cast<const floatx4*>(b + col);
    floatx4 y;
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = (x[i] - mu) * rs * gg[i] + bb[i];
    *reinterpret_cast<floatx4*>(out + (size_t)row * 768 + col) = y;
  }
}

extern "C" hipError_t ae_launch_layernorm_stats(const float* v, const uint64_t* stats,
                                                const float* g, const float* b, float eps, int M,
                                                float* out, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(layernorm_stats_kernel, dim3((M + 3) / 4), dim3(256), 0, st, v, stats, g, b,
                     eps, M, out);
  return hipGetLastError();
}

// v = A·W^T + bias + r over rows of N = 768 (the O-projection / FFN2), written as f32 C and packed
// planes Cp of v - shift (shift null: of v; the plane shift, FoldArgs), with the (mean, M2) of every
// row of v over each of its 4 192-column tiles into stats ([M][4] 8-B words).  r = R as it is when rstats is null, else r = LN(R) with R's own tile
// statistics rstats and gamma / beta (R a pre-LayerNorm row).  R may equal C.
extern "C" hipError_t ae_launch_gemm_packed_res_stats(
    const unsigned short* A, const unsigned short* W, const float* bias, const float* R,
    const uint64_t* rstats, const float* gamma, const float* beta, float eps, float* C,
    unsigned short* Cp, uint64_t* stats, int M, int N, int K, int np, const float* shift,
    hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (N != 768 || K % 64 != 0 || (np != 1 && np != 2) || !bias || !R || !C || !Cp || !stats ||
      (rstats && (!gamma || !beta)))
    return hipErrorInvalidValue;
  const StatArgs ln{gamma, beta, eps, reinterpret_cast<__bf16*>(Cp), stats, rstats, shift};
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  if (rstats)
    return np == 2 ? pp192_launch<2, PK_EPI_RES_STATS_LN>(a, w, bias, R, C, M, N, K, PK_GROUP_M, st, ln)
                   : pp192_launch<1, PK_EPI_RES_STATS_LN>(a, w, bias, R, C, M, N, K, PK_GROUP_M, st, ln);
  return np == 2 ? pp192_launch<2, PK_EPI_RES_STATS>(a, w, bias, R, C, M, N, K, PK_GROUP_M, st, ln)
                 : pp192_launch<1, PK_EPI_RES_STATS>(a, w, bias, R, C, M, N, K, PK_GROUP_M, st, ln);
}

#ifdef AE_TOOLS
// ---- tools library only (lib/libalert_engine_tools.so, -DAE_TOOLS): timing experiments whose
// variants give WRONG results on purpose; the product library exports none of this.

// ae_launch_gemm_packed_res_stats with an explicit kernel: variant 0 = gemm_pp192_kernel (one
// 256 x 192 workgroup per CU), 1 = gemm_p2_kernel (two 128 x 192 workgroups per CU, M-tiles
// grouped by `group` (0: 8)).  Exact results in both.
extern "C" hipError_t ae_bench_gemm_packed_res_stats(
    const unsigned short* A, const unsigned short* W, const float* bias, const float* R,
    const uint64_t* rstats, const float* gamma, const float* beta, float eps, float* C,
    unsigned short* Cp, uint64_t* stats, int M, int N, int K, int np, const float* shift,
    int variant, int group, hipStream_t st) {
  if (variant == 0)
    return ae_launch_gemm_packed_res_stats(A, W, bias, R, rstats, gamma, beta, eps, C, Cp, stats,
                                           M, N, K, np, shift, st);
  if (M <= 0) return hipSuccess;
  if ((variant != 1 && variant != 2) || N != 768 || K % 64 != 0 || (np != 1 && np != 2) || !bias ||
      !R || !C || !Cp || !stats || (rstats && (!gamma || !beta)))
    return hipErrorInvalidValue;
  const StatArgs ln{gamma, beta, eps, reinterpret_cast<__bf16*>(Cp), stats, rstats, shift};
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  const int gm = group > 0 ? group : 8;
  if (variant == 2) {  // fragment reads pipelined against the MFMAs (V 1)
    if (rstats)
      return np == 2 ? p2_launch<2, PK_EPI_RES_STATS_LN, 1>(a, w, bias, R, C, M, N, K, gm, st, ln)
                     : p2_launch<1, PK_EPI_RES_STATS_LN, 1>(a, w, bias, R, C, M, N, K, gm, st, ln);
    return np == 2 ? p2_launch<2, PK_EPI_RES_STATS, 1>(a, w, bias, R, C, M, N, K, gm, st, ln)
                   : p2_launch<1, PK_EPI_RES_STATS, 1>(a, w, bias, R, C, M, N, K, gm, st, ln);
  }
  if (rstats)
    return np == 2 ? p2_launch<2, PK_EPI_RES_STATS_LN>(a, w, bias, R, C, M, N, K, gm, st, ln)
                   : p2_launch<1, PK_EPI_RES_STATS_LN>(a, w, bias, R, C, M, N, K, gm, st, ln);
  return np == 2 ? p2_launch<2, PK_EPI_RES_STATS>(a, w, bias, R, C, M, N, K, gm, st, ln)
                 : p2_launch<1, PK_EPI_RES_STATS>(a, w, bias, R, C, M, N, K, gm, st, ln);
}

// ae_launch_gemm_packed_fold with an explicit kernel: variant 0 = gemm_pp_kernel (one 256 x 256
// workgroup per CU, the production launch), 1 = gemm_p2_kernel (two 128 x 192 workgroups per CU,
// M-tiles grouped by `group` (0: 8), kc added in the epilogue instead of preloaded: equal to the
// production results up to f32 rounding).  N % 192 == 0.
extern "C" hipError_t ae_bench_gemm_packed_fold(const unsigned short* A, const unsigned short* W,
                                                const float* bias, const float* s,
                                                const uint64_t* stats, float eps,
                                                unsigned short* Cp, int M, int N, int K, int gelu,
                                                int np, const float* kc, int variant, int group,
                                                hipStream_t st) {
  if (variant == 0)
    return ae_launch_gemm_packed_fold(A, W, bias, s, stats, eps, Cp, M, N, K, gelu, np, kc, st);
  if (M <= 0) return hipSuccess;
  if (variant != 1 || N % 192 != 0 || K % 64 != 0 || (np != 1 && np != 2) || !bias || !s ||
      !stats || !Cp)
    return hipErrorInvalidValue;
  StatArgs ln{};
  ln.xp = reinterpret_cast<__bf16*>(Cp);
  const FoldArgs fold{s, stats, eps, kc};
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  const int gm = group > 0 ? group : 8;
  if (np == 2)
    return gelu ? p2_launch<2, PK_EPI_GELU_FOLD>(a, w, bias, nullptr, nullptr, M, N, K, gm, st, ln, fold)
                : p2_launch<2, PK_EPI_BIAS_FOLD>(a, w, bias, nullptr, nullptr, M, N, K, gm, st, ln, fold);
  return gelu ? p2_launch<1, PK_EPI_GELU_FOLD>(a, w, bias, nullptr, nullptr, M, N, K, gm, st, ln, fold)
              : p2_launch<1, PK_EPI_BIAS_FOLD>(a, w, bias, nullptr, nullptr, M, N, K, gm, st, ln, fold);
}

// Kernel experiments (tools/gemm_bench.py, tests): explicit tile width (0 = the production choice)
// and a diagnostic variant (0 = the production kernel; see DIAG above — values 1-7 give WRONG
// results and exist only to time parts of the pipeline).  Variant 8 is exact and flips the store
// flavour of the epilogue: plain stores for the 256 x 256 kernel (production: non-temporal, about
// 2 % faster on FFN1 / QKV), non-temporal for the 256 x 192 kernel (production: plain; mixed
// +-3 % on O-proj / FFN2).  Not part of include/alert_engine.h.
extern "C" hipError_t ae_bench_gemm_packed(const unsigned short* A, const unsigned short* W,
                                           const float* bias, const float* R, float* C,
                                           unsigned short* Cp, int M, int N, int K, int epi,
                                           int np, int bn, int diag, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!pk_shape_ok(M, N, K, np) || (bn != 0 && bn != 192 && bn != 512))
    return hipErrorInvalidValue;
  if (bn == 0) bn = pp_choose(M, N, epi) == 192 ? 192 : 512;
  if (bn == 192)  // diag 8: non-temporal stores; 21-52: grouped order of diag - 20 M-tiles
    return pp192_dispatch(A, W, bias, R, C, Cp, M, N, K, epi, np,
                          diag >= 21 && diag <= 52 ? diag - 20 : PK_GROUP_M, st, diag == 8);
  if (bn == 512 && diag >= 21 && diag <= 52)  // production kernel, grouped order of diag - 20 M-tiles
    return pp_dispatch<0>(A, W, bias, R, C, Cp, M, N, K, epi, np, diag - 20, st);
  if (bn == 512) {  // the ping-pong 256 x 256 kernel
    switch (diag) {
      case 0: return pp_dispatch<0>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 1: return pp_dispatch<1>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 2: return pp_dispatch<2>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 3: return pp_dispatch<3>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 4: return pp_dispatch<4>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 5: return pp_dispatch<5>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 6: return pp_dispatch<6>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 7: return pp_dispatch<7>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 8: return pp_dispatch<8>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      case 9: return pp_dispatch<9>(A, W, bias, R, C, Cp, M, N, K, epi, np, PK_GROUP_M, st);
      default: return hipErrorInvalidValue;
    }
  }
  return hipErrorInvalidValue;
}
#endif  // AE_TOOLS
