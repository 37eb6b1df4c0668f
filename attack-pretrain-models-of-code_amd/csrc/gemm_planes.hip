// gemm_planes.hip — packed bf16-plane MFMA GEMM of the split-precision encoder
// (AE_PREC_BF16 / AE_PREC_F32X3).
//
// Operands arrive already split into bf16: the weights at engine creation (W = W_hi + W_lo), the
// activations by the kernel that produced them (LayerNorm, attention, the FFN1 epilogue), so the
// main loop moves and multiplies nothing but bf16.  Packed layout ("NP planes per 128-B block"):
//   NP = 2 (f32x3): row = K/32 blocks of 128 B, block b = [hi of k 32b..32b+31 | lo of the same]
//   NP = 1 (bf16):  row = K bf16 (the hi plane)
// so one K-tile of a row is always one full 128-B cache line.  With NP = 2 every product is
//     a·w ≈ a_hi·w_hi + a_hi·w_lo + a_lo·w_hi          (3 bf16 MFMAs, f32 accumulate)
// from ONE load of the four planes.
//
// gfx950 mapping:
//   * tile 256 x BN (BN = 256: 8 waves as 2 x 4, wave tile 128 x 64; BN = 128: 4 x 2, 64 x 64),
//     one 512-thread workgroup per CU, LDS NST x (256 + BN) x 128 B (NST = 3 stages for BN = 128,
//     2 for BN = 256)
//   * operands reach LDS by LDS-DMA (global_load_lds_dwordx4, one wave instruction = 8 rows x
//     128 B, lane-linear image); the 16-B chunk of row r is XOR-swizzled by (r >> 1) & 7 on the
//     SOURCE address, so fragment ds_read_b128s of 16 rows hit 16 different bank slots
//   * a K-tile's fragments are pulled from LDS into registers as soon as the tile has landed;
//     2 stages (BN = 256): once every wave holds them (a second barrier) the stage is refilled
//     with tile k+2; 3 stages (BN = 128): tile k+2 goes into tile k-1's stage right after the
//     K-tile's one barrier, so two K-tiles of DMA are in flight behind the MFMAs — the kernel is
//     bound by how many bytes a CU keeps in flight (tools/gemm_bench.py diag runs)
//   * the MFMAs of the first half of the tile run between the fragment reads and that barrier,
//     overlapping the LDS reads of the other waves
//   * DMA issued from inline asm with hand-counted vmcnt (the compiler's wait-count pass would
//     otherwise drain it before every fragment read); raw s_barrier; XCD-aware tile order
//   * epilogues: +bias -> f32, +bias+residual -> f32, +bias -> tanh -> f32, +bias -> GELU -> packed
//     bf16 planes (the FFN2 operand)
#include "common.h"


// m0 is written only by dma16 below; nothing else in these kernels reads it
#pragma clang diagnostic ignored "-Winline-asm"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

enum { PK_EPI_BIAS = 0, PK_EPI_GELU_PACKED = 1, PK_EPI_RES = 2, PK_EPI_TANH = 3 };

namespace {
constexpr int PK_BM = 256, PK_ROWB = 128;

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
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

// LDS stages of the DMA ring: 3 when they fit in 160 KiB (256 x 128 tiles: 3 x 48 KiB), else 2
template <int BN>
constexpr int pk_stages() { return 3 * (256 + BN) * 128 <= 160 * 1024 ? 3 : 2; }
}  // namespace

// keeps a value live in a diagnostic build whose consumer was cut out (rule 17)
__device__ __forceinline__ void keep_f32(float x) { asm volatile("" ::"v"(x)); }

// element offset of (row, col) in a packed [rows][NP*ld] matrix, plane p
__device__ __forceinline__ size_t pk_index(int row, int col, int ld, int np, int p) {
  return (size_t)row * np * ld + (size_t)(col >> 5) * 32 * np + 32 * p + (col & 31);
}

// DIAG (timing experiments only, reachable only through ae_bench_gemm_packed; results WRONG):
// 1 = no refill DMA after the first two K-tiles, 2 = no post-read barrier, 3 = no barriers at
// all, 4 = no fragment reads after the first K-tile, 5 = no MFMAs, 6 = epilogue only,
// 7 = no epilogue stores.  The production instantiations have DIAG = 0.
template <int BN, int NP, int EPI, int DIAG>
__global__ __launch_bounds__(512, 1) void gemm_pk_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ R, float* __restrict__ C, __bf16* __restrict__ Cp, int M, int N,
    int K, int group_m) {
  constexpr int diag = DIAG;
  extern __shared__ __attribute__((aligned(16))) unsigned char pk_smem[];
  constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  constexpr int TM = PK_BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_BYTES = PK_BM * PK_ROWB, W_BYTES = BN * PK_ROWB;
  constexpr int STAGE = A_BYTES + W_BYTES;
  constexpr int NST = pk_stages<BN>();                 // ring depth: NST-1 K-tiles in flight
  constexpr int A_DMA = PK_BM / 64, W_DMA = BN / 64;  // DMA instructions per wave per K-tile
  constexpr int DMA = A_DMA + W_DMA;
  constexpr int KB = 64 / NP;                          // k per K-tile
  constexpr int NS = KB / 16;                          // 16-deep MFMA steps per K-tile
  constexpr int NS0 = NS / 2;                          // steps multiplied before the refill

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + PK_BM - 1) / PK_BM;
  // XCD-contiguous tile order, then grouped: group_m M-tiles sweep the N-tiles together, so the
  // ~32 tiles an XCD runs at once share both their A rows and their W rows in its L2
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm = first_m + (t - g * per_group) % gsize, tn = (t - g * per_group) / gsize;
  const int m0 = tm * PK_BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, lh = lane >> 5;
  const size_t lda = (size_t)NP * K;  // packed row length (elements), A and W

  // ---- per-lane DMA sources at K-tile 0 (instruction u covers rows 8 * (DMA_X * wave + u) + lane/8)
  const char* a_src[A_DMA];
  const char* w_src[W_DMA];
#pragma unroll
  for (int u = 0; u < A_DMA; ++u) {
    const int r = 8 * (A_DMA * wave + u) + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = m0 + r < M ? m0 + r : M - 1;
    a_src[u] = reinterpret_cast<const char*>(A + gr * lda) + 16 * cs;
  }
#pragma unroll
  for (int u = 0; u < W_DMA; ++u) {
    const int r = 8 * (W_DMA * wave + u) + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = n0 + r < N ? n0 + r : N - 1;
    w_src[u] = reinterpret_cast<const char*>(W + gr * lda) + 16 * cs;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)pk_smem;
  const int nk = diag == 6 ? 0 : K / KB;

  auto issue = [&](int kt) {
    const int kb = kt * PK_ROWB;  // byte offset of K-tile kt in a packed row
    const uint32_t st = lds0 + (kt % NST) * STAGE;
#pragma unroll
    for (int u = 0; u < A_DMA; ++u) dma16(a_src[u] + kb, st + (A_DMA * wave + u) * 1024);
#pragma unroll
    for (int u = 0; u < W_DMA; ++u) dma16(w_src[u] + kb, st + A_BYTES + (W_DMA * wave + u) * 1024);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // fragment rows are 32-aligned + li, so the row swizzle is (li >> 1) & 7
  const int sw = (li >> 1) & 7;
  const int a_row0 = (wm * (PK_BM / WM) + li) * PK_ROWB;
  const int w_row0 = A_BYTES + (wn * (BN / WN) + li) * PK_ROWB;

  auto mfma_step = [&](const bf16x8 (&fa)[NP][TM], const bf16x8 (&fw)[NP][TN]) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        if (NP == 2) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][a], fw[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][a], fw[1][b], acc[a][b], 0, 0, 0);
        }
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][a], fw[0][b], acc[a][b], 0, 0, 0);
      }
  };

  auto keep_live = [&](const bf16x8 (&fa)[NP][TM], const bf16x8 (&fw)[NP][TN]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int a = 0; a < TM; ++a) asm volatile("" ::"v"(fa[p][a]));
#pragma unroll
      for (int b = 0; b < TN; ++b) asm volatile("" ::"v"(fw[p][b]));
    }
  };

  bf16x8 fa[NS][NP][TM], fw[NS][NP][TN];
  // prologue: tiles 0 and 1 (both ring depths refill with tile kt+2 during iteration kt)
  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's DMA; kt+1 may still be in flight), then visible to all waves
    if (kt + 1 < nk) wait_vm<DMA>();
    else wait_vm<0>();
    if (diag != 3) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const unsigned char* st = pk_smem + (kt % NST) * STAGE;
    if constexpr (NST == 3) {
      // 3-stage ring: every wave is past this barrier, so every wave has finished reading tile
      // kt-1 — its stage takes tile kt+2 during this K-tile, and one barrier per K-tile suffices.
      // Issue order, pinned: step-0 fragment reads, then the step-0.. MFMAs with the later
      // steps' fragment reads and the DMA pieces of tile kt+2 spread between them (a DMA piece
      // issued in a burst holds the wave's issue for ~60-100 cycles each; between MFMAs it
      // hides in their issue gaps), then the last step's MFMAs.
      constexpr int T = NP == 2 ? 3 : 1;
      constexpr int MPS = T * TM * TN;           // MFMAs per 16-deep step
      constexpr int RPS = NP * (TM + TN);         // fragment reads per step
      constexpr int MU = (NS - 1) * MPS, RU = (NS - 1) * RPS;
      auto read_one = [&](int s, int i) {        // i-th fragment read of step s
        const int p = i / (TM + TN), j = i % (TM + TN);
        const int coff = 16 * ((4 * p + 2 * s + lh) ^ sw);
        if (j < TN)
          fw[s][p][j] = *reinterpret_cast<const bf16x8*>(st + w_row0 + j * 32 * PK_ROWB + coff);
        else
          fa[s][p][j - TN] =
              *reinterpret_cast<const bf16x8*>(st + a_row0 + (j - TN) * 32 * PK_ROWB + coff);
      };
      auto mfma_one = [&](int s, int i) {        // i-th MFMA of step s
        const int a = i / (T * TN), b = (i / T) % TN, term = i % T;
        if (diag == 5) {
          keep_f32(acc[a][b][0]);
          return;
        }
        const bf16x8& x = (T == 3 && term == 0) ? fa[s][NP - 1][a] : fa[s][0][a];
        const bf16x8& y = (T == 3 && term == 1) ? fw[s][NP - 1][b] : fw[s][0][b];
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc[a][b], 0, 0, 0);
      };
      const bool refill = kt + 2 < nk && diag != 1;
      const int kb = (kt + 2) * PK_ROWB;
      const uint32_t nst = lds0 + ((kt + 2) % NST) * STAGE;
      auto dma_one = [&](int j) {
        if (!refill) return;
        if (j < A_DMA) dma16(a_src[j] + kb, nst + (A_DMA * wave + j) * 1024);
        else dma16(w_src[j - A_DMA] + kb, nst + A_BYTES + (W_DMA * wave + j - A_DMA) * 1024);
      };
#pragma unroll
      for (int i = 0; i < RPS; ++i)
        if (diag != 4 || kt == 0) read_one(0, i);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_sched_barrier(0);
      // MU MFMAs, RU reads and the DMA pieces in DMA groups, each group's share pinned in order
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int g = 0; g < DMA; ++g) {
#pragma unroll
        for (int i = g * MU / DMA; i < (g + 1) * MU / DMA; ++i) mfma_one(i / MPS, i % MPS);
#pragma unroll
        for (int i = g * RU / DMA; i < (g + 1) * RU / DMA; ++i)
          if (diag != 4 || kt == 0) read_one(1 + i / RPS, i % RPS);
        __builtin_amdgcn_sched_barrier(0);
        dma_one(g);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < MPS; ++i) mfma_one(NS - 1, i);
      __builtin_amdgcn_s_setprio(0);
      continue;
    }
    auto read_step = [&](int s) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int coff = 16 * ((4 * p + 2 * s + lh) ^ sw);
#pragma unroll
        for (int b = 0; b < TN; ++b)
          fw[s][p][b] = *reinterpret_cast<const bf16x8*>(st + w_row0 + b * 32 * PK_ROWB + coff);
#pragma unroll
        for (int a = 0; a < TM; ++a)
          fa[s][p][a] = *reinterpret_cast<const bf16x8*>(st + a_row0 + a * 32 * PK_ROWB + coff);
      }
    };
#pragma unroll
    for (int s = 0; s < NS0; ++s)
      if (diag != 4 || kt == 0) read_step(s);
    __builtin_amdgcn_sched_barrier(0);
    // first-half MFMAs interleaved with the second-half fragment reads (<= 15 LDS ops in flight)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = NS0; s < NS; ++s)
      if (diag != 4 || kt == 0) read_step(s);
#pragma unroll
    for (int s = 0; s < NS0; ++s) {
      if (diag != 5) mfma_step(fa[s], fw[s]);
      else keep_live(fa[s], fw[s]);
    }
    {
      constexpr int RD1 = (NS - NS0) * NP * (TM + TN);
      constexpr int MF0 = NS0 * (NP == 2 ? 3 : 1) * TM * TN;
      constexpr int PER = MF0 / RD1 > 0 ? MF0 / RD1 : 1;
#pragma unroll
      for (int i = 0; i < RD1; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
      }
      if (MF0 > PER * RD1) __builtin_amdgcn_sched_group_barrier(0x008, MF0 - PER * RD1, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NST == 2) {
      // every wave holds tile kt in registers: refill its stage with tile kt+2
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (diag != 2 && diag != 3) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk && diag != 1) issue(kt + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = NS0; s < NS; ++s) {
      if (diag != 5) mfma_step(fa[s], fw[s]);
      else keep_live(fa[s], fw[s]);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (DIAG == 7) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) keep_f32(acc[a][b][r]);
    return;
  }

  // ---- epilogue through LDS: each 32x32 accumulator tile is transposed through a private
  // 32 x 33-float LDS slab so that every global access is a 16-byte-per-lane row segment
  // (4 floats of C / R, or 8 hi + 8 lo bf16 of a packed block) instead of one element per lane
  __syncthreads();  // the stages are reused as scratch: every wave has finished the main loop
  float* slab = reinterpret_cast<float*>(pk_smem) + wave * 32 * 33;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int cb = n0 + wn * (BN / WN) + b * 32;  // first column of the tile (N % 32 == 0)
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int rb = m0 + wm * (PK_BM / WM) + a * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) slab[mfma32_row(r, lh) * 33 + li] = acc[a][b][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slab is written before it is read
      if (cb < N) {
        if (EPI == PK_EPI_GELU_PACKED) {
          // lane -> row (lane >> 2) + 16 pass, 8 columns c8 = 8 * (lane & 3)
          const int c8 = 8 * (lane & 3);
          floatx4 b0 = *reinterpret_cast<const floatx4*>(bias + cb + c8);
          floatx4 b1 = *reinterpret_cast<const floatx4*>(bias + cb + c8 + 4);
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const int rr = 16 * pass + (lane >> 2);
            const int row = rb + rr;
            bf16x8 h, l;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float v = gelu_erfc_fast(slab[rr * 33 + c8 + e] + (e < 4 ? b0[e] : b1[e - 4]));
              const __bf16 hv = (__bf16)v;
              h[e] = hv;
              l[e] = (__bf16)(v - (float)hv);
            }
            if (row < M) {
              __bf16* dst = Cp + (size_t)row * NP * N + (size_t)(cb >> 5) * 32 * NP + c8;
              *reinterpret_cast<bf16x8*>(dst) = h;
              if (NP == 2) *reinterpret_cast<bf16x8*>(dst + 32) = l;
            }
          }
        } else {
          // lane -> row (lane >> 3) + 8 pass, 4 columns c4 = 4 * (lane & 7)
          const int c4 = 4 * (lane & 7);
          const floatx4 bv = *reinterpret_cast<const floatx4*>(bias + cb + c4);
#pragma unroll
          for (int pass = 0; pass < 4; ++pass) {
            const int rr = 8 * pass + (lane >> 3);
            const int row = rb + rr;
            if (row < M) {
              const size_t o = (size_t)row * N + cb + c4;
              floatx4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = slab[rr * 33 + c4 + e] + bv[e];
              if (EPI == PK_EPI_TANH)
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = tanhf(v[e]);
              if (EPI == PK_EPI_RES) v += *reinterpret_cast<const floatx4*>(R + o);
              *reinterpret_cast<floatx4*>(C + o) = v;
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab reads done before the next tile overwrites it
    }
  }
}

namespace {
constexpr int PK_GROUP_M = 4;  // grouped tile order: 4 > 8 > 16 > 32 M-tiles by A/B (round 1)

template <int BN, int NP, int EPI, int DIAG>
hipError_t pk_launch(const __bf16* A, const __bf16* W, const float* bias, const float* R, float* C,
                     __bf16* Cp, int M, int N, int K, hipStream_t st) {
  constexpr int lds = pk_stages<BN>() * (PK_BM + BN) * PK_ROWB;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_pk_kernel<BN, NP, EPI, DIAG>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int tiles = ((M + PK_BM - 1) / PK_BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_pk_kernel<BN, NP, EPI, DIAG>), dim3(tiles), dim3(512), lds, st, A, W,
                     bias, R, C, Cp, M, N, K, PK_GROUP_M);
  return hipGetLastError();
}

template <int BN, int NP, int DIAG>
hipError_t pk_epi(int epi, const __bf16* A, const __bf16* W, const float* bias, const float* R,
                  float* C, __bf16* Cp, int M, int N, int K, hipStream_t st) {
  if constexpr (DIAG != 0) {  // diagnostic builds: split-bf16, bias / GELU epilogues only
    if (NP != 2 || (epi != PK_EPI_BIAS && epi != PK_EPI_GELU_PACKED)) return hipErrorInvalidValue;
    if (epi == PK_EPI_BIAS)
      return pk_launch<BN, 2, PK_EPI_BIAS, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
    return pk_launch<BN, 2, PK_EPI_GELU_PACKED, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
  }
  switch (epi) {
    case PK_EPI_BIAS: return pk_launch<BN, NP, PK_EPI_BIAS, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
    case PK_EPI_GELU_PACKED:
      return pk_launch<BN, NP, PK_EPI_GELU_PACKED, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
    case PK_EPI_RES: return pk_launch<BN, NP, PK_EPI_RES, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
    default: return pk_launch<BN, NP, PK_EPI_TANH, DIAG>(A, W, bias, R, C, Cp, M, N, K, st);
  }
}

// Tile width per problem: wall time ~ rounds of 256 CUs x per-tile time (256x128 ~0.55 of 256^2)
int pick_bn(int M, int N) {
  const long tm = (M + PK_BM - 1) / PK_BM;
  const long t256 = tm * ((N + 255) / 256), t128 = tm * ((N + 127) / 128);
  const double c256 = (double)((t256 + 255) / 256), c128 = 0.55 * (double)((t128 + 255) / 256);
  return c128 < c256 ? 128 : 256;
}

template <int DIAG>
hipError_t pk_dispatch(const unsigned short* A, const unsigned short* W, const float* bias,
                       const float* R, float* C, unsigned short* Cp, int M, int N, int K, int epi,
                       int np, int bn, hipStream_t st) {
  auto bf = [](const unsigned short* p) { return reinterpret_cast<const __bf16*>(p); };
  auto bfm = [](unsigned short* p) { return reinterpret_cast<__bf16*>(p); };
  if (np == 2) {
    if (bn == 256) return pk_epi<256, 2, DIAG>(epi, bf(A), bf(W), bias, R, C, bfm(Cp), M, N, K, st);
    return pk_epi<128, 2, DIAG>(epi, bf(A), bf(W), bias, R, C, bfm(Cp), M, N, K, st);
  }
  if (bn == 256) return pk_epi<256, 1, DIAG>(epi, bf(A), bf(W), bias, R, C, bfm(Cp), M, N, K, st);
  return pk_epi<128, 1, DIAG>(epi, bf(A), bf(W), bias, R, C, bfm(Cp), M, N, K, st);
}

bool pk_shape_ok(int M, int N, int K, int np) {
  return K % 64 == 0 && N % 32 == 0 && (np == 1 || np == 2) && N > 0 && M >= 0;
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
  return pk_dispatch<0>(A, W, bias, R, C, Cp, M, N, K, epi, np, pick_bn(M, N), st);
}

// Kernel experiments (tools/gemm_bench.py, tests): explicit tile width (0 = the production choice)
// and a diagnostic variant (0 = the production kernel; see DIAG above — other values give WRONG
// results and exist only to time parts of the pipeline).  Not part of include/alert_engine.h.
extern "C" hipError_t ae_bench_gemm_packed(const unsigned short* A, const unsigned short* W,
                                           const float* bias, const float* R, float* C,
                                           unsigned short* Cp, int M, int N, int K, int epi,
                                           int np, int bn, int diag, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!pk_shape_ok(M, N, K, np) || (bn != 0 && bn != 128 && bn != 256)) return hipErrorInvalidValue;
  if (bn == 0) bn = pick_bn(M, N);
  switch (diag) {
    case 0: return pk_dispatch<0>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 1: return pk_dispatch<1>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 2: return pk_dispatch<2>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 3: return pk_dispatch<3>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 4: return pk_dispatch<4>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 5: return pk_dispatch<5>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 6: return pk_dispatch<6>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    case 7: return pk_dispatch<7>(A, W, bias, R, C, Cp, M, N, K, epi, np, bn, st);
    default: return hipErrorInvalidValue;
  }
}
