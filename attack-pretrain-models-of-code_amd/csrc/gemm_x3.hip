// gemm_x3.hip — split-bf16 MFMA GEMM: f32-class accuracy at bf16 matrix-core rate.
//
// C[M,N] = A[M,K] · W[N,K]^T + bias (+GELU | +residual | tanh), A and C f32, W pre-split at
// engine creation into W = W_hi + W_lo (two bf16 arrays, round-to-nearest-even).  A is split the
// same way while it is staged into LDS.  With TERMS = 3 every product is
//     a·w ≈ a_hi·w_hi + a_hi·w_lo + a_lo·w_hi        (dropped a_lo·w_lo and split residual
//                                                      ~2^-16 relative per product)
// accumulated in f32 by v_mfma_f32_32x32x16_bf16 (bf16 products are exact in f32).  Measured on
// the full 12-layer victim: |Δp| ≤ 3e-5 against the exact-f32 oracle, inside the 1e-4 parity
// tolerance, at 3 bf16 MFMAs per product (5.3x the f32 MFMA peak before efficiency).  TERMS = 1
// is plain bf16 (the stated-tolerance bf16 mode).
//
// gfx950 mapping: 512-thread workgroup (8 waves) on a BM x BN tile, BK = 32 (two 16-deep MFMA
// steps).  LDS keeps A_hi, A_lo, W_hi, W_lo tiles as 64-byte rows (32 bf16) whose four 16-byte
// chunks are XOR-swizzled by (row >> 2) & 3, so the ds_read_b128 fragment reads of 16 different
// rows hit 16 different bank slots; two stages (double buffer).  Global loads of the next K-tile
// are issued before the current tile's MFMAs and written to LDS after them (T14 split), one
// barrier per K-tile.  Tile order is XCD-remapped so neighbouring tiles share an XCD's L2.
#include "common.h"

#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int BK = 32;
constexpr int ROWB = 64;  // bytes per LDS row (32 bf16)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
}  // namespace

enum { X3_EPI_BIAS = 0, X3_EPI_GELU = 1, X3_EPI_RES = 2, X3_EPI_TANH = 3 };

template <int BM, int BN, int WM, int WN, int TERMS, int EPI>
__global__ __launch_bounds__(512, (BM * BN >= 256 * 256 ? 2 : 4)) void gemm_x3_kernel(
    const float* __restrict__ A, const __bf16* __restrict__ Whi, const __bf16* __restrict__ Wlo,
    const float* __restrict__ bias, const float* __restrict__ R, float* __restrict__ C, int M,
    int N, int K, int lda, int ldw, int ldc) {
  constexpr int NA = TERMS == 3 ? 2 : 1;      // A planes (hi[, lo])
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
  constexpr int NB = TERMS == 3 ? 2 : 1;      // W planes
  constexpr int STAGE_B = NA * A_BYTES + NB * B_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * STAGE_B];

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, lh = lane >> 5;

  // ---- global staging map
  // A: BM rows x 32 f32 = BM*8 float4; thread covers float4 (row = q/8, c4 = q%8), q = tid + 512*i
  constexpr int A_F4 = BM * 8 / 512;
  // W: BN rows x 64 B per plane = BN*4 16-byte chunks per plane
  constexpr int W_C16 = BN * 4 / 512;
  static_assert(A_F4 >= 1 && W_C16 >= 1, "tile too small for 512 threads");
  const float* a_src[A_F4];
  int a_row[A_F4];
#pragma unroll
  for (int i = 0; i < A_F4; ++i) {
    const int q = tid + 512 * i;
    a_row[i] = q >> 3;
    int r = m0 + a_row[i];
    r = r < M ? r : M - 1;
    a_src[i] = A + (size_t)r * lda + (q & 7) * 4;
  }
  const __bf16* w_src[W_C16];
  const __bf16* w_lo_src[W_C16];
  int w_row[W_C16];
#pragma unroll
  for (int i = 0; i < W_C16; ++i) {
    const int q = tid + 512 * i;
    w_row[i] = q >> 2;
    int r = n0 + w_row[i];
    r = r < N ? r : N - 1;
    w_src[i] = Whi + (size_t)r * ldw + (q & 3) * 8;
    w_lo_src[i] = TERMS == 3 ? Wlo + (size_t)r * ldw + (q & 3) * 8 : nullptr;
  }

  floatx4 ra[A_F4];
  bf16x8 rwh[W_C16], rwl[W_C16];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) ra[i] = *reinterpret_cast<const floatx4*>(a_src[i] + k0);
#pragma unroll
    for (int i = 0; i < W_C16; ++i) {
      rwh[i] = *reinterpret_cast<const bf16x8*>(w_src[i] + k0);
      if (TERMS == 3) rwl[i] = *reinterpret_cast<const bf16x8*>(w_lo_src[i] + k0);
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* st = lds + buf * STAGE_B;
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int q = tid + 512 * i;
      const int row = a_row[i], c4 = q & 7;  // 4 floats -> 8 bytes per plane
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = ra[i][e];
        const __bf16 h = (__bf16)v;
        hi[e] = h;
        if (TERMS == 3) lo[e] = (__bf16)(v - (float)h);
      }
      const int chunk = c4 >> 1, half = c4 & 1;
      const int off = row * ROWB + swz(row, chunk) * 16 + half * 8;
      *reinterpret_cast<bf16x4*>(st + off) = hi;
      if (TERMS == 3) *reinterpret_cast<bf16x4*>(st + A_BYTES + off) = lo;
    }
    unsigned char* sb = st + NA * A_BYTES;
#pragma unroll
    for (int i = 0; i < W_C16; ++i) {
      const int q = tid + 512 * i;
      const int row = w_row[i], chunk = q & 3;
      const int off = row * ROWB + swz(row, chunk) * 16;
      *reinterpret_cast<bf16x8*>(sb + off) = rwh[i];
      if (TERMS == 3) *reinterpret_cast<bf16x8*>(sb + B_BYTES + off) = rwl[i];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  gload(0);
  lstore(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const unsigned char* st = lds + cur * STAGE_B;
    const unsigned char* sb = st + NA * A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = 2 * s + lh;  // k = 16s + 8h .. +8
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = wm * (BM / WM) + a * 32 + li;
        const int off = row * ROWB + swz(row, chunk) * 16;
        ah[a] = *reinterpret_cast<const bf16x8*>(st + off);
        if (TERMS == 3) al[a] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + off);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int row = wn * (BN / WN) + b * 32 + li;
        const int off = row * ROWB + swz(row, chunk) * 16;
        bh[b] = *reinterpret_cast<const bf16x8*>(sb + off);
        if (TERMS == 3) bl[b] = *reinterpret_cast<const bf16x8*>(sb + B_BYTES + off);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          if (TERMS == 3) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          }
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * (BN / WN) + b * 32 + li;
      if (col >= N) continue;
      const float bv = bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / WM) + a * 32 + mfma32_row(r, lh);
        if (row < M) {
          float v = acc[a][b][r] + bv;
          if (EPI == X3_EPI_GELU) v = gelu_erf(v);
          if (EPI == X3_EPI_TANH) v = tanhf(v);
          if (EPI == X3_EPI_RES) v += R[(size_t)row * ldc + col];
          C[(size_t)row * ldc + col] = v;
        }
      }
    }
  }
}

namespace {
template <int BM, int BN, int WM, int WN, int TERMS>
hipError_t launch_cfg(const float* A, const __bf16* Whi, const __bf16* Wlo, const float* bias,
                      const float* R, float* C, int M, int N, int K, int lda, int ldw, int ldc,
                      int epi, hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  dim3 grid(tiles), block(512);
#define X3_LAUNCH(E)                                                                         \
  hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, TERMS, E>), grid, block, 0, st, A, Whi, \
                     Wlo, bias, R, C, M, N, K, lda, ldw, ldc)
  switch (epi) {
    case X3_EPI_BIAS: X3_LAUNCH(X3_EPI_BIAS); break;
    case X3_EPI_GELU: X3_LAUNCH(X3_EPI_GELU); break;
    case X3_EPI_RES: X3_LAUNCH(X3_EPI_RES); break;
    default: X3_LAUNCH(X3_EPI_TANH);
  }
#undef X3_LAUNCH
  return hipGetLastError();
}
}  // namespace

// terms: 3 = split-bf16 (f32-class), 1 = plain bf16.  Tile shape chosen per problem so the grid
// has >= ~1.5 waves of workgroups over 256 CUs.
extern "C" hipError_t ae_launch_gemm_x3(const float* A, const unsigned short* Whi,
                                        const unsigned short* Wlo, const float* bias,
                                        const float* R, float* C, int M, int N, int K, int lda,
                                        int ldw, int ldc, int epi, int terms, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (K % BK != 0) return hipErrorInvalidValue;
  const __bf16* wh = reinterpret_cast<const __bf16*>(Whi);
  const __bf16* wl = reinterpret_cast<const __bf16*>(Wlo);
  const long big_tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  // 256x256 (1 workgroup / CU) only when it fills >= 2 full rounds of 256 CUs; otherwise
  // 128x128 (2 workgroups / CU, 4x the tiles).  AE_X3_TILE=128|256 forces a shape (A/B runs).
  static const int force = [] {
    const char* v = std::getenv("AE_X3_TILE");
    return v ? std::atoi(v) : 0;
  }();
  const bool big = force ? force == 256 : big_tiles >= 512;
  if (terms == 3) {
    if (big)
      return launch_cfg<256, 256, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
    return launch_cfg<128, 128, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
  }
  if (big)
    return launch_cfg<256, 256, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
  return launch_cfg<128, 128, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
}

// =================================================================================================
// gemm_x3g: the same split-bf16 GEMM fed by LDS-DMA (global_load_lds_dwordx4) through a 4-stage
// LDS ring, so three K-steps of loads are in flight while one is computed (the register-staged
// kernel above keeps only one and is latency-bound at 256x256 tiles: one workgroup per CU).
//   * tile 256 x 256, 8 waves (2 x 4), wave tile 128 x 64 = 4 x 2 MFMA 32x32 tiles
//   * one stage = BK 16: A as f32 (256 rows x 64 B), W_hi and W_lo as bf16 (256 rows x 32 B)
//   * LDS images are lane-linear (LDS-DMA writes base + 16*lane); bank-conflict freedom for the
//     ds_read_b128 fragment reads comes from XOR-swizzling the 16-B chunk on the SOURCE address and
//     applying the same involution on the read (cdna_hip_programming.md rule 21)
//   * A is split into hi/lo bf16 in registers right after its fragment read
//   * raw s_barrier + counted s_waitcnt vmcnt(N) (never __syncthreads inside the loop, which would
//     drain the DMA), all LDS in one dynamic array (no second __shared__ object)
namespace {
constexpr int G_BM = 256, G_BN = 256, G_BK = 16, G_NST = 4;
constexpr int G_A_BYTES = G_BM * 64, G_W_BYTES = G_BN * 32;

template <int TERMS>
constexpr int g_stage_bytes() { return G_A_BYTES + (TERMS == 3 ? 2 : 1) * G_W_BYTES; }
template <int TERMS>
constexpr int g_vm_per_stage() { return TERMS == 3 ? 4 : 3; }

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, lds_dst, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
}  // namespace

template <int TERMS, int EPI>
__global__ __launch_bounds__(512, 2) void gemm_x3g_kernel(
    const float* __restrict__ A, const __bf16* __restrict__ Whi, const __bf16* __restrict__ Wlo,
    const float* __restrict__ bias, const float* __restrict__ R, float* __restrict__ C, int M,
    int N, int K, int lda, int ldw, int ldc) {
  extern __shared__ __attribute__((aligned(16))) unsigned char glds_smem[];
  constexpr int SB = g_stage_bytes<TERMS>();
  constexpr int VPS = g_vm_per_stage<TERMS>();
  constexpr int TM = 4, TN = 2;

  const int tiles_n = (N + G_BN - 1) / G_BN;
  const int tiles_m = (M + G_BM - 1) / G_BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * G_BM, n0 = tn * G_BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int li = lane & 31, lh = lane >> 5;

  // ---- this wave's DMA sources (per lane) for one stage, k offset added per stage
  // A instrs 2w, 2w+1: rows 16j + lane/4, LDS chunk lane%4 <- source chunk ^ ((row>>2)&3)
  const float* a_src[2];
  int a_dst[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = 2 * wave + u;
    const int r = 16 * j + (lane >> 2);
    const int cl = lane & 3;
    const int cs = cl ^ ((r >> 2) & 3);
    int gr = m0 + r;
    gr = gr < M ? gr : M - 1;
    a_src[u] = A + (size_t)gr * lda + 4 * cs;
    a_dst[u] = j * 1024;
  }
  // W instr w: rows 32w + lane/2, LDS chunk lane%2 <- source chunk ^ ((row>>3)&1)
  const __bf16* wh_src;
  const __bf16* wl_src = nullptr;
  {
    const int r = 32 * wave + (lane >> 1);
    const int cl = lane & 1;
    const int cs = cl ^ ((r >> 3) & 1);
    int gr = n0 + r;
    gr = gr < N ? gr : N - 1;
    wh_src = Whi + (size_t)gr * ldw + 8 * cs;
    if (TERMS == 3) wl_src = Wlo + (size_t)gr * ldw + 8 * cs;
  }
  const int w_dst = wave * 1024;

  auto issue = [&](int kt) {
    unsigned char* st = glds_smem + (kt % G_NST) * SB;
    const int k0 = kt * G_BK;
    glds16(a_src[0] + k0, st + a_dst[0]);
    glds16(a_src[1] + k0, st + a_dst[1]);
    glds16(wh_src + k0, st + G_A_BYTES + w_dst);
    if (TERMS == 3) glds16(wl_src + k0, st + G_A_BYTES + G_W_BYTES + w_dst);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / G_BK;
  for (int s = 0; s < G_NST - 1 && s < nk; ++s) issue(s);

  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;  // stages issued after kt (capped at NST-2)
    if (ahead >= 2) wait_vm<2 * VPS>();
    else if (ahead == 1) wait_vm<VPS>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + G_NST - 1 < nk) issue(kt + G_NST - 1);

    const unsigned char* st = glds_smem + (kt % G_NST) * SB;
    // W fragments (hi, lo) for this wave's TN tiles: row, chunk lh ^ ((row>>3)&1)
    bf16x8 bh[TN], bl[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int row = wn * 64 + b * 32 + li;
      const int off = row * 32 + 16 * (lh ^ ((row >> 3) & 1));
      bh[b] = *reinterpret_cast<const bf16x8*>(st + G_A_BYTES + off);
      if (TERMS == 3) bl[b] = *reinterpret_cast<const bf16x8*>(st + G_A_BYTES + G_W_BYTES + off);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int row = wm * 128 + a * 32 + li;
      const int sw = (row >> 2) & 3;
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(st + row * 64 + 16 * ((2 * lh) ^ sw));
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(st + row * 64 + 16 * ((2 * lh + 1) ^ sw));
      bf16x8 ah, al;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[e] = h0;
        ah[4 + e] = h1;
        if (TERMS == 3) {
          al[e] = (__bf16)(x0[e] - (float)h0);
          al[4 + e] = (__bf16)(x1[e] - (float)h1);
        }
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        if (TERMS == 3) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[b], acc[a][b], 0, 0, 0);
        }
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[b], acc[a][b], 0, 0, 0);
      }
    }
  }

#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * 64 + b * 32 + li;
      if (col >= N) continue;
      const float bv = bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 128 + a * 32 + mfma32_row(r, lh);
        if (row < M) {
          float v = acc[a][b][r] + bv;
          if (EPI == X3_EPI_GELU) v = gelu_erf(v);
          if (EPI == X3_EPI_TANH) v = tanhf(v);
          if (EPI == X3_EPI_RES) v += R[(size_t)row * ldc + col];
          C[(size_t)row * ldc + col] = v;
        }
      }
    }
  }
}

namespace {
template <int TERMS, int EPI>
hipError_t launch_g(const float* A, const __bf16* Whi, const __bf16* Wlo, const float* bias,
                    const float* R, float* C, int M, int N, int K, int lda, int ldw, int ldc,
                    hipStream_t st) {
  const int lds = G_NST * g_stage_bytes<TERMS>();
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_x3g_kernel<TERMS, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int tiles = ((M + G_BM - 1) / G_BM) * ((N + G_BN - 1) / G_BN);
  hipLaunchKernelGGL((gemm_x3g_kernel<TERMS, EPI>), dim3(tiles), dim3(512), lds, st, A, Whi, Wlo,
                     bias, R, C, M, N, K, lda, ldw, ldc);
  return hipGetLastError();
}

template <int TERMS>
hipError_t launch_g_epi(const float* A, const __bf16* Whi, const __bf16* Wlo, const float* bias,
                        const float* R, float* C, int M, int N, int K, int lda, int ldw, int ldc,
                        int epi, hipStream_t st) {
  switch (epi) {
    case X3_EPI_BIAS: return launch_g<TERMS, X3_EPI_BIAS>(A, Whi, Wlo, bias, R, C, M, N, K, lda, ldw, ldc, st);
    case X3_EPI_GELU: return launch_g<TERMS, X3_EPI_GELU>(A, Whi, Wlo, bias, R, C, M, N, K, lda, ldw, ldc, st);
    case X3_EPI_RES: return launch_g<TERMS, X3_EPI_RES>(A, Whi, Wlo, bias, R, C, M, N, K, lda, ldw, ldc, st);
    default: return launch_g<TERMS, X3_EPI_TANH>(A, Whi, Wlo, bias, R, C, M, N, K, lda, ldw, ldc, st);
  }
}
}  // namespace

// LDS-DMA pipelined variant; requires K % 16 == 0.  kernel_variant: 0 = register-staged (above),
// 1 = LDS-DMA ring.
extern "C" hipError_t ae_launch_gemm_x3g(const float* A, const unsigned short* Whi,
                                         const unsigned short* Wlo, const float* bias,
                                         const float* R, float* C, int M, int N, int K, int lda,
                                         int ldw, int ldc, int epi, int terms, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (K % G_BK != 0) return hipErrorInvalidValue;
  const __bf16* wh = reinterpret_cast<const __bf16*>(Whi);
  const __bf16* wl = reinterpret_cast<const __bf16*>(Wlo);
  if (terms == 3) return launch_g_epi<3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
  return launch_g_epi<1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
}
