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
  // 128x128 (2 workgroups / CU, 4x the tiles)
  const bool big = big_tiles >= 512;
  if (terms == 3) {
    if (big)
      return launch_cfg<256, 256, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
    return launch_cfg<128, 128, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
  }
  if (big)
    return launch_cfg<256, 256, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
  return launch_cfg<128, 128, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st);
}
