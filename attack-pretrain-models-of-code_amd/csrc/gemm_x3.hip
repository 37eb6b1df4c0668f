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

// Split-K without losing batch invariance (SEG = true, the 128 x 128 configuration): the K range
// is cut into `segs` segments that depend on K only (splitk_segments); every output is
// acc(seg 0) + acc(seg 1) + ... summed in segment order.  Unsplit (part == nullptr) one workgroup
// walks all segments, adding each segment's accumulator into a running total; split, workgroup
// (tile, s) computes segment s alone into part[s][M][N] and splitk_reduce_kernel adds them in
// the same order — bit-identical, so a row's score does not depend on how many rows share the
// launch (small launches such as the last layer's CLS rows take the split form to fill the chip).
template <int BM, int BN, int WM, int WN, int TERMS, int EPI>
__global__ __launch_bounds__(512, (BM * BN >= 256 * 256 ? 2 : 4)) void gemm_x3_kernel(
    const float* __restrict__ A, const __bf16* __restrict__ Whi, const __bf16* __restrict__ Wlo,
    const float* __restrict__ bias, const float* __restrict__ R, float* __restrict__ C, int M,
    int N, int K, int lda, int ldw, int ldc, int segs, float* __restrict__ part) {
  constexpr bool SEG = BM * BN < 256 * 256;
  constexpr int NA = TERMS == 3 ? 2 : 1;      // A planes (hi[, lo])
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
  constexpr int NB = TERMS == 3 ? 2 : 1;      // W planes
  constexpr int STAGE_B = NA * A_BYTES + NB * B_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * STAGE_B];

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nsplit = part ? segs : 1;
  const int t_all = xcd_remap(blockIdx.x, tiles_m * tiles_n * nsplit);
  const int t = t_all / nsplit, sp = t_all % nsplit;
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

  // K-tiles [kb, ke): the whole K, or segment sp of a split launch
  const int nk_all = K / BK;
  const int kb = part ? sp * nk_all / segs : 0;
  const int ke = part ? (sp + 1) * nk_all / segs : nk_all;
  floatx16 tot[SEG ? TM : 1][SEG ? TN : 1];
  if (SEG) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) tot[a][b][r] = 0.f;
  }
  int seg = 0, seg_end = (SEG && !part) ? nk_all / segs : ke;
  gload(kb * BK);
  lstore(0);
  __syncthreads();

  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) & 1;
    if (kt + 1 < ke) gload((kt + 1) * BK);
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
    if (SEG && !part && kt + 1 == seg_end) {  // close a segment: total += its accumulator
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          tot[a][b] += acc[a][b];
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
        }
      ++seg;
      seg_end = (seg + 1) * nk_all / segs;
    }
    if (kt + 1 < ke) lstore(cur ^ 1);
    __syncthreads();
  }
  if (SEG && !part) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] = tot[a][b];
  }

#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * (BN / WN) + b * 32 + li;
      if (col >= N) continue;
      if (part) {  // raw segment accumulator; splitk_reduce_kernel adds bias + epilogue
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * (BM / WM) + a * 32 + mfma32_row(r, lh);
          if (row < M) part[((size_t)sp * M + row) * N + col] = acc[a][b][r];
        }
        continue;
      }
      const float bv = bias ? bias[col] : 0.f;  // null bias: same rule as splitk_reduce
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / WM) + a * 32 + mfma32_row(r, lh);
        if (row < M) {
          float v = (0.f + acc[a][b][r]) + bv;
          if (EPI == X3_EPI_GELU) v = gelu_erf(v);
          if (EPI == X3_EPI_TANH) v = tanhf(v);
          if (EPI == X3_EPI_RES) v += R[(size_t)row * ldc + col];
          C[(size_t)row * ldc + col] = v;
        }
      }
    }
  }
}

// part[s][M][N] (s < segs) -> C = epilogue(Σ_s part[s] + bias), summed in segment order
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part,
                                                            int segs, int M, int N,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ R,
                                                            float* __restrict__ C, int ldc,
                                                            int epi) {
  const int n4 = N >> 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)M * n4) return;
  const int row = (int)(i / n4), c = (int)(i % n4) * 4;
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  for (int sg = 0; sg < segs; ++sg)
    v += *reinterpret_cast<const floatx4*>(part + ((size_t)sg * M + row) * N + c);
  if (bias) v += *reinterpret_cast<const floatx4*>(bias + c);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (epi == X3_EPI_GELU) v[e] = gelu_erf(v[e]);
    if (epi == X3_EPI_TANH) v[e] = tanhf(v[e]);
  }
  if (epi == X3_EPI_RES) v += *reinterpret_cast<const floatx4*>(R + (size_t)row * ldc + c);
  *reinterpret_cast<floatx4*>(C + (size_t)row * ldc + c) = v;
}

// K segments of the split-K scheme: a function of K alone (batch invariance), ~6 K-tiles each
extern "C" int ae_splitk_segments(int K) {
  const int nk = K / BK;
  const int s = nk / 6;
  return s < 1 ? 1 : (s > 8 ? 8 : s);
}

// split when the tile grid covers less than half the CUs and the workspace holds the partials
extern "C" int ae_splitk_use(int tiles, int M, int N, int K, long ws_floats) {
  const int segs = ae_splitk_segments(K);
  return segs > 1 && tiles < 128 && (N % 4) == 0 && (long)segs * M * N <= ws_floats;
}

extern "C" hipError_t ae_launch_splitk_reduce(const float* part, int segs, int M, int N,
                                              const float* bias, const float* R, float* C, int ldc,
                                              int epi, hipStream_t st) {
  const long n = (long)M * (N / 4);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     part, segs, M, N, bias, R, C, ldc, epi);
  return hipGetLastError();
}

namespace {
template <int BM, int BN, int WM, int WN, int TERMS>
hipError_t launch_cfg(const float* A, const __bf16* Whi, const __bf16* Wlo, const float* bias,
                      const float* R, float* C, int M, int N, int K, int lda, int ldw, int ldc,
                      int epi, hipStream_t st, float* ws, long ws_floats) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  constexpr bool SEG = BM * BN < 256 * 256;
  const int segs = SEG ? ae_splitk_segments(K) : 1;
  float* part = (SEG && ae_splitk_use(tiles, M, N, K, ws_floats)) ? ws : nullptr;
  dim3 grid(tiles * (part ? segs : 1)), block(512);
#define X3_LAUNCH(E)                                                                         \
  hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, TERMS, E>), grid, block, 0, st, A, Whi, \
                     Wlo, bias, R, C, M, N, K, lda, ldw, ldc, segs, part)
  switch (epi) {
    case X3_EPI_BIAS: X3_LAUNCH(X3_EPI_BIAS); break;
    case X3_EPI_GELU: X3_LAUNCH(X3_EPI_GELU); break;
    case X3_EPI_RES: X3_LAUNCH(X3_EPI_RES); break;
    default: X3_LAUNCH(X3_EPI_TANH);
  }
#undef X3_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !part) return e;
  return ae_launch_splitk_reduce(part, segs, M, N, bias, R, C, ldc, epi, st);
}
}  // namespace

// terms: 3 = split-bf16 (f32-class), 1 = plain bf16.  Tile shape chosen per problem so the grid
// has >= ~1.5 waves of workgroups over 256 CUs; small grids take the split-K form when the
// caller's workspace ws (ws_floats f32) holds the partials (see gemm_x3_kernel).
extern "C" hipError_t ae_launch_gemm_x3(const float* A, const unsigned short* Whi,
                                        const unsigned short* Wlo, const float* bias,
                                        const float* R, float* C, int M, int N, int K, int lda,
                                        int ldw, int ldc, int epi, int terms, hipStream_t st,
                                        float* ws, long ws_floats) {
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
      return launch_cfg<256, 256, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st,
                                           nullptr, 0);
    return launch_cfg<128, 128, 2, 4, 3>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st,
                                         ws, ws_floats);
  }
  if (big)
    return launch_cfg<256, 256, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st,
                                         nullptr, 0);
  return launch_cfg<128, 128, 2, 4, 1>(A, wh, wl, bias, R, C, M, N, K, lda, ldw, ldc, epi, st, ws,
                                       ws_floats);
}
