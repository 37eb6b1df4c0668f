// gemm_f32.hip — exact-f32 MFMA GEMM with fused epilogues for the RoBERTa encoder (parity mode).
//
// C[M,N] = A[M,K] · W[N,K]^T + bias[N]  (+ GELU | + residual R[M,N] | tanh)
// This is every nn.Linear of the encoder the reference reaches through
// RobertaForSequenceClassification (CodeXGLUE/Defect-detection/code/model.py:25): QKV, attention
// output, intermediate (GELU) and output projections.  W keeps the HF nn.Linear layout
// [out_features, in_features], so both operands are K-contiguous.
//
// gfx950 mapping: v_mfma_f32_32x32x2_f32 (one f32 per lane per operand, exact fmaf chain,
// 64 FLOP/clk/SIMD = 157 TF/s chip).  Workgroup tile 128x128x32, 4 waves (2x2), 64x64 per wave
// = 2x2 MFMA tiles.  Operands are staged global->VGPR->LDS with the next K-tile's loads issued
// before the current tile's MFMAs (T14 split) and one barrier per K-tile.  LDS rows are padded to
// 36 floats (144 B) so the ds_read_b128 fragment reads of 16 different rows are conflict-free.
// Within a 32-deep K-tile, lane half h owns k in [16h, 16h+16): a lane reads 16 contiguous floats
// (4 x ds_read_b128) and MFMA step (c,e) pairs k = 4c+e (h=0) with k = 16+4c+e (h=1).
#include "common.h"

namespace {
constexpr int BM = 128, BN = 128, BK = 32, LDS_STRIDE = 36;
}

enum { EPI_BIAS = 0, EPI_BIAS_GELU = 1, EPI_BIAS_RESIDUAL = 2, EPI_BIAS_TANH = 3 };

// Segmented split-K as in gemm_x3.hip: the K range is cut into `segs` segments (a function of K
// alone); unsplit, one workgroup adds each segment's accumulator into a running total; split
// (part != nullptr), workgroup (tile, s) writes segment s to part[s][M][N] for
// ae_launch_splitk_reduce — the same sums in the same order, so scores stay batch-invariant.
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f32_nt_kernel(
    const float* __restrict__ A, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ R, float* __restrict__ C, int M, int N, int K, int lda, int ldw,
    int ldc, const int* __restrict__ row_map, int segs, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDS_STRIDE];

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int nsplit = part ? segs : 1;
  const int t_all = xcd_remap(blockIdx.x, nwg * nsplit);
  const int t = t_all / nsplit, sp = t_all % nsplit;
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;

  // global staging: 4 float4 of A and 4 of W per thread per K-tile
  const int ld_chunk = tid & 7;   // 8 float4 chunks per 32-float row
  const int ld_row = tid >> 3;    // rows ld_row + 32*i
  const float* a_src[4];
  const float* w_src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = m0 + ld_row + 32 * i;
    r = r < M ? r : M - 1;
    if (row_map) r = row_map[r];
    a_src[i] = A + (size_t)r * lda + ld_chunk * 4;
    int wr = n0 + ld_row + 32 * i;
    wr = wr < N ? wr : N - 1;
    w_src[i] = W + (size_t)wr * ldw + ld_chunk * 4;
  }
  floatx4 ra[4], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const floatx4*>(a_src[i] + k0);
      rw[i] = *reinterpret_cast<const floatx4*>(w_src[i] + k0);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (ld_row + 32 * i) * LDS_STRIDE + ld_chunk * 4;
      *reinterpret_cast<floatx4*>(&As[buf][off]) = ra[i];
      *reinterpret_cast<floatx4*>(&Bs[buf][off]) = rw[i];
    }
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk_all = K / BK;
  const int kb = part ? sp * nk_all / segs : 0;
  const int ke = part ? (sp + 1) * nk_all / segs : nk_all;
  floatx16 tot[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) tot[a][b][r] = 0.f;
  int seg = 0, seg_end = part ? ke : nk_all / segs;
  gload(kb * BK);
  lstore(0);
  __syncthreads();

  for (int kt = kb; kt < ke; ++kt) {
    const int cur = (kt - kb) & 1;
    if (kt + 1 < ke) gload((kt + 1) * BK);
    const float* as = &As[cur][(wm * 64 + li) * LDS_STRIDE + 16 * lh];
    const float* bs = &Bs[cur][(wn * 64 + li) * LDS_STRIDE + 16 * lh];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const floatx4 a0 = *reinterpret_cast<const floatx4*>(as + 4 * c);
      const floatx4 a1 = *reinterpret_cast<const floatx4*>(as + 32 * LDS_STRIDE + 4 * c);
      const floatx4 b0 = *reinterpret_cast<const floatx4*>(bs + 4 * c);
      const floatx4 b1 = *reinterpret_cast<const floatx4*>(bs + 32 * LDS_STRIDE + 4 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b0[e], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b1[e], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b0[e], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b1[e], acc[1][1], 0, 0, 0);
      }
    }
    if (!part && kt + 1 == seg_end) {  // close a segment: total += its accumulator
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
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

  // epilogue
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = n0 + wn * 64 + b * 32 + li;
      if (col >= N) continue;
      if (part) {  // raw segment accumulator; the reduce adds bias + epilogue
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + a * 32 + mfma32_row(r, lh);
          if (row < M) part[((size_t)sp * M + row) * N + col] = acc[a][b][r];
        }
        continue;
      }
      const float bv = bias ? bias[col] : 0.f;  // null bias: same rule as splitk_reduce
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + a * 32 + mfma32_row(r, lh);
        if (row < M) {
          float v = tot[a][b][r] + bv;
          if (EPI == EPI_BIAS_GELU) v = gelu_erf(v);
          if (EPI == EPI_BIAS_TANH) v = tanhf(v);
          if (EPI == EPI_BIAS_RESIDUAL) v += R[(size_t)row * ldc + col];
          C[(size_t)row * ldc + col] = v;
        }
      }
    }
  }
}

extern "C" hipError_t ae_launch_splitk_reduce(const float* part, int segs, int M, int N,
                                              const float* bias, const float* R, float* C, int ldc,
                                              int epi, hipStream_t st);

// K segments of this kernel (a function of K alone, ~3 K-tiles each, at most 8)
extern "C" int ae_splitk_segments_f32(int K) {
  const int s = (K / BK) / 3;
  return s < 1 ? 1 : (s > 8 ? 8 : s);
}

// Host launcher.  row_map (device, optional) gathers A rows: A row r of the product is
// A[row_map[r]] (used to run the last layer on CLS rows only).  A grid of fewer than 128 tiles
// takes the split-K form when ws (ws_floats f32) holds the segment partials.
extern "C" hipError_t ae_launch_gemm_f32(const float* A, const float* W, const float* bias,
                                         const float* R, float* C, int M, int N, int K, int lda,
                                         int ldw, int ldc, int epi, const int* row_map,
                                         hipStream_t stream, float* ws, long ws_floats) {
  if (M <= 0) return hipSuccess;
  if (K % BK != 0) return hipErrorInvalidValue;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int segs = ae_splitk_segments_f32(K);
  float* part = (segs > 1 && tiles < 128 && N % 4 == 0 && (long)segs * M * N <= ws_floats)
                    ? ws : nullptr;
  dim3 grid(tiles * (part ? segs : 1)), block(256);
  switch (epi) {
    case EPI_BIAS:
      hipLaunchKernelGGL(gemm_f32_nt_kernel<EPI_BIAS>, grid, block, 0, stream, A, W, bias, R, C, M,
                         N, K, lda, ldw, ldc, row_map, segs, part);
      break;
    case EPI_BIAS_GELU:
      hipLaunchKernelGGL(gemm_f32_nt_kernel<EPI_BIAS_GELU>, grid, block, 0, stream, A, W, bias, R,
                         C, M, N, K, lda, ldw, ldc, row_map, segs, part);
      break;
    case EPI_BIAS_TANH:
      hipLaunchKernelGGL(gemm_f32_nt_kernel<EPI_BIAS_TANH>, grid, block, 0, stream, A, W, bias, R,
                         C, M, N, K, lda, ldw, ldc, row_map, segs, part);
      break;
    default:
      hipLaunchKernelGGL(gemm_f32_nt_kernel<EPI_BIAS_RESIDUAL>, grid, block, 0, stream, A, W, bias,
                         R, C, M, N, K, lda, ldw, ldc, row_map, segs, part);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !part) return e;
  return ae_launch_splitk_reduce(part, segs, M, N, bias, R, C, ldc, epi, stream);
}
