// gemm_w2.hip — packed bf16-plane GEMM with TWO workgroups per CU, so that one workgroup's
// epilogue (bias / GELU / plane split / stores: MFMA-idle VALU and memory work) runs while the
// other workgroup on the same CU keeps the matrix cores busy.
//
// Same product and operand layout as gemm_planes.hip (packed planes: per 32 k of a row a 128-B
// block [hi 32 | lo 32]; NP = 2: 3 bf16 MFMAs per product, NP = 1: hi only).  Mapping:
//   * tile 128 (M) x 256 (N), 4 waves (256 threads), one per SIMD; wave w owns all 128 rows and
//     columns 64 w .. 64 w + 63 (acc[4][2] of 32 x 32, 128 registers) — the ping-pong kernel's
//     wave tile, so its epilogue is reused;
//   * K-tile = 16 k: a row's K-tile is two 32-B pieces (hi 16 | lo 16 of one half of a 128-B
//     block), 64 B per row in LDS; a stage holds A (128 rows, 8 KiB) + W (256 rows, 16 KiB);
//     3 stages = 72 KiB per workgroup, 2 workgroups = 144 KiB of the 160 KiB LDS;
//   * the 16-B chunk c of LDS row r holds logical chunk c ^ ((r >> 2) & 3) (chunks 0-1 hi,
//     2-3 lo): the ds_read_b128 fragment reads of 16 rows hit 16 different bank slots;
//   * operands reach LDS by LDS-DMA (global_load_lds_dwordx4, 16 rows x 64 B per wave
//     instruction, 6 per wave per K-tile), tile kt+3 issued right after the barrier that ends
//     every wave's reads of tile kt (its stage), spread between the MFMAs; one s_barrier per
//     K-tile (4 waves), counted vmcnt; the fragments of tile kt+1 are read into a second
//     register buffer while tile kt's MFMAs run;
//   * XCD-aware grouped tile order as the other packed GEMMs.
// No intra-workgroup staggering: the two co-resident workgroups interleave on every SIMD.
#include <type_traits>

#include "common.h"

#pragma clang diagnostic ignored "-Winline-asm"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {
// PK_EPI_* of gemm_planes.hip
enum { W2_EPI_BIAS = 0, W2_EPI_GELU_PACKED = 1, W2_EPI_RES = 2, W2_EPI_TANH = 3, W2_EPI_BIAS_PACKED = 4 };
constexpr int W2_BM = 128, W2_BN = 256, W2_ROWB = 64;  // LDS bytes per row per K-tile
constexpr int W2_A_BYTES = W2_BM * W2_ROWB, W2_STAGE = (W2_BM + W2_BN) * W2_ROWB;  // 24 KiB
constexpr int W2_NST = 3;
constexpr int W2_LDS = W2_NST * W2_STAGE;  // 72 KiB (the epilogue's 4 x 16 KiB fit inside)

__device__ __forceinline__ void w2_dma16(const void* gsrc, uint32_t lds_base) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(gsrc), "s"(lds_base)
      : "memory", "m0");
}
}  // namespace

template <int NP, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_w2_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ R, float* __restrict__ C, __bf16* __restrict__ Cp, int M, int N,
    int K, int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char w2_smem[];
  constexpr int T = NP == 2 ? 3 : 1;

  const int tiles_n = (N + W2_BN - 1) / W2_BN;
  const int tiles_m = (M + W2_BM - 1) / W2_BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int per_group = group_m * tiles_n;
  const int g = t / per_group, first_m = g * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm0 = first_m + (t - g * per_group) % gsize, tn0 = (t - g * per_group) / gsize;
  const int m0 = tm0 * W2_BM, n0 = tn0 * W2_BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const size_t lda = (size_t)NP * K;  // packed row length (elements)
  const int nk = K / 16;              // K-tiles of 16 k

  // ---- DMA: per K-tile 24 pieces of 16 rows x 64 B (A rows 0..127 = pieces 0..7, W rows
  // 0..255 = pieces 8..23); wave w issues pieces 6 w .. 6 w + 5.  Lane i of a piece writes LDS
  // bytes 16 i: row i / 4, physical chunk i % 4, holding logical chunk (i % 4) ^ ((row >> 2) & 3)
  // whose source is: hi 0..7 / 8..15 of the K-tile's half of its 128-B block, or lo (+64 B).
  const char* src[6];
  uint32_t dst[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int piece = 6 * wave + j;
    const bool is_a = piece < 8;
    const int r0 = (is_a ? piece : piece - 8) * 16;  // the piece's first row (wave-uniform)
    const int r = r0 + (lane >> 2);                   // this lane's row within A or W
    const int lc = (lane & 3) ^ ((r >> 2) & 3);                   // logical chunk
    const int boff = (lc >> 1) * 64 * (NP == 2 ? 1 : 0) + (lc & 1) * 16;  // within the half
    if (is_a) {
      const int gr = m0 + r < M ? m0 + r : M - 1;
      src[j] = reinterpret_cast<const char*>(A + gr * lda) + boff;
      dst[j] = r0 * W2_ROWB;
    } else {
      const int gr = n0 + r < N ? n0 + r : N - 1;
      src[j] = reinterpret_cast<const char*>(W + gr * lda) + boff;
      dst[j] = W2_A_BYTES + r0 * W2_ROWB;
    }
  }
  // byte offset of K-tile kt inside a packed row: NP = 2: block kt / 2 (128 B), half kt % 2 (32 B);
  // NP = 1: 32 B per K-tile (16 bf16 of hi)
  auto ktoff = [&](int kt) -> size_t {
    return NP == 2 ? (size_t)(kt >> 1) * 128 + (kt & 1) * 32 : (size_t)kt * 32;
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)w2_smem;
  auto dma_piece = [&](int j, int kt) {
    w2_dma16(src[j] + ktoff(kt), lds0 + (kt % W2_NST) * W2_STAGE + dst[j]);
  };

  floatx16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // fragment rows: 32-aligned + li, so the row swizzle is (li >> 2) & 3
  const int sw = (li >> 2) & 3;
  const int a_row = li * W2_ROWB;
  const int w_row = W2_A_BYTES + (wave * 64 + li) * W2_ROWB;

  // Software-pipelined: the fragments of K-tile kt+1 are read (into the other register buffer)
  // while the MFMAs of K-tile kt run, so the LDS read latency hides behind the matrix core even
  // when the two workgroups of a CU run in step.  3-stage ring: tiles kt+1, kt+2 resident or in
  // flight, tile kt+3 loading into kt's stage (its fragments already in registers).
  bf16x8 fa[2][4][NP], fw[2][2][NP];
  auto read_frags = [&](auto bufc, int kt) {
    constexpr int B = decltype(bufc)::value;
    const unsigned char* st = w2_smem + (kt % W2_NST) * W2_STAGE;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int coff = 16 * ((2 * p + lh) ^ sw);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        fw[B][b][p] = *reinterpret_cast<const bf16x8*>(st + w_row + b * 32 * W2_ROWB + coff);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        fa[B][a][p] = *reinterpret_cast<const bf16x8*>(st + a_row + a * 32 * W2_ROWB + coff);
    }
  };
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (k < nk)
#pragma unroll
      for (int j = 0; j < 6; ++j) dma_piece(j, k);
  if (nk > 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (nk > 0) read_frags(std::integral_constant<int, 0>(), 0);

  auto step = [&](auto bufc, int kt) {
    constexpr int B = decltype(bufc)::value;
    const bool more = kt + 1 < nk;
    const bool refill = kt + 3 < nk;
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      // tile kt+1 landed (this wave's pieces), this wave's reads of tile kt done, then every
      // wave's: tile kt's stage is free for tile kt+3, tile kt+1 is readable
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      read_frags(std::integral_constant<int, 1 - B>(), kt + 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8 * T; ++i) {
      const int a = i / (2 * T), b = (i / T) % 2, term = i % T;
      const bf16x8& x = (T == 3 && term == 1) ? fw[B][b][NP - 1] : fw[B][b][0];
      const bf16x8& y = (T == 3 && term == 0) ? fa[B][a][NP - 1] : fa[B][a][0];
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc[a][b], 0, 0, 0);
      // the 6 DMA pieces of tile kt+3 spread over the MFMAs (issue cost hidden in their gaps)
      constexpr int NM = 8 * T;
      if (refill && (i + 1) * 6 / NM > i * 6 / NM) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = i * 6 / NM; j < (i + 1) * 6 / NM; ++j) dma_piece(j, kt + 3);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(std::integral_constant<int, 0>(), kt);
    if (kt + 1 < nk) step(std::integral_constant<int, 1>(), kt + 1);
  }
  __syncthreads();  // every wave's last fragment reads done: the stages become epilogue scratch

  // ---- epilogue (gemm_planes.hip gemm_pp_kernel's, wave tile 128 x 64 at rows 0..127):
  // acc[tm][tn] register 4 j + i of lane l = output row tm*32 + (l & 31), column wave*64 +
  // tn*32 + 8 j + 4 (l >> 5) + i; per 64-row half the wave writes its 64 x 64 block into its
  // own 16-KiB LDS region in the output's byte image (XOR-ed 16-B chunks), then stores whole
  // row segments with 16-B lanes (+ residual / tanh on the coalesced side).
  constexpr bool PACKED = EPI == W2_EPI_GELU_PACKED || EPI == W2_EPI_BIAS_PACKED;
  constexpr int RB = PACKED ? 64 * 2 * NP : 256;
  constexpr int CPR = RB / 16;
  unsigned char* reg = w2_smem + wave * 16384;
  const int cb0 = n0 + wave * 64;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int lr = tt * 32 + li;
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const floatx16& c = acc[2 * half + tt][tn];
          const int cc = tn * 32 + 8 * j + 4 * lh;
          if (PACKED) {
            const int col = cb0 + cc < N ? cb0 + cc : N - 4;
            const floatx4 bv = *reinterpret_cast<const floatx4*>(bias + col);
            ushortx4 h, l;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float y = EPI == W2_EPI_GELU_PACKED ? gelu_erfc_fast(c[4 * j + i] + bv[i])
                                                        : c[4 * j + i] + bv[i];
              const __bf16 hv = (__bf16)y;
              h[i] = __builtin_bit_cast(unsigned short, hv);
              l[i] = f2bf(y - (float)hv);
            }
            const int hb = tn * 64 * NP + 2 * (8 * j + 4 * lh);
            const int ch = ((hb >> 4) ^ (lr & 15)) & (CPR - 1);
            *reinterpret_cast<ushortx4*>(reg + lr * RB + ch * 16 + (hb & 15)) = h;
            if (NP == 2) {
              const int lb = hb + 64;
              const int cl = ((lb >> 4) ^ (lr & 15)) & (CPR - 1);
              *reinterpret_cast<ushortx4*>(reg + lr * RB + cl * 16 + (lb & 15)) = l;
            }
          } else {
            floatx4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = c[4 * j + i];
            const int ch = (cc >> 2) ^ (lr & 15);
            *reinterpret_cast<floatx4*>(reg + lr * RB + ch * 16) = v;
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int RPI = 64 / CPR;
#pragma unroll
    for (int k = 0; k < 64 / RPI; ++k) {
      const int lr = k * RPI + lane / CPR, c = lane % CPR;
      const int row = m0 + half * 64 + lr;
      const bool ok = row < M;
      const uint4 v = *reinterpret_cast<const uint4*>(reg + lr * RB + ((c ^ (lr & 15)) & (CPR - 1)) * 16);
      if (PACKED) {
        const int col = cb0 + (c * 16) / (2 * NP);
        if (ok && col < N) {
          __bf16* dstp = Cp + (size_t)row * NP * N + (size_t)(cb0 >> 5) * 32 * NP + c * 8;
          __builtin_nontemporal_store(__builtin_bit_cast(floatx4, v), reinterpret_cast<floatx4*>(dstp));
        }
      } else {
        const int col = cb0 + 4 * c;
        if (ok && col < N) {
          const size_t o = (size_t)row * N + col;
          floatx4 f = __builtin_bit_cast(floatx4, v);
          if (bias) f += *reinterpret_cast<const floatx4*>(bias + col);
          if (EPI == W2_EPI_TANH)
#pragma unroll
            for (int i = 0; i < 4; ++i) f[i] = tanhf(f[i]);
          if (EPI == W2_EPI_RES) f += *reinterpret_cast<const floatx4*>(R + o);
          *reinterpret_cast<floatx4*>(C + o) = f;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

namespace {
template <int NP, int EPI>
hipError_t w2_launch(const __bf16* A, const __bf16* W, const float* bias, const float* R, float* C,
                     __bf16* Cp, int M, int N, int K, int group_m, hipStream_t st) {
  if (hipError_t e = ensure_dynamic_lds((const void*)gemm_w2_kernel<NP, EPI>, W2_LDS); e != hipSuccess)
    return e;
  const int tiles = ((M + W2_BM - 1) / W2_BM) * ((N + W2_BN - 1) / W2_BN);
  hipLaunchKernelGGL((gemm_w2_kernel<NP, EPI>), dim3(tiles), dim3(256), W2_LDS, st, A, W, bias,
                     R, C, Cp, M, N, K, group_m);
  return hipGetLastError();
}

template <int NP>
hipError_t w2_epi(int epi, const __bf16* A, const __bf16* W, const float* bias, const float* R,
                  float* C, __bf16* Cp, int M, int N, int K, int group_m, hipStream_t st) {
  switch (epi) {
    case W2_EPI_BIAS: return w2_launch<NP, W2_EPI_BIAS>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    case W2_EPI_GELU_PACKED:
      return w2_launch<NP, W2_EPI_GELU_PACKED>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    case W2_EPI_BIAS_PACKED:
      return w2_launch<NP, W2_EPI_BIAS_PACKED>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    case W2_EPI_RES: return w2_launch<NP, W2_EPI_RES>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    case W2_EPI_TANH: return w2_launch<NP, W2_EPI_TANH>(A, W, bias, R, C, Cp, M, N, K, group_m, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

// The two-workgroups-per-CU packed GEMM (same contract as ae_launch_gemm_packed: A [M][np*K],
// W [N][np*K] packed planes; f32 C or packed Cp; K % 64 == 0, N % 32 == 0).  group_m: M-tiles
// per grouped sweep of the N-tiles.
extern "C" hipError_t ae_launch_gemm_w2(const unsigned short* A, const unsigned short* W,
                                        const float* bias, const float* R, float* C,
                                        unsigned short* Cp, int M, int N, int K, int epi, int np,
                                        int group_m, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (K % 64 != 0 || N % 32 != 0 || N <= 0 || (np != 1 && np != 2) || group_m < 1)
    return hipErrorInvalidValue;
  auto a = reinterpret_cast<const __bf16*>(A);
  auto w = reinterpret_cast<const __bf16*>(W);
  auto cp = reinterpret_cast<__bf16*>(Cp);
  if (np == 2) return w2_epi<2>(epi, a, w, bias, R, C, cp, M, N, K, group_m, st);
  return w2_epi<1>(epi, a, w, bias, R, C, cp, M, N, K, group_m, st);
}
