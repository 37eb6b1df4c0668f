// attention_f32.hip — fused multi-head self-attention over ragged (pad-compacted) sequences, f32.
//
// Replaces HF eager_attention_forward as reached from the victim (CodeXGLUE/Defect-detection/
// code/model.py:25, attention_mask = input_ids.ne(1)): softmax(Q K^T / 8 + mask) V per head.
// The engine drops pad tokens before the encoder (a padded key is masked for every query and a
// pad query row never reaches the CLS output), so sequences arrive compacted: tokens of sequence
// s are rows cu[s] .. cu[s+1]-1 of the packed QKV matrix [T, 3*768] (Q | K | V, head h at 64h).
// Optional data-flow mask (GraphCodeBERT, GraphCodeBERT/Defect-detection/code/model.py:35 with
// utils.py:540-576): bit-packed [n][Lm][Lm/32 words] over the compacted index, bit k of row q
// set = query q may attend key k.
//
// gfx950 mapping (flash-style, online softmax, exact-f32 MFMA v_mfma_f32_32x32x2_f32):
//   workgroup = 4 waves = 128 queries of one (sequence, head); each wave owns 32 queries.
//   Both products are computed transposed so that the query index lives on the lane:
//     S^T[key][q]  = K · Q^T     A = K tile from LDS (row = key), B = this lane's Q row in VGPRs
//     O^T[d][q]   += V^T · P^T   A = V tile from LDS, B = P^T straight from the S^T accumulator
//   (register s of the S^T accumulator holds key (s&3)+8(s>>2)+4h, which is exactly the k-slot
//   the next MFMA needs), so the row max / sum / rescale are lane-local plus one xor-32 shuffle.
//   K/V tiles of 32 keys are double-buffered in LDS (K rows padded to 68 floats: conflict-free
//   ds_read_b128), next tile's global loads issued before the current tile's MFMAs.
#include <cfloat>
#include "common.h"

namespace {
constexpr int QPB = 128;      // queries per workgroup
constexpr int KT = 32;        // keys per tile
constexpr int KSTRIDE = 68;   // padded K row (floats)
constexpr int VSTRIDE = 64;
constexpr int OSTRIDE = 65;   // output staging row
constexpr int LDS_FLOATS = 2 * KT * KSTRIDE + 2 * KT * VSTRIDE;  // 8448 floats = 33 KiB
static_assert(4 * 32 * OSTRIDE <= LDS_FLOATS, "output staging must fit in the K/V buffers");
}  // namespace

template <bool HAS_MASK>
__global__ __launch_bounds__(256, 2) void attn_f32_kernel(const float* __restrict__ qkv,
                                                          float* __restrict__ out,
                                                          const int* __restrict__ cu,
                                                          const int* __restrict__ q_rows,
                                                          const uint32_t* __restrict__ mask,
                                                          int mask_L, float scale) {
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  float* Ks = lds;                       // [2][KT][KSTRIDE]
  float* Vs = lds + 2 * KT * KSTRIDE;    // [2][KT][VSTRIDE]

  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  // q_rows (optional): number of query rows to compute per sequence (1 = CLS only).
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QPB >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  constexpr int LDQKV = 3 * AE_HIDDEN;

  // this lane's query row (clamped; rows >= nq are computed and discarded)
  const int q = qb * QPB + wave * 32 + li;
  const int qr = q < nq ? q : nq - 1;
  float qreg[32];
  {
    const float* qp = qkv + (size_t)(start + qr) * LDQKV + head * AE_HEAD_DIM + 32 * lh;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(qp + 4 * c);
      qreg[4 * c + 0] = v[0] * scale;
      qreg[4 * c + 1] = v[1] * scale;
      qreg[4 * c + 2] = v[2] * scale;
      qreg[4 * c + 3] = v[3] * scale;
    }
  }

  // K/V tile staging: thread -> (row = tid>>4 and +16, float4 chunk = tid&15)
  const int st_row = tid >> 4, st_chunk = tid & 15;
  floatx4 rk[2], rv[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int key = kt * KT + st_row + 16 * i;
      key = key < len ? key : len - 1;
      const float* base = qkv + (size_t)(start + key) * LDQKV + head * AE_HEAD_DIM + st_chunk * 4;
      rk[i] = *reinterpret_cast<const floatx4*>(base + AE_HIDDEN);
      rv[i] = *reinterpret_cast<const floatx4*>(base + 2 * AE_HIDDEN);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = st_row + 16 * i;
      *reinterpret_cast<floatx4*>(&Ks[buf * KT * KSTRIDE + row * KSTRIDE + st_chunk * 4]) = rk[i];
      *reinterpret_cast<floatx4*>(&Vs[buf * KT * VSTRIDE + row * VSTRIDE + st_chunk * 4]) = rv[i];
    }
  };

  floatx16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o0[r] = 0.f; o1[r] = 0.f; }
  float m_run = -INFINITY, l_run = 0.f;

  const uint32_t* mrow = nullptr;
  if (HAS_MASK) mrow = mask + ((size_t)seq * mask_L + qr) * (mask_L / 32);

  const int nkt = (len + KT - 1) / KT;
  gload(0);
  lstore(0);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kt + 1);

    // S^T tile: 32 keys x 32 queries, contraction over d (half h owns d in [32h, 32h+32))
    floatx16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    const float* kp = &Ks[cur * KT * KSTRIDE + li * KSTRIDE + 32 * lh];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const floatx4 kv = *reinterpret_cast<const floatx4*>(kp + 4 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[e], qreg[4 * c + e], s, 0, 0, 0);
    }

    // mask + online softmax (lane = query; this lane holds 16 of the 32 keys, partner lane^32
    // the other 16)
    uint32_t mbits = 0xffffffffu;
    if (HAS_MASK) mbits = mrow[kt];
    float mt = -INFINITY;
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
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    // a fully masked prefix keeps m_new = -inf: guard the exp arguments
    const float alpha = (m_run == -INFINITY) ? 0.f : __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = (s[r] == -INFINITY) ? 0.f : __expf(s[r] - m_new);
      s[r] = p;
      psum += p;
    }
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }

    // O^T += V^T P^T
    const float* vp = &Vs[cur * KT * VSTRIDE + li];
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int kk = mfma32_row(st, lh);
      const float v0 = vp[kk * VSTRIDE];
      const float v1 = vp[kk * VSTRIDE + 32];
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, s[st], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, s[st], o1, 0, 0, 0);
    }

    if (kt + 1 < nkt) lstore(cur ^ 1);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;

  // stage O (q rows x 64 d) per wave through LDS, then write whole rows
  float* os = lds + wave * 32 * OSTRIDE;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = mfma32_row(r, lh);
    os[li * OSTRIDE + d] = o0[r] * inv;
    os[li * OSTRIDE + 32 + d] = o1[r] * inv;
  }
  __syncthreads();
  for (int rr = 0; rr < 32; ++rr) {
    const int qq = qb * QPB + wave * 32 + rr;
    if (qq < nq) out[(size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + lane] = os[rr * OSTRIDE + lane];
  }
}

// Launcher: grid = (ceil(max_len/128), heads, n).  q_rows (device, optional) limits the query
// rows per sequence (1 => CLS row only, used for the last encoder layer).
extern "C" hipError_t ae_launch_attention_f32(const float* qkv, float* out, const int* cu,
                                              const int* q_rows, int max_q, int n, int heads,
                                              const uint32_t* mask, int mask_L, hipStream_t stream) {
  if (n <= 0 || max_q <= 0) return hipSuccess;
  dim3 grid((max_q + QPB - 1) / QPB, heads, n), block(256);
  const float scale = 0.125f;  // 64^-0.5, exact power of two
  if (mask)
    hipLaunchKernelGGL(attn_f32_kernel<true>, grid, block, 0, stream, qkv, out, cu, q_rows, mask,
                       mask_L, scale);
  else
    hipLaunchKernelGGL(attn_f32_kernel<false>, grid, block, 0, stream, qkv, out, cu, q_rows, mask,
                       mask_L, scale);
  return hipGetLastError();
}
