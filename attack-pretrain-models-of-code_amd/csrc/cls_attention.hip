// cls_attention.hip — the last encoder layer's attention for the one row the task heads read.
//
// The heads read features[:, 0, :] only (RobertaClassificationHead via
// CodeXGLUE/Defect-detection/code/model.py:25; the clone / authorship heads likewise), so the last
// layer needs the attention output of ONE query per sequence, the CLS row.  Per head h with
// q = W_q x_0 + b_q (the CLS query) and keys / values k_j = W_k x_j + b_k, v_j = W_v x_j + b_v:
//   s_j  = q·k_j / 8 = x_j · (W_k^T q) / 8 + q·b_k / 8        (the last term is the same for every
//                                                           j, so softmax drops it)
//   ctx  = Σ_j p_j v_j = W_v (Σ_j p_j x_j) + b_v              (Σ_j p_j = 1)
// so W_k is absorbed into the query (u_h = W_k,h^T q_h: 768 values per head) and W_v is applied
// once to the p-weighted row sum.  The layer's K / V projections over all T rows (the QKV GEMM,
// 116 GFLOP at B=64 x L=512) are never computed: the attention reads the layer-input rows x_j
// (f32, 3 KB each) once, which makes it HBM-bound at ~T·3 KB.
//
// Kernels (all f32 arithmetic, exact-f32 MFMA products; per-sequence work only, with key chunks
// fixed at 64 keys, so a sequence's result does not depend on the batch it is in):
//   cls_u_kernel       u[s][h][:] = Σ_d q[s][64h+d] W_k[64h+d][:]  (VALU; 4 sequences x 256
//                      columns per workgroup: 576 workgroups at n = 64)
//   cls_attn_kernel    one workgroup per (sequence, 64-key chunk): scores of 16-key tiles by
//                      v_mfma_f32_16x16x4_f32 (16 keys x 16 head slots x 768), online softmax in
//                      the exp2 domain, y_h += Σ p x_j by the same MFMA (16 head slots x 768) ->
//                      per-chunk (max, sum, y[12][768])
//   cls_combine_kernel the chunks of a sequence merged in chunk order -> ybar[s][h][:], one
//                      workgroup per (sequence, head, 256 columns)
//   cls_vproj_kernel   ctx[s][64h+d] = b_v[64h+d] + Σ_c W_v[64h+d][c] ybar[s][h][c] by
//                      v_mfma_f32_16x16x4_f32, one workgroup per (16 sequences, head, 16 d)
// (round 4, first form: a 16-sequence u kernel, a combine over (sequence, head) and a VALU
// projection over 48 workgroups took 18.7 + 15.3 + 72.4 us of the ~145 us at B=64,
// profiles/r4g_*; merging the chunks in the sequence's last-arriving chunk workgroup instead of a
// combine kernel made the attention kernel 36 -> 163-204 us: one workgroup then reads all of a
// sequence's records, r4i)
// Round 6: the same kernels serve any fixed number qper of query rows per sequence (query qi of
// sequence qi / qper; its chunk records after the sequence's earlier queries', rec_base): the
// row windows of ae_encode_rows, where each config-3 candidate is read only at its own span
// (get_substitutes.py:98-108) — the last layer then costs O(rows) instead of a full layer.
// Masked (GraphCodeBERT) launches read row 0 of the sequence's bit-packed mask; the CLS row always
// attends itself (special tokens see [:max_length], utils.py:555-557), so a fully masked CLS row
// cannot occur — if it does the device error flag poisons the scores (alert_engine.h ae_score).
#include "common.h"

namespace {

constexpr int H = AE_HIDDEN;        // 768
constexpr int NH = 12;              // heads
constexpr int DH = AE_HEAD_DIM;     // 64
constexpr int KC = 64;              // keys per workgroup chunk
constexpr int KT = 16;              // keys per MFMA tile
constexpr int XS = H + 4;           // LDS row stride (floats) of the x / u tiles
constexpr int REC = 32 + NH * H;    // floats per chunk record: m[16], l[16], y[12][768]

// first chunk record of query qj of sequence s (rows [beg, beg + len)): qper·((beg >> 6) + s) bounds
// qper times the chunk records of the sequences before s, and query qj's ceil(len / 64) chunks
// follow the sequence's earlier queries' (CLS, qper 1: (beg >> 6) + s, as before)
__device__ __forceinline__ size_t rec_base(int beg, int s, int qper, int qj, int len) {
  return (size_t)qper * ((size_t)(beg >> 6) + s) + (size_t)qj * ((len + KC - 1) / KC);
}

__global__ __launch_bounds__(256) void cls_u_kernel(const float* __restrict__ q,
                                                    const float* __restrict__ wk, int n,
                                                    float* __restrict__ u) {
  constexpr int SB = 4;  // sequences per workgroup
  __shared__ float qs[SB][DH];
  const int h = blockIdx.y, s0 = blockIdx.x * SB, col = blockIdx.z * 256 + threadIdx.x;
  {
    const int r = threadIdx.x / DH, d = threadIdx.x % DH;  // 256 = SB x DH
    qs[r][d] = s0 + r < n ? q[(size_t)(s0 + r) * H + h * DH + d] : 0.f;
  }
  __syncthreads();
  float acc[SB];
#pragma unroll
  for (int r = 0; r < SB; ++r) acc[r] = 0.f;
  const float* w = wk + (size_t)h * DH * H + col;
#pragma unroll 8
  for (int d = 0; d < DH; ++d) {
    const float wv = w[(size_t)d * H];
#pragma unroll
    for (int r = 0; r < SB; ++r) acc[r] = fmaf(qs[r][d], wv, acc[r]);
  }
  for (int r = 0; r < SB && s0 + r < n; ++r) u[((size_t)(s0 + r) * NH + h) * H + col] = acc[r];
}

// one workgroup (8 waves) per (chunk c, sequence s); LDS: u [12][XS], x tile [16][XS], partial
// score tiles [8][256], p [16][16], alpha / running max / running sum [16] each.  (u held in 24
// registers per lane instead, for 59 KiB of LDS and two workgroups per CU: 63 vs 41 us at B=64,
// profiles/r4o — slower, not kept.)
__global__ __launch_bounds__(512) void cls_attn_kernel(
    const float* __restrict__ x, const float* __restrict__ u, const int* __restrict__ cu,
    const uint32_t* __restrict__ mask, int mask_L, float scale, int qper,
    float* __restrict__ part) {
  extern __shared__ float lds[];
  float* us = lds;                  // [12][XS]
  float* xs = us + NH * XS;         // [16][XS]
  float* sred = xs + KT * XS;       // [8][256]
  float* pt = sred + 8 * 256;       // [16 keys][16 heads]
  float* alpha = pt + 256;          // [16]
  float* mrun = alpha + 16;         // [16]
  float* lrun = mrun + 16;          // [16]
  // query qi = blockIdx.y of sequence s = qi / qper (CLS: qper 1, the query is the sequence)
  const int c = blockIdx.x, qi = blockIdx.y, s = qi / qper, qj = qi - s * qper;
  const int beg = cu[s], len = cu[s + 1] - beg, k0 = c * KC;
  if (k0 >= len) return;
  const int nk = min(KC, len - k0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, l4 = lane >> 4;
  const uint32_t* mrow = mask ? mask + (size_t)s * mask_L * (mask_L / 32) : nullptr;

  // u of this sequence -> LDS (12 x 192 float4)
  const float4* u4 = reinterpret_cast<const float4*>(u + (size_t)qi * NH * H);
  for (int i = tid; i < NH * (H / 4); i += 512) {
    const int r = i / (H / 4), c4 = i % (H / 4);
    *reinterpret_cast<float4*>(us + r * XS + 4 * c4) = u4[i];
  }
  if (tid < 16) {
    mrun[tid] = -INFINITY;
    lrun[tid] = 0.f;
  }
  floatx4 acc[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int ntile = (nk + KT - 1) / KT;
  float4 pre[6];  // the next x tile, 16 rows x 192 float4 over 512 threads
  auto load_tile = [&](int t) {
    const int r0 = k0 + t * KT;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int f = tid + 512 * j, r = f / (H / 4), c4 = f % (H / 4);
      pre[j] = r0 + r < len ? reinterpret_cast<const float4*>(x + (size_t)(beg + r0 + r) * H)[c4]
                            : float4{0.f, 0.f, 0.f, 0.f};
    }
  };
  load_tile(0);
  for (int t = 0; t < ntile; ++t) {
    __syncthreads();  // the previous tile's readers are done with xs
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int f = tid + 512 * j, r = f / (H / 4), c4 = f % (H / 4);
      *reinterpret_cast<float4*>(xs + r * XS + 4 * c4) = pre[j];
    }
    __syncthreads();
    if (t + 1 < ntile) load_tile(t + 1);  // in flight under this tile's MFMAs
    // scores: wave w contracts dims [96w, 96w + 96) -> D[key = 4*l4 + i][head slot = l15]
    floatx4 d = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* xa = xs + l15 * XS + 96 * w + l4;
    const float* ub = us + (l15 < NH ? l15 : 0) * XS + 96 * w + l4;
#pragma unroll
    for (int kk = 0; kk < 24; ++kk) {
      const float b = l15 < NH ? ub[4 * kk] : 0.f;
      d = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[4 * kk], b, d, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) sred[w * 256 + (4 * l4 + i) * 16 + l15] = d[i];
    __syncthreads();
    if (tid < 256) {  // key = tid >> 4, head slot = tid & 15
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += sred[q * 256 + tid];
      const int key = k0 + t * KT + (tid >> 4);
      bool ok = key < len;
      if (ok && mrow) ok = (mrow[key >> 5] >> (key & 31)) & 1u;
      pt[tid] = ok ? v * scale : -INFINITY;
    }
    __syncthreads();
    if (tid < 16) {  // online softmax of head slot tid over the tile's 16 keys
      const float mo = mrun[tid];
      float mx = mo;
#pragma unroll
      for (int j = 0; j < KT; ++j) mx = fmaxf(mx, pt[j * 16 + tid]);
      float a = 1.f, sum = 0.f;
      if (mx != -INFINITY) {
        a = __builtin_amdgcn_exp2f(mo - mx);
#pragma unroll
        for (int j = 0; j < KT; ++j) {
          const float p = __builtin_amdgcn_exp2f(pt[j * 16 + tid] - mx);
          pt[j * 16 + tid] = p;
          sum += p;
        }
      } else {
#pragma unroll
        for (int j = 0; j < KT; ++j) pt[j * 16 + tid] = 0.f;
      }
      alpha[tid] = a;
      mrun[tid] = mx;
      lrun[tid] = fmaf(lrun[tid], a, sum);
    }
    __syncthreads();
    // y[head slot][col] = alpha * y + Σ_key p[key][slot] x[key][col]; wave w owns cols [96w, +96)
    float al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) al[i] = alpha[4 * l4 + i];
    float pa[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pa[q] = pt[(4 * q + l4) * 16 + l15];
#pragma unroll
    for (int ct = 0; ct < 6; ++ct) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[ct][i] *= al[i];
      const float* xb = xs + l4 * XS + 96 * w + 16 * ct + l15;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[q], xb[4 * q * XS], acc[ct], 0, 0, 0);
    }
  }
  float* rec = part + (rec_base(beg, s, qper, qj, len) + c) * REC;
  __syncthreads();
  if (tid < 16) {
    rec[tid] = mrun[tid];
    rec[16 + tid] = lrun[tid];
  }
#pragma unroll
  for (int ct = 0; ct < 6; ++ct)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hs = 4 * l4 + i;
      if (hs < NH) rec[32 + hs * H + 96 * w + 16 * ct + l15] = acc[ct][i];
    }

}

// the chunks of sequence s merged in chunk order: ybar[s][h][c] = Σ_k 2^(m_k - M) y_k[h][c] / L
__global__ __launch_bounds__(256) void cls_combine_kernel(const float* __restrict__ part,
                                                          const int* __restrict__ cu, int qper,
                                                          float* __restrict__ ybar,
                                                          int* __restrict__ err) {
  const int qi = blockIdx.x, h = blockIdx.y, col = blockIdx.z * 256 + threadIdx.x;
  const int s = qi / qper, qj = qi - s * qper;
  const int beg = cu[s], len = cu[s + 1] - beg, nc = (len + KC - 1) / KC;
  const float* rec0 = part + rec_base(beg, s, qper, qj, len) * REC;
  float M = -INFINITY;
  for (int c = 0; c < nc; ++c) M = fmaxf(M, rec0[(size_t)c * REC + h]);
  float L = 0.f, y = 0.f;
  for (int c = 0; c < nc; ++c) {
    const float m = rec0[(size_t)c * REC + h];
    if (m != -INFINITY) {
      const float e = __builtin_amdgcn_exp2f(m - M);
      L = fmaf(rec0[(size_t)c * REC + 16 + h], e, L);
      y = fmaf(rec0[(size_t)c * REC + 32 + h * H + col], e, y);
    }
  }
  if (!(L > 0.f)) {  // no key attended: cannot happen for a CLS / unmasked row; poison the call
    if (threadIdx.x == 0 && blockIdx.z == 0) atomicOr(err, 2);
  }
  ybar[((size_t)qi * NH + h) * H + col] = y * (1.f / L);
}

// ctx[s][64h + d] = b_v[64h + d] + Σ_c W_v[64h + d][c] ybar[s][h][c]: one workgroup per (16
// sequences, head h, 16 d).  Wave w sums c in [192 w, 192 w + 192) by v_mfma_f32_16x16x4_f32: a
// lane loads 4 consecutive c of its row as one float4 and feeds them to 4 MFMAs as their k-slot —
// the same permutation of c on both operands, so the dot products are unchanged — and the 4
// waves' 16 x 16 tiles are added in wave order
__global__ __launch_bounds__(256) void cls_vproj_kernel(const float* __restrict__ ybar,
                                                        const float* __restrict__ wv,
                                                        const float* __restrict__ bv, int n,
                                                        float* __restrict__ ctx) {
  __shared__ float red[4][256];
  const int h = blockIdx.y, s0 = blockIdx.x * 16, d0 = blockIdx.z * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int s = min(s0 + i, n - 1);
  const float* a = ybar + ((size_t)s * NH + h) * H + 192 * w + 4 * kq;
  const float* b = wv + (size_t)(h * DH + d0 + i) * H + 192 * w + 4 * kq;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int blk = 0; blk < 12; ++blk) {
    const float4 av = *reinterpret_cast<const float4*>(a + 16 * blk);
    const float4 bw = *reinterpret_cast<const float4*>(b + 16 * blk);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bw.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bw.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bw.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bw.w, acc, 0, 0, 0);
  }
  // D[sequence 4 kq + r][d i] of the wave's c range
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][r * 64 + lane] = acc[r];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sidx = s0 + 4 * kq + r, d = d0 + i;
      const float v = ((red[0][r * 64 + lane] + red[1][r * 64 + lane]) + red[2][r * 64 + lane]) +
                      red[3][r * 64 + lane];
      if (sidx < n) ctx[(size_t)sidx * H + h * DH + d] = v + bv[h * DH + d];
    }
  }
}

}  // namespace

extern "C" {

// floats of the per-chunk partial records for sequences whose token rows total T (any lens), with
// qper queries per sequence
long ae_cls_attention_part_floats(long T, int n, int qper) {
  return (long)qper * ((T >> 6) + n + 2) * (long)REC;
}

// One query row per (sequence, slot): nq = n·qper queries, query qi of sequence qi / qper (the CLS
// path: qper 1, the CLS row of every sequence; ae_encode_rows: a window of rows per sequence).
// q: [nq][768] queries (the split modes' W_q carries log2(e)/8, so scale = 1; the exact mode's
// does not, scale = log2(e)/8); wk, wv: [768][768] row-major K / V projection weights; bv: [768];
// x: [T][768] layer-input rows (compacted, cu offsets); u_ws, ybar_ws: [nq][12][768];
// part_ws: ae_cls_attention_part_floats(T, n, qper) floats; ctx: [nq][768] out.  mask (the
// GraphCodeBERT bit mask, row 0 of each sequence) only with qper 1.
hipError_t ae_launch_cls_attention(const float* x, const float* q, const float* wk,
                                   const float* wv, const float* bv, const int* cu, int n,
                                   int qper, int max_len, const uint32_t* mask, int mask_L,
                                   float scale, float* u_ws, float* part_ws, float* ybar_ws,
                                   float* ctx, int* err, hipStream_t st) {
  if (n <= 0 || qper <= 0) return hipSuccess;
  if (mask && qper != 1) return hipErrorInvalidValue;
  const int nq = n * qper;
  hipLaunchKernelGGL(cls_u_kernel, dim3((nq + 3) / 4, NH, H / 256), dim3(256), 0, st, q, wk, nq,
                     u_ws);
  const size_t lds = (size_t)(NH * XS + KT * XS + 8 * 256 + 256 + 48) * sizeof(float);
  hipError_t e = ensure_dynamic_lds((const void*)cls_attn_kernel, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cls_attn_kernel, dim3((max_len + KC - 1) / KC, nq), dim3(512), lds, st, x,
                     u_ws, cu, mask, mask_L, scale, qper, part_ws);
  hipLaunchKernelGGL(cls_combine_kernel, dim3(nq, NH, H / 256), dim3(256), 0, st, part_ws, cu,
                     qper, ybar_ws, err);
  hipLaunchKernelGGL(cls_vproj_kernel, dim3((nq + 15) / 16, NH, DH / 16), dim3(256), 0, st,
                     ybar_ws, wv, bv, nq, ctx);
  return hipGetLastError();
}

}  // extern "C"
