// attention_x3.hip — the fused attention of attention_f32.hip on bf16 matrix cores.
//
// Same algorithm and layout (ragged pad-compacted sequences, 128 queries of one (sequence, head)
// per workgroup, online softmax with the query on the lane, optional bit-packed data-flow mask),
// but both products run on v_mfma_f32_32x32x16_bf16 with every operand split into bf16 hi + lo
// (TERMS = 3: x·y ≈ x_hi·y_hi + x_hi·y_lo + x_lo·y_hi, f32 accumulate) — f32-class accuracy at
// the bf16 matrix rate; TERMS = 1 is plain bf16 (the stated-tolerance mode).
//
//   S^T[key][q]  = K · Q^T   A = K (LDS, key rows, 16-B chunks XOR-swizzled by key&7), B = Q^T
//                            (this lane's query row, pre-scaled by 1/8 and split once, in VGPRs)
//   O^T[d][q]   += V^T · P^T A = V^T (LDS, stored transposed [d][key] with 72-B rows: the two
//                            4-key runs a lane reads are conflict-free ds_read_b64), B = P^T taken
//                            straight from the S^T accumulator: accumulator registers 8t..8t+7 of
//                            lane half h hold keys (j&3)+8(j>>2)+4h+16t — that permuted key order
//                            is used for the V^T operand of the same k-slot.
#include <cfloat>
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

namespace {
constexpr int QPB = 128, KT = 32;
constexpr int K_ROWB = 128;          // 64 d bf16 per key row
constexpr int K_PLANE = KT * K_ROWB; // 4 KiB
constexpr int VT_ROWB = 72;          // 32 keys bf16 + 8 B pad
constexpr int VT_PLANE = 64 * VT_ROWB;
constexpr int V_PLANE = KT * K_ROWB;  // row-major V (VAR_VTR): 64 d bf16 per key row
constexpr int OSTRIDE = 65;
template <int VAR>
constexpr int stage_bytes() { return 2 * K_PLANE + 2 * ((VAR & 1) ? V_PLANE : VT_PLANE); }
template <int VAR>
constexpr int lds_bytes() {
  return (2 * stage_bytes<VAR>() > 4 * 32 * OSTRIDE * 4) ? 2 * stage_bytes<VAR>() : 4 * 32 * OSTRIDE * 4;
}

__device__ __forceinline__ int kswz(int key, int chunk) { return chunk ^ (key & 7); }
// row-major V image: 16-B chunk c of key row r at c ^ 4 ((r >> 1) & 1), so the 4 rows of a
// ds_read_b64_tr_b16 block (keys 4m .. 4m+3) land on 4 distinct 16-bank ranges of a 32-lane half
__device__ __forceinline__ int vswz(int key, int chunk) { return chunk ^ (((key >> 1) & 1) << 2); }
}  // namespace

// Variant bits (VAR): 1 = V stored row-major and fed to the PV MFMA through the hardware
// transposed read ds_read_b64_tr_b16 (4-key x 16-d blocks; replaces the transposing 2-byte LDS
// scatter), 2 = exp2 domain (log2 e folded into the Q scale) and the O rescale skipped when no
// lane's running max moved (alpha == 1 exactly: the skip changes no bit).
// PLANES: write the context as packed bf16 planes (hi = bf16(o), lo = bf16(o - hi); layout of
// gemm_planes.hip) for the O-projection instead of f32 rows in out.
template <int TERMS, bool HAS_MASK, bool PLANES, int VAR>
__global__ __launch_bounds__(256, 2) void attn_x3_kernel(const float* __restrict__ qkv,
                                                         float* __restrict__ out,
                                                         unsigned short* __restrict__ op,
                                                         const int* __restrict__ cu,
                                                         const int* __restrict__ q_rows,
                                                         const uint32_t* __restrict__ mask,
                                                         int mask_L) {
  constexpr bool VTR = VAR & 1, EXP2 = VAR & 2;
  constexpr int STAGE = stage_bytes<VAR>();
  __shared__ __attribute__((aligned(16))) unsigned char lds[lds_bytes<VAR>()];
  const int seq = blockIdx.z, head = blockIdx.y, qb = blockIdx.x;
  const int start = cu[seq];
  const int len = cu[seq + 1] - start;
  const int nq = q_rows ? min(len, q_rows[0]) : len;
  if (qb * QPB >= nq) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  constexpr int LDQKV = 3 * AE_HIDDEN;

  // Q fragments: step s covers d = 16s + 8h .. +8 (B operand: B[k=d][j=q])
  const int q = qb * QPB + wave * 32 + li;
  const int qr = q < nq ? q : nq - 1;
  bf16x8 qh[4], ql[4];
  {
    const float* qp = qkv + (size_t)(start + qr) * LDQKV + head * AE_HEAD_DIM;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(qp + 16 * s + 8 * lh);
      const floatx4 b = *reinterpret_cast<const floatx4*>(qp + 16 * s + 8 * lh + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // 1/sqrt(64) (and log2 e in the exp2 domain)
        const float v = (e < 4 ? a[e] : b[e - 4]) * (EXP2 ? 0.18033688011112042f : 0.125f);
        const __bf16 h = (__bf16)v;
        qh[s][e] = h;
        ql[s][e] = (__bf16)(v - (float)h);
      }
    }
  }

  // staging: thread -> key row (tid>>4) and +16, float4 chunk (tid&15) of K and of V
  const int st_key = tid >> 4, st_c4 = tid & 15;
  floatx4 rk[2], rv[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int key = kt * KT + st_key + 16 * i;
      key = key < len ? key : len - 1;
      const float* base = qkv + (size_t)(start + key) * LDQKV + head * AE_HEAD_DIM + st_c4 * 4;
      rk[i] = *reinterpret_cast<const floatx4*>(base + AE_HIDDEN);
      rv[i] = *reinterpret_cast<const floatx4*>(base + 2 * AE_HIDDEN);
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* st = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = st_key + 16 * i;
      // K: 4 consecutive d at d0 = 4*st_c4 -> 8 B in chunk d0/8, half (d0/4)&1
      bf16x4 kh, kl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h = (__bf16)rk[i][e];
        kh[e] = h;
        kl[e] = (__bf16)(rk[i][e] - (float)h);
      }
      const int off = key * K_ROWB + kswz(key, st_c4 >> 1) * 16 + (st_c4 & 1) * 8;
      *reinterpret_cast<bf16x4*>(st + off) = kh;
      if (TERMS == 3) *reinterpret_cast<bf16x4*>(st + K_PLANE + off) = kl;
      if (VTR) {  // V row-major: the same 8 B per plane as K
        bf16x4 vh, vl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __bf16 h = (__bf16)rv[i][e];
          vh[e] = h;
          vl[e] = (__bf16)(rv[i][e] - (float)h);
        }
        const int voff = key * K_ROWB + vswz(key, st_c4 >> 1) * 16 + (st_c4 & 1) * 8;
        *reinterpret_cast<bf16x4*>(st + 2 * K_PLANE + voff) = vh;
        if (TERMS == 3) *reinterpret_cast<bf16x4*>(st + 2 * K_PLANE + V_PLANE + voff) = vl;
        continue;
      }
      // V^T: element (key, d) -> row d, column key
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d = st_c4 * 4 + e;
        const __bf16 h = (__bf16)rv[i][e];
        *reinterpret_cast<__bf16*>(st + 2 * K_PLANE + d * VT_ROWB + key * 2) = h;
        if (TERMS == 3)
          *reinterpret_cast<__bf16*>(st + 2 * K_PLANE + VT_PLANE + d * VT_ROWB + key * 2) =
              (__bf16)(rv[i][e] - (float)h);
      }
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
    const unsigned char* st = lds + cur * STAGE;

    // ---- S^T = K Q^T (4 k-steps of 16 d)
    floatx16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int off = li * K_ROWB + kswz(li, 2 * ks + lh) * 16;
      const bf16x8 kh = *reinterpret_cast<const bf16x8*>(st + off);
      if (TERMS == 3) {
        const bf16x8 kl = *reinterpret_cast<const bf16x8*>(st + K_PLANE + off);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[ks], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[ks], s, 0, 0, 0);
      }
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[ks], s, 0, 0, 0);
    }

    // ---- mask + online softmax (lane = query)
    uint32_t mbits = 0xffffffffu;
    if (HAS_MASK) mbits = mrow[kt];
    float mt = -INFINITY;
    // (EXP2 variants: a full tile without a mask needs no per-key select; the branch is
    // wave-uniform)
    if (EXP2 && !HAS_MASK && (kt + 1) * KT <= len) {
#pragma unroll
      for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[r]);
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
    const float m_new = fmaxf(m_run, mt);
    const float alpha = (m_run == -INFINITY) ? 0.f
                        : EXP2                ? __builtin_amdgcn_exp2f(m_run - m_new)
                                              : __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // exp2(-inf - m) = 0 for finite m; m_new is finite once any key of the row is present
      const float p = EXP2 ? __builtin_amdgcn_exp2f(s[r] - m_new)
                           : ((s[r] == -INFINITY) ? 0.f : __expf(s[r] - m_new));
      s[r] = p;
      psum += p;
    }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (!EXP2 || __any(alpha != 1.f)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) { o0[r] *= alpha; o1[r] *= alpha; }
    }

    // ---- O^T += V^T P^T (2 k-steps of 16 keys, 2 d-tiles)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 ph, pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = s[8 * t + j];
        const __bf16 h = (__bf16)p;
        ph[j] = h;
        pl[j] = (__bf16)(p - (float)h);
      }
      // keys of this k-slot: 16t + 4h + {0..3} and 16t + 8 + 4h + {0..3}
      const int k0 = 16 * t + 4 * lh;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        bf16x8 vh, vl;
        if (VTR) {
          // lane 16g + 4q + p addresses key row k0 + q (and k0 + 8 + q), d columns
          // 32 dt + 16 (g & 1) + 4p; it receives d = 32 dt + (lane & 31) of those 4 keys
          const int kq = k0 + ((lane >> 2) & 3);
          const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
          const unsigned char* vb = st + 2 * K_PLANE + (col & 7) * 2;
          const int o_a = kq * K_ROWB + vswz(kq, col >> 3) * 16;
          const int o_b = (kq + 8) * K_ROWB + vswz(kq + 8, col >> 3) * 16;
          const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb + o_a));
          const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb + o_b));
#pragma unroll
          for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = b[e]; }
          if (TERMS == 3) {
            const bf16x4 c = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb + V_PLANE + o_a));
            const bf16x4 d = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(vb + V_PLANE + o_b));
#pragma unroll
            for (int e = 0; e < 4; ++e) { vl[e] = c[e]; vl[4 + e] = d[e]; }
          }
        } else {
          const int d = dt * 32 + li;
          const unsigned char* vrow = st + 2 * K_PLANE + d * VT_ROWB;
          {
            const bf16x4 a = *reinterpret_cast<const bf16x4*>(vrow + 2 * k0);
            const bf16x4 b = *reinterpret_cast<const bf16x4*>(vrow + 2 * (k0 + 8));
#pragma unroll
            for (int e = 0; e < 4; ++e) { vh[e] = a[e]; vh[4 + e] = b[e]; }
          }
          if (TERMS == 3) {
            const bf16x4 a = *reinterpret_cast<const bf16x4*>(vrow + VT_PLANE + 2 * k0);
            const bf16x4 b = *reinterpret_cast<const bf16x4*>(vrow + VT_PLANE + 2 * (k0 + 8));
#pragma unroll
            for (int e = 0; e < 4; ++e) { vl[e] = a[e]; vl[4 + e] = b[e]; }
          }
        }
        floatx16& o = dt == 0 ? o0 : o1;
        if (TERMS == 3) {
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl, o, 0, 0, 0);
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph, o, 0, 0, 0);
      }
    }

    if (kt + 1 < nkt) lstore(cur ^ 1);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
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
      const size_t o = (size_t)(start + qq) * AE_HIDDEN + head * AE_HEAD_DIM + lane;
      const float v = os[rr * OSTRIDE + lane];
      if (PLANES) {  // packed planes (gemm_planes.hip layout), np = 2 for TERMS 3 else 1
        constexpr int NP = TERMS == 3 ? 2 : 1;
        const int c = head * AE_HEAD_DIM + lane;
        unsigned short* dst = op + (size_t)(start + qq) * NP * AE_HIDDEN + (c >> 5) * 32 * NP + (c & 31);
        const unsigned short h = f2bf(v);
        dst[0] = h;
        if (NP == 2) dst[32] = f2bf(v - __builtin_bit_cast(float, (uint32_t)h << 16));
      } else {
        out[o] = v;
      }
    }
  }
}

namespace {
template <int VAR>
hipError_t attn_launch(const float* qkv, float* out, unsigned short* op, const int* cu,
                       const int* q_rows, int max_q, int n, int heads, const uint32_t* mask,
                       int mask_L, int terms, hipStream_t stream) {
  if (n <= 0 || max_q <= 0) return hipSuccess;
  dim3 grid((max_q + QPB - 1) / QPB, heads, n), block(256);
#define ATT_LAUNCH(T, M, P)                                                                  \
  hipLaunchKernelGGL((attn_x3_kernel<T, M, P, VAR>), grid, block, 0, stream, qkv, out, op, cu, \
                     q_rows, mask, mask_L)
#define ATT_MP(T)                                              \
  if (op) {                                                    \
    if (mask) ATT_LAUNCH(T, true, true); else ATT_LAUNCH(T, false, true);   \
  } else {                                                     \
    if (mask) ATT_LAUNCH(T, true, false); else ATT_LAUNCH(T, false, false); \
  }
  if (terms == 3) {
    ATT_MP(3)
  } else {
    ATT_MP(1)
  }
#undef ATT_MP
#undef ATT_LAUNCH
  return hipGetLastError();
}
constexpr int ATT_VAR = 3;  // production variant (tools/attn_bench.py A/B: 227 -> 192 us at B=64, L=512)
}  // namespace

extern "C" hipError_t ae_launch_attention_x3(const float* qkv, float* out, unsigned short* op,
                                             const int* cu,
                                             const int* q_rows, int max_q, int n, int heads,
                                             const uint32_t* mask, int mask_L, int terms,
                                             hipStream_t stream) {
  return attn_launch<ATT_VAR>(qkv, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, terms,
                              stream);
}

// Kernel experiments (tools/attn_bench.py): the variant bits of attn_x3_kernel (0..3).  Every
// variant computes the same attention; not part of include/alert_engine.h.
extern "C" hipError_t ae_bench_attention_x3(const float* qkv, float* out, unsigned short* op,
                                            const int* cu, const int* q_rows, int max_q, int n,
                                            int heads, const uint32_t* mask, int mask_L, int terms,
                                            int variant, hipStream_t stream) {
  switch (variant) {
    case 0: return attn_launch<0>(qkv, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, terms, stream);
    case 1: return attn_launch<1>(qkv, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, terms, stream);
    case 2: return attn_launch<2>(qkv, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, terms, stream);
    case 3: return attn_launch<3>(qkv, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, terms, stream);
    default: return hipErrorInvalidValue;
  }
}
