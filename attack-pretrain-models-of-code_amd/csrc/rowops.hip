// rowops.hip — pad compaction, fused embedding gather + LayerNorm, LayerNorm, CLS gather and the
// task heads.  All are row kernels over 768-wide f32 rows: one wave per row, 12 floats per lane
// (3 x float4, coalesced 1 KiB per wave-instruction), wave-shuffle reductions.
//
// Reference semantics (HF RoBERTa eager, reached from CodeXGLUE/Defect-detection/code/model.py:25):
//   position ids  = cumsum(ids != pad) * (ids != pad) + pad   (modeling_roberta.py:142-155)
//   embeddings    = LN(word[id] + pos[position] + type[0]), eps 1e-5
//   heads: Devign   sigmoid(out_proj(tanh(dense(h_cls))))            model.py:24-34
//          AA       softmax(out_proj(tanh(dense(h_cls))))            Authorship-Attribution/code/model.py:13-54
//          clone    softmax(out_proj(tanh(dense(cat(h_cls_a, h_cls_b)))))  Clone-detection-BigCloneBench/code/model.py:13-53
#include "common.h"

// ---------------------------------------------------------------------------------------------
// Pad compaction: one workgroup per sequence.  Writes the non-pad ids of row s, in order, to
// tok_ids[cu[s] + j] and their position ids (explicit `pos` row, or the RoBERTa rule pad+1+j).
// keep_all (a model called without attention_mask, e.g. get_substitutes.py:62,73,105): the first
// cu[s+1]-cu[s] ids of the row are all kept — a pad id is then an ordinary, attended token whose
// position is `pad`, and only non-pad tokens advance the position counter (HF
// create_position_ids_from_input_ids).
// Also records where each compacted token came from (src_col) for ae_encode scatter-back.
// The segment of row s is exactly cu[s+1]-cu[s] tokens: a row whose non-pad count disagrees with
// that length (e.g. caller lens that count a literal "<pad>" token of the source text) never writes
// outside its segment; its unfilled slots get the pad id and `err` is set, which turns every
// output of the call into NaN (head_out / scatter_rows) instead of a silently wrong score.
__global__ __launch_bounds__(256) void compact_kernel(const int* __restrict__ ids,
                                                      const int* __restrict__ pos,
                                                      const int* __restrict__ cu, int L, int pad,
                                                      int keep_all,
                                                      int* __restrict__ tok_ids,
                                                      int* __restrict__ tok_pos,
                                                      int* __restrict__ src_col,
                                                      int* __restrict__ err) {
  __shared__ int wave_tot[4], wave_np[4];
  __shared__ int carry, carry_np;
  const int s = blockIdx.x;
  const int base = cu[s];
  const int len = cu[s + 1] - base;
  const int* row = ids + (size_t)s * L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = carry_np = 0;
  __syncthreads();
  for (int c0 = 0; c0 < L; c0 += 256) {
    const int c = c0 + tid;
    const int id = c < L ? row[c] : pad;
    const int nonpad = c < L && id != pad;
    const int keep = keep_all ? c < len : nonpad;
    const unsigned long long bal = __ballot(keep), bnp = __ballot(nonpad);
    const unsigned long long below = (1ull << lane) - 1ull;
    const int before = __popcll(bal & below), np_before = __popcll(bnp & below);
    if (lane == 0) {
      wave_tot[wave] = __popcll(bal);
      wave_np[wave] = __popcll(bnp);
    }
    __syncthreads();
    int off = carry, off_np = carry_np;
    for (int w = 0; w < wave; ++w) {
      off += wave_tot[w];
      off_np += wave_np[w];
    }
    if (keep && off + before < len) {
      const int j = off + before;
      tok_ids[base + j] = id;
      tok_pos[base + j] = pos ? pos[(size_t)s * L + c] : (nonpad ? pad + 1 + off_np + np_before : pad);
      if (src_col) src_col[base + j] = c;
    }
    __syncthreads();
    if (tid == 0) {
      carry += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
      carry_np += wave_np[0] + wave_np[1] + wave_np[2] + wave_np[3];
    }
    __syncthreads();
  }
  if (carry != len) {  // lens disagree with the row's ids: fill the rest in-bounds, flag the call
    for (int j = carry + tid; j < len; j += 256) {
      tok_ids[base + j] = pad;
      tok_pos[base + j] = pad;
      if (src_col) src_col[base + j] = L;  // outside every scatter window
    }
    if (tid == 0) atomicOr(err, 1);
  }
}

__device__ __forceinline__ void ln_row_store(float (&v)[12], const float* __restrict__ g,
                                             const float* __restrict__ b, float eps,
                                             float* __restrict__ out, int lane,
                                             unsigned short* __restrict__ op = nullptr,
                                             int np = 0) {
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 12; ++i) sum += v[i];
  const float mean = wave_sum(sum) * (1.f / AE_HIDDEN);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const float d = v[i] - mean;
    sq += d * d;
  }
  const float var = wave_sum(sq) * (1.f / AE_HIDDEN);
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    const floatx4 gg = *reinterpret_cast<const floatx4*>(g + col);
    const floatx4 bb = *reinterpret_cast<const floatx4*>(b + col);
    floatx4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[4 * c + e] - mean) * rstd * gg[e] + bb[e];
    *reinterpret_cast<floatx4*>(out + col) = o;
    if (op) {  // packed bf16 planes for the split-precision GEMMs (gemm_planes.hip): o = hi + lo
      ushortx4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h[e] = f2bf(o[e]);
        l[e] = f2bf(o[e] - __builtin_bit_cast(float, (uint32_t)h[e] << 16));
      }
      unsigned short* dst = op + (col >> 5) * 32 * np + (col & 31);
      *reinterpret_cast<ushortx4*>(dst) = h;
      if (np == 2) *reinterpret_cast<ushortx4*>(dst + 32) = l;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Embedding gather + add + LayerNorm.  4 rows per 256-thread workgroup.
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int* __restrict__ tok_ids, const int* __restrict__ tok_pos,
    const float* __restrict__ wemb, const float* __restrict__ pemb,
    const float* __restrict__ temb, const float* __restrict__ g, const float* __restrict__ b,
    float eps, int T, int max_pos, float* __restrict__ x, unsigned short* __restrict__ xp,
    int np, const uint32_t* __restrict__ node_mask, int mask_L, const int* __restrict__ cu,
    int n) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int id = tok_ids[row];
  const int p_raw = tok_pos[row];
  const int p = p_raw < 0 ? 0 : (p_raw >= max_pos ? max_pos - 1 : p_raw);  // GCB hazard, App. A
  const float* pe = pemb + (size_t)p * AE_HIDDEN;
  float w[12];
  if (node_mask && p_raw == 0) {
    // GraphCodeBERT data-flow node (GraphCodeBERT/Defect-detection/code/model.py:27-33): its input
    // embedding is the mean word embedding of the code tokens (position >= 2) its mask row
    // attends; 0 when it attends none (0 / (0 + 1e-10)).  Rows are pad-compacted with trailing
    // pads only, so the compacted index of a token equals its column in the mask row.
    int lo = 0, hi = n;  // sequence s with cu[s] <= row < cu[s+1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (cu[mid] <= row) lo = mid; else hi = mid;
    }
    const int base = cu[lo], len = cu[lo + 1] - base;
    const uint32_t* mrow = node_mask + ((size_t)lo * mask_L + (row - base)) * (mask_L / 32);
#pragma unroll
    for (int e = 0; e < 12; ++e) w[e] = 0.f;
    int cnt = 0;
    for (int wd = 0; wd * 32 < len; ++wd) {
      uint32_t bits = mrow[wd];
      if (len - wd * 32 < 32) bits &= (1u << (len - wd * 32)) - 1u;
      while (bits) {
        const int j = wd * 32 + __builtin_ctz(bits);
        bits &= bits - 1u;
        if (tok_pos[base + j] < 2) continue;
        ++cnt;
        const float* te = wemb + (size_t)tok_ids[base + j] * AE_HIDDEN;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const floatx4 a = *reinterpret_cast<const floatx4*>(te + c * 256 + lane * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) w[4 * c + e] += a[e];
        }
      }
    }
    const float inv = 1.0f / ((float)cnt + 1e-10f);
#pragma unroll
    for (int e = 0; e < 12; ++e) w[e] *= inv;
  } else {
    const float* we = wemb + (size_t)id * AE_HIDDEN;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(we + c * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * c + e] = a[e];
    }
  }
  float v[12];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    const floatx4 bb = *reinterpret_cast<const floatx4*>(pe + col);
    const floatx4 t = *reinterpret_cast<const floatx4*>(temb + col);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * c + e] = (w[4 * c + e] + t[e]) + bb[e];
  }
  const size_t o = (size_t)row * AE_HIDDEN;
  ln_row_store(v, g, b, eps, x + o, lane, xp ? xp + o * np : nullptr, np);
}

// In-place (or out-of-place) LayerNorm of T rows.
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ in,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ b, float eps,
                                                        int T, float* __restrict__ out,
                                                        unsigned short* __restrict__ op, int np) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const float* r = in + (size_t)row * AE_HIDDEN;
  float v[12];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(r + c * 256 + lane * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * c + e] = a[e];
  }
  const size_t o = (size_t)row * AE_HIDDEN;
  ln_row_store(v, g, b, eps, out + o, lane, op ? op + o * np : nullptr, np);
}

// Gather the first (CLS) row of every sequence from two [T,768] matrices into compact [n,768].
__global__ __launch_bounds__(256) void gather_cls_kernel(const float* __restrict__ a,
                                                         const float* __restrict__ b,
                                                         const int* __restrict__ cu, int n,
                                                         float* __restrict__ ac,
                                                         float* __restrict__ bc) {
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= n) return;
  const size_t src = (size_t)cu[s] * AE_HIDDEN;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    *reinterpret_cast<floatx4*>(ac + (size_t)s * AE_HIDDEN + col) =
        *reinterpret_cast<const floatx4*>(a + src + col);
    *reinterpret_cast<floatx4*>(bc + (size_t)s * AE_HIDDEN + col) =
        *reinterpret_cast<const floatx4*>(b + src + col);
  }
}

// ---------------------------------------------------------------------------------------------
// Classification head output layer.  The head's dense layer (+tanh) runs as an MFMA GEMM over the
// compact CLS rows (for the clone pair head the [n,768] CLS matrix IS the [n/2,1536] pair-feature
// matrix); this kernel applies out_proj and the final activation, one wave per output row.
//   kind 0: sigmoid1  -> out[row] = sigmoid(logit)        (C == 1)
//   kind 1: softmaxN / kind 2: pair2 -> out[row][0..C) = softmax(logits)
__global__ __launch_bounds__(256) void head_out_kernel(const float* __restrict__ hid,
                                                       const float* __restrict__ wo,
                                                       const float* __restrict__ bo, int kind,
                                                       int C, int n_out, float* __restrict__ out,
                                                       const int* __restrict__ err) {
  __shared__ float logit[4][128];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= n_out) return;
  if (err && *err) {  // compact_kernel found lens that disagree with the ids
    for (int c = lane; c < (kind == 0 ? 1 : C); c += 64) out[(size_t)row * (kind == 0 ? 1 : C) + c] = NAN;
    return;
  }
  const float* h = hid + (size_t)row * AE_HIDDEN;
  float hv[12];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(h + c * 256 + lane * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) hv[4 * c + e] = a[e];
  }
  for (int o = 0; o < C; ++o) {
    const float* wr = wo + (size_t)o * AE_HIDDEN;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const floatx4 w = *reinterpret_cast<const floatx4*>(wr + c * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += w[e] * hv[4 * c + e];
    }
    acc = wave_sum(acc);
    if (lane == 0) logit[wave][o] = acc + bo[o];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  if (kind == 0) {
    if (lane == 0) out[row] = 1.f / (1.f + expf(-logit[wave][0]));
    return;
  }
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, logit[wave][c]);
  mx = wave_max(mx);
  float sm = 0.f;
  for (int c = lane; c < C; c += 64) sm += expf(logit[wave][c] - mx);
  sm = wave_sum(sm);
  for (int c = lane; c < C; c += 64) out[(size_t)row * C + c] = expf(logit[wave][c] - mx) / sm;
}

// Scatter compacted rows back to the padded layout (ae_encode): token t of sequence s, from
// column c = src_col[t], goes to out[s, c - row0] when row0 <= c < row0 + nrows (out [n, nrows, 768]).
__global__ __launch_bounds__(256) void scatter_rows_kernel(const float* __restrict__ x,
                                                           const int* __restrict__ cu,
                                                           const int* __restrict__ src_col, int n,
                                                           int row0, int nrows, int T,
                                                           float* __restrict__ out,
                                                           const int* __restrict__ err) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const int c = src_col[t] - row0;
  if (c < 0 || c >= nrows) return;
  const bool bad = err && *err;  // lens disagreed with the ids (compact_kernel): poison the rows
  int lo = 0, hi = n;  // find s with cu[s] <= t < cu[s+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cu[mid] <= t) lo = mid; else hi = mid;
  }
  const size_t dst = ((size_t)lo * nrows + c) * AE_HIDDEN;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int col = k * 256 + lane * 4;
    floatx4 v = *reinterpret_cast<const floatx4*>(x + (size_t)t * AE_HIDDEN + col);
    if (bad) v = floatx4{NAN, NAN, NAN, NAN};
    *reinterpret_cast<floatx4*>(out + dst + col) = v;
  }
}

// Query rows of ae_encode_rows: sequence s asks for its columns [row0[s], row0[s] + nrows); slot
// s·nrows + j gets the compacted row t of column row0[s] + j (qrow pre-filled with -1 by the
// caller: a column past lens or a pad the compaction dropped stays -1 and is never written out).
__global__ __launch_bounds__(256) void query_rows_kernel(const int* __restrict__ cu,
                                                         const int* __restrict__ src_col,
                                                         const int* __restrict__ row0, int n,
                                                         int nrows, int T, int* __restrict__ qrow) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  int lo = 0, hi = n;  // s with cu[s] <= t < cu[s+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cu[mid] <= t) lo = mid; else hi = mid;
  }
  const int c = src_col[t] - row0[lo];
  if (c >= 0 && c < nrows) qrow[lo * nrows + c] = t;
}

// xq[i] = x[qrow[i]] (a slot without a row copies its sequence's first row: computed, never stored)
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ x,
                                                          const int* __restrict__ qrow,
                                                          const int* __restrict__ cu, int qper,
                                                          int nq, float* __restrict__ xq) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= nq) return;
  const int t = qrow[i] >= 0 ? qrow[i] : cu[i / qper];
  const size_t src = (size_t)t * AE_HIDDEN;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    *reinterpret_cast<floatx4*>(xq + (size_t)i * AE_HIDDEN + col) =
        *reinterpret_cast<const floatx4*>(x + src + col);
  }
}

// out[i] = xq[i] for the slots that have a row (NaN when the lens disagreed with the ids)
__global__ __launch_bounds__(256) void scatter_query_kernel(const float* __restrict__ xq,
                                                            const int* __restrict__ qrow, int nq,
                                                            float* __restrict__ out,
                                                            const int* __restrict__ err) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= nq || qrow[i] < 0) return;
  const bool bad = err && *err;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = c * 256 + lane * 4;
    floatx4 v = *reinterpret_cast<const floatx4*>(xq + (size_t)i * AE_HIDDEN + col);
    if (bad) v = floatx4{NAN, NAN, NAN, NAN};
    *reinterpret_cast<floatx4*>(out + (size_t)i * AE_HIDDEN + col) = v;
  }
}

// Token negative log-likelihood of the MLM logits (CrossEntropyLoss(reduction='none') of
// utils.py:238-239): nll[t] = logsumexp(logits[t, :]) - logits[t, target[t]].  One 256-thread
// workgroup per row; the 50265-wide row is read once (online max / rescaled sum per lane).
__global__ __launch_bounds__(256) void nll_rows_kernel(const float* __restrict__ logits,
                                                       const int* __restrict__ target, int V,
                                                       float* __restrict__ nll) {
  __shared__ float sm_m[4], sm_s[4];
  const int t = blockIdx.x;
  const float* row = logits + (size_t)t * V;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m = -INFINITY, sum = 0.f;
  for (int c = tid; c < V; c += 256) {
    const float v = row[c];
    if (v > m) {
      sum = sum * expf(m - v) + 1.f;
      m = v;
    } else {
      sum += expf(v - m);
    }
  }
  // wave reduce (m, sum)
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(sum, o);
    const float mm = fmaxf(m, m2);
    sum = (m == -INFINITY ? 0.f : sum * expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * expf(m2 - mm));
    m = mm;
  }
  if (lane == 0) {
    sm_m[wave] = m;
    sm_s[wave] = sum;
  }
  __syncthreads();
  if (tid == 0) {
    float M = sm_m[0];
    for (int w = 1; w < 4; ++w) M = fmaxf(M, sm_m[w]);
    float S = 0.f;
    for (int w = 0; w < 4; ++w) S += sm_s[w] * expf(sm_m[w] - M);
    nll[t] = logf(S) + M - row[target[t]];
  }
}

// ---------------------------------------------------------------------------------------------
// GraphCodeDataset.__getitem__'s graph-guided attention mask (GraphCodeBERT/*/code/run.py
// TextDataset / utils.py:547-570) built from the compact features of ah_gcb_features_batch, one
// workgroup per query, the [L, L/32] bit image assembled in LDS:
//   rows < node_index: keys [0, node_index)                (code tokens see code tokens)
//   rows with id 0 / 2 (CLS / SEP): keys [0, max_length)
//   node k (row node_index + k), span (a, b): keys [a, b), and rows a..b-1 see key node_index + k
//   edge (k, t): row node_index + k sees key node_index + t (t + node_index < L)
__device__ __forceinline__ uint32_t range_bits(int w, int a, int b) {
  const int lo = max(a, 32 * w), hi = min(b, 32 * w + 32);
  if (lo >= hi) return 0u;
  const int n = hi - lo;
  return (n == 32 ? 0xffffffffu : ((1u << n) - 1u)) << (lo - 32 * w);
}

__global__ __launch_bounds__(256) void graph_mask_kernel(const int* __restrict__ ids,
                                                         const int* __restrict__ meta,
                                                         const int* __restrict__ spans,
                                                         const int* __restrict__ edges, int L,
                                                         int e_cap, uint32_t* __restrict__ bits) {
  extern __shared__ uint32_t gm_words[];
  const int q = blockIdx.x, W = L >> 5;
  const int ni = meta[4 * q], ml = meta[4 * q + 1], nn = meta[4 * q + 2], ne = meta[4 * q + 3];
  const int* qid = ids + (size_t)q * L;
  const int* qsp = spans + (size_t)q * L;
  for (int x = threadIdx.x; x < L * W; x += blockDim.x) {
    const int r = x / W, w = x - r * W;
    uint32_t v = 0;
    if (r < ni) v |= range_bits(w, 0, ni);
    const int id = qid[r];
    if (id == 0 || id == 2) v |= range_bits(w, 0, ml);
    if (r >= ni && r - ni < nn) {
      const int sp = qsp[r - ni];
      if (sp >= 0) v |= range_bits(w, sp & 0xffff, sp >> 16);
    }
    gm_words[x] = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nn; k += blockDim.x) {
    const int sp = qsp[k];
    if (sp < 0) continue;
    const int col = ni + k;
    for (int r = sp & 0xffff; r < (sp >> 16); ++r) atomicOr(&gm_words[r * W + (col >> 5)], 1u << (col & 31));
  }
  for (int j = threadIdx.x; j < ne; j += blockDim.x) {
    const int e = edges[(size_t)q * e_cap + j];
    const int row = ni + (e & 0xffff), col = ni + (e >> 16);
    if (col < L) atomicOr(&gm_words[row * W + (col >> 5)], 1u << (col & 31));
  }
  __syncthreads();
  uint32_t* out = bits + (size_t)q * L * W;
  for (int x = threadIdx.x; x < L * W; x += blockDim.x) out[x] = gm_words[x];
}

extern "C" {
hipError_t ae_launch_graph_mask(const int* ids, const int* meta, const int* spans,
                                const int* edges, int n, int L, int e_cap, uint32_t* bits,
                                hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const size_t lds = (size_t)L * (L / 32) * 4;
  if (lds > 65536)
    if (hipError_t e = ensure_dynamic_lds((const void*)graph_mask_kernel, lds); e != hipSuccess)
      return e;
  hipLaunchKernelGGL(graph_mask_kernel, dim3(n), dim3(256), lds, st, ids, meta, spans, edges, L,
                     e_cap, bits);
  return hipGetLastError();
}
hipError_t ae_launch_query_rows(const int* cu, const int* src_col, const int* row0, int n,
                                int nrows, int T, int* qrow, hipStream_t st) {
  if (n <= 0 || nrows <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(qrow, 0xff, (size_t)n * nrows * sizeof(int), st);
  if (e != hipSuccess || T <= 0) return e;
  hipLaunchKernelGGL(query_rows_kernel, dim3((T + 255) / 256), dim3(256), 0, st, cu, src_col, row0,
                     n, nrows, T, qrow);
  return hipGetLastError();
}
hipError_t ae_launch_gather_rows(const float* x, const int* qrow, const int* cu, int qper, int nq,
                                 float* xq, hipStream_t st) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((nq + 3) / 4), dim3(256), 0, st, x, qrow, cu, qper,
                     nq, xq);
  return hipGetLastError();
}
hipError_t ae_launch_scatter_query(const float* xq, const int* qrow, int nq, float* out,
                                   const int* err, hipStream_t st) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_query_kernel, dim3((nq + 3) / 4), dim3(256), 0, st, xq, qrow, nq, out,
                     err);
  return hipGetLastError();
}
hipError_t ae_launch_scatter_rows(const float* x, const int* cu, const int* src_col, int n,
                                  int row0, int nrows, int T, float* out, const int* err,
                                  hipStream_t st) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((T + 3) / 4), dim3(256), 0, st, x, cu, src_col, n,
                     row0, nrows, T, out, err);
  return hipGetLastError();
}
hipError_t ae_launch_compact(const int* ids, const int* pos, const int* cu, int n, int L, int pad,
                             int keep_all, int* tok_ids, int* tok_pos, int* src_col, int* err,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(compact_kernel, dim3(n), dim3(256), 0, st, ids, pos, cu, L, pad, keep_all,
                     tok_ids, tok_pos, src_col, err);
  return hipGetLastError();
}
hipError_t ae_launch_nll_rows(const float* logits, const int* target, int T, int V, float* nll,
                              hipStream_t st) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(nll_rows_kernel, dim3(T), dim3(256), 0, st, logits, target, V, nll);
  return hipGetLastError();
}
hipError_t ae_launch_embed_ln(const int* tok_ids, const int* tok_pos, const float* wemb,
                              const float* pemb, const float* temb, const float* g, const float* b,
                              float eps, int T, int max_pos, float* x, unsigned short* xp,
                              int np, const uint32_t* node_mask, int mask_L, const int* cu, int n,
                              hipStream_t st) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(embed_ln_kernel, dim3((T + 3) / 4), dim3(256), 0, st, tok_ids, tok_pos, wemb,
                     pemb, temb, g, b, eps, T, max_pos, x, xp, np, node_mask, mask_L, cu, n);
  return hipGetLastError();
}
hipError_t ae_launch_layernorm(const float* in, const float* g, const float* b, float eps, int T,
                               float* out, unsigned short* op, int np, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(layernorm_kernel, dim3((T + 3) / 4), dim3(256), 0, st, in, g, b, eps, T, out,
                     op, np);
  return hipGetLastError();
}
hipError_t ae_launch_gather_cls(const float* a, const float* b, const int* cu, int n, float* ac,
                                float* bc, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_cls_kernel, dim3((n + 3) / 4), dim3(256), 0, st, a, b, cu, n, ac, bc);
  return hipGetLastError();
}
hipError_t ae_launch_head_out(const float* hid, const float* wo, const float* bo, int kind, int C,
                              int n_out, float* out, const int* err, hipStream_t st) {
  if (n_out <= 0) return hipSuccess;
  if (C < 1 || C > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_out_kernel, dim3((n_out + 3) / 4), dim3(256), 0, st, hid, wo, bo, kind,
                     C, n_out, out, err);
  return hipGetLastError();
}
}
