// splice_topk.hip — HBM-bound integer/byte kernels of the query path.
//
// ae_splice: the mutant population builder.  The reference builds every mutant as TEXT
//   (python_parser/run_parser.py:218-266 get_example / get_example_batch) and re-tokenises it
//   (CodeXGLUE/Defect-detection/code/attacker.py:38-45: ' '.join(code.split()) -> tokenize ->
//   [:block-2] -> [CLS]+..+[SEP] -> pad 1).  Byte-level BPE pre-tokenisation is word-local after
//   the whitespace normalisation, so a mutant is exactly the concatenation of the token runs of its
//   whitespace-delimited words.  The host reduces each mutant to a sequence of word ids (an index
//   into the example's table of distinct words and their token runs); this kernel gathers the runs,
//   truncates to L-2, adds CLS/SEP and pads.  One workgroup per mutant; word starts by a
//   wave-ballot exclusive scan, then every lane copies its word's run.
//
// ae_topk: row-wise top-k over a vocabulary-wide logit row (torch.topk(., 60, -1) at
//   CodeXGLUE/Defect-detection/preprocess/get_substitutes.py:63).  One workgroup per row, exact
//   radix select on the order-preserving u32 key of the f32 (4 passes x 8 bits, LDS histograms),
//   then collection of the k winners (ties at the threshold taken in index order) and a rank sort
//   (value descending, index ascending).
//
// ae_cosine_rank: sum over a sub-word span of CosineSimilarity(dim=1, eps) / span
//   (get_substitutes.py:75,108).  One wave per (candidate, position) row pair.
#include "common.h"

// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void splice_kernel(const int* __restrict__ word_tok,
                                                     const int* __restrict__ word_off,
                                                     const int* __restrict__ mut_words,
                                                     const int* __restrict__ mut_off, int L,
                                                     int cls_id, int sep_id, int pad_id,
                                                     int* __restrict__ ids_out,
                                                     int* __restrict__ lens_out) {
  __shared__ int wave_tot[4];
  __shared__ int carry_s, pads_s;
  const int m = blockIdx.x;
  const int w0 = mut_off[m], nw = mut_off[m + 1] - w0;
  int* out = ids_out + (size_t)m * L;
  const int cap = L - 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry_s = pads_s = 0;
  __syncthreads();
  int pads = 0;  // pad ids inside the kept tokens (a literal "<pad>" in the source text)
  for (int c0 = 0; c0 < nw; c0 += 256) {
    const int c = c0 + tid;
    int wlen = 0, wstart = 0;
    if (c < nw) {
      const int w = mut_words[w0 + c];
      wstart = word_off[w];
      wlen = word_off[w + 1] - wstart;
    }
    // exclusive scan of wlen across the workgroup (wave inclusive scan by shuffles)
    int incl = wlen;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wave_tot[wave] = incl;
    __syncthreads();
    int pos = carry_s + incl - wlen;
    for (int w = 0; w < wave; ++w) pos += wave_tot[w];
    for (int j = 0; j < wlen; ++j) {
      const int p = pos + j;
      if (p < cap) {
        const int id = word_tok[wstart + j];
        out[1 + p] = id;
        pads += id == pad_id;
      }
    }
    __syncthreads();
    if (tid == 0) carry_s += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
    __syncthreads();
  }
  if (pads) atomicAdd(&pads_s, pads);
  __syncthreads();
  const int total = carry_s;
  const int ntok = total < cap ? total : cap;
  for (int p = tid; p < L; p += 256) {
    if (p == 0) out[0] = cls_id;
    else if (p == ntok + 1) out[p] = sep_id;
    else if (p > ntok + 1) out[p] = pad_id;
  }
  if (tid == 0) lens_out[m] = ntok + 2 - pads_s;  // non-pad count (ae_score's lens)
}

// --------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ x, int cols, int k,
                                                   float* __restrict__ vals,
                                                   int* __restrict__ idx) {
  __shared__ unsigned int hist[256];
  __shared__ uint32_t s_prefix, s_mask;
  __shared__ int s_need;
  __shared__ int s_cnt_gt, s_tie_taken;
  __shared__ uint32_t cand_key[256];
  __shared__ int cand_idx[256];
  __shared__ int wave_tot[4];
  const int row = blockIdx.x;
  const float* xr = x + (size_t)row * cols;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) { s_prefix = 0u; s_mask = 0u; s_need = k; }
  __syncthreads();
  // radix select: find the k-th largest key
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0u;
    __syncthreads();
    const uint32_t prefix = s_prefix, pmask = s_mask;
    for (int c = tid; c < cols; c += 256) {
      const uint32_t key = f2key(xr[c]);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int need = s_need;
      int b = 255;
      for (; b >= 0; --b) {
        const int h = (int)hist[b];
        if (h >= need) break;
        need -= h;
      }
      s_prefix = prefix | ((uint32_t)b << shift);
      s_mask = pmask | (255u << shift);
      s_need = need;  // how many of the elements equal to the final key we still need
    }
    __syncthreads();
  }
  const uint32_t thr = s_prefix;
  const int need_eq = s_need;
  // collect: all keys > thr (exactly k - need_eq of them), then the first need_eq ties by index
  if (tid == 0) { s_cnt_gt = 0; s_tie_taken = 0; }
  __syncthreads();
  for (int c = tid; c < cols; c += 256) {
    const uint32_t key = f2key(xr[c]);
    if (key > thr) {
      const int p = atomicAdd(&s_cnt_gt, 1);
      cand_key[p] = key;
      cand_idx[p] = c;
    }
  }
  __syncthreads();
  const int n_gt = s_cnt_gt;
  for (int c0 = 0; c0 < cols && s_tie_taken < need_eq; c0 += 256) {
    const int c = c0 + tid;
    const int eq = (c < cols) && (f2key(xr[c]) == thr);
    const unsigned long long bal = __ballot(eq);
    if (lane == 0) wave_tot[wave] = __popcll(bal);
    __syncthreads();
    int before = s_tie_taken + __popcll(bal & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; ++w) before += wave_tot[w];
    if (eq && before < need_eq) {
      cand_key[n_gt + before] = thr;
      cand_idx[n_gt + before] = c;
    }
    __syncthreads();
    if (tid == 0) s_tie_taken += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
    __syncthreads();
  }
  // rank sort of the k candidates (value desc, index asc)
  if (tid < k) {
    const uint32_t mk = cand_key[tid];
    const int mi = cand_idx[tid];
    int rank = 0;
    for (int j = 0; j < k; ++j) {
      const uint32_t ok = cand_key[j];
      const int oi = cand_idx[j];
      rank += (ok > mk) || (ok == mk && oi < mi);
    }
    vals[(size_t)row * k + rank] = key2f(mk);
    idx[(size_t)row * k + rank] = mi;
  }
}

// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cosine_rank_kernel(const float* __restrict__ ref,
                                                          const float* __restrict__ cand, int n,
                                                          int span, int hidden, float eps,
                                                          float* __restrict__ sims) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  float total = 0.f;
  for (int t = 0; t < span; ++t) {
    const float* a = ref + (size_t)t * hidden;
    const float* b = cand + ((size_t)i * span + t) * hidden;
    float d = 0.f, na = 0.f, nb = 0.f;
    for (int c = lane; c < hidden; c += 64) {
      const float x = a[c], y = b[c];
      d += x * y;
      na += x * x;
      nb += y * y;
    }
    d = wave_sum(d);
    na = wave_sum(na);
    nb = wave_sum(nb);
    total += d / (fmaxf(sqrtf(na), eps) * fmaxf(sqrtf(nb), eps));
  }
  if (lane == 0) sims[i] = total / (float)span;
}

extern "C" {
hipError_t ae_launch_splice(const int* word_tok, const int* word_off, const int* mut_words,
                            const int* mut_off, int n_mut, int L, int cls_id, int sep_id,
                            int pad_id, int* ids_out, int* lens_out, hipStream_t st) {
  if (n_mut <= 0) return hipSuccess;
  hipLaunchKernelGGL(splice_kernel, dim3(n_mut), dim3(256), 0, st, word_tok, word_off, mut_words,
                     mut_off, L, cls_id, sep_id, pad_id, ids_out, lens_out);
  return hipGetLastError();
}
hipError_t ae_launch_topk(const float* x, int rows, int cols, int k, float* vals, int* idx,
                          hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(topk_kernel, dim3(rows), dim3(256), 0, st, x, cols, k, vals, idx);
  return hipGetLastError();
}
hipError_t ae_launch_cosine_rank(const float* ref, const float* cand, int n, int span, int hidden,
                                 float eps, float* sims, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cosine_rank_kernel, dim3((n + 3) / 4), dim3(256), 0, st, ref, cand, n, span,
                     hidden, eps, sims);
  return hipGetLastError();
}
}
