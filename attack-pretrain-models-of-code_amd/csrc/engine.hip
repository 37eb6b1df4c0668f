// engine.hip — host side of the C-ABI (include/alert_engine.h): weight residency, workspaces and
// the launch sequence of one victim query batch.
//
// One ae_score call = the whole of Model.get_results' device work for a batch
// (CodeXGLUE/Defect-detection/code/model.py:36-59): pad compaction -> embedding+LN ->
// 12 x [QKV GEMM -> fused attention -> O GEMM(+res) -> LN -> FFN1 GEMM(+GELU) -> FFN2 GEMM(+res)
// -> LN] -> task head.  The last layer only needs the CLS row of every sequence (the heads read
// features[:, 0, :]), so after its K/V are produced its attention, O-projection, LayerNorms and
// FFN run on the n CLS rows only.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/alert_engine.h"

extern "C" {
hipError_t ae_launch_gemm_f32(const float*, const float*, const float*, const float*, float*, int,
                              int, int, int, int, int, int, const int*, hipStream_t, float*, long);
hipError_t ae_launch_gemm_x3(const float*, const unsigned short*, const unsigned short*,
                             const float*, const float*, float*, int, int, int, int, int, int,
                             int, int, hipStream_t, float*, long);
hipError_t ae_launch_attention_f32(const float*, float*, const int*, const int*, int, int, int,
                                   const uint32_t*, int, hipStream_t);
hipError_t ae_launch_attention_pp(const unsigned short*, float*, unsigned short*, const int*,
                                  const int*, int, int, int, const uint32_t*, int, int, hipStream_t);
#ifdef AE_TOOLS
hipError_t ae_bench_attention_pp(const unsigned short*, float*, unsigned short*, const int*,
                                 const int*, int, int, int, const uint32_t*, int, int, int,
                                 hipStream_t);
hipError_t ae_bench_gemm_packed_fold(const unsigned short*, const unsigned short*, const float*,
                                     const float*, const uint64_t*, float, unsigned short*, int,
                                     int, int, int, int, const float*, int, int, hipStream_t);
hipError_t ae_bench_gemm_packed_res_stats(const unsigned short*, const unsigned short*,
                                          const float*, const float*, const uint64_t*,
                                          const float*, const float*, float, float*,
                                          unsigned short*, uint64_t*, int, int, int, int,
                                          const float*, int, int, hipStream_t);
#endif
hipError_t ae_launch_gemm_packed(const unsigned short*, const unsigned short*, const float*,
                                 const float*, float*, unsigned short*, int, int, int, int, int,
                                 hipStream_t);
hipError_t ae_launch_gemm_packed_fold(const unsigned short*, const unsigned short*, const float*,
                                      const float*, const uint64_t*, float, unsigned short*, int,
                                      int, int, int, int, const float*, hipStream_t);
hipError_t ae_launch_gemm_packed_res_stats(const unsigned short*, const unsigned short*,
                                           const float*, const float*, const uint64_t*,
                                           const float*, const float*, float, float*,
                                           unsigned short*, uint64_t*, int, int, int, int,
                                           const float*, hipStream_t);
hipError_t ae_launch_compact(const int*, const int*, const int*, int, int, int, int, int*, int*,
                             int*, int*, hipStream_t);
hipError_t ae_launch_embed_ln(const int*, const int*, const float*, const float*, const float*,
                              const float*, const float*, float, int, int, float*, unsigned short*,
                              int, const uint32_t*, int, const int*, int, hipStream_t);
hipError_t ae_launch_layernorm(const float*, const float*, const float*, float, int, float*,
                               unsigned short*, int, hipStream_t);
hipError_t ae_launch_gather_cls(const float*, const float*, const int*, int, float*, float*,
                                hipStream_t);
hipError_t ae_launch_head_out(const float*, const float*, const float*, int, int, int, float*,
                              const int*, hipStream_t);
hipError_t ae_launch_splice(const int*, const int*, const int*, const int*, int, int, int, int,
                            int, int*, int*, hipStream_t);
hipError_t ae_launch_topk(const float*, int, int, int, float*, int*, hipStream_t);
hipError_t ae_launch_cosine_rank(const float*, const float*, int, int, int, float, float*,
                                 hipStream_t);
hipError_t ae_launch_scatter_rows(const float*, const int*, const int*, int, int, int, int,
                                  float*, const int*, hipStream_t);
hipError_t ae_launch_nll_rows(const float*, const int*, int, int, float*, hipStream_t);
hipError_t ae_launch_graph_mask(const int*, const int*, const int*, const int*, int, int, int,
                                uint32_t*, hipStream_t);
long ae_cls_attention_part_floats(long, int, int);
hipError_t ae_launch_cls_attention(const float*, const float*, const float*, const float*,
                                   const float*, const int*, int, int, int, const uint32_t*, int,
                                   float, float*, float*, float*, float*, int*, hipStream_t);
hipError_t ae_launch_layernorm_stats(const float*, const uint64_t*, const float*, const float*,
                                     float, int, float*, hipStream_t);
hipError_t ae_launch_query_rows(const int*, const int*, const int*, int, int, int, int*,
                                hipStream_t);
hipError_t ae_launch_gather_rows(const float*, const int*, const int*, int, int, float*,
                                 hipStream_t);
hipError_t ae_launch_scatter_query(const float*, const int*, int, float*, const int*, hipStream_t);
}

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPC(x)                                                                         \
  do {                                                                                  \
    hipError_t _e = (x);                                                                \
    if (_e != hipSuccess)                                                               \
      return fail(AE_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e));          \
  } while (0)

enum { EPI_BIAS = 0, EPI_BIAS_GELU = 1, EPI_BIAS_RESIDUAL = 2, EPI_BIAS_TANH = 3, EPI_BIAS_PACKED = 4 };

struct LayerW {
  float *wqkv, *bqkv, *wo, *bo, *ln1g, *ln1b, *w1, *b1, *w2, *b2, *ln2g, *ln2b;
  // split-bf16 planes (AE_PREC_BF16: hi only; AE_PREC_F32X3: hi + lo)
  unsigned short *wqkv_h, *wo_h, *w1_h, *w2_h;
  unsigned short *wqkv_l, *wo_l, *w1_l, *w2_l;
  // packed planes for gemm_planes.hip (F32X3: [N][K/32][hi 32 | lo 32]; BF16: the hi plane).
  // wqkv_p of layers >= 1 and every w1_p carry the preceding LayerNorm's gain folded in
  // (gemm_planes.hip FoldArgs): W' = W·diag(g), with s = row sums of W' (as its planes hold it)
  // and the folded bias bias + W·b
  unsigned short *wqkv_p, *wo_p, *w1_p, *w2_p;
  float *sqkv, *bqkv_f, *s1, *b1_f;
  // plane shift (gemm_planes.hip FoldArgs): kappa of the O-projection / FFN2 outputs (their bias +
  // their residual's LayerNorm shift) and the accumulator starts kc = kappa·W'^T of FFN1 / QKV
  float *kap_o, *kap_f, *kc1, *kcqkv;
};

struct ProfRec {
  hipEvent_t a, b;
  double flop;
};
}  // namespace

struct ae_engine {
  ae_config cfg;
  int device = 0;
  std::vector<void*> allocs;
  float *wemb = nullptr, *pemb = nullptr, *temb = nullptr, *eg = nullptr, *eb = nullptr;
  std::vector<LayerW> layers;
  float *hd_w = nullptr, *hd_b = nullptr, *ho_w = nullptr, *ho_b = nullptr;
  // MLM head
  float *lm_dw = nullptr, *lm_db = nullptr, *lm_lg = nullptr, *lm_lb = nullptr, *lm_bias = nullptr;
  // workspaces
  size_t cap_T = 0, cap_n = 0;
  float *x = nullptr, *qkv = nullptr, *ctx = nullptr, *tmp = nullptr, *h1 = nullptr;
  float *xc = nullptr, *cc = nullptr, *tc = nullptr, *hc = nullptr;
  // packed bf16 activation planes of the split-precision path (gemm_planes.hip layout, np planes):
  // LN output, attention context, FFN1 output.  Allocated only when `planes` is on.
  unsigned short *xp = nullptr, *cp = nullptr, *hp = nullptr;
  // per-tile row statistics [T][4] of the pre-LayerNorm rows (gemm_planes.hip PK_EPI_RES_STATS):
  // lnst of the FFN2 output (read by the next layer's QKV and O-projection), lnst2 of the
  // O-projection output (read by FFN1 and FFN2)
  uint64_t* lnst = nullptr;
  uint64_t* lnst2 = nullptr;
  bool planes = false;
  int np = 1;
  // last-layer CLS attention with W_k absorbed into the query (cls_attention.hip): per-sequence
  // u = W_k^T q and p-weighted row sums [n][12][768], per-64-key-chunk partial records
  // (AE_CLS_ABSORB=0 at engine creation: the full-T QKV GEMM + one-query attention instead)
  bool cls_absorb = true;
  float *cls_u = nullptr, *cls_y = nullptr, *cls_part = nullptr;
  size_t cap_cls_part = 0;
  int *tok_ids = nullptr, *tok_pos = nullptr, *src_col = nullptr, *cu = nullptr, *one = nullptr;
  int* err = nullptr;  // device flag: some row's lens disagreed with its ids (compact_kernel)
  float* logits = nullptr;
  // split-K partials of the small GEMMs (last-layer CLS rows, classifier head): 64 MB
  static constexpr long kSplitKFloats = 16L << 20;
  float* skws = nullptr;
  size_t cap_logits = 0;
  int* pinned_cu = nullptr;
  size_t cap_pinned = 0;
  hipEvent_t pinned_ready = nullptr;
  // ae_encode_rows: per-sequence first column of the row window (host pinned -> device) and the
  // compacted row of every query slot [n][nrows] (-1: no row)
  int *pinned_r0 = nullptr, *row0_dev = nullptr, *qrow = nullptr;
  size_t cap_r0 = 0, cap_q = 0;
  hipEvent_t r0_ready = nullptr;
  // two-stream encoder (split-precision modes unless cfg.streams = AE_STREAMS_ONE; the tools
  // library's AE_SPLIT_STREAMS=0 too): the batch's sequences in two halves, each half's layers on
  // its own stream, the second half one kernel behind, so one half's memory-bound phases (GEMM
  // epilogue bursts) and tile-quantisation tails can run beside the other half's MFMA-bound main
  // loops; every row's arithmetic is the one-stream form's (layer_rows)
  static constexpr int kMaxParts = 4;
  bool split = false;
  int split_parts = 2;  // parts of the batch, each on its own stream (AE_SPLIT_PARTS, 2..4)
  int split_lag = 1;    // a part starts after this many of the previous part's layer-0 kernels
  // experiments (AE_ATTN_VARIANT, tools/engine_ab.py): an attention_pp loop variant other than the
  // production one for the unmasked launches (0 = production)
  int attn_variant = 0;
  // experiments (AE_GEMM_P2, tools/engine_ab.py): bit 1 QKV, 2 FFN1, 4 O-projection, 8 FFN2 on
  // the two-per-CU 128 x 192 kernel (gemm_p2_kernel) instead of the production launch
  int gemm_p2 = 0;
  hipStream_t sts[kMaxParts] = {};  // sts[0] unused: part 0 runs on the caller's stream
  hipEvent_t ev_fork = nullptr, ev_lag[kMaxParts] = {}, ev_join[kMaxParts] = {};
  // profiling: event pairs are created when profiling is switched on (never inside the timed
  // launches) and recycled by ae_kernel_time
  int prof_kind = -1;
  std::vector<ProfRec> prof;
  std::vector<ProfRec> prof_pool;
};

namespace {
int dev_alloc(ae_engine* e, void** p, size_t bytes) {
  hipError_t r = hipMalloc(p, bytes ? bytes : 16);
  if (r != hipSuccess) return fail(AE_ENOMEM, "hipMalloc " + std::to_string(bytes) + " B failed");
  e->allocs.push_back(*p);
  return AE_OK;
}
void dev_free(ae_engine* e, void* p) {
  if (!p) return;
  for (auto& a : e->allocs)
    if (a == p) { a = nullptr; }
  (void)hipFree(p);
}

struct WeightTable {
  std::map<std::string, const ae_weight_view*> by_name;
  const ae_weight_view* get(const std::string& n) const {
    auto it = by_name.find(n);
    return it == by_name.end() ? nullptr : it->second;
  }
};

int upload(ae_engine* e, const WeightTable& wt, const std::string& name, int64_t numel,
           float** dst) {
  const ae_weight_view* v = wt.get(name);
  if (!v) return fail(AE_ENOENT, "missing weight " + name);
  if (v->numel != numel)
    return fail(AE_EINVAL, "weight " + name + " has " + std::to_string(v->numel) +
                               " elements, expected " + std::to_string(numel));
  int rc = dev_alloc(e, (void**)dst, numel * sizeof(float));
  if (rc) return rc;
  HIPC(hipMemcpy(*dst, v->data, numel * sizeof(float), hipMemcpyHostToDevice));
  return AE_OK;
}

unsigned short host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

float host_bf2f(unsigned short b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// W = hi + lo with hi = bf16(W), lo = bf16(W - hi) (round-to-nearest-even); lo only if dst_lo
int upload_split(ae_engine* e, const float* host, size_t n, unsigned short** dst_hi,
                 unsigned short** dst_lo) {
  std::vector<unsigned short> h(n), l(dst_lo ? n : 0);
  for (size_t i = 0; i < n; ++i) {
    h[i] = host_f2bf(host[i]);
    if (dst_lo) l[i] = host_f2bf(host[i] - host_bf2f(h[i]));
  }
  int rc = dev_alloc(e, (void**)dst_hi, n * 2);
  if (rc) return rc;
  HIPC(hipMemcpy(*dst_hi, h.data(), n * 2, hipMemcpyHostToDevice));
  if (dst_lo) {
    if ((rc = dev_alloc(e, (void**)dst_lo, n * 2))) return rc;
    HIPC(hipMemcpy(*dst_lo, l.data(), n * 2, hipMemcpyHostToDevice));
  }
  return AE_OK;
}

// Packed planes of gemm_planes.hip for np = 2: row r = K/32 blocks of [hi(32) | lo(32)].
int upload_packed(ae_engine* e, const float* host, size_t rows, size_t K, unsigned short** dst) {
  if (K % 32) return fail(AE_EINVAL, "packed planes need K % 32 == 0");
  std::vector<unsigned short> pk(rows * K * 2);
  for (size_t r = 0; r < rows; ++r)
    for (size_t k = 0; k < K; ++k) {
      const float v = host[r * K + k];
      const unsigned short h = host_f2bf(v);
      unsigned short* blk = pk.data() + r * 2 * K + (k / 32) * 64;
      blk[k % 32] = h;
      blk[32 + k % 32] = host_f2bf(v - host_bf2f(h));
    }
  int rc = dev_alloc(e, (void**)dst, pk.size() * 2);
  if (rc) return rc;
  HIPC(hipMemcpy(*dst, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
  return AE_OK;
}

// A LayerNorm (gain g, shift b over the K inputs) folded into the packed-plane weight of the GEMM
// that consumes its output (gemm_planes.hip FoldArgs): uploads the planes of W' = W·diag(g)
// (np 2: hi | lo, np 1: hi), s[n] = sum_k W'[n][k] as those planes hold it, and the folded bias
// bias[n] + sum_k W[n][k]·b[k] (double sums).
// With kappa (the producer's plane shift, [K]), also kc[n] = sum_k kappa[k]·W'[n][k] as the planes
// hold W' (double sums): the consumer's accumulator start.
int upload_folded(ae_engine* e, const float* W, const float* bias, const float* g, const float* b,
                  size_t rows, size_t K, int np, unsigned short** planes, float** s_dev,
                  float** bias_dev, const float* kappa = nullptr, float** kc_dev = nullptr) {
  std::vector<float> wf(rows * K), sv(rows), bv(rows), kv(rows);
  for (size_t r = 0; r < rows; ++r) {
    double ss = 0.0, bb = bias[r], kk = 0.0;
    for (size_t k = 0; k < K; ++k) {
      const float x = W[r * K + k] * g[k];
      wf[r * K + k] = x;
      const float h = host_bf2f(host_f2bf(x));
      const double held = (double)h + (np == 2 ? (double)host_bf2f(host_f2bf(x - h)) : 0.0);
      ss += held;
      if (kappa) kk += (double)kappa[k] * held;
      bb += (double)W[r * K + k] * (double)b[k];
    }
    sv[r] = (float)ss;
    bv[r] = (float)bb;
    kv[r] = (float)kk;
  }
  int rc = np == 2 ? upload_packed(e, wf.data(), rows, K, planes)
                   : upload_split(e, wf.data(), wf.size(), planes, nullptr);
  if (rc) return rc;
  if ((rc = dev_alloc(e, (void**)s_dev, rows * 4)) || (rc = dev_alloc(e, (void**)bias_dev, rows * 4)))
    return rc;
  HIPC(hipMemcpy(*s_dev, sv.data(), rows * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(*bias_dev, bv.data(), rows * 4, hipMemcpyHostToDevice));
  if (kappa && kc_dev) {
    if ((rc = dev_alloc(e, (void**)kc_dev, rows * 4))) return rc;
    HIPC(hipMemcpy(*kc_dev, kv.data(), rows * 4, hipMemcpyHostToDevice));
  }
  return AE_OK;
}

// kappa = bias + beta (the per-column constant part of a residual add whose residual is a
// LayerNorm output with shift beta), uploaded; host copy in out
int upload_kappa(ae_engine* e, const float* bias, const float* beta, size_t n,
                 std::vector<float>& out, float** dev) {
  out.resize(n);
  for (size_t i = 0; i < n; ++i) out[i] = bias[i] + beta[i];
  int rc = dev_alloc(e, (void**)dev, n * 4);
  if (rc) return rc;
  HIPC(hipMemcpy(*dev, out.data(), n * 4, hipMemcpyHostToDevice));
  return AE_OK;
}

int ensure_workspace(ae_engine* e, size_t T, size_t n) {
  const size_t H = e->cfg.hidden, F = e->cfg.ffn;
  if (T > e->cap_T) {
    size_t nt = T + T / 4 + 128;
    HIPC(hipDeviceSynchronize());
    for (void* p : {(void*)e->x, (void*)e->qkv, (void*)e->ctx, (void*)e->tmp, (void*)e->h1,
                    (void*)e->tok_ids, (void*)e->tok_pos, (void*)e->src_col, (void*)e->xp,
                    (void*)e->cp, (void*)e->hp, (void*)e->lnst, (void*)e->lnst2})
      dev_free(e, p);
    e->xp = e->cp = e->hp = nullptr;
    e->lnst = e->lnst2 = nullptr;
    int rc = 0;
    if ((rc = dev_alloc(e, (void**)&e->x, nt * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->qkv, nt * 3 * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->ctx, nt * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->tmp, nt * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->h1, nt * F * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->tok_ids, nt * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->tok_pos, nt * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->src_col, nt * 4))) return rc;
    if (e->planes) {
      if ((rc = dev_alloc(e, (void**)&e->xp, nt * H * 2 * e->np))) return rc;
      if ((rc = dev_alloc(e, (void**)&e->cp, nt * H * 2 * e->np))) return rc;
      if ((rc = dev_alloc(e, (void**)&e->hp, nt * F * 2 * e->np))) return rc;
      const size_t blocks = (nt + 255) / 256;
      if ((rc = dev_alloc(e, (void**)&e->lnst, blocks * 256 * 4 * 8))) return rc;
      if ((rc = dev_alloc(e, (void**)&e->lnst2, blocks * 256 * 4 * 8))) return rc;
    }
    e->cap_T = nt;
  }
  if (n + 1 > e->cap_n) {
    size_t nn = n + n / 4 + 64;
    HIPC(hipDeviceSynchronize());
    for (void* p : {(void*)e->xc, (void*)e->cc, (void*)e->tc, (void*)e->hc, (void*)e->cu,
                    (void*)e->cls_u, (void*)e->cls_y})
      dev_free(e, p);
    int rc = 0;
    if ((rc = dev_alloc(e, (void**)&e->cls_u, nn * 12 * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->cls_y, nn * 12 * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->xc, nn * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->cc, nn * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->tc, nn * H * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->hc, nn * F * 4))) return rc;
    if ((rc = dev_alloc(e, (void**)&e->cu, (nn + 1) * 4))) return rc;
    e->cap_n = nn;
    if (e->pinned_cu) (void)hipHostFree(e->pinned_cu);
    HIPC(hipHostMalloc((void**)&e->pinned_cu, (nn + 1) * 4, hipHostMallocDefault));
    e->cap_pinned = nn + 1;
  }
  return AE_OK;
}

// Partial records of the last layer's CLS attention for T rows of n sequences.
int ensure_cls_part(ae_engine* e, int64_t T, int n, int qper) {
  const size_t need = (size_t)ae_cls_attention_part_floats((long)T, n, qper);
  if (need <= e->cap_cls_part) return AE_OK;
  HIPC(hipDeviceSynchronize());
  dev_free(e, e->cls_part);
  e->cls_part = nullptr;
  const size_t cap = need + need / 4;
  int rc = dev_alloc(e, (void**)&e->cls_part, cap * 4);
  if (rc) return rc;
  e->cap_cls_part = cap;
  return AE_OK;
}

// Upload cu_seqlens computed on the host; returns T.
int upload_cu(ae_engine* e, const int32_t* lens, int n, int L, hipStream_t st, int64_t* T_out) {
  // the previous upload must have left the pinned buffer
  HIPC(hipEventSynchronize(e->pinned_ready));
  int64_t T = 0;
  e->pinned_cu[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (lens[i] < 1 || lens[i] > L)
      return fail(AE_EINVAL, "lens[" + std::to_string(i) + "]=" + std::to_string(lens[i]) +
                                 " outside [1, L]");
    T += lens[i];
    e->pinned_cu[i + 1] = (int)T;
  }
  HIPC(hipMemcpyAsync(e->cu, e->pinned_cu, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, st));
  HIPC(hipEventRecord(e->pinned_ready, st));
  *T_out = T;
  return AE_OK;
}

// Profiled launch wrapper
struct Prof {
  ae_engine* e;
  hipStream_t st;
  bool on;
  ProfRec rec;
  Prof(ae_engine* e_, hipStream_t s, bool enabled, double flop) : e(e_), st(s), on(enabled) {
    if (on) {
      if (!e->prof_pool.empty()) {
        rec = e->prof_pool.back();
        e->prof_pool.pop_back();
      } else {  // pool exhausted (more launches than ae_set_profiling reserved)
        (void)hipEventCreate(&rec.a);
        (void)hipEventCreate(&rec.b);
      }
      rec.flop = flop;
      (void)hipEventRecord(rec.a, st);
    }
  }
  ~Prof() {
    if (on) {
      (void)hipEventRecord(rec.b, st);
      e->prof.push_back(rec);
    }
  }
};

int gemm(ae_engine* e, const float* A, const float* W, const unsigned short* Wh,
         const unsigned short* Wl, const float* bias, const float* R, float* C, int M, int N, int K,
         int epi, hipStream_t st, bool is_ffn1) {
  const bool prof = (e->prof_kind == AE_KIND_GEMM_ANY) || (e->prof_kind == AE_KIND_GEMM_FFN1 && is_ffn1);
  Prof p(e, st, prof, 2.0 * M * N * K);
  if (e->cfg.precision != AE_PREC_FP32 && Wh) {
    const int terms = e->cfg.precision == AE_PREC_F32X3 ? 3 : 1;
    HIPC(ae_launch_gemm_x3(A, Wh, Wl, bias, R, C, M, N, K, K, K, N, epi, terms, st, e->skws,
                           ae_engine::kSplitKFloats));
  } else {
    HIPC(ae_launch_gemm_f32(A, W, bias, R, C, M, N, K, K, K, N, epi, nullptr, st, e->skws,
                            ae_engine::kSplitKFloats));
  }
  return AE_OK;
}

// Packed-plane GEMM of the split-precision path: packed bf16 planes in, f32 (or packed planes for
// the GELU epilogue) out.
int gemm_pk(ae_engine* e, const unsigned short* A, const unsigned short* Wp, const float* bias,
            const float* R, float* C, unsigned short* Cp, int M, int N, int K, int epi,
            hipStream_t st, bool is_ffn1) {
  const bool prof = (e->prof_kind == AE_KIND_GEMM_ANY) || (e->prof_kind == AE_KIND_GEMM_FFN1 && is_ffn1);
  Prof p(e, st, prof, 2.0 * M * N * K);
  HIPC(ae_launch_gemm_packed(A, Wp, bias, R, C, Cp, M, N, K, epi, e->np, st));
  return AE_OK;
}

// attention over packed planes: the production loop, or an experiment variant (unmasked launches)
hipError_t attention_pp(ae_engine* e, const unsigned short* qkvp, float* out, unsigned short* op,
                        const int* cu, const int* q_rows, int max_q, int n, int heads,
                        const uint32_t* mask, int mask_L, int np, hipStream_t st) {
#ifdef AE_TOOLS
  if (e->attn_variant && !mask)
    return ae_bench_attention_pp(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np,
                                 e->attn_variant, st);
#endif
  return ae_launch_attention_pp(qkvp, out, op, cu, q_rows, max_q, n, heads, mask, mask_L, np, st);
}

// One full encoder layer li of the split-precision path over the token rows [t0, t0 + M) of the
// sequences [s0, s0 + ns) on stream st, with both LayerNorms folded into the GEMMs that follow
// them (gemm_planes.hip FoldArgs): between layers the rows stay pre-LayerNorm (v in e->tmp, its
// planes in e->xp, its tile statistics in e->lnst / e->lnst2), and
//   QKV   = fold(v, LN2 of layer li-1)                    (layer 0: the embedding LN's x as it is)
//   v     = ctx·Wo^T + bo + LN2_{li-1}(v)                 (+ tile statistics -> lnst2)
//   h     = GELU(fold(v, LN1 of layer li))
//   v     = h·W2^T + b2 + LN1_li(v)                        (+ tile statistics -> lnst)
// no LayerNorm pass over the rows, and no exchange between workgroups.  last: the encoder's last
// full layer, whose output LN2_li(v) is written to e->x (f32) for the CLS path / MLM head.
// Every row's arithmetic is independent of the part boundaries and of M.
int layer_rows(ae_engine* e, int li, int64_t t0, int M, int s0, int ns, int max_len,
               const uint32_t* mask_bits, int L, hipStream_t st, bool last,
               hipEvent_t mark = nullptr, int mark_after = 1) {
  const int H = e->cfg.hidden, F = e->cfg.ffn, np = e->np;
  const LayerW& w = e->layers[li];
  const LayerW* prev = li > 0 ? &e->layers[li - 1] : nullptr;
  const float eps = e->cfg.ln_eps;
  unsigned short* qkvp = reinterpret_cast<unsigned short*>(e->qkv) + t0 * 3 * H * np;
  unsigned short* xp = e->xp + t0 * H * np;
  unsigned short* cp = e->cp + t0 * H * np;
  unsigned short* hp = e->hp + t0 * F * np;
  float* v = e->tmp + t0 * H;
  uint64_t* sa = e->lnst + t0 * 4;   // FFN2 output statistics
  uint64_t* sb = e->lnst2 + t0 * 4;  // O-projection output statistics
  int k = 0;
  // records `mark` on st after the mark_after-th kernel of the layer (the second stream's lag)
  auto done = [&]() -> int {
    if (mark && ++k == mark_after) HIPC(hipEventRecord(mark, st));
    return AE_OK;
  };
  const bool prof = e->prof_kind == AE_KIND_GEMM_ANY;
  {
    Prof p(e, st, prof, 2.0 * M * 3 * H * H);
#ifdef AE_TOOLS
    if (prev && (e->gemm_p2 & 1))
      HIPC(ae_bench_gemm_packed_fold(xp, w.wqkv_p, w.bqkv_f, w.sqkv, sa, eps, qkvp, M, 3 * H, H, 0,
                                     np, w.kcqkv, 1, 0, st));
    else
#endif
    if (prev)
      HIPC(ae_launch_gemm_packed_fold(xp, w.wqkv_p, w.bqkv_f, w.sqkv, sa, eps, qkvp, M, 3 * H, H,
                                      0, np, w.kcqkv, st));
    else
      HIPC(ae_launch_gemm_packed(xp, w.wqkv_p, w.bqkv, nullptr, nullptr, qkvp, M, 3 * H, H,
                                 EPI_BIAS_PACKED, np, st));
  }
  if (int rc = done()) return rc;
  {
    Prof p(e, st, e->prof_kind == AE_KIND_ATTENTION, 0.0);
    HIPC(attention_pp(e, reinterpret_cast<unsigned short*>(e->qkv), e->ctx, e->cp, e->cu + s0,
                      nullptr, max_len, ns, e->cfg.heads,
                      mask_bits ? mask_bits + (size_t)s0 * L * (L / 32) : nullptr, L, np, st));
  }
  if (int rc = done()) return rc;
  {
    Prof p(e, st, prof, 2.0 * M * H * H);
#ifdef AE_TOOLS
    if (e->gemm_p2 & 4)
      HIPC(ae_bench_gemm_packed_res_stats(cp, w.wo_p, w.bo, prev ? v : e->x + t0 * H,
                                          prev ? sa : nullptr, prev ? prev->ln2g : nullptr,
                                          prev ? prev->ln2b : nullptr, eps, v, xp, sb, M, H, H, np,
                                          w.kap_o, 1, 0, st));
    else
#endif
    HIPC(ae_launch_gemm_packed_res_stats(cp, w.wo_p, w.bo, prev ? v : e->x + t0 * H,
                                         prev ? sa : nullptr, prev ? prev->ln2g : nullptr,
                                         prev ? prev->ln2b : nullptr, eps, v, xp, sb, M, H, H, np,
                                         w.kap_o, st));
  }
  if (int rc = done()) return rc;
  {
    Prof p(e, st, prof || e->prof_kind == AE_KIND_GEMM_FFN1, 2.0 * M * F * H);
#ifdef AE_TOOLS
    if (e->gemm_p2 & 2)
      HIPC(ae_bench_gemm_packed_fold(xp, w.w1_p, w.b1_f, w.s1, sb, eps, hp, M, F, H, 1, np, w.kc1,
                                     1, 0, st));
    else
#endif
    HIPC(ae_launch_gemm_packed_fold(xp, w.w1_p, w.b1_f, w.s1, sb, eps, hp, M, F, H, 1, np, w.kc1,
                                    st));
  }
  if (int rc = done()) return rc;
  {
    Prof p(e, st, prof, 2.0 * M * H * F);
#ifdef AE_TOOLS
    if (e->gemm_p2 & 8)
      HIPC(ae_bench_gemm_packed_res_stats(hp, w.w2_p, w.b2, v, sb, w.ln1g, w.ln1b, eps, v, xp, sa,
                                          M, H, F, np, w.kap_f, 1, 0, st));
    else
#endif
    HIPC(ae_launch_gemm_packed_res_stats(hp, w.w2_p, w.b2, v, sb, w.ln1g, w.ln1b, eps, v, xp, sa,
                                         M, H, F, np, w.kap_f, st));
  }
  if (int rc = done()) return rc;
  // the last full layer's output x = LN2(v) for the CLS path / MLM head / encode outputs, from
  // FFN2's tile statistics in the folded consumers' merge order (the same bits they see)
  if (last) HIPC(ae_launch_layernorm_stats(v, sa, w.ln2g, w.ln2b, eps, M, e->x + t0 * H, st));
  return AE_OK;
}

// Runs the encoder over compacted tokens; on return the last-layer CLS rows are in e->xc
// (cls_only) or all rows in e->x.  lens: the host copy of the sequence lengths (two-stream mode).
// qper > 0 (cls_only): the last layer runs for the query rows e->qrow [n][qper] (ae_encode_rows)
// instead of the CLS rows; on return they are in e->xc [n·qper][H].
int run_encoder(ae_engine* e, const int32_t* ids, const int32_t* pos, const uint32_t* mask_bits,
                int n, int L, int64_t T, int max_len, bool cls_only, hipStream_t st,
                int keep_all = 0, bool node_avg = false, const int32_t* lens = nullptr,
                int qper = 0) {
  const int H = e->cfg.hidden, F = e->cfg.ffn, NL = e->cfg.layers, heads = e->cfg.heads;
  const float eps = e->cfg.ln_eps;
  HIPC(hipMemsetAsync(e->err, 0, sizeof(int), st));
  HIPC(ae_launch_compact(ids, pos, e->cu, n, L, e->cfg.pad_id, keep_all, e->tok_ids, e->tok_pos,
                         e->src_col, e->err, st));
  // ae_encode_rows: the compacted row of every query slot (columns row0_dev[s] + j)
  if (qper > 0)
    HIPC(ae_launch_query_rows(e->cu, e->src_col, e->row0_dev, n, qper, (int)T, e->qrow, st));
  const bool pl = e->planes;
  HIPC(ae_launch_embed_ln(e->tok_ids, e->tok_pos, e->wemb, e->pemb, e->temb, e->eg, e->eb, eps,
                          (int)T, e->cfg.max_pos, e->x, pl ? e->xp : nullptr, e->np,
                          node_avg ? mask_bits : nullptr, L, e->cu, n, st));
  unsigned short* qkvp = reinterpret_cast<unsigned short*>(e->qkv);  // planes mode: [T][np·3H]
  int first = 0;  // first layer the single-stream loop below runs
  if (pl) {
    // the full layers (layer_rows): with two streams in P parts of the batch (sequence ranges,
    // each on its own stream, every part one lag behind the previous; one part when n == 1),
    // else one part of all rows on st.  Every row's arithmetic is the same either way.
    const int NLs = cls_only ? NL - 1 : NL;
    const int P = e->split && lens ? (n < e->split_parts ? n : e->split_parts) : (n > 0 ? 1 : 0);
    int s_beg[ae_engine::kMaxParts + 1], ml[ae_engine::kMaxParts];
    int64_t r_beg[ae_engine::kMaxParts + 1];
    for (int p = 0; p <= P; ++p) s_beg[p] = (int)((int64_t)n * p / (P ? P : 1));
    for (int p = 0; p < P; ++p) {
      ml[p] = 0;
      if (lens)
        for (int i = s_beg[p]; i < s_beg[p + 1]; ++i) ml[p] = lens[i] > ml[p] ? lens[i] : ml[p];
      else
        ml[p] = max_len;
    }
    // row ranges: host prefix sums of the uploaded lens (all rows for one part)
    for (int p = 0; p <= P; ++p) r_beg[p] = P == 1 ? (p ? T : 0) : e->pinned_cu[s_beg[p]];
    auto stream_of = [&](int p) { return p == 0 ? st : e->sts[p]; };
    if (P > 1) {
      HIPC(hipEventRecord(e->ev_fork, st));
      for (int p = 1; p < P; ++p) HIPC(hipStreamWaitEvent(e->sts[p], e->ev_fork, 0));
    }
    for (int li = 0; li < NLs; ++li) {
      for (int p = 0; p < P; ++p) {
        if (li == 0 && p > 0) HIPC(hipStreamWaitEvent(e->sts[p], e->ev_lag[p - 1], 0));
        const int64_t t0 = r_beg[p];
        const int M = (int)(r_beg[p + 1] - t0);
        int rc;
        if ((rc = layer_rows(e, li, t0, M, s_beg[p], s_beg[p + 1] - s_beg[p], ml[p], mask_bits, L,
                             stream_of(p), li == NLs - 1,
                             li == 0 && p + 1 < P ? e->ev_lag[p] : nullptr, e->split_lag)))
          return rc;
      }
    }
    for (int p = 1; p < P; ++p) {
      HIPC(hipEventRecord(e->ev_join[p], e->sts[p]));
      HIPC(hipStreamWaitEvent(st, e->ev_join[p], 0));
    }
    first = NLs;
  }
  for (int li = first; li < NL; ++li) {
    const LayerW& w = e->layers[li];
    const bool last_cls = cls_only && li == NL - 1;
    const int nq = qper > 0 ? n * qper : n;  // rows of the last layer's query path
    int rc;
    if (last_cls && !e->cls_absorb && qper > 0)
      return fail(AE_EINVAL, "row windows need the absorbed last layer (AE_CLS_ABSORB)");
    if (last_cls && e->cls_absorb) {
      // the CLS query per sequence (or the query rows of ae_encode_rows), then attention with W_k
      // absorbed / W_v deferred over the layer-input rows (cls_attention.hip); no K / V
      // projection of the T rows
      if (qper > 0)
        HIPC(ae_launch_gather_rows(e->x, e->qrow, e->cu, qper, nq, e->xc, st));
      else
        HIPC(ae_launch_gather_cls(e->x, e->x, e->cu, n, e->cc, e->xc, st));
      if ((rc = gemm(e, e->xc, w.wqkv, w.wqkv_h, w.wqkv_l, w.bqkv, nullptr, e->hc, nq, H, H,
                     EPI_BIAS, st, false)))
        return rc;
      if ((rc = ensure_cls_part(e, T, n, qper > 0 ? qper : 1))) return rc;
      Prof p(e, st, e->prof_kind == AE_KIND_ATTENTION, 0.0);
      // split modes fold log2(e)/8 into W_q (ae_create); the exact mode scales here
      const float scale = e->cfg.precision == AE_PREC_FP32 ? 0.18033688011112042f : 1.0f;
      HIPC(ae_launch_cls_attention(e->x, e->hc, w.wqkv + (size_t)H * H,
                                   w.wqkv + (size_t)2 * H * H, w.bqkv + 2 * H, e->cu, n,
                                   qper > 0 ? qper : 1, max_len, mask_bits, L, scale, e->cls_u,
                                   e->cls_part, e->cls_y, e->cc, e->err, st));
    } else if (pl && li > 0) {
      // Q | K | V as packed planes (Q pre-scaled) straight into the attention's LDS-DMA, from the
      // previous layer's pre-LayerNorm rows (the LayerNorm folded in)
      Prof p(e, st, e->prof_kind == AE_KIND_GEMM_ANY, 2.0 * T * 3 * H * H);
      HIPC(ae_launch_gemm_packed_fold(e->xp, w.wqkv_p, w.bqkv_f, w.sqkv, e->lnst, eps, qkvp,
                                      (int)T, 3 * H, H, 0, e->np, w.kcqkv, st));
    } else if (pl) {
      if ((rc = gemm_pk(e, e->xp, w.wqkv_p, w.bqkv, nullptr, nullptr, qkvp, (int)T, 3 * H, H,
                        EPI_BIAS_PACKED, st, false)))
        return rc;
    } else if ((rc = gemm(e, e->x, w.wqkv, w.wqkv_h, w.wqkv_l, w.bqkv, nullptr, e->qkv, (int)T,
                          3 * H, H, EPI_BIAS, st, false))) {
      return rc;
    }
    if (!(last_cls && e->cls_absorb)) {
      const double flop = 0.0;  // attention FLOP are accounted by the caller
      Prof p(e, st, e->prof_kind == AE_KIND_ATTENTION, flop);
      if (e->cfg.precision == AE_PREC_FP32)
        HIPC(ae_launch_attention_f32(e->qkv, e->ctx, e->cu, last_cls ? e->one : nullptr,
                                     last_cls ? 1 : max_len, n, heads, mask_bits, L, st));
      else
        HIPC(attention_pp(e, qkvp, e->ctx, last_cls ? nullptr : e->cp, e->cu,
                          last_cls ? e->one : nullptr, last_cls ? 1 : max_len, n, heads,
                          mask_bits, L, e->np, st));
    }
    if (!last_cls) {  // the exact-fp32 mode (the split modes ran their full layers above)
      if ((rc = gemm(e, e->ctx, w.wo, w.wo_h, w.wo_l, w.bo, e->x, e->tmp, (int)T, H, H, EPI_BIAS_RESIDUAL,
                     st, false)))
        return rc;
      HIPC(ae_launch_layernorm(e->tmp, w.ln1g, w.ln1b, eps, (int)T, e->x, nullptr, 0, st));
      if ((rc = gemm(e, e->x, w.w1, w.w1_h, w.w1_l, w.b1, nullptr, e->h1, (int)T, F, H, EPI_BIAS_GELU, st,
                     true)))
        return rc;
      if ((rc = gemm(e, e->h1, w.w2, w.w2_h, w.w2_l, w.b2, e->x, e->tmp, (int)T, H, F, EPI_BIAS_RESIDUAL,
                     st, false)))
        return rc;
      HIPC(ae_launch_layernorm(e->tmp, w.ln2g, w.ln2b, eps, (int)T, e->x, nullptr, 0, st));
    } else {
      if (!e->cls_absorb) HIPC(ae_launch_gather_cls(e->ctx, e->x, e->cu, n, e->cc, e->xc, st));
      if ((rc = gemm(e, e->cc, w.wo, w.wo_h, w.wo_l, w.bo, e->xc, e->tc, nq, H, H, EPI_BIAS_RESIDUAL,
                     st, false)))
        return rc;
      HIPC(ae_launch_layernorm(e->tc, w.ln1g, w.ln1b, eps, nq, e->xc, nullptr, 0, st));
      if ((rc = gemm(e, e->xc, w.w1, w.w1_h, w.w1_l, w.b1, nullptr, e->hc, nq, F, H, EPI_BIAS_GELU,
                     st, false)))
        return rc;
      if ((rc = gemm(e, e->hc, w.w2, w.w2_h, w.w2_l, w.b2, e->xc, e->tc, nq, H, F, EPI_BIAS_RESIDUAL,
                     st, false)))
        return rc;
      HIPC(ae_launch_layernorm(e->tc, w.ln2g, w.ln2b, eps, nq, e->xc, nullptr, 0, st));
    }
  }
  return AE_OK;
}

int check_common(ae_engine* e, const int32_t* ids, const int32_t* lens, int n, int L) {
  if (!e) return fail(AE_EINVAL, "null engine");
  if (!ids || !lens) return fail(AE_EINVAL, "null ids/lens");
  if (n < 0 || L < 2 || L > 4096) return fail(AE_EINVAL, "bad n/L");
  return AE_OK;
}
}  // namespace

extern "C" {

const char* ae_last_error(void) { return g_err.c_str(); }
const char* ae_version(void) { return "alert-mi355x 0.1 (gfx950)"; }

int ae_create(const ae_config* cfg, const ae_weight_view* weights, int32_t n_weights,
              int32_t device, ae_engine** out) {
  if (!cfg || !out || (!weights && n_weights)) return fail(AE_EINVAL, "null argument");
  if (cfg->hidden != 768 || cfg->heads != 12)
    return fail(AE_EINVAL, "kernels are specialised for hidden=768, heads=12");
  if (cfg->ffn % 32 || cfg->layers < 1) return fail(AE_EINVAL, "bad ffn/layers");
  if (cfg->num_labels < 1 || cfg->num_labels > 128) return fail(AE_EINVAL, "num_labels in [1,128]");
  if (cfg->head_kind == AE_HEAD_SIGMOID1 && cfg->num_labels != 1)
    return fail(AE_EINVAL, "sigmoid head needs num_labels=1");
  if (cfg->head_kind == AE_HEAD_PAIR2 && cfg->num_labels != 2)
    return fail(AE_EINVAL, "pair head needs num_labels=2");
  if (cfg->precision < AE_PREC_FP32 || cfg->precision > AE_PREC_F32X3)
    return fail(AE_EINVAL, "precision must be AE_PREC_FP32, AE_PREC_BF16 or AE_PREC_F32X3");
  if (cfg->streams != AE_STREAMS_TWO && cfg->streams != AE_STREAMS_ONE)
    return fail(AE_EINVAL, "streams must be AE_STREAMS_TWO or AE_STREAMS_ONE");
  HIPC(hipSetDevice(device));
  ae_engine* e = new ae_engine();
  e->cfg = *cfg;
  e->device = device;
  // split-precision modes run the full-length GEMMs on bf16 activation planes (gemm_planes.hip)
  e->planes = cfg->precision != AE_PREC_FP32;
  e->np = cfg->precision == AE_PREC_F32X3 ? 2 : 1;
  WeightTable wt;
  for (int i = 0; i < n_weights; ++i) wt.by_name[weights[i].name] = &weights[i];
  const int64_t H = cfg->hidden, F = cfg->ffn, V = cfg->vocab;
  int rc = 0;
#define UP(name, numel, dst)                                   \
  if ((rc = upload(e, wt, name, numel, dst))) {                \
    std::string m = g_err;                                     \
    ae_destroy(e);                                             \
    return fail(rc, m);                                        \
  }
  UP("embeddings.word_embeddings.weight", V * H, &e->wemb);
  UP("embeddings.position_embeddings.weight", (int64_t)cfg->max_pos * H, &e->pemb);
  UP("embeddings.token_type_embeddings.weight", (int64_t)cfg->type_vocab * H, &e->temb);
  UP("embeddings.LayerNorm.weight", H, &e->eg);
  UP("embeddings.LayerNorm.bias", H, &e->eb);
  e->layers.resize(cfg->layers);
  std::vector<float> prev_kap_f;  // the previous layer's FFN2 plane shift (its QKV consumer's)
  for (int l = 0; l < cfg->layers; ++l) {
    LayerW& w = e->layers[l];
    std::memset(&w, 0, sizeof(w));
    const std::string p = "encoder.layer." + std::to_string(l) + ".";
    // fused QKV: rows [q; k; v]
    const ae_weight_view* q = wt.get(p + "attention.self.query.weight");
    const ae_weight_view* k = wt.get(p + "attention.self.key.weight");
    const ae_weight_view* v = wt.get(p + "attention.self.value.weight");
    const ae_weight_view* qb = wt.get(p + "attention.self.query.bias");
    const ae_weight_view* kb = wt.get(p + "attention.self.key.bias");
    const ae_weight_view* vb = wt.get(p + "attention.self.value.bias");
    if (!q || !k || !v || !qb || !kb || !vb) {
      ae_destroy(e);
      return fail(AE_ENOENT, "missing attention.self weights of layer " + std::to_string(l));
    }
    if (q->numel != H * H || k->numel != H * H || v->numel != H * H || qb->numel != H ||
        kb->numel != H || vb->numel != H) {
      ae_destroy(e);
      return fail(AE_EINVAL, "bad attention.self shapes in layer " + std::to_string(l));
    }
    std::vector<float> hw(3 * H * H), hb(3 * H);
    std::memcpy(hw.data(), q->data, H * H * 4);
    std::memcpy(hw.data() + H * H, k->data, H * H * 4);
    std::memcpy(hw.data() + 2 * H * H, v->data, H * H * 4);
    std::memcpy(hb.data(), qb->data, H * 4);
    std::memcpy(hb.data() + H, kb->data, H * 4);
    std::memcpy(hb.data() + 2 * H, vb->data, H * 4);
    if (cfg->precision != AE_PREC_FP32) {
      // split-precision modes: the packed QKV output feeds attention_pp.hip, which runs its
      // softmax in the exp2 domain over Q·K^T·log2(e)/8 — fold that scale into Wq and bq (these
      // copies serve only the split path; the fp32 mode keeps the HF weights unchanged)
      constexpr float kQScale = 0.18033688011112042f;  // log2(e) / sqrt(64)
      for (int64_t i = 0; i < (int64_t)H * H; ++i) hw[i] *= kQScale;
      for (int i = 0; i < H; ++i) hb[i] *= kQScale;
    }
    if ((rc = dev_alloc(e, (void**)&w.wqkv, hw.size() * 4)) ||
        (rc = dev_alloc(e, (void**)&w.bqkv, hb.size() * 4))) {
      std::string m = g_err;
      ae_destroy(e);
      return fail(rc, m);
    }
    if (hipMemcpy(w.wqkv, hw.data(), hw.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(w.bqkv, hb.data(), hb.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      ae_destroy(e);
      return fail(AE_EDEVICE, "weight upload failed");
    }
    UP(p + "attention.output.dense.weight", H * H, &w.wo);
    UP(p + "attention.output.dense.bias", H, &w.bo);
    UP(p + "attention.output.LayerNorm.weight", H, &w.ln1g);
    UP(p + "attention.output.LayerNorm.bias", H, &w.ln1b);
    UP(p + "intermediate.dense.weight", F * H, &w.w1);
    UP(p + "intermediate.dense.bias", F, &w.b1);
    UP(p + "output.dense.weight", H * F, &w.w2);
    UP(p + "output.dense.bias", H, &w.b2);
    UP(p + "output.LayerNorm.weight", H, &w.ln2g);
    UP(p + "output.LayerNorm.bias", H, &w.ln2b);
    if (cfg->precision != AE_PREC_FP32) {
      const bool lo = cfg->precision == AE_PREC_F32X3;
      auto view = [&](const std::string& n) { return wt.get(n); };
      const ae_weight_view* vo = view(p + "attention.output.dense.weight");
      const ae_weight_view* v1 = view(p + "intermediate.dense.weight");
      const ae_weight_view* v2 = view(p + "output.dense.weight");
      if ((rc = upload_split(e, hw.data(), hw.size(), &w.wqkv_h, lo ? &w.wqkv_l : nullptr)) ||
          (rc = upload_split(e, vo->data, vo->numel, &w.wo_h, lo ? &w.wo_l : nullptr)) ||
          (rc = upload_split(e, v1->data, v1->numel, &w.w1_h, lo ? &w.w1_l : nullptr)) ||
          (rc = upload_split(e, v2->data, v2->numel, &w.w2_h, lo ? &w.w2_l : nullptr))) {
        std::string m = g_err;
        ae_destroy(e);
        return fail(rc, m);
      }
      // the planes GEMMs: W_o and W_2 as they are; FFN1 with this layer's LN1 folded in, the QKV
      // of layers >= 1 with the previous layer's LN2 (layer 0's input is the embedding LN's x)
      const std::string pp = "encoder.layer." + std::to_string(l - 1) + ".";
      const ae_weight_view* g1 = view(p + "attention.output.LayerNorm.weight");
      const ae_weight_view* b1 = view(p + "attention.output.LayerNorm.bias");
      const ae_weight_view* bi = view(p + "intermediate.dense.bias");
      const int np = lo ? 2 : 1;
      // plane shifts: the O-projection's v = ... + b_o + LN(prev) (layer 0: the embedding LN's
      // x) and FFN2's v = ... + b_2 + LN1(v_o) carry the constant columns b + beta; their planes
      // hold v - kappa, and FFN1 / the next layer's QKV start their accumulators at kappa·W'^T
      std::vector<float> kap_o, kap_f;
      if ((rc = upload_kappa(e, view(p + "attention.output.dense.bias")->data,
                             view(l == 0 ? std::string("embeddings.LayerNorm.bias")
                                         : pp + "output.LayerNorm.bias")->data,
                             H, kap_o, &w.kap_o)) ||
          (rc = upload_kappa(e, view(p + "output.dense.bias")->data, b1->data, H, kap_f,
                             &w.kap_f))) {
        std::string m = g_err;
        ae_destroy(e);
        return fail(rc, m);
      }
      if (lo) {
        if ((l == 0 && (rc = upload_packed(e, hw.data(), 3 * H, H, &w.wqkv_p))) ||
            (rc = upload_packed(e, vo->data, H, H, &w.wo_p)) ||
            (rc = upload_packed(e, v2->data, H, F, &w.w2_p))) {
          std::string m = g_err;
          ae_destroy(e);
          return fail(rc, m);
        }
      } else {
        if (l == 0) w.wqkv_p = w.wqkv_h;
        w.wo_p = w.wo_h;
        w.w2_p = w.w2_h;
      }
      if ((rc = upload_folded(e, v1->data, bi->data, g1->data, b1->data, F, H, np, &w.w1_p, &w.s1,
                              &w.b1_f, kap_o.data(), &w.kc1)) ||
          (l > 0 && (rc = upload_folded(e, hw.data(), hb.data(),
                                        view(pp + "output.LayerNorm.weight")->data,
                                        view(pp + "output.LayerNorm.bias")->data, 3 * H, H, np,
                                        &w.wqkv_p, &w.sqkv, &w.bqkv_f, prev_kap_f.data(),
                                        &w.kcqkv)))) {
        std::string m = g_err;
        ae_destroy(e);
        return fail(rc, m);
      }
      prev_kap_f = kap_f;
    }
  }
  if (cfg->head_kind != AE_HEAD_NONE) {
    const int64_t in_dim = cfg->head_kind == AE_HEAD_PAIR2 ? 2 * H : H;
    UP("classifier.dense.weight", H * in_dim, &e->hd_w);
    UP("classifier.dense.bias", H, &e->hd_b);
    UP("classifier.out_proj.weight", (int64_t)cfg->num_labels * H, &e->ho_w);
    UP("classifier.out_proj.bias", cfg->num_labels, &e->ho_b);
  }
  if (cfg->with_mlm) {
    UP("lm_head.dense.weight", H * H, &e->lm_dw);
    UP("lm_head.dense.bias", H, &e->lm_db);
    UP("lm_head.layer_norm.weight", H, &e->lm_lg);
    UP("lm_head.layer_norm.bias", H, &e->lm_lb);
    UP("lm_head.bias", V, &e->lm_bias);  // decoder weight is tied to word_embeddings
  }
#undef UP
  if ((rc = dev_alloc(e, (void**)&e->one, 16)) || (rc = dev_alloc(e, (void**)&e->err, 16)) ||
      (rc = dev_alloc(e, (void**)&e->skws, (size_t)ae_engine::kSplitKFloats * 4))) {
    ae_destroy(e);
    return fail(rc, "alloc");
  }
  const int one_host[4] = {1, 1, 1, 1};
  HIPC(hipMemcpy(e->one, one_host, 16, hipMemcpyHostToDevice));
  HIPC(hipEventCreateWithFlags(&e->pinned_ready, hipEventDisableTiming));
  HIPC(hipEventRecord(e->pinned_ready, nullptr));
  HIPC(hipEventCreateWithFlags(&e->r0_ready, hipEventDisableTiming));
  HIPC(hipEventRecord(e->r0_ready, nullptr));
#ifdef AE_TOOLS
  // A/B knobs of the tools library (lib/libalert_engine_tools.so, tools/engine_ab.py and the
  // alternative-form parity tests); the product library has the defaults compiled in
  {
    const char* ca = std::getenv("AE_CLS_ABSORB");  // A/B runs: 0 = full-T QKV + attention
    e->cls_absorb = !(ca && ca[0] == '0');
  }
#endif
  if (e->planes) {
    // two streams unless cfg.streams == AE_STREAMS_ONE (tools/split_ab.py,
    // profiles/r3s_split_streams_ab.json: B=64 x L=512 16.58 -> 16.35 ms per step, ragged lens
    // 40..512 11.36 -> 9.53 ms)
    e->split = e->cfg.streams != AE_STREAMS_ONE;
#ifdef AE_TOOLS
    const char* sp = std::getenv("AE_SPLIT_STREAMS");
    if (sp && sp[0] == '0') e->split = false;
    // experiments: 1 (after QKV) .. 5 (after the whole layer 0: QKV, attention, O-projection,
    // FFN1, FFN2 — layer_rows' five kernels)
    const char* lag = std::getenv("AE_SPLIT_LAG");
    if (lag && lag[0] >= '1' && lag[0] <= '5') e->split_lag = lag[0] - '0';
    const char* av = std::getenv("AE_ATTN_VARIANT");  // A/B runs: 6, 66, 72 (67 = production)
    if (av) {
      const int v = std::atoi(av);
      if (v != 0 && v != 6 && v != 66 && v != 67 && v != 72) {
        ae_destroy(e);
        return fail(AE_EINVAL, "AE_ATTN_VARIANT must be 6, 66, 67 or 72 (the exact loops)");
      }
      e->attn_variant = v == 67 ? 0 : v;
    }
    const char* g2 = std::getenv("AE_GEMM_P2");  // experiments: bit mask, see ae_engine::gemm_p2
    if (g2) e->gemm_p2 = std::atoi(g2) & 15;
    const char* parts = std::getenv("AE_SPLIT_PARTS");  // experiments: 2 (default) .. 4
    if (parts && parts[0] >= '2' && parts[0] <= '4') e->split_parts = parts[0] - '0';
#endif
    if (e->split) {
      HIPC(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
      for (int p = 0; p < ae_engine::kMaxParts; ++p) {
        if (p > 0) {
          const char* sp2 = nullptr;
#ifdef AE_TOOLS
          // experiments (AE_SPLIT_PRIO): the lagging parts' streams at the lowest ("lo") or the
          // highest ("hi") stream priority instead of the default
          sp2 = std::getenv("AE_SPLIT_PRIO");
#endif
          if (sp2) {
            int least = 0, greatest = 0;
            HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIPC(hipStreamCreateWithPriority(&e->sts[p], hipStreamNonBlocking,
                                             sp2[0] == 'h' ? greatest : least));
          } else {
            HIPC(hipStreamCreateWithFlags(&e->sts[p], hipStreamNonBlocking));
          }
        }
        HIPC(hipEventCreateWithFlags(&e->ev_lag[p], hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&e->ev_join[p], hipEventDisableTiming));
      }
    }
  }
  HIPC(hipDeviceSynchronize());
  *out = e;
  return AE_OK;
}

int ae_destroy(ae_engine* e) {
  if (!e) return AE_OK;
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  for (void* p : e->allocs)
    if (p) (void)hipFree(p);
  if (e->pinned_cu) (void)hipHostFree(e->pinned_cu);
  if (e->pinned_ready) (void)hipEventDestroy(e->pinned_ready);
  if (e->pinned_r0) (void)hipHostFree(e->pinned_r0);
  if (e->r0_ready) (void)hipEventDestroy(e->r0_ready);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  for (int p = 0; p < ae_engine::kMaxParts; ++p) {
    if (e->ev_lag[p]) (void)hipEventDestroy(e->ev_lag[p]);
    if (e->ev_join[p]) (void)hipEventDestroy(e->ev_join[p]);
    if (e->sts[p]) (void)hipStreamDestroy(e->sts[p]);
  }
  for (auto* v : {&e->prof, &e->prof_pool})
    for (auto& r : *v) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
  delete e;
  return AE_OK;
}

static int score_impl(ae_engine* e, const int32_t* ids, const int32_t* lens, const int32_t* pos,
                      const uint32_t* mask_bits, int32_t n, int32_t L, float* probs_out,
                      void* stream, bool node_avg);

int ae_score(ae_engine* e, const int32_t* ids, const int32_t* lens, const int32_t* pos,
             const uint32_t* mask_bits, int32_t n, int32_t L, float* probs_out, void* stream) {
  return score_impl(e, ids, lens, pos, mask_bits, n, L, probs_out, stream, false);
}

int ae_score_graph(ae_engine* e, const int32_t* ids, const int32_t* lens, const int32_t* pos,
                   const uint32_t* mask_bits, int32_t n, int32_t L, float* probs_out,
                   void* stream) {
  if (!pos || !mask_bits) return fail(AE_EINVAL, "ae_score_graph needs pos and mask_bits");
  return score_impl(e, ids, lens, pos, mask_bits, n, L, probs_out, stream, true);
}

static int score_impl(ae_engine* e, const int32_t* ids, const int32_t* lens, const int32_t* pos,
                      const uint32_t* mask_bits, int32_t n, int32_t L, float* probs_out,
                      void* stream, bool node_avg) {
  int rc = check_common(e, ids, lens, n, L);
  if (rc) return rc;
  if (e->cfg.head_kind == AE_HEAD_NONE) return fail(AE_EINVAL, "engine has no task head");
  if (e->cfg.head_kind == AE_HEAD_PAIR2 && (n & 1)) return fail(AE_EINVAL, "pair head needs even n");
  if (mask_bits && (L % 32)) return fail(AE_EINVAL, "mask_bits needs L % 32 == 0");
  if (!probs_out) return fail(AE_EINVAL, "null probs_out");
  if (n == 0) return AE_OK;
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  if ((rc = ensure_workspace(e, (size_t)n * L, n))) return rc;
  int64_t T = 0;
  if ((rc = upload_cu(e, lens, n, L, st, &T))) return rc;
  int max_len = 0;
  for (int i = 0; i < n; ++i) max_len = lens[i] > max_len ? lens[i] : max_len;
  if ((rc = run_encoder(e, ids, pos, mask_bits, n, L, T, max_len, true, st, node_avg ? 1 : 0,
                        node_avg, lens)))
    return rc;
  const int kind = e->cfg.head_kind == AE_HEAD_SIGMOID1 ? 0 : (e->cfg.head_kind == AE_HEAD_PAIR2 ? 2 : 1);
  const int n_out = kind == 2 ? n / 2 : n;
  // head: dense (+tanh) as a GEMM over the compact CLS rows (pair head: [n/2, 1536] view), then
  // out_proj + sigmoid/softmax
  const int in_dim = kind == 2 ? 2 * e->cfg.hidden : e->cfg.hidden;
  HIPC(ae_launch_gemm_f32(e->xc, e->hd_w, e->hd_b, nullptr, e->tc, n_out, e->cfg.hidden, in_dim,
                          in_dim, in_dim, e->cfg.hidden, EPI_BIAS_TANH, nullptr, st, e->skws,
                          ae_engine::kSplitKFloats));
  HIPC(ae_launch_head_out(e->tc, e->ho_w, e->ho_b, kind, e->cfg.num_labels, n_out, probs_out,
                          e->err, st));
  return AE_OK;
}

int ae_encode_ex(ae_engine* e, const int32_t* ids, const int32_t* lens, int32_t n, int32_t L,
                 int32_t flags, int32_t row0, int32_t nrows, float* hidden_out, void* stream) {
  int rc = check_common(e, ids, lens, n, L);
  if (rc) return rc;
  if (!hidden_out) return fail(AE_EINVAL, "null hidden_out");
  if (row0 < 0 || nrows < 1 || row0 + nrows > L) return fail(AE_EINVAL, "bad row window");
  if (flags & ~AE_ENC_ATTEND_PAD) return fail(AE_EINVAL, "unknown flags");
  if (n == 0) return AE_OK;
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  if ((rc = ensure_workspace(e, (size_t)n * L, n))) return rc;
  int64_t T = 0;
  if ((rc = upload_cu(e, lens, n, L, st, &T))) return rc;
  int max_len = 0;
  for (int i = 0; i < n; ++i) max_len = lens[i] > max_len ? lens[i] : max_len;
  if ((rc = run_encoder(e, ids, nullptr, nullptr, n, L, T, max_len, false, st,
                        (flags & AE_ENC_ATTEND_PAD) ? 1 : 0, false, lens)))
    return rc;
  HIPC(ae_launch_scatter_rows(e->x, e->cu, e->src_col, n, row0, nrows, (int)T, hidden_out, e->err,
                              st));
  return AE_OK;
}

int ae_encode(ae_engine* e, const int32_t* ids, const int32_t* lens, int32_t n, int32_t L,
              float* hidden_out, void* stream) {
  return ae_encode_ex(e, ids, lens, n, L, 0, 0, L, hidden_out, stream);
}

int ae_encode_rows(ae_engine* e, const int32_t* ids, const int32_t* lens, int32_t n, int32_t L,
                   int32_t flags, const int32_t* row0, int32_t nrows, float* hidden_out,
                   void* stream) {
  int rc = check_common(e, ids, lens, n, L);
  if (rc) return rc;
  if (!hidden_out || !row0) return fail(AE_EINVAL, "null hidden_out/row0");
  if (nrows < 1 || nrows > L) return fail(AE_EINVAL, "bad nrows");
  for (int i = 0; i < n; ++i)
    if (row0[i] < 0 || row0[i] + nrows > L)
      return fail(AE_EINVAL, "row0[" + std::to_string(i) + "]=" + std::to_string(row0[i]) +
                                 ": window outside [0, L)");
  if (flags & ~AE_ENC_ATTEND_PAD) return fail(AE_EINVAL, "unknown flags");
  if (!e->cls_absorb) return fail(AE_EINVAL, "row windows need the absorbed last layer");
  if (n == 0) return AE_OK;
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t nq = (size_t)n * nrows;
  if ((rc = ensure_workspace(e, (size_t)n * L, nq > (size_t)n ? nq : (size_t)n))) return rc;
  if ((size_t)n > e->cap_r0) {
    HIPC(hipDeviceSynchronize());
    const size_t c = n + n / 4 + 64;
    dev_free(e, e->row0_dev);
    e->row0_dev = nullptr;
    if (e->pinned_r0) (void)hipHostFree(e->pinned_r0);
    e->pinned_r0 = nullptr;
    if ((rc = dev_alloc(e, (void**)&e->row0_dev, c * 4))) return rc;
    HIPC(hipHostMalloc((void**)&e->pinned_r0, c * 4, hipHostMallocDefault));
    e->cap_r0 = c;
  }
  if (nq > e->cap_q) {
    HIPC(hipDeviceSynchronize());
    const size_t c = nq + nq / 4 + 64;
    dev_free(e, e->qrow);
    e->qrow = nullptr;
    if ((rc = dev_alloc(e, (void**)&e->qrow, c * 4))) return rc;
    e->cap_q = c;
  }
  int64_t T = 0;
  if ((rc = upload_cu(e, lens, n, L, st, &T))) return rc;
  HIPC(hipEventSynchronize(e->r0_ready));  // the previous call's copy has left the pinned buffer
  std::memcpy(e->pinned_r0, row0, (size_t)n * 4);
  HIPC(hipMemcpyAsync(e->row0_dev, e->pinned_r0, (size_t)n * 4, hipMemcpyHostToDevice, st));
  HIPC(hipEventRecord(e->r0_ready, st));
  int max_len = 0;
  for (int i = 0; i < n; ++i) max_len = lens[i] > max_len ? lens[i] : max_len;
  // the query slots (e->qrow) are built from row0_dev by run_encoder right after compaction
  if ((rc = run_encoder(e, ids, nullptr, nullptr, n, L, T, max_len, true, st,
                        (flags & AE_ENC_ATTEND_PAD) ? 1 : 0, false, lens, nrows)))
    return rc;
  HIPC(ae_launch_scatter_query(e->xc, e->qrow, (int)nq, hidden_out, e->err, st));
  return AE_OK;
}

}  // extern "C"

namespace {
// lm_head over the T encoder rows in e->x: dense -> gelu -> LN -> decoder (tied word embeddings)
// + bias, into e->logits [T, V] (RobertaLMHead, reached from get_substitutes.py:62)
int mlm_logits(ae_engine* e, int64_t T, hipStream_t st) {
  const int V = e->cfg.vocab, H = e->cfg.hidden;
  int rc;
  if ((size_t)T * V > e->cap_logits) {
    HIPC(hipDeviceSynchronize());
    dev_free(e, e->logits);
    if ((rc = dev_alloc(e, (void**)&e->logits, (size_t)T * V * 4))) return rc;
    e->cap_logits = (size_t)T * V;
  }
  HIPC(ae_launch_gemm_f32(e->x, e->lm_dw, e->lm_db, nullptr, e->tmp, (int)T, H, H, H, H, H,
                          EPI_BIAS_GELU, nullptr, st, e->skws, ae_engine::kSplitKFloats));
  HIPC(ae_launch_layernorm(e->tmp, e->lm_lg, e->lm_lb, e->cfg.ln_eps, (int)T, e->ctx, nullptr, 0,
                           st));
  HIPC(ae_launch_gemm_f32(e->ctx, e->wemb, e->lm_bias, nullptr, e->logits, (int)T, V, H, H, H, V,
                          EPI_BIAS, nullptr, st, e->skws, ae_engine::kSplitKFloats));
  return AE_OK;
}
}  // namespace

extern "C" {

int ae_mlm_topk(ae_engine* e, const int32_t* ids, int32_t L, int32_t k, float* scores_out,
                int32_t* ids_out, void* stream) {
  if (!e || !ids || !scores_out || !ids_out) return fail(AE_EINVAL, "null argument");
  if (!e->lm_dw) return fail(AE_EINVAL, "engine created without the MLM head (with_mlm=0)");
  if (L < 1 || L > 4096 || k < 1 || k > 256) return fail(AE_EINVAL, "bad L/k");
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if ((rc = ensure_workspace(e, (size_t)L, 1))) return rc;
  const int32_t lens[1] = {L};
  int64_t T = 0;
  if ((rc = upload_cu(e, lens, 1, L, st, &T))) return rc;
  // codebert_mlm(input_ids_) is called without attention_mask: every id is attended
  if ((rc = run_encoder(e, ids, nullptr, nullptr, 1, L, T, L, false, st, 1))) return rc;
  if ((rc = mlm_logits(e, T, st))) return rc;
  HIPC(ae_launch_topk(e->logits, L, e->cfg.vocab, k, scores_out, ids_out, st));
  return AE_OK;
}

int ae_mlm_nll(ae_engine* e, const int32_t* ids, int32_t n, int32_t L, float* nll_out,
               void* stream) {
  if (!e || !ids || !nll_out) return fail(AE_EINVAL, "null argument");
  if (!e->lm_dw) return fail(AE_EINVAL, "engine created without the MLM head (with_mlm=0)");
  if (n < 0 || L < 1 || L > 4096) return fail(AE_EINVAL, "bad n/L");
  if (n == 0) return AE_OK;
  HIPC(hipSetDevice(e->device));
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if ((rc = ensure_workspace(e, (size_t)n * L, n))) return rc;
  std::vector<int32_t> lens((size_t)n, L);
  int64_t T = 0;
  if ((rc = upload_cu(e, lens.data(), n, L, st, &T))) return rc;
  // mlm_model(all_substitutes) without attention_mask (utils.py:237): every id is attended;
  // with all rows full the compact token order is row-major [n, L]
  if ((rc = run_encoder(e, ids, nullptr, nullptr, n, L, T, L, false, st, 1))) return rc;
  if ((rc = mlm_logits(e, T, st))) return rc;
  HIPC(ae_launch_nll_rows(e->logits, e->tok_ids, (int)T, e->cfg.vocab, nll_out, st));
  return AE_OK;
}

int ae_splice(const int32_t* word_tok, const int32_t* word_off, const int32_t* mut_words,
              const int32_t* mut_off, int32_t n_mut, int32_t L, int32_t cls_id, int32_t sep_id,
              int32_t pad_id, int32_t* ids_out, int32_t* lens_out, void* stream) {
  if (!word_tok || !word_off || !mut_words || !mut_off || !ids_out || !lens_out)
    return fail(AE_EINVAL, "null argument");
  if (n_mut < 0 || L < 2) return fail(AE_EINVAL, "bad n_mut/L");
  HIPC(ae_launch_splice(word_tok, word_off, mut_words, mut_off, n_mut, L, cls_id, sep_id, pad_id,
                        ids_out, lens_out, (hipStream_t)stream));
  return AE_OK;
}

int ae_topk(const float* x, int32_t rows, int32_t cols, int32_t k, float* vals_out,
            int32_t* idx_out, void* stream) {
  if (!x || !vals_out || !idx_out) return fail(AE_EINVAL, "null argument");
  if (rows < 0 || cols < 1 || k < 1 || k > 256 || k > cols) return fail(AE_EINVAL, "bad shape");
  HIPC(ae_launch_topk(x, rows, cols, k, vals_out, idx_out, (hipStream_t)stream));
  return AE_OK;
}

int ae_graph_mask(const int32_t* ids, const int32_t* meta, const int32_t* spans,
                  const int32_t* edges, int32_t n, int32_t L, int32_t e_cap, uint32_t* mask_bits,
                  void* stream) {
  if (n > 0 && (!ids || !meta || !spans || !edges || !mask_bits))
    return fail(AE_EINVAL, "null argument");
  if (n < 0 || L < 32 || L % 32 || L > 1024 || e_cap < 1) return fail(AE_EINVAL, "bad shape");
  HIPC(ae_launch_graph_mask(ids, meta, spans, edges, n, L, e_cap, mask_bits, (hipStream_t)stream));
  return AE_OK;
}

int ae_cosine_rank(const float* ref, const float* cand, int32_t n, int32_t span_len,
                   int32_t hidden, float eps, float* sims_out, void* stream) {
  if (!ref || !cand || !sims_out) return fail(AE_EINVAL, "null argument");
  if (n < 0 || span_len < 1 || hidden < 1) return fail(AE_EINVAL, "bad shape");
  HIPC(ae_launch_cosine_rank(ref, cand, n, span_len, hidden, eps, sims_out, (hipStream_t)stream));
  return AE_OK;
}

int ae_set_profiling(ae_engine* e, int32_t kind, int32_t enabled) {
  if (!e) return fail(AE_EINVAL, "null engine");
  if (enabled) {  // reserve the events now, outside whatever region the caller times
    HIPC(hipSetDevice(e->device));
    while (e->prof_pool.size() < 1024) {
      ProfRec r{};
      HIPC(hipEventCreate(&r.a));
      HIPC(hipEventCreate(&r.b));
      e->prof_pool.push_back(r);
    }
  }
  e->prof_kind = enabled ? kind : -1;
  return AE_OK;
}

int ae_kernel_time(ae_engine* e, double* ms_total, int64_t* launches, double* flop_total) {
  if (!e || !ms_total || !launches || !flop_total) return fail(AE_EINVAL, "null argument");
  HIPC(hipSetDevice(e->device));
  double ms = 0, fl = 0;
  int64_t cnt = 0;
  for (auto& r : e->prof) {
    HIPC(hipEventSynchronize(r.b));
    float t = 0.f;
    HIPC(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    fl += r.flop;
    ++cnt;
    e->prof_pool.push_back(r);
  }
  e->prof.clear();
  *ms_total = ms;
  *launches = cnt;
  *flop_total = fl;
  return AE_OK;
}

}  // extern "C"
