/*
 * alert_engine.h — C-ABI of the MI355X victim-query engine.
 *
 * This is the drop-in boundary below ALERT's `Model.get_results` (the victim
 * query boundary) and below the masked-LM substitute generation path.  Every
 * entry point is plain C: pointers, sizes, ints, no C++ or torch types.  The
 * Python host side (`attack-pretrain-models-of-code_amd/engine.py`) binds it
 * with ctypes on torch-owned device buffers; INTEGRATION.md shows the binding a
 * maintainer adds on the reference side.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference snapshot):
 *   ae_create     <- RobertaForSequenceClassification/RobertaForMaskedLM construction +
 *                    Model.load_state_dict(...) + .to("cuda")
 *                    (CodeXGLUE/Defect-detection/code/gi_attack.py:122-152)
 *   ae_score      <- Model.forward + the per-batch loop of Model.get_results
 *                    (CodeXGLUE/Defect-detection/code/model.py:24-59; clone head
 *                    CodeXGLUE/Clone-detection-BigCloneBench/code/model.py:13-85;
 *                    authorship head CodeXGLUE/Authorship-Attribution/code/model.py:13-91;
 *                    GraphCodeBERT mask/positions without node averaging)
 *   ae_score_graph<- GraphCodeBERT Model.forward incl. data-flow node averaging
 *                    (GraphCodeBERT/Defect-detection/code/model.py:24-45,
 *                    GraphCodeBERT/clonedetection/code/model.py:41-64)
 *   ae_splice     <- the text-level mutant construction + re-tokenisation
 *                    (python_parser/run_parser.py:218-266 get_example/get_example_batch,
 *                    CodeXGLUE/Defect-detection/code/attacker.py:38-45 convert_code_to_features)
 *                    expressed on token ids: word-id sequences -> padded [n, L] ids.
 *   ae_mlm_topk   <- codebert_mlm(input_ids)[0] + torch.topk(., 60, -1)
 *                    (CodeXGLUE/Defect-detection/preprocess/get_substitutes.py:62-63)
 *   ae_encode     <- codebert_mlm.roberta(ids)[0] (get_substitutes.py:73,105); ae_encode_ex adds
 *                    the no-attention_mask call form and a row window (the cosine span);
 *                    ae_encode_rows a window per sequence (get_substitutes.py:98-108)
 *   ae_mlm_nll    <- mlm_model(all_substitutes)[0] + CrossEntropyLoss(reduction='none')
 *                    (utils.py:237-239 get_bpe_substitues)
 *   ae_cosine_rank<- CosineSimilarity(dim=1) summed over the sub-word span / L_sub
 *                    (get_substitutes.py:75,108)
 *   ae_graph_mask <- GraphCodeDataset.__getitem__'s bool [L, L] graph-guided attention mask
 *                    (GraphCodeBERT/Defect-detection/code/utils.py:547-570 and the run.py
 *                    TextDataset of each GraphCodeBERT task), built on the device
 *
 * Conventions
 *   - Every function returns 0 on success or a negative AE_E* code; the
 *     message of the last failure on the calling thread is ae_last_error().
 *   - The engine owns its weights and workspaces (HBM); the caller owns all
 *     I/O buffers.  Pointers documented "device" are HIP device pointers.
 *   - Calls are asynchronous on the caller's stream (hipStream_t passed as
 *     void*; NULL = legacy default stream).  Nothing synchronises unless the
 *     function says so.
 *   - One engine per GPU per process; a handle is not re-entrant across host
 *     threads.
 */
#ifndef ALERT_ENGINE_H
#define ALERT_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AE_OK 0
#define AE_EINVAL (-22)  /* bad argument / shape */
#define AE_ENOMEM (-12)  /* device allocation failed */
#define AE_EDEVICE (-5)  /* HIP runtime error */
#define AE_ENOENT (-2)   /* weight tensor missing */

/* Task head on top of the CLS vector (reference model.py of each task). */
#define AE_HEAD_SIGMOID1 0 /* Devign: RobertaClassificationHead(num_labels=1) -> sigmoid   */
#define AE_HEAD_SOFTMAXN 1 /* Authorship: dense->tanh->out_proj(num_labels) -> softmax      */
#define AE_HEAD_PAIR2 2    /* Clone: cat(CLS_a, CLS_b) 1536->768->tanh->2 -> softmax        */
#define AE_HEAD_NONE 3     /* encoder only (MLM / cosine paths)                             */

#define AE_PREC_FP32 0  /* exact-f32 MFMA (v_mfma_f32_32x32x2_f32) for every GEMM           */
#define AE_PREC_BF16 1  /* GEMMs on bf16 MFMA (one term), f32 accumulate / residual stream  */
#define AE_PREC_F32X3 2 /* GEMMs as split-bf16 (hi*hi + hi*lo + lo*hi) on bf16 MFMA:
                           f32-class accuracy (probabilities within 1e-4) at 3 bf16 MFMAs  */

/* Encoder schedule of the split-precision modes (ignored by AE_PREC_FP32). */
#define AE_STREAMS_TWO 0 /* default: the batch as two halves on two HIP streams, one kernel apart
                            (one half's memory-bound phases beside the other's MFMA loops)   */
#define AE_STREAMS_ONE 1 /* every kernel on the caller's stream (bit-identical scores; what
                            the bench's roofline pass times)                                  */

typedef struct ae_config {
  int32_t layers;      /* 12 */
  int32_t hidden;      /* 768 (kernels are specialised for 768) */
  int32_t heads;       /* 12  (head dim 64) */
  int32_t ffn;         /* 3072 */
  int32_t vocab;       /* 50265 */
  int32_t max_pos;     /* 514 */
  int32_t type_vocab;  /* 1 */
  int32_t num_labels;  /* 1 (Devign), 2 (clone), 66 (authorship) */
  int32_t head_kind;   /* AE_HEAD_* */
  int32_t precision;   /* AE_PREC_* */
  int32_t pad_id;      /* 1 */
  int32_t with_mlm;    /* 1: also upload the lm_head (MLM paths) */
  float ln_eps;        /* 1e-5 */
  int32_t streams;     /* AE_STREAMS_*: how the split-precision encoder is scheduled */
} ae_config;

/* One named host tensor (fp32, row-major, HF state_dict naming). */
typedef struct ae_weight_view {
  const char *name;
  const float *data; /* host pointer */
  int64_t numel;
} ae_weight_view;

typedef struct ae_engine ae_engine;

int ae_create(const ae_config *cfg, const ae_weight_view *weights, int32_t n_weights,
              int32_t device, ae_engine **out);
int ae_destroy(ae_engine *eng);

/* Score n sequences of row length L.
 *   ids       device int32 [n, L]  token ids, pad = cfg.pad_id anywhere in the row
 *   lens      HOST  int32 [n]      count of non-pad ids of each row (the engine skips
 *                                  pad rows entirely: they never influence the CLS row).  A row
 *                                  whose ids disagree with its lens entry makes every output of
 *                                  the call NaN (the engine never reads or writes out of bounds)
 *   pos       device int32 [n, L] or NULL  explicit position ids (GraphCodeBERT); NULL =
 *                                  RoBERTa rule cumsum(ids!=pad)*(ids!=pad)+pad
 *   mask_bits device uint32 [n, L, ceil(L/32)] or NULL  explicit attention mask (GraphCodeBERT
 *                                  data-flow mask, bit j of row i = query i may attend key j);
 *                                  NULL = key-padding mask ids!=pad
 *   probs_out device float [n_out, C]  n_out = n (n/2 for AE_HEAD_PAIR2), C = max(num_labels,1)
 *                                  sigmoid head writes p (C=1); softmax heads write the row.
 */
int ae_score(ae_engine *eng, const int32_t *ids, const int32_t *lens, const int32_t *pos,
             const uint32_t *mask_bits, int32_t n, int32_t L, float *probs_out, void *stream);

/* GraphCodeBERT Model.forward (GraphCodeBERT/Defect-detection/code/model.py:24-45, clone pair
 * GraphCodeBERT/clonedetection/code/model.py:41-64): ae_score with explicit positions and the
 * data-flow mask, where each data-flow node row (pos == 0) first takes as its input embedding the
 * mean word embedding of the code tokens (pos >= 2) its mask row attends (model.py:27-33).
 * pos and mask_bits are required.  Here lens[i] is the number of leading columns of row i that
 * take part, pad ids included (normally L): as in HF's additive finfo(f32).min mask, a query row
 * whose mask excludes every key (a data-flow node whose code span was truncated away, a pad row)
 * attends all lens[i] keys uniformly, so pads are not dropped on this path. */
int ae_score_graph(ae_engine *eng, const int32_t *ids, const int32_t *lens, const int32_t *pos,
                   const uint32_t *mask_bits, int32_t n, int32_t L, float *probs_out, void *stream);

/* Encoder hidden states of n sequences: hidden_out device float [n, L, hidden]
 * (rows of pad positions are left untouched). */
int ae_encode(ae_engine *eng, const int32_t *ids, const int32_t *lens, int32_t n, int32_t L,
              float *hidden_out, void *stream);

/* ae_encode with options.
 *   flags     AE_ENC_ATTEND_PAD: the model is called without attention_mask (get_substitutes.py
 *             :73,105 codebert_mlm.roberta(ids)): the first lens[i] ids of row i are all attended,
 *             a pad id included (position = pad_id, only non-pad ids advance positions)
 *   row0/nrows  only rows [row0, row0 + nrows) of each sequence are written:
 *             hidden_out device float [n, nrows, hidden] */
#define AE_ENC_ATTEND_PAD 1
int ae_encode_ex(ae_engine *eng, const int32_t *ids, const int32_t *lens, int32_t n, int32_t L,
                 int32_t flags, int32_t row0, int32_t nrows, float *hidden_out, void *stream);

/* ae_encode_ex with a row window PER SEQUENCE, for the cosine naturalness filter's re-encodes
 * (get_substitutes.py:98-108: each candidate sequence is read only at the span of the occurrence
 * it substitutes, orig_embeddings / new_embeddings[0][keys[0]+1:keys[1]+1]).  The last layer runs
 * for the window rows only (its attention with W_k absorbed into each query and W_v applied to the
 * p-weighted row sum, cls_attention.hip; O-projection / FFN for nrows rows per sequence), so a
 * call costs 11 full layers plus O(n·nrows) rows, not 12 full layers.
 *   row0      HOST int32 [n]: sequence i's window is columns [row0[i], row0[i] + nrows)
 *             (0 <= row0[i], row0[i] + nrows <= L)
 *   hidden_out device float [n, nrows, hidden]; a column past lens[i] (or a pad id the call form
 *             drops) is left untouched, as in ae_encode_ex.  Same flags. */
int ae_encode_rows(ae_engine *eng, const int32_t *ids, const int32_t *lens, int32_t n, int32_t L,
                   int32_t flags, const int32_t *row0, int32_t nrows, float *hidden_out,
                   void *stream);

/* Per-token masked-LM negative log-likelihood of n full rows (no attention_mask: every id is
 * attended):  nll_out[i, t] = logsumexp(logits[i, t, :]) - logits[i, t, ids[i, t]]
 * (CrossEntropyLoss(reduction='none') of utils.py:238, the BPE-substitute perplexity).
 *   ids device int32 [n, L];  nll_out device float [n, L]. */
int ae_mlm_nll(ae_engine *eng, const int32_t *ids, int32_t n, int32_t L, float *nll_out,
               void *stream);

/* Masked-LM logits + top-k over the vocabulary for ONE sequence (no attention_mask: every id is
 * attended, as codebert_mlm(input_ids_) in get_substitutes.py:62):
 *   scores_out device float [L, k], ids_out device int32 [L, k] (descending, ties by lower id). */
int ae_mlm_topk(ae_engine *eng, const int32_t *ids, int32_t L, int32_t k, float *scores_out,
                int32_t *ids_out, void *stream);

/* Mutant population builder on token ids.
 *   word_tok   device int32 [n_word_tok]     concatenated token ids of every distinct word
 *   word_off   device int32 [n_words+1]      offsets into word_tok
 *   mut_words  device int32 [sum n_words_m]  word-id sequence of each mutant
 *   mut_off    device int32 [n_mut+1]        offsets into mut_words
 *   ids_out    device int32 [n_mut, L]       [cls] + first L-2 tokens + [sep] + pad
 *   lens_out   device int32 [n_mut]          non-pad count of each row (ae_score's lens)
 */
int ae_splice(const int32_t *word_tok, const int32_t *word_off, const int32_t *mut_words,
              const int32_t *mut_off, int32_t n_mut, int32_t L, int32_t cls_id, int32_t sep_id,
              int32_t pad_id, int32_t *ids_out, int32_t *lens_out, void *stream);

/* Row-wise top-k of a [rows, cols] float matrix (device), descending, ties by lower index. */
int ae_topk(const float *x, int32_t rows, int32_t cols, int32_t k, float *vals_out,
            int32_t *idx_out, void *stream);

/* sims_out[i] = (1/span_len) * sum_{t<span_len} cos(ref[t], cand[i, t]) with eps clamp
 *   ref  device float [span_len, hidden], cand device float [n, span_len, hidden]. */
int ae_cosine_rank(const float *ref, const float *cand, int32_t n, int32_t span_len, int32_t hidden,
                   float eps, float *sims_out, void *stream);

/* The bit-packed mask ae_score_graph reads (mask_bits device uint32 [n, L, L/32], bit j of word
 * w = key 32 w + j) from the compact per-query features ah_gcb_features_batch emits (all device
 * int32): ids [n, L]; meta [n, 4] = node_index, max_length, nodes, edges; spans [n, L] = node k's
 * code span a | b << 16 or -1; edges [n, e_cap] = node | target << 16.  L % 32 == 0, L <= 1024. */
int ae_graph_mask(const int32_t *ids, const int32_t *meta, const int32_t *spans,
                  const int32_t *edges, int32_t n, int32_t L, int32_t e_cap, uint32_t *mask_bits,
                  void *stream);

/* Profiling of the dominant kernel: when enabled, the engine brackets every launch of kernel
 * class `kind` with HIP events on the launch stream.  ae_kernel_time synchronises and returns the
 * summed milliseconds, launch count and algorithmic FLOP of those launches, then resets. */
#define AE_KIND_GEMM_FFN1 0
#define AE_KIND_GEMM_ANY 1
#define AE_KIND_ATTENTION 2
int ae_set_profiling(ae_engine *eng, int32_t kind, int32_t enabled);
int ae_kernel_time(ae_engine *eng, double *ms_total, int64_t *launches, double *flop_total);

const char *ae_last_error(void);
const char *ae_version(void);
/* Hash of the sources this library was built from (attack-pretrain-models-of-code_amd/
 * buildinfo.py); the Python loader refuses a library whose hash differs from its tree. */
const char *ae_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* ALERT_ENGINE_H */
