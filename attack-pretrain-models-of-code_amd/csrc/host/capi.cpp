// capi.cpp — extern "C" surface of libalert_host.so (include/alert_host.h).
#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>

#include "../../../include/alert_host.h"
#include "host.h"

struct ah_tokenizer {
  ah::Tokenizer t;
  // worker clones for the multi-threaded featurisers (the BPE caches are per object)
  std::mutex mu;
  std::vector<std::unique_ptr<ah::Tokenizer>> clones;
  std::vector<std::unique_ptr<std::unordered_map<std::string, std::vector<int32_t>>[]>> leaf_caches;
};

namespace ah {
struct GcbArgs {
  Lang lang;
  DfgVariant variant;
  bool normalize, run_trunc;
  int code_length, dfl, e_cap;
};
bool gcb_features_one(Tokenizer& t, std::unordered_map<std::string, std::vector<int32_t>>* cache,
                      const std::string& code_in, const GcbArgs& a, int32_t* ids, int32_t* pos,
                      int32_t* meta, int32_t* spans, int32_t* edges, std::string* err);
}  // namespace ah

struct ah_example {
  ah::Example ex;
  // word table for the device splice: (word, first) -> id, token runs
  std::unordered_map<std::string, int32_t> word_id[2];
  std::vector<int32_t> word_tok;
  std::vector<int32_t> word_off{0};
  // the word ids of every line of the original text (its first word in the "first" BPE form
  // when it is the text's first word), so a mutant re-splits only the lines its edits touch;
  // first_line: the first line that has words (-2: not built yet)
  std::vector<std::vector<int32_t>> line_ids;
  int32_t first_line = -2;
};

namespace {
thread_local std::string g_err;
int32_t fail(const std::string& m) {
  g_err = m;
  return -1;
}

// ' '.join(code.split()) -> tokenize -> [:L-2] -> [CLS] .. [SEP] -> pad (attacker.py:38-45)
void featurize_words(ah::Tokenizer& t, const std::vector<std::string>& words, int32_t L,
                     int32_t* ids, int32_t* len) {
  const int32_t cap = L - 2;
  int32_t n = 0;
  ids[0] = t.cls_id;
  for (size_t w = 0; w < words.size() && n < cap; ++w) {
    const std::vector<int32_t>& run = t.word_ids(words[w], w == 0);
    for (int32_t id : run) {
      if (n >= cap) break;
      ids[1 + n++] = id;
    }
  }
  ids[1 + n] = t.sep_id;
  for (int32_t k = n + 2; k < L; ++k) ids[k] = t.pad_id;
  // ae_score's lens = the non-pad count: a literal "<pad>" in the text tokenises to the pad id,
  // which the reference masks (attention_mask = ids.ne(1)) and the engine drops
  int32_t pads = 0;
  for (int32_t k = 1; k <= n; ++k) pads += ids[k] == t.pad_id;
  *len = n + 2 - pads;
}

// convert_code_to_features WITHOUT the whitespace normalisation (the Authorship-Attribution
// victim tokenises the raw source: CodeXGLUE/Authorship-Attribution/code/attacker.py:31-37)
void featurize_raw(ah::Tokenizer& t, const std::string& code, int32_t L, int32_t* ids,
                   int32_t* len) {
  std::vector<int32_t> toks;
  t.encode(code, toks);
  const int32_t n = std::min<int32_t>((int32_t)toks.size(), L - 2);
  ids[0] = t.cls_id;
  int32_t pads = 0;
  for (int32_t k = 0; k < n; ++k) {
    ids[1 + k] = toks[k];
    pads += toks[k] == t.pad_id;
  }
  ids[1 + n] = t.sep_id;
  for (int32_t k = n + 2; k < L; ++k) ids[k] = t.pad_id;
  *len = n + 2 - pads;
}

bool build_mutant(ah_example* e, int32_t mode, int32_t b, int32_t end, const char* const* tgts,
                  const char* const* subs, std::string& out) {
  if (mode == AH_MODE_SINGLE) {
    if (end - b != 1) return false;
    out = ah::get_example(e->ex, tgts[b], subs[b]);
    return true;
  }
  std::vector<std::string> tv, sv;
  for (int32_t k = b; k < end; ++k) {
    tv.emplace_back(tgts[k]);
    sv.emplace_back(subs[k]);
  }
  out = ah::get_example_batch(e->ex, tv, sv);
  return true;
}
}  // namespace

extern "C" {

const char* ah_last_error(void) { return g_err.c_str(); }

int32_t ah_gcb_features_batch(ah_tokenizer* tok, int32_t n, const char* const* codes, int32_t lang,
                              int32_t variant, int32_t flags, int32_t code_length,
                              int32_t data_flow_length, int32_t e_cap, int32_t threads,
                              int32_t* ids_out, int32_t* pos_out, int32_t* meta_out,
                              int32_t* spans_out, int32_t* edges_out) {
  if (!tok || (n > 0 && (!codes || !ids_out || !pos_out || !meta_out || !spans_out || !edges_out)))
    return fail("null argument");
  if (lang < 0 || lang > 2) return fail("unknown language");
  if (variant != AH_DFG_RUN_PARSER && variant != AH_DFG_GCB_RUN) return fail("unknown DFG variant");
  if (variant == AH_DFG_GCB_RUN && lang == AH_LANG_C)
    return fail("the GraphCodeBERT run.py data flow has no C walk (parser/DFG.py)");
  const int32_t L = code_length + data_flow_length;
  if (code_length < 4 || data_flow_length < 0 || L > 65535 || e_cap < 1) return fail("bad lengths");
  ah::GcbArgs a{(ah::Lang)lang, (ah::DfgVariant)variant, (flags & AH_GCB_NORMALIZE) != 0,
                (flags & AH_GCB_RUN_TRUNC) != 0, code_length, data_flow_length, e_cap};
  const int nthr = std::max(1, std::min(std::min(threads, n), 64));
  // the whole batch holds the tokenizer: its worker clones and their BPE / leaf caches are
  // shared state, so concurrent calls on one tokenizer serialise here
  std::lock_guard<std::mutex> g(tok->mu);
  while ((int)tok->clones.size() < nthr) {
    tok->clones.emplace_back(new ah::Tokenizer(tok->t));
    tok->leaf_caches.emplace_back(new std::unordered_map<std::string, std::vector<int32_t>>[2]);
  }
  std::vector<std::string> errs(nthr);
  std::vector<char> ok(nthr, 1);
  auto work = [&](int w) {
    for (int32_t i = w; i < n; i += nthr) {
      if (!ah::gcb_features_one(*tok->clones[w], tok->leaf_caches[w].get(), codes[i], a,
                                ids_out + (size_t)i * L, pos_out + (size_t)i * L,
                                meta_out + (size_t)i * 4, spans_out + (size_t)i * L,
                                edges_out + (size_t)i * e_cap, &errs[w])) {
        ok[w] = 0;
        return;
      }
    }
  };
  if (nthr == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int w = 1; w < nthr; ++w) pool.emplace_back(work, w);
    work(0);
    for (auto& th : pool) th.join();
  }
  for (int w = 0; w < nthr; ++w)
    if (!ok[w]) return fail(errs[w]);
  return n;
}

ah_tokenizer* ah_tokenizer_load(const char* vocab_json, const char* merges_txt) {
  auto* t = new ah_tokenizer();
  std::string err;
  if (!t->t.load(vocab_json, merges_txt, &err)) {
    g_err = err;
    delete t;
    return nullptr;
  }
  return t;
}

void ah_tokenizer_free(ah_tokenizer* t) { delete t; }

int32_t ah_tokenizer_special(ah_tokenizer* t, int32_t which) {
  switch (which) {
    case 0: return t->t.cls_id;
    case 1: return t->t.pad_id;
    case 2: return t->t.sep_id;
    case 3: return t->t.unk_id;
    case 4: return t->t.mask_id;
  }
  return fail("bad special index");
}

int32_t ah_tokenize(ah_tokenizer* t, const char* text, int32_t* out, int32_t cap) {
  if (!t || !text) return fail("null argument");
  std::vector<int32_t> ids;
  t->t.encode(text, ids);
  for (int32_t k = 0; k < (int32_t)ids.size() && k < cap; ++k) out[k] = ids[k];
  return (int32_t)ids.size();
}

int32_t ah_decode(ah_tokenizer* t, const int32_t* ids, int32_t n, char* out, int32_t cap) {
  if (!t || (!ids && n)) return fail("null argument");
  const std::string s = t->t.decode(ids, n);
  if (out && cap > 0) {
    const int32_t m = std::min<int32_t>(cap - 1, (int32_t)s.size());
    std::memcpy(out, s.data(), m);
    out[m] = 0;
  }
  return (int32_t)s.size() + 1;
}

int32_t ah_featurize_batch(ah_tokenizer* t, int32_t n, const char* const* codes, int32_t L,
                           int32_t* ids_out, int32_t* lens_out) {
  if (!t || !codes || !ids_out || !lens_out || L < 2) return fail("bad argument");
  for (int32_t i = 0; i < n; ++i)
    featurize_words(t->t, ah::py_split(codes[i]), L, ids_out + (size_t)i * L, lens_out + i);
  return n;
}

int32_t ah_featurize_batch_raw(ah_tokenizer* t, int32_t n, const char* const* codes, int32_t L,
                               int32_t* ids_out, int32_t* lens_out) {
  if (!t || !codes || !ids_out || !lens_out || L < 2) return fail("bad argument");
  for (int32_t i = 0; i < n; ++i)
    featurize_raw(t->t, codes[i], L, ids_out + (size_t)i * L, lens_out + i);
  return n;
}

int32_t ah_tokens_to_ids(ah_tokenizer* t, int32_t n, const char* const* tokens, int32_t* ids_out) {
  if (!t || (n && (!tokens || !ids_out))) return fail("bad argument");
  for (int32_t i = 0; i < n; ++i) ids_out[i] = t->t.token_to_id(tokens[i]);
  return n;
}

ah_example* ah_example_new(const char* code, int32_t lang) {
  if (!code || lang < 0 || lang > 2) {
    fail("bad argument");
    return nullptr;
  }
  auto* e = new ah_example();
  ah::example_init(e->ex, code, (ah::Lang)lang);
  return e;
}

void ah_example_free(ah_example* e) { delete e; }

int32_t ah_example_num_leaves(ah_example* e, int32_t which) {
  return (int32_t)(which ? e->ex.id_leaves : e->ex.leaves).size();
}

int32_t ah_example_leaves(ah_example* e, int32_t which, char* buf, int32_t cap) {
  const std::vector<ah::Leaf>& lv = which ? e->ex.id_leaves : e->ex.leaves;
  size_t need = 0;
  for (auto& lf : lv) need += lf.text.size() + 1;
  if (buf && (size_t)cap >= need) {
    size_t p = 0;
    for (auto& lf : lv) {
      std::memcpy(buf + p, lf.text.data(), lf.text.size());
      p += lf.text.size();
      buf[p++] = 0;
    }
  }
  return (int32_t)need;
}

int32_t ah_example_mutant_text(ah_example* e, int32_t mode, int32_t n_pairs,
                               const char* const* tgts, const char* const* subs, char* out,
                               int32_t cap) {
  if (!e) return fail("null example");
  std::string s;
  if (!build_mutant(e, mode, 0, n_pairs, tgts, subs, s)) return fail("single mode needs 1 pair");
  if (out && cap > 0) {
    const int32_t m = std::min<int32_t>(cap - 1, (int32_t)s.size());
    std::memcpy(out, s.data(), m);
    out[m] = 0;
  }
  return (int32_t)s.size() + 1;
}

int32_t ah_example_mutants(ah_example* e, ah_tokenizer* t, int32_t mode, int32_t n_mut,
                           const int32_t* pair_off, const char* const* tgts,
                           const char* const* subs, int32_t L, int32_t* ids_out,
                           int32_t* lens_out) {
  if (!e || !t || !pair_off || !ids_out || !lens_out || L < 2) return fail("bad argument");
  const bool raw = (mode & AH_MODE_RAW) != 0;
  mode &= ~AH_MODE_RAW;
  std::string code;
  for (int32_t m = 0; m < n_mut; ++m) {
    if (!build_mutant(e, mode, pair_off[m], pair_off[m + 1], tgts, subs, code))
      return fail("single mode needs 1 pair per mutant");
    if (raw) featurize_raw(t->t, code, L, ids_out + (size_t)m * L, lens_out + m);
    else featurize_words(t->t, ah::py_split(code), L, ids_out + (size_t)m * L, lens_out + m);
  }
  return n_mut;
}

namespace {
// id of (word, first) in the example's word table, added with its token run on first sight
int32_t word_lookup(ah_example* e, ah_tokenizer* t, const std::string& w, int first) {
  auto it = e->word_id[first].find(w);
  if (it != e->word_id[first].end()) return it->second;
  const std::vector<int32_t>& run = t->t.word_ids(w, first);
  const int32_t id = (int32_t)e->word_off.size() - 1;
  e->word_tok.insert(e->word_tok.end(), run.begin(), run.end());
  e->word_off.push_back((int32_t)e->word_tok.size());
  e->word_id[first].emplace(w, id);
  return id;
}

// the words of one line: py_split of its text (lines are joined by '\n', so the text's split is
// the concatenation of its lines' splits), each word assembled in one reused buffer
void line_words(ah_example* e, ah_tokenizer* t, const std::vector<uint32_t>& cps, int32_t line,
                std::vector<int32_t>& out) {
  thread_local std::string w;
  w.clear();
  int first = line == e->first_line ? 1 : 0;
  for (uint32_t cp : cps) {
    if (ah::py_isspace(cp)) {
      if (!w.empty()) {
        out.push_back(word_lookup(e, t, w, first));
        first = 0;
        w.clear();
      }
    } else {
      ah::utf8_append(w, cp);
    }
  }
  if (!w.empty()) out.push_back(word_lookup(e, t, w, first));
}

void ensure_line_ids(ah_example* e, ah_tokenizer* t) {
  if (e->first_line != -2) return;
  const auto& lines = e->ex.lines_cp;
  e->first_line = -1;
  for (size_t i = 0; i < lines.size() && e->first_line < 0; ++i)
    if (!ah::py_split(ah::utf8_encode(lines[i], 0, lines[i].size())).empty())
      e->first_line = (int32_t)i;
  e->line_ids.assign(lines.size(), {});
  for (size_t i = 0; i < lines.size(); ++i) line_words(e, t, lines[i], (int32_t)i, e->line_ids[i]);
}

// a substitute that cannot change which line holds the text's first word: non-empty, no
// whitespace (py_isspace over the ASCII and the common Unicode spaces, conservatively)
bool plain_sub(const char* s) {
  if (!s || !*s) return false;
  for (const unsigned char* p = (const unsigned char*)s; *p; ++p)
    if (*p <= 0x20 || *p == 0x7f || *p >= 0x80) return false;
  return true;
}
}  // namespace

int32_t ah_example_mutant_words(ah_example* e, ah_tokenizer* t, int32_t mode, int32_t n_mut,
                                const int32_t* pair_off, const char* const* tgts,
                                const char* const* subs, int32_t L, int32_t* mut_words,
                                int32_t cap_words, int32_t* mut_off, int32_t* lens_out) {
  if (!e || !t || !pair_off || !mut_off || !lens_out || L < 2) return fail("bad argument");
  ensure_line_ids(e, t);
  std::string code;
  std::vector<int32_t> seq;
  std::vector<std::string> tv, sv;
  mut_off[0] = 0;
  for (int32_t m = 0; m < n_mut; ++m) {
    const size_t seq0 = seq.size();
    const int32_t b = pair_off[m], end = pair_off[m + 1];
    if (mode == AH_MODE_SINGLE && end - b != 1) return fail("single mode needs 1 pair per mutant");
    bool plain = true;
    for (int32_t k = b; k < end && plain; ++k) plain = plain_sub(subs[k]);
    if (plain) {
      // only the lines the edits touch are re-split (ASCII identifiers in, so the text's first
      // word stays on first_line); the others reuse the original's word ids
      tv.assign(tgts + b, tgts + end);
      sv.assign(subs + b, subs + end);
      auto edited = ah::edit_lines(e->ex, tv, sv);  // in line order
      size_t q = 0;
      for (int32_t i = 0; i < (int32_t)e->line_ids.size(); ++i) {
        if (q < edited.size() && edited[q].first == i) {
          line_words(e, t, edited[q].second, i, seq);
          ++q;
        } else {
          seq.insert(seq.end(), e->line_ids[i].begin(), e->line_ids[i].end());
        }
      }
    } else {
      if (!build_mutant(e, mode, b, end, tgts, subs, code))
        return fail("single mode needs 1 pair per mutant");
      const std::vector<std::string> words = ah::py_split(code);
      for (size_t w = 0; w < words.size(); ++w)
        seq.push_back(word_lookup(e, t, words[w], w == 0 ? 1 : 0));
    }
    int32_t ntok = 0, pads = 0;
    for (size_t w = seq0; w < seq.size(); ++w) {
      const int32_t id = seq[w];
      for (int32_t k = e->word_off[id]; k < e->word_off[id + 1]; ++k, ++ntok)
        if (ntok < L - 2 && e->word_tok[k] == t->t.pad_id) ++pads;  // literal "<pad>" text
    }
    mut_off[m + 1] = (int32_t)seq.size();
    lens_out[m] = std::min(ntok, L - 2) + 2 - pads;  // non-pad count (ae_score's lens)
  }
  if ((int32_t)seq.size() > cap_words) return -(int32_t)seq.size();
  if (mut_words) std::memcpy(mut_words, seq.data(), seq.size() * 4);
  return (int32_t)seq.size();
}

int32_t ah_example_word_table(ah_example* e, int32_t* word_tok, int32_t cap_tok,
                              int32_t* word_off, int32_t cap_off, int32_t* n_words_out) {
  const int32_t nt = (int32_t)e->word_tok.size();
  const int32_t nw = (int32_t)e->word_off.size() - 1;
  *n_words_out = nw;
  if (word_tok && cap_tok >= nt) std::memcpy(word_tok, e->word_tok.data(), nt * 4);
  if (word_off && cap_off >= nw + 1) std::memcpy(word_off, e->word_off.data(), (nw + 1) * 4);
  return nt;
}

int32_t ah_example_identifiers(ah_example* e, char* buf, int32_t cap) {
  if (!e) return fail("null example");
  const std::vector<std::string> names = ah::dfg_names(e->ex.id_leaves, e->ex.lang);
  size_t need = 0;
  for (auto& s : names) need += s.size() + 1;
  if (buf && (size_t)cap >= need) {
    size_t p = 0;
    for (auto& s : names) {
      std::memcpy(buf + p, s.data(), s.size());
      p += s.size();
      buf[p++] = 0;
    }
  }
  return (int32_t)need;
}

int32_t ah_example_dfg(ah_example* e, int32_t* rows, int32_t cap_rows, int32_t* from_idx,
                       int32_t cap_from) {
  return ah_example_dfg_variant(e, AH_DFG_RUN_PARSER, rows, cap_rows, from_idx, cap_from);
}

int32_t ah_example_dfg_variant(ah_example* e, int32_t variant, int32_t* rows, int32_t cap_rows,
                               int32_t* from_idx, int32_t cap_from) {
  if (!e) return fail("null example");
  if (variant != AH_DFG_RUN_PARSER && variant != AH_DFG_GCB_RUN) return fail("unknown DFG variant");
  if (variant == AH_DFG_GCB_RUN && e->ex.lang == ah::LANG_C)
    return fail("the GraphCodeBERT run.py data flow has no C walk (parser/DFG.py)");
  const std::vector<ah::DfgEdge> d =
      ah::dfg_of(e->ex.id_leaves, e->ex.lang, (ah::DfgVariant)variant);
  int32_t nf = 0;
  for (auto& x : d) nf += (int32_t)x.from_idx.size();
  if (rows && cap_rows >= (int32_t)d.size() && from_idx && cap_from >= nf) {
    int32_t f = 0;
    for (size_t i = 0; i < d.size(); ++i) {
      rows[4 * i + 0] = d[i].idx;
      rows[4 * i + 1] = d[i].computed ? 1 : 0;
      rows[4 * i + 2] = f;
      rows[4 * i + 3] = (int32_t)d[i].from_idx.size();
      for (int k : d[i].from_idx) from_idx[f++] = k;
    }
  }
  if (cap_from < nf && rows) return -nf - 1;
  return (int32_t)d.size();
}

int32_t ah_remove_comments(const char* code, char* out, int32_t cap) {
  if (!code) return fail("null argument");
  const std::string s = ah::remove_comments(code);
  if (out && cap > 0) {
    const int32_t m = std::min<int32_t>(cap - 1, (int32_t)s.size());
    std::memcpy(out, s.data(), m);
    out[m] = 0;
  }
  return (int32_t)s.size() + 1;
}

}  // extern "C"
