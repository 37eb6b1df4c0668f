// host.h — internal C++ API of the host featurisation library (libalert_host.so).
//
// Replaces, on the host side of the victim query boundary:
//   RobertaTokenizer.tokenize / convert_tokens_to_ids   (byte-level BPE; reference call sites
//       CodeXGLUE/Defect-detection/code/attacker.py:38-45, utils.py:174-189)
//   tree-sitter leaf extraction                          (python_parser/parser_folder/utils.py:89-129)
//   get_example / get_example_batch                       (python_parser/run_parser.py:218-266)
//   convert_code_to_features                              (attacker.py:38-45)
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace ah {

// ------------------------------------------------------------------------------------ utf-8
// Decode one code point at s[i] (advances i).  Invalid bytes decode as themselves (U+FFFD-free).
uint32_t utf8_next(const std::string& s, size_t& i);
void utf8_append(std::string& out, uint32_t cp);
std::vector<uint32_t> utf8_decode(const std::string& s);
std::string utf8_encode(const std::vector<uint32_t>& cps, size_t b, size_t e);
bool py_isspace(uint32_t cp);  // Python str.split() whitespace

// ------------------------------------------------------------------------------------ BPE
class Tokenizer {
 public:
  bool load(const std::string& vocab_json, const std::string& merges_txt, std::string* err);
  // tokenize(text) ids, RobertaTokenizer semantics (special tokens split first).
  void encode(const std::string& text, std::vector<int32_t>& out);
  // ids of one whitespace-delimited word, with (" " + word) when !first; cached.
  const std::vector<int32_t>& word_ids(const std::string& word, bool first);
  int32_t cls_id = 0, sep_id = 2, pad_id = 1, unk_id = 3, mask_id = 50264;
  const std::string& id_to_token(int32_t id) const { return inv_[id]; }
  // convert_tokens_to_ids of one token string (unk_id when it is not in the vocabulary)
  int32_t token_to_id(const std::string& token) const {
    auto it = vocab_.find(token);
    return it == vocab_.end() ? unk_id : it->second;
  }
  size_t vocab_size() const { return inv_.size(); }
  // decode byte-level tokens to text (tokenizer._decode / convert_tokens_to_string)
  std::string decode(const int32_t* ids, int n) const;

 private:
  void encode_plain(const std::string& seg, std::vector<int32_t>& out);
  void bpe(const std::string& pretok, std::vector<int32_t>& out);
  std::unordered_map<std::string, int32_t> vocab_;
  std::vector<std::string> inv_;
  std::unordered_map<std::string, int32_t> ranks_;  // "a b" -> rank
  std::vector<std::string> byte_enc_;               // byte -> utf-8 of its unicode stand-in
  std::unordered_map<uint32_t, uint8_t> byte_dec_;  // stand-in code point -> byte
  std::unordered_map<std::string, std::vector<int32_t>> bpe_cache_;
  std::unordered_map<std::string, std::vector<int32_t>> word_cache_[2];
  std::vector<std::string> specials_;
};

// ------------------------------------------------------------------------------------ lexer
enum Lang { LANG_C = 0, LANG_JAVA = 1, LANG_PYTHON = 2 };

struct Leaf {
  int sl, sc, el, ec;  // start/end line, byte column (tree-sitter Point semantics)
  std::string text;    // index_to_code_token(start, end, lines): the code the reference records
  std::string raw;     // the token's own bytes (what the parser sees; differs from `text` on
                       // lines with non-ASCII code points, where the byte-column slice shifts)
  bool joined = false; // Python: a backslash line continuation precedes this leaf
};

// Leaves of `code` (already '\\n'-replaced by the caller when the reference does so).
std::vector<Leaf> lex(const std::string& code, Lang lang);

// ------------------------------------------------------------------------------------ mutants
std::vector<std::string> split_lines(const std::string& code);
std::string join_lines(const std::vector<std::string>& lines);

struct Example {
  Lang lang;
  std::string code;                // as given (func text)
  std::string rcode;               // code.replace("\\n", "\n")
  std::vector<Leaf> leaves;        // lex(rcode): the leaves get_example(_batch) edits
  std::vector<Leaf> id_leaves;     // lex(remove_comments(rcode)): get_identifiers code tokens
  std::vector<std::vector<uint32_t>> lines_cp;  // rcode.split('\n') as code points
  // leaf text -> indices into leaves, in leaf order (the edits get_example(_batch) makes for a
  // name, without scanning every leaf per name)
  std::unordered_map<std::string, std::vector<int>> leaf_index;
  std::vector<std::vector<int>> line_leaves;  // leaf indices by start line, in leaf order
};

void example_init(Example& ex, const std::string& code, Lang lang);
std::string remove_comments(const std::string& src);
// get_example (single variable, run_parser.py:218-239)
std::string get_example(const Example& ex, const std::string& tgt, const std::string& sub);
// get_example_batch (chromosome in dict order, run_parser.py:242-266)
std::string get_example_batch(const Example& ex, const std::vector<std::string>& tgts,
                              const std::vector<std::string>& subs);
// the lines either of them changes, in line order, with their new code points (every other
// line of ex.lines_cp is unchanged); both are this plus a join
std::vector<std::pair<int, std::vector<uint32_t>>> edit_lines(const Example& ex,
                                                              const std::vector<std::string>& tgts,
                                                              const std::vector<std::string>& subs);

// ------------------------------------------------------------------------------------ DFG
// One DFG_c entry (python_parser/parser_folder/DFG_c.py): (code, idx, 'comesFrom' |
// 'computedFrom', [from codes], [from idxs]); idx = leaf index.
struct DfgEdge {
  std::string code;
  int idx;
  bool computed;  // 'computedFrom' (update_expression) vs 'comesFrom'
  std::vector<std::string> from_code;
  std::vector<int> from_idx;
};
// DFG of C leaves (dfg.cpp), sorted by idx as extract_dataflow returns it (run_parser.py:213)
std::vector<DfgEdge> dfg_c(const std::vector<Leaf>& leaves);
// DFG_java / DFG_python over Java / Python leaves (dfg_java.cpp, dfg_python.cpp); ms = the
// GraphCodeBERT parser/DFG.py variant of the walk (GraphCodeBERT/*/code/parser/DFG.py)
std::vector<DfgEdge> dfg_java(const std::vector<Leaf>& leaves, bool ms = false);
std::vector<DfgEdge> dfg_python(const std::vector<Leaf>& leaves, bool ms = false);
// the DFG of a language: variant 0 = python_parser/run_parser.py extract_dataflow; variant 1 =
// GraphCodeBERT/*/code/run.py extract_dataflow (parser/DFG.py walk, then only entries that have
// or are the source of an edge); C has variant 0 only
enum DfgVariant { DFG_RUN_PARSER = 0, DFG_GCB_RUN = 1 };
std::vector<DfgEdge> dfg_of(const std::vector<Leaf>& leaves, Lang lang,
                            DfgVariant variant = DFG_RUN_PARSER);
// unique DFG names in graph order (get_identifiers before the validity filter, run_parser.py:272)
std::vector<std::string> dfg_names(const std::vector<Leaf>& leaves, Lang lang);

// ' '.join(code.split()) words
std::vector<std::string> py_split(const std::string& s);

}  // namespace ah
