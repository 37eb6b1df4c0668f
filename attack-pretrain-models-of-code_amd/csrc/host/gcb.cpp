// gcb.cpp — GraphCodeBERT query featurisation for a batch of texts, multi-threaded.
//
// convert_code_to_features of the GraphCodeBERT attackers
// (GraphCodeBERT/Defect-detection/code/attacker.py:30-63, Authorship-Attribution/code/
// attacker.py:52-88, clonedetection/code/attacker.py:33-72 and run.py:148-192 for the original
// pair) restated over the host lexer / DFG builders, with the graph mask left COMPACT: instead of
// the bool [L, L] GraphCodeDataset builds per query (utils.py:547-570), every query leaves
//   meta  [4]      node_index (= code-segment length), max_length (= node_index + nodes),
//                  nodes, edges
//   spans [L]      node k: dfg_to_code[k] as a | b << 16 when both ends lie inside the code
//                  segment (the only spans the mask uses), else -1
//   edges [e_cap]  node | target << 16 for every dfg_to_dfg entry whose column is inside L
// and the device builds the bits from them (ae_graph_mask, rowops.hip).  Queries are independent:
// they are split over worker threads, each with its own tokenizer clone (the BPE caches are not
// shared).  Parity with graph.py convert_code_to_features: tests/test_graph.py.
#include <algorithm>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "host.h"

namespace ah {

struct GcbArgs {  // keep in sync with capi.cpp
  Lang lang;
  DfgVariant variant;
  bool normalize, run_trunc;
  int code_length, dfl, e_cap;
};

namespace {
// tokenizer.tokenize(x) (first leaf) or tokenizer.tokenize('@ ' + x)[1:] (attacker.py:35)
const std::vector<int32_t>& leaf_ids(Tokenizer& t, std::unordered_map<std::string, std::vector<int32_t>>* cache,
                                     const std::string& leaf, bool first) {
  auto& c = cache[first ? 0 : 1];
  auto it = c.find(leaf);
  if (it != c.end()) return it->second;
  std::vector<int32_t> ids;
  if (first) {
    t.encode(leaf, ids);
  } else {
    t.encode("@ " + leaf, ids);
    if (!ids.empty()) ids.erase(ids.begin());
  }
  return c.emplace(leaf, std::move(ids)).first->second;
}
}  // namespace

// One query.  Returns false (with *err) if the edges exceed e_cap.
bool gcb_features_one(Tokenizer& t, std::unordered_map<std::string, std::vector<int32_t>>* cache,
                      const std::string& code_in, const GcbArgs& a, int32_t* ids, int32_t* pos,
                      int32_t* meta, int32_t* spans, int32_t* edges, std::string* err) {
  std::string code = code_in;
  if (a.normalize) {
    const std::vector<std::string> w = py_split(code_in);
    code.clear();
    for (size_t k = 0; k < w.size(); ++k) {
      if (k) code.push_back(' ');
      code += w[k];
    }
  }
  Example ex;
  example_init(ex, code, a.lang);
  const std::vector<DfgEdge> dfg_all = dfg_of(ex.id_leaves, a.lang, a.variant);
  const size_t nt = ex.id_leaves.size();
  std::vector<int64_t> ends(nt + 1, 0);
  std::vector<int32_t> flat;
  for (size_t i = 0; i < nt; ++i) {
    const std::vector<int32_t>& r = leaf_ids(t, cache, ex.id_leaves[i].text, i == 0);
    flat.insert(flat.end(), r.begin(), r.end());
    ends[i + 1] = (int64_t)flat.size();
  }
  const int total = a.code_length + a.dfl;
  const int ndfg = (int)dfg_all.size();
  size_t keep;
  if (a.run_trunc) {  // clonedetection/code/run.py:166: one token fewer, at most 509
    const long k1 = (long)total - 3 - std::min(ndfg, a.dfl);
    keep = (size_t)std::max<long>(0, std::min<long>({k1, (long)flat.size(), 512 - 3}));
  } else {
    const long k1 = (long)total - 2 - std::min(ndfg, a.dfl);
    keep = (size_t)std::max<long>(0, std::min<long>(k1, (long)flat.size()));
  }
  const int pad = t.pad_id;
  int L = 0;
  ids[L] = t.cls_id;
  pos[L] = pad + 1;
  ++L;
  for (size_t k = 0; k < keep; ++k, ++L) {
    ids[L] = flat[k];
    pos[L] = pad + 1 + L;
  }
  ids[L] = t.sep_id;
  pos[L] = pad + 1 + L;
  ++L;
  const int ni = L;                                      // code segment (positions > 1)
  const int nn = std::max(0, std::min(ndfg, total - ni));  // dfg[:total - len(source)]
  for (int k = 0; k < nn; ++k, ++L) {
    ids[L] = t.unk_id;
    pos[L] = 0;
  }
  for (; L < total; ++L) {
    ids[L] = pad;
    pos[L] = pad;
  }
  // reverse_index = {x[1]: i for i, x in enumerate(dfg)}: the last entry of a leaf index wins
  std::unordered_map<int, int> rev;
  for (int k = 0; k < nn; ++k) rev[dfg_all[k].idx] = k;
  int ne = 0;
  for (int k = 0; k < nn; ++k) {
    const DfgEdge& d = dfg_all[k];
    const int64_t sa = ends[d.idx] + 1, sb = ends[d.idx + 1] + 1;  // dfg_to_code[k]
    spans[k] = (sa < ni && sb < ni) ? (int32_t)(sa | (sb << 16)) : -1;
    for (int f : d.from_idx) {
      auto it = rev.find(f);
      if (it == rev.end() || ni + it->second >= total) continue;
      if (ne >= a.e_cap) {
        *err = "graph features: more than e_cap data-flow edges in one query";
        return false;
      }
      edges[ne++] = k | (it->second << 16);
    }
  }
  for (int k = nn; k < total; ++k) spans[k] = -1;
  meta[0] = ni;
  meta[1] = ni + nn;
  meta[2] = nn;
  meta[3] = ne;
  return true;
}

}  // namespace ah
