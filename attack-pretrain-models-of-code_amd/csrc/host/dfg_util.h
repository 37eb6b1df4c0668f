// dfg_util.h — the bookkeeping shared by the DFG_c / DFG_java / DFG_python restatements
// (python_parser/parser_folder/DFG_*.py): idx-stable sorting, the (code, idx, relation) merge of
// loop bodies, and the state union of if statements.
#pragma once
#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "host.h"

namespace ah {

using DfgStates = std::map<std::string, std::vector<int>>;

// sorted(DFG, key=lambda x: x[1]) — Python's sort is stable
inline void dfg_sort(std::vector<DfgEdge>& d) {
  std::stable_sort(d.begin(), d.end(),
                   [](const DfgEdge& a, const DfgEdge& b) { return a.idx < b.idx; });
}

inline void dfg_append(std::vector<DfgEdge>& a, std::vector<DfgEdge>&& b) {
  a.insert(a.end(), std::make_move_iterator(b.begin()), std::make_move_iterator(b.end()));
}

// for / while bodies: entries with the same (code, idx, relation) are merged — from-codes as a
// set, from-idxs as a sorted set — then ordered by idx over first-seen order (DFG_*.py `dic`)
inline void dfg_merge_dup(std::vector<DfgEdge>& d) {
  std::map<std::tuple<std::string, int, int>, size_t> pos;
  std::vector<DfgEdge> out;
  for (auto& e : d) {
    auto key = std::make_tuple(e.code, e.idx, (int)e.computed);
    auto it = pos.find(key);
    if (it == pos.end()) {
      pos[key] = out.size();
      out.push_back(e);
    } else {
      DfgEdge& m = out[it->second];
      for (auto& c : e.from_code)
        if (std::find(m.from_code.begin(), m.from_code.end(), c) == m.from_code.end())
          m.from_code.push_back(c);
      std::set<int> s(m.from_idx.begin(), m.from_idx.end());
      s.insert(e.from_idx.begin(), e.from_idx.end());
      m.from_idx.assign(s.begin(), s.end());
    }
  }
  dfg_sort(out);
  d.swap(out);
}

// if statements: the union of every branch's states (and the incoming states when there is no
// else), each list deduplicated and sorted
inline DfgStates dfg_union(const std::vector<DfgStates>& dicts) {
  DfgStates merged;
  for (auto& dic : dicts)
    for (auto& kv : dic) {
      auto& m = merged[kv.first];
      m.insert(m.end(), kv.second.begin(), kv.second.end());
    }
  for (auto& kv : merged) {
    std::set<int> s(kv.second.begin(), kv.second.end());
    kv.second.assign(s.begin(), s.end());
  }
  return merged;
}

}  // namespace ah
