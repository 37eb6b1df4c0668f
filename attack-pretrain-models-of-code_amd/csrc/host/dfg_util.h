// dfg_util.h — the bookkeeping shared by the DFG_c / DFG_java / DFG_python restatements
// (python_parser/parser_folder/DFG_*.py): idx-stable sorting, the (code, idx, relation) merge of
// loop bodies, and the state union of if statements.
#pragma once
#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "host.h"

namespace ah {

using DfgStates = std::map<std::string, std::vector<int>>;

// sorted(DFG, key=lambda x: x[1]) — Python's sort is stable
// (a stable sort of an already ordered list is the identity, and most walk results arrive in leaf
// order, so the O(n) check skips the sort's buffer and moves)
inline void dfg_sort(std::vector<DfgEdge>& d) {
  auto by_idx = [](const DfgEdge& a, const DfgEdge& b) { return a.idx < b.idx; };
  if (std::is_sorted(d.begin(), d.end(), by_idx)) return;
  std::stable_sort(d.begin(), d.end(), by_idx);
}

inline void dfg_append(std::vector<DfgEdge>& a, std::vector<DfgEdge>&& b) {
  if (a.empty()) {
    a.swap(b);
    return;
  }
  a.insert(a.end(), std::make_move_iterator(b.begin()), std::make_move_iterator(b.end()));
}

// for / while bodies: entries with the same (code, idx, relation) are merged — from-codes as a
// set, from-idxs as a sorted set — then ordered by idx over first-seen order (DFG_*.py `dic`)
inline void dfg_merge_dup(std::vector<DfgEdge>& d) {
  // (idx, relation) -> positions in out; the code string is compared within the bucket
  std::unordered_map<long long, std::vector<size_t>> pos;
  pos.reserve(d.size());
  std::vector<DfgEdge> out;
  out.reserve(d.size());
  for (auto& e : d) {
    auto& bucket = pos[(long long)e.idx * 2 + (e.computed ? 1 : 0)];
    size_t hit = (size_t)-1;
    for (size_t p : bucket)
      if (out[p].code == e.code) {
        hit = p;
        break;
      }
    if (hit == (size_t)-1) {
      bucket.push_back(out.size());
      out.push_back(std::move(e));
    } else {
      DfgEdge& m = out[hit];
      for (auto& c : e.from_code)
        if (std::find(m.from_code.begin(), m.from_code.end(), c) == m.from_code.end())
          m.from_code.push_back(c);
      m.from_idx.insert(m.from_idx.end(), e.from_idx.begin(), e.from_idx.end());
      std::sort(m.from_idx.begin(), m.from_idx.end());
      m.from_idx.erase(std::unique(m.from_idx.begin(), m.from_idx.end()), m.from_idx.end());
    }
  }
  dfg_sort(out);
  d.swap(out);
}

// if statements: the union of every branch's states (and the incoming states when there is no
// else), each list deduplicated and sorted.  The maps are key-ordered, so the union merges each
// into the first in one linear pass; a key's lists are concatenated (a list equal to the one
// already there adds nothing to the set) and sorted + deduplicated at the end (= sorted(set)).
inline DfgStates dfg_union(std::vector<DfgStates>&& dicts) {
  if (dicts.empty()) return {};
  DfgStates merged = std::move(dicts[0]);
  for (size_t d = 1; d < dicts.size(); ++d) {
    auto bi = merged.begin();
    for (auto& kv : dicts[d]) {
      while (bi != merged.end() && bi->first < kv.first) ++bi;
      if (bi != merged.end() && bi->first == kv.first) {
        if (bi->second != kv.second)
          bi->second.insert(bi->second.end(), kv.second.begin(), kv.second.end());
      } else {
        bi = merged.emplace_hint(bi, kv.first, std::move(kv.second));
      }
    }
  }
  for (auto& kv : merged) {
    auto& v = kv.second;
    if (std::adjacent_find(v.begin(), v.end(), [](int a, int b) { return a >= b; }) != v.end()) {
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
    }
  }
  return merged;
}

}  // namespace ah
