// mutate.cpp — identifier substitution at the text level, exactly as the reference applies it.
//
//   get_example        python_parser/run_parser.py:218-239
//   get_example_batch  python_parser/run_parser.py:242-266 (map_chromesome, utils.py:116-120)
//
// Both re-parse `code.replace("\\n", "\n")` (so "\n" escape sequences inside string literals turn
// into real line breaks in every mutant), collect the leaves whose text equals a target word, and
// splice the substitute into the LINE strings at the leaf's tree-sitter columns.  tree-sitter
// columns are byte offsets but the reference slices Python str lines with them, i.e. uses them as
// code-point indices; lines are therefore kept as code-point arrays and indexed with byte columns.
// get_example shifts the k-th same-line occurrence by k*diff; get_example_batch applies a line's
// edits in chromosome-key order with a running diff (the documented offset quirk).
#include <algorithm>
#include "host.h"

namespace ah {

namespace {
std::string replace_backslash_n(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 1 < s.size() && s[i + 1] == 'n') {
      out.push_back('\n');
      ++i;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

// Python slicing semantics on a code-point line: line[:a] + sub + line[b:] with clamped indices
void splice_line(std::vector<uint32_t>& line, long a, long b, const std::vector<uint32_t>& sub) {
  const long n = (long)line.size();
  auto clamp = [n](long x) {
    if (x < 0) x += n;
    if (x < 0) x = 0;
    if (x > n) x = n;
    return x;
  };
  const long ca = clamp(a), cb = clamp(b);
  std::vector<uint32_t> out(line.begin(), line.begin() + ca);
  out.insert(out.end(), sub.begin(), sub.end());
  out.insert(out.end(), line.begin() + cb, line.end());
  line.swap(out);
}

std::string lines_to_string(const std::vector<std::vector<uint32_t>>& lines) {
  std::string out;
  for (size_t k = 0; k < lines.size(); ++k) {
    if (k) out.push_back('\n');
    for (uint32_t cp : lines[k]) utf8_append(out, cp);
  }
  return out;
}
}  // namespace

// remove_comments_and_docstrings(source, lang) for C / Java
// (python_parser/parser_folder/utils.py:30-87, non-Python branch): re.sub of
//   //.*?$ | /\*.*?\*/ | '(?:\\.|[^\\'])*' | "(?:\\.|[^\\"])*"   (DOTALL | MULTILINE)
// where comments become " " and literals are kept, then whitespace-only lines are dropped.
// Emulated by a leftmost scanner (all pattern characters are ASCII, so bytes == code points).
std::string remove_comments(const std::string& src) {
  std::string out;
  const size_t n = src.size();
  size_t i = 0;
  auto quoted = [&](size_t p, char q, size_t& end) {
    size_t j = p + 1;
    while (j < n) {
      if (src[j] == '\\') {
        if (j + 1 >= n) return false;
        j += 2;
        continue;
      }
      if (src[j] == q) {
        end = j + 1;
        return true;
      }
      ++j;
    }
    return false;
  };
  while (i < n) {
    const char c = src[i];
    if (c == '/' && i + 1 < n && src[i + 1] == '/') {
      size_t j = i + 2;
      while (j < n && src[j] != '\n') ++j;
      out.push_back(' ');
      i = j;
      continue;
    }
    if (c == '/' && i + 1 < n && src[i + 1] == '*') {
      const size_t e = src.find("*/", i + 2);
      if (e != std::string::npos) {
        out.push_back(' ');
        i = e + 2;
        continue;
      }
    }
    if (c == '\'' || c == '"') {
      size_t end = 0;
      if (quoted(i, c, end)) {
        out.append(src, i, end - i);
        i = end;
        continue;
      }
    }
    out.push_back(c);
    ++i;
  }
  // drop lines whose strip() is empty
  std::string res;
  bool first = true;
  for (const std::string& line : split_lines(out)) {
    bool blank = true;
    for (size_t k = 0; k < line.size() && blank;) {
      if (!py_isspace(utf8_next(line, k))) blank = false;
    }
    if (blank) continue;
    if (!first) res.push_back('\n');
    res += line;
    first = false;
  }
  return res;
}

void example_init(Example& ex, const std::string& code, Lang lang) {
  ex.lang = lang;
  ex.code = code;
  ex.rcode = replace_backslash_n(code);
  ex.leaves = lex(ex.rcode, lang);
  // get_identifiers -> extract_dataflow (run_parser.py:190-216): '\\n' -> newline, comments
  // removed (C / Java), then the leaves of that text are the code tokens
  ex.id_leaves = lang == LANG_PYTHON ? ex.leaves : lex(remove_comments(ex.rcode), lang);
  ex.lines_cp.clear();
  for (auto& l : split_lines(ex.rcode)) ex.lines_cp.push_back(utf8_decode(l));
  ex.leaf_index.clear();
  ex.line_leaves.assign(ex.lines_cp.size(), {});
  for (size_t i = 0; i < ex.leaves.size(); ++i) {
    ex.leaf_index[ex.leaves[i].text].push_back((int)i);
    if (ex.leaves[i].sl >= 0 && ex.leaves[i].sl < (int)ex.line_leaves.size())
      ex.line_leaves[ex.leaves[i].sl].push_back((int)i);
  }
}

std::vector<std::pair<int, std::vector<uint32_t>>> edit_lines(const Example& ex,
                                                              const std::vector<std::string>& tgts,
                                                              const std::vector<std::string>& subs) {
  // get_example(_batch) edits, per line, every occurrence of every chromosome name — names in
  // chromosome order, a name's occurrences in leaf order — each shifted by the diffs applied
  // before it on that line.  A line changes iff one of its edits changes the text: a name mapped
  // to itself splices its own text back with diff 0, which alters nothing on a line where every
  // edit is such, but after a real edit on the same line it lands shifted (the reference's
  // offset quirk), so it is applied there like any other.
  const size_t n = tgts.size();
  std::unordered_map<std::string, int> name_k;
  name_k.reserve(n * 2);
  for (size_t k = 0; k < n; ++k) name_k.emplace(tgts[k], (int)k);
  std::vector<int> touched;
  for (size_t k = 0; k < n; ++k) {
    if (tgts[k] == subs[k]) continue;
    auto hit = ex.leaf_index.find(tgts[k]);
    if (hit == ex.leaf_index.end()) continue;
    for (int li : hit->second) touched.push_back(ex.leaves[li].sl);
  }
  std::sort(touched.begin(), touched.end());
  touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
  std::vector<std::vector<uint32_t>> subcps(n);
  std::vector<long> diffs(n, 0);
  std::vector<char> decoded(n, 0);
  struct Edit {
    int k, li;
  };
  std::vector<Edit> edits;
  std::vector<std::pair<int, std::vector<uint32_t>>> out;
  out.reserve(touched.size());
  for (int line : touched) {
    edits.clear();
    for (int li : ex.line_leaves[line]) {
      auto it = name_k.find(ex.leaves[li].text);
      if (it != name_k.end()) edits.push_back({it->second, li});
    }
    std::sort(edits.begin(), edits.end(),
              [](const Edit& a, const Edit& b) { return a.k != b.k ? a.k < b.k : a.li < b.li; });
    std::vector<uint32_t> l = ex.lines_cp[line];
    long shift = 0;
    for (const Edit& e : edits) {
      if (!decoded[e.k]) {
        subcps[e.k] = utf8_decode(subs[e.k]);
        diffs[e.k] = (long)subcps[e.k].size() - (long)utf8_decode(tgts[e.k]).size();
        decoded[e.k] = 1;
      }
      const Leaf& lf = ex.leaves[e.li];
      splice_line(l, lf.sc + shift, lf.ec + shift, subcps[e.k]);
      shift += diffs[e.k];
    }
    out.emplace_back(line, std::move(l));
  }
  return out;
}

namespace {
std::string apply_edits(const Example& ex,
                        std::vector<std::pair<int, std::vector<uint32_t>>>&& edited) {
  std::vector<std::vector<uint32_t>> lines = ex.lines_cp;
  for (auto& e : edited) lines[e.first] = std::move(e.second);
  return lines_to_string(lines);
}
}  // namespace

std::string get_example(const Example& ex, const std::string& tgt, const std::string& sub) {
  return apply_edits(ex, edit_lines(ex, {tgt}, {sub}));
}

std::string get_example_batch(const Example& ex, const std::vector<std::string>& tgts,
                              const std::vector<std::string>& subs) {
  return apply_edits(ex, edit_lines(ex, tgts, subs));
}

std::vector<std::string> py_split(const std::string& s) {
  std::vector<std::string> words;
  size_t i = 0, start = std::string::npos;
  while (i < s.size()) {
    size_t j = i;
    const uint32_t cp = utf8_next(s, j);
    if (py_isspace(cp)) {
      if (start != std::string::npos) {
        words.push_back(s.substr(start, i - start));
        start = std::string::npos;
      }
    } else if (start == std::string::npos) {
      start = i;
    }
    i = j;
  }
  if (start != std::string::npos) words.push_back(s.substr(start));
  return words;
}

}  // namespace ah
