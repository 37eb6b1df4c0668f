// bpe.cpp — byte-level BPE with RobertaTokenizer semantics.
//
// Semantics pinned by tests/test_host.py against the installed transformers 5.15.0
// RobertaTokenizer (tokenizers 0.22.2 ByteLevel pre-tokeniser + BPE) on the same vocab/merges:
//   1. special (added) tokens <s> <pad> </s> <unk> <mask> are split out of the text first
//      (leftmost-longest, no lstrip/rstrip);
//   2. each remaining segment is split by the GPT-2 pattern
//      's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
//   3. each piece is mapped byte -> printable stand-in (bytes_to_unicode) and merged by rank.
#include <algorithm>
#include <climits>
#include <cstring>
#include <fstream>
#include <sstream>

#include "host.h"
#include "unicode_tables.h"

namespace ah {

uint32_t utf8_next(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  auto cont = [&](size_t k) { return k < s.size() && ((unsigned char)s[k] & 0xC0) == 0x80; };
  if (c < 0x80) { i += 1; return c; }
  if ((c & 0xE0) == 0xC0 && cont(i + 1)) {
    uint32_t cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F);
    i += 2;
    return cp;
  }
  if ((c & 0xF0) == 0xE0 && cont(i + 1) && cont(i + 2)) {
    uint32_t cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    i += 3;
    return cp;
  }
  if ((c & 0xF8) == 0xF0 && cont(i + 1) && cont(i + 2) && cont(i + 3)) {
    uint32_t cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) |
                  (s[i + 3] & 0x3F);
    i += 4;
    return cp;
  }
  i += 1;  // invalid byte: pass through (input comes from Python str -> valid UTF-8)
  return c;
}

void utf8_append(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

std::vector<uint32_t> utf8_decode(const std::string& s) {
  std::vector<uint32_t> out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) out.push_back(utf8_next(s, i));
  return out;
}

std::string utf8_encode(const std::vector<uint32_t>& cps, size_t b, size_t e) {
  std::string out;
  for (size_t i = b; i < e && i < cps.size(); ++i) utf8_append(out, cps[i]);
  return out;
}

bool py_isspace(uint32_t cp) {
  if (cp <= 0x20) return cp == 0x20 || (cp >= 0x09 && cp <= 0x0D) || (cp >= 0x1C && cp <= 0x1F);
  return cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) ||
         cp == 0x2028 || cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000;
}

namespace {
template <size_t N>
bool in_ranges(const uint32_t (&r)[N][2], uint32_t cp) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (cp < r[mid][0]) hi = mid;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}
bool is_L(uint32_t cp) {
  if (cp < 0x80) return (cp >= 'a' && cp <= 'z') || (cp >= 'A' && cp <= 'Z');
  return in_ranges(kUniLetter, cp);
}
bool is_N(uint32_t cp) {
  if (cp < 0x80) return cp >= '0' && cp <= '9';
  return in_ranges(kUniNumber, cp);
}
// regex \s (Unicode White_Space)
bool is_S(uint32_t cp) {
  if (cp <= 0x20) return cp == 0x20 || (cp >= 0x09 && cp <= 0x0D);
  return cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) ||
         cp == 0x2028 || cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000;
}
bool is_P(uint32_t cp) { return !is_S(cp) && !is_L(cp) && !is_N(cp); }

// JSON string literal parser (vocab.json keys), returns position after closing quote.
size_t json_string(const std::string& s, size_t i, std::string& out) {
  // s[i] == '"'
  ++i;
  out.clear();
  while (i < s.size() && s[i] != '"') {
    if (s[i] == '\\') {
      const char e = s[i + 1];
      i += 2;
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'u': {
          uint32_t cp = (uint32_t)std::stoul(s.substr(i, 4), nullptr, 16);
          i += 4;
          if (cp >= 0xD800 && cp <= 0xDBFF && s[i] == '\\' && s[i + 1] == 'u') {
            const uint32_t lo = (uint32_t)std::stoul(s.substr(i + 2, 4), nullptr, 16);
            i += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8_append(out, cp);
          break;
        }
        default: out.push_back(e);
      }
    } else {
      out.push_back(s[i++]);
    }
  }
  return i + 1;
}
}  // namespace

bool Tokenizer::load(const std::string& vocab_json, const std::string& merges_txt,
                     std::string* err) {
  std::ifstream fv(vocab_json, std::ios::binary);
  if (!fv) { *err = "cannot open " + vocab_json; return false; }
  std::stringstream ss;
  ss << fv.rdbuf();
  const std::string s = ss.str();
  size_t i = s.find('{');
  if (i == std::string::npos) { *err = "bad vocab json"; return false; }
  ++i;
  std::string key;
  int32_t max_id = -1;
  while (true) {
    while (i < s.size() && s[i] != '"' && s[i] != '}') ++i;
    if (i >= s.size() || s[i] == '}') break;
    i = json_string(s, i, key);
    while (i < s.size() && (s[i] == ':' || s[i] == ' ')) ++i;
    size_t j = i;
    while (j < s.size() && (s[j] == '-' || (s[j] >= '0' && s[j] <= '9'))) ++j;
    const int32_t id = (int32_t)std::stol(s.substr(i, j - i));
    i = j;
    vocab_[key] = id;
    max_id = std::max(max_id, id);
  }
  inv_.assign(max_id + 1, std::string());
  for (auto& kv : vocab_) inv_[kv.second] = kv.first;
  std::ifstream fm(merges_txt, std::ios::binary);
  if (!fm) { *err = "cannot open " + merges_txt; return false; }
  std::string line;
  int32_t rank = 0;
  while (std::getline(fm, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.rfind("#version", 0) == 0 || line.empty()) continue;
    ranks_[line] = rank++;
  }
  // GPT-2 bytes_to_unicode
  byte_enc_.assign(256, std::string());
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
  std::vector<bool> have(256, false);
  for (int b : bs) have[b] = true;
  int n = 0;
  for (int b = 0; b < 256; ++b) {
    uint32_t cp;
    if (have[b]) cp = (uint32_t)b;
    else cp = 256 + (n++);
    std::string u;
    utf8_append(u, cp);
    byte_enc_[b] = u;
    byte_dec_[cp] = (uint8_t)b;
  }
  auto id_of = [&](const char* t, int32_t dflt) {
    auto it = vocab_.find(t);
    return it == vocab_.end() ? dflt : it->second;
  };
  cls_id = id_of("<s>", 0);
  pad_id = id_of("<pad>", 1);
  sep_id = id_of("</s>", 2);
  unk_id = id_of("<unk>", 3);
  mask_id = id_of("<mask>", 50264);
  specials_ = {"<s>", "<pad>", "</s>", "<unk>", "<mask>"};
  return true;
}

void Tokenizer::bpe(const std::string& pretok, std::vector<int32_t>& out) {
  auto it = bpe_cache_.find(pretok);
  if (it != bpe_cache_.end()) {
    out.insert(out.end(), it->second.begin(), it->second.end());
    return;
  }
  std::vector<std::string> sym;
  for (unsigned char c : pretok) sym.push_back(byte_enc_[c]);
  std::string key;
  while (sym.size() > 1) {
    int32_t best = INT32_MAX;
    size_t bi = 0;
    for (size_t k = 0; k + 1 < sym.size(); ++k) {
      key.assign(sym[k]);
      key.push_back(' ');
      key.append(sym[k + 1]);
      auto r = ranks_.find(key);
      if (r != ranks_.end() && r->second < best) {
        best = r->second;
        bi = k;
      }
    }
    if (best == INT32_MAX) break;
    const std::string a = sym[bi], b = sym[bi + 1];
    std::vector<std::string> nxt;
    nxt.reserve(sym.size());
    for (size_t k = 0; k < sym.size();) {
      if (k + 1 < sym.size() && sym[k] == a && sym[k + 1] == b) {
        nxt.push_back(a + b);
        k += 2;
      } else {
        nxt.push_back(sym[k]);
        k += 1;
      }
    }
    sym.swap(nxt);
  }
  std::vector<int32_t> ids;
  ids.reserve(sym.size());
  for (auto& t : sym) {
    auto v = vocab_.find(t);
    ids.push_back(v == vocab_.end() ? unk_id : v->second);
  }
  out.insert(out.end(), ids.begin(), ids.end());
  bpe_cache_.emplace(pretok, std::move(ids));
}

void Tokenizer::encode_plain(const std::string& seg, std::vector<int32_t>& out) {
  const std::vector<uint32_t> cp = utf8_decode(seg);
  const size_t n = cp.size();
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    const uint32_t c = cp[i];
    // 's|'t|'re|'ve|'m|'ll|'d
    if (c == '\'' && i + 1 < n) {
      const uint32_t d = cp[i + 1];
      if (d == 's' || d == 't' || d == 'm' || d == 'd') j = i + 2;
      else if (i + 2 < n && ((d == 'r' && cp[i + 2] == 'e') || (d == 'v' && cp[i + 2] == 'e') ||
                             (d == 'l' && cp[i + 2] == 'l')))
        j = i + 3;
    }
    if (j == i) {
      const size_t s0 = (c == ' ' && i + 1 < n) ? i + 1 : i;  // optional leading space
      auto run = [&](size_t from, bool (*pred)(uint32_t)) {
        size_t k = from;
        while (k < n && pred(cp[k])) ++k;
        return k;
      };
      for (auto pred : {is_L, is_N, is_P}) {
        if (s0 < n && pred(cp[s0])) { j = run(s0, pred); break; }
        if (s0 != i && pred(cp[i])) { j = run(i, pred); break; }
      }
    }
    if (j == i) {
      // whitespace run
      size_t k = i;
      while (k < n && is_S(cp[k])) ++k;
      const size_t r = k - i;
      if (k == n) j = k;                 // \s+(?!\S) at end
      else if (r >= 2) j = k - 1;        // backtrack one: followed by the last space
      else j = k;                        // \s+
    }
    if (j == i) j = i + 1;  // unreachable safeguard
    bpe(utf8_encode(cp, i, j), out);
    i = j;
  }
}

void Tokenizer::encode(const std::string& text, std::vector<int32_t>& out) {
  size_t start = 0, i = 0;
  while (i < text.size()) {
    if (text[i] == '<') {
      size_t best = 0;
      int32_t bid = -1;
      for (auto& sp : specials_) {
        if (sp.size() > best && text.compare(i, sp.size(), sp) == 0) {
          best = sp.size();
          bid = vocab_[sp];
        }
      }
      if (best) {
        if (i > start) encode_plain(text.substr(start, i - start), out);
        out.push_back(bid);
        i += best;
        start = i;
        continue;
      }
    }
    ++i;
  }
  if (start < text.size()) encode_plain(text.substr(start), out);
}

const std::vector<int32_t>& Tokenizer::word_ids(const std::string& word, bool first) {
  auto& cache = word_cache_[first ? 1 : 0];
  auto it = cache.find(word);
  if (it != cache.end()) return it->second;
  std::vector<int32_t> ids;
  encode(first ? word : " " + word, ids);
  return cache.emplace(word, std::move(ids)).first->second;
}

std::string Tokenizer::decode(const int32_t* ids, int n) const {
  std::string stand, bytes;
  for (int k = 0; k < n; ++k) {
    const int32_t id = ids[k];
    if (id < 0 || (size_t)id >= inv_.size()) continue;
    const std::string& t = inv_[id];
    if (t == "<s>" || t == "</s>" || t == "<pad>" || t == "<unk>" || t == "<mask>") {
      // special tokens pass through as text
      for (size_t i = 0; i < t.size(); ++i) utf8_append(stand, 0x110000 + (unsigned char)t[i]);
      continue;
    }
    stand += t;
  }
  for (size_t i = 0; i < stand.size();) {
    const uint32_t cp = utf8_next(stand, i);
    if (cp >= 0x110000) { bytes.push_back((char)(cp - 0x110000)); continue; }
    auto it = byte_dec_.find(cp);
    if (it != byte_dec_.end()) bytes.push_back((char)it->second);
  }
  // bytes.decode("utf-8", errors="replace")
  std::string out;
  for (size_t i = 0; i < bytes.size();) {
    const unsigned char c = (unsigned char)bytes[i];
    size_t len = c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
    bool ok = len > 0 && i + len <= bytes.size();
    for (size_t k = 1; ok && k < len; ++k) ok = ((unsigned char)bytes[i + k] & 0xC0) == 0x80;
    if (ok) {
      out.append(bytes, i, len);
      i += len;
    } else {
      out += "\xEF\xBF\xBD";
      i += 1;
    }
  }
  return out;
}

}  // namespace ah
