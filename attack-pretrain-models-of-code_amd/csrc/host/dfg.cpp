// dfg.cpp — C data-flow graph and identifier list without tree-sitter.
//
// The reference derives the attackable identifiers of a function from GraphCodeBERT's data-flow
// graph: run_parser.py:272-281 get_identifiers = unique valid names over extract_dataflow
// (run_parser.py:190-216), whose graph comes from DFG_c (python_parser/parser_folder/DFG_c.py:
// 10-191) walking a tree-sitter-c parse.  tree-sitter is absent here, so this file
// builds its own C syntax tree over the lexer's leaves (lexer.cpp) with the node kinds DFG_c
// looks at, then restates the DFG_c walk on it.  The tree follows tree-sitter-c 0.20's shapes
// where DFG_c can see them:
//   declaration        specifiers, then declarators; a declarator with '=' is an init_declarator
//                      {declarator, value}; `T a;` puts the identifier directly under the
//                      declaration (the only identifier-leaf definition DFG_c recognises)
//   pointer_declarator / array_declarator / function_declarator / parenthesized_declarator,
//   parameter_list / parameter_declaration, function_definition, field_declaration
//   compound / if / while / do / for / expression statements
//   assignment_expression (=, op=), update_expression (++/--); every other expression node is
//   generic (DFG_c only recurses through it)
// and the walk keeps every DFG_c quirk that decides the output:
//   * 'init_declatator' is misspelt in DFG_c's def list, so `int a = 1;` defines nothing, while
//     pointer / array declarators define every non-keyword leaf of their declarator subtree
//     whether or not they are initialised;
//   * assignment_expression returns no entries at all (its body is commented out), so uses,
//     updates and calls inside an assignment never reach the graph;
//   * update_expression: every non-keyword leaf computedFrom every other;
//   * while bodies are walked twice (a name defined late in a loop flows to its earlier uses);
//   * the identifier leaf that names a function_declarator is skipped.
// Parity with tree-sitter itself is unpinned (no grammar here); the known answer is the set and
// order of the substitute keys of the reference's own jsonl fixtures (tests/test_host.py).
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <unordered_set>

#include "dfg_util.h"
#include "host.h"

namespace ah {
namespace {

enum NT : uint8_t {
  N_LEAF,
  N_GENERIC,
  N_TRANSLATION_UNIT,
  N_FUNCTION_DEFINITION,
  N_DECLARATION,
  N_FIELD_DECLARATION,
  N_TYPE_DEFINITION,
  N_INIT_DECLARATOR,
  N_POINTER_DECLARATOR,
  N_ARRAY_DECLARATOR,
  N_FUNCTION_DECLARATOR,
  N_PAREN_DECLARATOR,
  N_PARAMETER_LIST,
  N_PARAMETER_DECLARATION,
  N_COMPOUND,
  N_IF,
  N_WHILE,
  N_DO,
  N_FOR,
  N_ASSIGNMENT,
  N_UPDATE,
};

struct Node {
  NT type = N_GENERIC;
  int leaf = -1;          // N_LEAF: leaf index
  int parent = -1;
  int decl = -1;          // 'declarator' field
  int value = -1;         // 'value' field (init_declarator)
  bool tid = false;       // leaf is a type_identifier / primitive_type of the specifiers
  std::vector<int> kids;  // in source order
};

const std::unordered_set<std::string>& c_keywords() {
  // anonymous tokens of tree-sitter-c whose node type equals their text
  static const std::unordered_set<std::string> k = {
      "if", "else", "while", "for", "do", "switch", "case", "default", "return", "break",
      "continue", "goto", "sizeof", "struct", "union", "enum", "typedef", "static", "extern",
      "auto", "register", "inline", "const", "volatile", "restrict", "_Atomic", "signed",
      "unsigned", "long", "short", "true", "false", "__attribute__", "defined", "_Alignof",
      "offsetof", "_Generic", "asm", "__asm__", "__restrict", "__restrict__", "__inline",
      "__inline__", "__extension__", "_Noreturn", "noreturn", "thread_local", "__thread",
      "_Thread_local"};
  return k;
}
const std::unordered_set<std::string>& primitive_types() {
  static const std::unordered_set<std::string> k = {
      "bool", "char", "int", "float", "double", "void", "size_t", "ssize_t", "ptrdiff_t",
      "intptr_t", "uintptr_t", "charptr_t", "int8_t", "int16_t", "int32_t", "int64_t",
      "uint8_t", "uint16_t", "uint32_t", "uint64_t", "char8_t", "char16_t", "char32_t",
      "char64_t", "_Bool", "_Complex"};
  return k;
}
bool is_storage_or_qual(const std::string& t) {
  static const std::unordered_set<std::string> k = {
      "static", "extern", "auto", "register", "inline", "__inline", "__inline__", "const",
      "volatile", "restrict", "__restrict", "__restrict__", "_Atomic", "__extension__",
      "_Noreturn", "noreturn", "thread_local", "__thread", "_Thread_local"};
  return k.count(t) > 0;
}
bool is_sized(const std::string& t) {
  return t == "signed" || t == "unsigned" || t == "long" || t == "short";
}
bool id_like(const std::string& t) {
  return !t.empty() && ((t[0] >= 'a' && t[0] <= 'z') || (t[0] >= 'A' && t[0] <= 'Z') || t[0] == '_');
}
bool is_ident(const std::string& t) {
  return id_like(t) && !c_keywords().count(t) && !primitive_types().count(t);
}
bool is_assign_op(const std::string& t) {
  return t == "=" || t == "+=" || t == "-=" || t == "*=" || t == "/=" || t == "%=" ||
         t == "<<=" || t == ">>=" || t == "&=" || t == "^=" || t == "|=";
}
int binary_prec(const std::string& t) {
  if (t == "||") return 4;
  if (t == "&&") return 5;
  if (t == "|") return 6;
  if (t == "^") return 7;
  if (t == "&") return 8;
  if (t == "==" || t == "!=") return 9;
  if (t == "<" || t == ">" || t == "<=" || t == ">=") return 10;
  if (t == "<<" || t == ">>") return 11;
  if (t == "+" || t == "-") return 12;
  if (t == "*" || t == "/" || t == "%") return 13;
  return -1;
}

// anonymous leaf: tree-sitter node type == its text (punctuation, keywords, quotes, directives)
bool leaf_anon(const std::string& t) {
  if (t.empty()) return true;
  const unsigned char c = (unsigned char)t[0];
  if (t == "L\"" || t == "L'" || t == "u8\"" || t == "u\"" || t == "U\"" || t == "u'" ||
      t == "U'" || t == "u8'")
    return true;  // prefixed string / char opener
  if (id_like(t)) return c_keywords().count(t) > 0;
  if (c >= '0' && c <= '9') return false;                      // number_literal
  if ((c == '-' || c == '+' || c == '.') && t.size() > 1 && t[1] >= '0' && t[1] <= '9')
    return false;                                              // signed / .5 number
  if (c == '\\') return false;                                 // escape_sequence
  if (c == '<' && t.size() > 2 && t.back() == '>') return false;  // system_lib_string
  if (c == '#') return true;                                   // directive
  if (c >= 0x80) return false;
  // preproc_arg and other multi-character free text contain spaces or id characters
  for (unsigned char d : t)
    if (d == ' ' || (d >= 'a' && d <= 'z') || (d >= 'A' && d <= 'Z') || (d >= '0' && d <= '9'))
      return false;
  return true;
}

class CTree {
 public:
  explicit CTree(const std::vector<Leaf>& lv) : lv_(lv) {
    n_ = lv.size();
    match_.assign(n_, -1);
    std::vector<int> st;
    for (size_t i = 0; i < n_; ++i) {
      const std::string& t = lv[i].raw;
      if (t == "(" || t == "[" || t == "{") st.push_back((int)i);
      else if (t == ")" || t == "]" || t == "}") {
        const char open = t == ")" ? '(' : t == "]" ? '[' : '{';
        // pop to the nearest matching opener (tolerates unbalanced macro text)
        for (int k = (int)st.size() - 1; k >= 0; --k)
          if (lv[st[k]].raw[0] == open) {
            match_[st[k]] = (int)i;
            match_[i] = st[k];
            st.resize(k);
            break;
          }
      }
    }
  }

  int parse() {
    root_ = make(N_TRANSLATION_UNIT);
    while (p_ < n_) {
      const size_t before = p_;
      external(root_);
      if (p_ == before) add_leaf(root_, p_++);
    }
    return root_;
  }

  std::vector<Node> nodes;

 private:
  // ---------------------------------------------------------------------------- tree helpers
  int make(NT t) {
    nodes.push_back(Node());
    nodes.back().type = t;
    return (int)nodes.size() - 1;
  }
  void attach(int parent, int child) {
    if (child < 0) return;
    nodes[child].parent = parent;
    nodes[parent].kids.push_back(child);
  }
  int leaf_node(size_t i) {
    int x = make(N_LEAF);
    nodes[x].leaf = (int)i;
    return x;
  }
  void add_leaf(int parent, size_t i) { attach(parent, leaf_node(i)); }
  const std::string& t(size_t i) const {
    static const std::string empty;
    return i < n_ ? lv_[i].raw : empty;
  }
  bool at(const char* s) const { return p_ < n_ && lv_[p_].raw == s; }
  // consume the balanced group starting at p_ ('(' / '[' / '{') as generic leaves under parent
  void group(int parent) {
    const size_t e = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
    while (p_ <= e && p_ < n_) add_leaf(parent, p_++);
  }

  // ---------------------------------------------------------------------------- preprocessor
  bool directive() const { return p_ < n_ && !t(p_).empty() && t(p_)[0] == '#'; }
  void preproc(int parent) {
    const int g = make(N_GENERIC);
    attach(parent, g);
    int end_line = lv_[p_].el;
    add_leaf(g, p_++);
    while (p_ < n_ && lv_[p_].sl <= end_line) {
      end_line = std::max(end_line, lv_[p_].el);
      add_leaf(g, p_++);
    }
  }

  // ---------------------------------------------------------------------------- declarations
  bool type_start(size_t i) const {
    const std::string& s = t(i);
    return is_storage_or_qual(s) || primitive_types().count(s) || is_sized(s) || s == "struct" ||
           s == "union" || s == "enum" || s == "__attribute__" || s == "typedef";
  }
  // statement-level: is the construct at p_ a declaration?
  bool looks_like_declaration() const {
    if (p_ >= n_) return false;
    if (type_start(p_)) return true;
    if (!is_ident(t(p_))) return false;
    size_t q = p_ + 1;
    if (is_ident(t(q))) return true;  // T x
    if (t(q) == "*") {
      while (t(q) == "*" || is_storage_or_qual(t(q))) ++q;
      if (!is_ident(t(q))) return false;
      const std::string& f = t(q + 1);
      return f == ";" || f == "=" || f == "," || f == "[" || f == ")";
    }
    if (t(q) == "(" && t(q + 1) == "*" && is_ident(t(q + 2)) && t(q + 3) == ")" && t(q + 4) == "(")
      return true;  // T (*fp)(...)
    return false;
  }

  void attribute(int parent) {  // __attribute__((...))
    add_leaf(parent, p_++);
    if (at("(")) group(parent);
  }

  // declaration specifiers; returns true if a type was seen
  bool specifiers(int parent) {
    bool seen_type = false;
    while (p_ < n_) {
      const std::string& s = t(p_);
      if (s == "__attribute__") {
        attribute(parent);
      } else if (is_storage_or_qual(s) || s == "typedef") {
        add_leaf(parent, p_++);
      } else if (primitive_types().count(s) || is_sized(s)) {
        add_leaf(parent, p_++);
        seen_type = true;
      } else if (s == "struct" || s == "union" || s == "enum") {
        const int g = make(N_GENERIC);
        attach(parent, g);
        add_leaf(g, p_++);
        while (at("__attribute__")) attribute(g);
        if (p_ < n_ && is_ident(t(p_))) add_leaf(g, p_++);
        if (at("{")) {
          if (s == "enum") group(g);
          else struct_body(g);
        }
        seen_type = true;
      } else if (!seen_type && is_ident(s) &&
                 !(t(p_ + 1) == "(" && !(t(p_ + 2) == "*"))) {
        add_leaf(parent, p_++);  // type_identifier
        nodes[nodes[parent].kids.back()].tid = true;
        seen_type = true;
      } else {
        break;
      }
    }
    return seen_type;
  }

  void struct_body(int parent) {
    const int body = make(N_GENERIC);
    attach(parent, body);
    const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
    add_leaf(body, p_++);
    while (p_ < close) {
      const size_t before = p_;
      if (directive()) {
        preproc(body);
        continue;
      }
      const int fd = make(N_FIELD_DECLARATION);
      attach(body, fd);
      specifiers(fd);
      while (p_ < close && !at(";")) {
        const size_t b2 = p_;
        const int d = declarator(false);
        flush_strays(fd);
        attach(fd, d);
        if (at(":")) {  // bitfield
          add_leaf(fd, p_++);
          expression(fd, close, false);
        }
        if (at(",")) add_leaf(fd, p_++);
        else if (p_ == b2) add_leaf(fd, p_++);
        else if (!at(";")) break;
      }
      if (at(";")) add_leaf(fd, p_++);
      if (p_ == before) add_leaf(body, p_++);
    }
    if (p_ == close) add_leaf(body, p_++);
  }

  // declarator (abstract allowed: returns a node possibly without an identifier, or -1)
  int declarator(bool in_param) {
    if (at("*")) {
      const int pd = make(N_POINTER_DECLARATOR);
      add_leaf(pd, p_++);
      while (p_ < n_ && (is_storage_or_qual(t(p_)) || t(p_) == "__attribute__")) {
        const int q = make(N_GENERIC);
        attach(pd, q);
        if (t(p_) == "__attribute__") attribute(q);
        else add_leaf(q, p_++);
      }
      const int inner = declarator(in_param);
      flush_strays(pd);
      if (inner >= 0) {
        attach(pd, inner);
        nodes[pd].decl = inner;
      }
      return pd;
    }
    int base = -1;
    if (p_ < n_ && is_ident(t(p_))) {
      // `av_unused x`, `* attribute_align_arg f(...)`: a stray macro identifier before the
      // declarator is skipped by tree-sitter's error recovery (an ERROR node, no definition)
      while (!in_param && is_ident(t(p_ + 1))) strays_.push_back(p_++);
      base = leaf_node(p_++);
    } else if (at("(") && match_[p_] > 0 && !type_start(p_ + 1) &&
               (t(p_ + 1) == "*" || t(p_ + 1) == "(" || is_ident(t(p_ + 1))) &&
               !(in_param && is_ident(t(p_ + 1)) && t(p_ + 2) != ")")) {
      const size_t close = (size_t)match_[p_];
      const int pd = make(N_PAREN_DECLARATOR);
      add_leaf(pd, p_++);
      const int inner = declarator(in_param);
      if (inner >= 0) {
        attach(pd, inner);
        nodes[pd].decl = inner;
      }
      while (p_ < close) add_leaf(pd, p_++);  // tolerate leftovers
      if (p_ == close) add_leaf(pd, p_++);
      base = pd;
    }
    while (p_ < n_) {
      if (at("[")) {
        const int ad = make(N_ARRAY_DECLARATOR);
        if (base >= 0) {
          attach(ad, base);
          nodes[ad].decl = base;
        }
        const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
        add_leaf(ad, p_++);
        if (p_ < close) expression(ad, close, false);
        while (p_ < close) add_leaf(ad, p_++);
        if (p_ == close) add_leaf(ad, p_++);
        base = ad;
      } else if (at("(") && base >= 0) {
        const int fd = make(N_FUNCTION_DECLARATOR);
        attach(fd, base);
        nodes[fd].decl = base;
        attach(fd, parameter_list());
        base = fd;
      } else if (at("__attribute__")) {
        if (!in_param && base >= 0 && nodes[base].type == N_LEAF) {
          // `TCGReg addrhi __attribute__((unused));`, `int x __attribute__((unused)) = 0;`:
          // tree-sitter keeps the identifier as the declarator and puts the attribute (and an
          // initialiser after it) in an ERROR node, so the name is defined (fixture keys)
          while (p_ < n_ && !at(",") && !at(";")) {
            const size_t q = p_;
            const size_t end = (at("(") && match_[p_] > 0) ? (size_t)match_[p_] : p_;
            for (size_t k = q; k <= end; ++k) strays_.push_back(k);
            p_ = end + 1;
          }
          break;
        }
        const int g = make(N_GENERIC);
        if (base >= 0) attach(g, base);
        attribute(g);
        base = g;
      } else {
        break;
      }
    }
    return base;
  }

  int parameter_list() {
    const int pl = make(N_PARAMETER_LIST);
    const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
    add_leaf(pl, p_++);
    while (p_ < close) {
      const size_t before = p_;
      if (at("...") || at(",")) {
        add_leaf(pl, p_++);
        continue;
      }
      const int pd = make(N_PARAMETER_DECLARATION);
      attach(pl, pd);
      specifiers(pd);
      if (p_ < close && !at(",")) {
        int d = declarator(true);
        // `T a MACRO`: tree-sitter's error recovery skips the stray identifier and keeps the
        // last one as the declarator (e.g. softfloat's `flag ieee STATUS_PARAM`)
        while (d >= 0 && nodes[d].type == N_LEAF && p_ < close && is_ident(t(p_))) {
          attach(pd, d);  // the skipped identifier stays a plain leaf of the parameter
          d = leaf_node(p_++);
        }
        if (d >= 0) {
          attach(pd, d);
          nodes[pd].decl = d;
        }
      }
      while (p_ < close && !at(",")) add_leaf(pd, p_++);  // tolerate leftovers
      if (p_ == before) add_leaf(pl, p_++);
    }
    if (p_ == close) add_leaf(pl, p_++);
    return pl;
  }

  // declaration body after the specifiers: declarators (with initialisers) up to ';'
  void init_declarators(int decl, size_t limit) {
    // `uint32_t av_unused auxtag;`, `struct {...} QEMU_PACKED name;`: two identifiers then ';' as
    // the first declarator — tree-sitter keeps the first as the declarator and puts the second in
    // an ERROR node (fixture keys: av_unused / QEMU_PACKED defined, auxtag / name not; after a
    // ',' or with '=' / '*' following, the second identifier is the declarator: declarator())
    if (p_ + 2 < limit && is_ident(t(p_)) && is_ident(t(p_ + 1)) && t(p_ + 2) == ";") {
      attach(decl, leaf_node(p_++));
      const int err = make(N_GENERIC);
      attach(decl, err);
      add_leaf(err, p_++);
      return;
    }
    while (p_ < limit && !at(";")) {
      const size_t before = p_;
      const int d = declarator(false);
      flush_strays(decl);
      if (at("=")) {
        const int id = make(N_INIT_DECLARATOR);
        attach(decl, id);
        if (d >= 0) {
          attach(id, d);
          nodes[id].decl = d;
        }
        add_leaf(id, p_++);
        const int v = initializer(limit);
        if (v >= 0) {
          attach(id, v);
          nodes[id].value = v;
        }
      } else {
        attach(decl, d);
      }
      if (at(",")) {
        add_leaf(decl, p_++);
      } else if (p_ == before) {
        // not a declarator (e.g. `volatile ("\t":::"memory")` once a raw newline broke the
        // asm string): tree-sitter wraps the rest of the statement in an ERROR node, so no
        // identifier in it sits directly under the declaration
        const int err = make(N_GENERIC);
        attach(decl, err);
        while (p_ < limit && !at(";")) add_leaf(err, p_++);
      } else if (!at(";")) {
        break;
      }
    }
  }

  int initializer(size_t limit) {
    if (at("{")) return init_list();
    const int g = make(N_GENERIC);
    assignment_expr(g, limit);
    if (nodes[g].kids.size() == 1) {
      const int k = nodes[g].kids[0];
      nodes[k].parent = -1;
      return k;
    }
    return g;
  }

  int init_list() {
    const int g = make(N_GENERIC);
    const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
    add_leaf(g, p_++);
    while (p_ < close) {
      const size_t before = p_;
      if (at(",")) {
        add_leaf(g, p_++);
        continue;
      }
      if (at(".") || at("[")) {  // designated initializer: initializer_pair (no assignment)
        const int pair = make(N_GENERIC);
        attach(g, pair);
        while (p_ < close && (at(".") || at("["))) {
          if (at(".")) {
            add_leaf(pair, p_++);
            if (p_ < close) add_leaf(pair, p_++);
          } else {
            group(pair);
          }
        }
        if (at("=")) add_leaf(pair, p_++);
        if (p_ < close) attach(pair, initializer(close));
      } else {
        attach(g, initializer(close));
      }
      if (p_ == before) add_leaf(g, p_++);
    }
    if (p_ == close) add_leaf(g, p_++);
    return g;
  }

  // ---------------------------------------------------------------------------- expressions
  // Pratt parser; `limit` bounds the scan (exclusive).  with_comma: comma_expression allowed.
  void expression(int parent, size_t limit, bool with_comma) {
    if (!with_comma) {
      assignment_expr(parent, limit);
      return;
    }
    const int g = make(N_GENERIC);
    assignment_expr(g, limit);
    while (p_ < limit && at(",")) {
      add_leaf(g, p_++);
      assignment_expr(g, limit);
    }
    if (nodes[g].kids.size() == 1) {
      const int k = nodes[g].kids[0];
      nodes[k].parent = -1;
      attach(parent, k);
    } else {
      attach(parent, g);
    }
  }

  bool operand_start() const {
    if (p_ >= n_) return false;
    const std::string& s = t(p_);
    if (s == ";" || s == ")" || s == "]" || s == "}" || s == "," || s == ":") return false;
    if (binary_prec(s) > 0 && s != "*" && s != "&" && s != "-" && s != "+") return false;
    if (is_assign_op(s) || s == "?") return false;
    return true;
  }

  // parse one assignment-expression into parent; returns its node
  int assignment_expr(int parent, size_t limit) {
    const int lhs = conditional(limit);
    if (lhs < 0) return -1;
    if (p_ < limit && is_assign_op(t(p_))) {
      const int a = make(N_ASSIGNMENT);
      attach(a, lhs);
      add_leaf(a, p_++);
      const int tmp = make(N_GENERIC);
      const int r = assignment_expr(tmp, limit);
      if (r >= 0) {
        nodes[r].parent = -1;
        attach(a, r);
      }
      attach(parent, a);
      return a;
    }
    attach(parent, lhs);
    return lhs;
  }

  int conditional(size_t limit) {
    const int c = binary(limit, 4);
    if (c < 0) return -1;
    if (p_ < limit && at("?")) {
      const int g = make(N_GENERIC);
      attach(g, c);
      add_leaf(g, p_++);
      if (!at(":")) expression(g, limit, true);
      if (at(":")) add_leaf(g, p_++);
      assignment_expr(g, limit);
      return g;
    }
    return c;
  }

  int binary(size_t limit, int min_prec) {
    int lhs = unary(limit);
    if (lhs < 0) return -1;
    while (p_ < limit) {
      const int pr = binary_prec(t(p_));
      if (pr < min_prec) break;
      const int g = make(N_GENERIC);
      attach(g, lhs);
      add_leaf(g, p_++);
      const int rhs = binary(limit, pr + 1);
      if (rhs >= 0) attach(g, rhs);
      lhs = g;
    }
    return lhs;
  }

  bool paren_is_type(size_t i) const {  // '(' at i starts a type name (cast / compound literal)
    if (match_[i] < 0) return false;
    const size_t close = (size_t)match_[i];
    const size_t q = i + 1;
    if (q >= close) return false;
    if (type_start(q)) return true;
    if (!is_ident(t(q))) return false;
    size_t r = q + 1;
    while (r < close && (t(r) == "*" || is_storage_or_qual(t(r)))) ++r;
    if (r != close) return false;
    if (r > q + 1) return true;  // (T *)
    // (T) followed by an operand
    const std::string& f = t(close + 1);
    return is_ident(f) || (!f.empty() && ((f[0] >= '0' && f[0] <= '9') || f[0] == '"' ||
                                          f[0] == '\'')) ||
           f == "(" || f == "{" || f == "!" || f == "~" || f == "&";
  }

  int unary(size_t limit) {
    if (p_ >= limit) return -1;
    const std::string& s = t(p_);
    if (s == "++" || s == "--") {
      const int u = make(N_UPDATE);
      add_leaf(u, p_++);
      const int e = unary(limit);
      if (e >= 0) attach(u, e);
      return u;
    }
    if (s == "*" || s == "&" || s == "-" || s == "+" || s == "!" || s == "~" ||
        s == "__extension__") {
      const int g = make(N_GENERIC);
      add_leaf(g, p_++);
      const int e = unary(limit);
      if (e >= 0) attach(g, e);
      return g;
    }
    if (s == "sizeof" || s == "_Alignof" || s == "__alignof__") {
      const int g = make(N_GENERIC);
      add_leaf(g, p_++);
      if (at("(") && paren_is_type(p_)) {
        group(g);
      } else {
        const int e = unary(limit);
        if (e >= 0) attach(g, e);
      }
      return g;
    }
    if (s == "(" && paren_is_type(p_)) {  // cast / compound literal
      const int g = make(N_GENERIC);
      group(g);
      if (at("{")) attach(g, init_list());
      else {
        const int e = unary(limit);
        if (e >= 0) attach(g, e);
      }
      return postfix(g, limit);
    }
    return postfix(primary(limit), limit);
  }

  int primary(size_t limit) {
    if (p_ >= limit) return -1;
    const std::string& s = t(p_);
    if (s == "(") {
      const int g = make(N_GENERIC);
      const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)limit - 1);
      add_leaf(g, p_++);
      if (at("{")) {  // GNU statement expression
        compound(g);
      } else if (p_ < close) {
        expression(g, close, true);
      }
      while (p_ < close) add_leaf(g, p_++);
      if (p_ == close) add_leaf(g, p_++);
      return g;
    }
    if (s == "{") return init_list();
    if (is_string_open(s)) return strings(limit);
    if (s == ";" || s == "}" || s == ")" || s == "]") return -1;
    return leaf_node(p_++);
  }

  static bool is_string_open(const std::string& s) {
    return s == "\"" || s == "'" || s == "L\"" || s == "L'" || s == "u\"" || s == "U\"" ||
           s == "u8\"" || s == "u'" || s == "U'" || s == "u8'";
  }
  int strings(size_t limit) {
    const int g = make(N_GENERIC);
    while (p_ < limit && is_string_open(t(p_))) {
      const char q = t(p_).back();
      const int line = lv_[p_].sl;
      const int lit = make(N_GENERIC);
      attach(g, lit);
      add_leaf(lit, p_++);
      while (p_ < limit && !t(p_).empty() && t(p_)[0] == '\\' && lv_[p_].sl == line)
        add_leaf(lit, p_++);
      if (p_ < limit && t(p_).size() == 1 && t(p_)[0] == q) add_leaf(lit, p_++);
    }
    return g;
  }

  int postfix(int e, size_t limit) {
    if (e < 0) return -1;
    while (p_ < limit) {
      const std::string& s = t(p_);
      if (s == "++" || s == "--") {
        const int u = make(N_UPDATE);
        attach(u, e);
        add_leaf(u, p_++);
        e = u;
      } else if (s == "[" || s == "(") {
        const int g = make(N_GENERIC);
        attach(g, e);
        const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)limit - 1);
        const int args = make(N_GENERIC);
        attach(g, args);
        add_leaf(args, p_++);
        while (p_ < close) {
          const size_t before = p_;
          if (at(",")) {
            add_leaf(args, p_++);
            continue;
          }
          if (s == "(" && looks_like_type_arg()) {
            // macro argument that is a type (container_of(p, T, f)): keep generic leaves
            while (p_ < close && !at(",")) add_leaf(args, p_++);
          } else {
            expression(args, close, s == "[");
          }
          if (p_ == before) add_leaf(args, p_++);
        }
        if (p_ == close) add_leaf(args, p_++);
        e = g;
      } else if (s == "." || s == "->") {
        const int g = make(N_GENERIC);
        attach(g, e);
        add_leaf(g, p_++);
        if (p_ < limit && id_like(t(p_))) add_leaf(g, p_++);
        e = g;
      } else if (is_string_open(s) && nodes[e].type == N_LEAF) {
        // macro string pieces: "a" PRIx64 "b" — keep them in one expression
        const int g = make(N_GENERIC);
        attach(g, e);
        attach(g, strings(limit));
        e = g;
      } else {
        break;
      }
    }
    return e;
  }
  bool looks_like_type_arg() const {
    return (type_start(p_) && !(t(p_) == "sizeof")) ;
  }

  // ---------------------------------------------------------------------------- statements
  void external(int parent) {
    if (directive()) {
      preproc(parent);
      return;
    }
    if (at(";")) {
      add_leaf(parent, p_++);
      return;
    }
    // function definition or declaration
    const size_t start = p_;
    const int d = make(N_DECLARATION);
    const bool typed = specifiers(d);
    if (!typed) {
      // no type specifier: not a function definition or declaration for tree-sitter-c (its
      // declaration specifiers need a type) — e.g. `name (T *a, ...) {` is a call expression
      // statement followed by a compound statement, so its "parameters" define nothing
      p_ = start;
      nodes[d].kids.clear();
      nodes[d].type = N_GENERIC;
      attach(parent, d);
      statement(d, n_);
      return;
    }
    // `static av_always_inline av_flatten void f(...)`: the second identifier closes a
    // declaration of its own (an identifier directly under a declaration) and the function
    // definition starts at the type keyword that follows
    if (p_ + 1 < n_ && is_ident(t(p_)) && type_start(p_ + 1)) {
      add_leaf(d, p_++);
      attach(parent, d);
      return;
    }
    // `uint32_t av_unused auxtag;`, `struct {...} QEMU_PACKED name;`: two identifiers then ';'
    // as the first declarator — tree-sitter keeps the first as the declarator and puts the
    // second in an ERROR node (fixture keys: av_unused / QEMU_PACKED defined, auxtag / name not;
    // with '=' or '*' after the second identifier it is the declarator instead, below)
    if (p_ + 2 < n_ && is_ident(t(p_)) && is_ident(t(p_ + 1)) && t(p_ + 2) == ";") {
      attach(d, leaf_node(p_++));
      const int err = make(N_GENERIC);
      attach(d, err);
      add_leaf(err, p_++);
      add_leaf(d, p_++);
      attach(parent, d);
      return;
    }
    // `static int coroutine_fn name(...)`: a macro between the type and the declarator is an
    // error node tree-sitter skips; the last identifier starts the declarator
    while (p_ + 1 < n_ && is_ident(t(p_)) && (is_ident(t(p_ + 1)) || t(p_ + 1) == "*"))
      add_leaf(d, p_++);
    const size_t after_spec = p_;
    const int decl = declarator(false);
    if (decl >= 0 && nodes[decl].type != N_LEAF && contains_function_declarator(decl)) {
      // K&R parameter declarations up to the body
      size_t q = p_;
      while (q < n_ && t(q) != "{" && t(q) != ";") ++q;
      if (q < n_ && t(q) == "{") {
        // a body whose '{' is never closed (truncated Devign functions, cut between statements)
        // does not reduce to a function_definition: tree-sitter's recovery leaves the declarator
        // under an ERROR node, so a pointer declarator then defines every leaf of its function
        // declarator (the function name, parameter types and names) as DFG_c does outside a
        // definition.  A function cut inside an open '(' recovers as a definition.
        nodes[d].type = match_[q] >= 0 || open_paren_at_eof() ? N_FUNCTION_DEFINITION : N_GENERIC;
        flush_strays(d);
        attach(d, decl);
        nodes[d].decl = decl;
        while (p_ < q) {
          const size_t before = p_;
          const int kr = make(N_DECLARATION);
          attach(d, kr);
          specifiers(kr);
          init_declarators(kr, q);
          if (at(";")) add_leaf(kr, p_++);
          if (p_ == before) add_leaf(d, p_++);
        }
        compound(d);
        attach(parent, d);
        return;
      }
    }
    // plain declaration: re-parse the declarators with initialisers
    strays_.clear();
    p_ = after_spec;
    init_declarators(d, n_);
    if (at(";")) add_leaf(d, p_++);
    attach(parent, d);
  }

  bool open_paren_at_eof() const {
    for (size_t i = 0; i < n_; ++i)
      if (lv_[i].raw == "(" && match_[i] < 0) return true;
    return false;
  }

  bool contains_function_declarator(int x) const {
    while (x >= 0) {
      if (nodes[x].type == N_FUNCTION_DECLARATOR) return true;
      x = nodes[x].decl;
    }
    return false;
  }

  void compound(int parent) {
    const int c = make(N_COMPOUND);
    attach(parent, c);
    const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_);
    add_leaf(c, p_++);
    while (p_ < close && p_ < n_) {
      const size_t before = p_;
      statement(c, close);
      if (p_ == before) add_leaf(c, p_++);
    }
    if (p_ == close && p_ < n_) add_leaf(c, p_++);
  }

  void paren_expr(int parent) {
    if (!at("(")) return;
    const int g = make(N_GENERIC);
    attach(parent, g);
    const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
    add_leaf(g, p_++);
    if (p_ < close) expression(g, close, true);
    while (p_ < close) add_leaf(g, p_++);
    if (p_ == close) add_leaf(g, p_++);
  }

  void statement(int parent, size_t limit) {
    if (p_ >= limit) return;
    if (directive()) {
      preproc(parent);
      return;
    }
    const std::string& s = t(p_);
    if (s == "{") {
      compound(parent);
      return;
    }
    if (s == ";") {
      add_leaf(parent, p_++);
      return;
    }
    if (s == "if") {
      const int n = make(N_IF);
      attach(parent, n);
      add_leaf(n, p_++);
      paren_expr(n);
      statement(n, limit);
      if (at("else")) {
        add_leaf(n, p_++);
        statement(n, limit);
      }
      return;
    }
    if (s == "while") {
      const int n = make(N_WHILE);
      attach(parent, n);
      add_leaf(n, p_++);
      paren_expr(n);
      statement(n, limit);
      return;
    }
    if (s == "switch") {
      const int n = make(N_GENERIC);
      attach(parent, n);
      add_leaf(n, p_++);
      paren_expr(n);
      statement(n, limit);
      return;
    }
    if (s == "do") {
      const int n = make(N_DO);
      attach(parent, n);
      add_leaf(n, p_++);
      statement(n, limit);
      if (at("while")) {
        add_leaf(n, p_++);
        paren_expr(n);
      }
      if (at(";")) add_leaf(n, p_++);
      return;
    }
    if (s == "for") {
      const int n = make(N_FOR);
      attach(parent, n);
      add_leaf(n, p_++);
      if (at("(")) {
        const size_t close = (size_t)(match_[p_] >= 0 ? match_[p_] : (int)n_ - 1);
        add_leaf(n, p_++);
        // initializer: declaration (its ';' included) or expression + ';'
        if (looks_like_declaration()) {
          const int d = make(N_DECLARATION);
          attach(n, d);
          specifiers(d);
          init_declarators(d, close);
          if (at(";")) add_leaf(d, p_++);
        } else {
          if (!at(";")) expression(n, close, true);
          if (at(";")) add_leaf(n, p_++);
        }
        if (!at(";") && p_ < close) expression(n, close, true);
        if (at(";")) add_leaf(n, p_++);
        if (p_ < close) expression(n, close, true);
        while (p_ < close) add_leaf(n, p_++);
        if (p_ == close) add_leaf(n, p_++);
      }
      statement(n, limit);
      return;
    }
    if (s == "return" || s == "goto" || s == "break" || s == "continue") {
      const int n = make(N_GENERIC);
      attach(parent, n);
      add_leaf(n, p_++);
      if (!at(";") && p_ < limit) expression(n, limit, true);
      if (at(";")) add_leaf(n, p_++);
      return;
    }
    if (s == "case" || s == "default") {
      const int n = make(N_GENERIC);
      attach(parent, n);
      add_leaf(n, p_++);
      if (!at(":") && p_ < limit) conditional_into(n, limit);
      if (at(":")) add_leaf(n, p_++);
      return;
    }
    if (is_ident(s) && t(p_ + 1) == ":") {  // label
      const int n = make(N_GENERIC);
      attach(parent, n);
      add_leaf(n, p_++);
      add_leaf(n, p_++);
      return;
    }
    if (looks_like_declaration()) {
      const int d = make(N_DECLARATION);
      attach(parent, d);
      if (at("typedef")) nodes[d].type = N_TYPE_DEFINITION;
      specifiers(d);
      init_declarators(d, limit);
      if (at(";")) add_leaf(d, p_++);
      return;
    }
    // expression statement (a macro call followed by a block ends before the block)
    const int n = make(N_GENERIC);
    attach(parent, n);
    expression(n, limit, true);
    if (at(";")) add_leaf(n, p_++);
  }

  void conditional_into(int parent, size_t limit) {
    const int c = conditional(limit);
    if (c >= 0) attach(parent, c);
  }

  void flush_strays(int parent) {
    if (strays_.empty()) return;
    const int g = make(N_GENERIC);  // tree-sitter ERROR node
    for (size_t i : strays_) add_leaf(g, i);
    strays_.clear();
    attach(parent, g);
  }

  const std::vector<Leaf>& lv_;
  std::vector<size_t> strays_;
  size_t n_ = 0, p_ = 0;
  int root_ = -1;
  std::vector<int> match_;
};

// ------------------------------------------------------------------------------ DFG_c walk
struct Walker {
  const std::vector<Node>& nd;
  const std::vector<Leaf>& lv;
  std::vector<char> anon;
  using States = std::map<std::string, std::vector<int>>;

  Walker(const std::vector<Node>& n, const std::vector<Leaf>& l) : nd(n), lv(l) {
    anon.resize(l.size());
    for (size_t i = 0; i < l.size(); ++i) anon[i] = leaf_anon(l[i].raw) && l[i].text == l[i].raw;
  }

  // tree_to_variable_index: non-anonymous leaves of a subtree (utils.py:98-113)
  void var_index(int x, std::vector<int>& out) const {
    if (x < 0) return;
    if (nd[x].type == N_LEAF) {
      if (!anon[nd[x].leaf]) out.push_back(nd[x].leaf);
      return;
    }
    for (int k : nd[x].kids) var_index(k, out);
  }

  static void sort_by_idx(std::vector<DfgEdge>& d) {
    std::stable_sort(d.begin(), d.end(),
                     [](const DfgEdge& a, const DfgEdge& b) { return a.idx < b.idx; });
  }

  // for / while: merge entries with the same (code, idx, rel) (DFG_c.py:130-138, :145-153)
  static void merge_dup(std::vector<DfgEdge>& d) {
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
    // sorted(dic.items(), key=idx): python sort is stable over first-seen order
    sort_by_idx(out);
    d.swap(out);
  }

  std::vector<DfgEdge> walk(int x, States& states) const {
    const Node& n = nd[x];
    std::vector<DfgEdge> dfg;
    if (n.type == N_LEAF) {
      const int idx = n.leaf;
      const std::string& code = lv[idx].text;
      const int par = n.parent;
      if (anon[idx] || (par >= 0 && nd[par].type == N_FUNCTION_DECLARATOR)) return dfg;
      auto it = states.find(code);
      if (it != states.end()) {
        dfg.push_back({code, idx, false, {code}, it->second});
        return dfg;
      }
      if (is_ident(lv[idx].raw) && !n.tid && !primitive_types().count(code) && par >= 0 &&
          nd[par].type == N_DECLARATION) {
        states[code] = {idx};
        dfg.push_back({code, idx, false, {}, {}});
      }
      return dfg;
    }
    switch (n.type) {
      case N_POINTER_DECLARATOR:
      case N_ARRAY_DECLARATOR: {
        const int par = n.parent;
        if (par >= 0 && nd[par].type == N_FUNCTION_DEFINITION) {
          int r = x;
          while (nd[r].type == N_POINTER_DECLARATOR && nd[r].decl >= 0 &&
                 nd[nd[r].decl].type == N_POINTER_DECLARATOR)
            r = nd[r].decl;
          for (int k : nd[r].kids) append(dfg, walk(k, states));
          sort_by_idx(dfg);
          return dfg;
        }
        std::vector<int> idxs;
        var_index(n.decl, idxs);
        for (int i : idxs) {
          dfg.push_back({lv[i].text, i, false, {}, {}});
          states[lv[i].text] = {i};
        }
        sort_by_idx(dfg);
        return dfg;
      }
      case N_ASSIGNMENT:
        return dfg;
      case N_UPDATE: {
        std::vector<int> idxs;
        var_index(x, idxs);
        for (int i1 : idxs) {
          for (int i2 : idxs) dfg.push_back({lv[i1].text, i1, true, {lv[i2].text}, {i2}});
          states[lv[i1].text] = {i1};
        }
        sort_by_idx(dfg);
        return dfg;
      }
      case N_IF: {
        States current = states;
        std::vector<States> others;
        bool flag = false;
        for (int k : n.kids) {
          const bool is_else = nd[k].type == N_LEAF && lv[nd[k].leaf].raw == "else";
          const bool in_if_list = is_else || nd[k].type == N_IF;
          if (!in_if_list && !flag) {
            append(dfg, walk(k, current));
          } else {
            flag = true;
            States ns = states;
            append(dfg, walk(k, ns));
            others.push_back(std::move(ns));
          }
        }
        others.push_back(std::move(current));
        // DFG_c.py also folds the incoming states in, with or without an else
        others.push_back(std::move(states));
        states = dfg_union(std::move(others));
        sort_by_idx(dfg);
        return dfg;
      }
      case N_FOR: {
        for (int k : n.kids) append(dfg, walk(k, states));
        merge_dup(dfg);
        return dfg;
      }
      case N_WHILE: {
        for (int rep = 0; rep < 2; ++rep)
          for (int k : n.kids) append(dfg, walk(k, states));
        merge_dup(dfg);
        return dfg;
      }
      case N_PARAMETER_DECLARATION: {
        int c = n.decl;
        if (c < 0) return dfg;
        while (!(nd[c].type == N_LEAF && is_ident(lv[nd[c].leaf].raw))) {
          c = nd[c].decl;  // parenthesized: its inner declarator is children[1] == decl
          if (c < 0) return dfg;
        }
        const int idx = nd[c].leaf;
        states[lv[idx].text] = {idx};
        dfg.push_back({lv[idx].text, idx, false, {}, {}});
        return dfg;
      }
      default: {
        for (int k : n.kids) append(dfg, walk(k, states));
        sort_by_idx(dfg);
        return dfg;
      }
    }
  }

  static void append(std::vector<DfgEdge>& a, std::vector<DfgEdge>&& b) {
    a.insert(a.end(), std::make_move_iterator(b.begin()), std::make_move_iterator(b.end()));
  }
};

}  // namespace

std::vector<DfgEdge> dfg_c(const std::vector<Leaf>& leaves) {
  CTree tree(leaves);
  const int root = tree.parse();
  Walker w(tree.nodes, leaves);
  std::map<std::string, std::vector<int>> states;
  std::vector<DfgEdge> d = w.walk(root, states);
  std::stable_sort(d.begin(), d.end(),
                   [](const DfgEdge& a, const DfgEdge& b) { return a.idx < b.idx; });
  return d;
}

std::vector<DfgEdge> dfg_of(const std::vector<Leaf>& leaves, Lang lang, DfgVariant variant) {
  if (variant == DFG_RUN_PARSER) {
    if (lang == LANG_JAVA) return dfg_java(leaves);
    if (lang == LANG_PYTHON) return dfg_python(leaves);
    return dfg_c(leaves);
  }
  std::vector<DfgEdge> d =
      lang == LANG_JAVA ? dfg_java(leaves, true) : dfg_python(leaves, true);
  // GraphCodeBERT/*/code/run.py:96-106: keep the entries that have an edge or are an edge's source
  std::set<int> linked;
  for (const DfgEdge& e : d) {
    if (!e.from_idx.empty()) linked.insert(e.idx);
    linked.insert(e.from_idx.begin(), e.from_idx.end());
  }
  std::vector<DfgEdge> out;
  for (DfgEdge& e : d)
    if (linked.count(e.idx)) out.push_back(std::move(e));
  return out;
}

std::vector<std::string> dfg_names(const std::vector<Leaf>& leaves, Lang lang) {
  std::vector<std::string> out;
  std::unordered_set<std::string> seen;
  for (const DfgEdge& e : dfg_of(leaves, lang))
    if (seen.insert(e.code).second) out.push_back(e.code);
  return out;
}

}  // namespace ah
