// dfg_python.cpp — Python data-flow graph and identifier list without tree-sitter.
//
// Restates python_parser/parser_folder/DFG_python.py:11-178 (the walk) over a Python syntax tree
// this file builds from the lexer's leaves (lexer.cpp): logical lines from the leaves' line
// positions, bracket depth and backslash continuations, blocks from their indentation, and
// expressions with tree-sitter-python's node shapes, because DFG_python pairs the CHILDREN of an
// assignment's left and right sides (`a, b = c, d` pairs a<-c and b<-d; unequal counts fall back
// to the whole sides).  The node kinds DFG_python looks at:
//   assignment / augmented_assignment {left, right}   (`x: T` without a value: nothing)
//   for_in_clause {left, last child}                  walked before its siblings
//   default_parameter {name, value}                   (also inside lambda parameters)
//   parameters: identifier children are definitions   (not *args / **kw / typed / lambda ones)
//   if_statement (elif_clause / else_clause walked from the incoming states), for_statement
//   (twice; the body only when it is the last child), while_statement (twice)
// and every other node generic.  Leaf classes: keywords and punctuation are anonymous; names,
// numbers, True / False / None, `...` and strings (taken whole) are named; `print` / `exec`
// starting a statement are the Python 2 statement keywords.  Known answer: the substitute keys
// of CodeXGLUE/Authorship-Attribution/dataset/data_folder/processed_gcjpy/valid_subs.jsonl
// (tests/test_host.py measures the match).
#include <cstring>
#include <unordered_set>

#include "dfg_util.h"

namespace ah {
namespace {

enum PT : uint8_t {
  P_LEAF,
  P_GENERIC,
  P_BLOCK,
  P_PARAMS,         // parameters
  P_DEFAULT_PARAM,  // a = name leaf node, b = value
  P_ASSIGN,         // assignment / augmented_assignment: a = left, b = right (-1: none)
  P_FOR_IN,         // for_in_clause: a = left
  P_IF,
  P_ELIF,
  P_ELSE,
  P_FOR,            // a = left, b = right
  P_WHILE,
};

struct PNode {
  PT type = P_GENERIC;
  int leaf = -1;
  int parent = -1;
  int a = -1, b = -1;
  std::vector<int> kids;
};

const std::unordered_set<std::string>& py_keywords() {
  static const std::unordered_set<std::string> k = {
      "and",   "as",     "assert", "async", "await",    "break", "class",  "continue",
      "def",   "del",    "elif",   "else",  "except",   "finally", "for",  "from",
      "global", "if",    "import", "in",    "is",       "lambda", "nonlocal", "not",
      "or",    "pass",   "raise",  "return", "try",     "while", "with",   "yield"};
  return k;
}
bool id_like(const std::string& t) {
  if (t.empty()) return false;
  const unsigned char c = (unsigned char)t[0];
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c >= 0x80;
}
bool is_name(const std::string& t) { return id_like(t) && !py_keywords().count(t); }
bool is_string(const std::string& t) {
  size_t p = 0;
  while (p < t.size() && p < 3 && std::strchr("rRbBuUfF", t[p])) ++p;
  return p < t.size() && (t[p] == '"' || t[p] == '\'');
}
bool is_number(const std::string& t) {
  if (t.empty()) return false;
  const unsigned char c = (unsigned char)t[0];
  return (c >= '0' && c <= '9') || (c == '.' && t.size() > 1 && t[1] >= '0' && t[1] <= '9');
}
bool is_atom_start(const std::string& t) {
  return is_name(t) || is_string(t) || is_number(t) || t == "(" || t == "[" || t == "{" ||
         t == "..." || t == "`";
}
bool is_aug_op(const std::string& t) {
  return t == "+=" || t == "-=" || t == "*=" || t == "/=" || t == "//=" || t == "%=" ||
         t == "**=" || t == ">>=" || t == "<<=" || t == "&=" || t == "^=" || t == "|=" ||
         t == "@=";
}
bool is_comp_op(const std::string& t) {
  return t == "<" || t == ">" || t == "==" || t == ">=" || t == "<=" || t == "!=" || t == "<>" ||
         t == "in" || t == "is" || t == "not";
}
int bin_prec(const std::string& t) {
  if (t == "|") return 1;
  if (t == "^") return 2;
  if (t == "&") return 3;
  if (t == "<<" || t == ">>") return 4;
  if (t == "+" || t == "-") return 5;
  if (t == "*" || t == "/" || t == "//" || t == "%" || t == "@") return 6;
  return -1;
}

class PyTree {
 public:
  explicit PyTree(const std::vector<Leaf>& lv) : lv_(lv), n_(lv.size()) {
    kw.assign(n_, 0);
    match_.assign(n_, -1);
    // token classes of find0's scan (integer compares instead of string compares per token)
    cls_.assign(n_, 0);
    for (size_t i = 0; i < n_; ++i) cls_[i] = (uint8_t)tok_class(lv[i].raw);
    std::vector<int> st;
    int depth = 0;
    for (size_t i = 0; i < n_; ++i) {
      const std::string& s = lv[i].raw;
      if (i == 0 || (depth == 0 && lv[i].sl > lv[i - 1].el && !lv[i].joined))
        lines_.push_back({i, i, lv[i].sc});
      lines_.back().e = i + 1;
      if (s == "(" || s == "[" || s == "{") {
        st.push_back((int)i);
        ++depth;
      } else if (s == ")" || s == "]" || s == "}") {
        const char open = s == ")" ? '(' : s == "]" ? '[' : '{';
        for (int k = (int)st.size() - 1; k >= 0; --k)
          if (lv[st[k]].raw[0] == open) {
            match_[st[k]] = (int)i;
            match_[i] = st[k];
            st.resize(k);
            break;
          }
        depth = (int)st.size();
      }
    }
  }

  int parse() {
    const int root = make(P_GENERIC);  // module
    while (li_ < lines_.size()) {
      const size_t before = li_;
      block_lines(root, lines_[li_].indent);
      if (li_ == before) ++li_;
    }
    return root;
  }

  std::vector<PNode> nodes;
  std::vector<char> kw;  // leaf consumed as a statement keyword (print / exec)

 private:
  struct Line {
    size_t b, e;
    int indent;
  };
  const std::vector<Leaf>& lv_;
  size_t n_;
  std::vector<int> match_;
  std::vector<uint8_t> cls_;
  std::vector<Line> lines_;
  size_t li_ = 0;
  size_t p_ = 0, lim_ = 0;

  // ------------------------------------------------------------------------ tree helpers
  int make(PT t) {
    nodes.push_back(PNode());
    nodes.back().type = t;
    return (int)nodes.size() - 1;
  }
  void attach(int parent, int child) {
    if (child < 0) return;
    nodes[child].parent = parent;
    nodes[parent].kids.push_back(child);
  }
  int leaf_node(size_t i) {
    const int x = make(P_LEAF);
    nodes[x].leaf = (int)i;
    return x;
  }
  int add_leaf(int parent, size_t i) {
    const int x = leaf_node(i);
    attach(parent, x);
    return x;
  }
  const std::string& t(size_t i) const {
    static const std::string empty;
    return i < lim_ && i < n_ ? lv_[i].raw : empty;
  }
  bool more() const { return p_ < lim_; }
  bool at(const char* s) const { return more() && lv_[p_].raw == s; }
  size_t close_of(size_t i) const {
    const int m = match_[i];
    if (m < 0 || (size_t)m >= lim_) return lim_ - 1;
    return (size_t)m;
  }
  template <class F>
  void limited(size_t lim, F f) {
    const size_t saved = lim_;
    lim_ = std::min(lim, saved);
    f();
    lim_ = saved;
  }
  void leaves_to(int parent, size_t e) {
    while (more() && p_ < e) add_leaf(parent, p_++);
  }
  // find0's token classes: brackets, lambda, ':' and the targets it is called with
  enum { K_OTHER, K_OPEN, K_LAMBDA, K_COLON, K_IN, K_SEMI, K_EQ, K_ELSE, K_COMMA, K_FOR };
  static int tok_class(const std::string& x) {
    if (x == "(" || x == "[" || x == "{") return K_OPEN;
    if (x == "lambda") return K_LAMBDA;
    if (x == ":") return K_COLON;
    if (x == "in") return K_IN;
    if (x == ";") return K_SEMI;
    if (x == "=") return K_EQ;
    if (x == "else") return K_ELSE;
    if (x == ",") return K_COMMA;
    if (x == "for") return K_FOR;
    return K_OTHER;
  }
  // first depth-0 occurrence of `s` in [p_, lim_) (a lambda's own ':' skipped), or lim_
  size_t find0(const char* s) const {
    const int want = tok_class(s);
    if (want == K_OTHER || want == K_OPEN || want == K_LAMBDA) std::abort();  // not a target
    int lambdas = 0;
    const size_t end = std::min(lim_, n_);
    for (size_t q = p_; q < end;) {
      const int c = cls_[q];
      if (c == K_OPEN) {
        q = close_of(q) + 1;
        continue;
      }
      if (c == K_LAMBDA) ++lambdas;
      else if (c == K_COLON && lambdas > 0) {
        --lambdas;
        ++q;
        continue;
      }
      if (c == want) return q;
      ++q;
    }
    return lim_;
  }

  // ------------------------------------------------------------------------ statements
  void block_lines(int parent, int indent) {
    while (li_ < lines_.size() && lines_[li_].indent >= indent) {
      const size_t before = li_;
      line_statement(parent);
      if (li_ == before) ++li_;
    }
  }
  // the body after a compound header's ':' at p_ (already consumed)
  void suite(int parent, int header_indent) {
    const int blk = make(P_BLOCK);
    if (more()) {  // same-line simple statements
      simple_statements(blk);
      ++li_;
    } else {
      ++li_;
      if (li_ < lines_.size() && lines_[li_].indent > header_indent)
        block_lines(blk, lines_[li_].indent);
    }
    attach(parent, blk);
  }
  void begin_line() {
    p_ = lines_[li_].b;
    lim_ = lines_[li_].e;
  }
  bool line_starts(const char* s) const {
    return li_ < lines_.size() && lv_[lines_[li_].b].raw == s;
  }
  // a clause header `kw [expr...] :` on the current line; returns after the ':'
  void clause_header(int node, bool expr_part) {
    begin_line();
    add_leaf(node, p_++);
    const size_t colon = find0(":");
    if (expr_part && p_ < colon) limited(colon, [&] { expression_list_into(node); });
    leaves_to(node, colon);
    if (at(":")) add_leaf(node, p_++);
  }

  void line_statement(int parent) {
    begin_line();
    const int indent = lines_[li_].indent;
    std::string s = t(p_);
    if (s == "async" && (t(p_ + 1) == "def" || t(p_ + 1) == "for" || t(p_ + 1) == "with"))
      s = t(p_ + 1);
    if (s == "if") {
      const int g = make(P_IF);
      attach(parent, g);
      clause_header(g, true);
      suite(g, indent);
      while (li_ < lines_.size() && lines_[li_].indent == indent &&
             (line_starts("elif") || line_starts("else"))) {
        const bool el = line_starts("elif");
        const int c = make(el ? P_ELIF : P_ELSE);
        attach(g, c);
        clause_header(c, el);
        suite(c, indent);
      }
      return;
    }
    if (s == "while") {
      const int g = make(P_WHILE);
      attach(parent, g);
      clause_header(g, true);
      suite(g, indent);
      else_clause(g, indent);
      return;
    }
    if (s == "for") {
      const int g = make(P_FOR);
      attach(parent, g);
      if (t(p_) == "async") add_leaf(g, p_++);
      add_leaf(g, p_++);
      const size_t in = find0("in");
      limited(in, [&] {
        const int left = targets();
        attach(g, left);
        nodes[g].a = left;
        leaves_to(g, lim_);
      });
      if (at("in")) add_leaf(g, p_++);
      const size_t colon = find0(":");
      limited(colon, [&] {
        const int right = expression_list();
        attach(g, right);
        nodes[g].b = right;
        leaves_to(g, lim_);
      });
      if (at(":")) add_leaf(g, p_++);
      suite(g, indent);
      else_clause(g, indent);
      return;
    }
    if (s == "try") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      clause_header(g, false);
      suite(g, indent);
      while (li_ < lines_.size() && lines_[li_].indent == indent &&
             (line_starts("except") || line_starts("else") || line_starts("finally"))) {
        const int c = make(P_GENERIC);
        attach(g, c);
        clause_header(c, line_starts("except"));
        suite(c, indent);
      }
      return;
    }
    if (s == "with") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      if (t(p_) == "async") add_leaf(g, p_++);
      add_leaf(g, p_++);
      const size_t colon = find0(":");
      limited(colon, [&] {
        while (more()) {
          const size_t before = p_;
          const int item = make(P_GENERIC);  // with_item: value [as alias]
          attach(g, item);
          attach(item, expression());
          if (at("as")) {
            add_leaf(item, p_++);
            attach(item, targets());
          }
          if (at(",")) add_leaf(g, p_++);
          if (p_ == before) add_leaf(g, p_++);
        }
      });
      if (at(":")) add_leaf(g, p_++);
      suite(g, indent);
      return;
    }
    if (s == "def") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      if (t(p_) == "async") add_leaf(g, p_++);
      add_leaf(g, p_++);
      if (is_name(t(p_))) add_leaf(g, p_++);
      if (at("(")) parameters(g, P_PARAMS, true);
      const size_t colon = find0(":");
      if (at("->")) {
        add_leaf(g, p_++);
        limited(colon, [&] { attach(g, expression()); });
      }
      leaves_to(g, colon);
      if (at(":")) add_leaf(g, p_++);
      suite(g, indent);
      return;
    }
    if (s == "class") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      if (is_name(t(p_))) add_leaf(g, p_++);
      if (at("(")) attach(g, arguments());
      leaves_to(g, find0(":"));
      if (at(":")) add_leaf(g, p_++);
      suite(g, indent);
      return;
    }
    if (s == "@") {  // decorator line
      const int g = make(P_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      attach(g, expression());
      leaves_to(g, lim_);
      ++li_;
      return;
    }
    simple_statements(parent);
    ++li_;
  }
  void else_clause(int g, int indent) {
    if (li_ < lines_.size() && lines_[li_].indent == indent && line_starts("else")) {
      const int c = make(P_ELSE);
      attach(g, c);
      clause_header(c, false);
      suite(c, indent);
    }
  }

  // simple statements separated by ';' in [p_, lim_)
  void simple_statements(int parent) {
    while (more()) {
      const size_t semi = find0(";");
      limited(semi, [&] {
        const size_t before = p_;
        simple_statement(parent);
        while (more()) add_leaf(parent, p_++);
        if (p_ == before && more()) add_leaf(parent, p_++);
      });
      if (at(";")) add_leaf(parent, p_++);
    }
  }
  void simple_statement(int parent) {
    const std::string& s = t(p_);
    const std::string& nx = t(p_ + 1);
    const bool print_kw = (s == "print" || s == "exec") && nx != "=" && !is_aug_op(nx) &&
                          nx != "." && nx != "[" && nx != ",";
    if (print_kw || s == "return" || s == "del" || s == "raise" || s == "assert" ||
        s == "global" || s == "nonlocal" || s == "yield" || s == "await") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      if (print_kw) kw[p_] = 1;
      add_leaf(g, p_++);
      while (more()) {
        const size_t before = p_;
        if (at(">>") && print_kw) {  // chevron
          const int c = make(P_GENERIC);
          attach(g, c);
          add_leaf(c, p_++);
          attach(c, expression());
        } else {
          attach(g, expression());
        }
        if (at(",") || at("in") || at("from")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
      return;
    }
    if (s == "import" || s == "from" || s == "pass" || s == "break" || s == "continue") {
      const int g = make(P_GENERIC);
      attach(parent, g);
      leaves_to(g, lim_);
      return;
    }
    const int g = make(P_GENERIC);  // expression_statement
    attach(parent, g);
    attach(g, expr_statement());
  }
  // expression list, then `= rhs` (chained), `op= rhs`, or `: type [= rhs]`
  int expr_statement() {
    const int left = expression_list();
    if (left < 0) return left;
    if (at("=") || is_aug_op(t(p_))) {
      const int a = make(P_ASSIGN);
      attach(a, left);
      nodes[a].a = left;
      add_leaf(a, p_++);
      const int r = (find0("=") < lim_) ? expr_statement() : rhs();
      attach(a, r);
      nodes[a].b = r;
      return a;
    }
    if (at(":")) {  // annotated assignment
      const int a = make(P_ASSIGN);
      attach(a, left);
      nodes[a].a = left;
      add_leaf(a, p_++);
      const size_t eq = find0("=");
      limited(eq, [&] { attach(a, expression()); });
      if (at("=")) {
        add_leaf(a, p_++);
        const int r = rhs();
        attach(a, r);
        nodes[a].b = r;
      }
      return a;
    }
    return left;
  }
  int rhs() {
    if (at("yield")) {
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      if (at("from")) add_leaf(g, p_++);
      attach(g, expression_list());
      return g;
    }
    return expression_list();
  }

  // ------------------------------------------------------------------------ parameters
  // '(' parameter (',' parameter)* ')' — identifiers are direct children of `container`
  void parameters(int parent, PT container, bool parens) {
    const int g = make(container);
    attach(parent, g);
    size_t close = lim_;
    if (parens) {
      close = close_of(p_);
      add_leaf(g, p_++);
    }
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        parameter(g);
        if (at(",")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (parens && p_ == close && p_ < n_) add_leaf(g, p_++);
  }
  void parameter(int g) {
    const std::string& s = t(p_);
    if (s == "*" || s == "**") {  // list_splat_pattern / dictionary_splat_pattern / separator
      const int c = make(P_GENERIC);
      attach(g, c);
      add_leaf(c, p_++);
      if (is_name(t(p_))) add_leaf(c, p_++);
      if (at(":")) {
        add_leaf(c, p_++);
        attach(c, expression());
      }
      return;
    }
    if (s == "(") {  // Python 2 tuple parameter
      const int c = make(P_GENERIC);
      attach(g, c);
      const size_t close = close_of(p_);
      leaves_to(c, close + 1);
      return;
    }
    if (!is_name(s)) return;
    if (t(p_ + 1) == "=") {
      const int d = make(P_DEFAULT_PARAM);
      attach(g, d);
      nodes[d].a = add_leaf(d, p_++);
      add_leaf(d, p_++);
      const int v = expression();
      attach(d, v);
      nodes[d].b = v;
      return;
    }
    if (t(p_ + 1) == ":") {  // typed_parameter / typed_default_parameter
      const int c = make(P_GENERIC);
      attach(g, c);
      add_leaf(c, p_++);
      add_leaf(c, p_++);
      attach(c, expression());
      if (at("=")) {
        add_leaf(c, p_++);
        attach(c, expression());
      }
      return;
    }
    add_leaf(g, p_++);
  }

  // ------------------------------------------------------------------------ expressions
  // comma-separated expressions; a single one is returned as is, else an expression_list
  int expression_list() {
    const int first = star_or_expression();
    if (first < 0 || !at(",")) return first;
    const int g = make(P_GENERIC);
    attach(g, first);
    while (at(",")) {
      add_leaf(g, p_++);
      if (!more() || !(is_atom_start(t(p_)) || t(p_) == "-" || t(p_) == "+" || t(p_) == "~" ||
                       t(p_) == "not" || t(p_) == "*" || t(p_) == "lambda" || t(p_) == "await"))
        break;
      attach(g, star_or_expression());
    }
    return g;
  }
  void expression_list_into(int parent) {
    while (more()) {
      const size_t before = p_;
      attach(parent, expression_list());
      if (at(",")) add_leaf(parent, p_++);
      if (p_ == before) break;
    }
  }
  int targets() { return expression_list(); }
  int star_or_expression() {
    if (at("*") || at("**")) {
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      attach(g, or_test());
      return g;
    }
    return expression();
  }
  int expression() {
    if (!more()) return -1;
    if (at("lambda")) return lambda();
    const int c = or_test();
    if (c >= 0 && at("if")) {  // conditional_expression (flat)
      const size_t e = find0("else");
      if (e < lim_) {
        const int g = make(P_GENERIC);
        attach(g, c);
        add_leaf(g, p_++);
        limited(e, [&] { attach(g, or_test()); });
        leaves_to(g, e);
        if (at("else")) add_leaf(g, p_++);
        attach(g, expression());
        return g;
      }
    }
    return c;
  }
  int lambda() {
    const int g = make(P_GENERIC);
    add_leaf(g, p_++);
    const size_t colon = find0(":");
    if (p_ < colon) limited(colon, [&] { parameters(g, P_GENERIC, false); });
    leaves_to(g, colon);
    if (at(":")) add_leaf(g, p_++);
    attach(g, expression());
    return g;
  }
  int or_test() {
    int l = and_test();
    while (l >= 0 && at("or")) {
      const int g = make(P_GENERIC);
      attach(g, l);
      add_leaf(g, p_++);
      attach(g, and_test());
      l = g;
    }
    return l;
  }
  int and_test() {
    int l = not_test();
    while (l >= 0 && at("and")) {
      const int g = make(P_GENERIC);
      attach(g, l);
      add_leaf(g, p_++);
      attach(g, not_test());
      l = g;
    }
    return l;
  }
  int not_test() {
    if (at("not")) {
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      attach(g, not_test());
      return g;
    }
    return comparison();
  }
  int comparison() {
    const int l = binary(1);
    if (l < 0 || !more() || !is_comp_op(t(p_)) || (at("not") && t(p_ + 1) != "in")) return l;
    const int g = make(P_GENERIC);  // comparison_operator: operands and operators flat
    attach(g, l);
    while (more() && is_comp_op(t(p_)) && !(at("not") && t(p_ + 1) != "in")) {
      if (at("not") || (at("is") && t(p_ + 1) == "not")) add_leaf(g, p_++);
      add_leaf(g, p_++);
      attach(g, binary(1));
    }
    return g;
  }
  int binary(int minprec) {
    int l = unary();
    for (;;) {
      if (l < 0 || !more()) break;
      const int prec = bin_prec(t(p_));
      if (prec < 0 || prec < minprec) break;
      const int g = make(P_GENERIC);
      attach(g, l);
      add_leaf(g, p_++);
      attach(g, binary(prec + 1));
      l = g;
    }
    return l;
  }
  int unary() {
    if (at("-") || at("+") || at("~")) {
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      attach(g, unary());
      return g;
    }
    return power();
  }
  int power() {
    int b = await_primary();
    if (b >= 0 && at("**")) {
      const int g = make(P_GENERIC);
      attach(g, b);
      add_leaf(g, p_++);
      attach(g, unary());
      b = g;
    }
    return b;
  }
  int await_primary() {
    if (at("await")) {
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      attach(g, await_primary());
      return g;
    }
    return trailers(atom());
  }
  int trailers(int node) {
    while (node >= 0 && more()) {
      if (at(".") && is_name(t(p_ + 1))) {  // attribute
        const int g = make(P_GENERIC);
        attach(g, node);
        add_leaf(g, p_++);
        add_leaf(g, p_++);
        node = g;
      } else if (at("(")) {  // call
        const int g = make(P_GENERIC);
        attach(g, node);
        attach(g, arguments());
        node = g;
      } else if (at("[")) {  // subscript
        const int g = make(P_GENERIC);
        attach(g, node);
        const size_t close = close_of(p_);
        add_leaf(g, p_++);
        limited(close, [&] {
          while (more()) {
            const size_t before = p_;
            attach(g, slice_or_expr());
            if (at(",")) add_leaf(g, p_++);
            if (p_ == before) add_leaf(g, p_++);
          }
        });
        if (p_ == close && p_ < n_) add_leaf(g, p_++);
        node = g;
      } else {
        break;
      }
    }
    return node;
  }
  int slice_or_expr() {
    const size_t colon = find0(":");
    const size_t comma = find0(",");
    if (colon < comma) {
      const int g = make(P_GENERIC);  // slice
      limited(comma, [&] {
        while (more()) {
          const size_t before = p_;
          if (at(":")) add_leaf(g, p_++);
          else attach(g, expression());
          if (p_ == before) add_leaf(g, p_++);
        }
      });
      return g;
    }
    return star_or_expression();
  }
  // argument_list, or a bare generator_expression as the whole call argument
  int arguments() {
    const size_t close = close_of(p_);
    const int g = make(P_GENERIC);
    add_leaf(g, p_++);
    limited(close, [&] {
      // f(x for x in y) and f(x for x, y in z): the first depth-0 `for` comes before any
      // depth-0 comma (a comma before it makes an argument list)
      if (find0("for") < lim_ && find0("for") < find0(",")) {
        attach(g, expression());
        comprehension_clauses(g);
      }
      while (more()) {
        const size_t before = p_;
        if (is_name(t(p_)) && t(p_ + 1) == "=") {  // keyword_argument
          const int k = make(P_GENERIC);
          attach(g, k);
          add_leaf(k, p_++);
          add_leaf(k, p_++);
          attach(k, expression());
        } else {
          attach(g, star_or_expression());
        }
        if (at(",")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
    return g;
  }
  // for_in_clause / if_clause sequence of a comprehension
  void comprehension_clauses(int g) {
    while (more() && (at("for") || at("if") || (at("async") && t(p_ + 1) == "for"))) {
      if (at("if")) {
        const int c = make(P_GENERIC);
        attach(g, c);
        add_leaf(c, p_++);
        attach(c, or_test_nocond());
        continue;
      }
      const int c = make(P_FOR_IN);
      attach(g, c);
      if (at("async")) add_leaf(c, p_++);
      add_leaf(c, p_++);
      const size_t in = find0("in");
      limited(in, [&] {
        const int left = targets();
        attach(c, left);
        nodes[c].a = left;
        leaves_to(c, lim_);
      });
      if (at("in")) add_leaf(c, p_++);
      attach(c, or_test_nocond());
      while (at(",") && !(t(p_ + 1) == "for" || t(p_ + 1) == "if" || t(p_ + 1).empty())) {
        add_leaf(c, p_++);
        attach(c, or_test_nocond());
      }
    }
  }
  int or_test_nocond() {
    if (at("lambda")) return lambda();
    return or_test();
  }
  int atom() {
    if (!more()) return -1;
    const std::string& s = t(p_);
    if (s == "(" || s == "[" || s == "{") {
      const size_t close = close_of(p_);
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      limited(close, [&] {
        if (at("yield")) {
          attach(g, rhs());
        } else if (s == "{") {
          while (more()) {
            const size_t before = p_;
            if (at("**")) {
              const int c = make(P_GENERIC);
              attach(g, c);
              add_leaf(c, p_++);
              attach(c, or_test());
            } else {
              const int k = star_or_expression();
              if (at(":")) {  // pair
                const int pr = make(P_GENERIC);
                attach(g, pr);
                attach(pr, k);
                add_leaf(pr, p_++);
                attach(pr, expression());
              } else {
                attach(g, k);
              }
            }
            if (at("for") || at("async")) comprehension_clauses(g);
            if (at(",")) add_leaf(g, p_++);
            if (p_ == before) add_leaf(g, p_++);
          }
        } else {
          while (more()) {
            const size_t before = p_;
            attach(g, star_or_expression());
            if (at("for") || at("async")) comprehension_clauses(g);
            if (at(",")) add_leaf(g, p_++);
            if (p_ == before) add_leaf(g, p_++);
          }
        }
      });
      if (p_ == close && p_ < n_) add_leaf(g, p_++);
      return g;
    }
    if (s == "`") {  // Python 2 repr backticks (no tree-sitter rule): leaves
      const int g = make(P_GENERIC);
      add_leaf(g, p_++);
      while (more() && !at("`")) add_leaf(g, p_++);
      if (at("`")) add_leaf(g, p_++);
      return g;
    }
    if (is_string(s)) {
      if (!is_string(t(p_ + 1))) return leaf_node(p_++);
      const int g = make(P_GENERIC);  // concatenated_string
      while (more() && is_string(t(p_))) add_leaf(g, p_++);
      return g;
    }
    if (is_name(s) || is_number(s) || s == "...") return leaf_node(p_++);
    if (s == "print" || s == "exec") return leaf_node(p_++);
    return -1;
  }
};

// ------------------------------------------------------------------------------ DFG_python walk
struct PWalker {
  const std::vector<PNode>& nd;
  const std::vector<Leaf>& lv;
  std::vector<char> anon, str, ident;
  // GraphCodeBERT's parser/DFG.py DFG_python: strings are not skipped and every named leaf
  // outside the states is an entry (identifiers define themselves on first sight)
  bool ms = false;

  PWalker(const std::vector<PNode>& n, const std::vector<Leaf>& l, const std::vector<char>& kw,
          bool ms_variant)
      : nd(n), lv(l), ms(ms_variant) {
    anon.resize(l.size());
    str.resize(l.size());
    ident.resize(l.size());
    for (size_t i = 0; i < l.size(); ++i) {
      const std::string& r = l[i].raw;
      bool a;
      if (is_string(r) || is_number(r) || r == "...") a = false;
      else if (id_like(r)) a = py_keywords().count(r) > 0 || kw[i];
      else a = true;
      // node type == recorded code only while the byte-column slice is intact
      anon[i] = a && l[i].text == r;
      str[i] = is_string(r);
      ident[i] = !a && is_name(r) && r != "True" && r != "False" && r != "None";
    }
  }

  void var_index(int x, std::vector<int>& out) const {  // tree_to_variable_index
    if (x < 0) return;
    if (nd[x].type == P_LEAF) {
      if (!anon[nd[x].leaf]) out.push_back(nd[x].leaf);
      return;
    }
    for (int k : nd[x].kids) var_index(k, out);
  }
  bool is_comma(int x) const { return nd[x].type == P_LEAF && lv[nd[x].leaf].raw == ","; }
  std::vector<int> split_children(int x) const {  // [c for c in x.children if c.type != ',']
    std::vector<int> out;
    if (x < 0 || nd[x].type == P_LEAF) return out;
    for (int k : nd[x].kids)
      if (!is_comma(k)) out.push_back(k);
    return out;
  }
  // the left <- right pairing of an assignment / for statement (DFG_python.py:49-76, :115-139)
  void pair_sides(int left, int right, std::vector<DfgEdge>& dfg, DfgStates& st) const {
    std::vector<int> ln = split_children(left), rn = split_children(right);
    if (rn.size() != ln.size()) {
      ln = {left};
      rn = {right};
    }
    if (ln.empty()) ln = {left};
    if (rn.empty()) rn = {right};
    for (int r : rn) dfg_append(dfg, walk(r, st));
    const size_t m = std::min(ln.size(), rn.size());
    for (size_t k = 0; k < m; ++k) {
      std::vector<int> li, ri;
      var_index(ln[k], li);
      var_index(rn[k], ri);
      std::vector<std::string> rc;
      for (int i : ri) rc.push_back(lv[i].text);
      for (int i1 : li) {
        dfg.push_back({lv[i1].text, i1, true, rc, ri});
        st[lv[i1].text] = {i1};
      }
    }
  }

  std::vector<DfgEdge> walk(int x, DfgStates& st) const {
    std::vector<DfgEdge> dfg;
    if (x < 0) return dfg;
    const PNode& n = nd[x];
    switch (n.type) {
      case P_LEAF: {
        const int idx = n.leaf;
        if (anon[idx] || (str[idx] && !ms)) return dfg;
        const std::string& code = lv[idx].text;
        auto it = st.find(code);
        if (it != st.end()) {
          dfg.push_back({code, idx, false, {code}, it->second});
        } else if (ms) {
          if (ident[idx]) st[code] = {idx};
          dfg.push_back({code, idx, false, {}, {}});
        } else if (n.parent >= 0 && nd[n.parent].type == P_PARAMS && is_name(lv[idx].raw)) {
          st[code] = {idx};
          dfg.push_back({code, idx, false, {}, {}});
        }
        return dfg;
      }
      case P_DEFAULT_PARAM: {
        std::vector<int> ni, vi;
        var_index(n.a, ni);
        if (n.b < 0) {
          for (int i : ni) {
            dfg.push_back({lv[i].text, i, false, {}, {}});
            st[lv[i].text] = {i};
          }
        } else {
          var_index(n.b, vi);
          dfg_append(dfg, walk(n.b, st));
          for (int i1 : ni) {
            for (int i2 : vi) dfg.push_back({lv[i1].text, i1, false, {lv[i2].text}, {i2}});
            st[lv[i1].text] = {i1};
          }
        }
        dfg_sort(dfg);
        return dfg;
      }
      case P_ASSIGN: {
        if (n.b < 0) return dfg;
        pair_sides(n.a, n.b, dfg, st);
        dfg_sort(dfg);
        return dfg;
      }
      case P_FOR_IN: {
        const int right = n.kids.empty() ? -1 : n.kids.back();
        dfg_append(dfg, walk(right, st));
        std::vector<int> li, ri;
        var_index(n.a, li);
        var_index(right, ri);
        std::vector<std::string> rc;
        for (int i : ri) rc.push_back(lv[i].text);
        for (int i1 : li) {
          dfg.push_back({lv[i1].text, i1, true, rc, ri});
          st[lv[i1].text] = {i1};
        }
        dfg_sort(dfg);
        return dfg;
      }
      case P_IF: {
        DfgStates current = st;
        std::vector<DfgStates> others;
        bool tag = false;
        for (int k : n.kids) {
          if (nd[k].type == P_ELSE) tag = true;
          if (nd[k].type != P_ELIF && nd[k].type != P_ELSE) {
            dfg_append(dfg, walk(k, current));
          } else {
            DfgStates ns = st;
            dfg_append(dfg, walk(k, ns));
            others.push_back(std::move(ns));
          }
        }
        others.push_back(std::move(current));
        if (!tag) others.push_back(std::move(st));
        st = dfg_union(std::move(others));
        dfg_sort(dfg);
        return dfg;
      }
      case P_FOR: {
        for (int rep = 0; rep < 2; ++rep) {
          pair_sides(n.a, n.b, dfg, st);
          if (!n.kids.empty() && nd[n.kids.back()].type == P_BLOCK)
            dfg_append(dfg, walk(n.kids.back(), st));
        }
        dfg_merge_dup(dfg);
        return dfg;
      }
      case P_WHILE: {
        for (int rep = 0; rep < 2; ++rep)
          for (int k : n.kids) dfg_append(dfg, walk(k, st));
        dfg_merge_dup(dfg);
        return dfg;
      }
      default: {
        for (int k : n.kids)
          if (nd[k].type == P_FOR_IN) dfg_append(dfg, walk(k, st));
        for (int k : n.kids)
          if (nd[k].type != P_FOR_IN) dfg_append(dfg, walk(k, st));
        dfg_sort(dfg);
        return dfg;
      }
    }
  }
};

}  // namespace

std::vector<DfgEdge> dfg_python(const std::vector<Leaf>& leaves, bool ms) {
  if (leaves.empty()) return {};
  PyTree tree(leaves);
  const int root = tree.parse();
  PWalker w(tree.nodes, leaves, tree.kw, ms);
  DfgStates states;
  std::vector<DfgEdge> d = w.walk(root, states);
  dfg_sort(d);
  return d;
}

}  // namespace ah
