// dfg_java.cpp — Java data-flow graph and identifier list without tree-sitter.
//
// Restates python_parser/parser_folder/DFG_java.py:10-191 (the walk) over a Java syntax tree this
// file builds from the lexer's leaves (lexer.cpp), with the tree-sitter-java node kinds DFG_java
// looks at:
//   variable_declarator {name, value}     local / field declarations, for-init, `T... args`
//   formal_parameter                       its identifier child is a definition (method, lambda
//                                          and constructor parameters; NOT catch parameters,
//                                          resources or inferred lambda parameters)
//   assignment_expression {left, right}    every operator (=, +=, ...)
//   update_expression                      ++ / -- (prefix and postfix)
//   method_invocation {object, arguments}  with an object only the object and the arguments are
//                                          walked (the method name never reaches the graph)
//   if_statement / for_statement / enhanced_for_statement {name, value, body} / while_statement
// and every other node generic (DFG_java only recurses through it).
//
// The snippets are bare methods, which tree-sitter-java's `program: repeat(statement)` cannot
// parse; its error recovery keeps `<modifiers> <type> name` as a local variable declaration
// without a value (the method name becomes a definition, first in the graph) and the parameter
// list as formal parameters.  The reference's own fixture keys (the substitute keys of
// CodeXGLUE/Clone-detection-BigCloneBench/dataset/test_subs_*.jsonl, which are
// get_identifiers(code1) in graph order filtered to names with substitutes) show exactly that
// pattern; tests/test_host.py measures the match.  Leaf classes: keywords, punctuation, `this`,
// `super`, `true`, `false` are anonymous (node type == text); identifiers, type names, literals,
// `null`, `boolean` and `void` (named leaf rules) are not.
#include <unordered_set>

#include "dfg_util.h"

namespace ah {
namespace {

enum JT : uint8_t {
  J_LEAF,
  J_GENERIC,
  J_LVD,         // local_variable_declaration (marks the for-init for DFG_java's second pass)
  J_DECLARATOR,  // a = name, b = value
  J_FORMAL,      // formal_parameter
  J_ASSIGN,      // a = left, b = right
  J_UPDATE,
  J_IF,
  J_FOR,
  J_ENH_FOR,     // a = name, b = value, c = body
  J_WHILE,
  J_INVOKE,      // a = object (or -1), b = arguments
};

struct JNode {
  JT type = J_GENERIC;
  int leaf = -1;
  int parent = -1;
  int a = -1, b = -1, c = -1;
  bool pname = false;  // J_LEAF: the identifier child of a formal_parameter
  bool tid = false;    // J_LEAF: a type name (type_identifier / scoped type), not an identifier
  std::vector<int> kids;
};

const std::unordered_set<std::string>& java_anon_words() {
  // keyword tokens whose node type equals their text ('this', 'super', 'true', 'false' are named
  // rules of one keyword each, which the walk treats alike since type == text)
  static const std::unordered_set<std::string> k = {
      "abstract", "assert",  "break",    "byte",       "case",      "catch",     "char",
      "class",    "continue", "default", "do",         "double",    "else",      "enum",
      "extends",  "final",   "finally",  "float",      "for",       "if",        "implements",
      "import",   "instanceof", "int",   "interface",  "long",      "native",    "new",
      "package",  "private", "protected", "public",    "return",    "short",     "static",
      "strictfp", "super",   "switch",   "synchronized", "this",    "throw",     "throws",
      "transient", "try",    "volatile", "while",      "true",      "false"};
  return k;
}
bool primitive_word(const std::string& s) {
  return s == "byte" || s == "short" || s == "int" || s == "long" || s == "char" ||
         s == "float" || s == "double" || s == "boolean" || s == "void";
}
bool id_like(const std::string& t) {
  if (t.empty()) return false;
  const unsigned char c = (unsigned char)t[0];
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c == '$' || c >= 0x80;
}
bool is_ident(const std::string& t) {
  return id_like(t) && !java_anon_words().count(t) && !primitive_word(t) && t != "null";
}
bool leaf_anon(const std::string& t) {
  if (t.empty()) return true;
  if (id_like(t)) return java_anon_words().count(t) > 0;
  const unsigned char c = (unsigned char)t[0];
  if (c >= '0' && c <= '9') return false;  // numeric literal
  if (c == '.' && t.size() > 1 && t[1] >= '0' && t[1] <= '9') return false;
  if (c == '"' || c == '\'') return false;  // string / character literal
  return true;                              // operators, punctuation, '@'
}
bool is_assign_op(const std::string& t) {
  return t == "=" || t == "+=" || t == "-=" || t == "*=" || t == "/=" || t == "%=" ||
         t == "&=" || t == "|=" || t == "^=" || t == "<<=" || t == ">>=" || t == ">>>=";
}
int binary_prec(const std::string& t) {
  if (t == "||") return 1;
  if (t == "&&") return 2;
  if (t == "|") return 3;
  if (t == "^") return 4;
  if (t == "&") return 5;
  if (t == "==" || t == "!=") return 6;
  if (t == "<" || t == ">" || t == "<=" || t == ">=" || t == "instanceof") return 7;
  if (t == "<<" || t == ">>" || t == ">>>") return 8;
  if (t == "+" || t == "-") return 9;
  if (t == "*" || t == "/" || t == "%") return 10;
  return -1;
}
bool is_literal(const std::string& t) {
  if (t.empty()) return false;
  const unsigned char c = (unsigned char)t[0];
  return (c >= '0' && c <= '9') || c == '"' || c == '\'' ||
         (c == '.' && t.size() > 1 && t[1] >= '0' && t[1] <= '9') || t == "null" ||
         t == "true" || t == "false";
}

class JTree {
 public:
  explicit JTree(const std::vector<Leaf>& lv) : lv_(lv), n_(lv.size()) {
    match_.assign(n_, -1);
    std::vector<int> st;
    for (size_t i = 0; i < n_; ++i) {
      const std::string& s = lv[i].raw;
      if (s == "(" || s == "[" || s == "{") {
        st.push_back((int)i);
      } else if (s == ")" || s == "]" || s == "}") {
        const char open = s == ")" ? '(' : s == "]" ? '[' : '{';
        for (int k = (int)st.size() - 1; k >= 0; --k)
          if (lv[st[k]].raw[0] == open) {
            match_[st[k]] = (int)i;
            match_[i] = st[k];
            st.resize(k);
            break;
          }
      }
    }
    lim_ = n_;
  }

  int parse() {
    const int root = make(J_GENERIC);
    method_header(root);
    while (p_ < n_) {
      const size_t before = p_;
      statement(root);
      if (p_ == before) add_leaf(root, p_++);
    }
    return root;
  }

  std::vector<JNode> nodes;

 private:
  const std::vector<Leaf>& lv_;
  size_t n_;
  size_t p_ = 0;
  size_t lim_;
  std::vector<int> match_;

  // ------------------------------------------------------------------------ tree helpers
  int make(JT t) {
    nodes.push_back(JNode());
    nodes.back().type = t;
    return (int)nodes.size() - 1;
  }
  void attach(int parent, int child) {
    if (child < 0) return;
    nodes[child].parent = parent;
    nodes[parent].kids.push_back(child);
  }
  int leaf_node(size_t i) {
    const int x = make(J_LEAF);
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
    return i < n_ && i < lim_ ? lv_[i].raw : empty;
  }
  bool more() const { return p_ < lim_ && p_ < n_; }
  bool at(const char* s) const { return more() && lv_[p_].raw == s; }
  // index of the closer matching the opener at i, clipped to the current limit
  size_t close_of(size_t i) const {
    const int m = match_[i];
    if (m < 0 || (size_t)m >= lim_) return lim_ > 0 ? lim_ - 1 : 0;
    return (size_t)m;
  }
  // run f with the parse limited to [p_, lim)
  template <class F>
  void limited(size_t lim, F f) {
    const size_t saved = lim_;
    lim_ = std::min(lim, saved);
    f();
    lim_ = saved;
  }
  // leaves up to (excluding) e
  void leaves_to(int parent, size_t e) {
    while (more() && p_ < e) add_leaf(parent, p_++);
  }
  // leaves of a type (modifiers, annotations, type arguments) up to e: names are type names
  void type_leaves(int parent, size_t e) {
    while (more() && p_ < e) nodes[add_leaf(parent, p_++)].tid = true;
  }
  void group_leaves(int parent) {  // a balanced group at p_ as plain leaves
    const size_t e = close_of(p_);
    while (more() && p_ <= e) add_leaf(parent, p_++);
  }

  // ------------------------------------------------------------------------ lookahead
  size_t skip_annotation(size_t q) const {  // '@' Name(.Name)* [ (...) ]
    if (t(q) != "@" || t(q + 1) == "interface") return q;
    ++q;
    if (id_like(t(q))) ++q;
    while (t(q) == "." && id_like(t(q + 1))) q += 2;
    if (t(q) == "(" && match_[q] >= 0) q = (size_t)match_[q] + 1;
    return q;
  }
  static bool modifier_word(const std::string& s) {
    return s == "public" || s == "private" || s == "protected" || s == "static" ||
           s == "final" || s == "abstract" || s == "native" || s == "synchronized" ||
           s == "transient" || s == "volatile" || s == "strictfp" || s == "default";
  }
  size_t skip_modifiers(size_t q) const {
    for (;;) {
      if (t(q) == "@" && t(q + 1) != "interface") {
        q = skip_annotation(q);
      } else if (modifier_word(t(q)) && !(t(q) == "synchronized" && t(q + 1) == "(") &&
                 !(t(q) == "default" && t(q + 1) == ":")) {
        ++q;
      } else {
        return q;
      }
    }
  }
  // '<' ... '>' of type arguments / parameters; returns the index after it, or 0 on failure
  size_t skip_type_args(size_t q) const {
    if (t(q) != "<") return 0;
    int depth = 0;
    for (; q < n_ && q < lim_; ++q) {
      const std::string& s = t(q);
      if (s == "<") ++depth;
      else if (s == ">") depth -= 1;
      else if (s == ">>") depth -= 2;
      else if (s == ">>>") depth -= 3;
      else if (!(id_like(s) || s == "." || s == "," || s == "?" || s == "[" || s == "]" ||
                 s == "&" || s == "@"))
        return 0;
      if (depth <= 0) return depth == 0 ? q + 1 : 0;
    }
    return 0;
  }
  // a type at q; returns the index after it, or 0
  size_t skip_type(size_t q) const {
    while (t(q) == "@") q = skip_annotation(q);
    const std::string& s = t(q);
    if (primitive_word(s)) {
      ++q;
    } else if (is_ident(s)) {
      ++q;
      for (;;) {
        if (t(q) == "<") {
          const size_t r = skip_type_args(q);
          if (!r) return 0;
          q = r;
        }
        if (t(q) == "." && is_ident(t(q + 1))) {
          q += 2;
          continue;
        }
        break;
      }
    } else {
      return 0;
    }
    while (t(q) == "[" && t(q + 1) == "]") q += 2;
    return q;
  }
  bool looks_like_lvd(size_t q) const {
    q = skip_modifiers(q);
    const size_t r = skip_type(q);
    if (!r || !is_ident(t(r))) return false;
    const std::string& f = t(r + 1);
    return f == "=" || f == ";" || f == "," || f == "[" || f == ":";
  }
  bool class_ahead(size_t q) const {
    q = skip_modifiers(q);
    const std::string& s = t(q);
    return s == "class" || s == "interface" || s == "enum" || (s == "@" && t(q + 1) == "interface");
  }

  // ------------------------------------------------------------------------ declarations
  // the top-level bare method: `<mods> <type> name (params) [throws ...] { body }` -> a local
  // variable declaration of `name` (no value), formal parameters, the rest, the body block
  void method_header(int root) {
    size_t q = skip_modifiers(0);
    if (t(q) == "<") {
      const size_t r = skip_type_args(q);
      if (!r) return;
      q = r;
    }
    size_t name = 0;
    bool typed = false;
    if (is_ident(t(q)) && t(q + 1) == "(") {
      name = q;  // constructor
    } else {
      const size_t r = skip_type(q);
      if (!r || !is_ident(t(r)) || t(r + 1) != "(") return;
      name = r;
      typed = true;
    }
    if (!typed && (q == 0 || (t(q + 1) == "(" && t(q + 2) == ")"))) {
      // a constructor with no modifier (`Name(T p) throws E {`), or with modifiers and no
      // parameters (`public Name() throws A, B {`): tree-sitter recovers it as a call — its
      // parameters are plain leaves, not definitions — followed by a declaration whose
      // declarators are the simple exception types of `throws` (the BigCloneBench fixture keys
      // of `HttpRepository`: its one type; of `FileChooserTestFrame`: both of its two)
      leaves_to(root, name + 1);
      leaves_to(root, close_of(p_) + 1);
      if (at("throws") && is_ident(t(p_ + 1))) {
        add_leaf(root, p_++);
        const int lvd0 = make(J_LVD);
        attach(root, lvd0);
        for (;;) {
          const int d = make(J_DECLARATOR);
          attach(lvd0, d);
          nodes[d].a = add_leaf(d, p_++);
          if (!(at(",") && is_ident(t(p_ + 1)) &&
                (t(p_ + 2) == "," || t(p_ + 2) == "{" || t(p_ + 2) == ";")))
            break;
          add_leaf(lvd0, p_++);
        }
      }
      while (more() && !at("{") && !at(";")) add_leaf(root, p_++);
      return;
    }
    int lvd = -1;
    if (typed) {
      lvd = make(J_LVD);
      attach(root, lvd);
      type_leaves(lvd, name);
      const int d = make(J_DECLARATOR);
      attach(lvd, d);
      nodes[d].a = add_leaf(d, p_++);
    } else {
      leaves_to(root, name + 1);
    }
    // parameter count (depth-0 commas of the parameter list + 1, 0 when empty)
    int nparams = 0;
    if (at("(")) {
      const size_t close = close_of(p_);
      if (close > p_ + 1) nparams = 1;
      int angle = 0;
      for (size_t q = p_ + 1; q < close; ++q) {
        const std::string& s = t(q);
        if (s == "(" || s == "[" || s == "{") q = close_of(q);
        else if (s == "<") ++angle;
        else if (s == ">") --angle;
        else if (s == ">>") angle -= 2;
        else if (s == "," && angle <= 0) ++nparams;
      }
    }
    formal_parameters(root);
    // `throws A, B, C`: after at most one parameter (or after a qualified A) the recovered
    // declaration continues past the first exception type, so every later simple name is one more
    // declarator — the fixture keys list B and C (never A) exactly in those headers and never
    // after two or more parameters
    // A header that starts with a marker annotation (`@Override`, no arguments) shifts the
    // recovery one type further: the declarators start at the third type, after at most two
    // parameters (`@Override ... (String message) throws A, B, C, D` keys C and D; `@Override ...
    // (URL url, String skin) throws A, B, C` keys C; no marker-annotated header with two types
    // keys either).
    bool more_decls = false;
    int skip_decls = 0;
    if (at("throws")) {
      size_t q = p_ + 1;
      bool qualified = false;
      while (is_ident(t(q)) && t(q + 1) == ".") {
        qualified = true;
        q += 2;
      }
      const bool marker = t(0) == "@" && is_ident(t(1)) && t(2) != "(" && t(2) != ".";
      if (marker && !qualified) {
        more_decls = nparams <= 2;
        skip_decls = 1;
      } else {
        more_decls = nparams <= 1 || qualified;
      }
    }
    while (more() && !at("{") && !at(";")) {
      if (lvd >= 0 && more_decls && at(",") && is_ident(t(p_ + 1)) &&
          (t(p_ + 2) == "," || t(p_ + 2) == "{" || t(p_ + 2) == ";")) {
        if (skip_decls > 0) {
          --skip_decls;
          add_leaf(root, p_++);
          add_leaf(root, p_++);
          continue;
        }
        add_leaf(lvd, p_++);
        const int d = make(J_DECLARATOR);
        attach(lvd, d);
        nodes[d].a = add_leaf(d, p_++);
        continue;
      }
      add_leaf(root, p_++);  // dims, throws, the first exception type
    }
  }

  // '(' formal_parameter (',' formal_parameter)* ')'
  void formal_parameters(int parent) {
    if (!at("(")) return;
    const int g = make(J_GENERIC);
    attach(parent, g);
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      while (more()) {
        // one parameter: up to the next depth-0 comma (type arguments nest with '<' '>')
        size_t e = p_;
        int angle = 0;
        while (e < lim_) {
          const std::string& s = t(e);
          if (s == "(" || s == "[" || s == "{") {
            e = close_of(e) + 1;
            continue;
          }
          if (s == "<") ++angle;
          else if (s == ">") --angle;
          else if (s == ">>") angle -= 2;
          else if (s == ">>>") angle -= 3;
          else if (s == "," && angle <= 0) break;
          ++e;
        }
        formal_parameter(g, e);
        if (at(",")) add_leaf(g, p_++);
        else if (more()) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
  }
  void formal_parameter(int parent, size_t e) {
    // name = the last identifier before trailing dims; `T... name` is a spread_parameter whose
    // name sits in a variable_declarator
    size_t end = e;
    while (end >= p_ + 2 && t(end - 1) == "]" && t(end - 2) == "[") end -= 2;
    const bool spread = end >= p_ + 2 && t(end - 2) == "...";
    const int f = make(J_FORMAL);
    attach(parent, f);
    if (end == p_ || !is_ident(t(end - 1))) {
      leaves_to(f, e);
      return;
    }
    const size_t name = end - 1;
    type_leaves(f, name);
    if (spread) {
      const int d = make(J_DECLARATOR);
      attach(f, d);
      nodes[d].a = add_leaf(d, p_++);
      leaves_to(d, e);
    } else {
      const int x = add_leaf(f, p_++);
      nodes[x].pname = true;
      leaves_to(f, e);
    }
  }

  // [modifiers] type declarator (',' declarator)* [';']
  int local_var_decl(int parent, JT kind = J_LVD) {
    const int g = make(kind);
    attach(parent, g);
    const size_t q = skip_type(skip_modifiers(p_));
    type_leaves(g, q);
    while (more()) {
      if (!is_ident(t(p_))) break;
      declarator(g);
      if (at(",")) {
        add_leaf(g, p_++);
        continue;
      }
      break;
    }
    while (more() && !at(";")) add_leaf(g, p_++);  // resync
    if (at(";")) add_leaf(g, p_++);
    return g;
  }
  void declarator(int parent) {
    const int d = make(J_DECLARATOR);
    attach(parent, d);
    nodes[d].a = add_leaf(d, p_++);
    while (at("[") && t(p_ + 1) == "]") {
      add_leaf(d, p_++);
      add_leaf(d, p_++);
    }
    if (at("=")) {
      add_leaf(d, p_++);
      const int v = at("{") ? array_initializer() : expr();
      attach(d, v);
      nodes[d].b = v;
    }
  }
  int array_initializer() {
    const int g = make(J_GENERIC);
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        attach(g, at("{") ? array_initializer() : expr());
        if (at(",")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
    return g;
  }

  void class_decl(int parent) {
    const int g = make(J_GENERIC);
    attach(parent, g);
    while (more() && !at("{")) add_leaf(g, p_++);
    if (at("{")) class_body(g);
  }
  void class_body(int parent) {
    const int g = make(J_GENERIC);
    attach(parent, g);
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        member(g);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
  }
  void member(int parent) {
    if (at(";")) {
      add_leaf(parent, p_++);
      return;
    }
    if (at("{")) {
      block(parent);
      return;
    }
    if (at("static") && t(p_ + 1) == "{") {
      const int g = make(J_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      block(g);
      return;
    }
    if (class_ahead(p_)) {
      class_decl(parent);
      return;
    }
    size_t q = skip_modifiers(p_);
    if (t(q) == "<") {
      const size_t r = skip_type_args(q);
      if (r) q = r;
    }
    size_t name = 0;
    if (is_ident(t(q)) && t(q + 1) == "(") {
      name = q;  // constructor
    } else {
      const size_t r = skip_type(q);
      if (r && is_ident(t(r)) && t(r + 1) == "(") name = r;  // method
      else if (r && is_ident(t(r))) {                        // field_declaration
        local_var_decl(parent, J_GENERIC);
        return;
      }
    }
    if (!name) {
      statement(parent);
      return;
    }
    const int g = make(J_GENERIC);  // method_declaration / constructor_declaration
    attach(parent, g);
    type_leaves(g, name);
    add_leaf(g, p_++);
    formal_parameters(g);
    while (more() && !at("{") && !at(";")) add_leaf(g, p_++);
    if (at("{")) block(g);
    else if (at(";")) add_leaf(g, p_++);
  }

  // ------------------------------------------------------------------------ statements
  void block(int parent) {
    const int g = make(J_GENERIC);
    attach(parent, g);
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        statement(g);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
  }
  void paren_expr(int parent) {  // parenthesized_expression
    if (!at("(")) return;
    const int g = make(J_GENERIC);
    attach(parent, g);
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      attach(g, expr());
      while (more()) add_leaf(g, p_++);
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
  }
  void end_statement(int g) {  // resync to the ';' of a statement
    while (more() && !at(";")) {
      if (at("{") || at("(") || at("[")) group_leaves(g);
      else add_leaf(g, p_++);
    }
    if (at(";")) add_leaf(g, p_++);
  }

  void statement(int parent) {
    if (!more()) return;
    const std::string& s = t(p_);
    if (s == "{") return block(parent);
    if (s == ";") {
      add_leaf(parent, p_++);
      return;
    }
    if (s == "if") {
      const int g = make(J_IF);
      attach(parent, g);
      add_leaf(g, p_++);
      paren_expr(g);
      statement(g);
      if (at("else")) {
        add_leaf(g, p_++);
        statement(g);
      }
      return;
    }
    if (s == "while") {
      const int g = make(J_WHILE);
      attach(parent, g);
      add_leaf(g, p_++);
      paren_expr(g);
      statement(g);
      return;
    }
    if (s == "do") {
      const int g = make(J_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      statement(g);
      if (at("while")) {
        add_leaf(g, p_++);
        paren_expr(g);
      }
      if (at(";")) add_leaf(g, p_++);
      return;
    }
    if (s == "for" && t(p_ + 1) == "(") return for_statement(parent);
    if (s == "try") return try_statement(parent);
    if (s == "switch") {
      switch_block(parent);
      return;
    }
    if (s == "synchronized" && t(p_ + 1) == "(") {
      const int g = make(J_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      paren_expr(g);
      if (at("{")) block(g);
      return;
    }
    if (s == "return" || s == "throw" || s == "break" || s == "continue" || s == "assert" ||
        (s == "yield" && !is_assign_op(t(p_ + 1)) && t(p_ + 1) != "(" && t(p_ + 1) != ".")) {
      const int g = make(J_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      while (more() && !at(";")) {
        const size_t before = p_;
        attach(g, expr());
        if (at(":") || at(",")) add_leaf(g, p_++);
        if (p_ == before) break;
      }
      end_statement(g);
      return;
    }
    if (class_ahead(p_)) return class_decl(parent);
    if (is_ident(s) && t(p_ + 1) == ":") {  // labeled_statement
      const int g = make(J_GENERIC);
      attach(parent, g);
      add_leaf(g, p_++);
      add_leaf(g, p_++);
      statement(g);
      return;
    }
    if (looks_like_lvd(p_)) {
      local_var_decl(parent);
      return;
    }
    const int g = make(J_GENERIC);  // expression_statement
    attach(parent, g);
    attach(g, expr());
    end_statement(g);
  }

  void for_statement(int parent) {
    const size_t open = p_ + 1;
    const size_t close = close_of(open);
    // enhanced for: a depth-0 ':' and no depth-0 ';' inside the parentheses
    bool colon = false, semi = false;
    for (size_t q = open + 1; q < close;) {
      const std::string& s = t(q);
      if (s == "(" || s == "[" || s == "{") {
        q = close_of(q) + 1;
        continue;
      }
      if (s == ":") colon = true;
      if (s == ";") semi = true;
      ++q;
    }
    if (colon && !semi) {
      const int g = make(J_ENH_FOR);
      attach(parent, g);
      add_leaf(g, p_++);
      add_leaf(g, p_++);
      limited(close, [&] {
        size_t c = p_;
        while (c < lim_ && t(c) != ":") ++c;
        size_t nm = c;
        while (nm >= p_ + 2 && t(nm - 1) == "]" && t(nm - 2) == "[") nm -= 2;
        if (nm > p_ && is_ident(t(nm - 1))) {
          type_leaves(g, nm - 1);
          nodes[g].a = add_leaf(g, p_++);
        }
        leaves_to(g, c);
        if (at(":")) add_leaf(g, p_++);
        const int v = expr();
        attach(g, v);
        nodes[g].b = v;
        while (more()) add_leaf(g, p_++);
      });
      if (p_ == close && p_ < n_) add_leaf(g, p_++);
      const size_t before = nodes[g].kids.size();
      statement(g);
      if (nodes[g].kids.size() > before) nodes[g].c = nodes[g].kids.back();
      return;
    }
    const int g = make(J_FOR);
    attach(parent, g);
    add_leaf(g, p_++);
    add_leaf(g, p_++);
    limited(close, [&] {
      if (looks_like_lvd(p_)) {
        local_var_decl(g);
      } else {
        while (more() && !at(";")) {
          const size_t before = p_;
          attach(g, expr());
          if (at(",")) add_leaf(g, p_++);
          if (p_ == before) add_leaf(g, p_++);
        }
        if (at(";")) add_leaf(g, p_++);
      }
      if (!at(";")) attach(g, expr());
      while (more() && !at(";")) add_leaf(g, p_++);
      if (at(";")) add_leaf(g, p_++);
      while (more()) {
        const size_t before = p_;
        attach(g, expr());
        if (at(",")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
    statement(g);
  }

  void try_statement(int parent) {
    const int g = make(J_GENERIC);
    attach(parent, g);
    add_leaf(g, p_++);
    if (at("(")) {  // resource_specification: resources are not declarators
      const int r = make(J_GENERIC);
      attach(g, r);
      const size_t close = close_of(p_);
      add_leaf(r, p_++);
      limited(close, [&] {
        while (more()) {
          const size_t before = p_;
          const int res = make(J_GENERIC);
          attach(r, res);
          const size_t q = skip_type(skip_modifiers(p_));
          if (q && is_ident(t(q)) && t(q + 1) == "=") {
            type_leaves(res, q);
            leaves_to(res, q + 2);
            attach(res, expr());
          } else {
            attach(res, expr());
          }
          if (at(";")) add_leaf(r, p_++);
          if (p_ == before) add_leaf(r, p_++);
        }
      });
      if (p_ == close && p_ < n_) add_leaf(r, p_++);
    }
    if (at("{")) block(g);
    while (at("catch")) {
      const int c = make(J_GENERIC);
      attach(g, c);
      add_leaf(c, p_++);
      if (at("(")) {
        const int fp = make(J_GENERIC);  // catch_formal_parameter: not a definition
        attach(c, fp);
        const size_t close = close_of(p_);
        size_t nm = close;  // the name: the last identifier before ')'
        while (nm > p_ && !is_ident(t(nm - 1))) --nm;
        add_leaf(fp, p_++);
        type_leaves(fp, nm > p_ ? nm - 1 : p_);
        leaves_to(fp, close + 1);
      }
      if (at("{")) block(c);
    }
    if (at("finally")) {
      const int f = make(J_GENERIC);
      attach(g, f);
      add_leaf(f, p_++);
      if (at("{")) block(f);
    }
  }

  int switch_block(int parent) {
    const int g = make(J_GENERIC);
    attach(parent, g);
    add_leaf(g, p_++);
    paren_expr(g);
    if (!at("{")) return g;
    const int body = make(J_GENERIC);
    attach(g, body);
    const size_t close = close_of(p_);
    add_leaf(body, p_++);
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        if (at("case")) {
          const int lab = make(J_GENERIC);
          attach(body, lab);
          add_leaf(lab, p_++);
          while (more() && !at(":") && !at("->")) {
            const size_t b2 = p_;
            attach(lab, expr());
            if (at(",")) add_leaf(lab, p_++);
            if (p_ == b2) add_leaf(lab, p_++);
          }
          if (more()) add_leaf(lab, p_++);
        } else if (at("default") && (t(p_ + 1) == ":" || t(p_ + 1) == "->")) {
          const int lab = make(J_GENERIC);
          attach(body, lab);
          add_leaf(lab, p_++);
          add_leaf(lab, p_++);
        } else {
          statement(body);
        }
        if (p_ == before) add_leaf(body, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(body, p_++);
    return g;
  }

  // ------------------------------------------------------------------------ expressions
  bool lambda_ahead() const {
    if (is_ident(t(p_)) && t(p_ + 1) == "->") return true;
    if (at("(") && match_[p_] >= 0 && (size_t)match_[p_] + 1 < lim_ &&
        t((size_t)match_[p_] + 1) == "->")
      return true;
    return false;
  }
  int lambda() {
    const int g = make(J_GENERIC);
    if (at("(")) {
      // inferred_parameters (identifiers only) vs formal_parameters
      const size_t close = close_of(p_);
      bool inferred = true;
      for (size_t q = p_ + 1; q < close; ++q)
        if (!(is_ident(t(q)) || t(q) == ",")) inferred = false;
      if (inferred) group_leaves(g);
      else formal_parameters(g);
    } else {
      add_leaf(g, p_++);
    }
    if (at("->")) add_leaf(g, p_++);
    if (at("{")) block(g);
    else attach(g, expr());
    return g;
  }

  int expr() {
    if (!more()) return -1;
    if (lambda_ahead()) return lambda();
    const int lhs = ternary();
    if (lhs >= 0 && more() && is_assign_op(t(p_))) {
      const int n = make(J_ASSIGN);
      attach(n, lhs);
      nodes[n].a = lhs;
      add_leaf(n, p_++);
      const int r = expr();
      attach(n, r);
      nodes[n].b = r;
      return n;
    }
    return lhs;
  }
  int ternary() {
    const int c = binary(1);
    if (c < 0 || !at("?")) return c;
    const int g = make(J_GENERIC);
    attach(g, c);
    add_leaf(g, p_++);
    attach(g, expr());
    if (at(":")) {
      add_leaf(g, p_++);
      attach(g, expr());
    }
    return g;
  }
  int binary(int minprec) {
    int lhs = unary();
    if (lhs < 0) return lhs;
    for (;;) {
      if (!more()) break;
      const std::string& op = t(p_);
      const int prec = binary_prec(op);
      if (prec < 0 || prec < minprec) break;
      const int g = make(J_GENERIC);
      attach(g, lhs);
      add_leaf(g, p_++);
      if (op == "instanceof") {
        if (at("final")) add_leaf(g, p_++);
        const size_t q = skip_type(p_);
        if (q) type_leaves(g, q);
        if (is_ident(t(p_)) && binary_prec(t(p_ + 1)) < 0 && !is_assign_op(t(p_ + 1)) &&
            t(p_ + 1) != "(" && t(p_ + 1) != ".")
          add_leaf(g, p_++);  // pattern binding
      } else {
        attach(g, binary(prec + 1));
      }
      lhs = g;
    }
    return lhs;
  }
  bool cast_ahead() const {
    if (!at("(")) return false;
    const size_t close = close_of(p_);
    size_t q = skip_type(p_ + 1);
    while (q && t(q) == "&") q = skip_type(q + 1);
    if (!q || q != close) return false;
    if (primitive_word(t(p_ + 1))) return true;
    const std::string& nx = t(close + 1);
    if (nx.empty()) return false;
    if (is_ident(nx) || is_literal(nx) || nx == "(" || nx == "!" || nx == "~" || nx == "this" ||
        nx == "super" || nx == "new" || primitive_word(nx))
      return true;
    return false;
  }
  int unary() {
    if (!more()) return -1;
    const std::string& s = t(p_);
    if (s == "+" || s == "-" || s == "!" || s == "~") {
      const int g = make(J_GENERIC);
      add_leaf(g, p_++);
      attach(g, unary());
      return g;
    }
    if (s == "++" || s == "--") {
      const int g = make(J_UPDATE);
      add_leaf(g, p_++);
      attach(g, unary());
      return g;
    }
    if (cast_ahead()) {
      const int g = make(J_GENERIC);
      const size_t close = close_of(p_);
      add_leaf(g, p_++);
      type_leaves(g, close);
      if (p_ == close) add_leaf(g, p_++);
      if (lambda_ahead()) attach(g, lambda());
      else attach(g, unary());
      return g;
    }
    return postfix(primary());
  }
  int arguments() {
    const int g = make(J_GENERIC);  // argument_list
    const size_t close = close_of(p_);
    add_leaf(g, p_++);
    limited(close, [&] {
      while (more()) {
        const size_t before = p_;
        attach(g, expr());
        if (at(",")) add_leaf(g, p_++);
        if (p_ == before) add_leaf(g, p_++);
      }
    });
    if (p_ == close && p_ < n_) add_leaf(g, p_++);
    return g;
  }
  int creation() {
    const int g = make(J_GENERIC);
    add_leaf(g, p_++);  // 'new'
    if (at("<")) {
      const size_t r = skip_type_args(p_);
      if (r) type_leaves(g, r);
    }
    while (at("@")) leaves_to(g, skip_annotation(p_));
    if (primitive_word(t(p_)) || is_ident(t(p_))) {
      nodes[add_leaf(g, p_++)].tid = true;
      for (;;) {
        if (at("<")) {
          const size_t r = skip_type_args(p_);
          if (r) {
            type_leaves(g, r);
            continue;
          }
          if (t(p_ + 1) == ">") {  // diamond
            add_leaf(g, p_++);
            add_leaf(g, p_++);
            continue;
          }
          break;
        }
        if (at(".") && is_ident(t(p_ + 1))) {
          add_leaf(g, p_++);
          nodes[add_leaf(g, p_++)].tid = true;
          continue;
        }
        break;
      }
    }
    if (at("(")) {
      attach(g, arguments());
      if (at("{")) class_body(g);
    } else {
      while (at("[")) {  // dimensions_expr / dimensions
        const size_t close = close_of(p_);
        add_leaf(g, p_++);
        limited(close, [&] {
          attach(g, expr());
          while (more()) add_leaf(g, p_++);
        });
        if (p_ == close && p_ < n_) add_leaf(g, p_++);
      }
      if (at("{")) attach(g, array_initializer());
    }
    return g;
  }
  int primary() {
    if (!more()) return -1;
    const std::string& s = t(p_);
    if (s == "(") {
      const int g = make(J_GENERIC);
      const size_t close = close_of(p_);
      add_leaf(g, p_++);
      limited(close, [&] {
        attach(g, expr());
        while (more()) add_leaf(g, p_++);
      });
      if (p_ == close && p_ < n_) add_leaf(g, p_++);
      return g;
    }
    if (s == "new") return creation();
    if (s == "switch") {
      const int g = make(J_GENERIC);
      switch_block(g);
      return g;
    }
    if (s == "{") return array_initializer();
    if (s == "@") {  // annotation in expression position: skip it
      const int g = make(J_GENERIC);
      leaves_to(g, std::max(skip_annotation(p_), p_ + 1));
      attach(g, primary());
      return g;
    }
    if (primitive_word(s)) {  // int.class, int[].class
      const int g = make(J_GENERIC);
      add_leaf(g, p_++);
      while (at("[") && t(p_ + 1) == "]") {
        add_leaf(g, p_++);
        add_leaf(g, p_++);
      }
      return g;
    }
    if (id_like(s) || is_literal(s)) {
      if ((is_ident(s) || s == "this" || s == "super") && t(p_ + 1) == "(") {
        const int g = make(J_INVOKE);  // method_invocation without object / ctor invocation
        add_leaf(g, p_++);
        const int args = arguments();
        attach(g, args);
        nodes[g].b = args;
        return g;
      }
      return leaf_node(p_++);
    }
    return -1;
  }
  int postfix(int node) {
    if (node < 0) return node;
    for (;;) {
      if (!more()) break;
      const std::string& s = t(p_);
      if (s == ".") {
        const std::string& nx = t(p_ + 1);
        if (nx == "<") {  // obj.<T>m(args)
          const size_t r = skip_type_args(p_ + 1);
          if (!r || !id_like(t(r)) || t(r + 1) != "(") break;
          const int g = make(J_INVOKE);
          attach(g, node);
          nodes[g].a = node;
          leaves_to(g, r + 1);
          const int args = arguments();
          attach(g, args);
          nodes[g].b = args;
          node = g;
          continue;
        }
        if (nx == "new") {
          const int g = make(J_GENERIC);
          attach(g, node);
          add_leaf(g, p_++);
          attach(g, creation());
          node = g;
          continue;
        }
        if (!id_like(nx)) break;
        if (t(p_ + 2) == "(" && nx != "class") {
          const int g = make(J_INVOKE);
          attach(g, node);
          nodes[g].a = node;
          add_leaf(g, p_++);
          add_leaf(g, p_++);
          const int args = arguments();
          attach(g, args);
          nodes[g].b = args;
          node = g;
          continue;
        }
        const int g = make(J_GENERIC);  // field_access / class literal / scoped name
        attach(g, node);
        add_leaf(g, p_++);
        add_leaf(g, p_++);
        node = g;
        continue;
      }
      if (s == "[") {
        const int g = make(J_GENERIC);
        attach(g, node);
        const size_t close = close_of(p_);
        add_leaf(g, p_++);
        limited(close, [&] {
          attach(g, expr());
          while (more()) add_leaf(g, p_++);
        });
        if (p_ == close && p_ < n_) add_leaf(g, p_++);
        node = g;
        continue;
      }
      if (s == "++" || s == "--") {
        const int g = make(J_UPDATE);
        attach(g, node);
        add_leaf(g, p_++);
        node = g;
        continue;
      }
      if (s == "::") {
        const int g = make(J_GENERIC);
        attach(g, node);
        add_leaf(g, p_++);
        if (more() && (id_like(t(p_)))) add_leaf(g, p_++);
        node = g;
        continue;
      }
      if (s == "<" ) {  // generic type in expression position: Foo<Bar>::new / .class
        const size_t r = skip_type_args(p_);
        if (r && (t(r) == "::" || (t(r) == "." && t(r + 1) == "class"))) {
          const int g = make(J_GENERIC);
          attach(g, node);
          leaves_to(g, r);
          node = g;
          continue;
        }
      }
      break;
    }
    return node;
  }
};

// ------------------------------------------------------------------------------ DFG_java walk
struct JWalker {
  const std::vector<JNode>& nd;
  const std::vector<Leaf>& lv;
  std::vector<char> anon;
  // GraphCodeBERT's parser/DFG.py DFG_java: every named leaf outside the states is an entry
  // (identifiers define themselves on first sight), and method_invocation has no special case
  bool ms = false;

  JWalker(const std::vector<JNode>& n, const std::vector<Leaf>& l, bool ms_variant)
      : nd(n), lv(l), ms(ms_variant) {
    anon.resize(l.size());
    // anonymous = node type == recorded code: a keyword / punctuation token whose byte-column
    // slice is intact
    for (size_t i = 0; i < l.size(); ++i) anon[i] = leaf_anon(l[i].raw) && l[i].text == l[i].raw;
  }

  void var_index(int x, std::vector<int>& out) const {  // tree_to_variable_index
    if (x < 0) return;
    if (nd[x].type == J_LEAF) {
      if (!anon[nd[x].leaf]) out.push_back(nd[x].leaf);
      return;
    }
    for (int k : nd[x].kids) var_index(k, out);
  }

  // name <- value entries (relation rel); the state of every name is its own idx
  void def_from(int name, int value, bool rel, std::vector<DfgEdge>& dfg, DfgStates& st) const {
    std::vector<int> ni, vi;
    var_index(name, ni);
    var_index(value, vi);
    for (int i1 : ni) {
      for (int i2 : vi) dfg.push_back({lv[i1].text, i1, rel, {lv[i2].text}, {i2}});
      st[lv[i1].text] = {i1};
    }
  }

  std::vector<DfgEdge> walk(int x, DfgStates& st) const {
    std::vector<DfgEdge> dfg;
    if (x < 0) return dfg;
    const JNode& n = nd[x];
    switch (n.type) {
      case J_LEAF: {
        const int idx = n.leaf;
        if (anon[idx]) return dfg;
        const std::string& code = lv[idx].text;
        auto it = st.find(code);
        if (it != st.end()) {
          dfg.push_back({code, idx, false, {code}, it->second});
        } else if (ms) {
          if (!n.tid && is_ident(lv[idx].raw)) st[code] = {idx};
          dfg.push_back({code, idx, false, {}, {}});
        } else if (n.pname) {
          st[code] = {idx};
          dfg.push_back({code, idx, false, {}, {}});
        }
        return dfg;
      }
      case J_DECLARATOR: {
        if (n.b < 0) {
          std::vector<int> ni;
          var_index(n.a, ni);
          for (int i : ni) {
            dfg.push_back({lv[i].text, i, false, {}, {}});
            st[lv[i].text] = {i};
          }
        } else {
          dfg_append(dfg, walk(n.b, st));
          def_from(n.a, n.b, false, dfg, st);
        }
        dfg_sort(dfg);
        return dfg;
      }
      case J_ASSIGN: {
        dfg_append(dfg, walk(n.b, st));
        def_from(n.a, n.b, true, dfg, st);
        dfg_sort(dfg);
        return dfg;
      }
      case J_UPDATE: {
        std::vector<int> idxs;
        var_index(x, idxs);
        for (int i1 : idxs) {
          for (int i2 : idxs) dfg.push_back({lv[i1].text, i1, true, {lv[i2].text}, {i2}});
          st[lv[i1].text] = {i1};
        }
        dfg_sort(dfg);
        return dfg;
      }
      case J_IF: {
        DfgStates current = st;
        std::vector<DfgStates> others;
        bool flag = false, tag = false;
        for (int k : n.kids) {
          const bool is_else = nd[k].type == J_LEAF && lv[nd[k].leaf].raw == "else";
          if (is_else) tag = true;
          if (!(is_else || nd[k].type == J_IF) && !flag) {
            dfg_append(dfg, walk(k, current));
          } else {
            flag = true;
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
      case J_FOR: {
        for (int k : n.kids) dfg_append(dfg, walk(k, st));
        bool flag = false;
        for (int k : n.kids) {
          if (flag) dfg_append(dfg, walk(k, st));
          else if (nd[k].type == J_LVD) flag = true;
        }
        dfg_merge_dup(dfg);
        return dfg;
      }
      case J_ENH_FOR: {
        for (int rep = 0; rep < 2; ++rep) {
          dfg_append(dfg, walk(n.b, st));
          def_from(n.a, n.b, true, dfg, st);
          dfg_append(dfg, walk(n.c, st));
        }
        dfg_merge_dup(dfg);
        return dfg;
      }
      case J_WHILE: {
        for (int rep = 0; rep < 2; ++rep)
          for (int k : n.kids) dfg_append(dfg, walk(k, st));
        dfg_merge_dup(dfg);
        return dfg;
      }
      case J_INVOKE:
        if (n.a >= 0 && !ms) {
          dfg_append(dfg, walk(n.a, st));
          dfg_append(dfg, walk(n.b, st));
          dfg_sort(dfg);
          return dfg;
        }
        [[fallthrough]];
      default:
        for (int k : n.kids) dfg_append(dfg, walk(k, st));
        dfg_sort(dfg);
        return dfg;
    }
  }
};

}  // namespace

std::vector<DfgEdge> dfg_java(const std::vector<Leaf>& leaves, bool ms) {
  JTree tree(leaves);
  const int root = tree.parse();
  JWalker w(tree.nodes, leaves, ms);
  DfgStates states;
  std::vector<DfgEdge> d = w.walk(root, states);
  dfg_sort(d);
  return d;
}

}  // namespace ah
