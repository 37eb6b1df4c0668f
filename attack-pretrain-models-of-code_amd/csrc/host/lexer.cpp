// lexer.cpp — tree-sitter-free leaf extraction.
//
// The reference obtains code tokens as the leaves of a tree-sitter parse
// (python_parser/parser_folder/utils.py:89-96 tree_to_token_index: every childless node, or a
// whole node of type 'string', except comments; text by utils.py:115-129 index_to_code_token).
// tree-sitter and its grammars are un-vendored and absent here, so this lexer DEFINES
// the leaf sequence with the rules below (mirrored exactly by oracle/featurize_ref.py); they follow
// the token rules of the tree-sitter-c / -java / -python grammars of the reference's era.
//
// C (tree-sitter-c 0.20.x):
//   * whitespace and backslash-newline are extras; // and /* */ comments are dropped (an
//     unterminated /* is not a comment: its characters lex as operators / identifiers);
//   * identifiers [A-Za-z_][A-Za-z0-9_]*; numbers (optional sign when an operand is expected,
//     0x/0b, digits, '.', exponent sign after e/E/p/P, suffix letters);
//   * string literal: opening quote (with L/u/U/u8 prefix) and closing quote are leaves, escape
//     sequences are leaves, plain content is a hidden token (no leaf); at an unescaped newline a
//     string literal closes if the next non-blank character is its quote (the closing quote may
//     follow whitespace), else it ends unterminated at the line break;  char literal: ends at
//     the line break;
//   * operators: longest match over the C punctuators;
//   * preprocessor line (# first on its line): directive leaf "#<ws>name"; #include <..> is one
//     leaf; #define NAME [ (params) ] then the rest of the line (with \-continuations, up to a
//     comment start) is one preproc_arg leaf; #if/#elif/#ifdef/#ifndef conditions are lexed as
//     code; unknown directives take the rest of the line as one preproc_arg leaf;
//   * any other code point is a one-character leaf.
// Java: as C without the preprocessor; string and char literals are single leaves (one token in
//   tree-sitter-java 0.19), text blocks likewise; '@' annotations are leaves.
// Python: strings (any prefix, ''' / """ included) are single leaves (node type 'string' is taken
//   whole); '#' comments dropped; NEWLINE/INDENT/DEDENT produce no leaf.
#include <cstring>

#include "host.h"

namespace ah {
namespace {

bool is_id_start(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; }
bool is_id_char(unsigned char c) { return is_id_start(c) || (c >= '0' && c <= '9'); }
bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

const char* kCOps[] = {"...", ">>=", "<<=", "->", "++", "--", "<<", ">>", "<=", ">=", "==", "!=",
                       "&&", "||", "+=", "-=", "*=", "/=", "%=", "&=", "^=", "|=", nullptr};
const char* kJavaOps[] = {">>>=", "<<=", ">>=", ">>>", "...", "->", "::", "++", "--", "<<", ">>",
                          "<=", ">=", "==", "!=", "&&", "||", "+=", "-=", "*=", "/=", "%=", "&=",
                          "^=", "|=", nullptr};
const char* kPyOps[] = {"**=", "//=", ">>=", "<<=", "...", "->", ":=", "**", "//", "<<", ">>", "<=",
                        ">=", "==", "!=", "<>", "+=", "-=", "*=", "/=", "%=", "&=", "^=", "|=",
                        "@=", nullptr};

struct Cursor {
  const std::string& s;
  size_t i = 0;
  int line = 0;
  size_t line_start = 0;
  explicit Cursor(const std::string& str) : s(str) {}
  bool eof() const { return i >= s.size(); }
  unsigned char at(size_t k = 0) const { return i + k < s.size() ? (unsigned char)s[i + k] : 0; }
  int col() const { return (int)(i - line_start); }
  void adv() {
    if (s[i] == '\n') {
      ++line;
      line_start = i + 1;
    }
    ++i;
  }
  void adv(size_t n) {
    for (size_t k = 0; k < n && !eof(); ++k) adv();
  }
};

class Lexer {
 public:
  Lexer(const std::string& code, Lang lang) : c_(code), lang_(lang), lines_(split_lines(code)) {
    for (auto& l : lines_) lines_cp_.push_back(utf8_decode(l));
  }

  std::vector<Leaf> run() {
    bool line_has_token = false;  // for '#' at line start
    int cur_line = 0;
    while (!c_.eof()) {
      if (c_.line != cur_line) {
        cur_line = c_.line;
        line_has_token = false;
      }
      const unsigned char ch = c_.at();
      // extras
      if (ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n' || ch == '\v' || ch == '\f') {
        c_.adv();
        continue;
      }
      if (ch == '\\' && lang_ != LANG_PYTHON && (c_.at(1) == '\n' || (c_.at(1) == '\r' && c_.at(2) == '\n'))) {
        c_.adv(c_.at(1) == '\n' ? 2 : 3);
        continue;
      }
      if (lang_ == LANG_PYTHON && ch == '\\' && (c_.at(1) == '\n' || (c_.at(1) == '\r' && c_.at(2) == '\n'))) {
        c_.adv(c_.at(1) == '\n' ? 2 : 3);
        joined_ = true;
        continue;
      }
      // comments
      if (lang_ != LANG_PYTHON && ch == '/' && c_.at(1) == '/') {
        skip_line_comment();
        continue;
      }
      if (lang_ != LANG_PYTHON && ch == '/' && c_.at(1) == '*' && block_comment_closes()) {
        skip_block_comment();
        continue;
      }
      if (lang_ == LANG_PYTHON && ch == '#') {
        while (!c_.eof() && c_.at() != '\n') c_.adv();
        continue;
      }
      if (lang_ == LANG_C && ch == '#' && !line_has_token) {
        preprocessor();
        line_has_token = true;
        continue;
      }
      line_has_token = true;
      token();
    }
    return std::move(out_);
  }

 private:
  void emit(size_t b, int sl, int sc) {
    Leaf lf;
    lf.sl = sl;
    lf.sc = sc;
    lf.el = c_.line;
    lf.ec = c_.col();
    // index_to_code_token (utils.py:115-129): same line -> slice; else concatenation of the
    // start line tail, the middle lines and the end line head (line breaks dropped).  The
    // reference slices Python str lines with tree-sitter's BYTE columns, so on a line holding
    // non-ASCII code points the text is taken at code-point indices equal to the byte columns.
    lf.raw = c_.s.substr(b, c_.i - b);
    lf.joined = joined_;
    joined_ = false;
    if (lf.sl == lf.el) {
      lf.text = utf8_encode(lines_cp_[lf.sl], lf.sc, lf.ec);
    } else {
      lf.text = utf8_encode(lines_cp_[lf.sl], lf.sc, lines_cp_[lf.sl].size());
      for (int k = lf.sl + 1; k < lf.el; ++k) lf.text += lines_[k];
      lf.text += utf8_encode(lines_cp_[lf.el], 0, lf.ec);
    }
    last_kind_ = kind_;
    out_.push_back(std::move(lf));
  }

  void skip_line_comment() {
    while (!c_.eof() && c_.at() != '\n') {
      if (c_.at() == '\\' && c_.at(1) == '\n') c_.adv(2);
      else if (c_.at() == '\\' && c_.at(1) == '\r' && c_.at(2) == '\n') c_.adv(3);
      else c_.adv();
    }
  }
  // an unterminated /* is not a comment token: '/' and '*' lex as operators (tree-sitter-c's
  // comment regex needs the closing */)
  bool block_comment_closes() const { return c_.s.find("*/", c_.i + 2) != std::string::npos; }
  void skip_block_comment() {
    c_.adv(2);
    while (!c_.eof() && !(c_.at() == '*' && c_.at(1) == '/')) c_.adv();
    if (!c_.eof()) c_.adv(2);
  }

  // operand-ending previous leaf => a following +/- is a binary operator, not a number sign
  bool expect_operand() const { return last_kind_ != K_OPERAND; }

  void token() {
    const size_t b = c_.i;
    const int sl = c_.line, sc = c_.col();
    const unsigned char ch = c_.at();
    // string / char literals (with prefixes)
    if (lang_ == LANG_C) {
      size_t pre = 0;
      if (ch == 'L' || ch == 'U') pre = 1;
      else if (ch == 'u') pre = (c_.at(1) == '8') ? 2 : 1;
      if (pre && (c_.at(pre) == '"' || c_.at(pre) == '\'')) {
        c_literal(pre);
        return;
      }
      if (ch == '"' || ch == '\'') {
        c_literal(0);
        return;
      }
    } else if (lang_ == LANG_JAVA) {
      if (ch == '"' || ch == '\'') {
        java_literal();
        return;
      }
    } else {
      if (py_string_start()) return;
    }
    if (is_id_start(ch)) {
      while (!c_.eof() && is_id_char(c_.at())) c_.adv();
      kind_ = K_OPERAND;
      emit(b, sl, sc);
      return;
    }
    // numbers (optional sign when an operand is expected — tree-sitter-c number_literal)
    const bool sign = (ch == '-' || ch == '+') && lang_ == LANG_C && expect_operand() &&
                      (is_digit(c_.at(1)) || (c_.at(1) == '.' && is_digit(c_.at(2))));
    if (is_digit(ch) || (ch == '.' && is_digit(c_.at(1))) || sign) {
      if (sign) c_.adv();
      number();
      kind_ = K_OPERAND;
      emit(b, sl, sc);
      return;
    }
    // operators
    const char* const* ops = lang_ == LANG_C ? kCOps : lang_ == LANG_JAVA ? kJavaOps : kPyOps;
    for (const char* const* op = ops; *op; ++op) {
      const size_t n = std::strlen(*op);
      if (c_.s.compare(c_.i, n, *op) == 0) {
        c_.adv(n);
        kind_ = (!std::strcmp(*op, "++") || !std::strcmp(*op, "--")) ? K_OPERAND : K_OP;
        emit(b, sl, sc);
        return;
      }
    }
    // single code point
    size_t k = c_.i;
    utf8_next(c_.s, k);
    c_.adv(k - c_.i);
    kind_ = (ch == ')' || ch == ']') ? K_OPERAND : K_OP;
    emit(b, sl, sc);
  }

  void number() {
    // 0x / 0b prefix, digits/letters/dots, exponent signs
    while (!c_.eof()) {
      const unsigned char d = c_.at();
      if (is_id_char(d) || d == '.' || d == '\'') {
        const bool exp = (d == 'e' || d == 'E' || d == 'p' || d == 'P');
        const bool hex = c_.i >= 2 && (c_.s[c_.i - 1] == 'x' || c_.s[c_.i - 1] == 'X');
        (void)hex;
        c_.adv();
        if (exp && (c_.at() == '+' || c_.at() == '-') && is_digit(c_.at(1))) c_.adv();
        continue;
      }
      break;
    }
  }

  // C string / char literal: quote leaves, escape leaves, hidden content.
  void c_literal(size_t pre) {
    const unsigned char q = c_.at(pre);
    {
      const size_t b = c_.i;
      const int sl = c_.line, sc = c_.col();
      c_.adv(pre + 1);
      kind_ = K_OP;
      emit(b, sl, sc);
    }
    while (!c_.eof()) {
      const unsigned char d = c_.at();
      if (d == '\n') {
        // a raw newline inside the literal: tree-sitter-c's content token is immediate and
        // excludes '\n', but the closing quote is not immediate, so whitespace (the newline and
        // the next line's indentation) may precede it — if the next non-blank character is the
        // closing quote the literal closes there; otherwise it is unterminated and ends here
        size_t k = c_.i;
        while (k < c_.s.size() && (c_.s[k] == '\n' || c_.s[k] == ' ' || c_.s[k] == '\t' ||
                                   c_.s[k] == '\r'))
          ++k;
        if (q != '"' || k >= c_.s.size() || (unsigned char)c_.s[k] != q) return;
        while (c_.i < k) c_.adv();
        continue;
      }
      if (d == q) {
        const size_t b = c_.i;
        const int sl = c_.line, sc = c_.col();
        c_.adv();
        kind_ = K_OPERAND;
        emit(b, sl, sc);
        return;
      }
      if (d == '\\') {
        const size_t b = c_.i;
        const int sl = c_.line, sc = c_.col();
        escape();
        kind_ = K_OP;
        emit(b, sl, sc);
        continue;
      }
      size_t k = c_.i;
      utf8_next(c_.s, k);
      c_.adv(k - c_.i);  // hidden content
    }
  }

  // escape_sequence: \ followed by octal{1,3} | x hex+ | u hex{4} | U hex{8} | any one char
  // (a backslash-newline inside a literal is a line continuation escape)
  void escape() {
    c_.adv();  // backslash
    if (c_.eof()) return;
    const unsigned char d = c_.at();
    auto hexc = [](unsigned char x) {
      return (x >= '0' && x <= '9') || (x >= 'a' && x <= 'f') || (x >= 'A' && x <= 'F');
    };
    if (d >= '0' && d <= '7') {
      for (int k = 0; k < 3 && c_.at() >= '0' && c_.at() <= '7'; ++k) c_.adv();
    } else if (d == 'x') {
      c_.adv();
      while (hexc(c_.at())) c_.adv();
    } else if (d == 'u' || d == 'U') {
      const int n = d == 'u' ? 4 : 8;
      c_.adv();
      for (int k = 0; k < n && hexc(c_.at()); ++k) c_.adv();
    } else if (d == '\r' && c_.at(1) == '\n') {
      c_.adv(2);
    } else {
      size_t k = c_.i;
      utf8_next(c_.s, k);
      c_.adv(k - c_.i);
    }
  }

  void java_literal() {
    const size_t b = c_.i;
    const int sl = c_.line, sc = c_.col();
    const unsigned char q = c_.at();
    if (q == '"' && c_.at(1) == '"' && c_.at(2) == '"') {  // text block
      c_.adv(3);
      while (!c_.eof() && !(c_.at() == '"' && c_.at(1) == '"' && c_.at(2) == '"')) {
        if (c_.at() == '\\') c_.adv();
        c_.adv();
      }
      c_.adv(3);
    } else {
      // one regex token that cannot hold a raw newline: an unterminated literal is a lexing
      // error, tree-sitter skips the opening quote alone and lexes what follows as code
      c_.adv();
      const size_t qi = c_.i, qls = c_.line_start;
      const int ql = c_.line;
      while (!c_.eof() && c_.at() != q && c_.at() != '\n') {
        if (c_.at() == '\\') c_.adv();
        c_.adv();
      }
      if (c_.at() == q) {
        c_.adv();
      } else {
        c_.i = qi;
        c_.line = ql;
        c_.line_start = qls;
      }
    }
    kind_ = K_OPERAND;
    emit(b, sl, sc);
  }

  bool py_string_start() {
    size_t p = 0;
    while (p < 3) {
      const unsigned char d = c_.at(p);
      if (d == 'r' || d == 'R' || d == 'b' || d == 'B' || d == 'u' || d == 'U' || d == 'f' ||
          d == 'F')
        ++p;
      else
        break;
    }
    const unsigned char q = c_.at(p);
    if (q != '"' && q != '\'') return false;
    if (p > 0 && (c_.i > 0 && is_id_char((unsigned char)c_.s[c_.i - 1]))) return false;
    const size_t b = c_.i;
    const int sl = c_.line, sc = c_.col();
    c_.adv(p);
    const bool triple = c_.at(1) == q && c_.at(2) == q;
    if (triple) {
      c_.adv(3);
      while (!c_.eof() && !(c_.at() == q && c_.at(1) == q && c_.at(2) == q)) {
        if (c_.at() == '\\') c_.adv();
        c_.adv();
      }
      c_.adv(3);
    } else {
      // tree-sitter-python's external scanner: string content may begin with a raw newline
      // (then it runs on to the next quote), but a newline after content is an error — the
      // string is then only its opening quote, and what follows lexes as code
      bool raw = false;
      for (size_t k = 0; k < p; ++k) raw |= (c_.s[b + k] == 'r' || c_.s[b + k] == 'R');
      c_.adv();
      const size_t qi = c_.i;
      const int ql = c_.line;
      const size_t qls = c_.line_start;
      bool has_content = false, broken = false;
      while (!c_.eof()) {
        const unsigned char d = c_.at();
        if (d == '\\') {
          if (raw) {
            c_.adv();
            if (c_.at() == q || c_.at() == '\\') c_.adv();
          } else {
            c_.adv(py_escape_len());
            has_content = false;  // the scanner resumes after an escape token
          }
          continue;
        }
        if (d == q) {
          c_.adv();
          break;
        }
        if (d == '\n' && has_content) {
          broken = true;
          break;
        }
        c_.adv();
        has_content = true;
      }
      if (broken) {
        c_.i = qi;
        c_.line = ql;
        c_.line_start = qls;
      }
    }
    kind_ = K_OPERAND;
    emit(b, sl, sc);
    return true;
  }

  // length of the escape token at a backslash in a non-raw Python string (1: a lone '\\')
  size_t py_escape_len() const {
    auto hex = [&](size_t k) {
      const unsigned char d = c_.at(k);
      return (d >= '0' && d <= '9') || (d >= 'a' && d <= 'f') || (d >= 'A' && d <= 'F');
    };
    const unsigned char d = c_.at(1);
    auto hexrun = [&](size_t n) {
      for (size_t k = 0; k < n; ++k)
        if (!hex(2 + k)) return false;
      return true;
    };
    if (d == 'u') return hexrun(4) ? 6 : 1;
    if (d == 'U') return hexrun(8) ? 10 : 1;
    if (d == 'x') return hexrun(2) ? 4 : 1;
    if (is_digit(d)) return (is_digit(c_.at(2)) && is_digit(c_.at(3))) ? 4 : 1;
    if (d == '\n') return 2;
    if (d == '\r') return c_.at(2) == '\n' ? 3 : 1;
    if (d && std::strchr("'\"abfrntv\\", d)) return 2;
    return 1;
  }

  void preprocessor() {
    // directive leaf: '#' [ \t]* name
    const size_t b = c_.i;
    const int sl = c_.line, sc = c_.col();
    c_.adv();
    while (c_.at() == ' ' || c_.at() == '\t') c_.adv();
    const size_t nb = c_.i;
    while (!c_.eof() && is_id_char(c_.at())) c_.adv();
    const std::string name = c_.s.substr(nb, c_.i - nb);
    kind_ = K_OP;
    emit(b, sl, sc);
    const int dline = c_.line;
    auto skip_ws = [&]() {
      while (c_.at() == ' ' || c_.at() == '\t') c_.adv();
    };
    if (name == "include") {
      skip_ws();
      if (c_.at() == '<') {
        const size_t b2 = c_.i;
        const int sl2 = c_.line, sc2 = c_.col();
        while (!c_.eof() && c_.at() != '>' && c_.at() != '\n') c_.adv();
        if (c_.at() == '>') c_.adv();
        kind_ = K_OPERAND;
        emit(b2, sl2, sc2);
      }
      lex_rest_of_line(dline);
      return;
    }
    if (name == "define") {
      skip_ws();
      if (is_id_start(c_.at())) {
        const size_t b2 = c_.i;
        const int sl2 = c_.line, sc2 = c_.col();
        while (is_id_char(c_.at())) c_.adv();
        kind_ = K_OPERAND;
        emit(b2, sl2, sc2);
        if (c_.at() == '(') {
          while (!c_.eof() && c_.at() != '\n') {
            skip_ws();
            const size_t b3 = c_.i;
            const int sl3 = c_.line, sc3 = c_.col();
            if (c_.at() == ')') {
              c_.adv();
              kind_ = K_OPERAND;
              emit(b3, sl3, sc3);
              break;
            }
            if (is_id_start(c_.at())) {
              while (is_id_char(c_.at())) c_.adv();
            } else if (c_.s.compare(c_.i, 3, "...") == 0) {
              c_.adv(3);
            } else {
              size_t k = c_.i;
              utf8_next(c_.s, k);
              c_.adv(k - c_.i);
            }
            kind_ = K_OP;
            emit(b3, sl3, sc3);
          }
        }
        preproc_arg();
      }
      return;
    }
    if (name == "if" || name == "elif" || name == "ifdef" || name == "ifndef" || name == "else" ||
        name == "endif") {
      lex_rest_of_line(dline);
      return;
    }
    preproc_arg();
  }

  // rest of the line (with \-continuations, stopping before "/*") as one leaf
  void preproc_arg() {
    while (c_.at() == ' ' || c_.at() == '\t') c_.adv();
    if (c_.eof() || c_.at() == '\n' || (c_.at() == '\r' && c_.at(1) == '\n')) return;
    if (c_.at() == '/' && (c_.at(1) == '*' || c_.at(1) == '/')) return;
    const size_t b = c_.i;
    const int sl = c_.line, sc = c_.col();
    while (!c_.eof()) {
      const unsigned char d = c_.at();
      if (d == '\n') break;
      if (d == '\\' && c_.at(1) == '\n') { c_.adv(2); continue; }
      if (d == '\\' && c_.at(1) == '\r' && c_.at(2) == '\n') { c_.adv(3); continue; }
      if (d == '/' && c_.at(1) == '*') break;
      c_.adv();
    }
    kind_ = K_OP;
    emit(b, sl, sc);
  }

  // lex ordinary tokens until the end of the directive's (continued) line
  void lex_rest_of_line(int dline) {
    (void)dline;
    while (!c_.eof()) {
      const unsigned char ch = c_.at();
      if (ch == '\n') return;
      if (ch == ' ' || ch == '\t' || ch == '\r' || ch == '\v' || ch == '\f') { c_.adv(); continue; }
      if (ch == '\\' && c_.at(1) == '\n') { c_.adv(2); continue; }
      if (ch == '\\' && c_.at(1) == '\r' && c_.at(2) == '\n') { c_.adv(3); continue; }
      if (ch == '/' && c_.at(1) == '/') { skip_line_comment(); continue; }
      if (ch == '/' && c_.at(1) == '*' && block_comment_closes()) { skip_block_comment(); continue; }
      token();
    }
  }

  enum Kind { K_OP = 0, K_OPERAND = 1 };
  Cursor c_;
  Lang lang_;
  std::vector<std::string> lines_;
  std::vector<std::vector<uint32_t>> lines_cp_;
  std::vector<Leaf> out_;
  int kind_ = K_OP, last_kind_ = K_OP;
  bool joined_ = false;
};

}  // namespace

std::vector<std::string> split_lines(const std::string& code) {
  std::vector<std::string> lines;
  size_t b = 0;
  for (size_t i = 0; i <= code.size(); ++i) {
    if (i == code.size() || code[i] == '\n') {
      lines.push_back(code.substr(b, i - b));
      b = i + 1;
    }
  }
  return lines;
}

std::string join_lines(const std::vector<std::string>& lines) {
  std::string out;
  for (size_t k = 0; k < lines.size(); ++k) {
    if (k) out.push_back('\n');
    out += lines[k];
  }
  return out;
}

std::vector<Leaf> lex(const std::string& code, Lang lang) { return Lexer(code, lang).run(); }

}  // namespace ah
