"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

Pure-Python restatement of the host featurisation the reference performs per mutant:
  * leaf extraction with the lexing rules documented in csrc/host/lexer.cpp (the reference uses
    tree-sitter leaves, python_parser/parser_folder/utils.py:89-129; tree-sitter is absent here, so
    these rules are the definition — parity with tree-sitter itself is UNPINNED);
  * get_example / get_example_batch restated line for line from python_parser/run_parser.py:218-266;
  * convert_code_to_features from CodeXGLUE/Defect-detection/code/attacker.py:38-45 with the
    installed transformers RobertaTokenizer (tokenizers-backed) on data/tokenizer.

This is an independent implementation (byte scanner in Python) of the same rules as the C++
library; tests/test_host.py requires the two to agree exactly.
"""
from __future__ import annotations

import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]

C_OPS = ["...", ">>=", "<<=", "->", "++", "--", "<<", ">>", "<=", ">=", "==", "!=", "&&", "||",
         "+=", "-=", "*=", "/=", "%=", "&=", "^=", "|="]
JAVA_OPS = [">>>=", "<<=", ">>=", ">>>", "...", "->", "::", "++", "--", "<<", ">>", "<=", ">=",
            "==", "!=", "&&", "||", "+=", "-=", "*=", "/=", "%=", "&=", "^=", "|="]
PY_OPS = ["**=", "//=", ">>=", "<<=", "...", "->", ":=", "**", "//", "<<", ">>", "<=", ">=", "==",
          "!=", "<>", "+=", "-=", "*=", "/=", "%=", "&=", "^=", "|=", "@="]


def _idstart(c):
    return c.isascii() and (c.isalpha() or c == "_")


def _idchar(c):
    return c.isascii() and (c.isalnum() or c == "_")


def _digit(c):
    return c.isascii() and c.isdigit()


class _Lex:
    """Scanner over the UTF-8 bytes (columns are byte offsets, like tree-sitter points)."""

    def __init__(self, code: str, lang: str):
        self.b = code.encode("utf-8")
        self.s = [chr(x) for x in self.b]  # byte-wise characters for scanning
        self.lang = lang
        self.lines = code.split("\n")
        self.i = 0
        self.line = 0
        self.line_start = 0
        self.out = []
        self.kind = 0
        self.last_kind = 0

    def at(self, k=0):
        j = self.i + k
        return self.s[j] if j < len(self.s) else "\0"

    def eof(self):
        return self.i >= len(self.s)

    def adv(self, n=1):
        for _ in range(n):
            if self.eof():
                return
            if self.s[self.i] == "\n":
                self.line += 1
                self.line_start = self.i + 1
            self.i += 1

    def col(self):
        return self.i - self.line_start

    def emit(self, b, sl, sc):
        el, ec = self.line, self.col()
        # index_to_code_token (utils.py:115-129) slices the str lines with tree-sitter's BYTE
        # columns (the reference's behaviour on non-ASCII lines, reproduced on purpose)
        if sl == el:
            text = self.lines[sl][sc:ec]
        else:
            text = self.lines[sl][sc:]
            for k in range(sl + 1, el):
                text += self.lines[k]
            text += self.lines[el][:ec]
        self.last_kind = self.kind
        self.out.append((sl, sc, el, ec, text))

    def cp_len(self):
        c = ord(self.at())
        return 1 if c < 0x80 else 2 if c >> 5 == 6 else 3 if c >> 4 == 14 else 4 if c >> 3 == 30 else 1

    def nl_cont(self):
        if self.at() == "\\" and self.at(1) == "\n":
            return 2
        if self.at() == "\\" and self.at(1) == "\r" and self.at(2) == "\n":
            return 3
        return 0

    def skip_line_comment(self):
        while not self.eof() and self.at() != "\n":
            k = self.nl_cont()
            self.adv(k if k else 1)

    def closes(self):
        return self.b.find(b"*/", self.i + 2) >= 0

    def skip_block_comment(self):
        self.adv(2)
        while not self.eof() and not (self.at() == "*" and self.at(1) == "/"):
            self.adv()
        if not self.eof():
            self.adv(2)

    def run(self):
        line_has_token, cur_line = False, 0
        while not self.eof():
            if self.line != cur_line:
                cur_line, line_has_token = self.line, False
            ch = self.at()
            if ch in " \t\r\n\v\f":
                self.adv()
                continue
            k = self.nl_cont()
            if k:
                self.adv(k)
                continue
            if self.lang != "python" and ch == "/" and self.at(1) == "/":
                self.skip_line_comment()
                continue
            if self.lang != "python" and ch == "/" and self.at(1) == "*" and self.closes():
                self.skip_block_comment()
                continue
            if self.lang == "python" and ch == "#":
                while not self.eof() and self.at() != "\n":
                    self.adv()
                continue
            if self.lang == "c" and ch == "#" and not line_has_token:
                self.preprocessor()
                line_has_token = True
                continue
            line_has_token = True
            self.token()
        return self.out

    def token(self):
        b, sl, sc = self.i, self.line, self.col()
        ch = self.at()
        if self.lang == "c":
            pre = 0
            if ch in "LU":
                pre = 1
            elif ch == "u":
                pre = 2 if self.at(1) == "8" else 1
            if pre and self.at(pre) in "\"'":
                self.c_literal(pre)
                return
            if ch in "\"'":
                self.c_literal(0)
                return
        elif self.lang == "java":
            if ch in "\"'":
                self.java_literal()
                return
        else:
            if self.py_string():
                return
        if _idstart(ch):
            while not self.eof() and _idchar(self.at()):
                self.adv()
            self.kind = 1
            self.emit(b, sl, sc)
            return
        sign = (ch in "-+" and self.lang == "c" and self.last_kind != 1 and
                (_digit(self.at(1)) or (self.at(1) == "." and _digit(self.at(2)))))
        if _digit(ch) or (ch == "." and _digit(self.at(1))) or sign:
            if sign:
                self.adv()
            while not self.eof():
                d = self.at()
                if _idchar(d) or d in ".'":
                    self.adv()
                    if d in "eEpP" and self.at() in "+-" and _digit(self.at(1)):
                        self.adv()
                    continue
                break
            self.kind = 1
            self.emit(b, sl, sc)
            return
        ops = C_OPS if self.lang == "c" else JAVA_OPS if self.lang == "java" else PY_OPS
        for op in ops:
            if "".join(self.s[self.i:self.i + len(op)]) == op:
                self.adv(len(op))
                self.kind = 1 if op in ("++", "--") else 0
                self.emit(b, sl, sc)
                return
        self.adv(self.cp_len())
        self.kind = 1 if ch in ")]" else 0
        self.emit(b, sl, sc)

    def escape(self):
        self.adv()  # backslash
        if self.eof():
            return
        d = self.at()
        hexc = lambda x: x in "0123456789abcdefABCDEF"  # noqa: E731
        if "0" <= d <= "7":
            for _ in range(3):
                if "0" <= self.at() <= "7":
                    self.adv()
                else:
                    break
        elif d == "x":
            self.adv()
            while hexc(self.at()):
                self.adv()
        elif d in "uU":
            n = 4 if d == "u" else 8
            self.adv()
            for _ in range(n):
                if hexc(self.at()):
                    self.adv()
                else:
                    break
        elif d == "\r" and self.at(1) == "\n":
            self.adv(2)
        else:
            self.adv(self.cp_len())

    def c_literal(self, pre):
        q = self.at(pre)
        b, sl, sc = self.i, self.line, self.col()
        self.adv(pre + 1)
        self.kind = 0
        self.emit(b, sl, sc)
        while not self.eof():
            d = self.at()
            if d == "\n":
                # the closing quote (not an immediate token) may follow blanks and newlines
                k = self.i
                while k < len(self.s) and self.s[k] in "\n \t\r":
                    k += 1
                if q != '"' or k >= len(self.s) or self.s[k] != q:
                    return
                while self.i < k:
                    self.adv()
                continue
            if d == q:
                b, sl, sc = self.i, self.line, self.col()
                self.adv()
                self.kind = 1
                self.emit(b, sl, sc)
                return
            if d == "\\":
                b, sl, sc = self.i, self.line, self.col()
                self.escape()
                self.kind = 0
                self.emit(b, sl, sc)
                continue
            self.adv(self.cp_len())

    def java_literal(self):
        b, sl, sc = self.i, self.line, self.col()
        q = self.at()
        if q == '"' and self.at(1) == '"' and self.at(2) == '"':
            self.adv(3)
            while not self.eof() and not (self.at() == '"' and self.at(1) == '"' and self.at(2) == '"'):
                if self.at() == "\\":
                    self.adv()
                self.adv()
            self.adv(3)
        else:
            # an unterminated literal (raw newline) is a lexing error: only the quote is skipped
            self.adv()
            saved = (self.i, self.line, self.line_start)
            while not self.eof() and self.at() != q and self.at() != "\n":
                if self.at() == "\\":
                    self.adv()
                self.adv()
            if self.at() == q:
                self.adv()
            else:
                self.i, self.line, self.line_start = saved
        self.kind = 1
        self.emit(b, sl, sc)

    def py_string(self):
        p = 0
        while p < 3 and self.at(p) in "rRbBuUfF":
            p += 1
        q = self.at(p)
        if q not in "\"'":
            return False
        if p > 0 and self.i > 0 and _idchar(self.s[self.i - 1]):
            return False
        b, sl, sc = self.i, self.line, self.col()
        self.adv(p)
        if self.at(1) == q and self.at(2) == q:
            self.adv(3)
            while not self.eof() and not (self.at() == q and self.at(1) == q and self.at(2) == q):
                if self.at() == "\\":
                    self.adv()
                self.adv()
            self.adv(3)
        else:
            # content may begin with a raw newline; a newline after content breaks the string
            # (it is then only its opening quote)
            raw = any(ch in "rR" for ch in self.s[b:b + p])
            self.adv()
            saved = (self.i, self.line, self.line_start)
            has_content = broken = False
            while not self.eof():
                d = self.at()
                if d == "\\":
                    if raw:
                        self.adv()
                        if self.at() in (q, "\\"):
                            self.adv()
                    else:
                        self.adv(self._py_escape_len())
                        has_content = False
                    continue
                if d == q:
                    self.adv()
                    break
                if d == "\n" and has_content:
                    broken = True
                    break
                self.adv()
                has_content = True
            if broken:
                self.i, self.line, self.line_start = saved
        self.kind = 1
        self.emit(b, sl, sc)
        return True

    def _py_escape_len(self):
        """tree-sitter-python escape_sequence length at a backslash (1: a lone backslash)."""
        hexd = "0123456789abcdefABCDEF"
        d = self.at(1)

        def run(n):
            return all(self.at(2 + k) in hexd for k in range(n))

        if d == "u":
            return 6 if run(4) else 1
        if d == "U":
            return 10 if run(8) else 1
        if d == "x":
            return 4 if run(2) else 1
        dig = "0123456789"
        if d in dig:
            return 4 if (self.at(2) in dig and self.at(3) in dig) else 1
        if d == "\n":
            return 2
        if d == "\r":
            return 3 if self.at(2) == "\n" else 1
        if d in "'\"abfrntv\\":
            return 2
        return 1

    def preprocessor(self):
        b, sl, sc = self.i, self.line, self.col()
        self.adv()
        while self.at() in " \t":
            self.adv()
        nb = self.i
        while not self.eof() and _idchar(self.at()):
            self.adv()
        name = "".join(self.s[nb:self.i])
        self.kind = 0
        self.emit(b, sl, sc)
        if name == "include":
            while self.at() in " \t":
                self.adv()
            if self.at() == "<":
                b2, sl2, sc2 = self.i, self.line, self.col()
                while not self.eof() and self.at() not in ">\n":
                    self.adv()
                if self.at() == ">":
                    self.adv()
                self.kind = 1
                self.emit(b2, sl2, sc2)
            self.rest_of_line()
            return
        if name == "define":
            while self.at() in " \t":
                self.adv()
            if _idstart(self.at()):
                b2, sl2, sc2 = self.i, self.line, self.col()
                while _idchar(self.at()):
                    self.adv()
                self.kind = 1
                self.emit(b2, sl2, sc2)
                if self.at() == "(":
                    while not self.eof() and self.at() != "\n":
                        while self.at() in " \t":
                            self.adv()
                        b3, sl3, sc3 = self.i, self.line, self.col()
                        if self.at() == ")":
                            self.adv()
                            self.kind = 1
                            self.emit(b3, sl3, sc3)
                            break
                        if _idstart(self.at()):
                            while _idchar(self.at()):
                                self.adv()
                        elif "".join(self.s[self.i:self.i + 3]) == "...":
                            self.adv(3)
                        else:
                            self.adv(self.cp_len())
                        self.kind = 0
                        self.emit(b3, sl3, sc3)
                self.preproc_arg()
            return
        if name in ("if", "elif", "ifdef", "ifndef", "else", "endif"):
            self.rest_of_line()
            return
        self.preproc_arg()

    def preproc_arg(self):
        while self.at() in " \t":
            self.adv()
        if self.eof() or self.at() == "\n" or (self.at() == "\r" and self.at(1) == "\n"):
            return
        if self.at() == "/" and self.at(1) in "*/":
            return
        b, sl, sc = self.i, self.line, self.col()
        while not self.eof():
            d = self.at()
            if d == "\n":
                break
            k = self.nl_cont()
            if k:
                self.adv(k)
                continue
            if d == "/" and self.at(1) == "*":
                break
            self.adv()
        self.kind = 0
        self.emit(b, sl, sc)

    def rest_of_line(self):
        while not self.eof():
            ch = self.at()
            if ch == "\n":
                return
            if ch in " \t\r\v\f":
                self.adv()
                continue
            k = self.nl_cont()
            if k:
                self.adv(k)
                continue
            if ch == "/" and self.at(1) == "/":
                self.skip_line_comment()
                continue
            if ch == "/" and self.at(1) == "*" and self.closes():
                self.skip_block_comment()
                continue
            self.token()


def leaves(code: str, lang: str = "c"):
    """[(start_line, start_byte_col, end_line, end_byte_col, text)]"""
    return _Lex(code, lang).run()


def code_tokens(code: str, lang: str = "c"):
    return [t[4] for t in leaves(code, lang)]


def remove_comments_and_docstrings(source, lang="c"):
    """python_parser/parser_folder/utils.py:73-87 (the non-Python branch), restated."""
    import re

    def replacer(match):
        s = match.group(0)
        return " " if s.startswith("/") else s

    pattern = re.compile(r'//.*?$|/\*.*?\*/|\'(?:\\.|[^\\\'])*\'|"(?:\\.|[^\\"])*"',
                         re.DOTALL | re.MULTILINE)
    temp = [x for x in re.sub(pattern, replacer, source).split("\n") if x.strip() != ""]
    return "\n".join(temp)


def remove_python_comments_and_docstrings(source):
    """python_parser/parser_folder/utils.py:30-70, restated: re-emit the stdlib tokenize stream
    with the original column spacing, dropping comments and every STRING token that starts a
    logical line (after INDENT or NEWLINE, or at column 0); then drop blank lines."""
    import io
    import tokenize

    pieces, prev, row, col = [], tokenize.INDENT, -1, 0
    for tt, text, (srow, scol), (erow, ecol), _ in tokenize.generate_tokens(
            io.StringIO(source).readline):
        if srow > row:
            col = 0
        if scol > col:
            pieces.append(" " * (scol - col))
        if tt == tokenize.COMMENT:
            pass
        elif tt == tokenize.STRING:
            if prev not in (tokenize.INDENT, tokenize.NEWLINE) and scol > 0:
                pieces.append(text)
        else:
            pieces.append(text)
        prev, row, col = tt, erow, ecol
    return "\n".join(l for l in "".join(pieces).split("\n") if l.strip() != "")


def identifier_code_tokens(code: str, lang: str = "c"):
    """get_identifiers(code, lang)[1] (run_parser.py:190-216,272-281): '\\n' -> newline, comments
    (and for Python docstrings; left as is when that raises) removed, then the leaves."""
    code = code.replace("\\n", "\n")
    if lang != "python":
        code = remove_comments_and_docstrings(code, lang)
    else:
        try:
            code = remove_python_comments_and_docstrings(code)
        except Exception:
            pass
    return code_tokens(code, lang)


def get_example(code, tgt_word, substitute, lang="c"):
    """python_parser/run_parser.py:218-239 over this lexer's leaves."""
    code = code.replace("\\n", "\n")
    lv = leaves(code, lang)
    code = code.split("\n")
    replace_pos = {}
    for (sl, sc, el, ec, text) in lv:
        if text == tgt_word:
            replace_pos.setdefault(sl, []).append((sc, ec))
    diff = len(substitute) - len(tgt_word)
    for line in replace_pos.keys():
        for index, pos in enumerate(replace_pos[line]):
            code[line] = code[line][:pos[0] + index * diff] + substitute + code[line][pos[1] + index * diff:]
    return "\n".join(code)


def get_example_batch(code, chromesome, lang="c"):
    """python_parser/run_parser.py:242-266 over this lexer's leaves."""
    code = code.replace("\\n", "\n")
    lv = leaves(code, lang)
    code = code.split("\n")
    replace_pos = {}
    for tgt_word in chromesome.keys():
        diff = len(chromesome[tgt_word]) - len(tgt_word)
        for (sl, sc, el, ec, text) in lv:
            if text == tgt_word:
                replace_pos.setdefault(sl, []).append((tgt_word, chromesome[tgt_word], diff, sc, ec))
    for line in replace_pos.keys():
        diff = 0
        for index, pos in enumerate(replace_pos[line]):
            code[line] = code[line][:pos[3] + diff] + pos[1] + code[line][pos[4] + diff:]
            diff += pos[2]
    return "\n".join(code)


_TOK = None


def tokenizer():
    """transformers RobertaTokenizer (tokenizers-backed) on data/tokenizer — the oracle tokenizer."""
    global _TOK
    if _TOK is None:
        import random

        # importing / constructing the transformers tokenizer draws from Python's global random
        # stream; the attack oracles share that stream with the product under one seed, so the
        # first load must leave it untouched
        state = random.getstate()
        from transformers import RobertaTokenizer
        v = json.load(open(ROOT / "data" / "tokenizer" / "vocab.json", encoding="utf-8"))
        merges = [tuple(l.rstrip("\n").split(" ")) for l in
                  open(ROOT / "data" / "tokenizer" / "merges.txt", encoding="utf-8")
                  if not l.startswith("#version")]
        _TOK = RobertaTokenizer(vocab=v, merges=merges)
        random.setstate(state)
    return _TOK


def convert_code_to_features(code, block_size=512, tok=None):
    """CodeXGLUE/Defect-detection/code/attacker.py:38-45 -> ids list of length block_size."""
    tok = tok or tokenizer()
    code = " ".join(code.split())
    code_tokens = tok.tokenize(code)[:block_size - 2]
    source_tokens = [tok.cls_token] + code_tokens + [tok.sep_token]
    source_ids = tok.convert_tokens_to_ids(source_tokens)
    padding_length = block_size - len(source_ids)
    source_ids += [tok.pad_token_id] * padding_length
    return source_ids
