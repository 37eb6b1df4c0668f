"""CPU: host featurisation library (C++) against the Python oracle (oracle/featurize_ref.py) and
the installed transformers RobertaTokenizer, on the reference's own attack fixtures
(data/devign/test_subs_*.jsonl, copied from CodeXGLUE/Defect-detection/preprocess/dataset)."""
import gzip
import json
import random

import numpy as np
import pytest

from conftest import ROOT
from oracle import featurize_ref as ref

DEVIGN = sorted((ROOT / "data" / "devign").glob("test_subs_*.jsonl"))
BCB_KEYS = ROOT / "tests" / "golden" / "bcb_java_keys.jsonl.gz"


def load(path, limit=None):
    out = []
    with open(path) as f:
        for i, line in enumerate(f):
            if limit is not None and i >= limit:
                break
            out.append(json.loads(line))
    return out


@pytest.fixture(scope="module")
def tok():
    from apmc_amd.host import Tokenizer
    return Tokenizer()


@pytest.fixture(scope="module")
def devign_small():
    return load(DEVIGN[0], 120)


def test_tokenizer_matches_transformers_on_all_fixture_functions(tok):
    rt = ref.tokenizer()
    n = 0
    for path in DEVIGN:
        for js in load(path):
            text = " ".join(js["func"].split())
            assert tok.encode_ids(text) == rt.convert_tokens_to_ids(rt.tokenize(text))
            n += 1
    assert n == 2732


@pytest.mark.parametrize("s", ["a <unk> b", "x<mask>y <s></s>", "  foo  ", "\t\tx\n\n  y",
                               "it's 'll 're 've", "说啊 ab12 3.5e-3", "\xa0x\u2003y", "", "<pad>",
                               "'z' \"s\\n\" /* c */ // d"])
def test_tokenizer_edge_cases(tok, s):
    rt = ref.tokenizer()
    assert tok.encode_ids(s) == rt.convert_tokens_to_ids(rt.tokenize(s))


def test_decode_roundtrip(tok):
    for s in ["int x = 1; // 说", " foo_bar", "\tq"]:
        assert tok.decode(tok.encode_ids(s)) == s


def test_leaves_match_oracle(devign_small):
    from apmc_amd.host import Example
    for js in devign_small:
        code = js["func"].replace("\\n", "\n")
        ex = Example(js["func"])
        assert ex.leaves() == ref.code_tokens(code, "c")
        assert ex.leaves(identifiers=True) == ref.identifier_code_tokens(js["func"], "c")


def test_remove_comments_matches_regex():
    from apmc_amd.host import Example
    cases = ["a = 1; // c\nb = '/*'; /* x\n y */ c = \"//\";",
             "don't /* it's */ x = 'a';\n  \n\t\ny", "/* open", "'\\'' // q"]
    for c in cases:
        assert Example(c).leaves(identifiers=True) == ref.identifier_code_tokens(c), c


def test_leaf_edge_cases():
    from apmc_amd.host import Example
    cases = [
        'int a = -1; b = a-1; c = x[2]-3; s = "a\\tb\\x41\\101"; ch = \'\\n\';',
        "#include <stdio.h>\n#define MAX(a, b) ((a) > (b) ? (a) : (b)) /* c */\nint x;",
        "#if defined(FOO) && BAR > 2\n  y++;\n#endif\n#pragma once\n  # undef Z",
        'x = L"wide" u8"u" U\'c\'; y = 0x1Fu + 1.5e-3f + .5 + 1e+10;',
        "p->q.r ... a >>= b <<= c; d = e ? f : g;",
        'line "unterminated\nnext = 1; /* multi\nline */ z;',
        "a = 1; /* never closed\n b = c;",
        'a = "说"; b = c; // 说\n d = e;',
        "q = 'x'; r = '\\'';",
    ]
    for c in cases:
        assert Example(c).leaves() == ref.code_tokens(c.replace("\\n", "\n"), "c"), c


def _random_chromosomes(js, rng, n):
    subs = js["substitutes"]
    keys = list(subs.keys())
    out = []
    for _ in range(n):
        chrom = {}
        for k in keys:
            if subs[k] and rng.random() < 0.6:
                chrom[k] = rng.choice(subs[k])
            else:
                chrom[k] = k
        out.append(chrom)
    return out


def test_get_example_batch_text_and_ids_match_oracle(devign_small, tok):
    from apmc_amd.host import Example
    rng = random.Random(0)
    for js in devign_small[:60]:
        if not js["substitutes"]:
            continue
        ex = Example(js["func"])
        chroms = _random_chromosomes(js, rng, 4)
        pops = [list(c.items()) for c in chroms]
        ids, lens = ex.mutant_ids(tok, pops, 512)
        for c, pairs, row, ln in zip(chroms, pops, ids, lens):
            text = ref.get_example_batch(js["func"], c, "c")
            assert ex.mutant_text(pairs) == text
            exp = ref.convert_code_to_features(text, 512)
            assert row.tolist() == exp
            assert ln == int((np.asarray(exp) != 1).sum())


def test_get_example_single_matches_oracle(devign_small, tok):
    from apmc_amd.host import MODE_SINGLE, Example
    for js in devign_small[:60]:
        ex = Example(js["func"])
        pops = []
        for var, subs in js["substitutes"].items():
            for s in subs[:5]:
                pops.append([(var, s)])
        if not pops:
            continue
        ids, lens = ex.mutant_ids(tok, pops, 512, mode=MODE_SINGLE)
        for pairs, row in zip(pops, ids):
            text = ref.get_example(js["func"], pairs[0][0], pairs[0][1], "c")
            assert ex.mutant_text(pairs, mode=MODE_SINGLE) == text
            assert row.tolist() == ref.convert_code_to_features(text, 512)


def test_offset_quirk_reproduced():
    """get_example_batch applies same-line edits in key order with a running diff."""
    from apmc_amd.host import Example
    code = "b = a;\nint c = b + a;"
    chrom = {"a": "xyz", "b": "b"}
    exp = ref.get_example_batch(code, chrom)
    assert exp != "b = xyz;\nint c = b + xyz;"  # the quirk garbles the line
    assert Example(code).mutant_text(list(chrom.items())) == exp


@pytest.mark.parametrize("single", [False, True])
def test_mutant_words_feed_the_same_ids(devign_small, tok, single):
    """The device-splice inputs (word table + per-mutant word ids; only the lines a mutant's
    edits touch are re-split, the others reuse the original's ids) give exactly the ids of the
    text path (get_example(_batch) -> ' '.join(split()) -> BPE), in both edit modes, incl.
    substitutes with spaces or non-ASCII text (the fallback that re-splits the whole text)."""
    from apmc_amd.host import MODE_SINGLE, Example
    rng = random.Random(1)
    odd = ["a b", "ü", "x\ty", "<pad>"]
    for js in devign_small[:40]:
        if not js["substitutes"]:
            continue
        ex = Example(js["func"])
        pops = [list(c.items()) for c in _random_chromosomes(js, rng, 5)]
        if single:
            pops = [[p[0]] for p in pops if p]
        pops.append([(pops[0][0][0], odd[rng.randrange(len(odd))])])
        kw = {"mode": MODE_SINGLE} if single else {}
        ids, lens = ex.mutant_ids(tok, pops, 512, **kw)
        word_tok, word_off, mut_words, mut_off, lens2 = ex.mutant_words(tok, pops, 512, **kw)
        assert (lens == lens2).all()
        for m in range(len(pops)):
            ws = mut_words[mut_off[m]:mut_off[m + 1]]
            toks = [t for w in ws for t in word_tok[word_off[w]:word_off[w + 1]]][:510]
            assert [0] + toks + [2] + [1] * (510 - len(toks)) == ids[m].tolist()


@pytest.mark.slow
def test_fixture_keys_are_lexer_identifiers():
    """Known-answer check: every substitute key of every Devign fixture example is an
    identifier leaf of our lexer (the reference took the keys from tree-sitter DFG identifiers)."""
    from apmc_amd.host import Example
    missing, total = [], 0
    for path in DEVIGN:
        for js in load(path):
            leaves = set(Example(js["func"]).leaves(identifiers=True))
            for k in js["substitutes"]:
                total += 1
                if k not in leaves:
                    missing.append(k)
    assert total == 17427
    # the only misses: 'm' / 'memory' GNU-asm constraint and clobber strings
    # (test_subs_800_1200 #151, test_subs_1200_1600 #161/#341), which tree-sitter's error
    # recovery surfaced as identifiers; parity with tree-sitter is unpinned there
    assert sorted(missing) == ["m", "m", "memory", "memory"], missing


# ------------------------------------------------------------------------------ data-flow graph
def _idents(code):
    from apmc_amd.attacker import get_identifiers
    return [i[0] for i in get_identifiers(code, "c")[0]]


def test_dfg_identifiers_known_answers():
    """DFG_c quirks (python_parser/parser_folder/DFG_c.py) the identifier list depends on."""
    # params first; `int a = 1` is an init_declarator, which DFG_c's misspelt 'init_declatator'
    # never matches -> not defined; pointer / array declarators are defined with or without '='
    code = "int f(int p, char *q) {\n int a = 1;\n int b;\n char *c = q;\n char d[4];\n}"
    assert _idents(code) == ["p", "q", "b", "c", "d"]
    # update_expression defines its operands; an assignment returns no entries at all
    code = "void g() {\n x = y++;\n z++;\n s->n--;\n}"
    assert _idents(code) == ["z", "s", "n"]
    # while bodies are walked twice: a late definition flows to an earlier use in the loop
    code = "void h(int k) {\n while (k) {\n if (k) use(late);\n int late;\n }\n}"
    ids = _idents(code)
    assert ids == ["k", "late"]
    from apmc_amd.host import Example
    ex = Example(code, "c")
    leaves = ex.leaves(True)
    first_late = min(i for i, _, _ in ex.dfg() if leaves[i] == "late")
    assert first_late == leaves.index("late")  # the use inside `use(late)`, before `int late;`
    # the identifier naming a function_declarator is skipped; prototypes' params are defined
    code = "void m(void) {\n int proto(int pa);\n}"
    assert _idents(code) == ["pa"]
    # macros: `static int coroutine_fn f(...)` (skipped), `int a, av_unused b;` (skipped)
    code = "static int coroutine_fn f(int u) {\n int a, av_unused b;\n}"
    assert _idents(code) == ["u", "a", "b"]


def dfg_key_parity():
    """Known answer from the reference's own output: the substitute keys of every Devign fixture
    function are get_substitutes.py:47-137 applied to get_identifiers(remove_comments(func)): the
    DFG names (run_parser.py:272-281) that occur as words (utils.get_identifier_posistions_from_code),
    are valid C names, have an occurrence inside the MLM's 510 sub-words, and keep >= 1 substitute.
    Returns (exact, consistent, total, residue): exact = our list after the same filters equals the
    keys; consistent = exact, or (function longer than 380 of our sub-words) equal once cut at the
    last key's first occurrence — the reference tokenizer's 510-sub-word boundary is unknowable
    offline (codebert vocab absent), so for long functions only a prefix is pinned."""
    from apmc_amd.host import Tokenizer, remove_comments
    from apmc_amd.utils import _tokenize, get_identifier_posistions_from_code, is_valid_variable_name
    tok = Tokenizer()
    exact = consistent = tot = 0
    residue = []
    for path in DEVIGN:
        for line, js in enumerate(load(path)):
            tot += 1
            keys = list(js["substitutes"].keys())
            from apmc_amd.attacker import get_identifiers
            idents, code_tokens = get_identifiers(remove_comments(js["func"]), "c")
            words, sub_words, kk = _tokenize(" ".join(code_tokens), tok)
            names = [i[0] for i in idents if " " not in i[0].strip()]
            pos = get_identifier_posistions_from_code(words, names)
            ours = [n for n in pos if is_valid_variable_name(n, "c")]
            if ours == keys:
                exact += 1
                consistent += 1
                continue
            if keys and len(sub_words) > 380 and all(k in pos for k in keys):
                last = max(kk[pos[k][0]][0] for k in keys)
                if [n for n in ours if kk[pos[n][0]][0] <= last] == keys:
                    consistent += 1
                    continue
            residue.append((path.name, line, [n for n in ours if n not in keys],
                            [k for k in keys if k not in ours]))
    return exact, consistent, tot, residue


def test_dfg_identifiers_vs_reference_fixture_keys():
    """tree-sitter's error recovery on macro-heavy code is not reproducible without the grammar,
    so the bar is a measured rate (DESIGN.md §5 lists the residue by cause): exact on >= 89% of the
    2732 functions, truncation-consistent on >= 98%."""
    exact, consistent, tot, residue = dfg_key_parity()
    assert tot == 2732
    assert exact / tot >= 0.89, (exact, tot)
    assert consistent / tot >= 0.98, (consistent, tot, residue[:5])


CLONE = ROOT / "data" / "clone" / "test_subs_0_500.jsonl"
AA = ROOT / "data" / "authorship" / "valid_subs.jsonl"


def test_java_python_leaves_match_oracle():
    """Java (BigCloneBench code1 and code2) and Python (authorship) leaves and identifier-pass
    leaves of the C++ lexer equal the oracle's, including the broken-literal rules (a Java literal
    cut by a raw newline is its quote alone; a Python string may start with a raw newline)."""
    from apmc_amd.host import Example
    n = 0
    for js in load(CLONE):
        for code in (js["code1"], js["code2"]):
            ex = Example(code, "java")
            assert ex.leaves() == ref.code_tokens(code.replace("\\n", "\n"), "java")
            assert ex.leaves(identifiers=True) == ref.identifier_code_tokens(code, "java")
            n += 1
    for js in load(AA):
        code = js["code"].replace("\\n", "\n")
        assert Example(code, "python").leaves() == ref.code_tokens(code, "python")
        n += 1
    assert n == 1132


def key_parity(task):
    """dfg_key_parity for the Java (clone code1, CodeXGLUE/Clone-detection-BigCloneBench/
    dataset/get_substitutes.py:74-165) and Python (authorship, CodeXGLUE/Authorship-Attribution/
    dataset/get_substitutes.py:52-140) fixtures: (exact, consistent, subsequence, total).
    subsequence = the keys are an ordered subsequence of our names (the only difference is names
    the reference kept no substitute for).  Java runs over all 4,000 code1 functions of the eight
    BigCloneBench test_subs_*.jsonl files the reference holds (tests/golden/bcb_java_keys.jsonl.gz,
    made by tests/golden/make_bcb_java_keys.py); the classification is tools/java_key_parity.py's."""
    from apmc_amd.host import Tokenizer
    from apmc_amd.substitutes import substitute_identifiers
    from apmc_amd.utils import _tokenize, get_identifier_posistions_from_code, is_valid_variable_name
    tok = Tokenizer()
    lang = "java" if task == "clone" else "python"
    exact = consistent = subseq = tot = 0
    distinct = {}
    if task == "clone":
        with gzip.open(BCB_KEYS, "rt", encoding="utf-8") as f:
            items = [(js["code1"], js["keys"]) for js in map(json.loads, f)]
    else:
        items = [(js["code"], list(js["substitutes"].keys())) for js in load(AA)]
    for code, keys in items:
        tot += 1
        # the stored text as the task's get_substitutes.py reads it (the authorship programs with
        # their newlines as literal '\\n': its comment remover runs on that one-line form)
        idents, toks = substitute_identifiers(code, lang)
        words, sub_words, kk = _tokenize(" ".join(toks), tok)
        names = [i[0] for i in idents if " " not in i[0].strip()]
        pos = get_identifier_posistions_from_code(words, names)
        ours = [n for n in pos if is_valid_variable_name(n, lang)]
        it = iter(ours)
        is_sub = all(k in it for k in keys)
        subseq += is_sub
        cls = "other"
        if ours == keys:
            cls = "exact"
        elif keys and len(sub_words) > 380 and all(k in pos for k in keys):
            last = max(kk[pos[k][0]][0] for k in keys)
            if [n for n in ours if kk[pos[n][0]][0] <= last] == keys:
                cls = "consistent"
        if cls == "other" and is_sub:
            cls = "subsequence"
        exact += cls == "exact"
        consistent += cls in ("exact", "consistent")
        distinct.setdefault(code, cls)
    key_parity.distinct = distinct
    return exact, consistent, subseq, tot


def test_dfg_java_python_vs_reference_fixture_keys():
    """DFG_java / DFG_python (dfg_java.cpp, dfg_python.cpp) against the reference's own keys, at
    the measured counts (DESIGN.md §5 classifies every remaining function by cause).  Java: all
    4,000 BigCloneBench code1 functions of the eight fixture files (749 distinct texts), 3,415 /
    3,848 / 3,916 exact / truncation-consistent / ordered subsequence; by distinct text 648 exact,
    721 consistent, 13 more an ordered subsequence (names the reference's MLM kept no substitute
    for) and 15 other (tree-sitter's recovery after a string literal broken by the \\n rewrite,
    DESIGN §5).  Python 90 / 130 / 130 of the 132 authorship programs (the two left: a broken
    string literal whose tree-sitter recovery defines two names, and a program that is Haskell)."""
    e, c, s, t = key_parity("clone")
    assert t == 4000 and e >= 3415 and c >= 3848 and s >= 3916, (e, c, s, t)
    d = list(key_parity.distinct.values())
    assert len(d) == 749 and d.count("exact") >= 648, (len(d), d.count("exact"))
    assert d.count("exact") + d.count("consistent") >= 721
    assert len(d) - d.count("other") >= 734, d.count("other")
    e, c, s, t = key_parity("authorship")
    assert t == 132 and e >= 90 and c >= 130 and s >= 130, (e, c, s, t)


def _names(code, lang):
    from apmc_amd.host import Example
    return Example(code, lang).dfg_names()


def test_dfg_java_known_answers():
    """DFG_java quirks (python_parser/parser_folder/DFG_java.py) the identifier list depends on."""
    # the bare method: name and parameters are definitions (recovered declaration)
    assert _names("void f(int a, String b) { int c = a; }", "java") == ["f", "a", "b", "c"]
    # a declarator whose value has no named leaf (`false`) defines the name without an entry:
    # it enters the graph at its first use
    assert _names("void f() { boolean x = false; int y = 1; g(y, x); }", "java") == \
        ["f", "y", "x"]
    # catch parameters and inferred lambda parameters are not definitions
    assert _names("void f() { try { g(); } catch (Exception e) { e.h(); } }", "java") == ["f"]
    assert _names("void f() { r(x -> x + 1); r((p, q) -> p); }", "java") == ["f"]
    assert _names("void f() { r((int p) -> p); }", "java") == ["f", "p"]
    # a method name called on an object is never walked; unqualified it is (if defined)
    assert _names("void f() { int g = 1; o.g(); g(); }", "java") == ["f", "g"]
    # enhanced for / assignment / update definitions
    assert _names("void f() { for (String s : xs) { t = s; i++; } }", "java") == \
        ["f", "s", "t", "i"]
    # throws: later simple names are declarators after <= 1 parameter
    assert _names("void f(int a) throws A, B { }", "java") == ["f", "a", "B"]
    assert _names("void f(int a, int b) throws A, B { }", "java") == ["f", "a", "b"]
    # a constructor recovered as a call (no modifier, or modifiers and no parameters): its
    # parameters are leaves and every exception type of `throws` is a declarator
    assert _names("F(int p) throws A, B { }", "java") == ["A", "B"]
    assert _names("public F() throws A, B { int x = 1; }", "java") == ["A", "B", "x"]
    assert _names("public F(int p) throws A, B { }", "java") == ["p"]
    # a marker annotation shifts the throws declarators to the third type, <= 2 parameters
    assert _names("@Override public void f(String m) throws A, B, C, D { }", "java") == \
        ["f", "m", "C", "D"]
    assert _names("@Override void f(int a, int b) throws A, B, C { }", "java") == \
        ["f", "a", "b", "C"]
    assert _names("@Override void f(int a, int b, int c) throws A, B, C { }", "java") == \
        ["f", "a", "b", "c"]
    assert _names('@SuppressWarnings("x") void f(int a) throws A, B, C { }', "java") == \
        ["f", "a", "B", "C"]


def test_dfg_python_known_answers():
    """DFG_python quirks (python_parser/parser_folder/DFG_python.py)."""
    # parameters: plain identifiers define, *args / **kw / typed do not; default_parameter with
    # a value without named leaves ([]) defines without an entry
    assert _names("def f(a, b=1, c=[], *d, **e):\n    return a + c", "python") == \
        ["a", "b", "c"]
    # tuple assignment pairs children; attribute targets define every named leaf
    assert _names("x, y = 1, 2\nself.z = x", "python") == ["x", "y", "self", "z"]
    # comprehension variables are defined before the element is walked
    assert _names("r = [v * 2 for v in xs]", "python") == ["r", "v"]
    # for: the body is walked only when it is the last child — with an else clause neither the
    # body nor the else clause reaches the graph
    assert _names("for i in a:\n    k = i\nelse:\n    m = 1", "python") == ["i"]
    assert _names("for i in a:\n    k = i", "python") == ["i", "k"]
    # lambda parameters are not definitions (default parameters are)
    assert _names("g = lambda u, w=1: u", "python") == ["g", "w"]


def _leaf_spans(code, leaves):
    """(line, column) start / end of every leaf, found left to right in the code text — the
    tree_to_token_index points (run_parser.py:199-204) of a lexer whose leaves are the text's."""
    lines, spans, ln, col = code.split("\n"), [], 0, 0
    for t in leaves:
        while True:
            c = lines[ln].find(t, col)
            if c >= 0:
                break
            ln, col = ln + 1, 0
        spans.append(((ln, c), (ln, c + len(t))))
        col = c + len(t)
    return spans


def test_python_junda_known_answer():
    """The reference's one known answer for the Python leaf lexer, python_parser/junda_test.md:1-18:
    for its snippet, the occurrences of c, d, e, f are leaves c -> [5, 12], d -> [10, 17, 22],
    e -> [15], f -> [20] at exactly the (line, column) spans listed there.  The same page's
    name set includes the typed parameter `c: int`; DFG_python.py:19-27 defines a parameter
    only when the identifier's parent is `parameters` (a `typed_parameter` is not), so
    get_identifiers (run_parser.py:272-281) of the snippet is [d, e, f] — our graph says the
    same (test_dfg_python_known_answers: typed parameters do not define)."""
    from apmc_amd.host import Example
    code = "import a\ndef b(c: int):\n    d = c + 10\n    e = d + 10\n    f = d + 20"
    want = {
        "c": ([5, 12], [((1, 6), (1, 7)), ((2, 8), (2, 9))]),
        "d": ([10, 17, 22], [((2, 4), (2, 5)), ((3, 8), (3, 9)), ((4, 8), (4, 9))]),
        "e": ([15], [((3, 4), (3, 5))]),
        "f": ([20], [((4, 4), (4, 5))]),
    }
    ex = Example(code, "python")
    for which in (0, 1):  # get_example's leaves and get_identifiers' (comment-stripped) leaves
        leaves = ex.leaves(identifiers=bool(which))
        spans = _leaf_spans(code, leaves)
        for name, (idx, pos) in want.items():
            got = [i for i, t in enumerate(leaves) if t == name]
            assert got == idx, (name, got)
            assert [spans[i] for i in got] == pos, (name, [spans[i] for i in got])
    # every data-flow entry sits on one of those occurrences
    leaves = ex.leaves(identifiers=True)
    names = ex.dfg_names()
    assert names == ["d", "e", "f"]
    for i, _, _ in ex.dfg():
        assert i in want[leaves[i]][0]
