"""ctypes binding of include/alert_host.h (lib/libalert_host.so): tokeniser, leaf lexer and the
text-level identifier substitution that builds mutant inputs.  No pure-Python fallback."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import DATA_DIR, HOSTLIB_PATH

LANG = {"c": 0, "java": 1, "python": 2}
MODE_BATCH, MODE_SINGLE = 0, 1
MODE_RAW = 16  # flag: featurise the raw mutant text (Authorship-Attribution victim)
DFG_RUN_PARSER = 0  # python_parser/run_parser.py extract_dataflow
DFG_GCB_RUN = 1     # GraphCodeBERT/*/code/run.py extract_dataflow (parser/DFG.py + edge filter)

_LIB = None


def load_host_library(path=None) -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    p = str(path or HOSTLIB_PATH)
    if not os.path.exists(p):
        raise RuntimeError(f"host featurisation library not built: {p} missing (run `make`)")
    lib = ctypes.CDLL(p)
    if path is None:
        from .buildinfo import source_hash

        lib.ah_source_hash.restype = ctypes.c_char_p
        built, here = lib.ah_source_hash().decode(), source_hash("host")
        if built != here:
            raise RuntimeError(f"{p} was built from other sources (hash {built}, this tree "
                               f"{here}): rebuild it (`make` or __graft_entry__.build())")
    vp, i32, cp = ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p
    pp = ctypes.POINTER(ctypes.c_char_p)
    lib.ah_tokenizer_load.restype = vp
    lib.ah_tokenizer_load.argtypes = [cp, cp]
    lib.ah_tokenizer_free.argtypes = [vp]
    lib.ah_tokenizer_special.argtypes = [vp, i32]
    lib.ah_tokenize.argtypes = [vp, cp, vp, i32]
    lib.ah_decode.argtypes = [vp, vp, i32, vp, i32]
    lib.ah_featurize_batch.argtypes = [vp, i32, pp, i32, vp, vp]
    lib.ah_featurize_batch_raw.argtypes = [vp, i32, pp, i32, vp, vp]
    lib.ah_tokens_to_ids.argtypes = [vp, i32, pp, vp]
    lib.ah_example_new.restype = vp
    lib.ah_example_new.argtypes = [cp, i32]
    lib.ah_example_free.argtypes = [vp]
    lib.ah_example_num_leaves.argtypes = [vp, i32]
    lib.ah_example_leaves.argtypes = [vp, i32, vp, i32]
    lib.ah_example_mutant_text.argtypes = [vp, i32, i32, pp, pp, vp, i32]
    lib.ah_example_mutants.argtypes = [vp, vp, i32, i32, vp, pp, pp, i32, vp, vp]
    lib.ah_example_mutant_words.argtypes = [vp, vp, i32, i32, vp, pp, pp, i32, vp, i32, vp, vp]
    lib.ah_example_word_table.argtypes = [vp, vp, i32, vp, i32, ctypes.POINTER(i32)]
    lib.ah_example_identifiers.argtypes = [vp, vp, i32]
    lib.ah_example_dfg.argtypes = [vp, vp, i32, vp, i32]
    lib.ah_example_dfg_variant.argtypes = [vp, i32, vp, i32, vp, i32]
    lib.ah_remove_comments.argtypes = [cp, vp, i32]
    lib.ah_gcb_features_batch.argtypes = [vp, i32, pp] + [i32] * 7 + [vp] * 5
    lib.ah_last_error.restype = ctypes.c_char_p
    for f in ("ah_example_identifiers", "ah_example_dfg", "ah_example_dfg_variant",
              "ah_remove_comments", "ah_gcb_features_batch",
              "ah_tokenizer_special", "ah_tokenize", "ah_decode", "ah_featurize_batch",
              "ah_featurize_batch_raw", "ah_tokens_to_ids",
              "ah_example_num_leaves", "ah_example_leaves", "ah_example_mutant_text",
              "ah_example_mutants", "ah_example_mutant_words", "ah_example_word_table"):
        getattr(lib, f).restype = i32
    _LIB = lib
    return lib


def gcb_threads() -> int:
    """Worker threads of the batch featurisers: this process's CPU share (sched affinity), at
    most 16 (the GPU box's share per GPU), overridable with APMC_HOST_THREADS."""
    import os
    env = os.environ.get("APMC_HOST_THREADS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _err(what):
    raise RuntimeError(f"{what}: {_LIB.ah_last_error().decode(errors='replace')}")


def _cstrs(strs):
    arr = (ctypes.c_char_p * max(len(strs), 1))()
    for i, s in enumerate(strs):
        arr[i] = s.encode("utf-8")
    return arr


def _i32p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def remove_comments(code: str) -> str:
    """remove_comments_and_docstrings(code, 'c' | 'java') (parser_folder/utils.py:30-87)."""
    lib = load_host_library()
    b = code.encode("utf-8")
    need = lib.ah_remove_comments(b, None, 0)
    buf = ctypes.create_string_buffer(need)
    lib.ah_remove_comments(b, buf, need)
    return buf.raw[:need - 1].decode("utf-8")


class Tokenizer:
    """Byte-level BPE with RobertaTokenizer.tokenize semantics (C++)."""

    def __init__(self, vocab_json=None, merges_txt=None):
        self.lib = load_host_library()
        vocab_json = str(vocab_json or DATA_DIR / "tokenizer" / "vocab.json")
        merges_txt = str(merges_txt or DATA_DIR / "tokenizer" / "merges.txt")
        h = self.lib.ah_tokenizer_load(vocab_json.encode(), merges_txt.encode())
        if not h:
            _err("ah_tokenizer_load")
        self.h = ctypes.c_void_p(h)
        self.cls_token_id, self.pad_token_id, self.sep_token_id, self.unk_token_id, \
            self.mask_token_id = (self.lib.ah_tokenizer_special(self.h, k) for k in range(5))
        self.cls_token, self.sep_token, self.pad_token, self.unk_token = "<s>", "</s>", "<pad>", "<unk>"

    def __del__(self):
        try:
            self.lib.ah_tokenizer_free(self.h)
        except Exception:
            pass

    def encode_ids(self, text: str) -> list[int]:
        b = text.encode("utf-8")
        cap = max(16, len(b) * 2 + 16)
        out = np.empty(cap, dtype=np.int32)
        n = self.lib.ah_tokenize(self.h, b, _i32p(out), cap)
        if n > cap:
            out = np.empty(n, dtype=np.int32)
            n = self.lib.ah_tokenize(self.h, b, _i32p(out), n)
        return out[:n].tolist()

    def decode(self, ids) -> str:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int32).reshape(-1))
        need = self.lib.ah_decode(self.h, _i32p(a), a.size, None, 0)
        buf = ctypes.create_string_buffer(need)
        self.lib.ah_decode(self.h, _i32p(a), a.size, buf, need)
        return buf.value.decode("utf-8")

    def featurize(self, codes: list[str], L: int, raw: bool = False):
        """convert_code_to_features of each text -> (ids int32 [n, L], lens int32 [n]).
        raw: tokenize the text as is (Authorship-Attribution) instead of ' '.join(code.split())."""
        n = len(codes)
        ids = np.empty((n, L), dtype=np.int32)
        lens = np.empty((n,), dtype=np.int32)
        fn = self.lib.ah_featurize_batch_raw if raw else self.lib.ah_featurize_batch
        if n and fn(self.h, n, _cstrs(codes), L, _i32p(ids), _i32p(lens)) < 0:
            _err("ah_featurize_batch")
        return ids, lens

    def gcb_features(self, codes: list[str], lang: str, variant: int, normalize: bool,
                     code_length: int, data_flow_length: int, run_trunc: bool = False,
                     threads: int | None = None, e_cap: int | None = None):
        """GraphCodeBERT convert_code_to_features of each text on host worker threads, the graph
        mask left compact (ah_gcb_features_batch): -> dict of ids, pos [n, L], meta [n, 4]
        (node_index, max_length, nodes, edges), spans [n, L], edges [n, e_cap] int32."""
        n, L = len(codes), code_length + data_flow_length
        e_cap = e_cap or 4 * L
        threads = threads or gcb_threads()
        flags = (1 if normalize else 0) | (2 if run_trunc else 0)
        strs = _cstrs(codes)
        while True:
            out = {"ids": np.empty((n, L), np.int32), "pos": np.empty((n, L), np.int32),
                   "meta": np.empty((n, 4), np.int32), "spans": np.empty((n, L), np.int32),
                   "edges": np.zeros((n, e_cap), np.int32)}
            if not n or self.lib.ah_gcb_features_batch(
                    self.h, n, strs, LANG[lang], variant, flags, code_length, data_flow_length,
                    e_cap, threads, *(_i32p(out[k]) for k in
                                      ("ids", "pos", "meta", "spans", "edges"))) >= 0:
                return out
            msg = _LIB.ah_last_error().decode(errors="replace")
            # the reference has no edge limit: an edge-heavy query (long comesFrom lists) gets a
            # wider edge array; every consumer pads widths when it joins batches
            if "e_cap" not in msg or e_cap >= 64 * L:
                _err("ah_gcb_features_batch")
            e_cap *= 4

    def convert_tokens_to_ids(self, tokens):
        """tokenizer.convert_tokens_to_ids (a token string not in the vocabulary -> unk id)."""
        one = isinstance(tokens, str)
        toks = [tokens] if one else list(tokens)
        out = np.empty((max(len(toks), 1),), dtype=np.int32)
        if toks and self.lib.ah_tokens_to_ids(self.h, len(toks), _cstrs(toks), _i32p(out)) < 0:
            _err("ah_tokens_to_ids")
        return int(out[0]) if one else out[:len(toks)].tolist()


class Example:
    """One attacked program: its leaves and the mutant builder."""

    def __init__(self, code: str, lang: str = "c"):
        self.lib = load_host_library()
        self.code = code
        self.lang = lang
        h = self.lib.ah_example_new(code.encode("utf-8"), LANG[lang])
        if not h:
            _err("ah_example_new")
        self.h = ctypes.c_void_p(h)

    def __del__(self):
        try:
            self.lib.ah_example_free(self.h)
        except Exception:
            pass

    def leaves(self, identifiers: bool = False) -> list[str]:
        """identifiers=False: leaves get_example edits; True: get_identifiers' code tokens."""
        w = int(identifiers)
        need = self.lib.ah_example_leaves(self.h, w, None, 0)
        buf = ctypes.create_string_buffer(max(need, 1))
        self.lib.ah_example_leaves(self.h, w, buf, need)
        n = self.lib.ah_example_num_leaves(self.h, w)
        parts = buf.raw[:need].split(b"\0")[:n]
        return [p.decode("utf-8") for p in parts]

    def dfg_names(self) -> list[str]:
        """Unique data-flow-graph names in graph order (get_identifiers before its validity
        filter, run_parser.py:272-281): DFG_c / DFG_java / DFG_python by the example's language."""
        need = self.lib.ah_example_identifiers(self.h, None, 0)
        if need < 0:
            _err("ah_example_identifiers")
        buf = ctypes.create_string_buffer(max(need, 1))
        self.lib.ah_example_identifiers(self.h, buf, need)
        return [p.decode("utf-8") for p in buf.raw[:need].split(b"\0")[:-1]] if need else []

    def dfg(self, variant: int = DFG_RUN_PARSER):
        """extract_dataflow(code, lang)[0] as (idx, computed, from_idx list) per entry, sorted by
        leaf index (run_parser.py:190-216; DFG_c.py / DFG_java.py / DFG_python.py), or with
        variant=DFG_GCB_RUN GraphCodeBERT run.py's (parser/DFG.py + edge filter).  The entry's
        code is leaves(True)[idx]."""
        n = self.lib.ah_example_dfg_variant(self.h, variant, None, 0, None, 0)
        if n < 0:
            _err("ah_example_dfg_variant")
        rows = np.zeros((max(n, 1), 4), dtype=np.int32)
        cap = 16
        while True:
            fr = np.zeros((cap,), dtype=np.int32)
            r = self.lib.ah_example_dfg_variant(self.h, variant, _i32p(rows), n, _i32p(fr), cap)
            if r >= 0:
                break
            cap = -r - 1
        return [(int(a), bool(b), fr[o:o + c].tolist()) for a, b, o, c in rows[:n]]

    def mutant_text(self, pairs: list[tuple[str, str]], mode: int = MODE_BATCH) -> str:
        tg, sb = _cstrs([p[0] for p in pairs]), _cstrs([p[1] for p in pairs])
        need = self.lib.ah_example_mutant_text(self.h, mode, len(pairs), tg, sb, None, 0)
        if need < 0:
            _err("ah_example_mutant_text")
        buf = ctypes.create_string_buffer(need)
        self.lib.ah_example_mutant_text(self.h, mode, len(pairs), tg, sb, buf, need)
        return buf.raw[:need - 1].decode("utf-8")

    @staticmethod
    def _flatten(population):
        off, tg, sb = [0], [], []
        for pairs in population:
            for t, s in pairs:
                tg.append(t)
                sb.append(s)
            off.append(len(tg))
        return np.asarray(off, dtype=np.int32), _cstrs(tg), _cstrs(sb)

    def mutant_ids(self, tok: Tokenizer, population, L: int, mode: int = MODE_BATCH):
        """population: list of [(tgt, sub), ...] (chromosome items in dict order)."""
        n = len(population)
        off, tg, sb = self._flatten(population)
        ids = np.empty((n, L), dtype=np.int32)
        lens = np.empty((n,), dtype=np.int32)
        if n and self.lib.ah_example_mutants(self.h, tok.h, mode, n, _i32p(off), tg, sb, L,
                                             _i32p(ids), _i32p(lens)) < 0:
            _err("ah_example_mutants")
        return ids, lens

    def mutant_words(self, tok: Tokenizer, population, L: int, mode: int = MODE_BATCH):
        """-> (word_tok, word_off, mut_words, mut_off, lens) numpy int32 (ae_splice inputs)."""
        n = len(population)
        off, tg, sb = self._flatten(population)
        mut_off = np.empty((n + 1,), dtype=np.int32)
        lens = np.empty((n,), dtype=np.int32)
        cap = 1024 * max(n, 1)
        words = np.empty((cap,), dtype=np.int32)
        r = self.lib.ah_example_mutant_words(self.h, tok.h, mode, n, _i32p(off), tg, sb, L,
                                             _i32p(words), cap, _i32p(mut_off), _i32p(lens))
        if r < -1:
            cap = -r
            words = np.empty((cap,), dtype=np.int32)
            r = self.lib.ah_example_mutant_words(self.h, tok.h, mode, n, _i32p(off), tg, sb, L,
                                                 _i32p(words), cap, _i32p(mut_off), _i32p(lens))
        if r < 0:
            _err("ah_example_mutant_words")
        nw = ctypes.c_int32()
        nt = self.lib.ah_example_word_table(self.h, None, 0, None, 0, ctypes.byref(nw))
        word_tok = np.empty((max(nt, 1),), dtype=np.int32)
        word_off = np.empty((nw.value + 1,), dtype=np.int32)
        self.lib.ah_example_word_table(self.h, _i32p(word_tok), word_tok.size, _i32p(word_off),
                                       word_off.size, ctypes.byref(nw))
        return word_tok, word_off, words[:r], mut_off, lens
