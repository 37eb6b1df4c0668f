"""Masked-LM substitute generation over the engine — the reference's preprocessing step that
builds every example's `substitutes` dict (CodeXGLUE/Defect-detection/preprocess/get_substitutes.py
:46-139) and the helpers it calls (utils.py:209-248 get_bpe_substitues, :251-277 get_substitues).

Per example (one `item` of the jsonl):
  1. identifiers and code tokens of the comment-stripped function (get_identifiers over the host
     data-flow graph, host/dfg.cpp); words / sub-word keys (utils.py:174-189 _tokenize);
  2. ONE masked-LM pass over [CLS] + sub-words[:block-2] + [SEP] with a vocabulary-wide top-60
     (ae_mlm_topk: MFMA logits GEMM + radix-select top-k kernel);
  3. per occurrence of every valid identifier: the 60 candidate rewrites of its sub-word span are
     re-encoded as ONE device batch (ae_encode_rows: the last layer runs for each candidate's own
     span rows only, and only those are written back) and
     ranked by sum-of-cosine / span length against the original's span (ae_cosine_rank); the top
     30 survive (Python's stable sort on the host, as the reference);
  4. single-sub-word spans decode their 30 ids; multi-sub-word spans take the capped cartesian
     product of the first 4 candidates of the first 12 rows (<= 24 rows), score each by masked-LM
     perplexity (ae_mlm_nll) and sort ascending (utils.py:209-248);
  5. the union, minus names already in the function and invalid names, is the entry.
GraphCodeBERT's variant (cosine=False; GraphCodeBERT/Defect-detection/preprocess/get_substitutes.py
:72-134, where the cosine block is commented out) skips step 3: all 60 candidates of every
occurrence go straight to step 4 (no re-encodes).
Every reference call of the MLM is made without attention_mask, so every call here uses the
attend-pad form.  The per-item output (`item["substitutes"]`) has the reference's schema; list order
inside an entry follows Python set iteration in the reference and is not reproduced (compare as
sets).
"""
from __future__ import annotations

import json
import time

import numpy as np

from .attacker import get_identifiers
from .host import Tokenizer, remove_comments
from .utils import _tokenize, get_identifier_posistions_from_code, is_valid_substitue, \
    is_valid_variable_name

K_TOP = 60  # get_substitutes.py:63


def substitute_identifiers(code: str, lang: str):
    """get_identifiers as each task's get_substitutes.py calls it on the stored program text.
    C (Defect-detection/preprocess/get_substitutes.py:54) and Java (Clone-detection-BigCloneBench/
    dataset/get_substitutes.py): get_identifiers(remove_comments_and_docstrings(code, lang)).
    Python (Authorship-Attribution/dataset/get_substitutes.py:54-57): the stored program is ONE
    line whose newlines are the two characters '\\n', and the tokenize-based comment / docstring
    remover runs on that form before get_identifiers turns them into newlines — so a '#' comment
    removes the rest of the program, and a program tokenize rejects keeps its comments (the
    except branch).  Pinned by the fixture keys (tests/test_host.py::key_parity)."""
    if lang == "python":
        from .attacker import remove_python_docstrings
        try:
            return get_identifiers(remove_python_docstrings(code), lang)
        except Exception:
            return get_identifiers(code, lang)
    return get_identifiers(remove_comments(code), lang)


class SubstituteGenerator:
    """`engine` is an Engine built with_mlm=True (head "none" is enough).  cosine=False is the
    GraphCodeBERT preprocessing (no naturalness re-encode: every top-60 candidate is kept)."""

    def __init__(self, engine, tokenizer: Tokenizer | None = None, block_size: int = 512,
                 lang: str = "c", cosine: bool = True):
        self.engine = engine
        self.tok = tokenizer or Tokenizer()
        self.block_size = block_size
        self.lang = lang
        self.cosine = cosine
        self.tokens_per_call = 1 << 18  # candidate tokens per re-encode call (workspace bound)
        self.stats = {"examples": 0, "occurrences": 0, "encoded_seqs": 0, "encoded_tokens": 0,
                      "bpe_batches": 0, "encoder_flop": 0.0}

    def _enc_flop(self, L: int) -> float:
        """Algorithmic FLOP of one encoder pass over L tokens (SURVEY §8(d) F_enc)."""
        sh = self.engine.shape
        per_tok = 2 * (4 * sh.hidden * sh.hidden + 2 * sh.hidden * sh.ffn)
        return sh.layers * (L * per_tok + 4 * L * L * sh.hidden)

    # ------------------------------------------------------------------------------------------
    def _bpe_words(self, substitutes: np.ndarray, trace=None) -> list[str]:
        """get_bpe_substitues (utils.py:209-248) with the perplexity on the device."""
        import torch

        substitutes = substitutes[0:12, 0:4]
        all_subs: list[list[int]] = []
        for i in range(substitutes.shape[0]):
            if len(all_subs) == 0:
                all_subs = [[int(c)] for c in substitutes[i]]
            else:
                all_subs = [a + [int(j)] for a in all_subs[:24] for j in substitutes[i]]
        cand = np.asarray(all_subs[:24], dtype=np.int32)
        dev = f"cuda:{self.engine.device}"
        nll = self.engine.mlm_nll(torch.from_numpy(cand).to(dev)).double().cpu().numpy()
        self.stats["bpe_batches"] += 1
        ppl = np.exp(nll.astype(np.float32).mean(axis=1, dtype=np.float32))
        if trace is not None:
            trace.setdefault("bpe", []).append((cand.copy(), ppl.copy()))
        order = np.argsort(ppl, kind="stable")
        return [self.tok.decode(cand[i]) for i in order]

    def _words(self, similar: np.ndarray, trace=None) -> list[str]:
        """get_substitues(similar, tok, mlm, use_bpe=1, scores, threshold=0) (utils.py:251-277)."""
        sub_len = similar.shape[0]
        if sub_len == 0:
            return []
        if sub_len == 1:
            return [self.tok.decode([int(i)]) for i in similar[0]]
        return self._bpe_words(similar, trace)

    # ------------------------------------------------------------------------------------------
    def generate(self, func: str, trace=None) -> dict[str, list[str]]:
        """`item["substitutes"]` for one function (get_substitutes.py:54-137)."""
        identifiers, code_tokens = substitute_identifiers(func, self.lang)
        variable_names = [name[0] for name in identifiers if " " not in name[0].strip()]
        return self.generate_from_tokens(code_tokens, variable_names, trace)

    def generate_from_tokens(self, code_tokens, variable_names, trace=None):
        import torch

        tok = self.tok
        words, sub_ids, keys = _tokenize(" ".join(code_tokens), tok)
        ids = [tok.cls_token_id] + list(sub_ids[:self.block_size - 2]) + [tok.sep_token_id]
        L = len(ids)
        dev = f"cuda:{self.engine.device}"
        ids_np = np.asarray(ids, dtype=np.int32)
        ids_dev = torch.from_numpy(ids_np).to(dev)
        scores, preds = self.engine.mlm_topk(ids_dev, K_TOP)
        # rows 1 .. L-1 (word_predictions[1:len(sub_words)+1], get_substitutes.py:66-67)
        preds = preds[1:].cpu().numpy()
        n_pred = preds.shape[0]
        orig = (self.engine.encode(ids_dev[None], np.array([L], np.int32), attend_pad=True)[0]
                if self.cosine else None)
        if trace is not None:
            trace["ids"] = ids_np.copy()
            trace["topk_ids"] = preds.copy()
            trace["topk_scores"] = scores[1:].cpu().numpy()
            trace["sims"] = []
        from .engine import cosine_rank

        positions = get_identifier_posistions_from_code(words, variable_names)
        # every (word, occurrence) that reaches the cosine filter, in the reference's loop order
        occ = []
        for tgt_word, tgt_positions in positions.items():
            if not is_valid_variable_name(tgt_word, self.lang):
                continue
            for one_pos in tgt_positions:
                k0, k1 = keys[one_pos]
                if k0 < n_pred:
                    occ.append((tgt_word, one_pos, k0, min(k1, n_pred)))  # slices clip at L - 1
        # re-encode the 60 candidates of several occurrences per device call (rows of a batch are
        # independent, so batching changes nothing but float rounding); one host sync per chunk
        per_call = max(1, min(16, self.tokens_per_call // (K_TOP * L)))
        sims_of = {}
        for c0 in range(0, len(occ) if self.cosine else 0, per_call):
            chunk = occ[c0:c0 + per_call]
            # each candidate sequence is read only at its own occurrence's span (rows k0+1 ..
            # k1e): one window of the chunk's widest span per sequence, so the last layer runs for
            # those rows only (ae_encode_rows); a window that would pass L - 1 starts earlier
            nrows = max(k1e - k0 for _, _, k0, k1e in chunk)
            batch = np.repeat(ids_np[None], K_TOP * len(chunk), axis=0)
            row0 = np.empty(len(batch), dtype=np.int32)
            for j, (_, _, k0, k1e) in enumerate(chunk):
                batch[j * K_TOP:(j + 1) * K_TOP, k0 + 1:k1e + 1] = preds[k0:k1e].T
                row0[j * K_TOP:(j + 1) * K_TOP] = min(k0 + 1, L - nrows)
            bdev = torch.from_numpy(batch).to(dev)
            hid = self.engine.encode_rows(bdev, np.full((len(batch),), L, np.int32), row0, nrows,
                                          attend_pad=True)
            sims = torch.empty((len(chunk), K_TOP), dtype=torch.float32, device=dev)
            for j, (_, _, k0, k1e) in enumerate(chunk):
                r = k0 + 1 - int(row0[j * K_TOP])
                cand = hid[j * K_TOP:(j + 1) * K_TOP, r:r + k1e - k0].contiguous()
                sims[j] = cosine_rank(orig[k0 + 1:k1e + 1].contiguous(), cand, eps=1e-6)
            sims = sims.cpu().numpy()
            for j, o in enumerate(chunk):
                sims_of[o] = sims[j]
            self.stats["occurrences"] += len(chunk)
            self.stats["encoded_seqs"] += len(batch)
            self.stats["encoded_tokens"] += len(batch) * L
            self.stats["encoder_flop"] += len(batch) * self._enc_flop(L)
        result: dict[str, list[str]] = {}
        all_subs: dict[str, list[str]] = {}
        for o in occ:
            tgt_word, one_pos, k0, k1e = o
            cand_ids = preds[k0:k1e]  # [span, 60]
            if not self.cosine:  # GraphCodeBERT: get_substitues on all 60 candidates
                self.stats["occurrences"] += 1
                all_subs.setdefault(tgt_word, []).extend(self._words(cand_ids, trace))
                continue
            sims = sims_of[o]
            if trace is not None:
                trace["sims"].append((tgt_word, one_pos, [float(v) for v in sims],
                                      [tuple(int(x) for x in c) for c in cand_ids.T]))
            # sorted(sims, key=sim, reverse=True): stable, ties keep candidate order
            order = sorted(range(K_TOP), key=lambda i: sims[i], reverse=True)[:K_TOP // 2]
            all_subs.setdefault(tgt_word, []).extend(self._words(cand_ids[:, order], trace))
        for tgt_word, subs in all_subs.items():
            for s in set(subs):
                if s.strip() in variable_names:
                    continue
                if not is_valid_substitue(s.strip(), tgt_word, self.lang):
                    continue
                result.setdefault(tgt_word, []).append(s)
        self.stats["examples"] += 1
        return result


def generate_file(gen: SubstituteGenerator, in_path, out_path, start=0, end=None, queue=None,
                  log=None):
    """get_substitutes.py main loop over items [start, end) of a jsonl (`func` or `code` field);
    writes item + "substitutes" per line.  queue: optional callable returning the next item index
    (multi-GPU sharding; then `out_path` receives this rank's items, merge with merge_shards)."""
    items = []
    with open(in_path) as f:
        for i, line in enumerate(f):
            if i < start or (end is not None and i >= end):
                continue
            items.append((i, json.loads(line.strip())))
    t0 = time.time()
    done = []
    with open(out_path, "w") as wf:
        pos = 0
        while True:
            if queue is not None:
                k = queue()
                if k is None or k >= len(items):
                    break
            else:
                if pos >= len(items):
                    break
                k = pos
                pos += 1
            idx, item = items[k]
            code = item["func"] if "func" in item else item["code"]
            item["substitutes"] = gen.generate(code)
            wf.write(json.dumps({"_line": idx, **item}) + "\n" if queue is not None
                     else json.dumps(item) + "\n")
            done.append(idx)
            if log:
                log(idx, item)
    return {"items": len(done), "wall_s": time.time() - t0, **gen.stats}


def merge_shards(shard_paths, out_path):
    """Merge per-rank shard files (lines tagged with their input line) into input order."""
    rows = []
    for p in shard_paths:
        with open(p) as f:
            for line in f:
                js = json.loads(line)
                rows.append((js.pop("_line"), js))
    rows.sort(key=lambda r: r[0])
    with open(out_path, "w") as wf:
        for _, js in rows:
            wf.write(json.dumps(js) + "\n")
    return len(rows)
