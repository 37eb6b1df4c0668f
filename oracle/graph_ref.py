"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

Pure-Python restatement of GraphCodeBERT's per-query host work and forward, line for line:
  * convert_code_to_features (GCB)  GraphCodeBERT/Defect-detection/code/attacker.py:30-63
    (list-of-token-lists, ori2cur_pos dict, reverse_index remap) with the installed transformers
    RobertaTokenizer (featurize_ref.tokenizer());
  * GraphCodeDataset.__getitem__ mask  utils.py:547-576 (Python loops over a numpy bool matrix);
  * Model.forward                     GraphCodeBERT/Defect-detection/code/model.py:24-45 and
    GraphCodeBERT/clonedetection/code/model.py:41-64: nodes_to_token_mask normalised by
    (sum + 1e-10), einsum average, then RoBERTa with inputs_embeds, the 3-D mask and explicit
    position ids (roberta_cpu.encoder_forward).

The data-flow graph itself (extract_dataflow) comes from the product's C DFG
(csrc/host/dfg.cpp, tree-sitter absent — parity with tree-sitter UNPINNED, pinned instead to the
reference's fixture key lists in tests/test_host.py); this oracle checks everything downstream
of the DFG: sub-token spans, truncation, node remapping, the mask and the node-averaged forward.
"""
from __future__ import annotations

import numpy as np
import torch

from . import featurize_ref
from . import roberta_cpu


def convert_code_to_features(dfg, code_tokens, code_length=512, data_flow_length=128,
                             run_trunc=False):
    """dfg: [(code, idx, rel, [names], [idx])] sorted by idx; code_tokens: leaf strings.
    Returns (input_ids, position_idx, dfg_to_code, dfg_to_dfg) exactly as attacker.py:30-63
    (run_trunc: GraphCodeBERT/clonedetection/code/run.py:166's truncation)."""
    tokenizer = featurize_ref.tokenizer()
    dfg = list(dfg)
    code_tokens = [tokenizer.tokenize('@ ' + x)[1:] if idx != 0 else tokenizer.tokenize(x)
                   for idx, x in enumerate(code_tokens)]
    ori2cur_pos = {}
    ori2cur_pos[-1] = (0, 0)
    for i in range(len(code_tokens)):
        ori2cur_pos[i] = (ori2cur_pos[i - 1][1], ori2cur_pos[i - 1][1] + len(code_tokens[i]))
    code_tokens = [y for x in code_tokens for y in x]
    if run_trunc:
        code_tokens = code_tokens[:code_length + data_flow_length - 3
                                  - min(len(dfg), data_flow_length)][:512 - 3]
    else:
        code_tokens = code_tokens[:code_length + data_flow_length - 2
                                  - min(len(dfg), data_flow_length)]
    source_tokens = [tokenizer.cls_token] + code_tokens + [tokenizer.sep_token]
    source_ids = tokenizer.convert_tokens_to_ids(source_tokens)
    position_idx = [i + tokenizer.pad_token_id + 1 for i in range(len(source_tokens))]
    dfg = dfg[:code_length + data_flow_length - len(source_tokens)]
    source_tokens += [x[0] for x in dfg]
    position_idx += [0 for x in dfg]
    source_ids += [tokenizer.unk_token_id for x in dfg]
    padding_length = code_length + data_flow_length - len(source_ids)
    position_idx += [tokenizer.pad_token_id] * padding_length
    source_ids += [tokenizer.pad_token_id] * padding_length
    reverse_index = {}
    for idx, x in enumerate(dfg):
        reverse_index[x[1]] = idx
    for idx, x in enumerate(dfg):
        dfg[idx] = x[:-1] + ([reverse_index[i] for i in x[-1] if i in reverse_index],)
    dfg_to_dfg = [x[-1] for x in dfg]
    dfg_to_code = [ori2cur_pos[x[1]] for x in dfg]
    length = len([tokenizer.cls_token])
    dfg_to_code = [(x[0] + length, x[1] + length) for x in dfg_to_code]
    return source_ids, position_idx, dfg_to_code, dfg_to_dfg


def graph_mask(input_ids, position_idx, dfg_to_code, dfg_to_dfg, L):
    """utils.py:547-570 with its loops."""
    attn_mask = np.zeros((L, L), dtype=bool)
    node_index = sum([i > 1 for i in position_idx])
    max_length = sum([i != 1 for i in position_idx])
    attn_mask[:node_index, :node_index] = True
    for idx, i in enumerate(input_ids):
        if i in [0, 2]:
            attn_mask[idx, :max_length] = True
    for idx, (a, b) in enumerate(dfg_to_code):
        if a < node_index and b < node_index:
            attn_mask[idx + node_index, a:b] = True
            attn_mask[a:b, idx + node_index] = True
    for idx, nodes in enumerate(dfg_to_dfg):
        for a in nodes:
            if a + node_index < len(position_idx):
                attn_mask[idx + node_index, a + node_index] = True
    return attn_mask


@torch.no_grad()
def graph_score(sd, inputs_ids, attn_mask, position_idx, kind="sigmoid1", layers=12):
    """GraphCodeBERT Model.forward (devign: sigmoid1; clone: pair2 over interleaved rows)."""
    inputs_ids = torch.as_tensor(np.asarray(inputs_ids), dtype=torch.long)
    position_idx = torch.as_tensor(np.asarray(position_idx), dtype=torch.long)
    attn_mask = torch.as_tensor(np.asarray(attn_mask), dtype=torch.bool)
    nodes_mask = position_idx.eq(0)
    token_mask = position_idx.ge(2)
    inputs_embeddings = roberta_cpu._t(sd, "embeddings.word_embeddings.weight")[inputs_ids]
    nodes_to_token_mask = nodes_mask[:, :, None] & token_mask[:, None, :] & attn_mask
    nodes_to_token_mask = nodes_to_token_mask / (nodes_to_token_mask.sum(-1) + 1e-10)[:, :, None]
    avg_embeddings = torch.einsum("abc,acd->abd", nodes_to_token_mask, inputs_embeddings)
    inputs_embeddings = inputs_embeddings * (~nodes_mask)[:, :, None] + \
        avg_embeddings * nodes_mask[:, :, None]
    h = roberta_cpu.encoder_forward(sd, inputs_ids, pos=position_idx, attn_mask=attn_mask,
                                    layers=layers, inputs_embeds=inputs_embeddings)
    return roberta_cpu.head_forward(sd, h, kind).numpy()


class GraphTextVictim:
    """Text-driven GraphCodeBERT victim for oracle/attack_ref.py's greedy / ga: every query text
    is featurised here (the product's data-flow graph of the text, then this file's features and
    mask) and scored by `score(ids, pos, bits) -> head outputs` (pair rows interleaved).

    task: gcb_devign (C, ' '.join(split()), run_parser flow), gcb_clone (Java pairs: mutants and
    code2 with the run_parser flow; the dataset example with GraphCodeBERT run.py's flow and
    truncation; importance rows against ' '.join(leaves of code2)), gcb_authorship (Python,
    run.py's flow for every query)."""

    def __init__(self, score, task, code0, code_length=512, data_flow_length=128, code2=None):
        from . import attack_ref

        self._fmt = attack_ref.Victim(None, code_length + data_flow_length, task=task)
        self.lang, self.base = self._fmt.lang, self._fmt.base
        self.ga_children, self.empty_pool_exit = self._fmt.ga_children, self._fmt.empty_pool_exit
        self.task, self.score, self.code0, self.code2 = task, score, code0, code2
        self.cl, self.dl = code_length, data_flow_length
        self.query = 0
        if task == "gcb_clone":
            self.code2_words = " ".join(featurize_ref.identifier_code_tokens(code2, "java"))

    def _feats(self, code, variant, run_trunc=False):
        # a pure function of its arguments; MHM chains re-score the same candidate texts many
        # times, so results are memoised per victim
        key = (code, variant, run_trunc)
        memo = self.__dict__.setdefault("_memo", {})
        if key not in memo:
            memo[key] = self._feats_uncached(code, variant, run_trunc)
        return memo[key]

    def _feats_uncached(self, code, variant, run_trunc=False):
        from apmc_amd.graph import extract_dataflow

        if self.base == "devign":
            code = " ".join(code.split())
        dfg, _, toks = extract_dataflow(code, self.lang, variant)
        ids, pos, d2c, d2d = convert_code_to_features(dfg, toks, self.cl, self.dl, run_trunc)
        L = len(ids)
        m = graph_mask(ids, pos, d2c, d2d, L)
        return ids, pos, np.packbits(m, axis=-1, bitorder="little").view("<i4")

    def _variant(self):
        return 1 if self.base == "authorship" else 0

    def _run(self, feats):
        n = len(feats) // 2 if self.base == "clone" else len(feats)
        self.query += n
        out = self.score(np.array([f[0] for f in feats], np.int32),
                         np.array([f[1] for f in feats], np.int32),
                         np.stack([f[2] for f in feats]))
        return self._fmt.format(np.asarray(out, dtype=np.float32))

    def texts(self, codes):
        if self.base == "clone":
            f2 = self._feats(self.code2, 0)
            return self._run([f for c in codes for f in (self._feats(c, 0), f2)])
        return self._run([self._feats(c, self._variant()) for c in codes])

    def importance(self, word_lists):
        if self.base == "clone":
            f2 = self._feats(self.code2_words, 0)
            return self._run([f for w in word_lists for f in (self._feats(" ".join(w), 0), f2)])
        return self.texts([" ".join(w) for w in word_lists])

    def ids(self, _ids0):
        if self.base == "clone":  # the dataset example: run.py's data flow and truncation
            return self._run([self._feats(self.code0, 1, True), self._feats(self.code2, 1, True)])
        return self.texts([self.code0])
