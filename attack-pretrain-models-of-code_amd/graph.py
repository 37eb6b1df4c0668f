"""GraphCodeBERT victims: data-flow featurisation, the graph-guided attention mask, and the drop-in
`Model` whose forward averages data-flow node embeddings (ae_score_graph).

Mirrors:
  convert_code_to_features (GCB)   GraphCodeBERT/Defect-detection/code/attacker.py:30-63,
                                   GraphCodeBERT/Authorship-Attribution/code/attacker.py:52-88
  pair features (clone)            GraphCodeBERT/clonedetection/code/attacker.py:33-72; the
                                   original example: clonedetection/code/run.py:148-192
  GraphCodeDataset / CodePairDataset  utils.py:540-639
  Model.forward / get_results      GraphCodeBERT/Defect-detection/code/model.py:24-60,
                                   GraphCodeBERT/clonedetection/code/model.py:41-85
  extract_dataflow                 python_parser/run_parser.py:190-216 (variant DFG_RUN_PARSER) and
                                   GraphCodeBERT/*/code/run.py:72-109 (DFG_GCB_RUN: parser/DFG.py
                                   walk + edge filter) — both in csrc/host/dfg*.cpp

Which builder, language and whitespace handling each GraphCodeBERT victim uses (TASK_FEATURES):
  devign      C,      ' '.join(code.split()), run_parser      (attacker.py:30-32, run.py:89-92)
  clone       Java,   text as is,             run_parser for attack-time mutants; the original
                                              pair from run.py (DFG_GCB_RUN, truncation -3 and
                                              at most 509 code tokens)
  authorship  Python, text as is,             DFG_GCB_RUN for every query (attacker.py imports
                                              run.extract_dataflow)

The reference builds a bool [L, L] mask per query in Python loops and ships it to the GPU as
L*L bytes.  The attack-time queries here go through the C++ batch featuriser
(Tokenizer.gcb_features: worker threads, one tokenizer clone each) which leaves the mask compact
(per query: node_index, max_length, node code spans, node->node edges, ~4 KB instead of 400 KB),
and the device builds the bit-packed mask (uint32 [L, L/32], bit j of word w = key 32*w + j) that
the attention kernel reads (ae_graph_mask).  The numpy builder below (graph_mask / pack_mask)
remains for the dataset example and as the reference the device path is tested against.
"""
from __future__ import annotations

import numpy as np

from .host import DFG_GCB_RUN, DFG_RUN_PARSER, Example
from .model import Model, Payload

DFG_REL = ("comesFrom", "computedFrom")
# task -> (language, normalise whitespace, data-flow builder of the attack-time queries)
TASK_FEATURES = {"devign": ("c", True, DFG_RUN_PARSER), "clone": ("java", False, DFG_RUN_PARSER),
                 "authorship": ("python", False, DFG_GCB_RUN)}


class GraphInputFeatures:
    """GraphCodeBERT/Defect-detection/code/run.py InputFeatures (input_tokens, input_ids,
    position_idx, dfg_to_code, dfg_to_dfg, idx, label)."""

    def __init__(self, input_tokens, input_ids, position_idx, dfg_to_code, dfg_to_dfg, idx, label):
        self.input_tokens = input_tokens
        self.input_ids = input_ids
        self.position_idx = position_idx
        self.dfg_to_code = dfg_to_code
        self.dfg_to_dfg = dfg_to_dfg
        self.idx = str(idx)
        self.label = label


def extract_dataflow(code: str, lang: str = "c", variant: int = DFG_RUN_PARSER):
    """run_parser.py:190-216 -> (DFG sorted by leaf index, index_table, code_tokens).  DFG entries
    are (code, idx, relation, [from names], [from idx]) as DFG_c / DFG_java / DFG_python build
    them; index_table is not reproduced (no caller on the query path reads it) and is returned
    as None.  variant=DFG_GCB_RUN: GraphCodeBERT run.py's builder (parser/DFG.py + edge filter)."""
    ex = Example(code, lang)
    toks = ex.leaves(identifiers=True)
    dfg = [(toks[i], i, DFG_REL[int(comp)], [toks[j] for j in fr], fr)
           for i, comp, fr in ex.dfg(variant)]
    return dfg, None, toks


class _LeafIds:
    """Per-tokenizer cache of `tokenize('@ ' + leaf)[1:]` ids (attacker.py:35): leaf strings repeat
    heavily across a mutant population, so each distinct leaf is tokenised once."""

    def __init__(self, tok):
        self.tok = tok
        self.first: dict[str, list[int]] = {}
        self.rest: dict[str, list[int]] = {}

    def __call__(self, leaf: str, first: bool) -> list[int]:
        d = self.first if first else self.rest
        r = d.get(leaf)
        if r is None:
            r = self.tok.encode_ids(leaf) if first else self.tok.encode_ids("@ " + leaf)[1:]
            d[leaf] = r
        return r


def _leaf_ids(tokenizer):
    c = getattr(tokenizer, "_apmc_leaf_ids", None)
    if c is None:
        c = _LeafIds(tokenizer)
        tokenizer._apmc_leaf_ids = c
    return c


def convert_code_to_features(code, tokenizer, label, args, lang: str = "c", normalize: bool = True,
                             variant: int = DFG_RUN_PARSER, run_trunc: bool = False):
    """GraphCodeBERT/Defect-detection/code/attacker.py:30-63 (code_length + data_flow_length
    row; DFG nodes appended as <unk> ids at position 0; pads at position pad_id).  normalize:
    ' '.join(code.split()) first (Devign only); run_trunc: clonedetection/code/run.py:166's
    truncation (one token fewer, at most 509 code tokens)."""
    if normalize:
        code = " ".join(code.split())
    dfg, _, code_tokens = extract_dataflow(code, lang, variant)
    leaf = _leaf_ids(tokenizer)
    runs = [leaf(x, idx == 0) for idx, x in enumerate(code_tokens)]
    ends = np.cumsum([0] + [len(r) for r in runs])  # ori2cur_pos[i] = (ends[i], ends[i+1])
    flat = [y for r in runs for y in r]
    total = args.code_length + args.data_flow_length
    if run_trunc:
        flat = flat[:total - 3 - min(len(dfg), args.data_flow_length)][:512 - 3]
    else:
        flat = flat[:total - 2 - min(len(dfg), args.data_flow_length)]
    pad, cls, sep, unk = (tokenizer.pad_token_id, tokenizer.cls_token_id, tokenizer.sep_token_id,
                          tokenizer.unk_token_id)
    source_ids = [cls] + flat + [sep]
    position_idx = list(range(pad + 1, pad + 1 + len(source_ids)))
    dfg = dfg[:total - len(source_ids)]
    source_ids += [unk] * len(dfg)
    position_idx += [0] * len(dfg)
    padding = total - len(source_ids)
    position_idx += [pad] * padding
    source_ids += [pad] * padding
    reverse_index = {x[1]: i for i, x in enumerate(dfg)}
    dfg_to_dfg = [[reverse_index[i] for i in x[-1] if i in reverse_index] for x in dfg]
    dfg_to_code = [(int(ends[x[1]]) + 1, int(ends[x[1] + 1]) + 1) for x in dfg]
    # input_tokens (strings) are not read by any query-path consumer
    return GraphInputFeatures(None, source_ids, position_idx, dfg_to_code, dfg_to_dfg, 0, label)


def task_features(code, tokenizer, label, args, task: str, **kw):
    """convert_code_to_features with the language / whitespace / builder of a task's attacker."""
    lang, normalize, variant = TASK_FEATURES[task]
    kw.setdefault("variant", variant)
    return convert_code_to_features(code, tokenizer, label, args, lang, normalize, **kw)


def pair_features(code1, code2, tokenizer, label, args, original: bool = False):
    """One clone query: GraphPairFeatures of (code1, code2).  original=True builds them as
    clonedetection/code/run.py does for the dataset example (DFG_GCB_RUN, run.py truncation);
    otherwise as attacker.py:33-72 does for every mutant (run_parser builder)."""
    kw = dict(variant=DFG_GCB_RUN, run_trunc=True) if original else {}
    f1 = task_features(code1, tokenizer, label, args, "clone", **kw)
    f2 = task_features(code2, tokenizer, label, args, "clone", **kw)
    return GraphPairFeatures(f1, f2, label)


def graph_mask(input_ids, position_idx, dfg_to_code, dfg_to_dfg, L: int | None = None) -> np.ndarray:
    """GraphCodeDataset.__getitem__'s graph-guided mask (utils.py:547-570) as bool [L, L]."""
    pos = np.asarray(position_idx)
    ids = np.asarray(input_ids)
    L = L or len(pos)
    m = np.zeros((L, L), dtype=bool)
    node_index = int((pos > 1).sum())
    max_length = int((pos != 1).sum())
    m[:node_index, :node_index] = True  # sequence attends to sequence
    m[np.nonzero((ids == 0) | (ids == 2))[0], :max_length] = True  # special tokens attend to all
    for idx, (a, b) in enumerate(dfg_to_code):  # nodes <-> the code tokens they come from
        if a < node_index and b < node_index:
            m[idx + node_index, a:b] = True
            m[a:b, idx + node_index] = True
    n_pos = len(pos)
    for idx, nodes in enumerate(dfg_to_dfg):  # nodes attend to adjacent nodes
        cols = [a + node_index for a in nodes if a + node_index < n_pos]
        if cols:
            m[idx + node_index, cols] = True
    return m


def pack_mask(m: np.ndarray) -> np.ndarray:
    """bool [..., L, L] -> int32 [..., L, L/32] (bit j of word w = key 32*w + j)."""
    L = m.shape[-1]
    if L % 32:
        raise ValueError(f"mask width {L} is not a multiple of 32")
    return np.packbits(m, axis=-1, bitorder="little").view("<i4")


class GraphCodeDataset:
    """utils.py:540-576.  Items are the reference's (ids, attn_mask bool [L,L], pos, label)
    tensors; `packed()` is the engine's fast path (no bool mask materialised per query)."""

    def __init__(self, examples, args=None):
        self.examples = examples
        self.args = args

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, item):
        import torch

        f = self.examples[item]
        m = graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg)
        return (torch.tensor(f.input_ids), torch.tensor(m), torch.tensor(f.position_idx),
                torch.tensor(f.label))

    def packed(self):
        """-> ids int32 [n, L], pos int32 [n, L], mask bits int32 [n, L, L/32]."""
        ids = np.asarray([f.input_ids for f in self.examples], dtype=np.int32)
        pos = np.asarray([f.position_idx for f in self.examples], dtype=np.int32)
        bits = np.stack([pack_mask(graph_mask(f.input_ids, f.position_idx, f.dfg_to_code,
                                              f.dfg_to_dfg)) for f in self.examples])
        return ids, pos, bits


def compact_features(f, e_cap: int | None = None) -> dict:
    """One GraphInputFeatures -> the compact arrays of Tokenizer.gcb_features ([1, ...] each)."""
    ids = np.asarray(f.input_ids, dtype=np.int32)
    pos = np.asarray(f.position_idx, dtype=np.int32)
    L = len(ids)
    e_cap = e_cap or 4 * L
    ni, nn = int((pos > 1).sum()), len(f.dfg_to_code)
    spans = np.full((L,), -1, np.int32)
    for k, (a, b) in enumerate(f.dfg_to_code):
        if a < ni and b < ni:
            spans[k] = a | (b << 16)
    edges = [k | (t << 16) for k, ts in enumerate(f.dfg_to_dfg) for t in ts if ni + t < L]
    e = np.zeros((max(e_cap, len(edges)),), np.int32)
    e[:len(edges)] = edges
    meta = np.asarray([ni, int((pos != 1).sum()), nn, len(edges)], np.int32)
    return {"ids": ids[None], "pos": pos[None], "meta": meta[None], "spans": spans[None],
            "edges": e[None]}


def graph_mask_from_compact(ids, meta, spans, edges) -> np.ndarray:
    """bool [L, L] from one query's compact arrays (what ae_graph_mask builds on the device)."""
    L = len(ids)
    ni, ml, nn, ne = (int(x) for x in meta)
    m = np.zeros((L, L), dtype=bool)
    m[:ni, :ni] = True
    m[np.nonzero((ids == 0) | (ids == 2))[0], :ml] = True
    for k in range(nn):
        sp = int(spans[k])
        if sp >= 0:
            a, b = sp & 0xFFFF, sp >> 16
            m[ni + k, a:b] = True
            m[a:b, ni + k] = True
    for e in edges[:ne]:
        k, t = int(e) & 0xFFFF, int(e) >> 16
        if ni + t < L:
            m[ni + k, ni + t] = True
    return m


def _pad_edges(arrays):
    """Edge arrays of one width (zero-padded; meta[:, 3] says how many are real)."""
    w = max(a.shape[1] for a in arrays)
    return [a if a.shape[1] == w else np.pad(a, ((0, 0), (0, w - a.shape[1]))) for a in arrays]


def _cat_compact(parts):
    out = {k: np.concatenate([p[k] for p in parts]) for k in parts[0] if k != "edges"}
    out["edges"] = np.concatenate(_pad_edges([p["edges"] for p in parts]))
    return out


class CompactGraphDataset:
    """Queries featurised by Tokenizer.gcb_features: the arrays stay compact until the device
    builds the mask.  pairs=True: rows interleaved code1, code2 (len = rows / 2).  Indexing and
    packed() rebuild the reference's tuples / bits on the host (compatibility, tests)."""

    def __init__(self, arrays: dict, labels=None, pairs: bool = False):
        self.c = arrays
        self.pairs = pairs
        rows = len(arrays["ids"])
        self.n = rows // 2 if pairs else rows
        self.labels = list(labels) if labels is not None else [0] * self.n

    def __len__(self):
        return self.n

    def _row(self, r):
        c = self.c
        m = graph_mask_from_compact(c["ids"][r], c["meta"][r], c["spans"][r], c["edges"][r])
        return c["ids"][r], c["pos"][r], m

    def __getitem__(self, item):
        import torch

        if self.pairs:
            out = []
            for r in (2 * item, 2 * item + 1):
                ids, pos, m = self._row(r)
                out += [torch.tensor(ids), torch.tensor(pos), torch.tensor(m)]
            return tuple(out) + (torch.tensor(self.labels[item]),)
        ids, pos, m = self._row(item)
        return (torch.tensor(ids), torch.tensor(m), torch.tensor(pos),
                torch.tensor(self.labels[item]))

    def packed(self):
        rows = len(self.c["ids"])
        bits = np.stack([pack_mask(self._row(r)[2]) for r in range(rows)])
        return self.c["ids"], self.c["pos"], bits


def payload_rows_host(live):
    """(ids, pos, mask bits) numpy arrays of every row of GraphModel payloads, the compact ones'
    masks built on the host (graph_mask_from_compact) — for victims without an engine."""
    ids, pos, bits = [], [], []
    for p in live:
        ids.append(p.ids)
        if p.extra[0] == "bits":
            pos.append(p.extra[1])
            bits.append(p.extra[2])
        else:
            c = p.extra[1]
            pos.append(c["pos"])
            bits.append(np.stack([pack_mask(graph_mask_from_compact(c["ids"][r], c["meta"][r],
                                                                    c["spans"][r], c["edges"][r]))
                                  for r in range(len(c["ids"]))]))
    return np.concatenate(ids), np.concatenate(pos), np.concatenate(bits)


def gcb_dataset_from_texts(texts, tokenizer, args, task: str, label=0):
    """The task's convert_code_to_features of many query texts through the batch featuriser."""
    lang, normalize, variant = TASK_FEATURES[task]
    c = tokenizer.gcb_features(list(texts), lang, variant, normalize, args.code_length,
                               args.data_flow_length)
    return CompactGraphDataset(c, [label] * len(texts))


def compact_pairs(c1: dict, c2_one: dict) -> CompactGraphDataset:
    """Clone queries: rows of c1 (mutated code1) each paired with the single code2 query c2_one,
    rows interleaved code1, code2 (clonedetection/code/model.py:42-45)."""
    n = len(c1["ids"])
    out = {}
    for k in c1:
        a, b = c1[k], np.repeat(c2_one[k], n, axis=0)
        if k == "edges":
            a, b = _pad_edges([a, b])
        if a.shape[1:] != b.shape[1:]:
            raise ValueError(f"pair feature widths differ for {k}")
        out[k] = np.stack([a, b], 1).reshape((2 * n,) + a.shape[1:])
    return CompactGraphDataset(out, pairs=True)


class GraphPairFeatures:
    """GraphCodeBERT/clonedetection/code/run.py InputFeatures of a pair (field suffixes _1/_2)."""

    def __init__(self, f1: GraphInputFeatures, f2: GraphInputFeatures, label, url1="", url2=""):
        for k in ("input_tokens", "input_ids", "position_idx", "dfg_to_code", "dfg_to_dfg"):
            setattr(self, k + "_1", getattr(f1, k))
            setattr(self, k + "_2", getattr(f2, k))
        self.label = label
        self.url1, self.url2 = url1, url2


class CodePairDataset:
    """utils.py:578-639 — items (ids1, pos1, mask1, ids2, pos2, mask2, label)."""

    def __init__(self, examples, args=None):
        self.examples = examples
        self.args = args

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, item):
        import torch

        f = self.examples[item]
        out = []
        for s in ("_1", "_2"):
            ids, pos = getattr(f, "input_ids" + s), getattr(f, "position_idx" + s)
            m = graph_mask(ids, pos, getattr(f, "dfg_to_code" + s), getattr(f, "dfg_to_dfg" + s))
            out += [torch.tensor(ids), torch.tensor(pos), torch.tensor(m)]
        return tuple(out) + (torch.tensor(f.label),)

    def packed(self):
        """Rows interleaved code1, code2 per pair (clonedetection/code/model.py:42-45)."""
        ids, pos, bits = [], [], []
        for f in self.examples:
            for s in ("_1", "_2"):
                i, p = getattr(f, "input_ids" + s), getattr(f, "position_idx" + s)
                ids.append(i)
                pos.append(p)
                bits.append(pack_mask(graph_mask(i, p, getattr(f, "dfg_to_code" + s),
                                                 getattr(f, "dfg_to_dfg" + s))))
        return (np.asarray(ids, dtype=np.int32), np.asarray(pos, dtype=np.int32),
                np.stack(bits))


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _pack_items(dataset, pair: bool):
    """Generic dataset of the reference's tuples -> packed arrays (rows interleaved for pairs)."""
    ids, pos, bits = [], [], []
    for i in range(len(dataset)):
        it = dataset[i]
        groups = [(it[0], it[1], it[2]), (it[3], it[4], it[5])] if pair else \
            [(it[0], it[2], it[1])]  # (ids, mask, pos, label) -> (ids, pos, mask)
        for a, p, m in groups:
            ids.append(_np(a).reshape(-1))
            pos.append(_np(p).reshape(-1))
            bits.append(pack_mask(_np(m).astype(bool)))
    return (np.asarray(ids, dtype=np.int32), np.asarray(pos, dtype=np.int32), np.stack(bits))


class GraphModel(Model):
    """GraphCodeBERT victim: task "devign" (sigmoid head, GraphCodeBERT/Defect-detection),
    "clone" (pair head over interleaved code1/code2 rows, GraphCodeBERT/clonedetection) or
    "authorship" (66-way softmax, GraphCodeBERT/Authorship-Attribution/code/model.py:29-60)."""

    # mutant rows are data-flow features, never spliced token ids (MHM_Attacker checks this)
    population_rows = None

    def __init__(self, encoder, config=None, tokenizer=None, args=None, task: str = "devign",
                 precision: str = "fp32", device: int = 0):
        super().__init__(encoder, config, tokenizer, args, task=task, precision=precision,
                         device=device)

    def score_packed(self, ids: np.ndarray, pos: np.ndarray, bits: np.ndarray) -> np.ndarray:
        import torch

        n, L = ids.shape
        if bits.shape != (n, L, L // 32) or pos.shape != (n, L):
            raise ValueError(f"graph inputs disagree: ids {ids.shape} pos {pos.shape} "
                             f"mask bits {bits.shape}")
        outs = []
        dev = f"cuda:{self.engine.device}"
        step = self.max_rows_per_launch
        for s in range(0, n, step):
            e = min(n, s + step)
            # every column takes part (pads too): a fully masked query row attends all L keys
            # uniformly under HF's finfo.min additive mask (alert_engine.h ae_score_graph)
            lens = np.full((e - s,), L, dtype=np.int32)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a[s:e])).to(dev)  # noqa: E731
            outs.append(self.engine.score_graph(t(ids), lens, t(pos), t(bits)))
        return torch.cat(outs, 0).cpu().numpy() if len(outs) > 1 else outs[0].cpu().numpy()

    def prepare(self, dataset) -> Payload:
        """(probs, pred_labels) request of GraphCodeBERT/*/code/model.py get_results: packed
        ids / positions / mask bits (rows interleaved code1, code2 for clone pairs), or the compact
        arrays of a CompactGraphDataset (mask built on the device)."""
        n = len(dataset)
        if n == 0:
            return Payload(None, None, 0)
        if isinstance(dataset, CompactGraphDataset):
            return Payload(dataset.c["ids"], None, n, ("compact", dataset.c))
        if hasattr(dataset, "packed"):
            ids, pos, bits = dataset.packed()
        else:
            ids, pos, bits = _pack_items(dataset, self.task == "clone")
        return Payload(ids, None, n, ("bits", pos, bits))

    def _bits_rows(self, p, dev):
        """Device mask bits of one payload's rows."""
        import torch

        from .model import to_device

        kind = p.extra[0]
        if kind == "bits":
            return to_device(p.extra[2], dev)
        c = p.extra[1]
        t = lambda a: to_device(a, dev)  # noqa: E731
        return self.engine.graph_mask(t(c["ids"]), t(c["meta"]), t(c["spans"]), t(c["edges"]))

    def score_payload_rows(self, live):
        """Logits of every row of the live payloads (device mask build for compact ones)."""
        return self._score_payload_rows_dev(live).cpu().numpy()

    def _score_payload_rows_dev(self, live):
        import torch

        dev = f"cuda:{self.engine.device}"
        ids = np.concatenate([p.ids for p in live])
        pos = np.concatenate([p.extra[1]["pos"] if p.extra[0] == "compact" else p.extra[1]
                              for p in live])
        n, L = ids.shape
        step = self.max_rows_per_launch
        outs, off, pi = [], 0, 0
        bits_parts = []
        for p in live:
            bits_parts.append(self._bits_rows(p, dev))
        bits = torch.cat(bits_parts, 0) if len(bits_parts) > 1 else bits_parts[0]
        from .model import to_device

        ids_d = to_device(ids, dev)
        pos_d = to_device(pos, dev)
        for s0 in range(0, n, step):
            e = min(n, s0 + step)
            lens = np.full((e - s0,), L, dtype=np.int32)
            outs.append(self.engine.score_graph(ids_d[s0:e], lens, pos_d[s0:e], bits[s0:e]))
        return torch.cat(outs, 0) if len(outs) > 1 else outs[0]

    def prepare_population(self, example, tokenizer, population, mode: int, block_size: int):
        """A population of chromosomes of one program: mutant texts (host get_example(_batch))
        -> data-flow features (len(population) queries)."""
        texts = [example.mutant_text(pairs, mode) for pairs in population]
        return self.prepare(self.dataset_from_texts(texts, tokenizer, self.args))

    def score_prepared(self, payloads, threshold: float = 0.5):
        self.query += sum(p.n for p in payloads)
        live = [p for p in payloads if p.n]
        if not live:
            return [([], []) for _ in payloads]
        logits = self.score_payload_rows(live)
        out, off = [], 0
        for p in payloads:
            out.append(self._format(logits[off:off + p.n], threshold) if p.n else ([], []))
            off += p.n
        return out

    def submit(self, payloads, threshold: float = 0.5):
        """score_prepared split in two (Model.submit): the batch is queued now, .result()
        answers it."""
        from .model import PendingScores, ScoresReady

        self.query += sum(p.n for p in payloads)
        live = [p for p in payloads if p.n]
        if not live:
            return ScoresReady([([], []) for _ in payloads])
        return PendingScores(self._score_payload_rows_dev(live), payloads, self._format,
                             threshold)

    def dataset_from_texts(self, texts, tokenizer, args, label=0):
        """Mutant texts -> the GCB attacker's convert_code_to_features of each
        (GraphCodeBERT/Defect-detection/code/attacker.py:30-63) with the task's language and
        builder, through the batch featuriser (compact mask).  Clone pairs are built by
        GraphCloneAttacker."""
        if self.task == "clone":
            raise ValueError("clone queries are pairs: build them with pair_features")
        if not hasattr(tokenizer, "gcb_features"):
            return GraphCodeDataset([task_features(t, tokenizer, label, args, self.task)
                                     for t in texts], args)
        return gcb_dataset_from_texts(texts, tokenizer, args, self.task, label)

    def prepare_pair_population(self, feats1, f2) -> Payload:
        """Clone queries of mutated code1 features against one fixed code2 (rows interleaved).
        feats1: a list of GraphInputFeatures, or the compact arrays of Tokenizer.gcb_features."""
        if isinstance(feats1, dict):
            c2 = f2 if isinstance(f2, dict) else compact_features(f2, feats1["edges"].shape[1])
            return self.prepare(compact_pairs(feats1, c2))
        return self.prepare(CodePairDataset([GraphPairFeatures(f, f2, 0) for f in feats1]))
