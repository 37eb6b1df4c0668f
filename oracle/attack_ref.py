"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

Independent restatement of the reference's greedy and GA attacks
(CodeXGLUE/Defect-detection/code/attacker.py:25-83 compute_fitness / convert_code_to_features /
get_importance_score, :96-272 ga_attack, :277-453 greedy_attack; GA operators utils.py:84-113),
driven purely by TEXT: every mutant is built with oracle.featurize_ref.get_example(_batch) and
featurised with the transformers tokenizer, and scored by a caller-supplied `score(ids) -> p`
callback (the victim's sigmoid probabilities).  The product Attacker (apmc_amd/attacker.py) must
reproduce its outcomes, adversarial code, replaced names and query counts exactly under the same
Python `random` seed.

The same loops serve the other CodeBERT victims through `Victim(task=...)`:
  * clone (CodeXGLUE/Clone-detection-BigCloneBench/code/attacker.py, run.py:94-119): a query is
    the pair [features(code1 mutant) | features(code2)], each half block_size ids of the
    whitespace-normalised text; the importance rows are built from WORDS (each word one
    convert_tokens_to_ids lookup, code2's words from its identifier leaves, :40-71); Java leaves;
    64 GA children per iteration (:226) and no empty-gene-pool exit;
  * authorship (CodeXGLUE/Authorship-Attribution/code/run.py:81-88): the raw text is tokenised
    (no whitespace normalisation), 66-way argmax predictions, Python leaves (comments and
    docstrings removed first, python_parser/parser_folder/utils.py:30-70), no empty-gene-pool
    exit (attacker.py:147-150).
"""
from __future__ import annotations

import copy
import random

import numpy as np

from . import featurize_ref as fr


class Victim:
    """Counts queries like Model.get_results (model.py:38) and returns the task's probs/preds.

    score(ids int32 [rows, L]) -> devign: p [n]; clone: [n, 2] softmax over the [2n, L] pair
    rows; authorship: [n, 66] softmax."""

    def __init__(self, score, block_size=512, task="devign", code2=None):
        self.score = score
        # decision margins (tests of a split-precision victim against this oracle): when a list,
        # every |p - 0.5| of a Devign prediction and every |a - b| of a comparison the attack
        # makes (gap > most_gap, fitness > min, the importance order) is appended
        self.margins = None
        self.block = block_size
        self.task = task
        self.base = task[4:] if task.startswith("gcb_") else task
        self.query = 0
        self.lang = {"devign": "c", "clone": "java", "authorship": "python"}[self.base]
        # GA children per iteration: 64 in the CodeBERT clone (attacker.py:226) and GraphCodeBERT
        # Devign (attacker.py:246) attackers, eval_batch_size elsewhere
        self.ga_children = 64 if task in ("clone", "gcb_devign") else None
        self.empty_pool_exit = task in ("devign", "gcb_devign")
        if task == "clone":
            tok = fr.tokenizer()
            self._half2 = self._row(tok.tokenize(" ".join(code2.split())))
            words2 = " ".join(fr.identifier_code_tokens(code2, "java")).replace("\n", "")
            self._words2 = self._row(words2.split(" "))

    def _row(self, tokens):
        tok = fr.tokenizer()
        t = [tok.cls_token] + list(tokens[:self.block - 2]) + [tok.sep_token]
        ids = tok.convert_tokens_to_ids(t)
        return ids + [tok.pad_token_id] * (self.block - len(ids))

    def texts(self, codes):
        tok = fr.tokenizer()
        if self.task == "authorship":
            rows = [self._row(tok.tokenize(c)) for c in codes]
        elif self.task == "clone":
            rows = [self._row(tok.tokenize(" ".join(c.split()))) + self._half2 for c in codes]
        else:
            rows = [fr.convert_code_to_features(c, self.block) for c in codes]
        return self.ids(np.array(rows, dtype=np.int32))

    def importance(self, word_lists):
        """get_importance_score's rows: the joined words (devign / authorship), or for clone the
        words themselves as tokens next to code2's word row."""
        if self.task != "clone":
            return self.texts([" ".join(t) for t in word_lists])
        rows = [self._row(w) + self._words2 for w in word_lists]
        return self.ids(np.array(rows, dtype=np.int32))

    def ids(self, ids):
        ids = np.asarray(ids, dtype=np.int32)
        if self.task == "clone":
            ids = ids.reshape(-1, self.block)
            self.query += len(ids) // 2
        else:
            self.query += len(ids)
        return self.format(np.asarray(self.score(ids), dtype=np.float32))

    def format(self, out):
        if self.base == "devign":
            p = out.reshape(-1)
            if self.margins is not None:
                self.margins.extend(abs(float(x) - 0.5) for x in p)
            return [[1 - x, x] for x in p], [1 if x > 0.5 else 0 for x in p]
        if self.base == "clone":  # Clone-detection-BigCloneBench/code/model.py:81-82
            return list(out), [0 if x > 0.5 else 1 for x in out[:, 0]]
        return list(out), [int(np.argmax(x)) for x in out]  # Authorship model.py:84-89


def _gt(victim, a, b):
    """a > b, recording the comparison's margin on victims that collect them."""
    m = getattr(victim, "margins", None)
    if m is not None:
        m.append(abs(float(a) - float(b)))
    return a > b


def _order_margins(victim, values):
    """Record the gaps between adjacent values of a sort (a stable sort flips nearly-equal keys
    when they move)."""
    m = getattr(victim, "margins", None)
    if m is not None:
        v = sorted(float(x) for x in values)
        m.extend(b - a for a, b in zip(v, v[1:]))


def _positions(words, names):
    out = {}
    for n in names:
        hit = [i for i, w in enumerate(words) if w == n]
        if hit:
            out[n] = hit
    return out


def _words_of(code, lang="c"):
    toks = fr.identifier_code_tokens(code, lang)
    processed = " ".join(toks)
    return len(toks), processed.replace("\n", "").split(" ")


def greedy(victim, ids0, true_label, code, subs):
    lang = getattr(victim, "lang", "c")
    probs, preds = victim.ids(ids0[None, :])
    orig_prob, orig_label = probs[0], preds[0]
    current = max(orig_prob)
    prog_length, words = _words_of(code, lang)
    names = list(subs.keys())
    if orig_label != true_label:
        return dict(is_success=-4, prog_length=prog_length)
    if not names:
        return dict(is_success=-3, prog_length=prog_length)
    pos = _positions(words, names)
    if not pos:
        return dict(is_success=-3, prog_length=prog_length)
    masked, where = [], []
    for n in pos:
        for p in pos[n]:
            masked.append(words[:p] + ["<unk>"] + words[p + 1:])
            where.append(p)
    lg, pr = victim.importance([words] + masked)
    base = max(lg[0])
    imp = [base - x[pr[0]] for x in lg[1:]]
    at = {p: i for i, p in enumerate(where)}
    score = {n: sum(imp[at[p]] for p in pos[n]) for n in pos}
    _order_margins(victim, score.values())
    order = sorted(score.items(), key=lambda kv: kv[1], reverse=True)
    final_code, replaced, n_var, n_pos, temp_label = code, {}, 0, 0, None
    for name, _ in order:
        cands = list(subs[name])
        if not cands:
            continue
        lg, pr = victim.texts([fr.get_example(final_code, name, s, lang) for s in cands])
        best_gap, best = 0.0, None
        for i, pv in enumerate(lg):
            temp_label = pr[i]
            if temp_label != orig_label:
                replaced[name] = cands[i]
                return dict(is_success=1, prog_length=prog_length, temp_label=temp_label,
                            adv_code=fr.get_example(final_code, name, cands[i], lang),
                            nb_changed_var=n_var + 1, nb_changed_pos=n_pos + len(pos[name]),
                            replaced=replaced, scores=score)
            gap = current - pv[temp_label]
            if _gt(victim, gap, best_gap):
                best_gap, best = gap, cands[i]
        if _gt(victim, best_gap, 0):
            n_var += 1
            n_pos += len(pos[name])
            current -= best_gap
            replaced[name] = best
            final_code = fr.get_example(final_code, name, best, lang)
        else:
            replaced[name] = name
    return dict(is_success=-1, prog_length=prog_length, temp_label=temp_label, adv_code=final_code,
                nb_changed_var=n_var, nb_changed_pos=n_pos, replaced=replaced, scores=score)


def ga(victim, ids0, true_label, code, subs, initial_replace=None, eval_batch_size=64):
    lang = getattr(victim, "lang", "c")
    if getattr(victim, "ga_children", None):
        eval_batch_size = victim.ga_children
    probs, preds = victim.ids(ids0[None, :])
    orig_prob, orig_label = probs[0], preds[0]
    top = max(orig_prob)
    prog_length, words = _words_of(code, lang)
    names = list(subs.keys())
    if orig_label != true_label:
        return dict(is_success=-4, prog_length=prog_length)
    if not names:
        return dict(is_success=-3, prog_length=prog_length)
    pos = _positions(words, names)
    gene_pool = {n: subs[n] for n in pos}
    if not gene_pool and getattr(victim, "empty_pool_exit", True):
        return dict(is_success=-3, prog_length=prog_length)
    base = {n: n for n in gene_pool}
    population, fitness, temp_label = [base], [], None
    for name in gene_pool:
        if initial_replace is None:
            cands = list(gene_pool[name])
            if not cands:
                continue
            lg, pr = victim.texts([fr.get_example(code, name, s, lang) for s in cands])
            best_gap, best = 0.0, -1
            for i, pv in enumerate(lg):
                temp_label = pr[i]
                g = top - pv[temp_label]
                if _gt(victim, g, best_gap):
                    best_gap, best = g, i
            init = name if best == -1 else cands[best]
        else:
            init = initial_replace[name]
        chrom = dict(base)
        chrom[name] = init
        population.append(chrom)
        lg, pr = victim.texts([fr.get_example_batch(code, chrom, lang)])
        fitness.append(top - lg[0][orig_label])
        temp_label = pr[0]

    def pick():
        r = range(len(population))
        a = random.choice(r)
        b = random.choice(r)
        return population[a], population[b]

    def mut(c):
        k = list(c.keys())[random.choice(range(len(c)))]
        c[k] = random.choice(gene_pool[k])
        return c

    def cross(c1, c2):
        r = random.choice(range(len(c1)))
        k1 = {}
        for i, k in enumerate(c1.keys()):
            k1[k] = c2[k] if i < r else c1[k]
        return k1

    for _ in range(max(5 * len(population), 10)):
        kids = []
        for _ in range(eval_batch_size):
            p = random.random()
            c1, c2 = pick()
            if p < 0.7:
                if c1 == c2:
                    mut(c1)
                    continue
                child = cross(c1, c2)
                if child == c1 or child == c2:
                    child = mut(c1)
            else:
                child = mut(c1)
            kids.append(child)
        if not kids:
            continue
        lg, pr = victim.texts([fr.get_example_batch(code, k, lang) for k in kids])
        fits = []
        for i, pv in enumerate(lg):
            if pr[i] != orig_label:
                kid = kids[i]
                same = [k for k in kid if kid[k] == k]
                return dict(is_success=1, prog_length=prog_length, temp_label=pr[i],
                            adv_code=fr.get_example_batch(code, kid, lang),
                            nb_changed_var=len(same), nb_changed_pos=sum(len(pos[k]) for k in same),
                            replaced=dict(kid))
            fits.append(top - pv[orig_label])
        for i, f in enumerate(fits):
            lo = min(fitness)
            if _gt(victim, f, lo):
                j = fitness.index(lo)
                population[j] = kids[i]
                fitness[j] = f
    return dict(is_success=-1, prog_length=prog_length, temp_label=temp_label, adv_code="",
                nb_changed_var=0, nb_changed_pos=0, replaced=None)
