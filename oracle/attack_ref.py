"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

Independent restatement of the reference's greedy and GA attacks
(CodeXGLUE/Defect-detection/code/attacker.py:25-83 compute_fitness / convert_code_to_features /
get_importance_score, :96-272 ga_attack, :277-453 greedy_attack; GA operators utils.py:84-113),
driven purely by TEXT: every mutant is built with oracle.featurize_ref.get_example(_batch) and
featurised with the transformers tokenizer, and scored by a caller-supplied `score(ids) -> p`
callback (the victim's sigmoid probabilities).  The product Attacker (apmc_amd/attacker.py) must
reproduce its outcomes, adversarial code, replaced names and query counts exactly under the same
Python `random` seed.
"""
from __future__ import annotations

import copy
import random

import numpy as np

from . import featurize_ref as fr


class Victim:
    """Counts queries like Model.get_results (model.py:38) and returns Devign probs/preds."""

    def __init__(self, score, block_size=512):
        self.score = score
        self.block = block_size
        self.query = 0

    def texts(self, codes):
        ids = np.array([fr.convert_code_to_features(c, self.block) for c in codes], dtype=np.int32)
        return self.ids(ids)

    def ids(self, ids):
        self.query += len(ids)
        p = np.asarray(self.score(ids), dtype=np.float32).reshape(-1)
        probs = [[1 - x, x] for x in p]
        preds = [1 if x > 0.5 else 0 for x in p]
        return probs, preds


def _positions(words, names):
    out = {}
    for n in names:
        hit = [i for i, w in enumerate(words) if w == n]
        if hit:
            out[n] = hit
    return out


def _words_of(code):
    toks = fr.identifier_code_tokens(code, "c")
    processed = " ".join(toks)
    return len(toks), processed.replace("\n", "").split(" ")


def greedy(victim, ids0, true_label, code, subs):
    probs, preds = victim.ids(ids0[None, :])
    orig_prob, orig_label = probs[0], preds[0]
    current = max(orig_prob)
    prog_length, words = _words_of(code)
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
    lg, pr = victim.texts([" ".join(t) for t in [words] + masked])
    base = max(lg[0])
    imp = [base - x[pr[0]] for x in lg[1:]]
    at = {p: i for i, p in enumerate(where)}
    score = {n: sum(imp[at[p]] for p in pos[n]) for n in pos}
    order = sorted(score.items(), key=lambda kv: kv[1], reverse=True)
    final_code, replaced, n_var, n_pos, temp_label = code, {}, 0, 0, None
    for name, _ in order:
        cands = list(subs[name])
        if not cands:
            continue
        lg, pr = victim.texts([fr.get_example(final_code, name, s, "c") for s in cands])
        best_gap, best = 0.0, None
        for i, pv in enumerate(lg):
            temp_label = pr[i]
            if temp_label != orig_label:
                replaced[name] = cands[i]
                return dict(is_success=1, prog_length=prog_length, temp_label=temp_label,
                            adv_code=fr.get_example(final_code, name, cands[i], "c"),
                            nb_changed_var=n_var + 1, nb_changed_pos=n_pos + len(pos[name]),
                            replaced=replaced, scores=score)
            gap = current - pv[temp_label]
            if gap > best_gap:
                best_gap, best = gap, cands[i]
        if best_gap > 0:
            n_var += 1
            n_pos += len(pos[name])
            current -= best_gap
            replaced[name] = best
            final_code = fr.get_example(final_code, name, best, "c")
        else:
            replaced[name] = name
    return dict(is_success=-1, prog_length=prog_length, temp_label=temp_label, adv_code=final_code,
                nb_changed_var=n_var, nb_changed_pos=n_pos, replaced=replaced, scores=score)


def ga(victim, ids0, true_label, code, subs, initial_replace=None, eval_batch_size=64):
    probs, preds = victim.ids(ids0[None, :])
    orig_prob, orig_label = probs[0], preds[0]
    top = max(orig_prob)
    prog_length, words = _words_of(code)
    names = list(subs.keys())
    if orig_label != true_label:
        return dict(is_success=-4, prog_length=prog_length)
    if not names:
        return dict(is_success=-3, prog_length=prog_length)
    pos = _positions(words, names)
    gene_pool = {n: subs[n] for n in pos}
    if not gene_pool:
        return dict(is_success=-3, prog_length=prog_length)
    base = {n: n for n in gene_pool}
    population, fitness, temp_label = [base], [], None
    for name in gene_pool:
        if initial_replace is None:
            cands = list(gene_pool[name])
            if not cands:
                continue
            lg, pr = victim.texts([fr.get_example(code, name, s, "c") for s in cands])
            best_gap, best = 0.0, -1
            for i, pv in enumerate(lg):
                temp_label = pr[i]
                g = top - pv[temp_label]
                if g > best_gap:
                    best_gap, best = g, i
            init = name if best == -1 else cands[best]
        else:
            init = initial_replace[name]
        chrom = dict(base)
        chrom[name] = init
        population.append(chrom)
        lg, pr = victim.texts([fr.get_example_batch(code, chrom, "c")])
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
        lg, pr = victim.texts([fr.get_example_batch(code, k, "c") for k in kids])
        fits = []
        for i, pv in enumerate(lg):
            if pr[i] != orig_label:
                kid = kids[i]
                same = [k for k in kid if kid[k] == k]
                return dict(is_success=1, prog_length=prog_length, temp_label=pr[i],
                            adv_code=fr.get_example_batch(code, kid, "c"),
                            nb_changed_var=len(same), nb_changed_pos=sum(len(pos[k]) for k in same),
                            replaced=dict(kid))
            fits.append(top - pv[orig_label])
        for i, f in enumerate(fits):
            lo = min(fitness)
            if f > lo:
                j = fitness.index(lo)
                population[j] = kids[i]
                fitness[j] = f
    return dict(is_success=-1, prog_length=prog_length, temp_label=temp_label, adv_code="",
                nb_changed_var=0, nb_changed_pos=0, replaced=None)
