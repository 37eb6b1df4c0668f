"""Attack drivers: the per-example loops of gi_attack.py (greedy, then GA on failure) and
mhm_attack.py (MHM-NS), over the engine, for the three CodeBERT victims:

  devign      CodeXGLUE/Defect-detection/code/gi_attack.py:154-218, mhm_attack.py:160-236
  clone       CodeXGLUE/Clone-detection-BigCloneBench/code/attack.py:160-231 (pairs; the attack
              perturbs code1; `code` = (id1, id2, code1, code2))
  authorship  CodeXGLUE/Authorship-Attribution/code/attack.py:199-266, mhm.py:160-233 (Python,
              66 authors, raw-text features; labels from valid.txt, codes from valid_subs.jsonl)
and their GraphCodeBERT counterparts (GraphModel victims, data-flow features):
  gcb_devign      GraphCodeBERT/Defect-detection/code/gi_attack.py:154-218 — with its extra
                  get_results([example]) per example (:161), one more query than the attack's
  gcb_clone       GraphCodeBERT/clonedetection/code/attack.py:170-223 (the CodeXGLUE
                  BigCloneBench pairs and substitutes; GraphCodeBERT ships none of its own)
  gcb_authorship  GraphCodeBERT/Authorship-Attribution/code/gi_attack.py:176-218

The original example's features come from the fixture (run.py of each task), substitutes from its
`substitutes`; one Recorder CSV row per example; success rate over examples the victim classified
correctly.  Also the multi-GPU form: examples are pulled from a dynamic queue shared by all ranks
(an atomic counter in the torch.distributed store; no tensor traffic) and the per-rank statistics
are all-gathered at the end.
"""
from __future__ import annotations

import dataclasses
import json
import random
import time

import numpy as np

from .attacker import (Attacker, AuthorshipAttacker, AuthorshipMHM_Attacker, CloneAttacker,
                       CloneMHM_Attacker, GraphAttacker, GraphAuthorshipAttacker,
                       GraphAuthorshipMHM_Attacker, GraphCloneAttacker, GraphCloneMHM_Attacker,
                       GraphMHM_Attacker, MHM_Attacker, get_identifiers)
from .host import Tokenizer
from .utils import Recorder, build_vocab, set_seed


@dataclasses.dataclass
class AttackArgs:
    block_size: int = 512
    eval_batch_size: int = 64
    use_ga: bool = True
    seed: int = 123456
    lang: str = "c"
    verbose: bool = False
    csv_store_path: str | None = None
    rng: str = "global"   # "global": one random stream in example order (reference);
                          # "per_example": random.seed(seed + index) before each example
    task: str = "devign"  # devign | clone | authorship (CodeBERT) | gcb_devign | gcb_clone |
                          # gcb_authorship (GraphCodeBERT)
    code_length: int = 512        # GraphCodeBERT rows: code_length + data_flow_length tokens
    data_flow_length: int = 128
    on_error: str = "raise"  # MHM chains: "raise" = the reference (its driver stops at the first
                             # exception); "record" = record is_success -5 and go on (one chain
                             # of the GraphCodeBERT clone copy can raise KeyError, see
                             # GraphCloneMHM_Attacker)


def load_fixture(path, start=0, end=None, labels_path=None):
    """codes, substitutes, labels of a test_subs / valid_subs jsonl.  Devign: `func`, `target`;
    clone: code = (id1, id2, code1, code2), `label` (Clone-detection-BigCloneBench/code/run.py:
    160-175); authorship: `code` with literal '\\n' turned into newlines (attack.py:205-211), the
    label from the `code <CODESPLIT> label` lines of `labels_path` (run.py:112-116)."""
    codes, subs, labels = [], [], []
    ext = None
    if labels_path is not None:
        ext = [int(line.split(" <CODESPLIT> ")[1]) for line in open(labels_path)]
    with open(path) as f:
        for i, line in enumerate(f):
            if i < start or (end is not None and i >= end):
                continue
            js = json.loads(line)
            if "code1" in js:
                codes.append((js.get("id1"), js.get("id2"), js["code1"], js["code2"]))
            elif "func" in js:
                codes.append(js["func"])
            else:
                codes.append(js["code"].replace("\\n", "\n"))
            subs.append(js["substitutes"])
            labels.append(ext[i] if ext is not None else int(js.get("target", js.get("label", 0))))
    return codes, subs, labels


def _example(tok, code, label, block, task="devign", args=None):
    """TextDataset item of each task: devign (ids of ' '.join(func.split()), label) (run.py:79-86);
    clone ([ids(code1) | ids(code2)], label) (Clone-detection-BigCloneBench/code/run.py:65-119);
    authorship (ids of the raw code, label) (Authorship-Attribution/code/run.py:81-89); the
    GraphCodeBERT tasks: the reference's dataset tuples of data-flow features (run.py of each)."""
    import torch

    if task.startswith("gcb_"):
        from .graph import CodePairDataset, GraphCodeDataset, pair_features, task_features

        t = task[4:]
        if t == "clone":
            return CodePairDataset([pair_features(code[2], code[3], tok, label, args,
                                                  original=True)], args)[0]
        return GraphCodeDataset([task_features(code, tok, label, args, t)], args)[0]
    if task == "clone":
        ids, _ = tok.featurize([code[2], code[3]], block)
        row = np.concatenate([ids[0], ids[1]])
    else:
        ids, _ = tok.featurize([code], block, raw=task == "authorship")
        row = ids[0]
    return torch.from_numpy(row.astype(np.int64)), torch.tensor(label)


ATTACKERS = {"devign": Attacker, "clone": CloneAttacker, "authorship": AuthorshipAttacker,
             "gcb_devign": GraphAttacker, "gcb_clone": GraphCloneAttacker,
             "gcb_authorship": GraphAuthorshipAttacker}


def make_attacker(args, model, tok):
    return ATTACKERS[getattr(args, "task", "devign")](args, model, tok, None, tok, use_bpe=1,
                                                      threshold_pred_score=0)


def _is_clone(task):
    return task in ("clone", "gcb_clone")


def attack_one(attacker, tok, code, subs, label, args):
    task = getattr(args, "task", "devign")
    example = _example(tok, code, label, args.block_size, task, args)
    if task == "gcb_devign":  # GraphCodeBERT/Defect-detection/code/gi_attack.py:161
        attacker.model_tgt.get_results([example], args.eval_batch_size)
    first = (subs, code) if _is_clone(task) else (code, subs)  # clone: (example, subs, code)
    res = attacker.greedy_attack(example, *first)
    attack_type = "Greedy"
    if res[6] == -1 and args.use_ga:
        res = attacker.ga_attack(example, *first, initial_replace=res[11])
        attack_type = "GA"
    return res, attack_type


def attack_one_gen(attacker, tok, code, subs, label, args, rng):
    """attack_one as a request generator (gi_attack.py:177-186): greedy, then GA on -1."""
    task = getattr(args, "task", "devign")
    example = _example(tok, code, label, args.block_size, task, args)
    if task == "gcb_devign":  # the driver's extra get_results([example]) (gi_attack.py:161)
        yield attacker.model_tgt.prepare([example])
    first = (subs, code) if _is_clone(task) else (code, subs)
    res = yield from attacker.greedy_gen(example, *first)
    attack_type = "Greedy"
    if res[6] == -1 and args.use_ga:
        res = yield from attacker.ga_gen(example, *first, res[11], rng)
        attack_type = "GA"
    return res, attack_type


def _record(index, res, attack_type, queries, dt_min, recorder):
    (code, prog_length, adv_code, true_label, orig_label, temp_label, is_success,
     variable_names, names_to_importance_score, nb_changed_var, nb_changed_pos,
     replaced_words) = res
    score_info = ""
    if names_to_importance_score is not None:
        for key in names_to_importance_score.keys():
            score_info += key + ":" + str(names_to_importance_score[key]) + ","
    replace_info = ""
    if replaced_words is not None:
        for key in replaced_words.keys():
            replace_info += key + ":" + replaced_words[key] + ","
    if recorder:
        recorder.write(index, code, prog_length, adv_code, true_label, orig_label, temp_label,
                       is_success, variable_names, score_info, nb_changed_var, nb_changed_pos,
                       replace_info, attack_type, queries, dt_min)
    return dict(index=index, is_success=is_success, attack_type=attack_type, queries=queries,
                adv_code=adv_code, replace_info=replace_info, nb_changed_var=nb_changed_var,
                nb_changed_pos=nb_changed_pos, prog_length=prog_length, time_s=dt_min * 60)


def _totals(records, wall):
    correct = sum(r["is_success"] >= -1 for r in records)
    succ = sum(r["is_success"] == 1 for r in records)
    return dict(records=records, examples=len(records), total_cnt=correct, success=succ,
                success_rate=(succ / correct) if correct else 0.0,
                queries=sum(r["queries"] for r in records), wall_s=wall)


class _InOrderWriter:
    """Recorder rows as examples finish, in the order they were taken (example order for a list
    or a rank's queue), so a crash or deadline mid-run keeps every finished row."""

    def __init__(self, recorder):
        self.recorder, self.taken, self.done, self.rows, self.pos = recorder, [], {}, {}, 0

    def take(self, index):
        self.taken.append(index)

    def finish(self, index, make_row):
        self.done[index] = make_row
        while self.pos < len(self.taken) and self.taken[self.pos] in self.done:
            i = self.taken[self.pos]
            self.rows[i] = self.done.pop(i)(self.recorder)
            self.pos += 1

    def records(self):
        return [self.rows[i] for i in sorted(self.rows)]

    def close(self):
        if self.recorder is not None:
            self.recorder.close()


def _source(order, queue, writer):
    pos = 0

    def next_index():
        nonlocal pos
        if queue is not None:
            index = queue()
        elif pos < len(order):
            index, pos = order[pos], pos + 1
        else:
            index = None
        if index is not None:
            writer.take(index)
        return index
    return next_index


def run_gi_attack_batched(model, codes, subs, labels, args: AttackArgs, indices=None, tok=None,
                          queue=None, log=None, max_inflight=64, pipeline=True):
    """greedy (+GA) over many examples at once: up to `max_inflight`
    examples' attacks are in flight, and every round answers all their pending victim requests
    with ONE device batch (batching.run_requests), so the GPU sees thousands of rows instead of
    one GA population of <= 64.  Example `index` draws from random.Random(args.seed + index),
    so each record is exactly the sequential run with rng="per_example" (same outcome, mutants,
    adversarial code and query count); records come back in example order, and the CSV rows are
    written as the examples finish (in the order they were taken)."""
    from .batching import run_requests

    tok = tok or Tokenizer()
    attacker = make_attacker(args, model, tok)
    writer = _InOrderWriter(Recorder(args.csv_store_path) if args.csv_store_path else None)
    order = list(range(len(codes))) if indices is None else list(indices)
    t0 = time.time()

    def start(index):
        return attack_one_gen(attacker, tok, codes[index], subs[index], labels[index], args,
                              random.Random(args.seed + index))

    def on_done(index, value, queries, ts):
        res, attack_type = value
        dt = (time.time() - ts) / 60
        if log:
            log(_record(index, res, attack_type, queries, dt, None))
        writer.finish(index, lambda rec: _record(index, res, attack_type, queries, dt, rec))

    try:
        run_requests(model, _source(order, queue, writer), start, on_done, max_inflight, pipeline)
    finally:
        writer.close()
    return _totals(writer.records(), time.time() - t0)


def run_gi_attack(model, codes, subs, labels, args: AttackArgs, indices=None, tok=None,
                  queue=None, log=None):
    """greedy (+GA) over the given examples; returns per-example records and totals.
    queue: optional callable returning the next example index (or None when drained)."""
    tok = tok or Tokenizer()
    attacker = make_attacker(args, model, tok)
    recorder = Recorder(args.csv_store_path) if args.csv_store_path else None
    if args.rng == "global":
        set_seed(args.seed)
    order = list(range(len(codes))) if indices is None else list(indices)
    records = []
    t0 = time.time()
    pos = 0
    try:
        while True:
            if queue is not None:
                index = queue()
                if index is None:
                    break
            else:
                if pos >= len(order):
                    break
                index = order[pos]
                pos += 1
            if args.rng == "per_example":
                random.seed(args.seed + index)
            q0 = model.query
            ts = time.time()
            res, attack_type = attack_one(attacker, tok, codes[index], subs[index], labels[index],
                                          args)
            records.append(_record(index, res, attack_type, model.query - q0,
                                   (time.time() - ts) / 60, recorder))
            if log:
                log(records[-1])
    finally:
        if recorder is not None:
            recorder.close()
    return _totals(records, time.time() - t0)


MHM_ATTACKERS = {"devign": MHM_Attacker, "authorship": AuthorshipMHM_Attacker,
                 "clone": CloneMHM_Attacker, "gcb_devign": GraphMHM_Attacker,
                 "gcb_authorship": GraphAuthorshipMHM_Attacker, "gcb_clone": GraphCloneMHM_Attacker}
# max_iter of each task's mhm driver: CodeXGLUE clone 10 (mhm_attack.py:196-203), GraphCodeBERT
# clone 400 (mhm_attack.py:200-206), 100 elsewhere
MHM_MAX_ITER = {"clone": 10, "gcb_clone": 400}


def _task_lang(task, args=None):
    base = task[4:] if task.startswith("gcb_") else task
    return {"devign": getattr(args, "lang", "c") or "c", "clone": "java",
            "authorship": "python"}[base]


def make_mhm_attacker(args, model, tok, codes):
    """mhm_attack.py's setup: build_vocab over every program's leaves (5000 names; code1 of the
    clone pairs, :168-172) and the task's MHM_Attacker copy."""
    task = getattr(args, "task", "devign")
    lang = _task_lang(task, args)
    texts = [c[2] for c in codes] if _is_clone(task) else codes
    code_tokens = [get_identifiers(c, lang)[1] for c in texts]
    id2token, token2id = build_vocab(code_tokens, 5000)
    return MHM_ATTACKERS[task](args, model, None, tok, token2id, id2token)


def _record_key_error(args, task):
    """on_error = "record" turns a chain's KeyError into is_success -5 for the one copy that is
    documented to raise it (GraphCloneMHM_Attacker: GraphCodeBERT/clonedetection/code/
    attacker.py never skips a candidate naming a variable); any other task's KeyError is a bug
    and propagates."""
    return getattr(args, "on_error", "raise") == "record" and task == "gcb_clone"


def mhm_one_gen(attacker, tok, code, subs, label, args, n_candi, max_iter, prob_threshold,
                original, rng):
    """One example of mhm_attack.py:188-230 (Authorship mhm.py:192-233, clone mhm_attack.py:
    186-221) as a request generator: the original-prediction query, then (if correctly
    classified) the MCMC chain.  Returns (is_success, result dict or None)."""
    task = getattr(args, "task", "devign")
    example = _example(tok, code, label, args.block_size, task, args)
    _, preds = yield attacker.classifier.prepare([example])
    if preds[0] != label:
        return -4, None
    try:
        res = yield from attacker.chain_gen(tok, subs, code, label, example, n_candi, max_iter,
                                            prob_threshold, original, rng)
    except KeyError as e:
        if not _record_key_error(args, task):
            raise
        return -5, {"error": f"KeyError: {e}"}
    return (1 if res["succ"] else (-1 if res["succ"] is not None else -3)), res


def _mhm_call(attacker, task, tok, code, subs, label, example, n_candi, max_iter,
              prob_threshold, original):
    """The task driver's mcmc / mcmc_random call, in its own argument form."""
    fn = attacker.mcmc_random if original else attacker.mcmc
    kw = dict(_n_candi=n_candi, _max_iter=max_iter, _prob_threshold=prob_threshold)
    if task in ("authorship", "gcb_authorship"):  # mhm.py:199-206: (tokenizer, code, ..., subs=)
        return fn(tok, code, _label=label, subs=subs, **kw)
    if _is_clone(task):  # clone mhm_attack.py:196-203: (example, substitute, tokenizer, code_pair)
        return fn(example, subs, tok, code, _label=label, **kw)
    return fn(tok, subs, code=code, _label=label, **kw)


# the task drivers whose writemhm call passes " ".join(_res['tokens']) — a string there, so every
# character comes out space-separated (CodeXGLUE/Clone-detection-BigCloneBench/code/
# mhm_attack.py:231, GraphCodeBERT/clonedetection/code/mhm_attack.py:221,
# GraphCodeBERT/Authorship-Attribution/code/mhm_attack.py:229); the other three pass it as is
MHM_JOINED_TOKENS = ("clone", "gcb_clone", "gcb_authorship")


def writemhm_columns(task, code, tokens, last_code=None):
    """(Original Code, Adversarial Code) of a writemhm row, with each task driver's own quirks:
    CodeXGLUE clone writes "CODE1: ... ||CODE2: ..." of the example's pair (mhm_attack.py:231);
    GraphCodeBERT clonedetection writes its leftover loop variable `code` — the LAST pair of
    source_codes (mhm_attack.py:162 then :221; the pickled pair's element type is not in the
    repository, a list is assumed: str(list(pair))); the rest write the example's code."""
    if task == "clone":
        text = ("CODE1: " + code[2].replace("\n", " ") + " ||CODE2: "
                + code[3].replace("\n", " "))
    elif task == "gcb_clone":
        text = str(list(last_code if last_code is not None else code))
    else:
        text = code
    adv = " ".join(tokens) if task in MHM_JOINED_TOKENS else tokens
    return text, adv


def _mhm_record(index, code, task, res, label, queries, dt_min, recorder, last_code=None):
    """One mhm_attack.py row (recoder.writemhm, :229) of a finished chain; res None: the
    example was skipped (-4 misclassified, or {'succ': None}: no substitutable name)."""
    if res is not None and "error" in res:
        return dict(index=index, is_success=-5, queries=queries, error=res["error"])
    ok = -4 if res is None else (1 if res["succ"] else (-1 if res["succ"] is not None else -3))
    rec = dict(index=index, is_success=ok, queries=queries)
    if res is not None and res["succ"] is not None:
        rec.update(attack_type=res["attack_type"], adv_code=res["tokens"],
                   replace_info=res["replace_info"], nb_changed_var=res["nb_changed_var"],
                   nb_changed_pos=res["nb_changed_pos"])
        if recorder is not None:
            text, adv = writemhm_columns(task, code, res["tokens"], last_code)
            recorder.writemhm(index, text, res["prog_length"], adv, label,
                              res.get("orig_label", label), res["new_pred"], res["is_success"],
                              res["old_uid"], res["score_info"], res["nb_changed_var"],
                              res["nb_changed_pos"], res["replace_info"], res["attack_type"],
                              queries, dt_min)
    return rec


def run_mhm_attack(model, codes, subs, labels, args: AttackArgs, indices=None, tok=None,
                   n_candi=30, max_iter=None, prob_threshold=1, original=False, max_inflight=1,
                   queue=None, last_code=None):
    """mhm_attack.py:160-236 (MHM-NS; `original` = MHM with the random-token candidates) for
    every task: devign / authorship / clone (CodeBERT) and their gcb_* GraphCodeBERT copies
    (MHM_ATTACKERS; max_iter defaults to each driver's own, MHM_MAX_ITER).

    max_inflight = 1 is the reference loop (one global `random` stream seeded once).  With
    max_inflight > 1 the examples run interleaved (batching.run_requests over mhm_one_gen): up
    to `max_inflight` chains share every device batch; example `index` then draws from
    `random.Random(args.seed + index)` — the same per-example seeding `rng="per_example"` gives
    the GA driver — and records stay in index order.  `queue` (batched form only) pulls the
    examples from a dist.DynamicQueue shared by all ranks instead of `indices`.  With
    args.csv_store_path every attacked example gets its writemhm row (mhm_attack.py:229).
    last_code: the eval list's LAST pair, which the GraphCodeBERT clone driver writes as every
    row's Original Code (its leftover loop variable, mhm_attack.py:162 then :221); default
    codes[-1], which is that pair only when `codes` is the whole eval list — a caller passing a
    slice passes the whole list's last element."""
    tok = tok or Tokenizer()
    task = getattr(args, "task", "devign")
    if max_iter is None:
        max_iter = MHM_MAX_ITER.get(task, 100)
    set_seed(args.seed)
    attacker = make_mhm_attacker(args, model, tok, codes)
    recorder = Recorder(args.csv_store_path) if args.csv_store_path else None
    order = list(range(len(codes))) if indices is None else list(indices)
    try:
        records, t0 = _run_mhm_loop(model, codes, subs, labels, args, attacker, tok, task, order,
                                    recorder, n_candi, max_iter, prob_threshold, original,
                                    max_inflight, queue,
                                    codes[-1] if last_code is None else last_code)
    finally:
        if recorder is not None:
            recorder.close()
    correct = sum(r["is_success"] >= -1 for r in records)
    succ = sum(r["is_success"] == 1 for r in records)
    return dict(records=records, examples=len(records), total_cnt=correct, success=succ,
                success_rate=(succ / correct) if correct else 0.0,
                errors=sum(r["is_success"] == -5 for r in records),
                queries=sum(r["queries"] for r in records), wall_s=time.time() - t0)


def _run_mhm_loop(model, codes, subs, labels, args, attacker, tok, task, order, recorder, n_candi,
                  max_iter, prob_threshold, original, max_inflight, queue, last_code):
    records, t0 = [], time.time()
    if max_inflight > 1 or queue is not None:
        from .batching import run_requests

        writer = _InOrderWriter(recorder)

        def start(index):
            return mhm_one_gen(attacker, tok, codes[index], subs[index], labels[index], args,
                               n_candi, max_iter, prob_threshold, original,
                               random.Random(args.seed + index))

        def on_done(index, value, queries, ts):
            dt = (time.time() - ts) / 60
            writer.finish(index, lambda rec: _mhm_record(index, codes[index], task, value[1],
                                                         labels[index], queries, dt, rec,
                                                         last_code))

        run_requests(model, _source(order, queue, writer), start, on_done, max(2, max_inflight))
        records = writer.records()
        order = []
    for index in order:
        example = _example(tok, codes[index], labels[index], args.block_size, task, args)
        q0 = model.query
        ts = time.time()
        probs, preds = model.get_results([example], args.eval_batch_size)
        if preds[0] != labels[index]:
            records.append(_mhm_record(index, codes[index], task, None, labels[index],
                                       model.query - q0, 0.0, None))
            continue
        try:
            res = _mhm_call(attacker, task, tok, codes[index], subs[index], labels[index],
                            example, n_candi, max_iter, prob_threshold, original)
        except KeyError as e:
            if not _record_key_error(args, task):
                raise
            res = {"error": f"KeyError: {e}"}
        records.append(_mhm_record(index, codes[index], task, res, labels[index],
                                   model.query - q0, (time.time() - ts) / 60, recorder,
                                   last_code))
    return records, t0
