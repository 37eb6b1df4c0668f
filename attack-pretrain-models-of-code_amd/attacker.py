"""ALERT attacks over the engine: greedy (importance-ordered), GA, and the MHM-NS baseline.

Same classes, signatures, return values and Python-`random` call order as the reference
(CodeXGLUE/Defect-detection/code/attacker.py): Attacker.greedy_attack :277-453,
Attacker.ga_attack :96-272, get_importance_score :48-83, compute_fitness :25-35,
convert_code_to_features :38-45, MHM_Attacker.mcmc / mcmc_random :466-608,
__replaceUID / __replaceUID_random :610-738.  Every victim query still goes through
Model.get_results semantics (query counter, probs/preds format); mutant text -> ids runs in the
C++ host library and the population's ids are built on the GPU by ae_splice.
"""
from __future__ import annotations

import copy
import random

import numpy as np

from .host import MODE_BATCH, MODE_RAW, MODE_SINGLE, Example
from .utils import (CodeDataset, InputFeatures, IdsDataset, _tokenize, crossover,
                    get_identifier_posistions_from_code, get_masked_code_by_position, isUID,
                    map_chromesome, mutate, select_parents)


def _label_of(example):
    lab = example[-1]  # (ids, label) / GCB (ids, mask, pos, label) / pairs: label is last
    return int(lab.item()) if hasattr(lab, "item") else int(lab)


def convert_code_to_features(code, tokenizer, label, args, raw: bool = False):
    """attacker.py:38-45 (host tokenizer; ' '.join(code.split()) -> [:block-2] -> CLS/SEP/pad).
    raw: the Authorship-Attribution form, which tokenizes the text as is
    (CodeXGLUE/Authorship-Attribution/code/attacker.py:31-37)."""
    ids, _ = tokenizer.featurize([code], args.block_size, raw=raw)
    return InputFeatures(None, ids[0].tolist(), 0, label)


def remove_python_docstrings(source: str) -> str:
    """remove_comments_and_docstrings(source, 'python') (python_parser/parser_folder/utils.py:
    31-68): re-emit the stdlib tokenize stream without comments and without string tokens that
    open a logical line (after INDENT / NEWLINE, or at column 0), then drop blank lines."""
    import io
    import tokenize

    out, prev, last_line, last_col = "", tokenize.INDENT, -1, 0
    for tok in tokenize.generate_tokens(io.StringIO(source).readline):
        ttype, text, (sl, sc), (el, ec), _ = tok
        if sl > last_line:
            last_col = 0
        if sc > last_col:
            out += " " * (sc - last_col)
        if ttype == tokenize.COMMENT:
            pass
        elif ttype == tokenize.STRING:
            if prev != tokenize.INDENT and prev != tokenize.NEWLINE and sc > 0:
                out += text
        else:
            out += text
        prev, last_col, last_line = ttype, ec, el
    return "\n".join(x for x in out.split("\n") if x.strip() != "")


def get_identifiers(code, lang):
    """run_parser.py:272-281 — (identifiers as [[name]], code_tokens): the unique valid names of
    the data-flow graph (host/dfg.cpp) and the comment-stripped leaves.  For Python,
    extract_dataflow (run_parser.py:190-199) first turns literal '\n' into newlines and strips
    comments and docstrings with the tokenize-based remover (left as is if that raises)."""
    from .utils import is_valid_variable_name

    if lang == "python":
        code = code.replace("\\n", "\n")
        try:
            code = remove_python_docstrings(code)
        except Exception:
            pass
    ex = Example(code, lang)
    toks = ex.leaves(identifiers=True)
    idents = [[n] for n in ex.dfg_names() if is_valid_variable_name(n, lang)]
    return idents, toks


class _Scorer:
    """Victim requests for one attacked program: ids built from chromosomes (host + device
    splice) or from texts."""

    def __init__(self, attacker, code, lang="c"):
        self.a = attacker
        self.ex = Example(code, lang)

    def population(self, pops, mode):
        """pops: list of [(tgt, sub), ...] -> a request (Payload) of len(pops) queries."""
        return self.a._population(self.ex, pops, mode)


def join_payloads(payloads):
    """Concatenate requests of one victim into one (rows in order, queries summed)."""
    from .model import Payload

    ps = [p for p in payloads if p.n]
    if len(ps) == 1:
        return ps[0]
    first = ps[0]
    if isinstance(first.ids, np.ndarray):
        ids = np.concatenate([p.ids for p in ps], 0)
    else:
        import torch

        ids = torch.cat([p.ids for p in ps], 0)
    lens = None if any(p.lens is None for p in ps) else np.concatenate([p.lens for p in ps])
    extra = None
    if first.extra is not None:
        extra = tuple(np.concatenate([p.extra[k] for p in ps]) for k in range(len(first.extra)))
    return Payload(ids, lens, sum(p.n for p in ps), extra)


def answer(model, gen):
    """Run an attack generator to completion, answering each request with its own
    get_results-equivalent call (the reference's one-example-at-a-time loop)."""
    try:
        req = next(gen)
        while True:
            req = gen.send(model.score_prepared([req])[0])
    except StopIteration as stop:
        return stop.value


def _importance_gen(args, words_list, variable_names, tgt_model, tokenizer, payload_fn=None):
    """get_importance_score as a request generator (attacker.py:48-83)."""
    positions = get_identifier_posistions_from_code(words_list, variable_names)
    if len(positions) == 0:
        return None, None, None
    masked_token_list, replace_token_positions = get_masked_code_by_position(words_list, positions)
    if payload_fn is not None:
        req = payload_fn([words_list] + masked_token_list)
    else:
        texts = [" ".join(tokens) for tokens in [words_list] + masked_token_list]
        req = tgt_model.prepare(tgt_model.dataset_from_texts(texts, tokenizer, args))
    logits, preds = yield req
    orig_probs = logits[0]
    orig_label = preds[0]
    orig_prob = max(orig_probs)
    importance_score = [orig_prob - prob[orig_label] for prob in logits[1:]]
    return importance_score, replace_token_positions, positions


def get_importance_score(args, example, code, words_list, sub_words, variable_names, tgt_model,
                         tokenizer, label_list, batch_size=16, max_length=512,
                         model_type="classification"):
    """attacker.py:48-83: 1 + #occurrences queries (original + one '<unk>' copy per occurrence)."""
    return answer(tgt_model, _importance_gen(args, words_list, variable_names, tgt_model,
                                             tokenizer))


def compute_fitness(chromesome, codebert_tgt, tokenizer_tgt, orig_prob, orig_label, true_label,
                    code, names_positions_dict, args, scorer=None):
    """attacker.py:25-35: one query for one chromosome."""
    if scorer is not None:
        new_logits, preds = codebert_tgt.score_prepared(
            [scorer.population([list(chromesome.items())], MODE_BATCH)])[0]
    else:
        temp_code = map_chromesome(chromesome, code, getattr(args, "lang", "c"))
        new_feature = convert_code_to_features(temp_code, tokenizer_tgt, true_label, args)
        new_logits, preds = codebert_tgt.get_results(CodeDataset([new_feature]), args.eval_batch_size)
    fitness_value = orig_prob - new_logits[0][orig_label]
    return fitness_value, preds[0]


class Attacker:
    """greedy_attack / ga_attack with the reference's signatures and 12-tuple results.

    Each attack is written once, as a generator that yields its victim requests (Payloads) and
    receives (probs, preds) back: greedy_attack / ga_attack answer every request with its own
    call (the reference loop, Python's global `random`), while drivers.run_gi_attack_batched
    keeps many examples' generators in flight and answers all their pending requests with ONE
    device batch (each example on its own `random.Random(seed + index)`).

    The same generators serve the task variants through a few hooks:
      Devign (CodeBERT)       CodeXGLUE/Defect-detection/code/attacker.py        lang 'c'
      Authorship-Attribution  CodeXGLUE/Authorship-Attribution/code/attacker.py  lang 'python',
                              raw-text featurisation (the Model of task 'authorship'), no -3
                              exit for an empty gene pool in ga_attack (:147-150)
      Clone (pairs)           CloneAttacker below
      GraphCodeBERT variants  the GraphModel victims (graph.py) behind the same hooks
    """

    ga_empty_check = True  # ga_attack returns -3 when no substitutable name occurs as a word

    def __init__(self, args, model_tgt, tokenizer_tgt, model_mlm, tokenizer_mlm, use_bpe,
                 threshold_pred_score) -> None:
        self.args = args
        self.model_tgt = model_tgt
        self.tokenizer_tgt = tokenizer_tgt
        self.model_mlm = model_mlm
        self.tokenizer_mlm = tokenizer_mlm
        self.use_bpe = use_bpe
        self.threshold_pred_score = threshold_pred_score
        self.lang = getattr(args, "lang", "c")
        # GA mutants per iteration: args.eval_batch_size (CodeBERT Devign, attacker.py:226);
        # the GraphCodeBERT Devign and CodeBERT clone attackers hard-code 64
        # (GraphCodeBERT/Defect-detection/code/attacker.py:246)
        self.ga_batch = None

    # ---- hooks ---------------------------------------------------------------------------------
    def _population(self, ex, pops, mode):
        return self.model_tgt.prepare_population(ex, self.tokenizer_tgt, pops, mode,
                                                 self.args.block_size)

    def _importance_payload(self):
        return None  # texts through Model.dataset_from_texts

    # ------------------------------------------------------------------------------------------
    def ga_attack(self, example, code, substituions, initial_replace=None):
        """Genetic attack (attacker.py:96-272); returns the reference's 12-tuple."""
        return answer(self.model_tgt, self.ga_gen(example, code, substituions, initial_replace,
                                                  random))

    def greedy_attack(self, example, code, substituions):
        """Importance-ordered greedy attack (attacker.py:277-453); returns the 12-tuple."""
        return answer(self.model_tgt, self.greedy_gen(example, code, substituions))

    # ------------------------------------------------------------------------------------------
    def ga_gen(self, example, code, substituions, initial_replace=None, rng=random):
        m = self.model_tgt
        logits, preds = yield m.prepare([example])
        orig_prob = logits[0]
        orig_label = preds[0]
        current_prob = max(orig_prob)
        true_label = _label_of(example)
        adv_code = ""
        temp_label = None

        identifiers, code_tokens = get_identifiers(code, self.lang)
        prog_length = len(code_tokens)
        processed_code = " ".join(code_tokens)
        words, sub_words, keys = _tokenize(processed_code, self.tokenizer_mlm)
        variable_names = list(substituions.keys())

        if not orig_label == true_label:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -4, \
                variable_names, None, None, None, None
        if len(variable_names) == 0:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -3, \
                variable_names, None, None, None, None

        names_positions_dict = get_identifier_posistions_from_code(words, variable_names)
        nb_changed_var = 0
        nb_changed_pos = 0
        is_success = -1
        variable_substitue_dict = {w: substituions[w] for w in names_positions_dict.keys()}
        if self.ga_empty_check and len(variable_substitue_dict) == 0:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -3, \
                variable_names, None, None, None, None

        scorer = _Scorer(self, code, self.lang)
        fitness_values = []
        base_chromesome = {word: word for word in variable_substitue_dict.keys()}
        population = [base_chromesome]
        for tgt_word in variable_substitue_dict.keys():
            if initial_replace is None:
                # pick the substitute with the largest probability gap (one batch per variable)
                current_prob = max(orig_prob)
                most_gap = 0.0
                substitute_list = list(variable_substitue_dict[tgt_word])
                if len(substitute_list) == 0:
                    continue
                logits, preds = yield scorer.population([[(tgt_word, s)] for s in substitute_list],
                                                        MODE_SINGLE)
                best = -1
                for index, temp_prob in enumerate(logits):
                    temp_label = preds[index]
                    gap = current_prob - temp_prob[temp_label]
                    if gap > most_gap:
                        most_gap = gap
                        best = index
                initial_candidate = tgt_word if best == -1 else substitute_list[best]
            else:
                initial_candidate = initial_replace[tgt_word]
            temp_chromesome = copy.deepcopy(base_chromesome)
            temp_chromesome[tgt_word] = initial_candidate
            population.append(temp_chromesome)
            # compute_fitness (attacker.py:25-35): one query
            new_logits, fpreds = yield scorer.population([list(temp_chromesome.items())],
                                                         MODE_BATCH)
            temp_fitness, temp_label = max(orig_prob) - new_logits[0][orig_label], fpreds[0]
            fitness_values.append(temp_fitness)

        cross_probability = 0.7
        max_iter = max(5 * len(population), 10)
        batch = self.ga_batch or self.args.eval_batch_size
        for i in range(max_iter):
            _temp_mutants = []
            for j in range(batch):
                p = rng.random()
                chromesome_1, index_1, chromesome_2, index_2 = select_parents(population, rng)
                if p < cross_probability:
                    if chromesome_1 == chromesome_2:
                        child_1 = mutate(chromesome_1, variable_substitue_dict, rng)
                        continue
                    child_1, child_2 = crossover(chromesome_1, chromesome_2, rng=rng)
                    if child_1 == chromesome_1 or child_1 == chromesome_2:
                        child_1 = mutate(chromesome_1, variable_substitue_dict, rng)
                else:
                    child_1 = mutate(chromesome_1, variable_substitue_dict, rng)
                _temp_mutants.append(child_1)
            if len(_temp_mutants) == 0:
                continue
            # the dicts are read only now, after every in-place mutate of this iteration
            mutate_logits, mutate_preds = yield scorer.population(
                [list(mt.items()) for mt in _temp_mutants], MODE_BATCH)
            mutate_fitness_values = []
            for index, logits in enumerate(mutate_logits):
                if mutate_preds[index] != orig_label:
                    adv_code = map_chromesome(_temp_mutants[index], code, self.lang, scorer.ex)
                    for old_word in _temp_mutants[index].keys():
                        if old_word == _temp_mutants[index][old_word]:
                            nb_changed_var += 1   # counts UNchanged names (reference quirk)
                            nb_changed_pos += len(names_positions_dict[old_word])
                    return code, prog_length, adv_code, true_label, orig_label, \
                        mutate_preds[index], 1, variable_names, None, nb_changed_var, \
                        nb_changed_pos, _temp_mutants[index]
                mutate_fitness_values.append(max(orig_prob) - logits[orig_label])
            for index, fitness_value in enumerate(mutate_fitness_values):
                min_value = min(fitness_values)
                if fitness_value > min_value:
                    min_index = fitness_values.index(min_value)
                    population[min_index] = _temp_mutants[index]
                    fitness_values[min_index] = fitness_value

        return code, prog_length, adv_code, true_label, orig_label, temp_label, is_success, \
            variable_names, None, nb_changed_var, nb_changed_pos, None

    # ------------------------------------------------------------------------------------------
    def greedy_gen(self, example, code, substituions):
        m = self.model_tgt
        logits, preds = yield m.prepare([example])
        orig_prob = logits[0]
        orig_label = preds[0]
        current_prob = max(orig_prob)
        true_label = _label_of(example)
        adv_code = ""
        temp_label = None

        identifiers, code_tokens = get_identifiers(code, self.lang)
        prog_length = len(code_tokens)
        processed_code = " ".join(code_tokens)
        words, sub_words, keys = _tokenize(processed_code, self.tokenizer_mlm)
        variable_names = list(substituions.keys())

        if not orig_label == true_label:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -4, \
                variable_names, None, None, None, None
        if len(variable_names) == 0:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -3, \
                variable_names, None, None, None, None

        importance_score, replace_token_positions, names_positions_dict = yield from \
            _importance_gen(self.args, words, variable_names, m, self.tokenizer_tgt,
                            self._importance_payload())
        if importance_score is None:
            return code, prog_length, adv_code, true_label, orig_label, temp_label, -3, \
                variable_names, None, None, None, None

        token_pos_to_score_pos = {pos: i for i, pos in enumerate(replace_token_positions)}
        names_to_importance_score = {}
        for name in names_positions_dict.keys():
            total_score = 0.0
            for token_pos in names_positions_dict[name]:
                total_score += importance_score[token_pos_to_score_pos[token_pos]]
            names_to_importance_score[name] = total_score
        sorted_list_of_names = sorted(names_to_importance_score.items(), key=lambda x: x[1],
                                      reverse=True)

        final_code = copy.deepcopy(code)
        nb_changed_var = 0
        nb_changed_pos = 0
        is_success = -1
        replaced_words = {}
        for name_and_score in sorted_list_of_names:
            tgt_word = name_and_score[0]
            all_substitues = substituions[tgt_word]
            most_gap = 0.0
            candidate = None
            substitute_list = list(all_substitues)
            if len(substitute_list) == 0:
                continue
            # get_example(final_code, tgt, sub) per substitute, one batch
            scorer = _Scorer(self, final_code, self.lang)
            logits, preds = yield scorer.population([[(tgt_word, s)] for s in substitute_list],
                                                    MODE_SINGLE)
            assert len(logits) == len(substitute_list)
            for index, temp_prob in enumerate(logits):
                temp_label = preds[index]
                if temp_label != orig_label:
                    is_success = 1
                    nb_changed_var += 1
                    nb_changed_pos += len(names_positions_dict[tgt_word])
                    candidate = substitute_list[index]
                    replaced_words[tgt_word] = candidate
                    adv_code = scorer.ex.mutant_text([(tgt_word, candidate)], MODE_SINGLE)
                    if getattr(self.args, "verbose", False):
                        print("%s SUC! %s => %s (%.5f => %.5f)" % (
                            ">>", tgt_word, candidate, current_prob, temp_prob[orig_label]),
                            flush=True)
                    return code, prog_length, adv_code, true_label, orig_label, temp_label, \
                        is_success, variable_names, names_to_importance_score, nb_changed_var, \
                        nb_changed_pos, replaced_words
                gap = current_prob - temp_prob[temp_label]
                if gap > most_gap:
                    most_gap = gap
                    candidate = substitute_list[index]
            if most_gap > 0:
                nb_changed_var += 1
                nb_changed_pos += len(names_positions_dict[tgt_word])
                current_prob = current_prob - most_gap
                replaced_words[tgt_word] = candidate
                final_code = scorer.ex.mutant_text([(tgt_word, candidate)], MODE_SINGLE)
            else:
                replaced_words[tgt_word] = tgt_word
            adv_code = final_code

        return code, prog_length, adv_code, true_label, orig_label, temp_label, is_success, \
            variable_names, names_to_importance_score, nb_changed_var, nb_changed_pos, \
            replaced_words


class AuthorshipAttacker(Attacker):
    """CodeXGLUE/Authorship-Attribution/code/attacker.py: the Devign attacker on Python code with a
    66-way victim (argmax predictions), raw-text featurisation (the 'authorship' Model) and no -3
    exit for an empty gene pool in ga_attack (:147-150: the reference then runs its GA loop on an
    empty chromosome and fails inside mutate, which this class reproduces by raising)."""

    ga_empty_check = False

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lang = "python"


class CloneAttacker(Attacker):
    """CodeXGLUE/Clone-detection-BigCloneBench/code/attacker.py: a pair (code1, code2) is one
    query; the victim reads [ids(code1) | ids(code2)] as two block-size rows and a 2-way pair
    head.  Only code1 is perturbed.  Differences from the Devign attacker this class keeps:
      * signatures greedy_attack(example, substitutes, code) / ga_attack(example, substitutes,
        code, initial_replace) with code = (id1, id2, code1, code2) (:89, :285); the returned
        code is that tuple;
      * Java leaves / mutants (get_identifiers(code1, 'java'), get_example(..., 'java'));
      * code2's half of every mutant row: tokenize(' '.join(code2.split())) (:128-129);
      * importance features from WORDS: convert_examples_to_features is handed whole words of
        code1 (masked with '<unk>') and of " ".join(get_identifiers(code2)[1]) split like
        _tokenize, so each word becomes ONE id through convert_tokens_to_ids (the unk id unless
        the word is itself a vocabulary token) (:48-71 with run.py:102-119);
      * 64 GA mutants per iteration whatever eval_batch_size is (:226); no -3 exit for an
        empty gene pool in ga_attack (:157-166)."""

    ga_empty_check = False

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lang = "java"
        self.ga_batch = 64
        self._code2 = None

    # ---- reference signatures ---------------------------------------------------------------
    def ga_attack(self, example, substitutes, code, initial_replace=None):
        return answer(self.model_tgt, self.ga_gen(example, substitutes, code, initial_replace,
                                                  random))

    def greedy_attack(self, example, substitutes, code):
        return answer(self.model_tgt, self.greedy_gen(example, substitutes, code))

    def ga_gen(self, example, substitutes, code, initial_replace=None, rng=random):
        res = yield from self._bound(code, super().ga_gen(example, code[2], substitutes,
                                                          initial_replace, rng))
        return (code,) + tuple(res[1:])

    def greedy_gen(self, example, substitutes, code):
        res = yield from self._bound(code, super().greedy_gen(example, code[2], substitutes))
        return (code,) + tuple(res[1:])

    # ---- pair requests ------------------------------------------------------------------------
    def _pair_state(self, code):
        """code2's fixed half of every row, and its word-level importance half."""
        L = self.args.block_size
        ids2, lens2 = self.tokenizer_tgt.featurize([code[3]], L)
        _, toks2 = get_identifiers(code[3], self.lang)
        words2 = " ".join(toks2).replace("\n", "").split(" ")
        return ids2[0], int(lens2[0]), self._word_row(words2)

    def _bound(self, code, gen):
        """Run `gen` with this pair's code2 state bound.  The binding is re-installed before
        every step, since the batched driver interleaves many pairs' generators over one
        attacker (requests are built before they are yielded, so each sees its own pair)."""
        bound = self._pair_state(code)
        self._code2 = bound
        try:
            req = next(gen)
            while True:
                ans = yield req
                self._code2 = bound
                req = gen.send(ans)
        except StopIteration as stop:
            return stop.value

    def _word_row(self, words):
        """[cls] + convert_tokens_to_ids(words[:L-2]) + [sep] + pad (run.py:102-119)."""
        t, L = self.tokenizer_tgt, self.args.block_size
        body = t.convert_tokens_to_ids(list(words[:L - 2]))
        row = [t.cls_token_id] + list(body) + [t.sep_token_id]
        return np.asarray(row + [t.pad_token_id] * (L - len(row)), dtype=np.int32)

    def _population(self, ex, pops, mode):
        m = self.model_tgt
        ids1, lens1 = m.population_rows(ex, self.tokenizer_tgt, pops, mode, self.args.block_size)
        ids2, len2, _ = self._code2
        return m.prepare_pairs(ids1, lens1, ids2, len2)

    def _importance_payload(self):
        ids2w = self._code2[2]

        def build(word_lists):
            ids1 = np.stack([self._word_row(w) for w in word_lists])
            lens1 = (ids1 != self.tokenizer_tgt.pad_token_id).sum(1).astype(np.int32)
            lens2 = int((ids2w != self.tokenizer_tgt.pad_token_id).sum())
            return self.model_tgt.prepare_pairs(ids1, lens1, ids2w, lens2)

        return build


class MHM_Attacker:
    """MHM-NS baseline (attacker.py:457-738).

    The six reference copies differ only in a few places, which the subclasses set:
      class                          reference                                      lang    skip known
                                                                                            subs / random  random label
      MHM_Attacker                   CodeXGLUE/Defect-detection/code/attacker.py    c       yes / yes      MHM-Origin
      AuthorshipMHM_Attacker         CodeXGLUE/Authorship-Attribution/.../attacker.py python yes / no      MHM-Origin
      CloneMHM_Attacker              CodeXGLUE/Clone-detection-BigCloneBench/...    java    yes / yes      Ori_MHM
      GraphMHM_Attacker              GraphCodeBERT/Defect-detection/.../attacker.py c       yes / yes      Ori_MHM
      GraphAuthorshipMHM_Attacker    GraphCodeBERT/Authorship-Attribution/...       python  yes / yes      Ori_MHM
      GraphCloneMHM_Attacker         GraphCodeBERT/clonedetection/.../attacker.py   java    no / no        Ori_MHM
    (skip known: a candidate that already names a variable of the chain is dropped,
    `if c in _uid.keys(): continue`).  The GraphCodeBERT copies featurise every candidate with
    their own convert_code_to_features (data flow + graph mask), which the GraphModel victim's
    dataset_from_texts applies; the clone copies query the dataset example first and score pairs
    (mutated code1 against the fixed code2)."""

    # __replaceUID drops substitutes that already name a variable (attacker.py:623-624)
    skip_known_subs = True
    # __replaceUID_random drops random-vocabulary candidates that already name a variable
    # (attacker.py:688-689); the CodeBERT Authorship-Attribution copy does not
    skip_known_uids = True
    # attack_type of mcmc_random's results (attacker.py:599,606)
    random_type = "MHM-Origin"

    def __init__(self, args, model_tgt, model_mlm, tokenizer_mlm, _token2idx, _idx2token) -> None:
        self.classifier = model_tgt
        self.model_mlm = model_mlm
        self.token2idx = _token2idx
        self.idx2token = _idx2token
        self.args = args
        self.tokenizer_mlm = tokenizer_mlm
        self.lang = getattr(args, "lang", "c")

    # The MCMC loop is written once, as a generator: every victim query is a `yield <Payload>`
    # (the victim's request API, model.py) that receives `(probs, preds)` back.  `_run` answers each request with its own get_results
    # call (the reference's one-example-at-a-time behaviour); `mcmc_batched` answers the pending
    # requests of many examples with ONE device batch.  Rows are scored batch-invariantly, so the
    # two give identical results; `rng` is the Python `random` module (sequential, as the
    # reference) or a per-example `random.Random(seed)` (batched: interleaved examples cannot
    # share one global stream).
    def _run(self, tokenizer, substituions, code, _label, _n_candi, _max_iter, _prob_threshold,
             replace, attack_type):
        gen = self._run_gen(tokenizer, substituions, code, _label, _n_candi, _max_iter,
                            _prob_threshold, replace, attack_type, random)
        return answer(self.classifier, gen)

    def _run_gen(self, tokenizer, substituions, code, _label, _n_candi, _max_iter, _prob_threshold,
                 replace, attack_type, rng, ctx=None):
        """ctx: per-chain request state handed to _candidates_request (the clone copies' fixed
        code2 half); chains of many examples interleave over one attacker, so it is never kept
        on self."""
        identifiers, code_tokens = get_identifiers(code, self.lang)
        prog_length = len(code_tokens)
        processed_code = " ".join(code_tokens)
        words, sub_words, keys = _tokenize(processed_code, tokenizer)
        raw_tokens = copy.deepcopy(words)
        variable_names = list(substituions.keys())
        uid = get_identifier_posistions_from_code(words, variable_names)
        if len(uid) <= 0:
            return {"succ": None, "tokens": None, "raw_tokens": None}
        variable_substitue_dict = {w: substituions[w] for w in uid.keys()}
        if len(variable_substitue_dict) <= 0:
            return {"succ": None, "tokens": None, "raw_tokens": None}
        old_uids = {}
        old_uid = ""
        res = None
        for iteration in range(1, 1 + _max_iter):
            res = yield from replace(rng, _tokens=code, _label=_label, _uid=uid,
                                     substitute_dict=variable_substitue_dict, _n_candi=_n_candi,
                                     _prob_threshold=_prob_threshold, ctx=ctx)
            self._print_res(iteration, res)
            if res["status"].lower() in ["s", "a"]:
                if iteration == 1:
                    old_uids[res["old_uid"]] = [res["new_uid"]]
                    old_uid = res["old_uid"]
                flag = 0
                for k in old_uids.keys():
                    if res["old_uid"] == old_uids[k][-1]:
                        flag = 1
                        old_uids[k].append(res["new_uid"])
                        old_uid = k
                        break
                if flag == 0:
                    old_uids[res["old_uid"]] = [res["new_uid"]]
                    old_uid = res["old_uid"]
                code = res["tokens"]
                uid[res["new_uid"]] = uid.pop(res["old_uid"])
                variable_substitue_dict[res["new_uid"]] = variable_substitue_dict.pop(res["old_uid"])
                for i in range(len(raw_tokens)):
                    if raw_tokens[i] == res["old_uid"]:
                        raw_tokens[i] = res["new_uid"]
                if res["status"].lower() == "s":
                    replace_info, nb_changed_pos = {}, 0
                    for uid_ in old_uids.keys():
                        replace_info[uid_] = old_uids[uid_][-1]
                        nb_changed_pos += len(uid[old_uids[uid_][-1]])
                    return {"succ": True, "tokens": code, "raw_tokens": raw_tokens,
                            "prog_length": prog_length, "new_pred": res["new_pred"],
                            "is_success": 1, "old_uid": old_uid,
                            "score_info": res["old_prob"][0] - res["new_prob"][0],
                            "nb_changed_var": len(old_uids), "nb_changed_pos": nb_changed_pos,
                            "replace_info": replace_info, "attack_type": attack_type}
        replace_info, nb_changed_pos = {}, 0
        for uid_ in old_uids.keys():
            replace_info[uid_] = old_uids[uid_][-1]
            nb_changed_pos += len(uid[old_uids[uid_][-1]])
        return {"succ": False, "tokens": res["tokens"], "raw_tokens": None,
                "prog_length": prog_length, "new_pred": res["new_pred"], "is_success": -1,
                "old_uid": old_uid, "score_info": res["old_prob"][0] - res["new_prob"][0],
                "nb_changed_var": len(old_uids), "nb_changed_pos": nb_changed_pos,
                "replace_info": replace_info, "attack_type": attack_type}

    def mcmc(self, tokenizer, substituions, code=None, _label=None, _n_candi=30, _max_iter=100,
             _prob_threshold=0.95):
        return self._run(tokenizer, substituions, code, _label, _n_candi, _max_iter,
                         _prob_threshold, self._replace_uid, "MHM")

    def mcmc_random(self, tokenizer, substituions, code=None, _label=None, _n_candi=30,
                    _max_iter=100, _prob_threshold=0.95):
        return self._run(tokenizer, substituions, code, _label, _n_candi, _max_iter,
                         _prob_threshold, self._replace_uid_random, self.random_type)

    def chain_gen(self, tokenizer, substituions, code, _label, example, _n_candi, _max_iter,
                  _prob_threshold, original, rng):
        """One mcmc (or mcmc_random if `original`) call as a request generator; `example` is the
        dataset item, read only by the copies whose mcmc queries it first (clone)."""
        replace = self._replace_uid_random if original else self._replace_uid
        kind = self.random_type if original else "MHM"
        return self._run_gen(tokenizer, substituions, code, _label, _n_candi, _max_iter,
                             _prob_threshold, replace, kind, rng)

    def mcmc_batched(self, tokenizer, jobs, _n_candi=30, _max_iter=100, _prob_threshold=0.95,
                     original=False, max_inflight=64, on_done=None):
        """Many examples' MCMC chains in flight at once.

        `jobs` = [(substituions, code, label, seed[, example])]; example j runs on
        `random.Random(seed)`, so its chain is exactly `random.seed(seed); mcmc(...)` (or
        `mcmc_random` if `original`).  Each round gathers the pending ≤(1+_n_candi)-candidate
        requests of up to `max_inflight` chains into ONE `get_results` call, so the device sees
        batches of hundreds of sequences instead of ≤31.  The victim's query counter advances by
        the same total as the sequential runs.  Returns `[(result_dict, queries)]` in job order;
        `on_done(j, result, queries)` is called as each chain finishes."""
        from .batching import list_source, run_requests

        out = [None] * len(jobs)

        def start(j):
            subs, code, label, seed = jobs[j][:4]
            example = jobs[j][4] if len(jobs[j]) > 4 else None
            return self.chain_gen(tokenizer, subs, code, label, example, _n_candi, _max_iter,
                                  _prob_threshold, original, random.Random(seed))

        def finish(j, value, q, _t0):
            out[j] = (value, q)
            if on_done is not None:
                on_done(j, value, q)

        run_requests(self.classifier, list_source(range(len(jobs))), start, finish,
                     max_inflight=max_inflight)
        return out

    def _candidates_result(self, rng, _tokens, _label, selected_uid, candi_token, candi_pairs,
                           _prob_threshold, ctx=None):
        """Shared tail of __replaceUID / __replaceUID_random (attacker.py:634-670)."""
        # candidate 0 is the unmodified code; the others are get_example(code, uid, c)
        ex = Example(_tokens, self.lang)
        tok = self.tokenizer_mlm
        L = self.args.block_size
        pops = [[(selected_uid, c)] for c in candi_pairs]
        prob, pred = yield self._candidates_request(ex, tok, _tokens, pops, L, ctx)
        candi_tokens = [_tokens] + [None] * len(pops)

        def text(i):
            if candi_tokens[i] is None:
                candi_tokens[i] = ex.mutant_text(pops[i - 1], MODE_SINGLE)
            return candi_tokens[i]

        for i in range(len(candi_token)):
            if pred[i] != _label:
                return {"status": "s", "alpha": 1, "tokens": text(i), "old_uid": selected_uid,
                        "new_uid": candi_token[i], "old_prob": prob[0], "new_prob": prob[i],
                        "old_pred": pred[0], "new_pred": pred[i],
                        "nb_changed_pos": _tokens.count(selected_uid)}
        candi_idx = 0
        min_prob = 1.0
        for idx, a_prob in enumerate(prob[1:]):
            if a_prob[_label] < min_prob:
                candi_idx = idx + 1
                min_prob = a_prob[_label]
        alpha = (1 - prob[candi_idx][_label] + 1e-10) / (1 - prob[0][_label] + 1e-10)
        # the reference reports candi_tokens[i] with i the LAST loop index (attacker.py:662-670)
        i = len(candi_token) - 1
        status = "r" if (rng.uniform(0, 1) > alpha or alpha < _prob_threshold) else "a"
        return {"status": status, "alpha": alpha, "tokens": text(i), "old_uid": selected_uid,
                "new_uid": candi_token[i], "old_prob": prob[0], "new_prob": prob[i],
                "old_pred": pred[0], "new_pred": pred[i],
                "nb_changed_pos": _tokens.count(selected_uid)}

    def _candidates_request(self, ex, tok, _tokens, pops, L, ctx=None):
        """One request: the unmodified code, then get_example(code, uid, c) per candidate."""
        m = self.classifier
        if getattr(m, "population_rows", None) is not None:
            first = m.prepare(m.dataset_from_texts([_tokens], tok, self.args))
            if not pops:
                return first
            rows = m.population_rows(ex, tok, pops, MODE_SINGLE, L)
            return join_payloads([first, type(first)(rows[0], rows[1], len(pops))])
        # victims whose rows are not spliced token ids (GraphModel: data-flow features): every
        # candidate text through the victim's own featuriser, one batch
        texts = [_tokens] + [ex.mutant_text(p, MODE_SINGLE) for p in pops]
        return m.prepare(m.dataset_from_texts(texts, tok, self.args))

    def _replace_uid(self, rng, _tokens, _label=None, _uid={}, substitute_dict={}, _n_candi=30,
                     _prob_threshold=0.95, _candi_mode="random", ctx=None):
        assert _candi_mode.lower() in ["random", "nearby"]
        selected_uid = rng.sample(list(substitute_dict.keys()), 1)[0]
        candi_token = [selected_uid]
        pairs = []
        pool = substitute_dict[selected_uid]
        for c in rng.sample(pool, min(_n_candi, len(pool))):
            if self.skip_known_subs and c in _uid.keys():
                continue
            if isUID(c):
                candi_token.append(c)
                pairs.append(c)
        return (yield from self._candidates_result(rng, _tokens, _label, selected_uid, candi_token,
                                                   pairs, _prob_threshold, ctx))

    def _replace_uid_random(self, rng, _tokens, _label=None, _uid={}, substitute_dict={},
                            _n_candi=30, _prob_threshold=0.95, _candi_mode="random", ctx=None):
        assert _candi_mode.lower() in ["random", "nearby"]
        selected_uid = rng.sample(list(substitute_dict.keys()), 1)[0]
        candi_token = [selected_uid]
        pairs = []
        for c in rng.sample(self.idx2token, _n_candi):
            if self.skip_known_uids and c in _uid.keys():
                continue
            if isUID(c):
                candi_token.append(c)
                pairs.append(c)
        return (yield from self._candidates_result(rng, _tokens, _label, selected_uid, candi_token,
                                                   pairs, _prob_threshold, ctx))

    def _print_res(self, _iter=None, _res=None, _prefix="  => "):
        if not getattr(self.args, "verbose", False):
            return
        tag = {"s": "SUCC!", "r": "REJ.", "a": "ACC!"}[_res["status"].lower()]
        print("%s iter %d, %s %s => %s (%d => %d, %.5f => %.5f) a=%.3f" % (
            _prefix, _iter, tag, _res["old_uid"], _res["new_uid"], _res["old_pred"],
            _res["new_pred"], _res["old_prob"][_res["old_pred"]],
            _res["new_prob"][_res["old_pred"]], _res["alpha"]), flush=True)


class AuthorshipMHM_Attacker(MHM_Attacker):
    """CodeXGLUE/Authorship-Attribution/code/attacker.py:425-700: Python leaves, the raw-text
    victim, the substitutes passed last (`mcmc(tokenizer, code, _label, ..., subs={})`, the call
    form of Authorship-Attribution/code/mhm.py:199-206), and no skip of known variable names
    among the random candidates of mcmc_random."""

    skip_known_uids = False

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lang = "python"

    def mcmc(self, tokenizer, code=None, _label=None, _n_candi=30, _max_iter=100,
             _prob_threshold=0.95, subs={}):
        return super().mcmc(tokenizer, subs, code, _label, _n_candi, _max_iter, _prob_threshold)

    def mcmc_random(self, tokenizer, code=None, _label=None, _n_candi=30, _max_iter=100,
                    _prob_threshold=0.95, subs={}):
        return super().mcmc_random(tokenizer, subs, code, _label, _n_candi, _max_iter,
                                   _prob_threshold)


class GraphMHM_Attacker(MHM_Attacker):
    """GraphCodeBERT/Defect-detection/code/attacker.py:467-737 over the GraphModel victim: the
    Devign chain (C leaves, same call form as mhm_attack.py:198-205), every candidate featurised
    by the GCB convert_code_to_features (:30-63: ' '.join(code.split()), run_parser data flow,
    GraphCodeDataset mask) and mcmc_random labelled "Ori_MHM" (:608,614)."""

    random_type = "Ori_MHM"


class GraphAuthorshipMHM_Attacker(AuthorshipMHM_Attacker):
    """GraphCodeBERT/Authorship-Attribution/code/attacker.py:479-741 over the GraphModel victim
    (mhm_attack.py:203-210 call form: mcmc(tokenizer, code, _label=..., subs=...)): Python
    leaves, candidates featurised with run.py's data flow (attacker.py:52-85 imports
    run.extract_dataflow), known names skipped in both modes (:634, :695) and mcmc_random
    labelled "Ori_MHM" (:613,619)."""

    skip_known_uids = True
    random_type = "Ori_MHM"


class CloneMHM_Attacker(MHM_Attacker):
    """CodeXGLUE/Clone-detection-BigCloneBench/code/attacker.py:469-800: the chain perturbs code1
    of a pair and every query is the pair [features(candidate code1) | features(code2)].
      * signature mcmc(example, substituions, tokenizer, code_pair, _label, ...) with code_pair =
        (id1, id2, code1, code2) (:478, :573); the call first queries the dataset example and
        returns {'succ': None, ...} when the victim misclassifies it (:485-512);
      * candidates: ' '.join(text.split()) tokenised and cut to block_size - 2 per half
        (run.py convert_examples_to_features, :689-699), code2's half fixed (:504-505);
      * the results carry "orig_label" (:565,571); mcmc_random is "Ori_MHM" (:659,666)."""

    random_type = "Ori_MHM"

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lang = "java"

    def mcmc(self, example, substituions, tokenizer, code_pair, _label=None, _n_candi=30,
             _max_iter=100, _prob_threshold=0.95):
        return answer(self.classifier, self.chain_gen(tokenizer, substituions, code_pair, _label,
                                                      example, _n_candi, _max_iter,
                                                      _prob_threshold, False, random))

    def mcmc_random(self, example, substituions, tokenizer, code_pair, _label=None, _n_candi=30,
                    _max_iter=100, _prob_threshold=0.95):
        return answer(self.classifier, self.chain_gen(tokenizer, substituions, code_pair, _label,
                                                      example, _n_candi, _max_iter,
                                                      _prob_threshold, True, random))

    def chain_gen(self, tokenizer, substituions, code, _label, example, _n_candi, _max_iter,
                  _prob_threshold, original, rng):
        """code = the pair tuple; the chain's text is code1 (code_pair[2])."""
        logits, preds = yield self.classifier.prepare([example])
        orig_label = preds[0]
        if orig_label != _label_of(example):
            return {"succ": None, "tokens": None, "raw_tokens": None}
        replace = self._replace_uid_random if original else self._replace_uid
        kind = self.random_type if original else "MHM"
        # _tokenize / candidates with tokenizer_mlm (:503, :692); the chain's text is code1
        res = yield from self._run_gen(self.tokenizer_mlm, substituions, code[2], _label,
                                       _n_candi, _max_iter, _prob_threshold, replace, kind, rng,
                                       ctx=self._pair_ctx(code))
        if res["succ"] is not None:
            res["orig_label"] = orig_label
        return res

    def _pair_ctx(self, code_pair):
        """code2's fixed half: its ids (tokenize(' '.join(code2.split()))[:block-2])."""
        ids2, lens2 = self.tokenizer_mlm.featurize([code_pair[3]], self.args.block_size)
        return ids2[0], int(lens2[0])

    def _candidates_request(self, ex, tok, _tokens, pops, L, ctx=None):
        m = self.classifier
        ids2, len2 = ctx
        ids0, lens0 = tok.featurize([_tokens], L)
        first = m.prepare_pairs(ids0, lens0, ids2, len2)
        if not pops:
            return first
        if getattr(m, "population_rows", None) is not None:
            rows, lens = m.population_rows(ex, tok, pops, MODE_SINGLE, L)
        else:
            rows, lens = tok.featurize([ex.mutant_text(p, MODE_SINGLE) for p in pops], L)
        return join_payloads([first, m.prepare_pairs(rows, lens, ids2, len2)])


class GraphCloneMHM_Attacker(CloneMHM_Attacker):
    """GraphCodeBERT/clonedetection/code/attacker.py:496-800 over the GraphModel clone victim:
    the CodeBERT clone chain, but every query is convert_code_to_features(candidate code1, code2)
    (:33-73: run_parser data flow of each Java text as is, one graph row per code), the dataset
    label is example[6] (:517), and NEITHER mode skips candidates that already name a variable
    (__replaceUID :704-709 and __replaceUID_random :766-771 have no `c in _uid` test).
    The reference's own driver calls mcmc(example, tokenizer, code_pair, ...) without the
    substitutes (mhm_attack.py:200-206), which raises TypeError; this class keeps the attacker's
    signature, the one the CodeBERT clone driver uses (its mhm_attack.py:195-203)."""

    skip_known_subs = False
    skip_known_uids = False

    def _pair_ctx(self, code_pair):
        from .graph import compact_features, task_features

        f2 = task_features(code_pair[3], self.tokenizer_mlm, 0, self.args, "clone")
        return compact_features(f2) if hasattr(self.tokenizer_mlm, "gcb_features") else f2

    def _candidates_request(self, ex, tok, _tokens, pops, L, ctx=None):
        from .graph import gcb_dataset_from_texts, task_features

        texts = [_tokens] + [ex.mutant_text(p, MODE_SINGLE) for p in pops]
        if hasattr(tok, "gcb_features"):
            feats = gcb_dataset_from_texts(texts, tok, self.args, "clone").c
        else:
            feats = [task_features(t, tok, 0, self.args, "clone") for t in texts]
        return self.classifier.prepare_pair_population(feats, ctx)


class GraphAttacker(Attacker):
    """GraphCodeBERT/Defect-detection/code/attacker.py: the Devign attacker over the GraphModel
    victim; the GA draws 64 children per iteration whatever eval_batch_size is (:246)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.ga_batch = 64


class GraphAuthorshipAttacker(AuthorshipAttacker):
    """GraphCodeBERT/Authorship-Attribution/code/attacker.py: the authorship attacker over the
    GraphModel victim (task 'authorship'); every query — original, importance rows, mutants — is
    featurised with run.py's data flow (DFG_GCB_RUN, attacker.py:18-52), which the victim's
    dataset_from_texts applies.  GA children per iteration: eval_batch_size (:260)."""


class GraphCloneAttacker(CloneAttacker):
    """GraphCodeBERT/clonedetection/code/attacker.py: pairs of data-flow features (the
    CodeBERT clone signatures and code tuple).
      * mutants of code1 and code2 itself are featurised with run_parser's data flow, Java text
        as is (attacker.py:33-72); the dataset example comes from run.py (pair_features
        original=True), so the first query of an attack sees different features than its
        mutants (the reference's quirk);
      * importance rows: ' '.join(words) of code1 against the features of
        ' '.join(get_identifiers(code2)[1]) (processed_code_2, :366-378 -> :84-85);
      * GA children per iteration: eval_batch_size (:261)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.ga_batch = None

    def _pair_state(self, code):
        from .graph import compact_features, task_features

        tok, args = self.tokenizer_tgt, self.args
        _, toks2 = get_identifiers(code[3], self.lang)
        f2 = task_features(code[3], tok, 0, args, "clone")
        f2w = task_features(" ".join(toks2), tok, 0, args, "clone")
        if hasattr(tok, "gcb_features"):  # code2 compact once per example
            return compact_features(f2), compact_features(f2w)
        return f2, f2w

    def _feats(self, texts):
        """code1 query features of many texts (run_parser data flow, Java text as is)."""
        from .graph import gcb_dataset_from_texts, task_features

        tok, args = self.tokenizer_tgt, self.args
        if hasattr(tok, "gcb_features"):
            return gcb_dataset_from_texts(texts, tok, args, "clone").c
        return [task_features(t, tok, 0, args, "clone") for t in texts]

    def _population(self, ex, pops, mode):
        feats = self._feats([ex.mutant_text(p, mode) for p in pops])
        return self.model_tgt.prepare_pair_population(feats, self._code2[0])

    def _importance_payload(self):
        f2w = self._code2[1]

        def build(word_lists):
            feats = self._feats([" ".join(w) for w in word_lists])
            return self.model_tgt.prepare_pair_population(feats, f2w)

        return build
