"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

Text-driven restatement of the MHM-NS baseline, CodeXGLUE/Defect-detection/code/attacker.py:
  mcmc :466-537 (iteration loop, old_uids chains, uid / substitute-dict renames, result dicts)
  __replaceUID :610-672 (random.sample of the variable and of <= n_candi substitutes, candidate 0 =
  the unmodified code, one get_results over all candidates, first flip wins, otherwise the
  acceptance test alpha = (1 - p_min + 1e-10) / (1 - p_0 + 1e-10); the reported candidate is the
  LAST loop index, :662-670).
Every candidate is built with oracle.featurize_ref.get_example and featurised with the
transformers tokenizer (featurize_ref.convert_code_to_features) and scored through a caller
Victim (oracle.attack_ref.Victim, or oracle.graph_ref.GraphTextVictim for the GraphCodeBERT
copies).  `is_uid` is passed in (utils.py:481-511 deny lists are data, checked on their own in
tests/test_host.py).

The other five copies of the class differ from the Devign one only in (all read as text):
  * which candidates are dropped for already naming a variable (`if c in _uid.keys()`):
    skip_known_subs (__replaceUID) / skip_known (__replaceUID_random) —
    CodeXGLUE Authorship-Attribution attacker.py:591 / none; GraphCodeBERT Defect-detection
    :629 / :691; GraphCodeBERT Authorship-Attribution :634 / :695; CodeXGLUE
    Clone-detection-BigCloneBench :681 / :748; GraphCodeBERT clonedetection: neither
    (:704-709, :766-771);
  * mcmc_random's attack_type: "MHM-Origin" (CodeXGLUE Devign / Authorship) or "Ori_MHM"
    (the clone and GraphCodeBERT copies);
  * the clone copies (Clone-detection-BigCloneBench :478-571, clonedetection :505-597) first
    query the dataset example (`pair_example`), return {'succ': None} when it is misclassified,
    and add "orig_label" to their results; the victim then scores pairs (Victim(task="clone",
    code2=...) / GraphTextVictim(task="gcb_clone", code2=...)).
"""
from __future__ import annotations

import copy
import random

from . import featurize_ref as fr
from .attack_ref import _positions, _words_of


def _replace_uid(victim, is_uid, tokens, label, uid, substitute_dict, n_candi, prob_threshold,
                 idx2token=None, lang="c", skip_known=True, skip_known_subs=True):
    selected_uid = random.sample(list(substitute_dict.keys()), 1)[0]
    candi_token = [selected_uid]
    candi_tokens = [copy.deepcopy(tokens)]
    # __replaceUID_random (:675-738, mcmc_random) draws from the whole vocabulary instead
    pool = random.sample(idx2token, n_candi) if idx2token is not None else \
        random.sample(substitute_dict[selected_uid], min(n_candi, len(substitute_dict[selected_uid])))
    for c in pool:
        # the Authorship-Attribution __replaceUID_random has no known-name skip (its :649-655)
        skip = skip_known_subs if idx2token is None else skip_known
        if skip and c in uid.keys():
            continue
        if is_uid(c):
            candi_token.append(c)
            candi_tokens.append(fr.get_example(copy.deepcopy(tokens), selected_uid, c, lang))
    prob, pred = victim.texts(candi_tokens)
    for i in range(len(candi_token)):
        if pred[i] != label:
            return {"status": "s", "alpha": 1, "tokens": candi_tokens[i],
                    "old_uid": selected_uid, "new_uid": candi_token[i],
                    "old_prob": prob[0], "new_prob": prob[i],
                    "old_pred": pred[0], "new_pred": pred[i],
                    "nb_changed_pos": tokens.count(selected_uid)}
    candi_idx = 0
    min_prob = 1.0
    for idx, a_prob in enumerate(prob[1:]):
        if a_prob[label] < min_prob:
            candi_idx = idx + 1
            min_prob = a_prob[label]
    alpha = (1 - prob[candi_idx][label] + 1e-10) / (1 - prob[0][label] + 1e-10)
    status = "r" if (random.uniform(0, 1) > alpha or alpha < prob_threshold) else "a"
    return {"status": status, "alpha": alpha, "tokens": candi_tokens[i],
            "old_uid": selected_uid, "new_uid": candi_token[i],
            "old_prob": prob[0], "new_prob": prob[i],
            "old_pred": pred[0], "new_pred": pred[i],
            "nb_changed_pos": tokens.count(selected_uid)}


def mcmc(victim, is_uid, substituions, code, label, n_candi=30, max_iter=100, prob_threshold=0.95,
         idx2token=None, lang="c", skip_known=True, skip_known_subs=True, random_type="MHM-Origin",
         pair_example=None):
    """mcmc (:466-537); with idx2token, mcmc_random (:539-608).  lang="python", skip_known=False
    with a Victim(task="authorship") is the Authorship-Attribution copy
    (CodeXGLUE/Authorship-Attribution/code/attacker.py:440-666: Python leaves and get_example,
    raw-text features, argmax predictions).  pair_example: the clone copies' first query (the
    dataset example's ids, handed to victim.ids); `code` is then code1."""
    attack_type = random_type if idx2token is not None else "MHM"
    orig_label = None
    if pair_example is not None:
        _, preds = victim.ids(pair_example)
        orig_label = preds[0]
        if orig_label != label:
            return {"succ": None, "tokens": None, "raw_tokens": None}
    prog_length, words = _words_of(code, lang)
    raw_tokens = copy.deepcopy(words)
    uid = _positions(words, list(substituions.keys()))
    if len(uid) <= 0:
        return {"succ": None, "tokens": None, "raw_tokens": None}
    variable_substitue_dict = {w: substituions[w] for w in uid.keys()}
    if len(variable_substitue_dict) <= 0:
        return {"succ": None, "tokens": None, "raw_tokens": None}
    old_uids = {}
    old_uid = ""
    res = None
    for iteration in range(1, 1 + max_iter):
        res = _replace_uid(victim, is_uid, code, label, uid, variable_substitue_dict, n_candi,
                           prob_threshold, idx2token, lang, skip_known, skip_known_subs)
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
                for u in old_uids.keys():
                    replace_info[u] = old_uids[u][-1]
                    nb_changed_pos += len(uid[old_uids[u][-1]])
                out = {"succ": True, "tokens": code, "raw_tokens": raw_tokens,
                       "prog_length": prog_length, "new_pred": res["new_pred"], "is_success": 1,
                       "old_uid": old_uid, "nb_changed_var": len(old_uids),
                       "nb_changed_pos": nb_changed_pos, "replace_info": replace_info,
                       "score_info": res["old_prob"][0] - res["new_prob"][0],
                       "attack_type": attack_type}
                if pair_example is not None:
                    out["orig_label"] = orig_label
                return out
    replace_info, nb_changed_pos = {}, 0
    for u in old_uids.keys():
        replace_info[u] = old_uids[u][-1]
        nb_changed_pos += len(uid[old_uids[u][-1]])
    out = {"succ": False, "tokens": res["tokens"], "raw_tokens": None,
           "prog_length": prog_length, "new_pred": res["new_pred"], "is_success": -1,
           "old_uid": old_uid, "nb_changed_var": len(old_uids),
           "nb_changed_pos": nb_changed_pos, "replace_info": replace_info,
           "score_info": res["old_prob"][0] - res["new_prob"][0], "attack_type": attack_type}
    if pair_example is not None:
        out["orig_label"] = orig_label
    return out
