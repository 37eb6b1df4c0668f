"""ORACLE — test infrastructure only (see oracle/roberta_cpu.py header for the import rule).

CPU restatement of ALERT's masked-LM substitute generation for one example, line for line from
CodeXGLUE/Defect-detection/preprocess/get_substitutes.py:54-137 and the helpers it calls
(utils.py:174-189 _tokenize, :192-206 get_identifier_posistions_from_code, :209-248
get_bpe_substitues, :251-277 get_substitues), on the PyTorch-CPU fp32 RoBERTa restatement
(roberta_cpu.py, pinned to the installed transformers).  Inputs the reference derives with
tree-sitter (the code tokens and the DFG identifier list) are passed in: their parity is tested on
their own (tests/test_host.py).

Two deliberate restatement choices, both arithmetic-neutral:
  * the 60 candidate re-encodes of one occurrence run as one batch of 60 (rows of a batch are
    independent, so this equals 60 batch-1 calls up to float rounding);
  * substitute order inside each list comes from Python set iteration in the reference (hash-seed
    dependent, get_substitutes.py:122-137): callers compare the lists as sets.
`trace` (optional dict) receives the intermediate top-k ids / scores and cosine ranks so tests can
tell a genuine mismatch from a near tie at a ranking boundary.
"""
from __future__ import annotations

import torch

from . import roberta_cpu as rc


def _tokenize(seq, tokenizer):
    """utils.py:174-189 (tokens, not ids)."""
    seq = seq.replace("\n", "")
    words = seq.split(" ")
    sub_words, keys, index = [], [], 0
    for word in words:
        sub = tokenizer.tokenize(word)
        sub_words += sub
        keys.append([index, index + len(sub)])
        index += len(sub)
    return words, sub_words, keys


def get_identifier_posistions_from_code(words_list, variable_names):
    positions = {}
    for name in variable_names:
        for index, token in enumerate(words_list):
            if name == token:
                positions.setdefault(name, []).append(index)
    return positions


@torch.no_grad()
def get_bpe_substitues(substitutes, tokenizer, sd, layers, trace=None):
    """utils.py:209-248 (mlm_model(all_substitutes) has no attention_mask)."""
    substitutes = substitutes[0:12, 0:4]
    all_substitutes = []
    for i in range(substitutes.size(0)):
        if len(all_substitutes) == 0:
            lev_i = substitutes[i]
            all_substitutes = [[int(c)] for c in lev_i]
        else:
            lev_i = []
            for all_sub in all_substitutes[:24]:
                for j in substitutes[i]:
                    lev_i.append(all_sub + [int(j)])
            all_substitutes = lev_i
    c_loss = torch.nn.CrossEntropyLoss(reduction="none")
    all_substitutes = torch.tensor(all_substitutes)[:24]
    N, L = all_substitutes.size()
    word_predictions = rc.mlm_logits(sd, all_substitutes.numpy(), layers=layers, no_mask=True)
    ppl = c_loss(word_predictions.view(N * L, -1), all_substitutes.view(-1))
    ppl = torch.exp(torch.mean(ppl.view(N, L), dim=-1))
    if trace is not None:
        trace.setdefault("bpe", []).append((all_substitutes.numpy().copy(), ppl.numpy().copy()))
    _, word_list = torch.sort(ppl)
    final_words = []
    for i in word_list:
        tokens = tokenizer.convert_ids_to_tokens([int(t) for t in all_substitutes[i]])
        final_words.append(tokenizer.convert_tokens_to_string(tokens))
    return final_words


def get_substitues(substitutes, tokenizer, sd, layers, use_bpe, substitutes_score=None,
                   threshold=3.0, trace=None):
    """utils.py:251-277."""
    words = []
    sub_len, k = substitutes.size()
    if sub_len == 0:
        return words
    if sub_len == 1:
        for (i, j) in zip(substitutes[0], substitutes_score[0]):
            if threshold != 0 and j < threshold:
                break
            words.append(tokenizer.decode([int(i)]))
    elif use_bpe == 1:
        words = get_bpe_substitues(substitutes, tokenizer, sd, layers, trace)
    return words


@torch.no_grad()
def substitutes_for_example(sd, tokenizer, code_tokens, variable_names, is_valid, block_size=512,
                            layers=12, trace=None, cosine=True):
    """get_substitutes.py:54-137 for one item; returns the `substitutes` dict (lists in set
    order).  is_valid(name) -> bool is is_valid_variable_name(name, 'c').  cosine=False restates
    GraphCodeBERT/Defect-detection/preprocess/get_substitutes.py:72-134 (cosine block commented
    out: get_substitues over all 60 candidates, use_bpe 1, threshold 0)."""
    processed_code = " ".join(code_tokens)
    words, sub_words, keys = _tokenize(processed_code, tokenizer)
    sub_words = [tokenizer.cls_token] + sub_words[:block_size - 2] + [tokenizer.sep_token]
    input_ids_ = torch.tensor([tokenizer.convert_tokens_to_ids(sub_words)])
    logits = rc.mlm_logits(sd, input_ids_.numpy(), layers=layers, no_mask=True)[0]
    word_pred_scores_all, word_predictions = torch.topk(logits, 60, -1)
    word_predictions = word_predictions[1:len(sub_words) + 1, :]
    word_pred_scores_all = word_pred_scores_all[1:len(sub_words) + 1, :]
    if trace is not None:
        trace["ids"] = input_ids_[0].numpy().copy()
        trace["topk_ids"] = word_predictions.numpy().copy()
        trace["topk_scores"] = word_pred_scores_all.numpy().copy()
        trace["logits"] = logits
        trace["sims"] = []
    names_positions_dict = get_identifier_posistions_from_code(words, variable_names)
    orig_embeddings = rc.encoder_forward(sd, input_ids_.numpy(), layers=layers, no_mask=True)
    cos = torch.nn.CosineSimilarity(dim=1, eps=1e-6)
    variable_substitue_dict = {}
    for tgt_word in names_positions_dict.keys():
        if not is_valid(tgt_word):
            continue
        all_substitues = []
        for one_pos in names_positions_dict[tgt_word]:
            k0, k1 = keys[one_pos]
            if k0 >= word_predictions.size()[0]:
                continue
            substitutes = word_predictions[k0:k1]
            word_pred_scores = word_pred_scores_all[k0:k1]
            if not cosine:
                all_substitues += get_substitues(substitutes, tokenizer, sd, layers, 1,
                                                 word_pred_scores, 0, trace)
                continue
            orig_word_embed = orig_embeddings[0][k0 + 1:k1 + 1]
            subwords_leng, nums_candis = substitutes.size()
            new_ids = input_ids_.repeat(nums_candis, 1)
            new_ids[:, k0 + 1:k1 + 1] = substitutes.t()
            new_emb = rc.encoder_forward(sd, new_ids.numpy(), layers=layers, no_mask=True)
            sims = []
            for i in range(nums_candis):
                new_word_embed = new_emb[i][k0 + 1:k1 + 1]
                sims.append((i, sum(cos(orig_word_embed, new_word_embed)) / subwords_leng))
            if trace is not None:
                trace["sims"].append((tgt_word, one_pos, [float(v) for _, v in sims],
                                      [tuple(int(x) for x in c) for c in substitutes.t()]))
            sims = sorted(sims, key=lambda x: x[1], reverse=True)
            similar_substitutes, similar_word_pred_scores = [], []
            for i in range(int(nums_candis / 2)):
                similar_substitutes.append(substitutes[:, sims[i][0]].reshape(subwords_leng, -1))
                similar_word_pred_scores.append(
                    word_pred_scores[:, sims[i][0]].reshape(subwords_leng, -1))
            similar_substitutes = torch.cat(similar_substitutes, 1)
            similar_word_pred_scores = torch.cat(similar_word_pred_scores, 1)
            all_substitues += get_substitues(similar_substitutes, tokenizer, sd, layers, 1,
                                             similar_word_pred_scores, 0, trace)
        for tmp_substitue in set(all_substitues):
            if tmp_substitue.strip() in variable_names:
                continue
            if not is_valid(tmp_substitue.strip()):
                continue
            variable_substitue_dict.setdefault(tgt_word, []).append(tmp_substitue)
    return variable_substitue_dict
