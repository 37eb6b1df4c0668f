"""Generates tests/golden/encoder_golden.npz — golden vectors for the victim-scoring path.

The arithmetic the reference calls at its query boundary is HuggingFace transformers' RoBERTa
(CodeXGLUE/Defect-detection/code/model.py:25 -> RobertaForSequenceClassification; MLM at
CodeXGLUE/Defect-detection/preprocess/get_substitutes.py:62).  The installed transformers 5.15.0 is
third-party code (not the reference), built here from a LOCAL RobertaConfig (never
from_pretrained; no network) with eager attention, fp32, and the seeded synthetic weights of
apmc_amd.weights.synthetic_state_dict.  Only inputs and outputs are stored; tests regenerate the
weights from the same seed.

Run:  python tests/golden/make_golden_encoder.py
"""
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import _apmc  # noqa: E402,F401
from apmc_amd.weights import synthetic_state_dict, to_hf_state_dict  # noqa: E402
from transformers import (RobertaConfig, RobertaForMaskedLM, RobertaForSequenceClassification,  # noqa: E402
                          RobertaModel)

OUT = pathlib.Path(__file__).with_name("encoder_golden.npz")


def config(num_labels=1):
    c = RobertaConfig(vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                      num_attention_heads=12, intermediate_size=3072, max_position_embeddings=514,
                      type_vocab_size=1, pad_token_id=1, bos_token_id=0, eos_token_id=2,
                      layer_norm_eps=1e-5, num_labels=num_labels, hidden_act="gelu",
                      hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    c._attn_implementation = "eager"
    return c


def make_ids(rng, n, L, lens, mid_pad_row=None):
    ids = np.full((n, L), 1, dtype=np.int64)
    for i, ln in enumerate(lens):
        ids[i, 0] = 0
        ids[i, 1:ln - 1] = rng.integers(4, 50264, size=ln - 2)
        ids[i, ln - 1] = 2
    if mid_pad_row is not None:
        ids[mid_pad_row, 5] = 1  # a literal <pad> inside a sequence (masked + position-skipped)
    return ids


def main():
    torch.manual_seed(0)
    rng = np.random.default_rng(1234)
    out = {}

    # --- Devign victim (sigmoid head), seed 0
    sd = synthetic_state_dict(seed=0, head="sigmoid1", num_labels=1)
    m = RobertaForSequenceClassification(config(1)).eval()
    missing, unexpected = m.load_state_dict(to_hf_state_dict(sd, "seqcls"), strict=False)
    assert not unexpected, unexpected
    assert all("position_ids" in k or "token_type_ids" in k for k in missing), missing
    L = 64
    lens = [64, 40, 17, 3, 64, 33]
    ids = make_ids(rng, len(lens), L, lens, mid_pad_row=4)
    with torch.no_grad():
        t = torch.from_numpy(ids)
        r = m(t, attention_mask=t.ne(1), output_hidden_states=True)
        probs = torch.sigmoid(r.logits).numpy()
        cls = r.hidden_states[-1][:, 0, :].numpy()
    out["devign_ids"] = ids.astype(np.int32)
    out["devign_probs"] = probs.astype(np.float32)
    out["devign_cls"] = cls.astype(np.float32)

    # --- Authorship victim (66-way softmax head on RobertaModel features), seed 1
    sd = synthetic_state_dict(seed=1, head="softmaxN", num_labels=66)
    enc = RobertaModel(config(66), add_pooling_layer=False).eval()
    enc.load_state_dict(to_hf_state_dict(sd, "model"), strict=False)
    L = 48
    lens = [48, 20, 31, 5]
    ids = make_ids(rng, len(lens), L, lens)
    with torch.no_grad():
        t = torch.from_numpy(ids)
        feat = enc(input_ids=t, attention_mask=t.ne(1))[0]
        # Authorship-Attribution/code/model.py:22-29 (dropout inactive in eval)
        x = feat[:, 0, :]
        x = torch.tanh(torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.dense.weight"]),
                                                  torch.from_numpy(sd["classifier.dense.bias"])))
        x = torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.out_proj.weight"]),
                                       torch.from_numpy(sd["classifier.out_proj.bias"]))
        probs = torch.softmax(x, dim=-1).numpy()
    out["aa_ids"] = ids.astype(np.int32)
    out["aa_probs"] = probs.astype(np.float32)

    # --- Clone victim (pair head: rows 2i, 2i+1 are one pair), seed 2
    sd = synthetic_state_dict(seed=2, head="pair2", num_labels=2)
    enc = RobertaModel(config(2), add_pooling_layer=False).eval()
    enc.load_state_dict(to_hf_state_dict(sd, "model"), strict=False)
    L = 32
    lens = [32, 12, 25, 32]
    ids = make_ids(rng, len(lens), L, lens)
    with torch.no_grad():
        t = torch.from_numpy(ids)
        feat = enc(input_ids=t, attention_mask=t.ne(1))[0]
        # Clone-detection-BigCloneBench/code/model.py:22-30
        x = feat[:, 0, :].reshape(-1, 768 * 2)
        x = torch.tanh(torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.dense.weight"]),
                                                  torch.from_numpy(sd["classifier.dense.bias"])))
        x = torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.out_proj.weight"]),
                                       torch.from_numpy(sd["classifier.out_proj.bias"]))
        probs = torch.softmax(x, dim=-1).numpy()
    out["clone_ids"] = ids.astype(np.int32)
    out["clone_probs"] = probs.astype(np.float32)

    # --- MLM top-60 (substitute generation), seed 3
    sd = synthetic_state_dict(seed=3, head="none", with_mlm=True)
    mlm = RobertaForMaskedLM(config(1)).eval()
    mlm.load_state_dict(to_hf_state_dict(sd, "mlm"), strict=False)
    L = 24
    ids = make_ids(rng, 1, L, [L])
    with torch.no_grad():
        logits = mlm(torch.from_numpy(ids))[0].squeeze(0)
        sc, ix = torch.topk(logits, 60, -1)
        hid = mlm.roberta(torch.from_numpy(ids))[0].squeeze(0)
    out["mlm_ids"] = ids.astype(np.int32)
    out["mlm_top_scores"] = sc.numpy().astype(np.float32)
    out["mlm_top_ids"] = ix.numpy().astype(np.int32)
    out["mlm_hidden"] = hid.numpy().astype(np.float32)

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
