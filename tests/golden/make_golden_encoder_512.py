"""Generates tests/golden/encoder_golden_512.npz — golden vectors for the three victim heads at the
block size the attacks run at (gi_attack.py:129-131: block_size = min(512, max_position_embeddings
- 2) ... the 510/512-token rows of the Devign GA config, BASELINE configs[1]).

Same provenance as make_golden_encoder.py: the installed transformers 5.15.0 RoBERTa (third-party
code the reference calls at CodeXGLUE/Defect-detection/code/model.py:24-34, not the reference
itself), built from a LOCAL RobertaConfig with eager attention in fp32 and the seeded synthetic
weights of apmc_amd.weights.synthetic_state_dict.  Only inputs and outputs are stored.

Rows per head (L = 512): one full 512-token row, one 510, two ragged rows (300, 129), a full row
with literal <pad> ids inside it (masked and skipped by the position ids) and a 200-token row.
The clone head scores rows (2i, 2i + 1) as one pair (Clone-detection-BigCloneBench/code/
model.py:22-30), so its 6 rows are 3 pairs of 2 x 512.

Run:  python tests/golden/make_golden_encoder_512.py
"""
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import _apmc  # noqa: E402,F401
from apmc_amd.weights import synthetic_state_dict, to_hf_state_dict  # noqa: E402
from make_golden_encoder import config  # noqa: E402
from transformers import RobertaForSequenceClassification, RobertaModel  # noqa: E402

OUT = pathlib.Path(__file__).with_name("encoder_golden_512.npz")
L = 512
LENS = [512, 510, 300, 129, 512, 200]
PAD_ROW, PAD_COLS = 4, (5, 6, 333)


def make_ids(rng):
    ids = np.full((len(LENS), L), 1, dtype=np.int64)
    for i, ln in enumerate(LENS):
        ids[i, 0] = 0
        ids[i, 1:ln - 1] = rng.integers(4, 50264, size=ln - 2)
        ids[i, ln - 1] = 2
    ids[PAD_ROW, list(PAD_COLS)] = 1
    return ids


def head(sd, feat, kind):
    x = feat[:, 0, :]
    if kind == "pair2":
        x = x.reshape(-1, 768 * 2)
    x = torch.tanh(torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.dense.weight"]),
                                              torch.from_numpy(sd["classifier.dense.bias"])))
    x = torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.out_proj.weight"]),
                                   torch.from_numpy(sd["classifier.out_proj.bias"]))
    return torch.softmax(x, dim=-1)


def main():
    torch.manual_seed(0)
    rng = np.random.default_rng(512)
    out = {}
    with torch.no_grad():
        # Devign (sigmoid head on RobertaForSequenceClassification), seed 0
        sd = synthetic_state_dict(seed=0, head="sigmoid1", num_labels=1)
        m = RobertaForSequenceClassification(config(1)).eval()
        _, unexpected = m.load_state_dict(to_hf_state_dict(sd, "seqcls"), strict=False)
        assert not unexpected, unexpected
        ids = make_ids(rng)
        t = torch.from_numpy(ids)
        r = m(t, attention_mask=t.ne(1), output_hidden_states=True)
        out["devign_ids"] = ids.astype(np.int32)
        out["devign_probs"] = torch.sigmoid(r.logits).numpy().astype(np.float32)
        out["devign_cls"] = r.hidden_states[-1][:, 0, :].numpy().astype(np.float32)

        # Authorship (66-way softmax on RobertaModel features), seed 1
        sd = synthetic_state_dict(seed=1, head="softmaxN", num_labels=66)
        enc = RobertaModel(config(66), add_pooling_layer=False).eval()
        enc.load_state_dict(to_hf_state_dict(sd, "model"), strict=False)
        ids = make_ids(rng)
        t = torch.from_numpy(ids)
        out["aa_ids"] = ids.astype(np.int32)
        out["aa_probs"] = head(sd, enc(input_ids=t, attention_mask=t.ne(1))[0], "softmaxN").numpy().astype(np.float32)

        # BigCloneBench (pair head), seed 2
        sd = synthetic_state_dict(seed=2, head="pair2", num_labels=2)
        enc = RobertaModel(config(2), add_pooling_layer=False).eval()
        enc.load_state_dict(to_hf_state_dict(sd, "model"), strict=False)
        ids = make_ids(rng)
        t = torch.from_numpy(ids)
        out["clone_ids"] = ids.astype(np.int32)
        out["clone_probs"] = head(sd, enc(input_ids=t, attention_mask=t.ne(1))[0], "pair2").numpy().astype(np.float32)

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
