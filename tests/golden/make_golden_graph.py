"""Generates tests/golden/graph_golden.npz — golden vectors for the GraphCodeBERT forward.

GraphCodeBERT's Model.forward (GraphCodeBERT/Defect-detection/code/model.py:24-45 and
clonedetection/code/model.py:41-64) averages each data-flow node's code-token embeddings
(nodes_to_token_mask / (sum + 1e-10), einsum) and calls RobertaModel with inputs_embeds, the
[L, L] graph-guided mask and explicit position ids.  The installed transformers 5.15.0 (third-party
code, not the reference; LOCAL config, eager attention, fp32, the seeded synthetic weights of
apmc_amd.weights) runs that encoder here at L = 640 (code_length 512 + data_flow_length 128).
transformers 5 no longer expands a 3-D mask, so the mask goes in as the 4-D additive float mask
(1 - m) * finfo(float32).min that the reference-era get_extended_attention_mask built from it.

Inputs: the data-flow features of Devign fixture functions (product featuriser; the features are
pinned separately against oracle/graph_ref.py), chosen with at most 510 code tokens so every
position id stays inside the 514-row position table.  Stored: ids, positions, the bit-packed
masks and the head outputs; tests regenerate the weights from the seed.

Run:  python tests/golden/make_golden_graph.py
"""
import json
import pathlib
import sys
import types

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import _apmc  # noqa: E402,F401
from apmc_amd.graph import convert_code_to_features, graph_mask, pack_mask  # noqa: E402
from apmc_amd.host import Tokenizer  # noqa: E402
from apmc_amd.weights import synthetic_state_dict, to_hf_state_dict  # noqa: E402
from make_golden_encoder import config  # noqa: E402
from transformers import RobertaModel  # noqa: E402

OUT = pathlib.Path(__file__).with_name("graph_golden.npz")
ARGS = types.SimpleNamespace(code_length=512, data_flow_length=128)


def features(codes):
    tok = Tokenizer()
    ids, pos, masks = [], [], []
    for code in codes:
        f = convert_code_to_features(code, tok, 0, ARGS)
        ids.append(f.input_ids)
        pos.append(f.position_idx)
        masks.append(graph_mask(f.input_ids, f.position_idx, f.dfg_to_code, f.dfg_to_dfg))
    return np.array(ids), np.array(pos), np.stack(masks)


def gcb_forward(enc, sd, ids, pos, mask, kind):
    ids_t, pos_t = torch.from_numpy(ids).long(), torch.from_numpy(pos).long()
    m = torch.from_numpy(mask)
    nodes_mask, token_mask = pos_t.eq(0), pos_t.ge(2)
    emb = enc.embeddings.word_embeddings(ids_t)
    n2t = nodes_mask[:, :, None] & token_mask[:, None, :] & m
    n2t = n2t / (n2t.sum(-1) + 1e-10)[:, :, None]
    avg = torch.einsum("abc,acd->abd", n2t, emb)
    emb = emb * (~nodes_mask)[:, :, None] + avg * nodes_mask[:, :, None]
    add = (~m[:, None, :, :]).float() * torch.finfo(torch.float32).min
    h = enc(inputs_embeds=emb, attention_mask=add, position_ids=pos_t)[0]
    x = h[:, 0, :]
    if kind == "pair2":
        x = x.reshape(-1, 768 * 2)
    x = torch.tanh(torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.dense.weight"]),
                                              torch.from_numpy(sd["classifier.dense.bias"])))
    x = torch.nn.functional.linear(x, torch.from_numpy(sd["classifier.out_proj.weight"]),
                                   torch.from_numpy(sd["classifier.out_proj.bias"]))
    out = torch.sigmoid(x) if kind == "sigmoid1" else torch.softmax(x, dim=-1)
    return out.numpy().astype(np.float32), h[:, 0, :].numpy().astype(np.float32)


def main():
    torch.manual_seed(0)
    codes = []
    with open(ROOT / "data" / "devign" / "test_subs_0_400.jsonl") as f:
        for line in f:
            codes.append(json.loads(line)["func"])
    ids, pos, mask = features(codes[:60])
    ok = [i for i in range(len(codes[:60])) if pos[i].max() <= 513]
    # varied sizes: short, medium, long (many nodes), and one with few nodes
    nodes = (pos == 0).sum(1)
    toks = (pos >= 2).sum(1)
    by_size = sorted(ok, key=lambda i: (toks[i], i))
    pick = sorted({by_size[0], by_size[len(by_size) // 3], by_size[2 * len(by_size) // 3],
                   by_size[-1]})
    assert len(pick) == 4, pick
    ids, pos, mask = ids[pick], pos[pick], mask[pick]
    out = {"gcb_ids": ids.astype(np.int32), "gcb_pos": pos.astype(np.int32),
           "gcb_bits": pack_mask(mask), "gcb_pick": np.array(pick, np.int32)}
    for name, seed, head, nl in [("devign", 6, "sigmoid1", 1), ("clone", 7, "pair2", 2)]:
        sd = synthetic_state_dict(seed=seed, head=head, num_labels=nl)
        enc = RobertaModel(config(nl), add_pooling_layer=False).eval()
        missing, unexpected = enc.load_state_dict(to_hf_state_dict(sd, "model"), strict=False)
        assert not unexpected, unexpected
        with torch.no_grad():
            probs, cls = gcb_forward(enc, sd, ids, pos, mask, head)
        out[f"gcb_{name}_probs"] = probs
        out[f"gcb_{name}_cls"] = cls
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()}, "picked", pick,
          "tokens", toks[pick].tolist(), "nodes", nodes[pick].tolist())


if __name__ == "__main__":
    main()
