"""RoBERTa-base weights for the engine: synthetic (seeded) construction and HF state-dict mapping.

No checkpoint or network is available, so the victim and the MLM run on seeded synthetic weights
of the exact codebert-base architecture (vocab 50265, hidden 768, 12 layers x 12 heads, ffn 3072,
max_pos 514, type_vocab 1, pad 1) — the architecture the reference loads with
`RobertaForSequenceClassification.from_pretrained` (CodeXGLUE/Defect-detection/code/gi_attack.py:
122-146) and `RobertaForMaskedLM.from_pretrained` (:150).

Names follow the HF state dict with the architecture prefix stripped ("embeddings.*",
"encoder.layer.{i}.*", "classifier.*", "lm_head.*").  `normalize_state_dict` maps a reference
checkpoint (`Model.state_dict()`: "encoder.roberta.*" / "encoder.classifier.*" for Devign,
"encoder.*" + "classifier.*" for clone / authorship) onto these names.
"""
from __future__ import annotations

import dataclasses

import numpy as np


@dataclasses.dataclass(frozen=True)
class RobertaShape:
    vocab: int = 50265
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 514
    type_vocab: int = 1
    pad_id: int = 1
    ln_eps: float = 1e-5


CODEBERT = RobertaShape()


def synthetic_state_dict(seed: int = 0, shape: RobertaShape = CODEBERT, head: str = "sigmoid1",
                         num_labels: int = 1, with_mlm: bool = False,
                         out_std: float = 0.5) -> dict[str, np.ndarray]:
    """Seeded RoBERTa weights (numpy PCG64; identical on every host of this image).

    Linear / embedding weights ~ N(0, 0.02) (HF _init_weights); biases ~ N(0, 0.02) and LayerNorm
    gamma ~ 1 + N(0, 0.05), beta ~ N(0, 0.02) so that every epilogue term is exercised by the
    parity tests; the classifier out_proj ~ N(0, out_std) so predicted probabilities spread away
    from the 0.5 decision boundary.
    head: "sigmoid1" (Devign), "softmaxN" (authorship, num_labels classes), "pair2" (clone).
    """
    rng = np.random.default_rng(seed)
    H, F, V = shape.hidden, shape.ffn, shape.vocab

    def n(*s, std=0.02):
        return (rng.standard_normal(s, dtype=np.float32) * np.float32(std)).astype(np.float32)

    def gamma(k):
        return (1.0 + rng.standard_normal(k, dtype=np.float32) * np.float32(0.05)).astype(np.float32)

    sd: dict[str, np.ndarray] = {}
    sd["embeddings.word_embeddings.weight"] = n(V, H)
    sd["embeddings.position_embeddings.weight"] = n(shape.max_pos, H)
    sd["embeddings.token_type_embeddings.weight"] = n(shape.type_vocab, H)
    sd["embeddings.LayerNorm.weight"] = gamma(H)
    sd["embeddings.LayerNorm.bias"] = n(H)
    for i in range(shape.layers):
        p = f"encoder.layer.{i}."
        for nm in ("query", "key", "value"):
            sd[p + f"attention.self.{nm}.weight"] = n(H, H)
            sd[p + f"attention.self.{nm}.bias"] = n(H)
        sd[p + "attention.output.dense.weight"] = n(H, H)
        sd[p + "attention.output.dense.bias"] = n(H)
        sd[p + "attention.output.LayerNorm.weight"] = gamma(H)
        sd[p + "attention.output.LayerNorm.bias"] = n(H)
        sd[p + "intermediate.dense.weight"] = n(F, H)
        sd[p + "intermediate.dense.bias"] = n(F)
        sd[p + "output.dense.weight"] = n(H, F)
        sd[p + "output.dense.bias"] = n(H)
        sd[p + "output.LayerNorm.weight"] = gamma(H)
        sd[p + "output.LayerNorm.bias"] = n(H)
    if head != "none":
        in_dim = 2 * H if head == "pair2" else H
        sd["classifier.dense.weight"] = n(H, in_dim)
        sd["classifier.dense.bias"] = n(H)
        sd["classifier.out_proj.weight"] = n(num_labels, H, std=out_std)
        sd["classifier.out_proj.bias"] = n(num_labels)
    if with_mlm:
        sd["lm_head.dense.weight"] = n(H, H)
        sd["lm_head.dense.bias"] = n(H)
        sd["lm_head.layer_norm.weight"] = gamma(H)
        sd["lm_head.layer_norm.bias"] = n(H)
        sd["lm_head.bias"] = n(V)
    return sd


def normalize_state_dict(sd: dict) -> dict[str, np.ndarray]:
    """Map reference / HF checkpoint keys onto the engine's names (see module docstring)."""
    out: dict[str, np.ndarray] = {}
    for k, v in sd.items():
        arr = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        arr = np.ascontiguousarray(arr, dtype=np.float32)
        key = k
        for pre in ("encoder.roberta.", "roberta.", "encoder.encoder.", "encoder.embeddings."):
            if key.startswith(pre):
                if pre == "encoder.encoder.":
                    key = "encoder." + key[len(pre):]
                elif pre == "encoder.embeddings.":
                    key = "embeddings." + key[len(pre):]
                else:
                    key = key[len(pre):]
                break
        if key.startswith("encoder.classifier."):
            key = key[len("encoder."):]
        if key.startswith(("encoder.pooler.", "pooler.")) or key.endswith("position_ids") \
                or key.endswith("token_type_ids") or key == "lm_head.decoder.weight" \
                or key == "lm_head.decoder.bias":
            continue
        out[key] = arr
    return out


def to_hf_state_dict(sd: dict[str, np.ndarray], arch: str = "seqcls") -> dict:
    """Engine names -> HF module names (arch "seqcls": RobertaForSequenceClassification,
    "mlm": RobertaForMaskedLM, "model": RobertaModel).  Used only by tests/golden generation."""
    import torch

    out = {}
    for k, v in sd.items():
        if k.startswith(("embeddings.", "encoder.")):
            key = k if arch == "model" else "roberta." + k
        elif k.startswith("classifier."):
            if arch != "seqcls":
                continue
            key = k
        elif k.startswith("lm_head."):
            if arch != "mlm":
                continue
            key = k
        else:
            continue
        out[key] = torch.from_numpy(np.array(v))
    if arch == "mlm":
        out["lm_head.decoder.weight"] = out["roberta.embeddings.word_embeddings.weight"]
        out["lm_head.decoder.bias"] = out["lm_head.bias"]
    return out


def load_checkpoint(path) -> dict[str, np.ndarray]:
    """Engine state dict from a local HF model directory or a reference `model.bin`.

    Accepts a directory holding model.safetensors or pytorch_model.bin (the from_pretrained
    layout the reference loads, gi_attack.py:122-152) or a single .bin / .safetensors file (the
    fine-tuned `model.bin` the attack scripts load_state_dict, gi_attack.py:138-146).  Loaded only
    with loaders that execute nothing from the file (safetensors, torch.load(weights_only=True)).
    """
    import pathlib

    p = pathlib.Path(path)
    if p.is_dir():
        for name in ("model.safetensors", "pytorch_model.bin", "model.bin"):
            if (p / name).exists():
                p = p / name
                break
        else:
            raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")
    if p.suffix == ".safetensors":
        from safetensors.numpy import load_file

        raw = load_file(str(p))
    else:
        import torch

        raw = torch.load(str(p), map_location="cpu", weights_only=True)
    return normalize_state_dict(raw)
