"""ORACLE — test infrastructure only.  CPU restatement (PyTorch-CPU, fp32, eager) of the victim
scoring the reference performs.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / CPU baseline; the product path never does.

What it restates (reference file:line; the encoder math is HF transformers RoBERTa, which the
reference reaches at CodeXGLUE/Defect-detection/code/model.py:25):
  - Model.forward / get_results of the Devign victim   CodeXGLUE/Defect-detection/code/model.py:24-59
  - clone head (pair of CLS vectors, 1536->768->2)     CodeXGLUE/Clone-detection-BigCloneBench/code/model.py:13-53
  - authorship head (768->768->66)                     CodeXGLUE/Authorship-Attribution/code/model.py:13-54
  - RoBERTa eager semantics (installed transformers 5.15.0, modeling_roberta.py:56-183): position ids
    cumsum(ids!=pad)*(ids!=pad)+pad, additive key mask of finfo(float32).min, softmax, exact-erf
    GELU, LayerNorm eps 1e-5.
  - GraphCodeBERT forward with explicit positions and a [L, L] attention mask
    (GraphCodeBERT/Defect-detection/code/model.py:24-45), the mask as a 4-D additive mask.

Pinning: tests/golden/make_golden_encoder.py runs the installed transformers 5.15.0
RobertaForSequenceClassification / RobertaForMaskedLM (third-party arithmetic the reference calls,
built from a local RobertaConfig, never from_pretrained) on seeded weights and commits the outputs;
tests/test_oracle.py checks this restatement against them.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v, dtype=np.float32))


def _ln(x, g, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), g, b, eps)


def position_ids(ids: torch.Tensor, pad: int = 1) -> torch.Tensor:
    m = ids.ne(pad).int()
    return (torch.cumsum(m, dim=1).type_as(m) * m).long() + pad


@torch.no_grad()
def encoder_forward(sd, ids, pos=None, attn_mask=None, layers: int = 12, heads: int = 12,
                    pad: int = 1, eps: float = 1e-5, inputs_embeds=None,
                    no_mask: bool = False) -> torch.Tensor:
    """Last hidden state [n, L, 768] of RoBERTa for int ids [n, L].

    attn_mask: None -> key padding mask ids != pad; else bool [n, L, L] (True = may attend).
    no_mask: the model is called without attention_mask (HF then attends every id, pad included;
    positions still follow the pad rule) — the MLM call sites of get_substitutes.py:62,73,105.
    """
    ids = torch.as_tensor(np.asarray(ids), dtype=torch.long)
    n, L = ids.shape
    if pos is None:
        pos = position_ids(ids, pad)
    else:
        pos = torch.as_tensor(np.asarray(pos), dtype=torch.long)
    if inputs_embeds is None:
        x = _t(sd, "embeddings.word_embeddings.weight")[ids]
    else:
        x = inputs_embeds
    x = x + _t(sd, "embeddings.token_type_embeddings.weight")[0]
    x = x + _t(sd, "embeddings.position_embeddings.weight")[pos]
    x = _ln(x, _t(sd, "embeddings.LayerNorm.weight"), _t(sd, "embeddings.LayerNorm.bias"), eps)
    neg = torch.finfo(torch.float32).min
    if no_mask:
        add = torch.zeros((n, 1, 1, L), dtype=torch.float32)
    elif attn_mask is None:
        add = torch.zeros((n, 1, 1, L), dtype=torch.float32)
        add.masked_fill_(~ids.ne(pad)[:, None, None, :], neg)
    else:
        m = torch.as_tensor(np.asarray(attn_mask), dtype=torch.bool)
        add = torch.zeros((n, 1, L, L), dtype=torch.float32)
        add.masked_fill_(~m[:, None, :, :], neg)
    H = x.shape[-1]
    D = H // heads
    scale = D ** -0.5
    for i in range(layers):
        p = f"encoder.layer.{i}."

        def lin(z, name):
            return torch.nn.functional.linear(z, _t(sd, p + name + ".weight"), _t(sd, p + name + ".bias"))

        q = lin(x, "attention.self.query").view(n, L, heads, D).transpose(1, 2)
        k = lin(x, "attention.self.key").view(n, L, heads, D).transpose(1, 2)
        v = lin(x, "attention.self.value").view(n, L, heads, D).transpose(1, 2)
        s = torch.matmul(q, k.transpose(2, 3)) * scale + add
        a = torch.softmax(s, dim=-1)
        ctx = torch.matmul(a, v).transpose(1, 2).reshape(n, L, H)
        o = lin(ctx, "attention.output.dense")
        x = _ln(o + x, _t(sd, p + "attention.output.LayerNorm.weight"),
                _t(sd, p + "attention.output.LayerNorm.bias"), eps)
        h = torch.nn.functional.gelu(lin(x, "intermediate.dense"))
        o = lin(h, "output.dense")
        x = _ln(o + x, _t(sd, p + "output.LayerNorm.weight"), _t(sd, p + "output.LayerNorm.bias"),
                eps)
    return x


@torch.no_grad()
def head_forward(sd, hidden: torch.Tensor, kind: str) -> torch.Tensor:
    """kind: sigmoid1 -> [n,1] probabilities; softmaxN -> [n,C]; pair2 -> [n/2, 2]."""
    x = hidden[:, 0, :]
    if kind == "pair2":
        x = x.reshape(-1, x.shape[-1] * 2)
    x = torch.nn.functional.linear(x, _t(sd, "classifier.dense.weight"), _t(sd, "classifier.dense.bias"))
    x = torch.tanh(x)
    x = torch.nn.functional.linear(x, _t(sd, "classifier.out_proj.weight"),
                                   _t(sd, "classifier.out_proj.bias"))
    if kind == "sigmoid1":
        return torch.sigmoid(x)
    return torch.softmax(x, dim=-1)


@torch.no_grad()
def score(sd, ids, kind: str = "sigmoid1", layers: int = 12, pos=None, attn_mask=None) -> np.ndarray:
    return head_forward(sd, encoder_forward(sd, ids, pos=pos, attn_mask=attn_mask, layers=layers),
                        kind).numpy()


@torch.no_grad()
def mlm_logits(sd, ids, layers: int = 12, no_mask: bool = False) -> torch.Tensor:
    """RobertaForMaskedLM logits [n, L, V] (lm_head: dense -> gelu -> LN -> tied decoder + bias)."""
    h = encoder_forward(sd, ids, layers=layers, no_mask=no_mask)
    x = torch.nn.functional.linear(h, _t(sd, "lm_head.dense.weight"), _t(sd, "lm_head.dense.bias"))
    x = torch.nn.functional.gelu(x)
    x = _ln(x, _t(sd, "lm_head.layer_norm.weight"), _t(sd, "lm_head.layer_norm.bias"), 1e-5)
    return torch.nn.functional.linear(x, _t(sd, "embeddings.word_embeddings.weight"), _t(sd, "lm_head.bias"))


def flops_per_query(L: int, layers: int = 12, hidden: int = 768, ffn: int = 3072, C: int = 1) -> float:
    """F(L) = 12*(2L*7,077,888 + 4L^2*768) + 2*768^2 + 2*768*C."""
    per_tok = 2 * (4 * hidden * hidden + 2 * hidden * ffn)
    return layers * (L * per_tok + 4 * L * L * hidden) + 2 * hidden * hidden + 2 * hidden * C


def gelu_erf(x):
    return 0.5 * x * (1.0 + math.erf(x / math.sqrt(2.0)))
