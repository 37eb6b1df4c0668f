"""CPU: the oracle (oracle/roberta_cpu.py) against the golden vectors produced by the installed
transformers RoBERTa (tests/golden/make_golden_encoder.py)."""
import numpy as np
import torch

from conftest import golden, synthetic_sd
from oracle import roberta_cpu as ora


def test_devign_probs_and_cls_match_hf():
    g = golden()
    sd = synthetic_sd(0, "sigmoid1")
    h = ora.encoder_forward(sd, g["devign_ids"])
    np.testing.assert_allclose(h[:, 0, :].numpy(), g["devign_cls"], atol=2e-5, rtol=0)
    p = ora.head_forward(sd, h, "sigmoid1").numpy()
    np.testing.assert_allclose(p, g["devign_probs"], atol=1e-6, rtol=0)


def test_authorship_probs_match_hf():
    g = golden()
    sd = synthetic_sd(1, "softmaxN", 66)
    p = ora.score(sd, g["aa_ids"], "softmaxN")
    np.testing.assert_allclose(p, g["aa_probs"], atol=1e-6, rtol=0)


def test_clone_pair_probs_match_hf():
    g = golden()
    sd = synthetic_sd(2, "pair2", 2)
    p = ora.score(sd, g["clone_ids"], "pair2")
    np.testing.assert_allclose(p, g["clone_probs"], atol=1e-6, rtol=0)


def test_mlm_topk_matches_hf():
    g = golden()
    sd = synthetic_sd(3, "none", 1, True)
    logits = ora.mlm_logits(sd, g["mlm_ids"])[0]
    sc, ix = torch.topk(logits, 60, -1)
    np.testing.assert_allclose(sc.numpy(), g["mlm_top_scores"], atol=1e-4, rtol=0)
    assert (ix.numpy() == g["mlm_top_ids"]).mean() > 0.99


def test_pad_rows_do_not_change_cls():
    """The engine's pad compaction relies on this: padding never influences the CLS output."""
    sd = synthetic_sd(0, "sigmoid1")
    rng = np.random.default_rng(5)
    ids = np.full((1, 40), 1, dtype=np.int64)
    ids[0, 0] = 0
    ids[0, 1:19] = rng.integers(4, 50000, 18)
    ids[0, 19] = 2
    a = ora.encoder_forward(sd, ids, layers=2)[0, 0]
    b = ora.encoder_forward(sd, ids[:, :20], layers=2)[0, 0]
    np.testing.assert_allclose(a.numpy(), b.numpy(), atol=1e-5)


def test_flop_model():
    assert ora.flops_per_query(512, C=0) - 2 * 768 * 768 == 12 * (2 * 512 * 7077888 + 4 * 512 * 512 * 768)


def test_heads_match_hf_at_block_512():
    """The oracle at the headline config's own length (L = 512: full, 510, ragged 300 / 129, a row
    with literal <pad> ids inside it) against transformers (make_golden_encoder_512.py)."""
    from conftest import golden512
    g = golden512()
    sd = synthetic_sd(0, "sigmoid1")
    h = ora.encoder_forward(sd, g["devign_ids"])
    np.testing.assert_allclose(h[:, 0, :].numpy(), g["devign_cls"], atol=5e-5, rtol=0)
    np.testing.assert_allclose(ora.head_forward(sd, h, "sigmoid1").numpy(), g["devign_probs"],
                               atol=2e-6, rtol=0)
    p = ora.score(synthetic_sd(1, "softmaxN", 66), g["aa_ids"], "softmaxN")
    np.testing.assert_allclose(p, g["aa_probs"], atol=2e-6, rtol=0)
    p = ora.score(synthetic_sd(2, "pair2", 2), g["clone_ids"], "pair2")
    np.testing.assert_allclose(p, g["clone_probs"], atol=2e-6, rtol=0)
