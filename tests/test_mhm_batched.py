"""Cross-example batched MHM-NS: `MHM_Attacker.mcmc_batched` interleaves many
examples' MCMC chains and answers all their pending candidate batches with one `get_results`
call.  Each chain must come out exactly as `random.seed(seed); mcmc(...)` run alone — same
outcome, adversarial code, replacement chain, per-example query count — and the victim's query
counter must advance by the same total.  The victim is a deterministic numpy stand-in over the
real featurised ids (C++ host library), so the batching/RNG logic is what is under test; the GPU
engine's batch-invariance is covered by tests/test_engine_gpu.py."""
import pathlib
import random
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
FIXTURE = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"
BLOCK = 128


class IdsVictim:
    """Devign-format victim: p = sigmoid(<ids, w> / 4); records every batch size it served."""

    def __init__(self):
        self.w = np.random.default_rng(1).standard_normal(50265)
        self.query = 0
        self.batches = []

    def get_results(self, dataset, batch_size=None):
        self.query += len(dataset)
        ids = dataset.ids if hasattr(dataset, "ids") else np.stack([np.asarray(d[0]) for d in dataset])
        self.batches.append(ids.shape[0])
        z = np.where(ids != 1, self.w[ids], 0.0).sum(1) / 4.0
        p = (1.0 / (1.0 + np.exp(-z))).astype(np.float32)
        return [[1 - x, x] for x in p], [1 if x > 0.5 else 0 for x in p]


@pytest.fixture(scope="module")
def setup():
    import _apmc  # noqa: F401
    from apmc_amd.drivers import load_fixture
    from apmc_amd.host import Tokenizer

    codes, subs, _ = load_fixture(FIXTURE, 0, 40)
    return codes, subs, Tokenizer()


def _labels(victim, tok, codes):
    from apmc_amd.utils import IdsDataset

    ids, lens = tok.featurize(codes, BLOCK)
    return victim.get_results(IdsDataset(ids, lens))[1]


@pytest.mark.parametrize("original", [False, True])
def test_batched_chains_equal_sequential(setup, original):
    from apmc_amd.attacker import MHM_Attacker
    from apmc_amd.drivers import AttackArgs

    codes, subs, tok = setup
    args = AttackArgs(block_size=BLOCK, eval_batch_size=32)
    vocab = sorted({w for s in subs for v in s.values() for w in v})
    victim = IdsVictim()
    labels = _labels(victim, tok, codes)
    att = MHM_Attacker(args, victim, None, tok, {w: i for i, w in enumerate(vocab)}, vocab)
    jobs = [(subs[i], codes[i], labels[i], 7000 + i) for i in range(len(codes))]

    seq = []
    q_start = victim.query
    for sb, code, lab, seed in jobs:
        random.seed(seed)
        q0 = victim.query
        fn = att.mcmc_random if original else att.mcmc
        res = fn(tok, sb, code, lab, _n_candi=30, _max_iter=15)
        seq.append((res, victim.query - q0))
    q_seq = victim.query - q_start

    victim.batches.clear()
    q0 = victim.query
    finished = []
    got = att.mcmc_batched(tok, jobs, _n_candi=30, _max_iter=15, original=original,
                           max_inflight=16, on_done=lambda j, r, q: finished.append(j))
    assert victim.query - q0 == q_seq
    assert sorted(finished) == list(range(len(jobs)))
    assert max(victim.batches) > 31  # chains really share device batches
    for j, ((r_seq, q_s), (r_bat, q_b)) in enumerate(zip(seq, got)):
        assert q_s == q_b, j
        assert r_seq == r_bat, j
    assert any(r["succ"] is not None for r, _ in seq)


def test_driver_batched_mode_counts(setup):
    from apmc_amd.drivers import AttackArgs, run_mhm_attack

    codes, subs, tok = setup
    victim = IdsVictim()
    labels = _labels(victim, tok, codes)
    labels = [lab if i % 5 else 1 - lab for i, lab in enumerate(labels)]  # some -4 early exits
    args = AttackArgs(block_size=BLOCK, eval_batch_size=32)
    q0 = victim.query
    out = run_mhm_attack(victim, codes, subs, labels, args, tok=tok, max_iter=10,
                         max_inflight=8)
    assert [r["index"] for r in out["records"]] == list(range(len(codes)))
    assert out["queries"] == victim.query - q0
    assert sum(r["is_success"] == -4 for r in out["records"]) == len(codes[::5])
