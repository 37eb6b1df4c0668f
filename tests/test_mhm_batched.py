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


def IdsVictim():
    """Devign-format victim: p = sigmoid(<ids, w> / 4) behind the product request API
    (HostIdsVictim); records every batch size it served in `.batches`."""
    import _apmc  # noqa: F401
    from apmc_amd.model import HostIdsVictim

    w = np.random.default_rng(1).standard_normal(50265)
    batches = []

    def score(ids):
        batches.append(ids.shape[0])
        z = np.where(ids != 1, w[ids], 0.0).sum(1) / 4.0
        return (1.0 / (1.0 + np.exp(-z))).astype(np.float32)[:, None]

    v = HostIdsVictim(score)
    v.batches = batches
    return v


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


def test_authorship_driver_batched_equals_sequential():
    """Authorship-Attribution MHM-NS (mhm.py:160-233): Python identifiers, raw-text features,
    the 66-way argmax victim; the batched driver's records equal the reference loop run with the
    same per-example seeds (random.seed(seed + index) before each chain)."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, _example, load_fixture, run_mhm_attack
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import HostIdsVictim

    codes, subs, _ = load_fixture(ROOT / "data" / "authorship" / "valid_subs.jsonl", 0, 12,
                                  labels_path=ROOT / "data" / "authorship" / "valid.txt")
    w = np.random.default_rng(5).standard_normal((50265, 66))

    def score(ids):
        z = (w[ids] * (ids != 1)[..., None]).sum(1) / 3.0
        z = np.exp(z - z.max(1, keepdims=True))
        return (z / z.sum(1, keepdims=True)).astype(np.float32)

    tok = Tokenizer()
    probe = HostIdsVictim(score, task="authorship")
    labels = [int(probe.get_results([_example(tok, c, 0, BLOCK, "authorship")])[1][0])
              for c in codes]
    args = AttackArgs(block_size=BLOCK, eval_batch_size=32, task="authorship", lang="python")
    v_bat = HostIdsVictim(score, task="authorship")
    bat = run_mhm_attack(v_bat, codes, subs, labels, args, tok=tok, max_iter=10, max_inflight=8)
    # the sequential reference loop, re-seeded per example the way the batched chains are
    import apmc_amd.drivers as D

    v_seq = HostIdsVictim(score, task="authorship")
    seq = []
    for i in range(len(codes)):
        orig_seed = args.seed
        args_i = AttackArgs(block_size=BLOCK, eval_batch_size=32, task="authorship",
                            lang="python", seed=orig_seed + i)
        q0 = v_seq.query
        out = D.run_mhm_attack(v_seq, codes, subs, labels, args_i, indices=[i], tok=tok,
                               max_iter=10)
        seq.append(dict(out["records"][0], index=i))
        assert out["queries"] == v_seq.query - q0
    assert [dict(r) for r in bat["records"]] == seq
    assert {r["is_success"] for r in seq} & {1, -1}


@pytest.mark.parametrize("kind", ["mcmc", "mcmc_random"])
def test_authorship_mhm_matches_text_oracle_cpu(kind):
    """AuthorshipMHM_Attacker (CodeXGLUE/Authorship-Attribution/code/attacker.py:440-666, driven as
    mhm.py:198-206: n_candi 30, threshold 1) against oracle/mhm_ref.py over text (Python leaves,
    raw-text features, 66-way argmax), same Python `random` seed, on a numpy stand-in victim: same
    outcome, adversarial code, replacement chain and query count."""
    import _apmc  # noqa: F401
    from apmc_amd.attacker import AuthorshipMHM_Attacker
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import HostIdsVictim
    from apmc_amd.utils import isUID
    from oracle import attack_ref, mhm_ref

    codes, subs, _ = load_fixture(ROOT / "data" / "authorship" / "valid_subs.jsonl", 0, 6,
                                  labels_path=ROOT / "data" / "authorship" / "valid.txt")
    w = np.random.default_rng(5).standard_normal((50265, 66))
    bias = np.random.default_rng(3).standard_normal(66) * 2.0

    def score(ids):  # sharpness chosen so the sample has successes and failures
        z = (w[ids] * (ids != 1)[..., None]).sum(1) / 20.0 + bias
        z = np.exp(z - z.max(1, keepdims=True))
        return (z / z.sum(1, keepdims=True)).astype(np.float32)

    tok = Tokenizer()
    victim = HostIdsVictim(score, task="authorship", block_size=BLOCK)
    labels = [int(victim.get_results([_example(tok, c, 0, BLOCK, "authorship")])[1][0])
              for c in codes]
    args = AttackArgs(block_size=BLOCK, eval_batch_size=64, task="authorship", lang="python")
    vocab = sorted({w_ for s in subs for v in s.values() for w_ in v})
    att = AuthorshipMHM_Attacker(args, victim, None, tok, {t: i for i, t in enumerate(vocab)},
                                 vocab)
    seen = []
    for i in range(len(codes)):
        random.seed(3100 + i)
        q0 = victim.query
        res = getattr(att, kind)(tok, codes[i], labels[i], _n_candi=30, _max_iter=20,
                                 _prob_threshold=1, subs=subs[i])
        q_prod = victim.query - q0
        random.seed(3100 + i)
        v = attack_ref.Victim(score, BLOCK, task="authorship")
        ref = mhm_ref.mcmc(v, isUID, subs[i], codes[i], labels[i], n_candi=30, max_iter=20,
                           prob_threshold=1, idx2token=vocab if kind == "mcmc_random" else None,
                           lang="python", skip_known=False)
        assert res["succ"] == ref["succ"], i
        assert q_prod == v.query, (i, q_prod, v.query)
        if res["succ"] is not None:
            for k in ("tokens", "replace_info", "nb_changed_var", "nb_changed_pos",
                      "prog_length", "new_pred"):
                assert res[k] == ref[k], (i, k)
        seen.append(res["succ"])
    assert True in seen and False in seen, seen
