"""Clone-pair and authorship attacks against the text oracle (oracle/attack_ref.py with
Victim(task=...)): the product attackers (CloneAttacker / AuthorshipAttacker: C++ featurisation,
host mutant rows, pair and raw-text requests) and the oracle (every mutant rebuilt as text by
oracle.featurize_ref and featurised with the transformers tokenizer) drive the SAME deterministic
numpy stand-in victim under the same Python `random` seed, and must agree on outcome, attack
kind, query count, adversarial code and replacements.  The GPU version, with the HIP engine as
the victim, is tests/test_attack_gpu.py::test_task_attack_matches_text_oracle."""
import random

import numpy as np
import pytest

from conftest import ROOT
from oracle import attack_ref

BLOCK = 128


def stand_in(task):
    """Deterministic numpy victims; their sharpness is chosen so the fixture sample exercises
    greedy successes and GA runs (successes and failures)."""
    rng = np.random.default_rng(11)
    if task == "clone":
        w = rng.standard_normal(50265)

        def score(ids):
            s = np.where(ids != 1, w[ids], 0.0).sum(1).reshape(-1, 2)
            p = 1.0 / (1.0 + np.exp(-(s[:, 0] - s[:, 1]) / 0.3))
            return np.stack([p, 1 - p], 1).astype(np.float32)
    else:
        w = rng.standard_normal((50265, 66))
        bias = np.random.default_rng(3).standard_normal(66) * 2.0

        def score(ids):
            z = (w[ids] * (ids != 1)[..., None]).sum(1) / 20.0 + bias
            z = np.exp(z - z.max(1, keepdims=True))
            return (z / z.sum(1, keepdims=True)).astype(np.float32)
    return score


def fixture(task, n):
    from apmc_amd.drivers import load_fixture

    if task == "clone":
        return load_fixture(ROOT / "data" / "clone" / "test_subs_0_500.jsonl", 0, n)
    return load_fixture(ROOT / "data" / "authorship" / "valid_subs.jsonl", 0, n,
                        labels_path=ROOT / "data" / "authorship" / "valid.txt")


def compare_task(task, victim, score, codes, subs, labels, block, batch, seed0, idx):
    """Run product and oracle on examples `idx`; returns [(kind, outcome)]."""
    from apmc_amd.drivers import AttackArgs, _example, attack_one, make_attacker
    from apmc_amd.host import Tokenizer

    tok = Tokenizer()
    args = AttackArgs(block_size=block, eval_batch_size=batch, task=task)
    att = make_attacker(args, victim, tok)
    seen = []
    for i in idx:
        code, sb, lab = codes[i], subs[i], labels[i]
        random.seed(seed0 + i)
        q0 = victim.query
        res, kind = attack_one(att, tok, code, sb, lab, args)
        q_prod = victim.query - q0
        random.seed(seed0 + i)
        ex = _example(tok, code, lab, block, task)
        v = attack_ref.Victim(score, block, task=task,
                              code2=code[3] if task == "clone" else None)
        text = code[2] if task == "clone" else code
        ids0 = ex[0].numpy().astype(np.int32)
        ref = attack_ref.greedy(v, ids0, lab, text, sb)
        ref_kind = "Greedy"
        if ref["is_success"] == -1:
            ref = attack_ref.ga(v, ids0, lab, text, sb, initial_replace=ref["replaced"],
                                eval_batch_size=batch)
            ref_kind = "GA"
        assert (res[6], kind) == (ref["is_success"], ref_kind), i
        assert q_prod == v.query, (i, kind, q_prod, v.query)
        assert res[1] == ref["prog_length"], i
        if res[6] == 1:
            assert res[2] == ref["adv_code"], i
            assert (res[9], res[10]) == (ref["nb_changed_var"], ref["nb_changed_pos"]), i
            assert dict(res[11]) == ref["replaced"], i
        seen.append((kind, res[6]))
    return seen


@pytest.mark.parametrize("task", ["clone", "authorship"])
def test_task_attack_matches_text_oracle_cpu(task):
    import _apmc  # noqa: F401
    from apmc_amd.drivers import _example
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import HostIdsVictim

    codes, subs, _ = fixture(task, 12)
    score = stand_in(task)
    tok = Tokenizer()
    probe = HostIdsVictim(score, task=task, block_size=BLOCK)
    # labels = the stand-in's own predictions, so every example is attacked
    labels = [int(probe.get_results([_example(tok, c, 0, BLOCK, task)])[1][0]) for c in codes]
    victim = HostIdsVictim(score, task=task, block_size=BLOCK)
    seen = compare_task(task, victim, score, codes, subs, labels, BLOCK, 16, 4000, range(12))
    assert ("Greedy", 1) in seen and any(k == "GA" for k, _ in seen), seen


# ---------------------------------------------------------------- GraphCodeBERT victims (CPU)
GCB_ARGS = dict(code_length=192, data_flow_length=64)


def graph_stand_in(base):
    """numpy scores of (ids, pos, mask bits) rows: token and mask terms, so a feature or mask
    difference between product and oracle changes the scores."""
    rng = np.random.default_rng(13)
    w = rng.standard_normal(50265)
    w66 = rng.standard_normal((50265, 66))

    def row_terms(ids, pos, bits):
        tok = np.where(pos > 1, w[ids], 0.0).sum(1)
        mk = (bits.astype(np.int64) % 7).sum(axis=(1, 2)) * 1e-3
        return tok, mk

    def score(ids, pos, bits):
        tok, mk = row_terms(ids, pos, bits)
        if base == "clone":
            z = (tok + mk).reshape(-1, 2)
            p = 1.0 / (1.0 + np.exp(-(z[:, 0] - z[:, 1]) / 0.5))
            return np.stack([p, 1 - p], 1).astype(np.float32)
        if base == "devign":
            return (1.0 / (1.0 + np.exp(-(tok + mk) / 3.0))).astype(np.float32)[:, None]
        z = (w66[ids] * (pos > 1)[..., None]).sum(1) / 20.0 + mk[:, None]
        z = np.exp(z - z.max(1, keepdims=True))
        return (z / z.sum(1, keepdims=True)).astype(np.float32)
    return score


def host_graph_victim(score, base):
    """The product GraphModel request API over a numpy scorer (no engine on this host)."""
    import _apmc  # noqa: F401
    from apmc_amd.graph import GraphModel

    class HostGraphVictim(GraphModel):
        def __init__(self):  # noqa: D107 — no engine
            self.task, self.query, self.raw = base, 0, False
            self.args = None

        def score_packed(self, ids, pos, bits):
            return np.asarray(score(ids, pos, bits))

        def score_payload_rows(self, live):  # compact masks rebuilt on the host
            from apmc_amd.graph import payload_rows_host
            return self.score_packed(*payload_rows_host(live))

        def submit(self, payloads, threshold=0.5):  # answered at once (host scoring)
            from apmc_amd.model import ScoresReady
            return ScoresReady(self.score_prepared(payloads, threshold))

    return HostGraphVictim()


def compare_gcb(task, codes, subs, labels, batch, seed0, idx):
    from apmc_amd.drivers import AttackArgs

    base = task[4:]
    args = AttackArgs(block_size=256, eval_batch_size=batch, task=task, **GCB_ARGS)
    score = graph_stand_in(base)
    victim = host_graph_victim(score, base)
    victim.args = args
    return compare_gcb_with(task, victim, score, codes, subs, labels, args, seed0, idx)


def compare_gcb_with(task, victim, score, codes, subs, labels, args, seed0, idx):
    """Product attack (sequential driver step) vs the text oracle on examples `idx`."""
    from apmc_amd.drivers import attack_one, make_attacker
    from apmc_amd.host import Tokenizer
    from oracle.graph_ref import GraphTextVictim

    base = task[4:]
    batch = args.eval_batch_size
    tok = Tokenizer()
    gcb = dict(code_length=args.code_length, data_flow_length=args.data_flow_length)
    att = make_attacker(args, victim, tok)
    seen = []
    for i in idx:
        code, sb, lab = codes[i], subs[i], labels[i]
        random.seed(seed0 + i)
        q0 = victim.query
        res, kind = attack_one(att, tok, code, sb, lab, args)
        q_prod = victim.query - q0
        random.seed(seed0 + i)
        text = code[2] if base == "clone" else code
        v = GraphTextVictim(score, task, text, code2=code[3] if base == "clone" else None, **gcb)
        extra = 0
        if task == "gcb_devign":  # the driver's extra get_results([example])
            v.ids(None)
            extra = 1
        ids0 = np.zeros(1, np.int32)  # unused: GraphTextVictim.ids featurises the text
        ref = attack_ref.greedy(v, ids0, lab, text, sb)
        ref_kind = "Greedy"
        if ref["is_success"] == -1:
            ref = attack_ref.ga(v, ids0, lab, text, sb, initial_replace=ref["replaced"],
                                eval_batch_size=batch)
            ref_kind = "GA"
        assert (res[6], kind) == (ref["is_success"], ref_kind), i
        assert q_prod == v.query, (i, kind, q_prod, v.query, extra)
        if res[6] == 1:
            assert res[2] == ref["adv_code"], i
            assert dict(res[11]) == ref["replaced"], i
        seen.append((kind, res[6]))
    return seen


@pytest.mark.parametrize("task", ["gcb_clone", "gcb_authorship", "gcb_devign"])
def test_gcb_task_attack_matches_text_oracle_cpu(task):
    """GraphCodeBERT attackers (GraphCloneAttacker / GraphAuthorshipAttacker / GraphAttacker and
    the gcb_* drivers) against the text oracle (oracle/graph_ref.GraphTextVictim) on a numpy
    scorer of the packed rows: same outcomes, query counts (incl. the gcb_devign driver's extra
    query, GraphCodeBERT/Defect-detection/code/gi_attack.py:161, and its 64-child GA),
    adversarial code and replacements.  Labels are the scorer's own predictions."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.host import Tokenizer

    base = task[4:]
    if base == "devign":
        codes, subs, _ = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl", 0, 40)
        pick = [i for i in range(40) if 1 <= len(subs[i]) <= 4 and len(codes[i]) < 900][:5]
    else:
        codes, subs, _ = fixture(base, 6)
        pick = list(range(6))
    tok = Tokenizer()
    args = AttackArgs(block_size=256, eval_batch_size=16, task=task, **GCB_ARGS)
    probe = host_graph_victim(graph_stand_in(base), base)
    labels = [0] * len(codes)
    for i in pick:
        labels[i] = int(probe.get_results([_example(tok, codes[i], 0, 256, task, args)])[1][0])
    seen = compare_gcb(task, codes, subs, labels, 16, 8000, pick)
    assert {o for _, o in seen} & {1, -1}, seen
