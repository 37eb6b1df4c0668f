"""GPU end-to-end parity of the attacks: the product Attacker (C++ featurisation, device splice,
HIP engine) against the text-driven restatement oracle/attack_ref.py scoring the SAME mutant texts
with the same engine (engine numerics are covered by test_engine_gpu.py).  Under one Python
`random` seed both must agree on outcome, adversarial code, replaced names and query count."""
import random

import numpy as np
import pytest
import torch

from conftest import ROOT, synthetic_sd
from oracle import attack_ref

pytestmark = pytest.mark.gpu
BLOCK = 256
FIXTURE = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"


@pytest.fixture(scope="module")
def victim():
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(seed=5, head="sigmoid1", out_std=8.0)
    return Model(sd, task="devign")


def _score_fn(model):
    def score(ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        lens = (ids != 1).sum(1).astype(np.int32)
        out = model.engine.score(torch.from_numpy(ids).cuda(), lens)
        return out.cpu().numpy()[:, 0]
    return score


def _pick(codes, subs, n, max_vars=6, max_chars=1500):
    idx = [i for i in range(len(codes))
           if 1 <= len(subs[i]) <= max_vars and len(codes[i]) < max_chars]
    return idx[:n]


# config-2 shape (gi_attack.py --block_size 512 --eval_batch_size 64): 16 fixture examples with
# up to 8 variables, in 4 chunks so each test stays well inside the per-test time limit
CONFIG2_BLOCK, CONFIG2_BATCH = 512, 64
_OUTCOMES = []


def _config2_examples(codes, subs):
    return _pick(codes, subs, 16, max_vars=8, max_chars=4000)


@pytest.mark.parametrize("chunk", [0, 1, 2, 3])
def test_greedy_then_ga_matches_text_oracle(victim, chunk):
    from apmc_amd.drivers import AttackArgs, _example
    from apmc_amd.attacker import Attacker
    from apmc_amd.host import Tokenizer
    from apmc_amd.drivers import load_fixture

    codes, subs, labels = load_fixture(FIXTURE, 0, 200)
    tok = Tokenizer()
    args = AttackArgs(block_size=CONFIG2_BLOCK, eval_batch_size=CONFIG2_BATCH)
    att = Attacker(args, victim, tok, None, tok, 1, 0)
    for i in _config2_examples(codes, subs)[4 * chunk:4 * chunk + 4]:
        code, sb, lab = codes[i], subs[i], labels[i]
        # product
        random.seed(1000 + i)
        q0 = victim.query
        ex = _example(tok, code, lab, CONFIG2_BLOCK)
        res = att.greedy_attack(ex, code, sb)
        kind = "greedy"
        if res[6] == -1:
            res = att.ga_attack(ex, code, sb, initial_replace=res[11])
            kind = "ga"
        q_prod = victim.query - q0
        # oracle
        random.seed(1000 + i)
        v = attack_ref.Victim(_score_fn(victim), CONFIG2_BLOCK)
        ids0 = ex[0].numpy().astype(np.int32)
        ref = attack_ref.greedy(v, ids0, lab, code, sb)
        if ref["is_success"] == -1:
            ref = attack_ref.ga(v, ids0, lab, code, sb, initial_replace=ref["replaced"],
                                eval_batch_size=CONFIG2_BATCH)
        assert res[6] == ref["is_success"], (i, kind)
        assert q_prod == v.query, (i, kind, q_prod, v.query)
        assert res[1] == ref["prog_length"]
        if res[6] == 1:
            assert res[2] == ref["adv_code"], i
            assert res[9] == ref["nb_changed_var"] and res[10] == ref["nb_changed_pos"]
            assert dict(res[11]) == ref["replaced"]
        _OUTCOMES.append((kind, res[6]))


# a GA success at config-2 shape: fixture example 55 with this victim and the per-example seed
# (found by tools/debug/find_ga_success.py: 1 GA success among the 289 config-2-sized examples)
GA_SUCCESS_INDEX = 55


def test_config2_ga_success_matches_text_oracle(victim):
    from apmc_amd.drivers import AttackArgs, _example, load_fixture, make_attacker
    from apmc_amd.host import Tokenizer

    codes, subs, labels = load_fixture(FIXTURE, 0, 200)
    tok = Tokenizer()
    args = AttackArgs(block_size=CONFIG2_BLOCK, eval_batch_size=CONFIG2_BATCH)
    att = make_attacker(args, victim, tok)
    i = GA_SUCCESS_INDEX
    code, sb, lab = codes[i], subs[i], labels[i]
    random.seed(args.seed + i)
    q0 = victim.query
    ex = _example(tok, code, lab, CONFIG2_BLOCK)
    res = att.greedy_attack(ex, code, sb)
    assert res[6] == -1
    res = att.ga_attack(ex, code, sb, initial_replace=res[11])
    q_prod = victim.query - q0
    random.seed(args.seed + i)
    v = attack_ref.Victim(_score_fn(victim), CONFIG2_BLOCK)
    ids0 = ex[0].numpy().astype(np.int32)
    ref = attack_ref.greedy(v, ids0, lab, code, sb)
    assert ref["is_success"] == -1
    ref = attack_ref.ga(v, ids0, lab, code, sb, initial_replace=ref["replaced"],
                        eval_batch_size=CONFIG2_BATCH)
    assert res[6] == ref["is_success"] == 1
    assert q_prod == v.query
    assert res[2] == ref["adv_code"]
    assert (res[9], res[10]) == (ref["nb_changed_var"], ref["nb_changed_pos"])
    assert dict(res[11]) == ref["replaced"]
    _OUTCOMES.append(("ga", res[6]))


def test_config2_sample_exercises_both_attacks():
    """The config-2 examples above include a greedy success and a GA success."""
    if len(_OUTCOMES) < 17:
        pytest.skip("needs the chunks of test_greedy_then_ga_matches_text_oracle and the GA case")
    assert ("greedy", 1) in _OUTCOMES and ("ga", 1) in _OUTCOMES, _OUTCOMES


# ---- the precision the bench runs: f32x3 attack decisions against the fp32 oracle ------------
# north_star: identical attack outcomes except where a probability lies within the tolerance
# (1e-4) of a decision boundary.  The oracle's fp32 run records the margin of every decision it
# makes (p vs 0.5, gap vs most_gap, fitness vs the population minimum, the importance order);
# an example may differ only if one of them was within X3_BOUNDARY (exact zeros are comparisons
# of identical rows, which score identically in both modes).
X3_BOUNDARY = 1e-4
_X3_OUT = []


@pytest.fixture(scope="module")
def victim_x3():
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(seed=5, head="sigmoid1", out_std=8.0)
    m = Model(sd, task="devign", precision="f32x3")
    yield m
    m.engine.close()


def _x3_examples(codes, subs):
    return _config2_examples(codes, subs) + [GA_SUCCESS_INDEX]


@pytest.mark.parametrize("chunk", [0, 1, 2, 3, 4])
def test_f32x3_attack_outcomes_match_fp32_oracle(victim, victim_x3, chunk):
    """The 17 config-2 examples above (block 512, batch 64, greedy -> GA, incl. the GA success)
    attacked through the f32x3 engine (the mode every bench attack leg runs) against the fp32
    text oracle: identical outcome, query count, adversarial code and replacements, except
    examples with a decision within X3_BOUNDARY of its boundary in the fp32 run (counted)."""
    from apmc_amd.drivers import AttackArgs, _example, load_fixture, make_attacker
    from apmc_amd.host import Tokenizer

    codes, subs, labels = load_fixture(FIXTURE, 0, 200)
    tok = Tokenizer()
    args = AttackArgs(block_size=CONFIG2_BLOCK, eval_batch_size=CONFIG2_BATCH)
    att = make_attacker(args, victim_x3, tok)
    for i in _x3_examples(codes, subs)[4 * chunk:4 * chunk + 4]:
        code, sb, lab = codes[i], subs[i], labels[i]
        seed = (args.seed + i) if i == GA_SUCCESS_INDEX else (1000 + i)
        random.seed(seed)
        q0 = victim_x3.query
        ex = _example(tok, code, lab, CONFIG2_BLOCK)
        res = att.greedy_attack(ex, code, sb)
        if res[6] == -1:
            res = att.ga_attack(ex, code, sb, initial_replace=res[11])
        q_x3 = victim_x3.query - q0
        random.seed(seed)
        v = attack_ref.Victim(_score_fn(victim), CONFIG2_BLOCK)
        v.margins = []
        ids0 = ex[0].numpy().astype(np.int32)
        ref = attack_ref.greedy(v, ids0, lab, code, sb)
        if ref["is_success"] == -1:
            ref = attack_ref.ga(v, ids0, lab, code, sb, initial_replace=ref["replaced"],
                                eval_batch_size=CONFIG2_BATCH)
        same = (res[6] == ref["is_success"] and q_x3 == v.query and
                (res[6] != 1 or (res[2] == ref["adv_code"] and dict(res[11]) == ref["replaced"])))
        near = min([m for m in v.margins if m > 0] or [1.0])
        _X3_OUT.append((i, same, near, res[6], q_x3, v.query))
        if not same:
            assert near < X3_BOUNDARY, (i, res[6], ref["is_success"], q_x3, v.query, near)


def test_f32x3_attack_outcomes_summary():
    """All 17 examples ran; report how many matched and how many were excused (a decision of
    the fp32 run within X3_BOUNDARY); the sample includes successes.  Every difference must be
    excused (each chunk already asserts it); the r4 GPU run had 14/17 identical and 3 excused,
    two of them at a fp32 decision margin of 1.19e-7 (one ulp at 1.0: two candidates whose
    fp32 probabilities differ in the last bit, which f32x3's 1e-5 rounding reorders)."""
    if len(_X3_OUT) < 17:
        pytest.skip("needs every chunk of test_f32x3_attack_outcomes_match_fp32_oracle")
    same = sum(1 for o in _X3_OUT if o[1])
    excused = [o for o in _X3_OUT if not o[1]]
    print(f"f32x3 vs fp32 oracle: {same}/{len(_X3_OUT)} identical, {len(excused)} excused "
          f"(decision margin < {X3_BOUNDARY}): {excused}")
    print("closest decision margins:", sorted((round(o[2], 8), o[0]) for o in _X3_OUT)[:5])
    assert all(o[2] < X3_BOUNDARY for o in excused), excused
    assert same >= (2 * len(_X3_OUT)) // 3, _X3_OUT
    assert any(o[3] == 1 for o in _X3_OUT if o[1])


def test_batched_gi_equals_sequential(victim):
    """Cross-example batching on the HIP engine (drivers.run_gi_attack_batched): 16 examples'
    greedy->GA attacks share every device batch; each record equals the sequential per-example
    run (random.seed(seed + index)) — outcome, adversarial code, replacements, query count."""
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack, run_gi_attack_batched

    codes, subs, labels = load_fixture(FIXTURE, 0, 200)
    idx = _config2_examples(codes, subs)
    args = AttackArgs(block_size=CONFIG2_BLOCK, eval_batch_size=CONFIG2_BATCH, rng="per_example")
    seq = run_gi_attack(victim, codes, subs, labels, args, indices=idx)
    bat = run_gi_attack_batched(victim, codes, subs, labels, args, indices=idx, max_inflight=16)
    keys = ["index", "is_success", "attack_type", "queries", "adv_code", "replace_info",
            "nb_changed_var", "nb_changed_pos"]
    assert [{k: r[k] for k in keys} for r in seq["records"]] == \
        [{k: r[k] for k in keys} for r in bat["records"]]
    assert seq["queries"] == bat["queries"]


def test_literal_pad_in_source(victim):
    """A literal "<pad>" in the source tokenises to the pad id (the reference masks it with
    attention_mask = ids.ne(1)); the featuriser's lens exclude it, the engine drops it, and the
    score equals the oracle's on the same ids.  Lens that disagree with the ids give an error,
    never a silently wrong score."""
    from apmc_amd.host import Tokenizer
    from apmc_amd.utils import IdsDataset
    from conftest import synthetic_sd
    from oracle import roberta_cpu as ora

    tok = Tokenizer()
    code = "int f(int a) { int <pad> = a; return a <pad> + 1; }"
    ids, lens = tok.featurize([code, "int g(void) { return 0; }"], 64)
    assert (ids[0, 1:lens[0]] == 1).any() and lens[0] == (ids[0] != 1).sum()
    probs, _ = victim.get_results(IdsDataset(ids, lens))
    ref = ora.score(synthetic_sd(seed=5, head="sigmoid1", out_std=8.0), ids, "sigmoid1")
    assert abs(probs[0][1] - ref[0, 0]) < 1e-4 and abs(probs[1][1] - ref[1, 0]) < 1e-4
    with pytest.raises(RuntimeError, match="non-finite"):
        victim.get_results(IdsDataset(ids, lens + 1))


def test_driver_runs_and_counts(victim):
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack
    codes, subs, labels = load_fixture(FIXTURE, 0, 6)
    out = run_gi_attack(victim, codes, subs, labels, AttackArgs(block_size=BLOCK,
                                                                eval_batch_size=16))
    assert out["examples"] == 6
    assert out["queries"] == sum(r["queries"] for r in out["records"])
    assert all(r["queries"] >= 1 for r in out["records"])


class _GraphVictim(attack_ref.Victim):
    """Text oracle victim for GraphCodeBERT: every mutant text featurised by oracle/graph_ref.py
    (reference-loop features and mask), scored by the same engine's graph forward."""

    def __init__(self, model, code0, args):
        super().__init__(None, 0)
        self.model, self.code0, self.args = model, code0, args

    def _feats(self, code):
        from apmc_amd.graph import extract_dataflow
        from oracle import graph_ref
        dfg, _, toks = extract_dataflow(" ".join(code.split()), "c")
        ids, pos, d2c, d2d = graph_ref.convert_code_to_features(
            dfg, toks, self.args.code_length, self.args.data_flow_length)
        L = len(ids)
        m = graph_ref.graph_mask(ids, pos, d2c, d2d, L)
        return ids, pos, np.packbits(m, axis=-1, bitorder="little").view("<i4")

    def texts(self, codes):
        fs = [self._feats(c) for c in codes]
        self.query += len(fs)
        p = self.model.score_packed(np.array([f[0] for f in fs], np.int32),
                                    np.array([f[1] for f in fs], np.int32),
                                    np.stack([f[2] for f in fs]))[:, 0]
        return [[1 - x, x] for x in p], [1 if x > 0.5 else 0 for x in p]

    def ids(self, _ids0):
        return self.texts([self.code0])


def test_graphcodebert_greedy_then_ga_matches_text_oracle():
    """GraphCodeBERT Devign victim (GraphCodeBERT/Defect-detection/code/attacker.py): mutants are
    re-featurised with the data-flow graph; product Attacker + GraphModel vs the text oracle."""
    import types
    from apmc_amd.attacker import Attacker
    from apmc_amd.drivers import load_fixture
    from apmc_amd.graph import GraphCodeDataset, GraphModel, convert_code_to_features
    from apmc_amd.host import Tokenizer
    from apmc_amd.weights import synthetic_state_dict

    args = types.SimpleNamespace(code_length=256, data_flow_length=64, block_size=320,
                                 eval_batch_size=16, lang="c")
    model = GraphModel(synthetic_state_dict(seed=5, head="sigmoid1", out_std=8.0), args=args)
    codes, subs, labels = load_fixture(FIXTURE, 0, 120)
    tok = Tokenizer()
    att = Attacker(args, model, tok, None, tok, 1, 0)
    kinds = []
    for i in _pick(codes, subs, 5):
        code, sb, lab = codes[i], subs[i], labels[i]
        ex = GraphCodeDataset([convert_code_to_features(code, tok, lab, args)], args)[0]
        random.seed(2000 + i)
        q0 = model.query
        res = att.greedy_attack(ex, code, sb)
        kind = "greedy"
        if res[6] == -1:
            res = att.ga_attack(ex, code, sb, initial_replace=res[11])
            kind = "ga"
        q_prod = model.query - q0
        random.seed(2000 + i)
        v = _GraphVictim(model, code, args)
        ref = attack_ref.greedy(v, np.zeros(1), lab, code, sb)
        if ref["is_success"] == -1:
            ref = attack_ref.ga(v, np.zeros(1), lab, code, sb, initial_replace=ref["replaced"],
                                eval_batch_size=16)
        assert res[6] == ref["is_success"], (i, kind)
        assert q_prod == v.query, (i, kind, q_prod, v.query)
        if res[6] == 1:
            assert res[2] == ref["adv_code"], i
            assert dict(res[11]) == ref["replaced"]
        kinds.append((kind, res[6]))
    assert kinds


# config-5 MHM-NS shape (mhm_attack.py:215-217 / Authorship mhm.py:198-206): block 512,
# n_candi 30, max_iter 100, _prob_threshold 1
MHM_BLOCK, MHM_ITERS, MHM_THRESHOLD = 512, 100, 1


@pytest.mark.parametrize("kind", ["mcmc", "mcmc_random"])
def test_mhm_matches_text_oracle(victim, kind):
    """MHM-NS baseline (attacker.py:466-738) at the config-5 shape: product MHM_Attacker (host
    mutants, engine scoring) vs oracle/mhm_ref.py over text, same Python `random` seed: identical
    outcome, adversarial code, replacement chain and query count over 100-iteration chains."""
    from apmc_amd.attacker import MHM_Attacker
    from apmc_amd.drivers import AttackArgs, load_fixture
    from apmc_amd.host import Tokenizer
    from apmc_amd.utils import isUID
    from oracle import mhm_ref

    codes, subs, labels = load_fixture(FIXTURE, 0, 120)
    tok = Tokenizer()
    args = AttackArgs(block_size=MHM_BLOCK, eval_batch_size=64)
    vocab = sorted({w for s in subs[:60] for v in s.values() for w in v})
    idx2token = vocab if kind == "mcmc_random" else None
    att = MHM_Attacker(args, victim, None, tok, {w: i for i, w in enumerate(vocab)}, vocab)
    seen = []
    for i in _pick(codes, subs, 5):
        code, sb, lab = codes[i], subs[i], labels[i]
        random.seed(3000 + i)
        q0 = victim.query
        res = getattr(att, kind)(tok, sb, code, lab, _n_candi=30, _max_iter=MHM_ITERS,
                                 _prob_threshold=MHM_THRESHOLD)
        q_prod = victim.query - q0
        random.seed(3000 + i)
        v = attack_ref.Victim(_score_fn(victim), MHM_BLOCK)
        ref = mhm_ref.mcmc(v, isUID, sb, code, lab, n_candi=30, max_iter=MHM_ITERS,
                           prob_threshold=MHM_THRESHOLD, idx2token=idx2token)
        assert res["succ"] == ref["succ"], i
        assert q_prod == v.query, (i, q_prod, v.query)
        if res["succ"] is not None:
            for k in ("tokens", "replace_info", "nb_changed_var", "nb_changed_pos",
                      "prog_length", "new_pred"):
                assert res[k] == ref[k], (i, k)
        seen.append(res["succ"])
    print(kind, seen)
    assert any(s is not None for s in seen)


def test_authorship_mhm_matches_text_oracle():
    """Config 5's baseline half: MHM-NS on the 66-way authorship victim
    (CodeXGLUE/Authorship-Attribution/code/attacker.py:440-666, driven as mhm.py:160-213: Python
    leaves, raw-text features, argmax predictions; block 512, n_candi 30, max_iter 100,
    _prob_threshold 1) on the HIP engine against oracle/mhm_ref.py scoring the same mutant texts
    with the same engine: identical outcome, adversarial code, replacement chain and query count.
    Labels are the victim's own predictions (the synthetic victim does not know the authors), so
    every program is attacked; the sample must include a success."""
    from apmc_amd.attacker import AuthorshipMHM_Attacker
    from apmc_amd.drivers import AttackArgs, _example
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import Model
    from apmc_amd.utils import isUID
    from oracle import mhm_ref
    from test_task_attacks import fixture

    model = Model(synthetic_sd(seed=5, head="softmaxN", num_labels=66, out_std=8.0),
                  task="authorship")

    def score(ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        lens = (ids != 1).sum(1).astype(np.int32)
        return model.engine.score(torch.from_numpy(ids).cuda(), lens).cpu().numpy()

    codes, subs, _ = fixture("authorship", 6)
    tok = Tokenizer()
    labels = [int(p) for p in model.get_results([_example(tok, c, 0, MHM_BLOCK, "authorship")
                                                 for c in codes])[1]]
    args = AttackArgs(block_size=MHM_BLOCK, eval_batch_size=64, task="authorship",
                      lang="python")
    vocab = sorted({w for s in subs for v in s.values() for w in v})
    att = AuthorshipMHM_Attacker(args, model, None, tok, {w: i for i, w in enumerate(vocab)},
                                 vocab)
    seen = []
    for i in range(len(codes)):
        random.seed(3300 + i)
        q0 = model.query
        res = att.mcmc(tok, codes[i], labels[i], _n_candi=30, _max_iter=MHM_ITERS,
                       _prob_threshold=MHM_THRESHOLD, subs=subs[i])
        q_prod = model.query - q0
        random.seed(3300 + i)
        v = attack_ref.Victim(score, MHM_BLOCK, task="authorship")
        ref = mhm_ref.mcmc(v, isUID, subs[i], codes[i], labels[i], n_candi=30,
                           max_iter=MHM_ITERS, prob_threshold=MHM_THRESHOLD, lang="python",
                           skip_known=False)
        assert res["succ"] == ref["succ"], i
        assert q_prod == v.query, (i, q_prod, v.query)
        if res["succ"] is not None:
            for k in ("tokens", "replace_info", "nb_changed_var", "nb_changed_pos",
                      "prog_length", "new_pred"):
                assert res[k] == ref[k], (i, k)
        seen.append((res["succ"], q_prod))
    print("authorship mhm", seen)
    assert sum(s is True for s, _ in seen) >= 1 and len(seen) >= 4, seen
    model.engine.close()


def test_mhm_batched_equals_sequential_on_engine(victim):
    """Cross-example batched MHM-NS (mcmc_batched) on the HIP engine at the
    config-5 shape: many chains share each device batch, and every chain still equals
    `random.seed(s); mcmc(...)` run alone (the engine scores rows batch-invariantly), with the
    same per-example query counts."""
    from apmc_amd.attacker import MHM_Attacker
    from apmc_amd.drivers import AttackArgs, load_fixture
    from apmc_amd.host import Tokenizer

    codes, subs, labels = load_fixture(FIXTURE, 0, 120)
    tok = Tokenizer()
    args = AttackArgs(block_size=MHM_BLOCK, eval_batch_size=64)
    vocab = sorted({w for s in subs[:60] for v in s.values() for w in v})
    att = MHM_Attacker(args, victim, None, tok, {w: i for i, w in enumerate(vocab)}, vocab)
    jobs = [(subs[i], codes[i], labels[i], 5000 + i) for i in _pick(codes, subs, 8)]
    seq = []
    for sb, code, lab, seed in jobs:
        random.seed(seed)
        q0 = victim.query
        res = att.mcmc(tok, sb, code, lab, _n_candi=30, _max_iter=MHM_ITERS,
                       _prob_threshold=MHM_THRESHOLD)
        seq.append((res, victim.query - q0))
    got = att.mcmc_batched(tok, jobs, _n_candi=30, _max_iter=MHM_ITERS,
                           _prob_threshold=MHM_THRESHOLD, max_inflight=8)
    for j, ((rs, qs), (rb, qb)) in enumerate(zip(seq, got)):
        assert qs == qb, j
        assert rs == rb, j


@pytest.mark.parametrize("task", ["clone", "authorship"])
def test_task_attack_matches_text_oracle(task):
    """CodeBERT clone-pair victim (pair2 head over [code1 | code2] rows, CloneAttacker) and the
    66-way authorship victim (raw-text features, AuthorshipAttacker) on the HIP engine, against
    the text oracle scoring the same mutant texts with the same engine: identical outcomes,
    query counts, adversarial code and replacements (block 512, batch 64 as the reference
    scripts run).  Labels are the victim's own predictions so every example is attacked."""
    from apmc_amd.drivers import _example
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import Model
    from test_task_attacks import compare_task, fixture

    head, nl = ("pair2", 2) if task == "clone" else ("softmaxN", 66)
    model = Model(synthetic_sd(seed=5, head=head, num_labels=nl, out_std=8.0), task=task)

    def score(ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        lens = (ids != 1).sum(1).astype(np.int32)
        return model.engine.score(torch.from_numpy(ids).cuda(), lens).cpu().numpy()

    codes, subs, _ = fixture(task, 6)
    tok = Tokenizer()
    labels = [int(p) for p in model.get_results([_example(tok, c, 0, CONFIG2_BLOCK, task)
                                                 for c in codes])[1]]
    seen = compare_task(task, model, score, codes, subs, labels, CONFIG2_BLOCK, CONFIG2_BATCH,
                        6000, range(len(codes)))
    print(task, seen)
    assert {o for _, o in seen} & {1, -1}, seen


@pytest.mark.parametrize("task", ["gcb_clone", "gcb_authorship", "gcb_devign"])
def test_gcb_task_attack_matches_text_oracle(task):
    """GraphCodeBERT victims on the HIP engine (graph forward, L = 512 + 128 = 640): the
    GraphCloneAttacker / GraphAuthorshipAttacker / GraphAttacker and the gcb_* drivers against
    the text oracle (oracle/graph_ref.GraphTextVictim) scoring the same texts with the same
    engine: identical outcomes, query counts, adversarial code and replacements."""
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.graph import GraphModel
    from apmc_amd.host import Tokenizer
    from test_task_attacks import compare_gcb_with, fixture

    base = task[4:]
    head, nl = {"clone": ("pair2", 2), "authorship": ("softmaxN", 66),
                "devign": ("sigmoid1", 1)}[base]
    args = AttackArgs(block_size=512, eval_batch_size=32, task=task, code_length=512,
                      data_flow_length=128)
    model = GraphModel(synthetic_sd(seed=5, head=head, num_labels=nl, out_std=8.0), task=base,
                       args=args)
    if base == "devign":
        codes, subs, _ = load_fixture(FIXTURE, 0, 120)
        pick = _pick(codes, subs, 4)
    else:
        codes, subs, _ = fixture(base, 4)
        pick = list(range(4))
    tok = Tokenizer()
    labels = [0] * len(codes)
    for i in pick:
        labels[i] = int(model.get_results([_example(tok, codes[i], 0, 512, task, args)])[1][0])
    seen = compare_gcb_with(task, model, model.score_packed, codes, subs, labels, args, 9000, pick)
    print(task, seen)
    assert {o for _, o in seen} & {1, -1}, seen


# ---- MHM-NS copies of the clone and GraphCodeBERT victims (config 5's GraphCodeBERT half) ----
# config shape: block 512 (CodeBERT clone: two 512-id halves per pair), GraphCodeBERT
# code_length 512 + data_flow_length 128, n_candi 30, 100 iterations, _prob_threshold 1
_MHM_VICTIMS = {}
_MHM_SEEN = {}
MHM_PROGRAMS = 4


def _mhm_victim(task):
    """(victim, oracle scorer, args, codes, subs, labels, programs) of one task, built once."""
    if task in _MHM_VICTIMS:
        return _MHM_VICTIMS[task]
    from apmc_amd.drivers import AttackArgs, _example, load_fixture
    from apmc_amd.graph import GraphModel
    from apmc_amd.host import Tokenizer
    from apmc_amd.model import Model
    from test_task_attacks import fixture

    base = task[4:] if task.startswith("gcb_") else task
    head, nl = {"clone": ("pair2", 2), "authorship": ("softmaxN", 66),
                "devign": ("sigmoid1", 1)}[base]
    sd = synthetic_sd(seed=5, head=head, num_labels=nl, out_std=8.0)
    args = AttackArgs(block_size=512, eval_batch_size=64, task=task, code_length=512,
                      data_flow_length=128)
    if task == "clone":
        model = Model(sd, task="clone")

        def score(ids):
            ids = np.ascontiguousarray(ids, dtype=np.int32)
            lens = (ids != 1).sum(1).astype(np.int32)
            return model.engine.score(torch.from_numpy(ids).cuda(), lens).cpu().numpy()
    else:
        model = GraphModel(sd, task=base, args=args)
        score = model.score_packed
    if base == "devign":
        codes, subs, _ = load_fixture(FIXTURE, 0, 120)
        pick = _pick(codes, subs, MHM_PROGRAMS)
    elif task == "gcb_clone":
        # the GraphCodeBERT clone copy skips no known name, so two variable names can merge and
        # its chain raise KeyError (the reference's own failure, reproduced); the pairs with the
        # fewest substitutable names chain longest without one
        codes, subs, _ = fixture(base, 40)
        pick = sorted(range(40), key=lambda i: (len(subs[i]), i))[:MHM_PROGRAMS]
    else:
        codes, subs, _ = fixture(base, MHM_PROGRAMS)
        pick = list(range(MHM_PROGRAMS))
    tok = Tokenizer()
    labels = [0] * len(codes)
    for i in pick:  # the victim's own predictions: every program is attacked
        labels[i] = int(model.get_results([_example(tok, codes[i], 0, 512, task, args)])[1][0])
    _MHM_VICTIMS[task] = (model, score, args, codes, subs, labels, pick)
    return _MHM_VICTIMS[task]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,prog", [("mcmc", p) for p in range(MHM_PROGRAMS)]
                         + [("mcmc_random", p) for p in range(2)])
@pytest.mark.parametrize("task", ["clone", "gcb_devign", "gcb_authorship", "gcb_clone"])
def test_mhm_variant_matches_text_oracle(task, kind, prog):
    """MHM-NS of the clone and GraphCodeBERT victims on the HIP engine (CloneMHM_Attacker,
    GraphMHM_Attacker, GraphAuthorshipMHM_Attacker, GraphCloneMHM_Attacker; reference
    CodeXGLUE/Clone-detection-BigCloneBench/code/attacker.py:469-800,
    GraphCodeBERT/{Defect-detection,Authorship-Attribution,clonedetection}/code/attacker.py
    MHM_Attacker) against oracle/mhm_ref.py scoring the same candidate texts (featurised by
    the oracle: transformers tokenizer, oracle/graph_ref.py features and masks) with the same
    engine: identical outcome, adversarial code, replacement chain, attack type and query count
    over 100-iteration chains at 512 + 128."""
    from test_mhm_variants import compare_mhm_with

    model, score, args, codes, subs, labels, pick = _mhm_victim(task)
    seen = compare_mhm_with(task, kind, model, score, args, codes, subs, labels, [pick[prog]],
                            MHM_ITERS, 3700, vocab_pick=pick)
    print(task, kind, prog, seen)
    _MHM_SEEN.setdefault(task, []).extend(s for s, _ in seen)


@pytest.mark.parametrize("task", ["clone", "gcb_devign", "gcb_authorship", "gcb_clone"])
def test_mhm_variant_sample_includes_success(task):
    """Each task's sample above includes a successful chain."""
    got = _MHM_SEEN.get(task, [])
    if len(got) < MHM_PROGRAMS + 2:
        pytest.skip("needs the runs of test_mhm_variant_matches_text_oracle")
    assert True in got, (task, got)
