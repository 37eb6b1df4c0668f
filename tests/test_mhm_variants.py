"""The MHM-NS copies of the clone and GraphCodeBERT victims against the text oracle
(oracle/mhm_ref.py), on deterministic numpy stand-in victims (no engine on this host):

  CloneMHM_Attacker            CodeXGLUE/Clone-detection-BigCloneBench/code/attacker.py:469-800
  GraphMHM_Attacker            GraphCodeBERT/Defect-detection/code/attacker.py:467-737
  GraphAuthorshipMHM_Attacker  GraphCodeBERT/Authorship-Attribution/code/attacker.py:479-741
  GraphCloneMHM_Attacker       GraphCodeBERT/clonedetection/code/attacker.py:496-800

Product (host mutants, C++ featurisation — spliced ids for CodeBERT, compact data-flow features
for GraphCodeBERT) and oracle (every candidate rebuilt as text by oracle.featurize_ref and
featurised by the transformers tokenizer / oracle.graph_ref) run under the same Python `random`
seed and must agree on outcome, adversarial code, replacement chain, attack type and query
count.  Then the batched driver (many chains per device batch) against the sequential loop.
The GPU versions: tests/test_attack_gpu.py::test_mhm_variant_matches_text_oracle."""
import random

import numpy as np
import pytest

from conftest import ROOT

BLOCK = 128
KEYS = ("tokens", "replace_info", "nb_changed_var", "nb_changed_pos", "prog_length", "new_pred",
        "attack_type", "old_uid", "is_success")
# skip rules and random label of each copy (read from the reference as text)
VARIANT = {"clone": dict(skip_known=True, skip_known_subs=True, random_type="Ori_MHM"),
           "gcb_devign": dict(skip_known=True, skip_known_subs=True, random_type="Ori_MHM"),
           "gcb_authorship": dict(skip_known=True, skip_known_subs=True, random_type="Ori_MHM"),
           "gcb_clone": dict(skip_known=False, skip_known_subs=False, random_type="Ori_MHM")}


def _load(task, n):
    from apmc_amd.drivers import load_fixture
    from test_task_attacks import fixture

    base = task[4:] if task.startswith("gcb_") else task
    if base == "devign":
        codes, subs, _ = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl", 0, 40)
        pick = [i for i in range(40) if 1 <= len(subs[i]) <= 4 and len(codes[i]) < 900][:n]
    else:
        codes, subs, _ = fixture(base, n)
        pick = list(range(n))
    return codes, subs, pick


def _victim(task, args):
    """(product victim, numpy score, labeller) of the task's stand-in."""
    from apmc_amd.model import HostIdsVictim
    from test_task_attacks import graph_stand_in, host_graph_victim, stand_in

    if task == "clone":
        score = stand_in("clone")
        return HostIdsVictim(score, task="clone", block_size=BLOCK), score
    base = task[4:]
    score = graph_stand_in(base)
    v = host_graph_victim(score, base)
    v.args = args
    return v, score


def _raised(fn, *a, **k):
    try:
        return fn(*a, **k)
    except (KeyError, ValueError) as e:
        return e


def compare_mhm(task, kind, n=5, max_iter=12, seed0=3500):
    """Product vs oracle on `n` fixture programs over the task's numpy stand-in."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, _example
    from apmc_amd.host import Tokenizer
    from test_task_attacks import GCB_ARGS

    codes, subs, pick = _load(task, n)
    gcb = task.startswith("gcb_")
    args = AttackArgs(block_size=256 if gcb else BLOCK, eval_batch_size=32, task=task,
                      **(GCB_ARGS if gcb else {}))
    victim, score = _victim(task, args)
    tok = Tokenizer()
    labels = [0] * len(codes)
    for i in pick:
        labels[i] = int(victim.get_results([_example(tok, codes[i], 0, args.block_size, task,
                                                     args)])[1][0])
    return compare_mhm_with(task, kind, victim, score, args, codes, subs, labels, pick,
                            max_iter, seed0)


def compare_mhm_with(task, kind, victim, score, args, codes, subs, labels, pick, max_iter, seed0,
                     vocab_pick=None):
    """Product MHM (the task's MHM_Attacker copy, driven in its reference call form) vs
    oracle/mhm_ref.mcmc over text, same seed per program; returns [(succ | "raised", queries)].
    score: the oracle victim's scorer (ids -> head outputs; GraphCodeBERT: (ids, pos, bits))."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import _example, _mhm_call, make_mhm_attacker
    from apmc_amd.host import Tokenizer
    from apmc_amd.utils import isUID
    from oracle import attack_ref, mhm_ref
    from oracle.graph_ref import GraphTextVictim

    gcb = task.startswith("gcb_")
    tok = Tokenizer()
    att = make_mhm_attacker(args, victim, tok, [codes[i] for i in (vocab_pick or pick)])
    vocab = att.idx2token
    clone = task in ("clone", "gcb_clone")
    seen = []
    for i in pick:
        code, sb, lab = codes[i], subs[i], labels[i]
        ex = _example(tok, code, lab, args.block_size, task, args)
        random.seed(seed0 + i)
        q0 = victim.query
        res = _raised(_mhm_call, att, task, tok, code, sb, lab, ex, 30, max_iter, 1,
                      kind == "mcmc_random")
        q_prod = victim.query - q0
        random.seed(seed0 + i)
        text = code[2] if clone else code
        if gcb:
            v = GraphTextVictim(score, task, text, code2=code[3] if clone else None,
                                code_length=args.code_length,
                                data_flow_length=args.data_flow_length)
        else:
            v = attack_ref.Victim(score, args.block_size, task=task,
                                  code2=code[3] if clone else None)
        pair_example = None
        if clone:
            pair_example = np.zeros(1) if gcb else ex[0].numpy().astype(np.int32)
        lang = {"clone": "java", "gcb_clone": "java", "gcb_devign": "c",
                "gcb_authorship": "python"}[task]
        ref = _raised(mhm_ref.mcmc, v, isUID, sb, text, lab, n_candi=30, max_iter=max_iter,
                      prob_threshold=1, idx2token=vocab if kind == "mcmc_random" else None,
                      lang=lang, pair_example=pair_example, **VARIANT[task])
        if isinstance(ref, Exception):
            # the reference's own failure (gcb_clone: a candidate that already names a variable
            # is accepted, two names merge in `uid`, and the chain's bookkeeping later raises
            # KeyError) must happen in the product too, at the same query
            assert type(res) is type(ref) and res.args == ref.args, (task, kind, i, res, ref)
            assert q_prod == v.query, (task, kind, i, q_prod, v.query)
            seen.append(("raised", q_prod))
            continue
        assert not isinstance(res, Exception), (task, kind, i, res)
        assert res["succ"] == ref["succ"], (task, kind, i)
        assert q_prod == v.query, (task, kind, i, q_prod, v.query)
        if res["succ"] is not None:
            for k in KEYS + (("orig_label",) if clone else ()):
                assert res[k] == ref[k], (task, kind, i, k, res[k], ref[k])
            assert abs(res["score_info"] - ref["score_info"]) == 0.0
        seen.append((res["succ"], q_prod))
    return seen


@pytest.mark.parametrize("kind", ["mcmc", "mcmc_random"])
@pytest.mark.parametrize("task", ["clone", "gcb_devign", "gcb_authorship", "gcb_clone"])
def test_mhm_variant_matches_text_oracle_cpu(task, kind):
    seen = compare_mhm(task, kind)
    print(task, kind, seen)
    assert any(s is not None for s, _ in seen), seen
    _SEEN.extend(s for s, _ in seen)


_SEEN = []


def test_mhm_variants_reach_success_and_failure_cpu():
    """Over the sample above the chains end both ways (the stand-ins are sharp enough to flip)."""
    if len(_SEEN) < 40:
        pytest.skip("needs the runs of test_mhm_variant_matches_text_oracle_cpu")
    assert True in _SEEN and False in _SEEN, _SEEN


@pytest.mark.parametrize("task", ["clone", "gcb_clone", "gcb_authorship"])
def test_mhm_variant_driver_batched_equals_sequential(task, tmp_path):
    """run_mhm_attack: batched chains (per-example random.Random(seed + index)) against the
    reference loop re-seeded per example — same records, queries and writemhm rows."""
    import csv

    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, _example, run_mhm_attack
    from apmc_amd.host import Tokenizer
    from test_task_attacks import GCB_ARGS

    codes, subs, pick = _load(task, 6)
    gcb = task.startswith("gcb_")
    mk = lambda seed, csv_path=None: AttackArgs(  # noqa: E731
        block_size=256 if gcb else BLOCK, eval_batch_size=32, task=task, seed=seed,
        csv_store_path=csv_path, on_error="record", **(GCB_ARGS if gcb else {}))
    args = mk(123456, str(tmp_path / "bat.csv"))
    victim, _ = _victim(task, args)
    tok = Tokenizer()
    labels = [int(victim.get_results([_example(tok, c, 0, args.block_size, task, args)])[1][0])
              for c in codes]
    labels[1] = 1 - labels[1] if task != "gcb_authorship" else (labels[1] + 1) % 66  # one -4 exit
    bat = run_mhm_attack(victim, codes, subs, labels, args, tok=tok, max_iter=8, max_inflight=4)
    seq = []
    for i in range(len(codes)):
        v_args = mk(123456 + i, str(tmp_path / f"seq{i}.csv"))
        q0 = victim.query
        out = run_mhm_attack(victim, codes, subs, labels, v_args, indices=[i], tok=tok,
                             max_iter=8)
        assert out["queries"] == victim.query - q0
        seq.append(out["records"][0])
    assert bat["records"] == seq
    assert bat["records"][1]["is_success"] == -4
    rows = list(csv.reader(open(tmp_path / "bat.csv")))
    attacked = [r for r in seq if r["is_success"] in (1, -1)]
    assert len(rows) == 1 + len(attacked)
    from apmc_amd.drivers import MHM_JOINED_TOKENS
    for row, r in zip(rows[1:], attacked):
        assert int(row[0]) == r["index"] and row[13] == r["attack_type"]
        assert int(row[14]) == r["queries"]
        # each task driver's own writemhm columns (drivers.writemhm_columns)
        adv = r["adv_code"]
        assert row[3] == (" ".join(adv) if task in MHM_JOINED_TOKENS else adv)
        if task == "clone":
            assert row[1].startswith("CODE1: ") and " ||CODE2: " in row[1]
        elif task == "gcb_clone":
            assert row[1] == str(list(codes[-1]))
        else:
            assert row[1] == codes[r["index"]]


def test_gcb_clone_writemhm_row_uses_the_eval_lists_last_pair():
    """GraphCodeBERT/clonedetection/code/mhm_attack.py:162/:221 writes its leftover loop variable
    — the eval list's LAST pair — as every row's Original Code: the driver takes it
    from `last_code` (default codes[-1]), so a caller attacking a slice still writes the whole
    list's last pair; the other tasks write the example's own code."""
    from apmc_amd.drivers import writemhm_columns
    pair = ["int a;", "int b;", "1", "2"]
    last = ["void f() {}", "void g() {}", "9", "10"]
    text, adv = writemhm_columns("gcb_clone", pair, ["x", "y"], last_code=last)
    assert text == str(last)
    text, _ = writemhm_columns("gcb_clone", pair, ["x", "y"])
    assert text == str(pair)
    text, _ = writemhm_columns("devign", "int main() {}", "x y")
    assert text == "int main() {}"
