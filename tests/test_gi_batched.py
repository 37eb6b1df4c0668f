"""Cross-example batched greedy -> GA attack:
`drivers.run_gi_attack_batched` keeps many examples' attacks in flight and answers all their
pending victim requests with ONE scoring call.  Every record must equal the sequential driver's
run under the per-example RNG (`random.seed(seed + index)` before each example): same outcome,
attack type, adversarial code, replacements and per-example query count, and the victim's query
counter must advance by the same total.  The victim is a deterministic numpy stand-in over the
real featurised ids (C++ host library) behind the product request API (HostIdsVictim); the GPU
version of this equivalence is tests/test_attack_gpu.py::test_batched_gi_equals_sequential."""
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
FIXTURE = ROOT / "data" / "devign" / "test_subs_0_400.jsonl"
N_EX = 24
KEYS = ["index", "is_success", "attack_type", "queries", "adv_code", "replace_info",
        "nb_changed_var", "nb_changed_pos", "prog_length"]


def _victim(batches=None):
    import _apmc  # noqa: F401
    from apmc_amd.model import HostIdsVictim

    w = np.random.default_rng(7).standard_normal(50265)

    def score(ids):
        if batches is not None:
            batches.append(ids.shape[0])
        z = np.where(ids != 1, w[ids], 0.0).sum(1) / 6.0
        return (1.0 / (1.0 + np.exp(-z))).astype(np.float32)[:, None]

    return HostIdsVictim(score)


def test_batched_gi_attack_equals_sequential(tmp_path):
    import _apmc  # noqa: F401
    from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack, run_gi_attack_batched

    codes, subs, labels = load_fixture(FIXTURE, 0, N_EX)
    args = AttackArgs(block_size=128, eval_batch_size=16, rng="per_example",
                      csv_store_path=str(tmp_path / "seq.csv"))
    v_seq = _victim()
    seq = run_gi_attack(v_seq, codes, subs, labels, args)
    batches = []
    v_bat = _victim(batches)
    args_b = AttackArgs(block_size=128, eval_batch_size=16, rng="per_example",
                        csv_store_path=str(tmp_path / "bat.csv"))
    bat = run_gi_attack_batched(v_bat, codes, subs, labels, args_b, max_inflight=8)
    a = [{k: r[k] for k in KEYS} for r in seq["records"]]
    b = [{k: r[k] for k in KEYS} for r in bat["records"]]
    assert a == b
    assert v_seq.query == v_bat.query == seq["queries"] == bat["queries"]
    # the sample exercises both attacks and at least one success
    kinds = {(r["attack_type"], r["is_success"]) for r in seq["records"]}
    assert any(k[0] == "GA" for k in kinds) and any(k[1] == 1 for k in kinds), kinds
    # many examples shared the scoring calls: far fewer, far larger batches
    assert max(batches) > 16 and len(batches) < v_seq.query / 4
    # the CSVs agree except the time column
    rows = lambda p: [r.rsplit(",", 1)[0] for r in p.read_text().splitlines()]  # noqa: E731
    assert rows(tmp_path / "seq.csv") == rows(tmp_path / "bat.csv")


def _task_victim(task, batches=None):
    """Deterministic stand-ins of the clone victim (pair rows [2n, L] -> [n, 2] softmax) and the
    authorship victim (rows -> [n, 66] softmax) behind the same request API."""
    import _apmc  # noqa: F401
    from apmc_amd.model import HostIdsVictim

    rng = np.random.default_rng(11)
    if task == "clone":
        w = rng.standard_normal(50265)

        def score(ids):
            if batches is not None:
                batches.append(ids.shape[0] // 2)
            s = np.where(ids != 1, w[ids], 0.0).sum(1).reshape(-1, 2)
            p = 1.0 / (1.0 + np.exp(-(s[:, 0] - s[:, 1]) / 4.0))
            return np.stack([p, 1 - p], 1).astype(np.float32)
    else:
        w = rng.standard_normal((50265, 66))

        def score(ids):
            if batches is not None:
                batches.append(ids.shape[0])
            z = (w[ids] * (ids != 1)[..., None]).sum(1) / 3.0
            z = np.exp(z - z.max(1, keepdims=True))
            return (z / z.sum(1, keepdims=True)).astype(np.float32)
    return HostIdsVictim(score, task=task, block_size=128)


@pytest.mark.parametrize("task", ["clone", "authorship"])
def test_batched_task_attack_equals_sequential(task, tmp_path):
    """Clone pairs (CloneAttacker: code1 perturbed, word-level importance rows, subs-first call)
    and authorship (raw-text features, Python identifiers) through the same batched driver.
    Labels are the stand-in victim's own predictions so every example is attacked."""
    import _apmc  # noqa: F401
    from apmc_amd.drivers import (AttackArgs, _example, load_fixture, run_gi_attack,
                                  run_gi_attack_batched)
    from apmc_amd.host import Tokenizer

    if task == "clone":
        codes, subs, labels = load_fixture(ROOT / "data" / "clone" / "test_subs_0_500.jsonl", 0, 10)
    else:
        codes, subs, labels = load_fixture(ROOT / "data" / "authorship" / "valid_subs.jsonl", 0, 10,
                                           labels_path=ROOT / "data" / "authorship" / "valid.txt")
    tok = Tokenizer()
    probe = _task_victim(task)
    labels = [int(probe.get_results([_example(tok, c, 0, 128, task)])[1][0]) for c in codes]
    mk = lambda name: AttackArgs(block_size=128, eval_batch_size=16, rng="per_example",  # noqa
                                 task=task, csv_store_path=str(tmp_path / name))
    v_seq = _task_victim(task)
    seq = run_gi_attack(v_seq, codes, subs, labels, mk("seq.csv"), tok=tok)
    batches = []
    v_bat = _task_victim(task, batches)
    bat = run_gi_attack_batched(v_bat, codes, subs, labels, mk("bat.csv"), tok=tok, max_inflight=8)
    a = [{k: r[k] for k in KEYS} for r in seq["records"]]
    b = [{k: r[k] for k in KEYS} for r in bat["records"]]
    assert a == b
    assert v_seq.query == v_bat.query == seq["queries"] == bat["queries"]
    outcomes = {r["is_success"] for r in seq["records"]}
    assert outcomes & {1, -1}, outcomes  # attacks ran (not all skipped)
    assert max(batches) > 16
