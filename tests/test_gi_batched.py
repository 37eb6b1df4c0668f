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
