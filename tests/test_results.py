"""get_res.py aggregation (apmc_amd.results) over Recorder CSVs written by the product's Recorder.
Known answers computed by hand for the rows below, per the reference scripts' rules:
GraphCodeBERT/Defect-detection/code/get_res.py (sum of Query Times), CodeXGLUE/Authorship-
Attribution/code/get_res.py (successes / rows with Is Success != -4), GraphCodeBERT/Authorship-
Attribution/code/get_res.py (Greedy successes, Index <= 42), CodeXGLUE/Clone-detection-
BigCloneBench/code/get_res.py (changed names of Greedy rows / extracted names)."""
from apmc_amd import results
from apmc_amd.utils import Recorder

ROWS = [  # index, is_success, names, nb_changed, attack_type, queries
    (0, 1, ["a", "b", "c"], 1, "Greedy", 40),
    (3, -1, ["x", "y"], "", "GA", 300),
    (7, -4, ["p"], "", "0", 0),
    (43, 1, ["u", "v"], 2, "GA", 120),
    (50, 1, ["m"], 1, "Greedy", 9),
]


def _write(path, rows):
    r = Recorder(str(path))
    for idx, succ, names, nb, typ, q in rows:
        r.write(idx, "code, with \"quotes\"\nand a newline", 12, "adv", 1, 1, 0, succ, names,
                "", nb, 0, "", typ, q, 0.5)
    r.f.close()


def test_get_res_statistics(tmp_path):
    a, b = tmp_path / "attack_0_400.csv", tmp_path / "attack_400_800.csv"
    _write(a, ROWS[:3])
    _write(b, ROWS[3:])
    both = [a, b]
    assert results.total_queries(both) == 469
    assert results.total_queries(both, "Greedy") == 49
    assert results.success_rate(both) == (3, 4, 0.75)
    assert results.success_rate(both, attack_type="Greedy", max_index=42) == (1, 2, 0.5)
    assert abs(results.changed_names_ratio(both) - 2 / 9) < 1e-12
    assert results.success_rate(a)[:2] == (1, 2)
