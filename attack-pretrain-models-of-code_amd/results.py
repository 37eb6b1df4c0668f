"""Aggregation of attack result CSVs (the Recorder files) — the reference's get_res.py scripts,
one function per statistic they print, over any list of per-shard CSVs (the reference hard-codes
its shard file names; run.sh writes one CSV per test_subs_* chunk):

  total_queries      GraphCodeBERT/Defect-detection/code/get_res.py:6-17 — sum of "Query Times"
                     over every row (its Greedy filter is commented out; attack_type restores it)
  success_rate       CodeXGLUE/Authorship-Attribution/code/get_res.py:7-21 — successes / rows whose
                     "Is Success" is not -4 (-4 = misclassified before the attack); with
                     attack_type="Greedy" and max_index=42 it is GraphCodeBERT/Authorship-
                     Attribution/code/get_res.py:7-22
  changed_names_ratio CodeXGLUE/Clone-detection-BigCloneBench/code/get_res.py:7-18 — "No. Changed
                     Names" summed over Greedy rows / number of extracted names over all rows
"""
from __future__ import annotations

import csv
import sys

csv.field_size_limit(sys.maxsize)


def read_rows(paths):
    """Rows (dicts keyed by the Recorder header) of every CSV in `paths`, in order."""
    if isinstance(paths, (str, bytes)) or hasattr(paths, "__fspath__"):
        paths = [paths]
    rows = []
    for p in paths:
        with open(p, newline="") as f:
            rows.extend(csv.DictReader(f))
    return rows


def total_queries(paths, attack_type=None):
    return sum(int(r["Query Times"]) for r in read_rows(paths)
               if attack_type is None or r["Attack Type"] == attack_type)


def success_rate(paths, attack_type=None, max_index=None):
    """(successes, attacked, rate): attacked = rows with "Is Success" != -4 (rows past
    max_index skipped); successes = rows with "Is Success" == 1 (and the given attack type)."""
    succ = total = 0
    for r in read_rows(paths):
        if max_index is not None and int(r["Index"]) > max_index:
            continue
        if r["Is Success"] != "-4":
            total += 1
        if r["Is Success"] == "1" and (attack_type is None or r["Attack Type"] == attack_type):
            succ += 1
    return succ, total, (succ / total if total else float("nan"))


def changed_names_ratio(paths):
    changed = names = 0
    for r in read_rows(paths):
        if r["No. Changed Names"] != "" and r["Attack Type"] == "Greedy":
            changed += int(r["No. Changed Names"])
        names += len(r["Extracted Names"].split(","))
    return changed / names if names else float("nan")


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="aggregate attack result CSVs (get_res.py)")
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--stat", choices=["queries", "success", "changed"], default="success")
    ap.add_argument("--attack_type", default=None)
    ap.add_argument("--max_index", type=int, default=None)
    a = ap.parse_args(argv)
    if a.stat == "queries":
        print(total_queries(a.csv, a.attack_type))
    elif a.stat == "success":
        s, t, r = success_rate(a.csv, a.attack_type, a.max_index)
        print(s)
        print(t)
        print(r)
    else:
        print(changed_names_ratio(a.csv))


if __name__ == "__main__":
    main()
