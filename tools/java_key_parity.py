"""Java DFG key parity over the 4,000 BigCloneBench code1 functions the reference holds
(tests/golden/bcb_java_keys.jsonl.gz, made by tests/golden/make_bcb_java_keys.py).

    python tools/java_key_parity.py [--dump out.jsonl] [--show N]

Prints exact / truncation-consistent / ordered-subsequence counts per fixture file and overall
(the same classification as tests/test_host.py::key_parity), and dumps every non-exact function
with our names, the reference keys and the set differences, for the residue table in DESIGN §5.
"""
import argparse
import gzip
import json
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _apmc  # noqa: F401,E402  (registers the package as apmc_amd)

FIXTURE = ROOT / "tests" / "golden" / "bcb_java_keys.jsonl.gz"


def classify(code, keys, tok):
    from apmc_amd.substitutes import substitute_identifiers
    from apmc_amd.utils import (_tokenize, get_identifier_posistions_from_code,
                                is_valid_variable_name)
    idents, toks = substitute_identifiers(code, "java")
    words, sub_words, kk = _tokenize(" ".join(toks), tok)
    names = [i[0] for i in idents if " " not in i[0].strip()]
    pos = get_identifier_posistions_from_code(words, names)
    ours = [n for n in pos if is_valid_variable_name(n, "java")]
    it = iter(ours)
    subseq = all(k in it for k in keys)
    if ours == keys:
        return "exact", ours, len(sub_words)
    if keys and len(sub_words) > 380 and all(k in pos for k in keys):
        last = max(kk[pos[k][0]][0] for k in keys)
        if [n for n in ours if kk[pos[n][0]][0] <= last] == keys:
            return "consistent", ours, len(sub_words)
    return ("subsequence" if subseq else "other"), ours, len(sub_words)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", default=None)
    ap.add_argument("--show", type=int, default=0)
    ap.add_argument("--only", default=None, help="one fixture span, e.g. 500_1000")
    a = ap.parse_args()
    from apmc_amd.host import Tokenizer
    tok = Tokenizer()
    per = {}
    dump = open(a.dump, "w") if a.dump else None
    shown = 0
    with gzip.open(FIXTURE, "rt", encoding="utf-8") as f:
        for line in f:
            js = json.loads(line)
            if a.only and js["file"] != a.only:
                continue
            cls, ours, nsub = classify(js["code1"], js["keys"], tok)
            c = per.setdefault(js["file"], Counter())
            c[cls] += 1
            c["total"] += 1
            if cls != "exact" and dump:
                dump.write(json.dumps({"file": js["file"], "row": js["row"], "cls": cls,
                                       "nsub": nsub, "ours": ours, "keys": js["keys"],
                                       "extra": [n for n in ours if n not in js["keys"]],
                                       "missing": [k for k in js["keys"] if k not in ours]})
                           + "\n")
            if cls in ("subsequence", "other") and shown < a.show:
                shown += 1
                print(js["file"], js["row"], cls, "extra", [n for n in ours if n not in js["keys"]],
                      "missing", [k for k in js["keys"] if k not in ours])
    tot = Counter()
    for span, c in per.items():
        tot.update(c)
        ex, cons = c["exact"], c["exact"] + c["consistent"]
        sub = cons + c["subsequence"]
        print(f"{span:>10}: exact {ex} consistent {cons} subsequence {sub} of {c['total']}")
    ex, cons = tot["exact"], tot["exact"] + tot["consistent"]
    print(f"{'all':>10}: exact {ex} consistent {cons} subsequence {cons + tot['subsequence']} "
          f"of {tot['total']}")


if __name__ == "__main__":
    main()
