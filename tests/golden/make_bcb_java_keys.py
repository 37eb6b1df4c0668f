"""Java DFG known answers from the reference's own BigCloneBench fixtures.

Reads the eight `CodeXGLUE/Clone-detection-BigCloneBench/dataset/test_subs_{a}_{b}.jsonl` files the
reference holds (4,000 code1 functions, produced by that directory's get_substitutes.py:74-165:
`get_identifiers(code1, 'java')` -> the validity filters -> names with at least one substitute)
and keeps, per function, only what the key-parity test reads: the code1 text and the ordered list
of substitute keys.  Data, not source: the keys are the reference's recorded outputs.

    python tests/golden/make_bcb_java_keys.py [/root/reference]

writes tests/golden/bcb_java_keys.jsonl.gz (one line per function, file order, `{"file", "row",
"code1", "keys"}`).
"""
import gzip
import json
import sys
from pathlib import Path

SPANS = ["0_500", "500_1000", "1000_1500", "1500_2000", "2000_2500", "2500_3000", "3000_3500",
         "3500_4000"]


def main(ref_root="/root/reference"):
    src = Path(ref_root) / "CodeXGLUE" / "Clone-detection-BigCloneBench" / "dataset"
    out = Path(__file__).resolve().parent / "bcb_java_keys.jsonl.gz"
    n = 0
    with gzip.open(out, "wt", encoding="utf-8", compresslevel=9) as f:
        for span in SPANS:
            with open(src / f"test_subs_{span}.jsonl", encoding="utf-8") as g:
                for row, line in enumerate(g):
                    js = json.loads(line)
                    f.write(json.dumps({"file": span, "row": row, "code1": js["code1"],
                                        "keys": list(js["substitutes"].keys())}) + "\n")
                    n += 1
    print(f"{n} functions -> {out}")


if __name__ == "__main__":
    main(*sys.argv[1:])
