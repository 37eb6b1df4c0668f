"""Builds data/tokenizer/{vocab.json,merges.txt}: a byte-level BPE with RoBERTa's layout.

The reference loads `RobertaTokenizer.from_pretrained("microsoft/codebert-base-mlm")`
(CodeXGLUE/Defect-detection/code/gi_attack.py:126,151) — unavailable offline.  This trains a
GPT-2/RoBERTa-style byte-level BPE with the installed `tokenizers` 0.22.2 on the attack fixtures'
source code (data/devign/*.jsonl `func`, data/authorship/valid_subs.jsonl `code`) and lays the
vocabulary out like codebert's: <s>=0, <pad>=1, </s>=2, <unk>=3, learned tokens from 4, and
<mask>=50264 (vocab size 50265; unused slots between the learned tokens and <mask> are filled with
unreachable placeholder strings).

Run:  python tools/make_tokenizer.py
"""
import json
import pathlib

from tokenizers import ByteLevelBPETokenizer

ROOT = pathlib.Path(__file__).resolve().parents[1]
OUT = ROOT / "data" / "tokenizer"
VOCAB = 50265


def corpus():
    for f in sorted((ROOT / "data" / "devign").glob("test_subs_*.jsonl")):
        for line in open(f):
            yield json.loads(line)["func"]
    for line in open(ROOT / "data" / "authorship" / "valid_subs.jsonl"):
        js = json.loads(line)
        yield js.get("code") or js.get("func") or ""


def main():
    tok = ByteLevelBPETokenizer(add_prefix_space=False)
    tok.train_from_iterator(corpus(), vocab_size=VOCAB - 1, min_frequency=2,
                            special_tokens=["<s>", "<pad>", "</s>", "<unk>"])
    vocab = json.loads(tok.to_str())["model"]["vocab"]
    merges = json.loads(tok.to_str())["model"]["merges"]
    ordered = sorted(vocab.items(), key=lambda kv: kv[1])
    assert [k for k, _ in ordered[:4]] == ["<s>", "<pad>", "</s>", "<unk>"]
    out = {k: i for i, (k, _) in enumerate(ordered)}
    n = len(out)
    assert n <= VOCAB - 1
    for i in range(n, VOCAB - 1):
        out[f"<unused_{i}>"] = i
    out["<mask>"] = VOCAB - 1
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "vocab.json").write_text(json.dumps(out, ensure_ascii=False))
    with open(OUT / "merges.txt", "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n")
        for m in merges:
            a, b = m if isinstance(m, (list, tuple)) else m.split(" ")
            f.write(f"{a} {b}\n")
    print(f"learned {n} tokens, {len(merges)} merges -> {OUT}")


if __name__ == "__main__":
    main()
