"""Tie analysis of two config-3 runs (GPU): why an entry differs between two of our full
get_substitutes runs made on different kernel versions (tools/config3_full.py rundiff).

For every item where the runs differ, the item is generated again here in f32x3 (this tree's
kernels) and in the exact-fp32 mode, with traces, and every cut the differing entries read is
measured on the fp32 run:
  * the 60th / 61st masked-LM logit of each sub-word row of the name's occurrences (top-60,
    get_substitutes.py:63; the 61st from ae_mlm_topk with k = 61),
  * the 30th / 31st cosine score of each occurrence (the naturalness cut, :104-107) and, for a
    multi-sub-word name, every adjacent pair among the first 5 (get_bpe_substitues reads the first
    4 columns in cosine order and caps their cartesian product at 24 in that order,
    utils.py:209-248), and every adjacent pair of its rows' top-60 logits (candidate j is the
    rank-j id of EVERY row of the span, so any swap re-pairs the columns).
The two runs' own f32x3 error is measured on the same items: eps_logit = max |f32x3 - fp32| over
the sorted top-60 scores, eps_sim = max |f32x3 - fp32| over the cosine scores of occurrences whose
60 candidates agree.  An entry is a NEAR TIE when some cut it reads has a gap below 2 eps (both runs
carry an f32x3 error of that size).  Each differing entry also records which run the exact-fp32
mode (pinned to the CPU oracle by the 12-layer substitute tests) agrees with, and whether this
tree's f32x3 reproduces run B (the run made on this tree's kernels).

  python tools/config3_ties.py A1.jsonl,A2.jsonl B1.jsonl,B2.jsonl > profiles/<round>_config3_ties.json
"""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
FUNCS = ROOT / "data" / "devign" / "test_funcs.jsonl"


def load(files):
    out = {}
    for f in files.split(","):
        for line in open(f):
            d = json.loads(line)
            out[d["idx"]] = d["substitutes"]
    return out


def main():
    import torch

    import _apmc  # noqa: F401
    from apmc_amd.engine import Engine
    from apmc_amd.host import Tokenizer
    from apmc_amd.substitutes import K_TOP, SubstituteGenerator, substitute_identifiers
    from apmc_amd.utils import _tokenize
    from apmc_amd.weights import synthetic_state_dict

    a, b = load(sys.argv[1]), load(sys.argv[2])
    funcs = {}
    for line in open(FUNCS):
        d = json.loads(line)
        funcs[d["idx"]] = d["func"]
    differing = {}
    for i in sorted(set(a) & set(b)):
        keys = {k for k in set(a[i]) | set(b[i])
                if k not in a[i] or k not in b[i] or set(a[i][k]) != set(b[i][k])}
        if keys:
            differing[i] = keys
    sd = synthetic_state_dict(seed=0, head="none", with_mlm=True)  # tools/get_substitutes.py's
    tok = Tokenizer()
    e32 = Engine(sd, head="none", with_mlm=True, precision="fp32")
    e3 = Engine(sd, head="none", with_mlm=True, precision="f32x3")
    g32, g3 = SubstituteGenerator(e32, tok, 512), SubstituteGenerator(e3, tok, 512)
    runs, eps_logit, eps_sim = [], 0.0, 0.0
    for i, keys in differing.items():
        idents, code_tokens = substitute_identifiers(funcs[i], "c")
        names = [x[0] for x in idents if " " not in x[0].strip()]
        t32, t3 = {}, {}
        r32 = g32.generate_from_tokens(code_tokens, names, trace=t32)
        r3 = g3.generate_from_tokens(code_tokens, names, trace=t3)
        eps_logit = max(eps_logit, float(np.abs(np.sort(t3["topk_scores"], 1) -
                                                np.sort(t32["topk_scores"], 1)).max()))
        for (w3, p3, s3, c3), (w32, p32, s32, c32) in zip(t3["sims"], t32["sims"]):
            if set(c3) == set(c32):
                d3, d32 = dict(zip(c3, s3)), dict(zip(c32, s32))
                eps_sim = max(eps_sim, max(abs(d3[c] - d32[c]) for c in d32))
        ids = torch.from_numpy(t32["ids"]).cuda()
        sc61, _ = e32.mlm_topk(ids, K_TOP + 1)
        runs.append((i, keys, code_tokens, t32, sc61[1:].cpu().numpy(), r32, r3))
        print(f"[config3_ties] item {i}: {len(runs)} / {len(differing)}", file=sys.stderr, flush=True)
    out = {"items_differing": len(differing), "eps_logit": eps_logit, "eps_sim": eps_sim,
           "entries": []}
    near = 0
    agree = {"fp32_eq_b": 0, "fp32_eq_a": 0, "fp32_eq_neither": 0, "f32x3_now_eq_b": 0}
    for i, keys, code_tokens, t32, sc61, r32, r3 in runs:
        _, _, kk = _tokenize(" ".join(code_tokens), tok)
        for key in sorted(keys):
            gaps_logit, gaps_sim = [], []
            for (w, pos, sims, cands) in t32["sims"]:
                if w != key:
                    continue
                k0, k1 = kk[pos]
                rows = range(k0, min(k1, sc61.shape[0]))
                multi = k1 - k0 > 1
                for r in rows:
                    if multi:  # candidate j pairs the rank-j ids of every row: any adjacent swap
                        gaps_logit.append(float(np.min(sc61[r, :K_TOP] - sc61[r, 1:K_TOP + 1])))
                    else:
                        gaps_logit.append(float(sc61[r, K_TOP - 1] - sc61[r, K_TOP]))
                s = np.sort(np.asarray(sims, np.float64))[::-1]
                gaps_sim.append(float(s[29] - s[30]))
                if multi:  # the first 4 columns, in cosine order (the capped cartesian product)
                    gaps_sim.append(float(np.min(s[:4] - s[1:5])))
            tie = ((gaps_logit and min(gaps_logit) < 2 * eps_logit) or
                   (gaps_sim and min(gaps_sim) < 2 * eps_sim))
            near += bool(tie)
            # which run the exact-fp32 mode (pinned to the CPU oracle) agrees with on this entry
            s32, sa, sb = set(r32.get(key, [])), set(a[i].get(key, [])), set(b[i].get(key, []))
            agree["fp32_eq_b" if s32 == sb else "fp32_eq_a" if s32 == sa else "fp32_eq_neither"] += 1
            agree["f32x3_now_eq_b"] += set(r3.get(key, [])) == sb
            out["entries"].append({"idx": i, "key": key, "near_tie": bool(tie),
                                   "fp32_agrees_with": "b" if s32 == sb else "a" if s32 == sa else None,
                                   "min_logit_gap": min(gaps_logit) if gaps_logit else None,
                                   "min_sim_gap": min(gaps_sim) if gaps_sim else None,
                                   "occurrences": len(gaps_sim)})
    out["entries_differing"] = len(out["entries"])
    out["entries_near_tie"] = near
    out["fp32_agreement"] = agree
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
