"""GPU debug: run the product greedy->GA attack and the text oracle on one fixture example with
the engine victim, record every victim call (ids digest, rows, probabilities) of both, and print
the first call where they differ.  Writes gpurun_out/ga_divergence.json."""
import hashlib
import json
import pathlib
import random
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _apmc  # noqa: E402,F401
from apmc_amd.attacker import Attacker  # noqa: E402
from apmc_amd.drivers import AttackArgs, _example, load_fixture  # noqa: E402
from apmc_amd.host import Tokenizer  # noqa: E402
from apmc_amd.model import Model  # noqa: E402
from apmc_amd.weights import synthetic_state_dict  # noqa: E402
from oracle import attack_ref  # noqa: E402

EX = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B, BS = 512, 64
log_p, log_o = [], []


def digest(ids):
    a = np.ascontiguousarray(np.asarray(ids, dtype=np.int32))
    return hashlib.sha1(a.tobytes()).hexdigest()[:12], a


class RecModel(Model):
    def score_prepared(self, payloads, threshold=0.5):
        out = super().score_prepared(payloads, threshold)
        for p, (pr, _) in zip(payloads, out):
            ids = p.ids.cpu().numpy() if hasattr(p.ids, "cpu") else p.ids
            d, a = digest(ids)
            log_p.append((d, a, np.asarray(pr, dtype=np.float64)[:, 1].tolist() if len(pr) else []))
        return out


victim = RecModel(synthetic_state_dict(seed=5, head="sigmoid1", out_std=8.0), task="devign")


def score(ids):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    lens = (ids != 1).sum(1).astype(np.int32)
    p = victim.engine.score(torch.from_numpy(ids).cuda(), lens).cpu().numpy()[:, 0]
    d, a = digest(ids)
    log_o.append((d, a, p.astype(np.float64).tolist()))
    return p


codes, subs, labels = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl", 0, 200)
tok = Tokenizer()
args = AttackArgs(block_size=B, eval_batch_size=BS)
att = Attacker(args, victim, tok, None, tok, 1, 0)
code, sb, lab = codes[EX], subs[EX], labels[EX]
random.seed(1000 + EX)
ex = _example(tok, code, lab, B)
res = att.greedy_attack(ex, code, sb)
kind = "greedy"
if res[6] == -1:
    res = att.ga_attack(ex, code, sb, initial_replace=res[11])
    kind = "ga"
random.seed(1000 + EX)
v = attack_ref.Victim(score, B)
ids0 = ex[0].numpy().astype(np.int32)
ref = attack_ref.greedy(v, ids0, lab, code, sb)
if ref["is_success"] == -1:
    ref = attack_ref.ga(v, ids0, lab, code, sb, initial_replace=ref["replaced"], eval_batch_size=BS)
out = {"example": EX, "kind": kind, "prod_success": res[6], "ref_success": ref["is_success"],
       "prod_calls": len(log_p), "ref_calls": len(log_o),
       "prod_queries": sum(len(x[2]) for x in log_p), "ref_queries": sum(len(x[2]) for x in log_o)}
for k, (a, b) in enumerate(zip(log_p, log_o)):
    if a[0] != b[0] or a[2] != b[2]:
        row = {"call": k, "prod_digest": a[0], "ref_digest": b[0], "prod_rows": len(a[2]),
               "ref_rows": len(b[2])}
        if a[1].shape == b[1].shape:
            diff_rows = np.nonzero((a[1] != b[1]).any(1))[0].tolist()
            row["ids_diff_rows"] = diff_rows[:10]
            pdiff = [i for i in range(len(a[2])) if a[2][i] != b[2][i]]
            row["prob_diff_rows"] = pdiff[:10]
            row["prob_pairs"] = [(a[2][i], b[2][i]) for i in pdiff[:5]]
            # same ids, different probability: re-score those rows alone and in the batch
            if pdiff and not diff_rows:
                one = score(a[1][pdiff[:1]])
                row["rescored_alone"] = float(one[0])
        out["first_divergence"] = row
        break
print(json.dumps(out))
(ROOT / "gpurun_out").mkdir(exist_ok=True)
(ROOT / "gpurun_out" / "ga_divergence.json").write_text(json.dumps(out))
