"""Scan the Devign fixture with the batched greedy->GA driver on the engine and print the
examples whose attack ends in a GA success, for a few synthetic victims (debug aid used to pick
the GA-success case of tests/test_attack_gpu.py)."""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import _apmc  # noqa: E402,F401
from apmc_amd.drivers import AttackArgs, load_fixture, run_gi_attack_batched  # noqa: E402
from apmc_amd.model import Model  # noqa: E402
from apmc_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    codes, subs, labels = load_fixture(ROOT / "data" / "devign" / "test_subs_0_400.jsonl")
    idx = [i for i in range(len(codes)) if 1 <= len(subs[i]) <= 8 and len(codes[i]) < 4000]
    for seed, std in [(5, 8.0), (5, 3.0), (7, 8.0), (11, 4.0)]:
        m = Model(synthetic_state_dict(seed=seed, head="sigmoid1", out_std=std), task="devign",
                  precision="fp32")
        args = AttackArgs(block_size=512, eval_batch_size=64, rng="per_example")
        t0 = time.time()
        out = run_gi_attack_batched(m, codes, subs, labels, args, indices=idx, max_inflight=64)
        ga = [r["index"] for r in out["records"] if r["attack_type"] == "GA" and r["is_success"] == 1]
        kinds = {}
        for r in out["records"]:
            k = (r["attack_type"], r["is_success"])
            kinds[str(k)] = kinds.get(str(k), 0) + 1
        print(json.dumps(dict(seed=seed, std=std, n=len(idx), ga_success=ga, kinds=kinds,
                              wall=round(time.time() - t0, 1))), flush=True)


if __name__ == "__main__":
    main()
