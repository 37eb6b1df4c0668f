"""Config 1 (BASELINE configs[0]) on the CPU reference path, run to completion.

The greedy attack (gi_attack.py without --use_ga) over test_subs_0_400 functions [0, 16) at block
512, with host featurisation and oracle/roberta_cpu.py fp32 eager scoring in batches of 64 — the
same loop as bench.py's config1.cpu leg, without its time cap.  It takes tens of minutes, so it
runs outside the bench; the record (per-function outcome, query count and a hash of the
adversarial code) goes to the JSON file given by --out, and bench.py compares its GPU records
against it.

    python tools/config1_cpu_full.py --threads 8 --out profiles/r3_config1_cpu_full.json
"""
import argparse
import hashlib
import json
import os
import pathlib
import platform
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def record_key(r):
    code = r.get("adv_code")
    return {"is_success": int(r["is_success"]), "queries": int(r["queries"]),
            "adv_code_sha1": hashlib.sha1(code.encode()).hexdigest() if code else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--out", required=True)
    args = ap.parse_args()

    import _apmc  # noqa: F401
    import bench
    from apmc_amd.drivers import load_fixture

    codes, subs, labels = load_fixture(bench.FIXTURE, 0, 16)
    cv = bench.cpu_victim(args.threads)
    cv.state["t0"] = time.time()
    c = bench.greedy_run(cv, codes, subs, labels, list(range(16)))
    rec = {"workload": "config 1: CodeBERT Devign greedy attack (gi_attack.py without --use_ga), "
                       "test_subs_0_400 functions [0, 16), block 512, eval_batch_size 64",
           "kind": "port", "path": "host featurisation + oracle/roberta_cpu.py fp32 eager",
           "cores": args.threads, "host": platform.node(), "cpu_count": os.cpu_count(),
           "examples_completed": c["examples"], "complete": c["examples"] == 16,
           "queries": c["queries"], "successes": c["successes"], "wall_s": round(c["wall_s"], 1),
           "victim_queries_per_s": round(c["queries"] / c["wall_s"], 3),
           "records": [record_key(r) for r in c["records"]]}
    pathlib.Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: v for k, v in rec.items() if k != "records"}))


if __name__ == "__main__":
    main()
