"""Where the config-2 attack leg's time goes (GPU): the bench's greedy -> GA attack over the first
--examples of test_subs_0_400 (cross-example batching, the bench's settings), once under cProfile
(host functions by own time) — run it under `rocprofv3 --kernel-trace` too and feed the trace to
`--busy` for the device-busy fraction over the leg.

  python tools/attack_profile.py --examples 200 [--profile out.txt]
  python tools/attack_profile.py --busy gpurun_out/<tag>/trace/run_kernel_trace.csv
"""
import argparse
import cProfile
import csv
import io
import json
import pathlib
import pstats
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def busy(path):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                  for r in csv.DictReader(open(path)))
    t0, t1 = rows[0][0], max(e for _, e in rows)
    tot, cs, ce = 0, None, None
    for s, e in rows:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print(json.dumps({"kernels": len(rows), "span_s": (t1 - t0) / 1e9, "busy_s": tot / 1e9,
                      "busy_frac": tot / (t1 - t0)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=200)
    ap.add_argument("--profile", default=None)
    ap.add_argument("--busy", default=None)
    args = ap.parse_args()
    if args.busy:
        return busy(args.busy)
    import torch

    import _apmc  # noqa: F401
    import bench
    from apmc_amd.dist import run_sharded_gi_batched
    from apmc_amd.drivers import AttackArgs, load_fixture
    from apmc_amd.model import Model
    from apmc_amd.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    codes, subs, labels = load_fixture(bench.FIXTURE, 0, args.examples)
    model = Model(synthetic_state_dict(seed=bench.VICTIM_SEED, head="sigmoid1",
                                       out_std=bench.VICTIM_OUT_STD),
                  task="devign", precision="f32x3", device=0)
    aargs = AttackArgs(block_size=512, eval_batch_size=64, seed=123456, rng="per_example")
    prof = cProfile.Profile() if args.profile else None
    t0 = time.time()
    if prof:
        prof.enable()
    _, t = run_sharded_gi_batched(model, codes, subs, labels, aargs, max_inflight=64,
                                  device=dev, deadline=time.time() + 600, key="prof_queue")
    if prof:
        prof.disable()
    wall = time.time() - t0
    print(json.dumps({"examples": t["examples"], "queries": t["queries"], "wall_s": round(wall, 2),
                      "victim_queries_per_s": round(t["queries"] / wall, 1)}))
    if prof:
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
        pathlib.Path(args.profile).write_text(s.getvalue())
    model.engine.close()


if __name__ == "__main__":
    main()
