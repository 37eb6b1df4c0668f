"""A/B of the split encoder (AE_SPLIT_STREAMS=1: AE_SPLIT_PARTS parts of the batch on as many
streams, each lagging the previous by AE_SPLIT_LAG kernels) against the single-stream fused path on the bench's scoring step (GPU): interleaved
rounds of `--steps` steps each, in one process, and the max |dp| between the engines'
probabilities (full-length and ragged batches).

  python tools/split_ab.py [--steps 10] [--rounds 5] [--lags 1,2,5] [--parts 2,3,4]
"""
import argparse
import json
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--precision", default="f32x3")
    ap.add_argument("--lags", default="1",
                    help="AE_SPLIT_LAG values of the split engines (comma-separated)")
    ap.add_argument("--parts", default="2",
                    help="AE_SPLIT_PARTS values of the split engines (comma-separated)")
    args = ap.parse_args()

    import numpy as np
    import torch

    import _apmc  # noqa: F401
    from apmc_amd.engine import Engine
    from apmc_amd.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    engines = {}
    os.environ["AE_SPLIT_STREAMS"] = "0"
    engines["single"] = Engine(sd, head="sigmoid1", num_labels=1, precision=args.precision, device=0, tools=True)
    os.environ["AE_SPLIT_STREAMS"] = "1"
    for parts in args.parts.split(","):
        for lag in args.lags.split(","):
            os.environ["AE_SPLIT_LAG"] = lag
            os.environ["AE_SPLIT_PARTS"] = parts
            engines[f"p{parts}lag{lag}"] = Engine(sd, head="sigmoid1", num_labels=1,
                                                  precision=args.precision, device=0, tools=True)
    for k in ("AE_SPLIT_STREAMS", "AE_SPLIT_LAG", "AE_SPLIT_PARTS"):
        os.environ.pop(k)
    B, L = 64, 512
    rng = np.random.default_rng(0)
    ids = rng.integers(4, 50264, size=(B, L)).astype(np.int32)
    ids[:, 0], ids[:, -1] = 0, 2
    full = np.full((B,), L, dtype=np.int32)
    ragged = rng.integers(40, L + 1, size=(B,)).astype(np.int32)
    ids_r = ids.copy()
    for i, n in enumerate(ragged):
        ids_r[i, n - 1] = 2
        ids_r[i, n:] = 1
    stream = torch.cuda.current_stream(dev)
    res = {"precision": args.precision}
    for name, x, lens in (("full", ids, full), ("ragged", ids_r, ragged)):
        xd = torch.from_numpy(x).to(dev)
        outs = {m: torch.empty((B, 1), device=dev) for m in engines}
        for m, eng in engines.items():
            for _ in range(3):
                eng.score(xd, lens, out=outs[m], stream=stream)
        torch.cuda.synchronize()
        times = {m: [] for m in engines}
        for _ in range(args.rounds):
            for m, eng in engines.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    eng.score(xd, lens, out=outs[m], stream=stream)
                torch.cuda.synchronize()
                times[m].append((time.perf_counter() - t0) * 1e3 / args.steps)
        res[name] = {"tokens": int(lens.sum())}
        for m in engines:
            res[name][f"ms_per_step_{m}"] = round(statistics.median(times[m]), 3)
            if m != "single":
                res[name][f"max_abs_dprob_{m}_vs_single"] = float((outs[m] - outs["single"]).abs().max())
        print(json.dumps({name: res[name]}), flush=True)
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
