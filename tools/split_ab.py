"""A/B of the two-stream encoder (AE_SPLIT_STREAMS=1) against the single-stream fused path on the
bench's scoring step (GPU): interleaved rounds of `--steps` steps each, in one process, and the
max |dp| between the two engines' probabilities (full-length and ragged batches).

  python tools/split_ab.py [--steps 10] [--rounds 5]
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
    args = ap.parse_args()

    import numpy as np
    import torch

    import _apmc  # noqa: F401
    from apmc_amd.engine import Engine
    from apmc_amd.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    sd = synthetic_state_dict(seed=0, head="sigmoid1")
    engines = {}
    for mode in ("0", "1"):
        os.environ["AE_SPLIT_STREAMS"] = mode
        engines[mode] = Engine(sd, head="sigmoid1", num_labels=1, precision=args.precision,
                               device=0)
    os.environ.pop("AE_SPLIT_STREAMS")
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
        d = float((outs["0"] - outs["1"]).abs().max())
        res[name] = {"ms_per_step_single": round(statistics.median(times["0"]), 3),
                     "ms_per_step_split": round(statistics.median(times["1"]), 3),
                     "tokens": int(lens.sum()), "max_abs_dprob_split_vs_single": d}
        print(json.dumps({name: res[name]}), flush=True)
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
