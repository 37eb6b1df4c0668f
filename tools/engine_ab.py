"""Same-box A/B of engine configurations on the bench's scoring step (GPU): one engine per
configuration (each built under its own AE_* environment — AE_ATTN_VARIANT, AE_SPLIT_STREAMS,
AE_SPLIT_PARTS, AE_SPLIT_LAG, AE_GEMM_P2), interleaved rounds of `--steps` steps each in one process, on a
full-length and a ragged B=64 x L=512 batch, with the max |dp| of each against the first.

  python tools/engine_ab.py --configs "prod:;pp6:AE_ATTN_VARIANT=6" [--steps 10] [--rounds 7]
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
KNOBS = ("AE_ATTN_VARIANT", "AE_SPLIT_STREAMS", "AE_SPLIT_PARTS", "AE_SPLIT_LAG",
         "AE_CLS_ABSORB", "AE_GEMM_P2", "AE_SPLIT_PRIO")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", required=True,
                    help="';'-separated name:K=V,K=V (an empty list = the defaults)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
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
    for spec in args.configs.split(";"):
        name, _, kv = spec.partition(":")
        for k in KNOBS:
            os.environ.pop(k, None)
        for item in filter(None, kv.split(",")):
            k, _, v = item.partition("=")
            os.environ[k] = v
        engines[name] = Engine(sd, head="sigmoid1", num_labels=1, precision=args.precision, device=0, tools=True)
    for k in KNOBS:
        os.environ.pop(k, None)
    first = next(iter(engines))
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
    res = {"precision": args.precision, "configs": args.configs}
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
            if m != first:
                res[name][f"max_abs_dprob_{m}_vs_{first}"] = float((outs[m] - outs[first]).abs().max())
        print(json.dumps({name: res[name]}), flush=True)
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
