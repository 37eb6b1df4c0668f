"""Same-box A/B of whole engine libraries (GPU): the headline scoring step (B = 64 x L = 512,
bench.py's id recipe, f32x3, sigmoid head, synthetic weights) and the ragged Devign-length batch
through Engine built on the library at --lib (default: the in-tree product library).  Run it in
alternating processes over two libraries (tools/engine_lib_ab.sh); one JSON line per process.

  python tools/engine_lib_ab.py [--lib lib/exp/libalert_engine_prefold.so] [--steps 20]
"""
import argparse
import json
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _apmc  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import apmc_amd.engine as em
    from apmc_amd.weights import synthetic_state_dict
    if args.lib:
        lib = em.load_library(args.lib)
        em.load_library = lambda path=None, tools=False: lib  # Engine binds this library
    eng = em.Engine(synthetic_state_dict(seed=0, head="sigmoid1"), head="sigmoid1",
                    precision="f32x3")
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    out = {"lib": args.lib or "in-tree"}
    n, L = 64, 512
    ids = rng.integers(4, 50264, size=(n, L)).astype(np.int32)
    ids[:, 0], ids[:, -1] = 0, 2
    cases = {"full": (ids, np.full(n, L, np.int32))}
    lens = np.clip(rng.lognormal(np.log(274), 0.6, n), 8, 512).astype(np.int32)
    rid = ids.copy()
    for i, x in enumerate(lens):
        rid[i, x - 1], rid[i, x:] = 2, 1
    cases["ragged"] = (rid, lens)
    # an attack round: 16 populations of 64 mutants, each population one program's length (the
    # fixture's length distribution), concatenated as the cross-example driver does
    nb, pop = 16, 64
    plen = np.clip(rng.lognormal(np.log(380), 0.5, nb), 40, 512).astype(np.int32)
    blens = np.repeat(plen, pop)
    bid = rng.integers(4, 50264, size=(nb * pop, L)).astype(np.int32)
    bid[:, 0] = 0
    for i, x in enumerate(blens):
        bid[i, x - 1], bid[i, x:] = 2, 1
    cases["blocks"] = (bid, blens)
    res = torch.empty((nb * pop, 1), device=dev)
    st = torch.cuda.current_stream(dev)
    for name, (x, ln) in cases.items():
        xd = torch.from_numpy(x).to(dev)
        steps = args.steps if x.shape[0] <= 64 else max(2, args.steps // 8)
        for _ in range(3):
            eng.score(xd, ln, out=res[:x.shape[0]], stream=st)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.score(xd, ln, out=res[:x.shape[0]], stream=st)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3 / steps)
        out[name + "_ms"] = round(statistics.median(ts), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
