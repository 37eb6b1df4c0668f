"""Microbenchmark of the packed split-bf16 GEMM kernels on the encoder's shapes (GPU).

Times every (shape, kernel variant) with HIP events on one stream, in interleaved rounds inside
one process (cdna_hip_programming.md §5.4 rule 24), on random operands, and prints one JSON line
per variant: median / min µs per launch and the algorithmic TFLOP/s (2·M·N·K per launch).

  python tools/gemm_bench.py [--shapes ffn1,ffn2,qkv,oproj] [--variants 0,5,1] [--rounds 7]

A variant is "diag" (ae_bench_gemm_packed's DIAG: 0 = production kernel, other values time parts
of the pipeline and give wrong results) optionally with "@bn" (kernel: 512 = the 256 x 256
ping-pong kernel, 192 = the 256 x 192 one, 0 = the production choice) and ":np".
(The folded-LayerNorm epilogues of the engine are timed against their plain forms by
tools/fold_bench.py.)
"""
import argparse
import ctypes
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import _apmc  # noqa: E402,F401

SHAPES = {  # name: (N, K, epilogue) with M = tokens (64 x 512 by default)
    "qkv": (2304, 768, 0),
    "oproj": (768, 768, 0),
    "ffn1": (3072, 768, 1),
    "ffn2": (768, 3072, 0),
    # the encoder's own epilogues: QKV -> packed planes, O-proj / FFN2 + residual (two-stream)
    "qkvp": (2304, 768, 4),
    "oproj_res": (768, 768, 2),
    "ffn2_res": (768, 3072, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64 * 512)
    ap.add_argument("--shapes", default="ffn1,ffn2,qkv,oproj")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--entry", default="ae_bench_gemm_packed")
    ap.add_argument("--lib", default=None, help="engine library to load (A/B of build flags)")
    args = ap.parse_args()

    from apmc_amd.engine import load_library
    lib = load_library(args.lib, tools=True)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    fn = getattr(lib, args.entry)
    fn.argtypes = [vp] * 6 + [i32] * 7 + [vp]
    fn.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    M = args.M
    g = torch.Generator(device=dev).manual_seed(0)

    def p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)

    variants = []
    for v in args.variants.split(","):
        np_ = 2
        if ":" in v:
            v, n = v.split(":")
            np_ = int(n)
        bn = 0
        if "@" in v:
            v, b = v.split("@")
            bn = int(b)
        variants.append((int(v), bn, np_))

    cases = []
    for name in args.shapes.split(","):
        N, K, epi = SHAPES[name]
        bufs = {}
        for np_ in sorted({v[2] for v in variants}):
            A = (torch.rand((M, np_ * K), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
            W = ((torch.rand((N, np_ * K), generator=g, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
            bufs[np_] = (A, W)
        bias = torch.zeros(N, device=dev)
        C = torch.empty((M, N), device=dev)
        Cp = torch.empty((M, 2 * N), dtype=torch.bfloat16, device=dev)
        R = None
        if epi == 2:
            R = torch.randn((M, N), generator=g, device=dev)
        for (diag, bn, np_) in variants:
            A, W = bufs[np_]
            call = (lambda A=A, W=W, bias=bias, C=C, Cp=Cp, N=N, K=K, epi=epi, np_=np_, bn=bn,
                    diag=diag, R=R: fn(p(A), p(W), p(bias), p(R), p(C), p(Cp), M, N, K, epi,
                                       np_, bn, diag, sp))
            rc = call()
            if rc != 0:
                print(json.dumps({"shape": name, "variant": [diag, bn, np_], "error": rc}))
                continue
            cases.append(dict(shape=name, diag=diag, bn=bn, np=np_, call=call, t=[],
                              flop=2.0 * M * N * K))
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c["call"]()
            e0.record(st)
            for _ in range(args.iters):
                c["call"]()
            e1.record(st)
            e1.synchronize()
            c["t"].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    for c in cases:
        med, mn = statistics.median(c["t"]), min(c["t"])
        print(json.dumps({"shape": c["shape"], "M": M, "diag": c["diag"], "bn": c["bn"],
                          "np": c["np"], "us_median": round(med, 2), "us_min": round(mn, 2),
                          "tflops_median": round(c["flop"] / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
