"""Microbenchmark + parity check of the split-bf16 fused attention kernels (GPU).

Random qkv [T, 2304] (f32, the QKV GEMM's output layout) over n sequences of length L (ragged
with --ragged), every variant of ae_bench_attention_x3 timed with HIP events in interleaved rounds
in one process, and checked against a float64 torch reference of the same attention (softmax of
Q·K^T/8 over each sequence's keys, times V).  One JSON line per variant: median / min µs per
launch, the algorithmic TFLOP/s (4·len²·64 per (sequence, head)) and max |out - ref|.

  python tools/attn_bench.py [--n 64] [--L 512] [--variants 0,1] [--terms 3] [--ragged] [--mask]

--mask adds a random bit-packed key mask (the GraphCodeBERT launch; ~60 % of the keys kept, key 0
always) to the pp variants and the reference.
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

H, HEADS, D = 768, 12, 64


def reference(qkv, cu, n, dense=None):
    outs = []
    for s in range(n):
        a, b = int(cu[s]), int(cu[s + 1])
        x = qkv[a:b].double()
        q = x[:, :H].view(-1, HEADS, D).transpose(0, 1)
        k = x[:, H:2 * H].view(-1, HEADS, D).transpose(0, 1)
        v = x[:, 2 * H:].view(-1, HEADS, D).transpose(0, 1)
        sc = q @ k.transpose(1, 2) / 8.0
        if dense is not None:  # HF's additive finfo(f32).min where the mask excludes a key
            sc = sc + (~dense[s, : b - a, : b - a]).to(sc.device).double() * torch.finfo(torch.float32).min
        p = torch.softmax(sc, dim=-1)
        outs.append((p @ v).transpose(0, 1).reshape(b - a, H))
    return torch.cat(outs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--terms", type=int, default=3)
    ap.add_argument("--ragged", action="store_true")
    ap.add_argument("--mask", action="store_true")
    ap.add_argument("--mask-gcb", action="store_true",
                    help="with --mask: GraphCodeBERT's mask structure (utils.py:547-570) instead "
                         "of random bits — the last 128 positions data-flow nodes over 1-3 code "
                         "tokens and 1-2 edges each, code rows attending all code rows")
    ap.add_argument("--mask-density", type=float, default=0.6,
                    help="fraction of keys each query keeps under --mask (1.0: the mask path "
                         "with nothing excluded)")
    ap.add_argument("--planes", action="store_true",
                    help="packed-plane context output (the engine's launch) instead of f32")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check-seqs", type=int, default=8)
    ap.add_argument("--lib", default=None, help="engine library to load (A/B of kernel sources)")
    args = ap.parse_args()

    from apmc_amd.engine import load_library
    lib = load_library(args.lib, tools=True)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    fn = lib.ae_bench_attention_x3
    fn.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    fn.restype = ctypes.c_int
    fpp = lib.ae_bench_attention_pp  # variants "pp" / "pp1": packed-plane input, LDS-DMA
    fpp.argtypes = [vp] * 5 + [i32] * 3 + [vp, i32, i32, i32, vp]
    fpp.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    g = torch.Generator().manual_seed(0)
    n, L = args.n, args.L
    if args.ragged:
        lens = torch.randint(L // 4, L + 1, (n,), generator=g)
    else:
        lens = torch.full((n,), L)
    cu = torch.zeros(n + 1, dtype=torch.int32)
    cu[1:] = torch.cumsum(lens, 0)
    T = int(cu[-1])
    qkv = (torch.randn((T, 3 * H), generator=g) * 1.5).to(dev)
    cu_d = cu.to(dev)
    flop = float(sum(4.0 * int(x) ** 2 * D * HEADS for x in lens))
    cs = min(args.check_seqs, n)
    dense, dmask = None, None
    if args.mask:
        if args.mask_gcb:
            nodes = min(128, L // 5)
            ncode = L - nodes
            dense = torch.zeros(n, L, L, dtype=torch.bool)
            dense[:, :ncode, :ncode] = True
            dense[:, 0, :] = True
            dense[:, ncode - 1, :] = True
            for s_ in range(n):
                for i in range(nodes):
                    a = int(torch.randint(1, ncode - 3, (1,), generator=g))
                    b = a + int(torch.randint(1, 4, (1,), generator=g))
                    dense[s_, ncode + i, a:b] = True
                    dense[s_, a:b, ncode + i] = True
                    for _ in range(int(torch.randint(1, 3, (1,), generator=g))):
                        dense[s_, ncode + i, ncode + int(torch.randint(0, nodes, (1,), generator=g))] = True
        else:
            dense = torch.rand(n, L, L, generator=g) < args.mask_density
            dense[:, :, 0] = True
        words = (dense.view(n, L, L // 32, 32).long() << torch.arange(32)).sum(-1)
        dmask = (words - (words >= 2 ** 31).long() * 2 ** 32).to(torch.int32).to(dev)
    ref = reference(qkv[:int(cu[cs])], cu, cs, dense)

    def p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)

    np_ = 2 if args.terms == 3 else 1
    x = qkv.clone()
    x[:, :H] *= 0.18033688011112042
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    planes = hi if np_ == 1 else torch.stack(
        [hi.view(T, -1, 32), lo.view(T, -1, 32)], 2).reshape(T, 2 * 3 * H).contiguous()
    cases = []
    for v in args.variants.split(","):
        var = v if v.startswith("pp") else int(v)
        out = torch.zeros((T, H), device=dev)
        opl = None
        if isinstance(var, str):
            pv = int(var[2:]) if len(var) > 2 else 0
            if args.planes:
                opl = torch.zeros((T, np_ * H), dtype=torch.int16, device=dev)
            call = (lambda out=out, pv=pv, opl=opl: fpp(p(planes), p(out), p(opl), p(cu_d), p(None),
                                                        int(lens.max()), n, HEADS, p(dmask),
                                                        L if args.mask else 0, np_, pv, sp))
        else:
            call = (lambda out=out, var=var: fn(p(qkv), p(out), p(None), p(cu_d), p(None),
                                                int(lens.max()), n, HEADS, p(None), 0, args.terms,
                                                var, sp))
        rc = call()
        torch.cuda.synchronize()
        if rc != 0:
            print(json.dumps({"variant": var, "error": rc}))
            continue
        if opl is not None:  # packed planes -> f32: per 32 columns [hi 32 | lo 32] (np 2)
            pl_ = opl.view(torch.bfloat16).float().view(T, H // 32, np_, 32)
            out = pl_.sum(2).reshape(T, H)
        err = float((out[:int(cu[cs])].double() - ref).abs().max())
        cases.append(dict(variant=var, call=call, t=[], err=err))
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
        print(json.dumps({"variant": c["variant"], "n": n, "L": L, "ragged": args.ragged,
                          "terms": args.terms, "planes": args.planes, "mask": args.mask, "us_median": round(med, 2), "us_min": round(mn, 2),
                          "tflops_median": round(flop / med / 1e6, 1),
                          "max_abs_err_vs_f64": c["err"]}), flush=True)


if __name__ == "__main__":
    main()
