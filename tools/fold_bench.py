"""Cost of the folded-LayerNorm epilogues (GPU): each encoder GEMM at B = 64 x 512 rows (M = 32768;
--m for the two-stream half) in its folded form against its plain form, HIP events in interleaved
rounds in one process.  One JSON line per pair, median µs:
  qkv   ae_launch_gemm_packed_fold(gelu 0)  vs ae_launch_gemm_packed(PK_EPI_BIAS_PACKED)
  ffn1  ae_launch_gemm_packed_fold(gelu 1)  vs ae_launch_gemm_packed(PK_EPI_GELU_PACKED)
  oproj / ffn2  ae_launch_gemm_packed_res_stats (residual normalised on the fly) vs the plain
        +residual f32 epilogue (PK_EPI_RES)

  python tools/fold_bench.py [--m 32768] [--rounds 7] [--lib PATH]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--p2", action="store_true",
                    help="also the two-per-CU 128 x 192 kernel (tools library): the statistics "
                         "epilogues (ae_bench_gemm_packed_res_stats variants 1 / 2) and the folded "
                         "QKV / FFN1 (ae_bench_gemm_packed_fold variant 1)")
    ap.add_argument("--only", default=None, help="comma-separated launch names")
    args = ap.parse_args()
    from apmc_amd.engine import load_library
    lib = load_library(args.lib, tools=args.p2)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    lib.ae_launch_gemm_packed.argtypes = [vp] * 6 + [i32] * 5 + [vp]
    lib.ae_launch_gemm_packed_fold.argtypes = [vp] * 5 + [f32, vp] + [i32] * 5 + [vp, vp]
    lib.ae_launch_gemm_packed_res_stats.argtypes = [vp] * 7 + [f32] + [vp] * 3 + [i32] * 4 + \
        [vp, vp]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    M, H, F = args.m, 768, 3072

    def p(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)

    def planes(r, k):
        return (torch.randn(r, 2 * k, device=dev) * 0.05).to(torch.bfloat16)

    g = torch.Generator(device=dev).manual_seed(0)
    x = planes(M, H)
    h = planes(M, F)
    ctx = planes(M, H)
    w = {"qkv": planes(3 * H, H), "ffn1": planes(F, H), "oproj": planes(H, H), "ffn2": planes(H, F)}
    bias = torch.randn(F, device=dev, generator=g) * 0.1
    s = torch.randn(F, device=dev, generator=g)
    gam, bet = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    # the plane shift as the engine runs it: kappa for the producers, kc for the consumers
    kap = torch.randn(H, device=dev, generator=g) * 0.1
    kc = torch.randn(F, device=dev, generator=g) * 0.1
    v = torch.randn(M, H, device=dev, generator=g)
    rv = torch.randn(M, H, device=dev, generator=g)
    stats = torch.zeros(M * 4, 2, device=dev)
    stats[:, 1] = 192.0  # (mean 0, M2 192): unit variance rows
    stats = stats.view(torch.int64)
    ostats = torch.zeros(M * 4, dtype=torch.int64, device=dev)
    outp = torch.zeros(M, 2 * F, dtype=torch.bfloat16, device=dev)
    vp_ = torch.zeros(M, 2 * H, dtype=torch.bfloat16, device=dev)
    calls = {
        "qkv_plain": lambda: lib.ae_launch_gemm_packed(p(x), p(w["qkv"]), p(bias), None, None, p(outp), M, 3 * H, H, 4, 2, st),
        "qkv_fold": lambda: lib.ae_launch_gemm_packed_fold(p(x), p(w["qkv"]), p(bias), p(s), p(stats), 1e-5, p(outp), M, 3 * H, H, 0, 2, p(kc), st),
        "ffn1_plain": lambda: lib.ae_launch_gemm_packed(p(x), p(w["ffn1"]), p(bias), None, None, p(outp), M, F, H, 1, 2, st),
        "ffn1_fold": lambda: lib.ae_launch_gemm_packed_fold(p(x), p(w["ffn1"]), p(bias), p(s), p(stats), 1e-5, p(outp), M, F, H, 1, 2, p(kc), st),
        "oproj_plain": lambda: lib.ae_launch_gemm_packed(p(ctx), p(w["oproj"]), p(bias), p(rv), p(v), None, M, H, H, 2, 2, st),
        "oproj_stats": lambda: lib.ae_launch_gemm_packed_res_stats(p(ctx), p(w["oproj"]), p(bias), p(rv), p(stats), p(gam), p(bet), 1e-5, p(v), p(vp_), p(ostats), M, H, H, 2, p(kap), st),
        "ffn2_plain": lambda: lib.ae_launch_gemm_packed(p(h), p(w["ffn2"]), p(bias), p(rv), p(v), None, M, H, F, 2, 2, st),
        "ffn2_stats": lambda: lib.ae_launch_gemm_packed_res_stats(p(h), p(w["ffn2"]), p(bias), p(rv), p(stats), p(gam), p(bet), 1e-5, p(v), p(vp_), p(ostats), M, H, F, 2, p(kap), st),
    }
    if args.p2:
        lib.ae_bench_gemm_packed_res_stats.argtypes = [vp] * 7 + [f32] + [vp] * 3 + [i32] * 4 + \
            [vp, i32, i32, vp]
        for nm, a_, w_, K_ in (("oproj", ctx, w["oproj"], H), ("ffn2", h, w["ffn2"], F)):
            for var in (1, 2):
                for grp in (8, 4, 16):
                    calls[f"{nm}_stats_p2v{var}_g{grp}"] = (
                        lambda a_=a_, w_=w_, K_=K_, grp=grp, var=var:
                        lib.ae_bench_gemm_packed_res_stats(
                            p(a_), p(w_), p(bias), p(rv), p(stats), p(gam), p(bet), 1e-5, p(v),
                            p(vp_), p(ostats), M, H, K_, 2, p(kap), var, grp, st))
    if args.p2:
        lib.ae_bench_gemm_packed_fold.argtypes = [vp] * 5 + [f32, vp] + [i32] * 5 + [vp, i32, i32, vp]
        for nm, gl, N_ in (("qkv", 0, 3 * H), ("ffn1", 1, F)):
            for grp in (8, 4, 16):
                calls[f"{nm}_fold_p2_g{grp}"] = (
                    lambda gl=gl, N_=N_, grp=grp, nm=nm:
                    lib.ae_bench_gemm_packed_fold(p(x), p(w[nm]), p(bias), p(s), p(stats), 1e-5,
                                                  p(outp), M, N_, H, gl, 2, p(kc), 1, grp, st))
    if args.only:
        calls = {k: c for k, c in calls.items() if k in args.only.split(",")}
    ts = {k: [] for k in calls}
    for k, c in calls.items():
        assert c() == 0, k
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, c in calls.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c()
            e0.record()
            for _ in range(args.iters):
                c()
            e1.record()
            e1.synchronize()
            ts[k].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    for k in calls:
        print(json.dumps({"launch": k, "M": M, "us_median": round(statistics.median(ts[k]), 1),
                          "us_min": round(min(ts[k]), 1)}), flush=True)


if __name__ == "__main__":
    main()
