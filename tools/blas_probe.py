"""Library-GEMM probe (GPU): how fast the vendor bf16 GEMM (torch.mm -> hipBLASLt / rocBLAS) runs
the encoder's f32x3 GEMMs written as ONE bf16 GEMM over a tripled K:
    [a_hi | a_hi | a_lo] · [w_hi | w_lo | w_hi]^T  (K' = 3K, f32 accumulate)
— the same three split products as gemm_planes.hip, without its fused epilogues (bias, GELU,
plane split, residual).  One JSON line per shape: median µs and bf16 TFLOP/s over K'.

  python tools/blas_probe.py [--m 32768] [--rounds 7]
"""
import argparse
import json
import statistics

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    shapes = {"qkv": (2304, 768), "oproj": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}
    for name, (n, k) in shapes.items():
        a = torch.randn(args.m, 3 * k, device=dev).to(torch.bfloat16)
        w = torch.randn(n, 3 * k, device=dev).to(torch.bfloat16)
        out = {}
        for dt in ("bf16", "f32"):
            ts = []
            for _ in range(args.rounds):
                if dt == "bf16":
                    f = lambda: torch.mm(a, w.t())  # noqa: E731
                else:  # f32 output of the same bf16 product (hipBLASLt out_dtype)
                    f = lambda: torch.mm(a, w.t(), out_dtype=torch.float32)  # noqa: E731
                try:
                    f()
                except (TypeError, RuntimeError) as exc:
                    ts = None
                    out[dt] = str(exc)[:80]
                    break
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / args.iters)
            if ts:
                med = statistics.median(ts)
                out[dt] = {"us": round(med, 1),
                           "bf16_tflops": round(2.0 * args.m * n * 3 * k / med / 1e6, 1)}
        print(json.dumps({"shape": name, "M": args.m, "N": n, "K_tripled": 3 * k, **out}), flush=True)


if __name__ == "__main__":
    main()
