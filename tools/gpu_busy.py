"""GPU busy fraction over time from a rocprofv3 kernel trace (GPU-side utilisation of an
end-to-end run such as the config-2 attack leg): the union of kernel intervals per --bucket
seconds, and over the whole window from --start-s (seconds after the first kernel).

  python tools/gpu_busy.py gpurun_out/<tag>/trace/run_kernel_trace.csv [--start-s S] [--bucket 5]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start-s", type=float, default=0.0)
    ap.add_argument("--bucket", type=float, default=5.0)
    args = ap.parse_args()
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(args.trace)))
    t0 = iv[0][0] + int(args.start_s * 1e9)
    iv = [(max(a, t0), b) for a, b in iv if b > t0]
    merged = []
    for a, b in iv:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    end = merged[-1][1]
    bk = int(args.bucket * 1e9)
    busy = [0] * ((end - t0) // bk + 1)
    for a, b in merged:
        while a < b:
            i = (a - t0) // bk
            e = min(b, t0 + (i + 1) * bk)
            busy[i] += e - a
            a = e
    for i, x in enumerate(busy):
        print(f"{args.start_s + i * args.bucket:8.1f} s  busy {x / bk:.3f}")
    tot = sum(b - a for a, b in merged)
    print(f"window {(end - t0) / 1e9:.2f} s  busy {tot / 1e9:.2f} s  frac {tot / (end - t0):.3f}")


if __name__ == "__main__":
    main()
