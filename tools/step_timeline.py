"""Per-step timeline of a rocprofv3 kernel trace (GPU): steps split at each embed_ln_kernel
launch; for each step the wall time to the next step, the union of kernel-busy time (the GPU
idle remainder is launch / dependency gaps), and per-kernel-class busy time summed over launches
(two-stream steps overlap, so the classes can sum past the wall).

  python tools/step_timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv [--grid-min N]
"""
import collections
import csv
import sys


def cls(name):
    for key, label in (("gemm_pp192_kernel<2, 2", "gemm192 +res (O-proj/FFN2)"),
                       ("gemm_pp192_kernel<2, 5", "gemm192 +res+LN"),
                       ("gemm_pp192_kernel<2, 8", "gemm192 +res+stats (layer 0)"),
                       ("gemm_pp192_kernel<2, 9", "gemm192 +LN(res)+stats (O-proj/FFN2)"),
                       ("gemm_pp_kernel<2, 1", "gemm256 GELU (FFN1)"),
                       ("gemm_pp_kernel<2, 6", "gemm256 fold GELU (FFN1)"),
                       ("gemm_pp_kernel<2, 7", "gemm256 fold packed (QKV)"),
                       ("gemm_pp_kernel<2, 4", "gemm256 packed (QKV)"),
                       ("gemm_pp192_kernel<2, 4", "gemm192 packed (QKV)"),
                       ("attn_pp_kernel", "attention"), ("layernorm_kernel", "layernorm"),
                       ("embed_ln", "embed+LN"), ("cls_", "CLS attention"),
                       ("gemm_x3", "last-layer CLS GEMMs"), ("splitk", "last-layer CLS GEMMs"),
                       ("gemm_f32_nt", "head"), ("gather_cls", "CLS gather")):
        if key in name:
            return label
    return name.split("(")[0][:40]


rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if "embed_ln_kernel" in r[2]]
out = []
for a, b in zip(starts, starts[1:]):
    seg = rows[a:b]
    t0, t1 = seg[0][0], rows[b][0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = collections.Counter()
    for s, e, n in seg:
        per[cls(n)] += e - s
    out.append(((t1 - t0) / 1e6, busy / 1e6, len(seg), per))
for wall, busy, n, per in out:
    top = ", ".join(f"{k} {v / 1e6:.2f}" for k, v in per.most_common(7))
    print(f"step {wall:7.3f} ms  busy {busy:7.3f}  idle {wall - busy:6.3f}  launches {n:4d} | {top}")
