"""Per-kernel SQ counter summary from scripts/gpu.sh `pmc` passes (one rocprofv3 --pmc run per
counter group, each with its kernel trace): the counters averaged per dispatch of each (kernel,
grid), the dispatch duration from the same pass's trace, and the ratios that say what bounds a
kernel (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles, 32 per 32x32x16 bf16 MFMA,
summed over the SIMDs; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave;
GRBM_GUI_ACTIVE is summed over the 8 XCDs).

  python tools/pmc_sq.py gpurun_out/<tag> [kernel substring ...] > profiles/<round>_pmc_sq.json
"""
import collections
import csv
import json
import pathlib
import statistics
import sys

SIMDS = 1024  # 256 CUs x 4

root = pathlib.Path(sys.argv[1])
# FFN1 / QKV (folded LayerNorm), O-projection / FFN2 (+ residual + statistics), attention
pats = sys.argv[2:] or ["gemm_pp_kernel<2, 6", "gemm_pp_kernel<2, 7", "gemm_pp192_kernel<2, 9",
                        "attn_pp_kernel<2, false, true"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for run in sorted(root.glob("pmc_p*")):
    f = run / "run_counter_collection.csv"
    if not f.exists():
        continue
    per_dispatch = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        if not any(p in key[0] for p in pats):
            continue
        per_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = key
    for d, cs in per_dispatch.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
    t = run / "run_kernel_trace.csv"
    if t.exists():
        for r in csv.DictReader(open(t)):
            key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1)
                   * int(r.get("Grid_Size_Z", 1) or 1))
            if any(p in key[0] for p in pats):
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

out = []
for (name, grid), cs in sorted(agg.items(), key=lambda kv: -len(kv[1])):
    m = {c: statistics.mean(v) for c, v in cs.items()}
    rec = {"kernel": name, "grid": grid, "dispatches": max(len(v) for v in cs.values()),
           "counters_mean": {c: round(v, 1) for c, v in sorted(m.items())}}
    us = statistics.mean(dur[(name, grid)]) if dur.get((name, grid)) else None
    rec["avg_duration_us_profiled"] = round(us, 2) if us else None
    g = m.get("GRBM_GUI_ACTIVE")
    if g and us:
        rec["clock_ghz"] = round(g / 8 / (us * 1e3), 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and g:
        rec["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * SIMDS), 4)
    if "SQ_INSTS_MFMA" in m and "SQ_INSTS_VALU" in m:
        rec["valu_insts_per_mfma"] = round((m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]) / m["SQ_INSTS_MFMA"], 2)
    wc = m.get("SQ_WAVE_CYCLES")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
        if c in m and wc:
            rec[c.lower().replace("sq_", "") + "_per_wave_cycle"] = round(m[c] / wc, 4)
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        rec["coexec_over_mfma_busy"] = round(m["SQ_VALU_MFMA_COEXEC_CYCLES"] / m["SQ_VALU_MFMA_BUSY_CYCLES"], 4)
    if "SQ_LDS_BANK_CONFLICT" in m and "SQ_ACTIVE_INST_LDS" in m and m["SQ_ACTIVE_INST_LDS"]:
        rec["lds_bank_conflict_over_active_lds"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_ACTIVE_INST_LDS"], 4)
    out.append(rec)
print(json.dumps(out, indent=1))
