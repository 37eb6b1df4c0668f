"""Average PMC counters per kernel (name substring, optional min grid size) from gpu_pmc.sh output.
Usage: python tools/pmc_table.py gpurun_out/pmc 'gemm_x3' [min_grid]"""
import collections
import csv
import pathlib
import sys

root = pathlib.Path(sys.argv[1])
pat = sys.argv[2]
min_grid = int(sys.argv[3]) if len(sys.argv) > 3 else 0
for run in sorted(p for p in root.iterdir() if p.is_dir() and p.name.startswith("pmc")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in run.glob("p*/**/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and int(r["Grid_Size"]) >= min_grid:
                name = r["Kernel_Name"].split("(")[0][:60]
                agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {run.name}")
    for name, cs in agg.items():
        print(f"  {name}")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
