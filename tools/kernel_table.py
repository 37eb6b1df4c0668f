"""Per-(kernel, grid) average durations from a rocprofv3 kernel-trace CSV."""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[(r["Kernel_Name"][:70], int(r["Grid_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) / tot > 0.002:
        print(f"{sum(v)/tot*100:5.1f}%  n={len(v):4d} avg={sum(v)/len(v):9.1f}us grid={k[1]:8d} {k[0]}")
