"""Per-dispatch kernel durations from a rocprofv3 kernel_trace.csv, grouped by kernel and grid
size (median / mean / count), so grouped and single launches of one kernel are told apart."""
import collections
import csv
import sys

import numpy as np

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    key = (name[:70], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]), int(r["Workgroup_Size_X"]))
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
print(f"{'kernel':70s} {'WGs':>7s} {'gy':>4s} {'thr':>5s} {'calls':>6s} {'median_us':>10s} {'mean_us':>9s}")
for k, v in sorted(d.items()):
    print(f"{k[0]:70s} {k[1]:7d} {k[2]:4d} {k[3]:5d} {len(v):6d} {np.median(v):10.2f} {np.mean(v):9.2f}")
