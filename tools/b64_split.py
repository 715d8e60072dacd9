"""Per-graph split of a kernel trace into kernels and the gaps between them (last N graphs)."""
import collections
import csv
import glob
import sys

d, per, ngraphs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-per * ngraphs:]
dur = collections.defaultdict(list)
gaps = collections.defaultdict(list)
prev_end, prev_name = None, None
for r in last:
    n = r["Kernel_Name"]
    n = n[:n.find("(", 20)] if "(" in n[20:] else n
    n = n[-60:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[n].append((e - s) / 1e3)
    if prev_end is not None:
        gaps[(prev_name, n)].append((s - prev_end) / 1e3)
    prev_end, prev_name = e, n
for k, v in dur.items():
    print(f"{k:60s} n={len(v):4d} avg {sum(v) / len(v):6.2f} us")
for (a, b), v in gaps.items():
    print(f"gap {a[-28:]:28s} -> {b[-28:]:28s} avg {sum(v) / len(v):6.2f} us")
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
print(f"per graph: {span / ngraphs:.2f} us (trace span of the last {ngraphs} graphs / {ngraphs})")
