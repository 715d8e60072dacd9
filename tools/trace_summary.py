"""Per-kernel durations of the last `tokens` decode tokens in a rocprofv3 kernel trace.
usage: python tools/trace_summary.py <trace dir> <kernels per token> <tokens>"""
import collections
import csv
import glob
import sys

d, per, ntok = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-per * ntok:]
agg = collections.defaultdict(list)
for r in last:
    n = r["Kernel_Name"]
    n = n[:n.find("(", 20)] if "(" in n[20:] else n
    agg[n[-64:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{k:64s} n={len(v):4d} avg {sum(v) / len(v):6.2f} us  per token {sum(v) / ntok:7.1f} us")
print(f"sum of kernel durations per token: {tot / ntok:.1f} us")
tok = last[-per:]
print(f"last token span: {(int(tok[-1]['End_Timestamp']) - int(tok[0]['Start_Timestamp'])) / 1e3:.1f} us")
