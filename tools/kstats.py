"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, share)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:n]:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>6} avg={float(r['AverageNs']) / 1e3:8.2f}us min={float(r['MinNs']) / 1e3:7.2f} share={float(r['TotalDurationNs']) / tot * 100:5.1f}%")
print(f"total {tot / 1e6:.3f} ms")
