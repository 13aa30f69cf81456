"""Summarise a rocprofv3 kernel_stats.csv: per-step ms per kernel (top N)."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms  per step {tot / 1e6 / steps:.3f} ms")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:6.1f} calls  {r['Name'][:120]}")
