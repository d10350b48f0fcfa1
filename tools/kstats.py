"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total / calls / average."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 18
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['Percentage']):5.1f}% n={r['Calls']:>5} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
print(f"total {tot/1e6:.2f} ms")
