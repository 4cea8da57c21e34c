"""Summarise a rocprofv3 kernel_stats.csv (per-step ms assuming `steps` timed+warmup steps)."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 13
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total GPU busy per step: {tot / 1e6 / steps:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r['Name'].replace('(anonymous namespace)::', '')[:90]
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step={int(r['Calls']) / steps:6.1f} avg={float(r['AverageNs']) / 1e3:8.2f}us  {name}")
