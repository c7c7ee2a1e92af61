"""Summarise a rocprofv3 kernel_stats.csv: python tools/prof_summary.py FILE [steps] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms over {steps:g} steps = {tot / 1e6 / steps:.3f} ms/step, {len(rows)} kernels")
for r in rows[:top]:
    n = r["Name"]
    n = n[:100]
    print(f'{float(r["TotalDurationNs"]) / 1e6 / steps:8.3f} ms/step {float(r["Percentage"]):5.1f}% '
          f'calls/step={int(r["Calls"]) / steps:7.1f} avg={float(r["AverageNs"]) / 1e3:7.2f}us  {n}')
