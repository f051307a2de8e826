"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: per-kernel
calls / average / share, plus per-token view for the decode forward."""
import csv
import os
import sys

d = sys.argv[1]  # a *_kernel_stats.csv, or a directory holding bench_kernel_stats.csv
rows = list(csv.DictReader(open(d if d.endswith(".csv") else os.path.join(d, "bench_kernel_stats.csv"))))
print(f"{'kernel':100s} {'calls':>7s} {'avg_us':>9s} {'min_us':>9s} {'%':>6s}")
for r in rows:
    print(f"{r['Name'][:100]:100s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} "
          f"{float(r['MinNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}")
print(f"total {sum(float(r['TotalDurationNs']) for r in rows) / 1e6:.3f} ms")
