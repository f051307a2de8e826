"""Top kernels of a rocprofv3 --kernel-trace --stats output directory (searched
recursively for *kernel_stats.csv): calls, average and total time.
usage: python tools/kstats.py DIR [N]"""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
print(f"# {f}")
for r in list(csv.DictReader(open(f)))[:n]:
    print(f"{r['Name'][:96]:96s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.1f} us "
          f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms")
