"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:100]:100s} n={r['Calls']:>7} avg={float(r['AverageNs'])/1e3:8.2f}us "
          f"tot={float(r['TotalDurationNs'])/1e6:8.2f}ms")
