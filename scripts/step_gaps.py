"""Per-step kernel durations and inter-kernel gaps from a rocprofv3 kernel trace (diagnostic).

    python scripts/step_gaps.py <kernel_trace.csv> [steps=10] [marker=commit_kernel]

Steps end at each dispatch whose name contains the marker.  For the last `steps` steps:
mean step span, sum of kernel time, sum of gaps, and per kernel class (name up to '<' or '(')
the mean duration, mean gap before it and count per step."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
marker = sys.argv[3] if len(sys.argv) > 3 else "commit_kernel"
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
steps = [(ends[k - 1] + 1, ends[k]) for k in range(len(ends) - n_steps, len(ends))]
span = kern = gap = 0.0
cls = collections.defaultdict(lambda: [0.0, 0.0, 0])
for a, b in steps:
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["End_Timestamp"])
    span += (t1 - t0) / 1e3
    prev_end = int(rows[a - 1]["End_Timestamp"])
    for i in range(a, b + 1):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        name = rows[i]["Kernel_Name"]
        key = name.split("(")[0][:70]
        d, g = (e - s) / 1e3, (s - prev_end) / 1e3
        kern += d
        gap += g
        c = cls[key]
        c[0] += d
        c[1] += g
        c[2] += 1
        prev_end = e
k = len(steps)
print(f"{k} steps: span {span / k:.1f} us/step, kernels {kern / k:.1f} us, gaps {gap / k:.1f} us"
      f" (incl. the gap before each step's first kernel)")
for key, (d, g, c) in sorted(cls.items(), key=lambda kv: -kv[1][0]):
    print(f"{d / c:8.2f} us  gap-before {g / c:6.2f} us  x{c / k:5.1f}/step  {key}")
