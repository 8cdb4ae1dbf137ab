"""Summarise a rocprofv3 kernel_trace.csv: per-kernel duration vs dispatch order.

    python scripts/trace_summary.py TRACE.csv [--kernel attn_kernel] [--bins 10]

Prints, for each kernel whose name contains --kernel, the mean duration (µs) in --bins
equal slices of its dispatch sequence (for decode steps: slices of the position range)."""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--bins", type=int, default=10)
    ap.add_argument("--by-grid", action="store_true", help="split each kernel by grid size")
    ap.add_argument("--gaps", action="store_true",
                    help="also print the mean idle gap before each kernel (same queue)")
    args = ap.parse_args()
    by = {}
    with open(args.trace) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name") or r.get("Name")
            if args.by_grid:
                grid = [r.get(k) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size")
                        if r.get(k)]
                name = f"{name[:70]} grid={'x'.join(grid)}"
            if args.kernel and args.kernel not in name:
                continue
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            by.setdefault(name, []).append((int(r["Start_Timestamp"]), t))
    if args.gaps:
        rows = []
        with open(args.trace) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name") or r.get("Name")
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
        rows.sort()
        gaps = {}
        for (s0, e0, _), (s1, e1, n1) in zip(rows, rows[1:]):
            g = (s1 - e0) / 1e3
            if 0 <= g < 50:  # same burst (graph replay), not host idle time
                gaps.setdefault(n1[:60], []).append(g)
        for n, v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
            print(f"gap before {n:60s} n={len(v):7d} mean={statistics.mean(v):6.2f}us")
    for name, v in by.items():
        v.sort()
        d = [t for _, t in v]
        n = len(d)
        if n < args.bins:
            continue
        step = n // args.bins
        bins = [round(statistics.mean(d[i * step:(i + 1) * step]), 2) for i in range(args.bins)]
        print(f"{name[:110]:110s} n={n:7d} mean={statistics.mean(d):8.2f}us bins={bins}")


if __name__ == "__main__":
    main()
