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
    args = ap.parse_args()
    by = {}
    with open(args.trace) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name") or r.get("Name")
            if args.kernel and args.kernel not in name:
                continue
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            by.setdefault(name, []).append((int(r["Start_Timestamp"]), t))
    for name, v in by.items():
        v.sort()
        d = [t for _, t in v]
        n = len(d)
        if n < args.bins:
            continue
        step = n // args.bins
        bins = [round(statistics.mean(d[i * step:(i + 1) * step]), 2) for i in range(args.bins)]
        print(f"{name[:60]:60s} n={n:7d} mean={statistics.mean(d):8.2f}us bins={bins}")


if __name__ == "__main__":
    main()
