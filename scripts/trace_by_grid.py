"""Per (kernel, grid) mean duration from a rocprofv3 kernel_trace.csv.

    python scripts/trace_by_grid.py FILE.csv [--kernel conv_gemm_tiled]"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="")
    args = ap.parse_args()
    acc = {}
    with open(args.csv) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            if args.kernel and args.kernel not in name:
                continue
            grid = "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            acc.setdefault((name[:90], grid), []).append(dur)
    for (name, grid), v in sorted(acc.items()):
        print(json.dumps({"kernel": name, "grid": grid, "n": len(v),
                          "median_us": statistics.median(v), "mean_us": statistics.mean(v)}))


if __name__ == "__main__":
    main()
