"""Summarise a rocprofv3 --pmc counter_collection.csv: per (kernel, grid) mean counter value.

    python scripts/pmc_summary.py FILE.csv [--kernel gemv1]

FETCH_SIZE / WRITE_SIZE are in KB; the gfx950 correction (MI355X_MICROARCH.md §HBM: FETCH_SIZE
reads exactly half the bytes of a wide coalesced 16-B-per-lane stream) is applied in the
"hbm_read_bytes" column = FETCH_SIZE * 1024 * 2."""
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
            name = r.get("Kernel_Name") or r.get("Name") or ""
            if args.kernel and args.kernel not in name:
                continue
            grid = r.get("Grid_Size") or "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            key = (name[:90], grid, r.get("Counter_Name"))
            acc.setdefault(key, []).append(float(r.get("Counter_Value", "nan")))
    out = []
    for (name, grid, ctr), v in sorted(acc.items()):
        row = {"kernel": name, "grid": grid, "counter": ctr, "n": len(v),
               "mean": statistics.mean(v), "median": statistics.median(v)}
        if ctr == "FETCH_SIZE":
            row["hbm_read_bytes"] = statistics.median(v) * 1024 * 2
        if ctr == "WRITE_SIZE":
            row["hbm_write_bytes"] = statistics.median(v) * 1024
        out.append(row)
        print(json.dumps(row))


if __name__ == "__main__":
    main()
