"""Print a rocprofv3 kernel trace in dispatch order for the last N dispatches (diagnostic):
    python scripts/trace_order.py <kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
for r in rows[-n:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    g = f'{r.get("Grid_Size_X", r.get("Grid_Size", ""))}x{r.get("Grid_Size_Y", "")}x{r.get("Grid_Size_Z", "")}'
    print(f'{d:9.1f} us  wg={r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))} grid={g}  {r["Kernel_Name"][:80]}')
