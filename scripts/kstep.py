"""One training step's kernels in launch order from a rocprofv3 kernel_trace.csv: the span
between the last two launches of the optimizer kernel (`--marker`), with each kernel's
duration, grid and workgroup size, so a product can be matched to its call site."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--marker", default="adamw_kernel")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
lo, hi = idx[-2] + 1, idx[-1] + 1
tot = 0.0
for r in rows[lo:hi]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    wg = r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?"))
    print(f"{d:9.1f} us  grid {grid:>9} wg {wg:>4}  {r['Kernel_Name'][:110]}")
span = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
print(f"kernels {hi - lo}  sum {tot:.1f} us  span {span:.1f} us")
