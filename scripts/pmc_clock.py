"""Per-kernel effective clock and issue profile from a rocprofv3 --pmc --kernel-trace run.

clock_GHz = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the counter over the 8 XCDs) / kernel wall
time (MI355X_MICROARCH.md 'DVFS give-back'; reads high below ~0.3 ms per dispatch).  Also the
MFMA-pipe share of SIMD-cycles, LDS instructions and LDS issue stalls per MFMA, and the share
of wave-cycles parked in s_waitcnt / s_barrier (SQ_WAIT_ANY).  Medians over the dispatches of
each (kernel, grid) pair.

    python scripts/pmc_clock.py <out_dir>     (the directory rocprofv3 -d wrote)
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    times = {}
    for path in kt:
        for r in csv.DictReader(open(path)):
            times[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(dict)
    meta = {}
    for path in cc:
        for r in csv.DictReader(open(path)):
            k = r["Dispatch_Id"]
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[k] = (r["Kernel_Name"], r.get("Grid_Size", ""))
            if k not in times and r.get("Start_Timestamp"):
                times[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    groups = defaultdict(list)
    for k, cs in per.items():
        if k in times and times[k] > 0:
            groups[meta[k]].append((times[k], cs))
    print(f"{'kernel':70s} {'grid':>9s} {'n':>4s} {'us':>8s} {'GHz':>5s} {'mfma%':>6s} {'lds/mfma':>8s} {'ldsstall/mfma':>13s} {'wait%':>6s}")
    for (name, grid), lst in sorted(groups.items(), key=lambda kv: -sum(t for t, _ in kv[1])):
        if len(lst) < 2:
            continue
        us = statistics.median(t for t, _ in lst) * 1e6
        ghz = statistics.median(cs.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 for t, cs in lst)
        mf = statistics.median(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, cs.get("GRBM_GUI_ACTIVE", 1) / 8 * 4 * 256)
                               for t, cs in lst)
        nm = statistics.median(max(1.0, cs.get("SQ_INSTS_MFMA", 1)) for _, cs in lst)
        lds = statistics.median(cs.get("SQ_INSTS_LDS", 0) for _, cs in lst) / nm
        ldsw = statistics.median(cs.get("SQ_WAIT_INST_LDS", 0) for _, cs in lst) / nm
        wait = statistics.median(cs.get("SQ_WAIT_ANY", 0) / max(1, cs.get("SQ_WAVE_CYCLES", 1)) for _, cs in lst)
        nm_ = name.replace("void ", "").replace("rtdc::", "").split("(")[0][:70]
        print(f"{nm_:70s} {grid:>9s} {len(lst):4d} {us:8.1f} {ghz:5.2f} {100 * mf:6.1f} {lds:8.3f} {ldsw:13.2f} {100 * wait:6.1f}")


if __name__ == "__main__":
    main()
