"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (name prefix), the mean per
dispatch of every collected counter.  usage: pmc_summary.py <csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if keys and not any(s in k for s in keys):
            continue
        k = k[:70]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, cs in tot.items():
        n = max(1, len(disp[k]))
        print(f"{k}  dispatches={n}")
        for c in sorted(cs):
            print(f"  {c:28s} {cs[c] / n:16.0f}")


if __name__ == "__main__":
    main()
