"""Summarise one rank's rocprofv3 --hip-trace of scripts/diag_postckpt.py: per HIP API function,
call count and total / max host time in the baseline window vs the window after DIAG_MODE's
ingredient (the windows are cut at the largest gap-free change of step rate: the script prints
its step timings; here the split is the first hipStreamCreate* call after the warm-up, or the
midpoint).  With a peer rank's trace directory as well, the kernel side: dispatches that ran far
longer than their kernel's median, and how much of each one the peer's kernels covered on the
same device (profiles/multiproc_slowdown_r6.md).
Usage: python scripts/diag_trace.py <rocprof dir> [<rank log>] [<peer rocprof dir>]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    rows = []
    for path in f:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                rows.append((r.get("Function") or r.get("Operation") or r.get("Kind"), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"]), r.get("Thread_Id", "")))
    rows.sort(key=lambda x: x[1])
    return rows


def main():
    rows = load(sys.argv[1])
    if not rows:
        print("no hip api trace found")
        return
    split = next((s for fn, s, e, t in rows if fn and fn.startswith("hipStreamCreate")), None)
    if split is None:
        split = rows[len(rows) // 2][1]
    t0, t1 = rows[0][1], rows[-1][2]
    print(f"trace {len(rows)} HIP calls over {(t1 - t0) / 1e9:.2f} s; split at +{(split - t0) / 1e9:.3f} s "
          f"({'first hipStreamCreate*' if any(r[0].startswith('hipStreamCreate') for r in rows) else 'midpoint'})")
    for name, sel in (("BEFORE", lambda s: s < split), ("AFTER", lambda s: s >= split)):
        agg = defaultdict(lambda: [0, 0, 0])
        span = [None, None]
        for fn, s, e, _t in rows:
            if not sel(s):
                continue
            a = agg[fn]
            a[0] += 1
            a[1] += e - s
            a[2] = max(a[2], e - s)
            span[0] = s if span[0] is None else min(span[0], s)
            span[1] = e if span[1] is None else max(span[1], e)
        wall = (span[1] - span[0]) / 1e9 if span[0] is not None else 0
        print(f"\n== {name} (window {wall:.2f} s): top HIP calls by total host time")
        print(f"{'function':40s} {'calls':>7s} {'total ms':>10s} {'max ms':>9s} {'mean us':>9s}")
        for fn, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
            print(f"{fn:40s} {n:7d} {tot / 1e6:10.1f} {mx / 1e6:9.2f} {tot / n / 1e3:9.1f}")
    if len(sys.argv) > 2 and os.path.exists(sys.argv[2]):
        print("\n== step timings (rank log)")
        for line in open(sys.argv[2]):
            if "ms/step" in line or "rc=" in line:
                print(line.rstrip())
    if len(sys.argv) > 3:
        kernel_side(kernels(sys.argv[1]), kernels(sys.argv[3]))


def kernels(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    out = []
    for path in f:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r["Queue_Id"]))
    return sorted(out)


def kernel_side(mine, peer, top=12):
    med = defaultdict(list)
    for s, e, n, _q in mine:
        med[n].append(e - s)
    med = {n: sorted(v)[len(v) // 2] for n, v in med.items()}
    slow = [k for k in mine if k[1] - k[0] > 50 * max(med[k[2]], 1000) and k[1] - k[0] > 5e6]
    print(f"\n== KERNELS: {len(slow)} of {len(mine)} dispatches ran > 50x their kernel's median (and > 5 ms); "
          f"{sum(k[1] - k[0] for k in slow) / 1e6:.0f} ms of dispatch time in all")
    print(f"{'ms':>8s} {'median us':>9s}  {'kernel':60s} peer-busy-share peer-queues")
    for s, e, n, q in sorted(slow, key=lambda k: k[0] - k[1])[:top]:
        ov = [k for k in peer if k[1] > s and k[0] < e]
        busy = sum(min(e, k[1]) - max(s, k[0]) for k in ov)
        print(f"{(e - s) / 1e6:8.1f} {med[n] / 1e3:9.1f}  {n:60s} {busy / (e - s):5.2f} {sorted(set(k[3] for k in ov))}")


if __name__ == "__main__":
    main()
