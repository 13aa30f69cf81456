"""Idle gaps in a rocprofv3 kernel_trace.csv: GPU busy fraction over the trace's last
`--window` seconds and the largest gaps (with the kernel that ends the gap)."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("path")
ap.add_argument("--last-ms", type=float, default=150.0)
ap.add_argument("--top", type=int, default=15)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.path)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
end = max(e for _, e, _ in ev)
t0 = end - a.last_ms * 1e6
ev = [x for x in ev if x[0] >= t0]
busy, gaps, cur = 0, [], ev[0][0]
for s, e, n in ev:
    if s > cur:
        gaps.append((s - cur, n, s))
    busy += max(0, e - max(s, cur))
    cur = max(cur, e)
span = cur - ev[0][0]
print(f"window {span / 1e6:.2f} ms  kernels {len(ev)}  busy {busy / span * 100:.1f}%  idle {(span - busy) / 1e6:.3f} ms")
for g, n, s in sorted(gaps, reverse=True)[: a.top]:
    print(f"  gap {g / 1e3:8.1f} us before {n[:100]}  @{(s - ev[0][0]) / 1e6:.3f} ms")
