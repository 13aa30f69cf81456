"""Per-kernel summary of a rocprofv3 SQLite output (rocprofv3 --kernel-trace -d DIR -o run):
total / per-step time and calls per kernel name.  usage: db_summary.py <results.db> <steps> [top]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    steps = float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    q = ("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    agg, cnt = collections.defaultdict(float), collections.Counter()
    for n, t in db.execute(q):
        agg[n] += t
        cnt[n] += 1
    tot = sum(agg.values())
    print(f"total {tot / 1e6:.3f} ms  per step {tot / 1e6 / steps:.3f} ms")
    for n in sorted(agg, key=lambda k: -agg[k])[:top]:
        print(f"{agg[n] / 1e6 / steps:8.3f} ms/step {cnt[n] / steps:6.1f} calls  {n[:110]}")


if __name__ == "__main__":
    main()
