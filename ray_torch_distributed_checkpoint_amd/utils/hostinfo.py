"""Host CPU budget as this process can actually use it.

`os.cpu_count()` reports every CPU of the machine, also inside a container or a job slot
limited by a cgroup CPU quota or an affinity mask (on the GPU boxes it reports many times the
16 CPUs a job may use).  Thread pools sized from it (checkpoint writers, per-rank intra-op
threads) then oversubscribe the host: the async-save writers of 2 ranks starved their training
threads."""
from __future__ import annotations

import os


def _cgroup_quota_cpus() -> float | None:
    try:  # cgroup v2
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:  # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = float(f.read())
        if q > 0 and p > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def available_cpus() -> int:
    """min(machine CPUs, affinity mask, cgroup quota), at least 1."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    q = _cgroup_quota_cpus()
    if q is not None:
        n = min(n, max(1, int(q)))
    return max(1, n)
