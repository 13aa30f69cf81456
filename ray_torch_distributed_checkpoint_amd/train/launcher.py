"""Process-per-GPU launcher and supervisor (replaces Ray's WorkerGroup + metaflow-ray gang).

`launch(payload, n, ...)` starts `n` worker processes (one per GPU, `python -m
ray_torch_distributed_checkpoint_amd.train._worker`), hosts the TCPStore that is both the
torch.distributed rendezvous (RCCL unique-id exchange / gloo) and the control plane
(reports, heartbeats, errors), and supervises them:

* a worker exiting non-zero, publishing an error, or missing heartbeats for
  `heartbeat_timeout_s` fails the attempt; every surviving worker of the gang is killed
  (SIGKILL to its process group - a partially failed RCCL communicator cannot recover);
* a worker whose training-thread step counter (`train.report_progress`; every `report` also
  counts as progress) stops advancing for `progress_timeout_s` fails the attempt the same way: this catches a rank
  stuck inside a collective (a dead or hung peer), which the heartbeat thread keeps hiding
  until the 30-minute process-group timeout;
* up to `FailureConfig.max_failures` restarts, each resuming from the latest committed
  checkpoint of the same trial (Ray FailureConfig semantics);
* fault injection for tests: env `RTDC_FAIL_AT_REPORT=K[:rank]` makes a worker SIGKILL itself
  right after its K-th report (only on the first attempt).

Workers see the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
NODE_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT) with all GPUs visible; rank r drives
`cuda:LOCAL_RANK`.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field

import cloudpickle
from torch.distributed import TCPStore


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class AttemptOutcome:
    ok: bool
    reports: list = field(default_factory=list)
    error: str | None = None
    failed_rank: int | None = None


class WorkerGroup:
    def __init__(self, num_workers: int, use_gpu: bool, verbose: int = 1):
        self.n = num_workers
        self.use_gpu = use_gpu
        self.verbose = verbose
        self.port = free_port()
        self.store = TCPStore("127.0.0.1", self.port, is_master=True, wait_for_workers=False,
                              timeout=__import__("datetime").timedelta(seconds=3600))
        self.procs: list[subprocess.Popen] = []

    def start(self, payload_path: str, attempt: int, extra_env: dict | None = None):
        pg_port = free_port()
        self.procs = []
        for r in range(self.n):
            env = dict(os.environ)
            env.update({
                "RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(self.n), "LOCAL_WORLD_SIZE": str(self.n),
                "NODE_RANK": "0", "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(pg_port),
                "RTDC_STORE_PORT": str(self.port), "RTDC_ATTEMPT": str(attempt), "RTDC_PAYLOAD": payload_path,
            })
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            # one intra-op thread pool per worker must not oversubscribe the host (gloo ranks
            # busy-poll): split the CPUs between the ranks unless the user chose
            from ..utils.hostinfo import available_cpus

            env.setdefault("OMP_NUM_THREADS", str(max(1, available_cpus() // self.n)))
            # workers import the user's modules (cloudpickle pickles module functions by
            # reference) and this package exactly as the driver does
            pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            paths = [pkg_root, os.getcwd()] + [p for p in sys.path if p]
            if env.get("PYTHONPATH"):
                paths.append(env["PYTHONPATH"])
            env["PYTHONPATH"] = os.pathsep.join(dict.fromkeys(paths))
            if extra_env:
                env.update(extra_env)
            cmd = [sys.executable, "-u", "-m", "ray_torch_distributed_checkpoint_amd.train._worker"]
            self.procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))

    def kill_all(self):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        for p in self.procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pass

    def supervise(self, attempt: int, heartbeat_timeout_s: float, on_report=None,
                  progress_timeout_s: float | None = None) -> AttemptOutcome:
        out = AttemptOutcome(ok=False)
        seen = 0
        t_start = time.time()
        t_prog_check = 0.0
        self._progress = {}  # rank -> (step, host time the step last changed)
        try:
            while True:
                n = self.store.add(f"a{attempt}/nreports", 0)
                while seen < n:
                    seen += 1
                    msg = json.loads(self.store.get(f"a{attempt}/report/{seen}").decode())
                    out.reports.append(msg)
                    if on_report:
                        on_report(msg)
                codes = [p.poll() for p in self.procs]
                nerr = self.store.add(f"a{attempt}/nerrors", 0)
                if nerr > 0 or any(c not in (None, 0) for c in codes):
                    out.error, out.failed_rank = self._collect_error(attempt, codes)
                    self.kill_all()
                    return out
                if all(c == 0 for c in codes):
                    # drain reports published right before exit
                    n = self.store.add(f"a{attempt}/nreports", 0)
                    while seen < n:
                        seen += 1
                        msg = json.loads(self.store.get(f"a{attempt}/report/{seen}").decode())
                        out.reports.append(msg)
                        if on_report:
                            on_report(msg)
                    out.ok = True
                    return out
                now = time.time()
                if progress_timeout_s and now - t_prog_check >= min(1.0, progress_timeout_s / 4):
                    t_prog_check = now
                    stalled = self._stalled_rank(attempt, progress_timeout_s, now)
                    if stalled is not None:
                        r, step = stalled
                        out.error = (f"worker rank {r} made no training progress for {progress_timeout_s}s "
                                     f"(stuck at step {step}: hung collective or kernel?)")
                        out.failed_rank = r
                        self.kill_all()
                        return out
                if heartbeat_timeout_s and time.time() - t_start > heartbeat_timeout_s:
                    stale = self._stale_rank(attempt, heartbeat_timeout_s)
                    if stale is not None:
                        out.error = f"worker rank {stale} missed heartbeats for {heartbeat_timeout_s}s (hang?)"
                        out.failed_rank = stale
                        self.kill_all()
                        return out
                time.sleep(0.05)
        except BaseException:
            self.kill_all()
            raise

    def _stalled_rank(self, attempt, timeout, now):
        """First rank whose published step counter has not changed for `timeout` seconds
        (ranks that never published, or finished, are not watched)."""
        for r in range(self.n):
            key = f"a{attempt}/prog/{r}"
            try:
                if not self.store.check([key]):
                    continue
                v = self.store.get(key).decode()
            except Exception:
                continue
            if v == "done":
                self._progress.pop(r, None)
                continue
            parts = v.split()
            step = int(parts[0])
            token = (step, parts[2] if len(parts) > 2 else "")  # step or report sequence advanced
            prev = self._progress.get(r)
            if prev is None or prev[0] != token:
                self._progress[r] = (token, now)
            elif now - prev[1] > timeout:
                return r, step
        return None

    def _stale_rank(self, attempt, timeout):
        now = time.time()
        for r in range(self.n):
            try:
                if not self.store.check([f"a{attempt}/hb/{r}"]):
                    continue
                t = float(self.store.get(f"a{attempt}/hb/{r}").decode())
                if now - t > timeout:
                    return r
            except Exception:
                continue
        return None

    def _collect_error(self, attempt, codes):
        for r in range(self.n):
            key = f"a{attempt}/error/{r}"
            if self.store.check([key]):
                return self.store.get(key).decode(), r
        for r, c in enumerate(codes):
            if c not in (None, 0):
                sig = f" (signal {-c})" if c < 0 else ""
                return f"worker rank {r} exited with code {c}{sig}", r
        return "unknown worker failure", None


def write_payload(obj) -> str:
    d = tempfile.mkdtemp(prefix="rtdc_payload_")
    p = os.path.join(d, "payload.pkl")
    with open(p, "wb") as f:
        cloudpickle.dump(obj, f)
    return p
