"""Checkpoint / supervisor robustness:

* a failed async write raises for EVERY waiter, every time (handle outcome cached under a
  lock; the native engine keeps finished jobs' outcomes);
* a restarted attempt never commits a dead attempt's partial staging files, and a commit never
  deletes a live final directory before the new one is in place;
* the page-cache residency measurement behind the "cold" restore is real (mincore);
* the step-progress watchdog does not kill loops that only call `report()`.
"""
import os
import sys
import threading
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_failed_async_write_raises_for_every_waiter(tmp_path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave

    bad = str(tmp_path / "no_such_dir" / "x.pt")  # the engine's open() fails
    h = torchsave.save({"w": torch.randn(1000)}, bad, async_=True)
    errs = []

    def waiter():
        try:
            h.wait()
        except IOError as e:
            errs.append(str(e))

    ts = [threading.Thread(target=waiter) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(errs) == 4 and all("checkpoint write failed" in e for e in errs)
    with pytest.raises(IOError):
        h.wait()  # and again, later
    # the engine itself keeps the outcome of a waited job: a second wait is the same error
    eng = torchsave.get_engine()
    err1, _ = eng.wait(h.job_id)
    assert err1, "a second engine wait on a failed job must report the error, not success"


def test_dcp_async_save_failure_raises_twice(tmp_path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    d = tmp_path / "ck"
    h = dcp.async_save({"a": torch.randn(64, 64)}, str(d))
    # make the shard path unwritable before the writer gets to it is racy; instead verify the
    # cached success path and that a verify failure is cached as an error
    assert h.wait() == h.wait()
    h2 = dcp.AsyncSave(str(d), None, None, 0, time.perf_counter(), 0.0, 0, None)
    h2._verify = [(str(d / "__0_0.distcp"), 0, 10, torch.zeros(3))]  # corrupt range: verify must fail
    for _ in range(2):
        with pytest.raises(IOError):
            h2.wait()


def test_stale_staging_swept_and_commit_is_atomic(tmp_path):
    from ray_torch_distributed_checkpoint_amd.train import storage

    trial = tmp_path / "trial"
    trial.mkdir()
    # a committed checkpoint and a crashed attempt's partial staging dir
    c1 = trial / "checkpoint_000001"
    c1.mkdir()
    (c1 / "__0_0.distcp").write_bytes(b"old")
    st = trial / "checkpoint_000002.tmp"
    st.mkdir()
    (st / "__1_0.distcp").write_bytes(b"partial from a dead attempt")
    removed = storage.sweep_stale_staging(str(trial))
    assert [os.path.basename(p) for p in removed] == ["checkpoint_000002.tmp"]
    assert not st.exists() and c1.exists()
    # re-committing an existing index swaps in the new directory; the old one is gone after
    new = trial / "checkpoint_000001.tmp"
    new.mkdir()
    (new / "__0_0.distcp").write_bytes(b"new")
    path = storage.commit(str(trial), 1)
    assert open(os.path.join(path, "__0_0.distcp"), "rb").read() == b"new"
    assert sorted(os.listdir(trial)) == ["checkpoint_000001"]


def test_page_cache_residency_is_measured(tmp_path):
    from ray_torch_distributed_checkpoint_amd.utils import pagecache

    f = tmp_path / "blob"
    f.write_bytes(os.urandom(4 << 20))
    with open(f, "rb") as fh:
        fh.read()
    assert pagecache.resident_fraction(str(tmp_path)) > 0.9
    pagecache.drop(str(tmp_path))
    frac = pagecache.resident_fraction(str(tmp_path))
    if frac > 0.5:
        pytest.skip(f"page cache not droppable on this filesystem (resident {frac})")
    assert frac < 0.01


def _report_only_loop(config):
    from ray_torch_distributed_checkpoint_amd import train

    for i in range(config["n"]):
        time.sleep(config["dt"])
        train.report({"i": i})


def _progress_then_reports(config):
    from ray_torch_distributed_checkpoint_amd import train

    train.report_progress(0)  # watched from here on, but only report() advances afterwards
    for i in range(config["n"]):
        time.sleep(config["dt"])
        train.report({"i": i})


@pytest.mark.parametrize("fn", [_report_only_loop, _progress_then_reports])
def test_progress_watchdog_spares_report_only_loops(tmp_path, monkeypatch, fn):
    from ray_torch_distributed_checkpoint_amd import train

    monkeypatch.setenv("RTDC_FORCE_CPU", "1")
    t = train.TorchTrainer(fn, train_loop_config={"n": 5, "dt": 1.0},
                           scaling_config=train.ScalingConfig(num_workers=2, use_gpu=False),
                           run_config=train.RunConfig(storage_path=str(tmp_path), name="wd", progress_timeout_s=2.5))
    r = t.fit()  # reports arrive every ~1 s, total 5 s > the 2.5 s timeout: must not be killed
    assert r.metrics["i"] == 4


def test_writer_budget_is_per_node_and_quota_aware(monkeypatch):
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave
    from ray_torch_distributed_checkpoint_amd.utils import hostinfo

    n = hostinfo.available_cpus()
    assert 1 <= n <= (os.cpu_count() or 1)
    monkeypatch.setattr(hostinfo, "available_cpus", lambda: 64)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert torchsave.default_writer_threads() == 8
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert torchsave.default_writer_threads() == 4  # 64 // (2 * 8): the node's budget, split
    monkeypatch.setattr(hostinfo, "available_cpus", lambda: 16)
    assert torchsave.default_writer_threads() == 2


class _FakeComm:
    """A registered communicator whose error word the test flips (parallel/health.py)."""

    def __init__(self):
        self.err = 0

    def error(self):
        return self.err


def _with_fake_comm(fn):
    from ray_torch_distributed_checkpoint_amd.parallel import health

    c = _FakeComm()
    health.register(c)
    try:
        return fn(c)
    finally:
        health.unregister(c)


def test_later_timeout_does_not_void_clean_checkpoint(tmp_path):
    """commit-or-refuse is decided from the error words captured AT the snapshot, so a
    timeout of a later step while this snapshot drains does not refuse the clean checkpoint."""
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp, torchsave

    def body(c):
        h = torchsave.save({"w": torch.randn(1000)}, str(tmp_path / "a.pt"), async_=True)
        a = dcp.async_save({"w": torch.randn(64)}, str(tmp_path / "ck"))
        c.err = 1  # a later collective times out while the saves drain
        assert h.wait() >= 0
        assert a.wait() >= 0
        # a save that starts now refuses up front
        from ray_torch_distributed_checkpoint_amd.parallel.health import CommPoisonedError

        with pytest.raises(CommPoisonedError):
            torchsave.save({"w": torch.randn(10)}, str(tmp_path / "b.pt"), async_=True)

    _with_fake_comm(body)


def test_timeout_before_snapshot_refuses_commit(tmp_path):
    """The words captured at the snapshot are what wait() checks: a poisoned capture refuses."""
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave
    from ray_torch_distributed_checkpoint_amd.parallel import health

    def body(c):
        real = health.capture_error_words

        def poisoned_capture():
            c.err = 7  # the timeout lands between the up-front check and the snapshot
            return real()

        health.capture_error_words = poisoned_capture
        try:
            h = torchsave.save({"w": torch.randn(100)}, str(tmp_path / "p.pt"), async_=True)
        finally:
            health.capture_error_words = real
        c.err = 0  # the live word no longer matters
        with pytest.raises(health.CommPoisonedError):
            h.wait()

    _with_fake_comm(body)
