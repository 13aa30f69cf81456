"""bf16-workload training loops under TorchTrainer on CPU/gloo (BASELINE configs 2-5 plumbing):
periodic async sharded checkpoints committed through report(), retention, kill at step K
with automatic restart, `train_flow.py --from-run ... --resume_mode exact`, and stall
detection of a rank hung before a collective.  Losses after every kind of resume must be
bit-identical to an uninterrupted run."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("RTDC_FORCE_CPU", "1")
    for k in ("RTDC_FAIL_AT_STEP", "RTDC_HANG_AT_STEP", "RTDC_FAIL_AT_REPORT"):
        monkeypatch.delenv(k, raising=False)


def _losses(result_path) -> dict:
    """step -> loss from result.json (every report carries the losses since the previous one);
    a step logged twice (before and after a restart) must have logged the same loss."""
    out = {}
    for line in open(os.path.join(result_path, "result.json")):
        row = json.loads(line)
        s = row["step"]
        for i, v in enumerate(reversed(row["losses"])):
            k = s - i
            if k in out:
                assert out[k] == v, f"step {k} logged twice with different losses: {out[k]} vs {v}"
            out[k] = v
    return out


def _fit(tmp, name, steps=8, workers=2, model="gpt2-tiny", **kw):
    from ray_torch_distributed_checkpoint_amd import workloads as W

    return W.train_workload(model, steps=steps, num_workers=workers, ckpt_every_n_steps=2,
                            checkpoint_storage_path=str(tmp / name), verbose=0, **kw)


def test_async_sharded_checkpoints_committed_with_retention(tmp_path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    r = _fit(tmp_path, "a", steps=6)
    kept = sorted(d for d in os.listdir(r.path) if d.startswith("checkpoint_"))
    assert kept == ["checkpoint_000001", "checkpoint_000002"]  # num_to_keep=2, nothing left in .tmp
    for d in kept:
        files = sorted(os.listdir(os.path.join(r.path, d)))
        assert files == [".metadata", "__0_0.distcp", "__1_0.distcp"]
    assert os.path.basename(r.checkpoint.path) == "checkpoint_000002"
    md = dcp.read_metadata(r.checkpoint.path)
    assert "model.wte" in md.state_dict_metadata and "optim.state.wte.exp_avg" in md.state_dict_metadata
    # stock torch DCP reads the model shard we wrote (format compatibility)
    import torch.distributed.checkpoint as tdcp
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    m = GPT2(GPT2Config.named("gpt2-tiny"))
    sd = {"model": m.state_dict()}
    tdcp.load(sd, checkpoint_id=r.checkpoint.path)
    # per-checkpoint stage/write/commit timings reach the metrics rows
    rows = [json.loads(line) for line in open(os.path.join(r.path, "result.json"))]
    assert rows[-1]["step"] == 6 and len(rows) == 3
    assert any("ckpt_write_s" in row and "ckpt_commit_s" in row for row in rows)
    assert all(row["samples_per_s"] > 0 for row in rows)


def test_kill_at_step_restart_is_bit_equal(tmp_path, monkeypatch):
    """BASELINE config 5: SIGKILL rank 1 at step 5, the supervisor restarts the gang from the
    latest committed sharded checkpoint, and every loss equals the uninterrupted run's."""
    a = _fit(tmp_path, "a")
    monkeypatch.setenv("RTDC_FAIL_AT_STEP", "5:1")
    b = _fit(tmp_path, "b", max_failures=1)
    la, lb = _losses(a.path), _losses(b.path)
    assert sorted(la) == list(range(1, 9)) and sorted(lb) == list(range(1, 9))
    assert la == lb
    assert b.metrics["step"] == 8


def test_from_run_exact_resume_via_train_flow(tmp_path):
    env = dict(os.environ, RTDC_HOME=str(tmp_path / ".rtdc"), RTDC_FORCE_CPU="1", PYTHONPATH=ROOT,
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("RTDC_FAIL_AT_STEP", None)

    def run(*args):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "train_flow.py"), "run", "--model", "gpt2-tiny",
                            "--num_workers", "2", "--ckpt_every_n_steps", "2", *args], cwd=str(tmp_path), env=env,
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]

    run("--steps", "8")                                   # RayTorchTrain/1: uninterrupted
    run("--steps", "4")                                   # RayTorchTrain/2: stops at step 4
    run("--steps", "8", "--from-run", "RayTorchTrain/2", "--resume_mode", "exact")  # /3 continues
    from ray_torch_distributed_checkpoint_amd.flow import registry

    os.environ["RTDC_HOME"] = str(tmp_path / ".rtdc")
    try:
        full = _losses(registry.Run("RayTorchTrain/1").data.result.path)
        first = _losses(registry.Run("RayTorchTrain/2").data.result.path)
        rest = _losses(registry.Run("RayTorchTrain/3").data.result.path)
    finally:
        os.environ.pop("RTDC_HOME", None)
    assert sorted(first) == [1, 2, 3, 4] and sorted(rest) == [5, 6, 7, 8]
    assert {**first, **rest} == full


def test_weights_only_resume_resets_step(tmp_path):
    a = _fit(tmp_path, "a", steps=4)
    b = _fit(tmp_path, "b", steps=2, checkpoint=a.checkpoint, resume_mode="weights")
    assert sorted(_losses(b.path)) == [1, 2]
    # warm start: the first loss is the trained model's, below a fresh model's
    assert _losses(b.path)[1] < _losses(a.path)[1]


def test_hung_rank_is_detected_and_gang_restarted(tmp_path, monkeypatch):
    """Rank 1 blocks forever before step 3's backward all-reduce; rank 0 then sits inside
    the collective (its heartbeat thread keeps beating).  The progress monitor must fail the
    gang within progress_timeout_s, and the restart resumes from the step-2 checkpoint."""
    import time

    ref = _fit(tmp_path, "ref", steps=6)
    monkeypatch.setenv("RTDC_HANG_AT_STEP", "3:1")
    t0 = time.time()
    r = _fit(tmp_path, "h", steps=6, max_failures=1, progress_timeout_s=6.0)
    assert time.time() - t0 < 120
    assert r.metrics["step"] == 6
    assert _losses(r.path) == _losses(ref.path)


@pytest.mark.parametrize("model", ["resnet18-tiny", "llama3-tiny"])
def test_other_workloads_restart_bit_equal(tmp_path, monkeypatch, model):
    a = _fit(tmp_path, "a", steps=4, model=model)
    monkeypatch.setenv("RTDC_FAIL_AT_STEP", "3:0")
    b = _fit(tmp_path, "b", steps=4, model=model, max_failures=1)
    assert _losses(a.path) == _losses(b.path)


def test_bf16_grad_comm_workload_runs(tmp_path):
    r = _fit(tmp_path, "c", steps=4, grad_comm_dtype="bf16")
    la = _losses(r.path)
    ref = _losses(_fit(tmp_path, "d", steps=4).path)
    assert la[1] == ref[1]  # identical init and data; the first update differs only by bf16 rounding
    assert all(abs(la[k] - ref[k]) < 0.05 for k in la)


def test_zero1_workload_kill_restart_bit_equal(tmp_path, monkeypatch):
    """ZeRO-1 under the trainer: the consolidated optimizer state goes into the async sharded
    checkpoint, a restart restores it, and the losses equal both the uninterrupted ZeRO run and
    the replicated-optimizer run."""
    a = _fit(tmp_path, "a", steps=6, zero_stage=1)
    ref = _fit(tmp_path, "r", steps=6)
    monkeypatch.setenv("RTDC_FAIL_AT_STEP", "5:1")
    b = _fit(tmp_path, "b", steps=6, zero_stage=1, max_failures=1)
    la, lb, lr = _losses(a.path), _losses(b.path), _losses(ref.path)
    assert la == lb
    assert la == lr
