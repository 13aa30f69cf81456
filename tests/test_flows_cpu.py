"""train_flow.py / eval_flow.py end to end on CPU: CLI parity, registry, --from-run, trigger."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(tmp_path):
    return dict(os.environ, RTDC_HOME=str(tmp_path / ".rtdc"), RTDC_FMNIST_TRAIN="1500", RTDC_FMNIST_TEST="400",
                RTDC_FORCE_CPU="1", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")


def _run(args, tmp_path, timeout=600):
    r = subprocess.run([sys.executable] + args, cwd=str(tmp_path), env=_env(tmp_path), capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_then_eval_from_run_and_trigger(tmp_path):
    from ray_torch_distributed_checkpoint_amd.flow import registry

    os.environ["RTDC_HOME"] = str(tmp_path / ".rtdc")
    try:
        # deploy the eval flow: it fires when RayTorchTrain finishes (R/eval_flow.py:19)
        _run([os.path.join(ROOT, "eval_flow.py"), "--environment=fast-bakery", "argo-workflows", "create"], tmp_path)
        out = _run([os.path.join(ROOT, "train_flow.py"), "--environment=fast-bakery", "run", "--epochs", "2",
                    "--num_workers", "2"], tmp_path)
        assert "Training from newly initialized" in out
        assert "triggering deployed flow RayTorchEval" in out
        run = registry.Run("RayTorchTrain/1")
        assert run.successful
        res = run.data.result
        assert res.checkpoint is not None and os.path.basename(res.checkpoint.path) == "checkpoint_000001"
        assert os.path.exists(os.path.join(res.checkpoint.path, "latest_model.pt"))
        # triggered eval consumed the train run's checkpoint
        ev = registry.Run("RayTorchEval/1")
        assert ev.successful and ev.meta["triggered_by"] == "RayTorchTrain/1"
        card = os.path.join(registry.task_dir("RayTorchEval", "1", "start", "1"), "cards", "error_analysis.html")
        assert "Misclassifications" in open(card).read()
        # resume training from the run (warm start) and evaluate it by pathspec
        _run([os.path.join(ROOT, "train_flow.py"), "run", "--epochs", "1", "--num_workers", "1",
              "--from-run", "RayTorchTrain/1"], tmp_path)
        t2 = registry.Run("RayTorchTrain/2")
        assert t2.successful and t2.meta["params"]["from-run"] == "RayTorchTrain/1"
        # --from-task precedence and the "null" sentinel
        _run([os.path.join(ROOT, "eval_flow.py"), "run", "--from-task", "RayTorchTrain/2/join/4",
              "--from-run", "null"], tmp_path)
        # unseeded 3-epoch warm-started toy run: well above chance (0.1), exact value varies
        assert registry.Run("RayTorchEval/3").data.accuracy > 0.2
    finally:
        os.environ.pop("RTDC_HOME", None)


def test_eval_without_checkpoint_source_fails(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "eval_flow.py"), "run"], cwd=str(tmp_path),
                       env=_env(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "must specify an upstream run or task id" in (r.stdout + r.stderr)


def test_show_lists_parameters(tmp_path):
    out = _run([os.path.join(ROOT, "train_flow.py"), "show"], tmp_path)
    d = json.loads(out.strip().splitlines()[-1])
    assert d["parameters"]["epochs"] == 3 and d["parameters"]["batch_size"] == 32
    assert d["parameters"]["learning_rate"] == 1e-3 and "from-run" in d["parameters"]
    assert d["schedule"] == "*/5 * * * *"
