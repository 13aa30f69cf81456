"""bench.py's N-rank path end to end on CPU gloo: the driver's 8-GPU run is
the first time this path meets RCCL, so everything except the fabric is rehearsed here -
torchrun launch, preflight all-reduce check, the timed loop, the post-run cross-rank checksum
(`ranks_in_sync`), the coalesced sharded restore and the bucket-size sweep."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(world, *extra, tmp):
    env = dict(os.environ, OMP_NUM_THREADS="1", RTDC_BENCH_CKPT_DIR=str(tmp))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--cpu", "--model", "gpt2-tiny", "--batch", "2", "--seq-len", "64",
           "--steps", "2", "--warmup", "1", "--overlap-steps", "1", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_n_rank_path_on_gloo(tmp_path):
    out = _bench(2, tmp=tmp_path)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["ranks_in_sync"] is True
    comm = out["comm"]
    assert comm["preflight"]["allreduce_check_ok_all_ranks"] is True
    assert len(comm["sweep"]) == 8 and all(s["ms_per_step"] > 0 for s in comm["sweep"])
    # no degenerate (< 1/4 of the first cap) first bucket
    assert comm["bucket_mb"][0] >= 0.5 or len(comm["bucket_mb"]) == 1
    # the checkpoint phase ran at full scope and restored with few collectives
    assert out["ckpt_scope"] == "model + optimizer + step", out.get("ckpt_unmeasured")
    assert out["ckpt_restore_collectives"] <= 16


def test_bench_n_rank_zero1_in_sync(tmp_path):
    out = _bench(2, "--zero", "1", "--sweep", "0", tmp=tmp_path)
    assert out["ranks_in_sync"] is True and out["comm"]["zero_stage"] == 1


def test_bench_watchdog_prints_headline_when_a_later_phase_hangs(tmp_path):
    """a hung post-headline phase (here an injected hang in the bucket
    sweep, as a stuck collective on a first 8-GPU contact would be) must not hide the measured
    throughput: rank 0's watchdog prints the JSON line with `phase_timed_out` and the run exits
    non-zero instead of blocking until the driver's limit."""
    env = dict(os.environ, OMP_NUM_THREADS="1", RTDC_BENCH_CKPT_DIR=str(tmp_path), RTDC_BENCH_HANG_PHASE="sweep")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--cpu", "--model", "gpt2-tiny", "--batch", "2", "--seq-len", "64",
           "--steps", "2", "--warmup", "1", "--overlap-steps", "1", "--sweep-budget-s", "4"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["phase_timed_out"] == "sweep"
    assert out["value"] > 0 and out["n_gpus"] == 2 and out["ranks_in_sync"] is True
    # the checkpoint phase finished before the hang and is reported
    assert out["ckpt_scope"] == "model + optimizer + step"
    assert len(out["ms_per_step_during_async_save_each"]) == 1


def test_ckpt_multiwriter_plumbing_on_gloo(tmp_path):
    """benchmarks/ckpt_multiwriter.py (8 ranks writing their ZeRO-1 Llama shards at once on
    one node) end to end on CPU: every rank's shard written, committed, restored cold and
    verified bitwise."""
    env = dict(os.environ, OMP_NUM_THREADS="1", RTDC_BENCH_CKPT_DIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "benchmarks", "ckpt_multiwriter.py"), "--cpu", "--model", "llama3-tiny"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["world"] == 3 and out["verified_bitwise"] is True and out["restore_cold"] is True
    assert len(out["per_rank_GB"]) == 3 and min(out["per_rank_GB"]) > 0
