"""Product path vs bench on one box (VERDICT r5 "next" #7): GPT-2-small through `train_flow.py`
(trainer + session + async sharded DCP commit), an exact resume, an uninterrupted reference run
and `bench.py`, each a child process under its own time limit; prints one JSON summary.

    A: train_flow.py run --model gpt2-small --steps 200 --ckpt_every_n_steps 50 --report_every_n_steps 10
    B: train_flow.py run --model gpt2-small --steps 250 ... --from-run RayTorchTrain/<A> --resume_mode exact
    C: train_flow.py run --model gpt2-small --steps 250 ... (uninterrupted)
    bench.py --model gpt2-small --steps 50 --warmup 10 --no-ckpt

    python scripts/product_path.py OUT_DIR
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(name, cmd, out, env, limit):
    log = os.path.join(out, f"{name}.log")
    with open(log, "w") as f:
        rc = subprocess.run(cmd, cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, timeout=limit).returncode
    print(f"[product] {name} rc={rc}", flush=True)
    if rc != 0:
        print(open(log).read()[-3000:], flush=True)
        sys.exit(rc)
    return open(log).read()


def rows(run_id, home):
    hits = glob.glob(os.path.join(home, "RayTorchTrain", str(run_id), "train", "*", "ray_storage_attempt*", "*", "*",
                                  "result.json"))
    assert hits, f"no result.json for run {run_id}"
    return [json.loads(line) for line in open(sorted(hits)[-1])]


def main():
    out = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/product")
    os.makedirs(out, exist_ok=True)
    home = "/tmp/rtdc_product_home"
    shutil.rmtree(home, ignore_errors=True)
    env = dict(os.environ, RTDC_HOME=home)
    flow = [sys.executable, "train_flow.py", "run", "--model", "gpt2-small", "--ckpt_every_n_steps", "50",
            "--report_every_n_steps", "10", "--num_workers", "1"]
    run("run_a", flow + ["--steps", "200"], out, env, 600)
    run("run_b", flow + ["--steps", "250", "--from-run", "RayTorchTrain/1", "--resume_mode", "exact"], out, env, 600)
    run("run_c", flow + ["--steps", "250"], out, env, 600)
    blog = run("bench", [sys.executable, "bench.py", "--model", "gpt2-small", "--steps", "50", "--warmup", "10",
                         "--no-ckpt"], out, env, 600)
    bench = json.loads([ln for ln in blog.splitlines() if ln.startswith("{")][-1])
    a, b, c = rows(1, home), rows(2, home), rows(3, home)
    for name, rr in (("run_a", a), ("run_b", b), ("run_c", c)):
        with open(os.path.join(out, f"{name}_result.json"), "w") as f:
            f.write("\n".join(json.dumps(r) for r in rr) + "\n")
    # a row whose 10 steps contain a checkpoint drain: the row after each commit step (50, 100, ...)
    drain = [r["samples_per_s"] for r in a if r["step"] > 10 and (r["step"] - 10) % 50 == 0 and r["step"] > 50]
    clean = [r["samples_per_s"] for r in a if r["step"] > 20 and (r["step"] - 10) % 50 != 0]
    resumed = {r["step"] - i: v for r in b for i, v in enumerate(reversed(r["losses"]))}
    ref = {r["step"] - i: v for r in c for i, v in enumerate(reversed(r["losses"]))}
    steps = sorted(k for k in resumed if k > 200)
    summary = {
        "bench_samples_per_s": bench["value"], "bench_ms_per_step": bench["ms_per_step"],
        "trainer_clean_rows": [min(clean), max(clean)], "trainer_drain_rows": [min(drain), max(drain)],
        "trainer_vs_bench": round(sum(clean) / len(clean) / bench["value"], 4),
        "drain_vs_clean": round(sum(drain) / len(drain) / (sum(clean) / len(clean)), 4),
        "resume_steps_compared": [steps[0], steps[-1]] if steps else None,
        "resume_bit_identical": bool(steps) and all(resumed[k] == ref[k] for k in steps),
    }
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
