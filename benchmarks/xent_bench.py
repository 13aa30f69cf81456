"""Fused LM-head cross-entropy kernel on the GPT-2 logits shape ([16384, 50304] bf16, 50257
real columns, gradient written in place): register-resident single-read kernel vs the
two-pass kernel (RTDC_XENT_TWO_PASS=1), interleaved rounds in one process.

    python benchmarks/xent_bench.py [--rows 16384] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--V", type=int, default=50257)
    ap.add_argument("--ld", type=int, default=50304)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    x0 = (torch.randn(a.rows, a.ld, device="cuda") * 2).bfloat16()
    tgt = torch.randint(0, a.V, (a.rows,), device="cuda")
    loss = torch.empty(a.rows, device="cuda")
    ext = gpu_ext()
    res = {"rows": a.rows, "ld": a.ld}
    bufs = {k: x0.clone() for k in ("reg", "two_pass")}
    times = {k: [] for k in bufs}
    for _ in range(5):
        for k, buf in bufs.items():
            if k == "two_pass":
                os.environ["RTDC_XENT_TWO_PASS"] = "1"
            else:
                os.environ.pop("RTDC_XENT_TWO_PASS", None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                buf.copy_(x0) if False else None
                ext.xent(buf, buf, tgt, loss, None, None, a.rows, a.V, a.ld, 1.0 / a.rows, -100)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.reps * 1e3)
    os.environ.pop("RTDC_XENT_TWO_PASS", None)
    nbytes = 2 * a.rows * a.ld * 2
    for k, ts in times.items():
        t = sorted(ts)[len(ts) // 2]
        res[f"{k}_us"] = round(t, 1)
        res[f"{k}_TBps_rw"] = round(nbytes / (t * 1e-6) / 1e12, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
