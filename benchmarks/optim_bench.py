"""Fused AdamW step over a flat parameter space (optim/fused.py FusedAdamW, optim.hip
adamw_kernel): time per step and the HBM rate it reaches (30 B per parameter: read p, g, m, v;
write p, m, v and the bf16 shadow).  Sizes: GPT-2-small (124.4 M) and Llama-3-8B (8.03 B).

    python benchmarks/optim_bench.py [--params 124.4e6,8.03e9] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="124.4e6,8.03e9")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    for n in (int(float(x)) for x in args.params.split(",")):
        # parameter shapes like a transformer's: square-ish matrices of ~n/64 elements
        per = max(1 << 16, n // 64)
        shapes, left = [], n
        while left > 0:
            k = min(per, left)
            shapes.append(k)
            left -= k
        params = [torch.nn.Parameter(torch.randn(k, device=dev) * 0.02) for k in shapes]
        opt = FusedAdamW(params, lr=1e-4, weight_decay=0.1)
        for p in params:
            p.grad = torch.randn_like(p)
        opt.step()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        best = float("inf")
        for _ in range(3):
            ev[0].record()
            for _ in range(args.reps):
                opt.step()
            ev[1].record()
            torch.cuda.synchronize()
            best = min(best, ev[0].elapsed_time(ev[1]) / args.reps)
        row = {"params": n, "ms": round(best, 3), "TBps": round(30.0 * n / (best * 1e-3) / 1e12, 2),
               "env": {k: v for k, v in os.environ.items() if k.startswith(("RTDC_ADAMW", "RTDC_OPT"))}}
        print(json.dumps(row), flush=True)
        del params, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
