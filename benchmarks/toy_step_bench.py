"""Reference toy model (BASELINE config 1 workload, R/my_ray_module.py:94-112) training-step
latency on one MI355X: eager native kernels vs one hipGraph replay per step
(utils/graphs.CapturedStep).  B = 16 per worker as in the reference flow.

    python benchmarks/toy_step_bench.py [--batch 16] [--steps 500]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_torch_distributed_checkpoint_amd import ops  # noqa: E402
from ray_torch_distributed_checkpoint_amd.models import NeuralNetwork  # noqa: E402
from ray_torch_distributed_checkpoint_amd.optim import FusedSGD  # noqa: E402
from ray_torch_distributed_checkpoint_amd.utils.graphs import CapturedStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=500)
    args = ap.parse_args()
    torch.manual_seed(0)
    res = {"batch": args.batch}
    for mode in ("eager", "hipgraph", "torch_stock"):
        m = NeuralNetwork().cuda() if mode != "torch_stock" else torch.nn.Sequential(
            torch.nn.Flatten(), torch.nn.Linear(784, 512), torch.nn.ReLU(), torch.nn.Dropout(0.25),
            torch.nn.Linear(512, 512), torch.nn.ReLU(), torch.nn.Dropout(0.25), torch.nn.Linear(512, 10),
            torch.nn.ReLU()).cuda()
        opt = FusedSGD(m.parameters(), lr=1e-3, momentum=0.9) if mode != "torch_stock" else \
            torch.optim.SGD(m.parameters(), lr=1e-3, momentum=0.9)
        x = torch.randn(args.batch, 1, 28, 28, device="cuda")
        y = torch.randint(0, 10, (args.batch,), device="cuda")
        lossf = ops.cross_entropy if mode != "torch_stock" else torch.nn.functional.cross_entropy

        def step():
            opt.zero_grad()
            loss = lossf(m(x), y)
            loss.backward()
            opt.step()
            return loss

        if mode == "hipgraph":
            cs = CapturedStep(step, warmup=3)
            run = cs.replay
        else:
            for _ in range(3):
                step()
            run = step
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        res[f"{mode}_us_per_step"] = round((time.perf_counter() - t0) / args.steps * 1e6, 2)
        if mode == "hipgraph":
            cs.close()
    res["samples_per_sec_hipgraph"] = round(args.batch / res["hipgraph_us_per_step"] * 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
