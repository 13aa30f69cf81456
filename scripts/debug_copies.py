"""Who issues the device copies of a GPT-2 training step?  (~43
`__amd_rocclr_copyBuffer` dispatches per step were unexplained.)

Runs the bench.py GPT-2-small step under a TorchDispatchMode that sees every ATen op the step
dispatches (including the ones autograd issues from C++), and prints, per copy-like op
(copy_, clone, _to_copy, contiguous copies, fills, cat), the count per step grouped by the
innermost frames of this repository in the Python stack.

    python scripts/debug_copies.py [--steps 3] [--model gpt2-small]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("copy", "clone", "_to_copy", "fill", "zero", "cat", "stack", "index", "scatter", "sort")


class CopyLog(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.by_site = collections.Counter()
        self.by_op = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket.__name__)
        if any(k in name for k in KEYS):
            dev = any(isinstance(a, torch.Tensor) and a.is_cuda for a in args)
            if dev:
                frames = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack()
                          if ("ray_torch_distributed_checkpoint_amd" in f.filename or f.filename.endswith("bench.py"))]
                self.by_op[name] += 1
                self.by_site[(name, " <- ".join(reversed(frames[-3:])) or "(no repo frame)")] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    args = ap.parse_args()
    import bench

    ns = argparse.Namespace(model=args.model, batch=None, seq_len=1024, batch_set=False, seq_len_set=False,
                            image_size=224)
    ns.batch = 16
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    wl = bench.build_workload(ns, dev, 0)
    model, opt, loss_fn = wl["model"], wl["opt"], wl["loss"]
    seed = torch.ones((), dtype=torch.float32, device=dev)

    def step(i):
        loss = loss_fn(model, i)
        loss.backward(seed)
        opt.step()
        opt.zero_grad()

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    log = CopyLog()
    with log:
        for i in range(args.steps):
            step(i)
    torch.cuda.synchronize()
    print(f"== copy-like ATen ops on device tensors, per step ({args.steps} steps)")
    for n, c in log.by_op.most_common():
        print(f"{c / args.steps:8.1f}  {n}")
    print("== by call site (per step), innermost repository frames first")
    for (n, site), c in log.by_site.most_common(60):
        print(f"{c / args.steps:8.1f}  {n:20s} {site}")


if __name__ == "__main__":
    main()
