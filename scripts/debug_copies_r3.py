"""Who issues the device copies of a GPT-2 training step?  (~43
`__amd_rocclr_copyBuffer` dispatches per step were unexplained.)

Runs the bench.py GPT-2-small step under torch.profiler with Python stacks and prints, per
copy-like op (aten::copy_, aten::clone, aten::contiguous, aten::to/_to_copy, Memcpy/Memset
runtime events), the count per step grouped by the innermost frames of this repository.

    python scripts/debug_copies_r3.py [--steps 3] [--model gpt2-small]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    args = ap.parse_args()
    import bench

    ns = argparse.Namespace(model=args.model, batch=16, seq_len=1024, batch_set=False, seq_len_set=False,
                            image_size=224)
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
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
    keys = ("copy", "clone", "contiguous", "_to_copy", "memcpy", "memset", "fill_", "zero_")
    by_site = collections.Counter()
    by_name = collections.Counter()
    for ev in prof.events():
        name = ev.name.lower()
        if not any(k in name for k in keys):
            continue
        by_name[ev.name] += 1
        frames = [f for f in (ev.stack or []) if "ray_torch_distributed_checkpoint_amd" in f or "bench.py" in f]
        by_site[(ev.name, " <- ".join(frames[:3]) or "(no repo frame)")] += 1
    print(f"== copy-like events per step ({args.steps} steps profiled)")
    for n, c in by_name.most_common():
        print(f"{c / args.steps:8.1f}  {n}")
    print("== by call site (per step)")
    for (n, site), c in by_site.most_common(40):
        print(f"{c / args.steps:8.1f}  {n:32s} {site}")
    kern = collections.Counter()
    for ev in prof.key_averages():
        if ev.device_type is not None and "cuda" in str(ev.device_type).lower():
            kern[ev.key] = ev.count
    print("== device-side events matching copy/fill (count over the profiled steps)")
    for k, c in kern.most_common():
        if any(x in k.lower() for x in ("copy", "fill", "memset", "memcpy")):
            print(f"{c / args.steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
