"""Host-vs-device time per training-step phase (GPT-2-small bench workload, 1 GPU).

For each phase (forward, backward, optimizer, zero_grad) prints the CPU time spent issuing it
and the GPU time the phase's kernels took (CUDA events).  A phase whose CPU time approaches its
GPU time is launch-bound; the step's idle gap before the optimizer is (CPU time of the backward
tail + optimizer issue) minus the lead the CPU built up.  Optional --cprofile dumps the top host
functions of the backward + optimizer."""
import argparse
import cProfile
import pstats
import sys
import time
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--cprofile", action="store_true")
    args = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(model=args.model, batch=16, seq_len=1024, batch_set=False, seq_len_set=False,
                            image_size=224)
    wl = bench.build_workload(ns, dev, 0)
    model, opt, fwd = wl["model"], wl["opt"], wl["loss"]
    names = ["fwd", "bwd", "opt", "zero"]
    for i in range(3):
        fwd(model, i).backward()
        opt.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    cpu = {n: [] for n in names}
    gpu = {n: [] for n in names}
    for i in range(args.steps):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        t = [time.perf_counter()]
        ev[0].record()
        loss = fwd(model, i)
        ev[1].record(); t.append(time.perf_counter())
        loss.backward()
        ev[2].record(); t.append(time.perf_counter())
        opt.step()
        ev[3].record(); t.append(time.perf_counter())
        opt.zero_grad()
        ev[4].record(); t.append(time.perf_counter())
        torch.cuda.synchronize()
        for k, n in enumerate(names):
            cpu[n].append((t[k + 1] - t[k]) * 1e3)
            gpu[n].append(ev[k].elapsed_time(ev[k + 1]))
    for n in names:
        c = sorted(cpu[n])[len(cpu[n]) // 2]
        g = sorted(gpu[n])[len(gpu[n]) // 2]
        print(f"{n:5s} cpu {c:8.3f} ms   gpu {g:8.3f} ms", flush=True)
    if args.cprofile:
        pr = cProfile.Profile()
        for i in range(3):
            loss = fwd(model, i)
            torch.cuda.synchronize()
            pr.enable()
            loss.backward()
            opt.step()
            pr.disable()
            opt.zero_grad()
            torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
