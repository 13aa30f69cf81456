"""Which ATen ops (and from which source lines) still launch GPU work in one training step of a
bench workload.  usage: python scripts/aten_ops.py [--model resnet18|gpt2-small]"""
import argparse
import os
import sys
from collections import Counter

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    args = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(model=args.model, batch=16 if "gpt" in args.model else 64, seq_len=1024,
                            batch_set=True, seq_len_set=False, image_size=224)
    wl = bench.build_workload(ns, dev, 0)
    model, opt, fwd = wl["model"], wl["opt"], wl["loss"]

    def step(i):
        fwd(model, i).backward()
        opt.step()
        opt.zero_grad()

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step(3)
        torch.cuda.synchronize()
    cnt = Counter()
    skip = ("aten::empty", "aten::view", "aten::as_strided", "aten::slice", "aten::detach", "aten::reshape",
            "aten::t", "aten::transpose", "aten::permute", "aten::expand", "aten::select", "aten::alias",
            "aten::unsqueeze", "aten::squeeze", "aten::_reshape_alias", "aten::empty_strided", "aten::empty_like",
            "aten::resolve_conj", "aten::resolve_neg", "aten::lift_fresh", "detach", "aten::split",
            "aten::narrow", "aten::result_type", "aten::is_nonzero", "aten::item", "aten::_local_scalar_dense")
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.name in skip:
            continue
        st = [s for s in (ev.stack or []) if "torch/" not in s and "<built-in" not in s][:2]
        cnt[(ev.name, " | ".join(st))] += 1
    for (name, st), v in cnt.most_common(40):
        print(f"{v:4d} {name:32s} {st}")


if __name__ == "__main__":
    main()
