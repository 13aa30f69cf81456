"""Diagnostic: per-parameter difference between the 1-rank forced-collective RCCL DDP gradient
and the single-process reference (tests/test_ddp_gpu.py), printed for every parameter."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import test_ddp_gpu as T  # noqa: E402


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    out = T._run(1, "nccl", dt, force=True)
    ref = T._reference(1)
    bad = 0
    for n, v in ref.items():
        g = torch.from_numpy(out[0][0][n])
        if dt != "fp32":
            v = v.to(torch.bfloat16).float()
        d = (g - v).abs().max().item()
        if d:
            bad += 1
            print(f"DIFF {n}: max abs {d:.3e} rel {(g - v).norm().item() / max(v.norm().item(), 1e-30):.3e}")
    print(f"{dt}: {bad} of {len(ref)} parameters differ")


if __name__ == "__main__":
    main()
