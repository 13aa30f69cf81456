"""What the fused epilogues cost: the GPT-2 forward products with and without their epilogue
work (bias, GELU + pre-activation side output, residual add), on random operands, interleaved
repetitions in one process.

    python benchmarks/epilogue_bench.py [--reps 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_torch_distributed_checkpoint_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = 16384
    out = []
    for name, K, N in (("qkv", 768, 2304), ("attn_proj", 768, 768), ("fc", 768, 3072), ("mlp_proj", 3072, 768)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        variants = {
            "plain": lambda: G.linear_fwd(x, w),
            "bias": lambda: G.linear_fwd(x, w, bias=b),
            "bias+res": lambda: G.linear_fwd(x, w, bias=b, residual=res),
            "bias+gelu+pre": lambda: G.linear_fwd(x, w, bias=b, act=G.ACT_GELU, aux_out=pre),
            "hipblaslt": lambda: torch.matmul(x, w.t()),
        }
        row = {"shape": name, "M": M, "K": K, "N": N}
        for _ in range(2):
            for k, f in variants.items():
                t = timeit(f, args.reps)
                row[k + "_us"] = round(min(t, row.get(k + "_us", 1e9)), 1)
        fl = 2.0 * M * N * K
        row["plain_TF"] = round(fl / row["plain_us"] / 1e6, 1)
        row["hipblaslt_TF"] = round(fl / row["hipblaslt_us"] / 1e6, 1)
        print(json.dumps(row), flush=True)
        out.append(row)


if __name__ == "__main__":
    main()
