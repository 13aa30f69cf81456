"""LM-head backward GEMMs at the GPT-2-small shape (16384 tokens x 768 -> 50304): native MFMA
kernels vs hipBLASLt (torch.mm; fp32-output weight gradient through `out_dtype`).
Random operands, interleaved repetitions in one process."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.gemm_bench import timeit, warm_up_clocks  # noqa: E402
from ray_torch_distributed_checkpoint_amd.ops import gemm as G  # noqa: E402


def main():
    M, C, V = 16384, 768, 50304
    dev = torch.device("cuda")
    dl = (torch.randn(M, V, device=dev) * 0.01).bfloat16()
    x = torch.randn(M, C, device=dev).bfloat16()
    w = (torch.randn(V, C, device=dev) * 0.02).bfloat16()
    alpha = torch.ones(1, device=dev)
    dw = torch.empty(V, C, device=dev)
    dw2 = torch.empty(V, C, device=dev)
    warm_up_clocks()
    fl = 2.0 * M * C * V
    res = {}
    for rnd in range(3):
        for name, fn in [
            ("wgrad_native", lambda: G.linear_wgrad(dl, x, out=dw, alpha_dev=alpha)),
            ("wgrad_blaslt", lambda: torch.mm(dl.t(), x, out_dtype=torch.float32, out=dw2)),
            ("dgrad_native", lambda: G.linear_dgrad(dl, w, alpha_dev=alpha)),
            ("dgrad_blaslt", lambda: torch.mm(dl, w)),
        ]:
            t = timeit(fn, 10)
            res.setdefault(name, []).append(round(fl / t / 1e12, 1))
    torch.cuda.synchronize()
    err = ((dw - dw2).abs().max() / dw2.abs().max()).item()
    print(json.dumps({"shape": [M, C, V], "tflops": res, "wgrad_rel_err": err}))


if __name__ == "__main__":
    main()
