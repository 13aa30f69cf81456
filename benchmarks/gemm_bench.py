"""GEMM microbenchmark: native gfx950 MFMA kernel vs torch.matmul (hipBLASLt) on the GPT-2
shapes, all three nn.Linear layouts.  Random operands (cdna_hip_programming.md §5.4 rule 25),
interleaved repetitions in one process (rule 24).

    python benchmarks/gemm_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_torch_distributed_checkpoint_amd.ops import gemm as G  # noqa: E402

SHAPES = [  # (name, M tokens, in K, out N)
    ("qkv", 16384, 768, 2304),
    ("attn_proj", 16384, 768, 768),
    ("fc", 16384, 768, 3072),
    ("mlp_proj", 16384, 3072, 768),
    ("lm_head", 16384, 768, 50304),
    ("sq4096", 4096, 4096, 4096),
]
LLAMA_SHAPES = [  # Llama-3-8B decoder layer at 1 x 2048 tokens (GQA 32/8 heads, SwiGLU 14336)
    ("l_qkv", 2048, 4096, 6144),
    ("l_o", 2048, 4096, 4096),
    ("l_gate_up", 2048, 4096, 28672),
    ("l_down", 2048, 14336, 4096),
]


def _mm_f32(a, b):
    """hipBLASLt bf16 x bf16 -> fp32 output (what our weight-gradient kernels write)."""
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        return (a @ b).float()


def timeit(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e-3


def warm_up_clocks(seconds: float = 0.5):
    """Run dense GEMMs until the GPU has left its idle clocks (the first shape's first timing
    otherwise reads a few % low)."""
    import time

    a = torch.randn(4096, 4096, device="cuda").bfloat16()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            a @ a
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--set", default="gpt2", choices=["gpt2", "llama", "all"])
    ap.add_argument("--sweep", action="store_true", help="also time forced tile configurations (all layouts)")
    ap.add_argument("--cfgs", default="0,6,7", help="tile configurations for --sweep")
    ap.add_argument("--layouts", default=None, help="comma list of the rows to time (e.g. fwd,dgrad,dgrad_kmaj)")
    ap.add_argument("--wgrad-group", default=None, choices=["llama", "gpt2"],
                    help="time one layer's grouped weight-gradient launch (gemm_bf16_grouped) against the "
                         "same products on hipBLASLt with fp32 output")
    args = ap.parse_args()
    torch.manual_seed(0)
    warm_up_clocks()
    if args.wgrad_group:
        return wgrad_group(args)
    res = []
    shapes = {"gpt2": SHAPES, "llama": LLAMA_SHAPES, "all": SHAPES + LLAMA_SHAPES}[args.set]
    for name, M, K, N in shapes:
        if args.only and args.only != name:
            continue
        xs = float(os.environ.get("GEMM_BENCH_XSCALE", "1"))  # e.g. 0.05: model-like magnitudes
        x = (torch.randn(M, K, device="cuda") * xs).bfloat16()
        w = (torch.randn(N, K, device="cuda") * xs).bfloat16()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        flops = 2.0 * M * N * K
        row = {"shape": name, "M": M, "K": K, "N": N}
        bias = torch.randn(N, device="cuda").bfloat16()
        bias32 = bias.float()  # the models pass their fp32 master bias
        res_in = torch.randn(M, N, device="cuda").bfloat16()
        pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        dxk = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        cs_out = torch.empty(K, device="cuda", dtype=torch.float32)
        for lay, ours, ref in [
            ("fwd", lambda: G.linear_fwd(x, w), lambda: x @ w.t()),
            # fused epilogues as the GPT-2 blocks use them (reference: unfused torch ops)
            ("fwd_bias_gelu", lambda: G.linear_fwd(x, w, bias, act=G.ACT_GELU, aux_out=pre),
             lambda: torch.nn.functional.gelu(torch.addmm(bias, x, w.t()), approximate="tanh")),
            ("fwd_f32bias_gelu", lambda: G.linear_fwd(x, w, bias32, act=G.ACT_GELU, aux_out=pre),
             lambda: torch.nn.functional.gelu(torch.addmm(bias32, x.float(), w.float().t()), approximate="tanh")),
            ("fwd_bias_res", lambda: G.linear_fwd(x, w, bias, residual=res_in),
             lambda: torch.addmm(bias, x, w.t()) + res_in),
            ("dgrad_gelu", lambda: G.linear_dgrad(dy, w, G.ACT_GELU_BWD, aux_in=x), lambda: dy @ w),
            # as the MLP backward runs it: + the bias-gradient column sums in the epilogue
            ("dgrad_gelu_cs", lambda: G.linear_dgrad(dy, w, G.ACT_GELU_BWD, aux_in=x, colsum_out=cs_out),
             lambda: dy @ w),
            # the same on a K-major image of w (persistent 8-wave kernel eligible)
            ("dgrad_gelu_cs_kmaj", lambda: G.gemm_bf16(dy, wt, dxk, M, K, N, N, N, K, True, True, aux_in=x,
                                                       act=G.ACT_GELU_BWD, colsum_out=cs_out), lambda: dy @ w),
            ("dgrad", lambda: G.linear_dgrad(dy, w), lambda: dy @ w),
            # the same product on a K-major (transposed) bf16 image of w
            ("dgrad_kmaj", lambda: G.gemm_bf16(dy, wt, dxk, M, K, N, N, N, K, True, True), lambda: dy @ w),
            ("wgrad", lambda: G.linear_wgrad(dy, x), lambda: (dy.t() @ x)),
            # same product, hipBLASLt writing fp32 like our kernel does
            ("wgrad_f32out", lambda: G.linear_wgrad(dy, x), lambda: _mm_f32(dy.t(), x)),
        ]:
            if args.layouts and lay not in args.layouts.split(","):
                continue
            # interleaved rounds, best of each: neither side is always timed first
            t_o = t_r = float("inf")
            for _ in range(3):
                t_o = min(t_o, timeit(ours, args.reps))
                t_r = min(t_r, timeit(ref, args.reps))
            row[lay] = {"ours_TF": round(flops / t_o / 1e12, 1), "hipblaslt_TF": round(flops / t_r / 1e12, 1),
                        "ours_us": round(t_o * 1e6, 1), "hipblaslt_us": round(t_r * 1e6, 1)}
        if args.sweep:
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
            dw = torch.empty(N, K, device="cuda", dtype=torch.float32)
            for cfg in [int(c) for c in args.cfgs.split(",")]:
                for lay, fn in [
                    ("fwd", lambda: G.gemm_bf16(x, w, y, M, N, K, K, K, N, tile_cfg=cfg)),
                    ("dgrad", lambda: G.gemm_bf16(dy, w, dx, M, K, N, N, K, K, True, False, tile_cfg=cfg)),
                    ("wgrad", lambda: G.gemm_bf16(dy, x, dw, N, K, M, N, K, K, False, False, tile_cfg=cfg)),
                ]:
                    t = min(timeit(fn, args.reps) for _ in range(3))
                    row[f"{lay}_cfg{cfg}_TF"] = round(flops / t / 1e12, 1)
        # correctness spot check (fwd)
        ref = (x.float() @ w.float().t())
        err = (G.linear_fwd(x, w).float() - ref).abs().max().item() / ref.abs().max().item()
        row["fwd_rel_err"] = err
        res.append(row)
        print(json.dumps(row), flush=True)


def wgrad_group(args):
    """One grouped launch of a layer's weight gradients (Llama-3-8B: qkv, o, gate_up, down at
    2048 tokens; GPT-2: two layers' qkv / proj / fc / mlp_proj at 16384 tokens) vs hipBLASLt."""
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    if args.wgrad_group == "llama":
        M, prods = 2048, [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    else:
        M, prods = 16384, [(2304, 768), (768, 768), (3072, 768), (768, 3072)] * 2
    dys = [torch.randn(M, n, device="cuda").bfloat16() for n, _ in prods]
    xs = [torch.randn(M, k, device="cuda").bfloat16() for _, k in prods]
    outs = [torch.empty(n, k, device="cuda") for n, k in prods]
    dims = []
    for n, k in prods:
        dims += [n, k, M, n, k, k]
    flops = sum(2.0 * M * n * k for n, k in prods)

    def ours():
        gpu_ext().gemm_bf16_grouped(dys, xs, outs, dims, False, False)

    def ref():
        for dy, x in zip(dys, xs):
            _mm_f32(dy.t(), x)

    t_o = t_r = float("inf")
    for _ in range(3):
        t_o = min(t_o, timeit(ours, args.reps))
        t_r = min(t_r, timeit(ref, args.reps))
    tiles = sum(((n + 255) // 256) * ((k + 255) // 256) for n, k in prods)
    row = {"wgrad_group": args.wgrad_group, "tokens": M, "products": len(prods), "tiles": tiles,
           "persistent": os.environ.get("RTDC_G8G_PERSIST", "1") != "0",
           "ours_TF": round(flops / t_o / 1e12, 1), "hipblaslt_TF": round(flops / t_r / 1e12, 1),
           "ours_us": round(t_o * 1e6, 1), "hipblaslt_us": round(t_r * 1e6, 1)}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
