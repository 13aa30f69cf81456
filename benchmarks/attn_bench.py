"""Causal flash attention microbenchmark (native fwd/bwd vs torch SDPA) on the GPT-2-small and
Llama-3-8B shapes; random operands, one process, interleaved repetitions.

    python benchmarks/attn_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext  # noqa: E402
from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention  # noqa: E402

SHAPES = [("gpt2", 16, 1024, 12, 12, 64), ("llama8b", 1, 2048, 32, 8, 128), ("llama8b_b4", 4, 2048, 32, 8, 128)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    torch.manual_seed(0)
    from gemm_bench import warm_up_clocks

    warm_up_clocks()
    for name, B, T, H, Hkv, Dh in SHAPES:
        if args.only and name != args.only:
            continue
        W = (H + 2 * Hkv) * Dh
        qkv = (torch.randn(B, T, W, device="cuda") * 0.5).bfloat16().requires_grad_(True)
        flops_f = 2 * 2 * B * H * T * T * Dh / 2  # causal
        y = causal_attention(qkv, H, Hkv)
        dy = torch.randn_like(y)
        t_f = min(timeit(lambda: causal_attention(qkv, H, Hkv), args.reps) for _ in range(3))

        def fb():
            out = causal_attention(qkv, H, Hkv)
            out.backward(dy)

        t_fb = min(timeit(fb, args.reps) for _ in range(3))
        # the kernels alone (what a training step pays; the autograd round trip above adds host
        # overhead the GPU can wait on in an isolated loop): flash_fwd, flash_bwd (dQ + dK/dV)
        ext = gpu_ext()
        scale = Dh ** -0.5
        q_ = qkv.detach()
        o_ = torch.empty((B, T, H * Dh), dtype=torch.bfloat16, device="cuda")
        lse = torch.empty((B * H, T), dtype=torch.float32, device="cuda")
        ext.flash_fwd(q_, o_, lse, B, T, H, Hkv, Dh, scale)
        dqkv = torch.empty_like(q_)
        delta = torch.empty((B * H, T), dtype=torch.float32, device="cuda")
        dyc = dy.contiguous()
        t_kf = min(timeit(lambda: ext.flash_fwd(q_, o_, lse, B, T, H, Hkv, Dh, scale), args.reps) for _ in range(3))
        t_kb = min(timeit(lambda: ext.flash_bwd(q_, o_, dyc, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, None), args.reps)
                   for _ in range(3))
        # the same backward with delta first and the dQ / dK/dV passes on two streams
        # (ops/attention.py RTDC_FA_CONCURRENT)
        side = torch.cuda.Stream()

        def conc():
            ext.flash_delta(o_, dyc, delta, B, T, H, Dh)
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                ext.flash_bwd(q_, o_, dyc, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, None, which=2, delta_ready=True)
            ext.flash_bwd(q_, o_, dyc, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, None, which=1, delta_ready=True)
            cur.wait_stream(side)

        t_kc = min(timeit(conc, args.reps) for _ in range(3))
        q = qkv.detach()[..., : H * Dh].view(B, T, H, Dh).transpose(1, 2).contiguous().requires_grad_(True)
        k = qkv.detach()[..., H * Dh:(H + Hkv) * Dh].view(B, T, Hkv, Dh).transpose(1, 2)
        v = qkv.detach()[..., (H + Hkv) * Dh:].view(B, T, Hkv, Dh).transpose(1, 2)
        k = k.repeat_interleave(H // Hkv, 1).contiguous().requires_grad_(True)
        v = v.repeat_interleave(H // Hkv, 1).contiguous().requires_grad_(True)
        t_sf = min(timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True), args.reps) for _ in range(3))
        do = torch.randn(B, H, T, Dh, device="cuda", dtype=torch.bfloat16)

        def sfb():
            F.scaled_dot_product_attention(q, k, v, is_causal=True).backward(do)

        t_sfb = min(timeit(sfb, args.reps) for _ in range(3))
        print(json.dumps({"shape": name, "B": B, "T": T, "H": H, "Hkv": Hkv, "Dh": Dh,
                          "fwd_us": round(t_f * 1e6, 1), "fwd_TF": round(flops_f / t_f / 1e12, 1),
                          "bwd_us": round((t_fb - t_f) * 1e6, 1),
                          "bwd_TF": round(2.5 * flops_f / (t_fb - t_f) / 1e12, 1),
                          "kernel_fwd_us": round(t_kf * 1e6, 1), "kernel_fwd_TF": round(flops_f / t_kf / 1e12, 1),
                          "kernel_bwd_us": round(t_kb * 1e6, 1),
                          "kernel_bwd_TF": round(2.5 * flops_f / t_kb / 1e12, 1),
                          "kernel_bwd_concurrent_us": round(t_kc * 1e6, 1),
                          "sdpa_fwd_us": round(t_sf * 1e6, 1), "sdpa_fwd_TF": round(flops_f / t_sf / 1e12, 1),
                          "sdpa_bwd_us": round((t_sfb - t_sf) * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
