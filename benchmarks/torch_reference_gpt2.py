"""Stock-PyTorch baseline of the headline workload on the same MI355X (for comparison only).

The reference repo trains with Ray Train -> torch DDP + ATen kernels and checkpoints with
torch.save / torch DCP.  It publishes no numbers, so this script measures what
that software stack does on MI355X for the bench.py workload: GPT-2-small, 16x1024 tokens
per GPU, bf16 autocast (hipBLASLt GEMMs, SDPA attention), torch DDP (25 MiB buckets),
torch.optim.AdamW(fused=True), torch.distributed.checkpoint save/load of model+optimizer.
Same JSON keys as bench.py so the two can be compared line by line.

    python benchmarks/torch_reference_gpt2.py --steps 10 --warmup 3
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import tempfile
import time

import torch
import torch.distributed as dist
import torch.distributed.checkpoint as tdcp
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, C, H):
        super().__init__()
        self.H = H
        self.ln_1 = nn.LayerNorm(C)
        self.c_attn = nn.Linear(C, 3 * C)
        self.c_proj = nn.Linear(C, C)
        self.ln_2 = nn.LayerNorm(C)
        self.c_fc = nn.Linear(C, 4 * C)
        self.mlp_proj = nn.Linear(4 * C, C)

    def forward(self, x):
        B, T, C = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).split(C, dim=2)
        q, k, v = (t.view(B, T, self.H, C // self.H).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, C)
        x = x + self.c_proj(y)
        return x + self.mlp_proj(F.gelu(self.c_fc(self.ln_2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, V=50304, T=1024, C=768, L=12, H=12):
        super().__init__()
        self.wte = nn.Embedding(V, C)
        self.wpe = nn.Embedding(T, C)
        self.h = nn.ModuleList([Block(C, H) for _ in range(L)])
        self.ln_f = nn.LayerNorm(C)

    def forward(self, idx, tgt):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in self.h:
            x = b(x)
        logits = F.linear(self.ln_f(x), self.wte.weight)
        return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), tgt.reshape(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(0)
    model = GPT().to(dev)
    net = nn.parallel.DistributedDataParallel(model, device_ids=[local]) if world > 1 else model
    opt = torch.optim.AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1, fused=True)
    B, T = args.batch, 1024
    data = torch.randint(0, 50257, (B, T + 1), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = net(data[:, :-1], data[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sps = world * B * args.steps / dt
    path = os.path.join(tempfile.gettempdir(), "torch_ref_ckpt")
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)
    state = {"model": model.state_dict(), "optim": opt.state_dict()}
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tdcp.save(state, checkpoint_id=path)
    t_save = time.perf_counter() - t1
    t2 = time.perf_counter()
    tdcp.load(state, checkpoint_id=path)
    opt.load_state_dict(state["optim"])
    torch.cuda.synchronize()
    t_load = time.perf_counter() - t2
    if rank == 0:
        print(json.dumps({"stack": "stock torch (autocast bf16, hipBLASLt, SDPA, DDP, fused AdamW, torch DCP)",
                          "value": round(sps, 3), "ms_per_step": round(dt / args.steps * 1e3, 3), "n_gpus": world,
                          "samples_per_sec_per_gpu": round(sps / world, 3), "final_loss": round(loss.item(), 4),
                          "ckpt_save_sync_s": round(t_save, 4), "ckpt_restore_s": round(t_load, 4),
                          "ckpt_save_plus_restore_s": round(t_save + t_load, 4)}), flush=True)
        shutil.rmtree(path, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
