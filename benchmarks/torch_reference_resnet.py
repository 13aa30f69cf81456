"""Stock-PyTorch baseline of BASELINE config 2 (ResNet-18, 10 classes, 224x224, bf16) on the
same MI355X, for comparison with `bench.py --model resnet18` (same model, batch, optimizer).

torchvision is not in this image, so the network is written with torch.nn modules (the
standard ResNet-18 topology).  Stack: bf16 autocast + channels_last (MIOpen convolutions),
nn.BatchNorm2d, torch.optim.SGD(fused) momentum 0.9, torch DCP save/load of model+optimizer.

    python benchmarks/torch_reference_resnet.py --steps 10 --warmup 3 [--batch 256]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import tempfile
import time

import torch
import torch.distributed.checkpoint as tdcp
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        h = F.relu(self.bn1(self.conv1(x)))
        h = self.bn2(self.conv2(h))
        return F.relu(h + (x if self.downsample is None else self.downsample(x)))


class ResNet18(nn.Module):
    def __init__(self, n=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers, cin = [], 64
        for i, w in enumerate((64, 128, 256, 512)):
            layers.append(nn.Sequential(Block(cin, w, 1 if i == 0 else 2), Block(w, w, 1)))
            cin = w
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, n)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(self.layers(x), 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--no-channels-last", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    mf = torch.contiguous_format if args.no_channels_last else torch.channels_last
    model = ResNet18().to(dev).to(memory_format=mf)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-5, fused=True)
    B = args.batch
    x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=mf)
    y = torch.randint(0, 10, (B,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
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
    path = os.path.join(tempfile.gettempdir(), "torch_ref_resnet_ckpt")
    shutil.rmtree(path, ignore_errors=True)
    state = {"model": model.state_dict(), "optim": opt.state_dict()}
    t1 = time.perf_counter()
    tdcp.save(state, checkpoint_id=path)
    t_save = time.perf_counter() - t1
    t2 = time.perf_counter()
    tdcp.load(state, checkpoint_id=path)
    opt.load_state_dict(state["optim"])
    torch.cuda.synchronize()
    t_load = time.perf_counter() - t2
    print(json.dumps({"stack": "stock torch (autocast bf16, %s, MIOpen conv, BatchNorm2d, fused SGD, torch DCP)"
                      % ("NCHW" if args.no_channels_last else "channels_last"),
                      "value": round(B * args.steps / dt, 3), "ms_per_step": round(dt / args.steps * 1e3, 3),
                      "batch": B, "final_loss": round(loss.item(), 4), "ckpt_save_sync_s": round(t_save, 4),
                      "ckpt_restore_s": round(t_load, 4), "ckpt_save_plus_restore_s": round(t_save + t_load, 4)}),
          flush=True)
    shutil.rmtree(path, ignore_errors=True)


if __name__ == "__main__":
    main()
