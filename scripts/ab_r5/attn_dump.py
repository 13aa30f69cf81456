"""Dump flash-attention forward + backward outputs (GPT-2 and Llama shapes, fixed seed) to a
.pt file, so two builds of the extension (RTDC_EXT_SO) can be compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention  # noqa: E402

out = {}
for name, B, T, H, Hkv, Dh in [("gpt2", 4, 1024, 12, 12, 64), ("gqa64", 2, 512, 8, 2, 64), ("llama", 1, 1024, 32, 8, 128)]:
    torch.manual_seed(7)
    qkv = (torch.randn(B, T, (H + 2 * Hkv) * Dh, device="cuda") * 0.5).bfloat16().requires_grad_(True)
    y = causal_attention(qkv, H, Hkv)
    g = torch.randn_like(y)
    y.backward(g)
    torch.cuda.synchronize()
    out[name] = (y.detach().cpu(), qkv.grad.detach().cpu())
torch.save(out, sys.argv[1])
