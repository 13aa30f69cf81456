"""Dump LayerNorm / RMSNorm forward + backward results (fixed seed, several widths) to a .pt
file, so two builds of the extension (RTDC_EXT_SO) can be compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ray_torch_distributed_checkpoint_amd.ops.norm import layer_norm, rms_norm  # noqa: E402

out = {}
for kind, M, D in [("rms", 2048, 4096), ("ln", 512, 4096), ("rms", 1024, 1024), ("ln", 4096, 768), ("ln", 256, 2048)]:
    torch.manual_seed(M + D)
    x = torch.randn(M, D, device="cuda").bfloat16().requires_grad_(True)
    w = torch.nn.Parameter(1 + 0.1 * torch.randn(D, device="cuda"))
    b = torch.nn.Parameter(0.1 * torch.randn(D, device="cuda"))
    y = rms_norm(x, w) if kind == "rms" else layer_norm(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    torch.cuda.synchronize()
    out[f"{kind}_{M}x{D}"] = (y.detach().cpu(), x.grad.cpu(), w.grad.cpu(), b.grad.cpu() if b.grad is not None else torch.zeros(1))
torch.save(out, sys.argv[1])
