"""Dump a ResNet-18 training step's outputs (loss, every parameter gradient, BN running stats)
to a .pt file, so two builds of the extension (RTDC_EXT_SO) can be compared bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ray_torch_distributed_checkpoint_amd import ops  # noqa: E402
from ray_torch_distributed_checkpoint_amd.models import ResNet18  # noqa: E402

torch.manual_seed(3)
model = ResNet18(num_classes=10).cuda()
x = torch.randn(32, 3, 128, 128, device="cuda")
y = torch.randint(0, 10, (32,), device="cuda")
loss = ops.cross_entropy(model(x), y)
loss.backward()
torch.cuda.synchronize()
out = {"loss": loss.detach().cpu()}
for n, p in model.named_parameters():
    out["grad." + n] = p.grad.detach().cpu()
for n, b in model.named_buffers():
    out["buf." + n] = b.detach().cpu()
torch.save(out, sys.argv[1])
