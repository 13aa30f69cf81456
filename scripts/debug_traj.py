"""Loss trajectory of GPT-2 (GPU native vs CPU reference) over a few fused-AdamW steps."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config  # noqa: E402
from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "gpt2-tiny"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
torch.manual_seed(0)
cfg = GPT2Config.named(name)
ref = GPT2(cfg)
gpu = copy.deepcopy(ref).cuda()
B, T = 4, 128
data = torch.randint(0, cfg.vocab_size, (4, B, T + 1))
for tag, m, dev in [("cpu", ref, "cpu"), ("gpu", gpu, "cuda")]:
    opt = FusedAdamW(m.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
    ls = []
    for i in range(steps):
        d = data[i % 4].to(dev)
        loss = m(d[:, :-1], d[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        ls.append(round(loss.item(), 4))
    print(tag, ls, flush=True)
