"""Which torch ops launch device copies in one GPT-2-small training step (torch.profiler)."""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config  # noqa: E402
from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW  # noqa: E402

cfg = GPT2Config.named("gpt2-small")
m = GPT2(cfg).cuda()
opt = FusedAdamW(m.parameters(), lr=6e-4)
data = torch.randint(0, cfg.vocab_size, (16, 1025), device="cuda")


def step():
    loss = m(data[:, :-1], data[:, 1:])
    loss.backward()
    opt.step()
    opt.zero_grad()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=40,
                                                   max_src_column_width=120))

from collections import Counter  # noqa: E402

cnt = Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::to", "aten::add_", "aten::zero_", "aten::fill_"):
        st = [s for s in (ev.stack or []) if "torch/" not in s][:3]
        cnt[(ev.name, str(ev.input_shapes)[:60], " | ".join(st))] += 1
for k, v in cnt.most_common(30):
    print(v, k)
tot = sum(e.self_cpu_time_total for e in prof.key_averages())
print("total self cpu us", tot)
