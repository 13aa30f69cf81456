"""End-to-end model numerics on the GPU: native bf16 path vs the fp32 PyTorch reference path."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gpt2_tiny_matches_reference_and_trains():
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    ref = GPT2(cfg)
    gpu = copy.deepcopy(ref).cuda()
    idx = torch.randint(0, cfg.vocab_size, (4, 128))
    loss_ref = ref(idx, idx.roll(-1, 1))
    loss_ref.backward()
    loss = gpu(idx.cuda(), idx.roll(-1, 1).cuda())
    loss.backward()
    assert abs(loss.item() - loss_ref.item()) < 0.02 * loss_ref.item()
    for (n, p), (_, q) in zip(ref.named_parameters(), gpu.named_parameters()):
        err = (p.grad - q.grad.cpu()).abs().max().item()
        mag = p.grad.abs().max().item() + 1e-8
        assert err < 0.08 * mag, f"{n}: grad err {err} vs {mag}"
    opt = FusedAdamW(gpu.parameters(), lr=3e-3, weight_decay=0.0)
    data = torch.randint(0, cfg.vocab_size, (4, 129), device="cuda")
    losses = []
    for _ in range(30):
        opt.zero_grad()
        l = gpu(data[:, :-1], data[:, 1:])
        l.backward()
        opt.step()
        losses.append(l.item())
    assert losses[-1] < losses[0] - 1.0, losses


def test_toy_mlp_native_fp32():
    from ray_torch_distributed_checkpoint_amd.models import NeuralNetwork
    from ray_torch_distributed_checkpoint_amd.ops import cross_entropy

    torch.manual_seed(0)
    ref = NeuralNetwork()
    ref.eval()
    gpu = copy.deepcopy(ref).cuda().eval()
    x = torch.randn(16, 1, 28, 28)
    y = torch.randint(0, 10, (16,))
    lr = torch.nn.functional.cross_entropy(ref(x), y)
    lr.backward()
    lg = cross_entropy(gpu(x.cuda()), y.cuda())
    lg.backward()
    assert abs(lg.item() - lr.item()) < 1e-4
    for p, q in zip(ref.parameters(), gpu.parameters()):
        assert (p.grad - q.grad.cpu()).abs().max().item() < 1e-4
