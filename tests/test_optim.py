"""Fused optimizers vs torch.optim with parameters that have no gradient (frozen, or unused in
a step): torch skips them entirely - no weight decay, no momentum, no step count - and so must
the flat chunk-table kernels.  Step counts are host integers internally but the
state_dict carries torch's per-parameter `step` tensors."""
import pytest
import torch

from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD


def _run(device, kind):
    torch.manual_seed(0)
    shapes = [(33, 17), (17,), (64, 8), (5,)]
    base = [torch.randn(s) for s in shapes]
    ps = [torch.nn.Parameter(b.clone().to(device)) for b in base]
    qs = [torch.nn.Parameter(b.clone().to(device)) for b in base]
    ps[3].requires_grad_(False)
    qs[3].requires_grad_(False)
    if kind == "adamw":
        opt = FusedAdamW(ps, lr=0.01, weight_decay=0.1)
        ref = torch.optim.AdamW(qs, lr=0.01, weight_decay=0.1, foreach=False)
    else:
        opt = FusedSGD(ps, lr=0.01, momentum=0.9, weight_decay=0.05)
        ref = torch.optim.SGD(qs, lr=0.01, momentum=0.9, weight_decay=0.05, foreach=False)
    g = torch.Generator().manual_seed(1)
    for step in range(5):
        opt.zero_grad(set_to_none=True)
        ref.zero_grad(set_to_none=True)
        for i, (p, q) in enumerate(zip(ps, qs)):
            if i == 3 or (i == 2 and step in (0, 3)):  # frozen / unused in steps 0 and 3
                continue
            gr = torch.randn(p.shape, generator=g).to(device)
            p.grad = gr.clone()
            q.grad = gr.clone()
        opt.step()
        ref.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.detach().cpu(), q.detach().cpu(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ps[3].detach().cpu(), base[3])  # frozen: bit-untouched
    sd, rsd = opt.state_dict(), ref.state_dict()
    assert sorted(sd["state"]) == sorted(rsd["state"]) == [0, 1, 2]
    for i in rsd["state"]:
        for k, v in rsd["state"][i].items():
            torch.testing.assert_close(sd["state"][i][k].detach().cpu().float(), v.detach().cpu().float(),
                                       rtol=1e-5, atol=1e-6)
    if kind == "adamw":
        assert float(sd["state"][2]["step"]) == 3.0 and float(sd["state"][0]["step"]) == 5.0
    # round trip: a fresh optimizer loaded from the state dict continues identically
    opt2 = (FusedAdamW if kind == "adamw" else FusedSGD)(ps, **{k: v for k, v in sd["param_groups"][0].items()
                                                               if k in ("lr", "weight_decay")})
    opt2.load_state_dict(sd)
    if kind == "adamw":
        assert opt2._steps[ps[2]] == 3


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_fused_optim_skips_gradless_params_cpu(kind):
    _run("cpu", kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_fused_optim_skips_gradless_params_gpu(kind):
    _run("cuda", kind)
