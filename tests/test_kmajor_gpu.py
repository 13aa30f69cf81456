"""K-major weight images for the input-gradient GEMMs (ops/shadow.py kmajor_*): the bf16 [in, out]
image of an fp32 master is built on a side stream during the forward and consumed by the
backward's dgrad GEMM with both operands K-major.

* dx through the image equals the fp32 reference and the MN-major path's result;
* after a fused optimizer step (masters changed in place, no version bump) the next backward
  uses a rebuilt image, not the stale one;
* the GPT-2 MLP / attention / LM-head backward with images equals the one without."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu


@pytest.fixture
def kmajor(monkeypatch):
    from ray_torch_distributed_checkpoint_amd.ops import shadow

    def set_mode(v):
        monkeypatch.setattr(shadow, "_KMAJOR", v)

    return set_mode


def _linear_grads(x, w, b):
    from ray_torch_distributed_checkpoint_amd import ops

    x = x.detach().clone().requires_grad_(True)
    w.grad = None
    b.grad = None
    y = ops.linear(x, w, b)
    y.backward(torch.ones_like(y) * 0.01)
    torch.cuda.synchronize()
    return x.grad.float(), w.grad.clone()


def test_linear_dgrad_on_kmajor_image_matches(kmajor):
    torch.manual_seed(0)
    M, K, N = 4096, 768, 2304
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.nn.Parameter(torch.randn(N, K, device="cuda") * 0.02)
    b = torch.nn.Parameter(torch.zeros(N, device="cuda"))
    kmajor("0")
    dx0, dw0 = _linear_grads(x, w, b)
    kmajor("1")
    dx1, dw1 = _linear_grads(x, w, b)
    assert getattr(w, "_rtdc_kimg", None) is not None  # the image path really ran
    ref = (torch.ones(M, N, device="cuda") * 0.01).bfloat16().float() @ w.detach().bfloat16().float()
    assert (dx1 - ref).abs().max() / ref.abs().max() < 1e-2
    assert (dx1 - dx0).abs().max() / dx0.abs().max() < 1e-2
    assert torch.equal(dw0, dw1)


def test_kmajor_image_rebuilt_after_fused_step(kmajor):
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    kmajor("1")
    torch.manual_seed(1)
    M, K, N = 2048, 512, 1024
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.nn.Parameter(torch.randn(N, K, device="cuda") * 0.02)
    b = torch.nn.Parameter(torch.zeros(N, device="cuda"))
    opt = FusedAdamW([w, b], lr=1e-2)
    _linear_grads(x, w, b)
    opt.step()  # masters (and shadows) change in place
    dx, _ = _linear_grads(x, w, b)
    img = w._rtdc_kimg["img"]
    assert torch.equal(img, w.detach().t().contiguous().bfloat16()), "stale K-major image after the step"
    ref = (torch.ones(M, N, device="cuda") * 0.01).bfloat16().float() @ w.detach().bfloat16().float()
    assert (dx - ref).abs().max() / ref.abs().max() < 1e-2


def test_gpt2_backward_with_kmajor_images_matches(kmajor):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    grads = {}
    for mode in ("0", "1"):
        kmajor(mode)
        torch.manual_seed(3)
        model = GPT2(GPT2Config(vocab_size=1000, n_positions=128, n_embd=256, n_layer=2, n_head=4)).cuda()
        idx = torch.randint(0, 1000, (4, 129), device="cuda", generator=torch.Generator("cuda").manual_seed(5))
        model(idx[:, :-1], idx[:, 1:]).backward()
        torch.cuda.synchronize()
        grads[mode] = {n: p.grad.float().clone() for n, p in model.named_parameters()}
    for n, g0 in grads["0"].items():
        g1 = grads["1"][n]
        err = (g1 - g0).norm() / max(g0.norm().item(), 1e-12)
        assert err < 2e-2, (n, float(err))


def test_bf16_transpose_multi_matches_torch():
    """The batched transpose behind the K-major images: several matrices (ragged edges, R and C
    multiples of 8) in one launch, bitwise torch's transpose."""
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    torch.manual_seed(7)
    shapes = [(2304, 768), (768, 3072), (50304, 768), (72, 136), (8, 8), (1000, 24)]
    src = [torch.randn(r, c, device="cuda").bfloat16() for r, c in shapes]
    dst = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes]
    jobs = torch.empty(gpu_ext().bf16_transpose_jobs_bytes(), dtype=torch.uint8, device="cuda")
    gpu_ext().bf16_transpose_multi(src, dst, jobs)
    torch.cuda.synchronize()
    for s, d in zip(src, dst):
        assert torch.equal(d, s.t().contiguous())
