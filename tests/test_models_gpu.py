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
        # relative-norm error of the whole gradient (bf16 activations vs the fp32 CPU path)
        err = ((p.grad - q.grad.cpu()).norm() / (p.grad.norm() + 1e-12)).item()
        assert err < 0.02, f"{n}: relative grad error {err:.3e}"
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


def test_gpt2_tied_embedding_grad_in_flat_space():
    """With the fused optimizer's flat gradient buffer in fresh mode, the tied token table's
    two contributions (LM head wgrad, then the embedding scatter-add accumulated in place)
    must equal the reference gradient."""
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    torch.manual_seed(3)
    cfg = GPT2Config.named("gpt2-tiny")
    ref = GPT2(cfg)
    gpu = copy.deepcopy(ref).cuda()
    opt = FusedAdamW(gpu.parameters(), lr=1e-3)
    opt.init_state()
    for _ in range(2):  # the second step exercises a reused buffer
        opt.zero_grad(set_to_none=True)
        idx = torch.randint(0, cfg.vocab_size, (4, 128))
        ref.zero_grad()
        ref(idx, idx.roll(-1, 1)).backward()
        gpu(idx.cuda(), idx.roll(-1, 1).cuda()).backward()
        g, r = gpu.wte.grad.cpu(), ref.wte.grad
        assert gpu.wte.grad.data_ptr() == opt.flat_space.grad_view(gpu.wte).data_ptr()
        err = ((g - r).norm() / r.norm()).item()
        assert err < 0.02, err


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


def test_rope_and_swiglu_kernels():
    import torch.nn.functional as F

    from ray_torch_distributed_checkpoint_amd.ops import llama_ops

    torch.manual_seed(1)
    B, T, H, Hkv, Dh = 2, 64, 4, 2, 128
    qkv = torch.randn(B, T, (H + 2 * Hkv) * Dh, device="cuda").to(torch.bfloat16)
    ref_in = qkv.float().requires_grad_(True)
    ref = llama_ops.rope_ref(ref_in, H, Hkv, 500000.0)
    g = torch.randn_like(ref)
    ref.backward(g)
    x = qkv.clone().requires_grad_(True)
    y = llama_ops.apply_rope(x, H, Hkv, 500000.0)
    assert (y.float() - ref).abs().max().item() < 0.03 * ref.abs().max().item()
    y.backward(g.to(torch.bfloat16))
    assert (x.grad.float() - ref_in.grad).abs().max().item() < 0.03 * ref_in.grad.abs().max().item()

    M, C, Fd = 128, 256, 512
    xm = (torch.randn(M, C, device="cuda") * 0.5).to(torch.bfloat16)
    w13 = torch.randn(2 * Fd, C, device="cuda") * 0.05
    w2 = torch.randn(C, Fd, device="cuda") * 0.05
    res = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    xr, w13r, w2r = xm.float().requires_grad_(True), w13.to(torch.bfloat16).float().requires_grad_(True), \
        w2.to(torch.bfloat16).float().requires_grad_(True)
    gg, uu = F.linear(xr, w13r).chunk(2, dim=-1)
    ref = F.linear(F.silu(gg) * uu, w2r) + res.float()
    gy = torch.randn_like(ref)
    ref.backward(gy)
    xi, w13i, w2i = xm.clone().requires_grad_(True), w13.clone().requires_grad_(True), w2.clone().requires_grad_(True)
    y = llama_ops.swiglu_mlp(xi, w13i, w2i, res)
    for out, r, n in [(y, ref, "y")]:
        assert (out.float() - r).abs().max().item() < 0.03 * r.abs().max().item(), n
    y.backward(gy.to(torch.bfloat16))
    for out, r, n in [(xi.grad, xr.grad, "dx"), (w13i.grad, w13r.grad, "dw13"), (w2i.grad, w2r.grad, "dw2")]:
        assert (out.float() - r).abs().max().item() < 0.04 * r.abs().max().item(), n


def test_llama_tiny_matches_reference_and_trains():
    from ray_torch_distributed_checkpoint_amd.models import Llama, LlamaConfig
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama3-tiny")
    ref = Llama(cfg)
    gpu = copy.deepcopy(ref).cuda()
    idx = torch.randint(0, cfg.vocab_size, (2, 128))
    loss_ref = ref(idx, idx.roll(-1, 1))
    loss_ref.backward()
    loss = gpu(idx.cuda(), idx.roll(-1, 1).cuda())
    loss.backward()
    assert abs(loss.item() - loss_ref.item()) < 0.02 * loss_ref.item()
    for (n, p), (_, q) in zip(ref.named_parameters(), gpu.named_parameters()):
        # relative-norm error of the whole gradient (bf16 activations vs the fp32 CPU path)
        err = ((p.grad - q.grad.cpu()).norm() / (p.grad.norm() + 1e-12)).item()
        assert err < 0.02, f"{n}: relative grad error {err:.3e}"
    opt = FusedAdamW(gpu.parameters(), lr=3e-3, weight_decay=0.0)
    data = torch.randint(0, cfg.vocab_size, (2, 129), device="cuda")
    losses = []
    for _ in range(30):
        opt.zero_grad()
        l = gpu(data[:, :-1], data[:, 1:])
        l.backward()
        opt.step()
        losses.append(l.item())
    assert losses[-1] < losses[0] - 1.0, losses


def test_toy_mlp_hipgraph_step_matches_eager():
    """Whole-step hipGraph capture (utils/graphs.py) of the toy model: replays reproduce the
    eager steps bit for bit, dropout masks included (device-side Philox base)."""
    import torch.nn.functional as F

    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.models import NeuralNetwork
    from ray_torch_distributed_checkpoint_amd.optim import FusedSGD
    from ray_torch_distributed_checkpoint_amd.utils.graphs import CapturedStep

    torch.manual_seed(0)
    base = NeuralNetwork()
    xs = torch.randn(12, 16, 1, 28, 28, device="cuda")
    ys = torch.randint(0, 10, (12, 16), device="cuda")

    def run(graph):
        m = copy.deepcopy(base).cuda()
        opt = FusedSGD(m.parameters(), lr=1e-2, momentum=0.9)
        ops.manual_seed(77)
        x, y = xs[0].clone(), ys[0].clone()

        def step():
            opt.zero_grad()
            loss = ops.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss.detach()

        losses = []
        if graph:
            cs = CapturedStep(step, warmup=3)  # the 3 warm-up steps consume batch 0
            for i in range(3):
                x.copy_(xs[0])
                y.copy_(ys[0])
            for i in range(3, 12):
                x.copy_(xs[i])
                y.copy_(ys[i])
                losses.append(cs.replay().clone())
            cs.close()
        else:
            for i in range(12):
                x.copy_(xs[0] if i < 3 else xs[i])
                y.copy_(ys[0] if i < 3 else ys[i])
                lo = step()
                if i >= 3:
                    losses.append(lo)
        return torch.stack(losses), [p.detach().clone() for p in m.parameters()], ops.default_stream().state_dict()

    le, pe, se = run(False)
    lg, pg, sg = run(True)
    assert torch.equal(le, lg), (le, lg)
    assert all(torch.equal(a, b) for a, b in zip(pe, pg))
    assert se == sg


def test_resnet18_two_captured_steps_replay_equals_eager():
    """bench.py --graph for ResNet-18: one captured step per synthetic batch (shared memory
    pool, replayed alternately in capture order) trains exactly as the eager steps do - loss,
    parameters and BatchNorm running statistics bitwise equal after the same step sequence."""
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.models import ResNet18
    from ray_torch_distributed_checkpoint_amd.optim import FusedSGD
    from ray_torch_distributed_checkpoint_amd.utils.graphs import CapturedStep

    torch.manual_seed(0)
    base = ResNet18(num_classes=10)
    pool = [(torch.randn(8, 3, 64, 64, device="cuda"), torch.randint(0, 10, (8,), device="cuda")) for _ in range(2)]
    seed = torch.ones((), device="cuda")

    def run(graph):
        m = copy.deepcopy(base).cuda()
        opt = FusedSGD(m.parameters(), lr=1e-2, momentum=0.9, weight_decay=5e-5)

        def step(i):
            x, y = pool[i % 2]
            loss = ops.cross_entropy(m(x), y)
            loss.backward(seed)
            opt.step()
            opt.zero_grad()
            return loss.detach()

        losses = [step(0).clone(), step(1).clone()]  # eager warm-up (the bench's warmup steps)
        if graph:
            gp = torch.cuda.graph_pool_handle()
            caps = [CapturedStep(lambda k=k: step(k), warmup=1, pool=gp) for k in range(2)]  # 2 more steps
            for i in range(2, 8):
                losses.append(caps[i % 2].replay().clone())
            caps[0].close()
        else:
            for i in range(2):  # what the two captures' warm-ups ran
                losses.append(step(i).clone())
            for i in range(2, 8):
                losses.append(step(i).clone())
        torch.cuda.synchronize()
        return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}

    le, se = run(False)
    lg, sg = run(True)
    assert len(le) == 10 and len(lg) == 8  # the two captures' warm-up steps return no loss here
    for a, b in zip(le[-6:], lg[-6:]):
        assert torch.equal(a, b)
    for k in se:
        assert torch.equal(se[k], sg[k]), k
