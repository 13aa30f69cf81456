"""Optimizer updates overlapped with backward (optim/overlap.py BackwardOverlap): bitwise the
same parameters and optimizer state as the plain `opt.step()` after several steps -
single process (AdamW on GPT-2-tiny, momentum SGD on a small ResNet), and data parallel (two
gloo ranks sharing the GPU with bf16 gradient communication: the engine's widen events order
the early updates); a second backward before `step()` raises."""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _gpt2_run(overlap: bool, steps: int = 4, bucket_mb: float = 0.05):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import BackwardOverlap, FusedAdamW

    torch.manual_seed(0)
    model = GPT2(GPT2Config.named("gpt2-tiny")).to(DEV)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)
    if overlap:
        ov = BackwardOverlap(opt, bucket_mb=bucket_mb)
        assert len(ov.groups) > 2
    g = torch.Generator(device=DEV).manual_seed(1)
    losses = []
    for _ in range(steps):
        data = torch.randint(0, 1000, (4, 65), device=DEV, generator=g)
        loss = model(data[:, :-1], data[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return losses, [p.detach().clone() for p in model.parameters()], opt._bufs["exp_avg_sq"].clone()


def test_adamw_overlap_bitwise_equal():
    l0, p0, v0 = _gpt2_run(False)
    l1, p1, v1 = _gpt2_run(True)
    assert l0 == l1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    assert torch.equal(v0, v1)


def test_sgd_overlap_bitwise_equal_resnet():
    from ray_torch_distributed_checkpoint_amd.models import ResNet18
    from ray_torch_distributed_checkpoint_amd.ops import cross_entropy
    from ray_torch_distributed_checkpoint_amd.optim import BackwardOverlap, FusedSGD

    out = []
    for overlap in (False, True):
        torch.manual_seed(0)
        model = ResNet18(num_classes=10).to(DEV)
        opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        if overlap:
            BackwardOverlap(opt, bucket_mb=1.0)
        g = torch.Generator(device=DEV).manual_seed(2)
        for _ in range(3):
            x = torch.randn(8, 3, 64, 64, device=DEV, generator=g)
            y = torch.randint(0, 10, (8,), device=DEV, generator=g)
            cross_entropy(model(x), y).backward()
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        out.append([p.detach().clone() for p in model.parameters()] + [b.clone() for b in model.buffers()])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_overlap_rejects_gradient_accumulation():
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import BackwardOverlap, FusedAdamW

    torch.manual_seed(0)
    model = GPT2(GPT2Config.named("gpt2-tiny")).to(DEV)
    opt = FusedAdamW(model.parameters(), lr=1e-3)
    BackwardOverlap(opt, bucket_mb=0.05)
    data = torch.randint(0, 1000, (4, 65), device=DEV)
    model(data[:, :-1], data[:, 1:]).backward()
    with pytest.raises(RuntimeError, match="already updated"):
        model(data[:, :-1], data[:, 1:]).backward()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, overlap, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
        from ray_torch_distributed_checkpoint_amd.optim import BackwardOverlap, FusedAdamW
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        torch.manual_seed(0)
        model = GPT2(GPT2Config.named("gpt2-tiny")).to(DEV)
        net = DistributedDataParallel(model, bucket_cap_mb=0.25, first_bucket_mb=0.05, grad_comm_dtype="bf16",
                                      defer_tail_to_optimizer=True)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)
        if overlap:
            BackwardOverlap(opt, ddp=net)
        g = torch.Generator().manual_seed(7)
        for _ in range(3):
            data = torch.randint(0, 1000, (2 * world, 65), generator=g).to(DEV)[2 * rank:2 * rank + 2]
            net(data[:, :-1], data[:, 1:]).backward()
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        q.put((rank, "ok", [p.detach().float().cpu().numpy() for p in model.parameters()]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _spawn(world, overlap):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, world, port, overlap, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, st, v = q.get(timeout=180)
            assert st == "ok", v
            out[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


def test_ddp_bf16_overlap_bitwise_equal():
    base = _spawn(2, False)
    ov = _spawn(2, True)
    for r in (0, 1):
        for a, b in zip(base[r], ov[r]):
            assert np.array_equal(a, b)
