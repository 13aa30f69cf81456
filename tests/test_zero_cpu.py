"""ZeRO-1 (DistributedDataParallel(zero_stage=1)) on CPU gloo: reduce-scatter of padded buckets,
the optimizer step, the parameter gather and the consolidated optimizer state equal plain DDP
(bitwise at 2 ranks, where a sum has one order; to rounding at 4)."""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(37, 129)
        self.b = torch.nn.Linear(129, 65)
        self.c = torch.nn.Linear(65, 10)

    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))


def _worker(rank, world, port, zero, opt_name, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        torch.manual_seed(0)
        model = _Net()
        # tiny buckets: several buckets, each padded to 64 x world under ZeRO
        net = DistributedDataParallel(model, bucket_cap_mb=0.02, first_bucket_mb=0.005, zero_stage=zero)
        opt = FusedAdamW(model.parameters(), lr=1e-2, weight_decay=0.1) if opt_name == "adamw" else \
            FusedSGD(model.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-3)
        g = torch.Generator().manual_seed(rank + 11)
        for _ in range(3):
            x = torch.randn(8, 37, generator=g)
            loss = net(x).square().mean()
            loss.backward()
            opt.step()
            opt.zero_grad()
        sd = opt.state_dict()
        state = {k: {n: v.numpy().copy() for n, v in st.items() if torch.is_tensor(v)} for k, st in sd["state"].items()}
        params = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
        q.put((rank, "ok", (params, state, len(net.buckets), net.comm_plan()["zero_stage"])))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _run(world, zero, opt_name):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, zero, opt_name, q)) for r in range(world)]
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
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world,opt_name", [(2, "adamw"), (2, "sgd"), (4, "adamw")])
def test_zero1_equals_replicated_optimizer(world, opt_name):
    base = _run(world, 0, opt_name)
    z = _run(world, 1, opt_name)
    assert z[0][3] == 1 and base[0][3] == 0
    assert z[0][2] > 2  # really several buckets
    exact = world == 2
    for r in range(world):
        for n, v in base[0][0].items():
            if exact:
                assert np.array_equal(z[r][0][n], v), (r, n)
            else:
                np.testing.assert_allclose(z[r][0][n], v, rtol=1e-5, atol=1e-6)
        for k, st in base[0][1].items():
            for name, v in st.items():
                if exact:
                    assert np.array_equal(z[r][1][k][name], v), (r, k, name)
                else:
                    np.testing.assert_allclose(z[r][1][k][name], v, rtol=1e-5, atol=1e-7)
