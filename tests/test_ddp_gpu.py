"""Data-parallel gradient engine on the GPU (bf16 GPT-2-tiny on the native kernels).

* Multi-process DDP gradients (flat buckets, C++ engine, fp32 or bf16 communication) equal
  the single-process gradient of the concatenated batch.  With >= 2 GPUs this runs over RCCL
  (one rank per GPU); on a 1-GPU box the same engine runs with two gloo ranks sharing cuda:0,
  which exercises the GPU side of the engine (bf16 rounding kernel, side-stream widening,
  event ordering) without RCCL.
* The bf16-workload trainer loop on one GPU: kill at step K, restart, bit-equal losses.
"""
import json
import os
import socket
import sys
import traceback

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
B, T = 2, 64


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(dev):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config.named("gpt2-tiny")).to(dev)


def _batch(world, dev):
    g = torch.Generator().manual_seed(7)
    return torch.randint(0, 1000, (world * B, T + 1), generator=g).to(dev)


def _worker(rank, world, port, backend, comm_dtype, q, force=False):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        ngpu = torch.cuda.device_count()
        dev = torch.device("cuda", rank % ngpu)
        torch.cuda.set_device(dev)
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        model = _model(dev)
        net = DistributedDataParallel(model, grad_comm_dtype=comm_dtype, bucket_cap_mb=0.25, first_bucket_mb=0.05,
                                      force_collectives=force)
        data = _batch(world, dev)[rank * B:(rank + 1) * B]
        for _ in range(2):  # second step: buckets reused, fresh-gradient mode
            net.space.zero_grad(set_to_none=True)
            loss = net(data[:, :-1], data[:, 1:])
            loss.backward()
        torch.cuda.synchronize()
        # numpy, not tensors: a torch.multiprocessing queue would pass shared-memory fds that
        # die with this process
        grads = {n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()}
        q.put((rank, "ok", (grads, len(net.buckets), net.comm_plan())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _run(world, backend, comm_dtype, force=False):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, comm_dtype, q, force)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, st, v = q.get(timeout=240)
            assert st == "ok", v
            out[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


def _reference(world):
    dev = torch.device("cuda", 0)
    model = _model(dev)
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    FlatParamSpace(list(reversed(list(model.parameters()))))  # same flat-gradient path as DDP
    data = _batch(world, dev)
    loss = model(data[:, :-1], data[:, 1:])
    loss.backward()
    return {n: p.grad.detach().float().cpu() for n, p in model.named_parameters()}


def _check(out, ref, tol):
    g0 = {n: torch.from_numpy(v) for n, v in out[0][0].items()}
    for r in out:  # every rank holds the same averaged gradient
        for n in g0:
            assert torch.equal(torch.from_numpy(out[r][0][n]), g0[n]), f"rank {r} differs on {n}"
    assert out[0][1] > 3  # really bucketed
    for n, v in ref.items():
        err = (g0[n] - v).norm() / v.norm().clamp_min(1e-12)
        assert err < tol, f"{n}: relative error {err:.3e}"


@pytest.mark.parametrize("comm_dtype,tol", [("fp32", 5e-3), ("bf16", 5e-3)])
def test_ddp_gloo_two_ranks_on_gpu_matches_concatenated_batch(comm_dtype, tol):
    out = _run(2, "gloo", comm_dtype)
    assert out[0][2]["grad_comm_dtype"] == comm_dtype
    _check(out, _reference(2), tol)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL DDP needs >= 2 GPUs (one rank per GPU)")
@pytest.mark.parametrize("comm_dtype,tol", [("fp32", 5e-3), ("bf16", 5e-3)])
def test_ddp_rccl_matches_concatenated_batch(comm_dtype, tol):
    world = min(torch.cuda.device_count(), 4)
    out = _run(world, "nccl", comm_dtype)
    _check(out, _reference(world), tol)


@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_ddp_rccl_one_rank_forced_collectives(comm_dtype):
    """RCCL on a one-GPU box: a 1-rank nccl group with force_collectives runs the real multi-GPU
    path - native bucket engine, c10d RCCL all-reduce (AVG) of every bucket on its side stream,
    bf16 rounding/widening - and must leave exactly the single-process gradient (fp32: an
    all-reduce over one rank is the identity) or its bf16 rounding."""
    out = _run(1, "nccl", comm_dtype, force=True)
    plan = out[0][2]
    assert plan["engine"] == "native" and plan["grad_comm_dtype"] == comm_dtype and out[0][1] > 3
    ref = _reference(1)
    for n, v in ref.items():
        g = torch.from_numpy(out[0][0][n])
        if comm_dtype == "fp32":
            assert torch.equal(g, v), n
        else:
            assert torch.equal(g, v.to(torch.bfloat16).float()), n


def _losses(path):
    out = {}
    for line in open(os.path.join(path, "result.json")):
        row = json.loads(line)
        for i, v in enumerate(reversed(row["losses"])):
            k = row["step"] - i
            assert out.get(k, v) == v
            out[k] = v
    return out


@pytest.mark.parametrize("model", ["gpt2-tiny", "resnet18-tiny"])
def test_workload_trainer_kill_restart_bit_equal_gpu(tmp_path, monkeypatch, model):
    from ray_torch_distributed_checkpoint_amd import workloads as W

    for k in ("RTDC_FAIL_AT_STEP", "RTDC_HANG_AT_STEP", "RTDC_FORCE_CPU"):
        monkeypatch.delenv(k, raising=False)
    kw = dict(steps=6, num_workers=1, use_gpu=True, ckpt_every_n_steps=2, verbose=0)
    a = W.train_workload(model, checkpoint_storage_path=str(tmp_path / "a"), **kw)
    monkeypatch.setenv("RTDC_FAIL_AT_STEP", "3")
    b = W.train_workload(model, checkpoint_storage_path=str(tmp_path / "b"), max_failures=1, **kw)
    la, lb = _losses(a.path), _losses(b.path)
    assert sorted(la) == list(range(1, 7))
    assert la == lb
    files = sorted(os.listdir(b.checkpoint.path))
    assert files == [".metadata", "__0_0.distcp"]


def _zero_worker(rank, world, port, zero, q):
    try:
        import numpy as np  # noqa: F401
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        model = _model(dev)
        net = DistributedDataParallel(model, bucket_cap_mb=0.25, first_bucket_mb=0.05, zero_stage=zero)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)
        data = _batch(world, dev)[rank * B:(rank + 1) * B]
        for _ in range(3):
            net(data[:, :-1], data[:, 1:]).backward()
            opt.step()
            opt.zero_grad()
        sd = opt.state_dict()  # ZeRO: consolidated (collective)
        torch.cuda.synchronize()
        params = {n: p.detach().float().cpu().numpy() for n, p in model.named_parameters()}
        shadows = float(sum(float(getattr(p, "_rtdc_shadow", p).float().sum()) for p in model.parameters()))
        state = {k: {n: v.float().cpu().numpy() for n, v in st.items() if torch.is_tensor(v) and v.dim() > 0}
                 for k, st in sd["state"].items()}
        q.put((rank, "ok", (params, state, shadows)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def test_zero1_native_optimizer_on_gpu_equals_replicated():
    """ZeRO-1 with the native engine and the fused AdamW on device (owned-shard chunk tables,
    fp32 parameter all-gather + bf16 shadow rebuild, consolidated state), two ranks on cuda:0
    over gloo: bitwise equal to the replicated optimizer."""
    import numpy as np
    import torch.multiprocessing as mp

    def run(zero):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_zero_worker, args=(r, 2, port, zero, q)) for r in range(2)]
        for p in ps:
            p.start()
        out = {}
        try:
            for _ in range(2):
                r, st, v = q.get(timeout=240)
                assert st == "ok", v
                out[r] = v
        finally:
            for p in ps:
                p.join(timeout=60)
                if p.is_alive():
                    p.kill()
        return out

    base, z = run(0), run(1)
    for r in range(2):
        for n, v in base[0][0].items():
            assert np.array_equal(z[r][0][n], v), (r, n)
        for k, st in base[0][1].items():
            for name, v in st.items():
                assert np.array_equal(z[r][1][k][name], v), (r, k, name)
        assert z[r][2] == base[0][2]  # bf16 compute shadows rebuilt identically
