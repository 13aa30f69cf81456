"""Sharded ZeRO-1 optimizer checkpoints on CPU gloo.

* optimizer-state bytes per rank are 1/world of the replicated state (compact shards);
* a 4-rank ZeRO-1 save writes every rank's shards as DCP chunks - no all-gather - and
  - reloads at 4 ranks (ZeRO) and continues bit-equal to the uninterrupted run,
  - reloads at 2 ranks (ZeRO, resharded) and at 2 ranks replicated with the saved state exactly,
  - its model part loads with stock `torch.distributed.checkpoint.load`.
"""
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


def _steps(net, opt, rank, k0, k1):
    losses = []
    for k in range(k0, k1):
        g = torch.Generator().manual_seed(1000 * k + rank)
        x = torch.randn(8, 37, generator=g)
        loss = net(x).square().mean()
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    return losses


def _worker(rank, world, port, mode, path, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
        from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import FlatShardedTensor
        from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict
        from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        zero = 1 if mode in ("save", "resume_zero", "reload_zero") else 0
        torch.manual_seed(0)
        model = _Net()
        net = DistributedDataParallel(model, bucket_cap_mb=0.02, first_bucket_mb=0.005, zero_stage=zero)
        opt = FusedAdamW(model.parameters(), lr=1e-2, weight_decay=0.1)
        out = {}
        if mode == "save":
            _steps(net, opt, rank, 0, 3)
            msd, osd = get_state_dict(model, opt)
            vals = [v for st in osd["state"].values() for v in st.values()]
            sharded = [v for v in vals if isinstance(v, FlatShardedTensor)]
            assert sharded, "ZeRO-1 optimizer state should be sharded"
            out["state_elems"] = sum(v.local_numel() for v in sharded)
            out["full_elems"] = sum(v.numel() for v in sharded)
            out["compact_bytes"] = sum(b.numel() * 4 for b in opt._bufs.values())
            dcp.save({"model": msd, "optim": osd, "step": 3}, path)
            out["params_at_save"] = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
            full = opt.state_dict()  # torch format (collective gather), for the comparisons
            out["state"] = {k: {n: v.numpy().copy() for n, v in st.items() if torch.is_tensor(v) and v.dim() > 0}
                            for k, st in full["state"].items()}
            out["losses"] = _steps(net, opt, rank, 3, 6)
        else:
            if mode != "resume_zero":
                # a fresh optimizer must be materialised to be a load target
                opt.init_state()
            msd, osd = get_state_dict(model, opt)
            sd = {"model": msd, "optim": osd, "step": 0}
            dcp.load(sd, path)
            set_state_dict(model, opt, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
            full = opt.state_dict()
            out["state"] = {k: {n: v.numpy().copy() for n, v in st.items() if torch.is_tensor(v) and v.dim() > 0}
                            for k, st in full["state"].items()}
            out["step"] = sd["step"]
            if mode == "resume_zero":
                out["losses"] = _steps(net, opt, rank, 3, 6)
        out["params"] = {n: p.detach().numpy().copy() for n, p in model.named_parameters()}
        q.put((rank, "ok", out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def _run(world, mode, path):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, path, q)) for r in range(world)]
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
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


def _same_state(a, b):
    assert set(a) == set(b)
    for k in a:
        for n in a[k]:
            assert np.array_equal(a[k][n], b[k][n]), (k, n)


def test_zero1_sharded_checkpoint_reshards(tmp_path):
    path = str(tmp_path / "ck")
    saved = _run(4, "save", path)
    s0 = saved[0]
    # 1/world of the optimizer state per rank (plus the 64 x world bucket padding)
    tot = sum(saved[r]["state_elems"] for r in range(4))
    assert tot == s0["full_elems"]
    for r in range(4):
        assert saved[r]["state_elems"] <= s0["full_elems"] / 4 * 1.15 + 64 * 4 * 6
        assert saved[r]["compact_bytes"] <= 2 * 4 * (s0["full_elems"] / 4 * 1.15 + 64 * 4 * 6)
    files = sorted(os.listdir(path))
    assert ".metadata" in files and all(f"__{r}_0.distcp" in files for r in range(4))

    # 4-rank ZeRO resume: bit-equal continuation
    res = _run(4, "resume_zero", path)
    for r in range(4):
        _same_state(res[r]["state"], s0["state"])
        assert res[r]["losses"] == saved[r]["losses"], (r, res[r]["losses"], saved[r]["losses"])
    # 2-rank ZeRO (resharded) and 2-rank replicated: the exact saved state and parameters
    for mode in ("reload_zero", "reload_repl"):
        got = _run(2, mode, path)
        for r in range(2):
            _same_state(got[r]["state"], s0["state"])
            for n, v in s0["params_at_save"].items():
                assert np.array_equal(got[r]["params"][n], v), (mode, r, n)
            assert got[r]["step"] == 3


def test_zero1_checkpoint_model_part_loads_with_stock_torch_dcp(tmp_path):
    import torch.distributed.checkpoint as tdcp

    path = str(tmp_path / "ck")
    saved = _run(2, "save", path)
    model = _Net()
    sd = {"model": model.state_dict()}
    tdcp.load(sd, checkpoint_id=path, no_dist=True)
    for n, v in saved[0]["params_at_save"].items():
        assert np.array_equal(sd["model"][n].numpy(), v), n
    # the optimizer state tensors keep the parameters' shapes (chunked on disk)
    md = tdcp.FileSystemReader(path).read_metadata()
    m = md.state_dict_metadata["optim.state.a.weight.exp_avg"]
    assert tuple(m.size) == (129, 37) and len(m.chunks) >= 2


def _per_rank_sharded_save(rank, world, path):
    """replicated=False: every rank writes its own items; one key is a FlatShardedTensor whose
    chunks are spread over both ranks, another a per-rank tensor with a rank-unique name."""
    import torch

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import FlatShardedTensor

    full = torch.arange(6 * 10, dtype=torch.float32).view(6, 10)
    ranges = [[(0, 25)], [(25, 60)]]
    flat = full.reshape(-1)
    local = [(a, flat[a:b].clone()) for a, b in ranges[rank]]
    sd = {"w": FlatShardedTensor((6, 10), torch.float32, local, ranges, rank),
          f"own_{rank}": torch.full((3,), float(rank))}
    dcp.save(sd, path, replicated=False)
    return True


def test_per_rank_metadata_merge_keeps_every_ranks_chunks(tmp_path):
    """Rank 0 merges the per-rank metadata of a replicated=False save: a key sharded over both
    ranks keeps the union of their chunk lists (dict.update kept only the last rank's)."""
    import torch

    from tests.mp_util import run
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    path = str(tmp_path / "ck")
    run(_per_rank_sharded_save, 2, path)
    md = dcp.read_metadata(path)
    assert len(md.state_dict_metadata["w"].chunks) >= 2
    sd = {"w": torch.zeros(6, 10), "own_0": torch.zeros(3), "own_1": torch.zeros(3)}
    dcp.load(sd, path)
    assert torch.equal(sd["w"], torch.arange(60, dtype=torch.float32).view(6, 10))
    assert torch.equal(sd["own_1"], torch.ones(3)) and torch.equal(sd["own_0"], torch.zeros(3))
