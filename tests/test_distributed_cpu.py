"""Multi-process gloo tests: DDP equivalence with torch DDP, sampler contract, sharded DCP
save/load with dedup and resharding across world sizes."""
import os

import torch
import torch.distributed as dist

from tests import mp_util


def _ddp_equiv(rank, world, seed, engine="native"):
    os.environ["RTDC_DDP_ENGINE"] = engine
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(seed)
    base = torch.nn.Sequential(torch.nn.Linear(20, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64), torch.nn.ReLU(),
                               torch.nn.Linear(64, 5))
    import copy

    ours_m = copy.deepcopy(base)
    ref_m = copy.deepcopy(base)
    ours = DistributedDataParallel(ours_m, bucket_cap_mb=0.01, first_bucket_mb=0.005)
    ref = torch.nn.parallel.DistributedDataParallel(ref_m)
    assert len(ours.buckets) > 1
    assert (ours._engine is not None) == (engine == "native")
    opt_o = torch.optim.SGD(ours.parameters(), lr=0.1, momentum=0.9)
    opt_r = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(3):
        x = torch.randn(8, 20, generator=g)
        y = torch.randint(0, 5, (8,), generator=g)
        for m, opt in ((ours, opt_o), (ref, opt_r)):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
    diffs = [float((a - b).abs().max()) for a, b in zip(ours_m.parameters(), ref_m.parameters())]
    return max(diffs)


def test_ddp_matches_torch_ddp():
    out = mp_util.run(_ddp_equiv, 2, 0)
    assert max(out) < 1e-5, out


def test_ddp_python_engine_matches_torch_ddp():
    out = mp_util.run(_ddp_equiv, 2, 1, "python")
    assert max(out) < 1e-5, out


def _ddp_deferred_tail(rank, world, opt_kind, piece_mb=32.0, comm="fp32"):
    """defer_tail_to_optimizer: backward returns with the last bucket's all-reduce pending; the
    fused optimizer steps the rest first and waits for it before the last slice - the same
    parameters as torch DDP + torch optimizer after several steps."""
    import copy

    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(7)
    base = torch.nn.Sequential(torch.nn.Linear(20, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64), torch.nn.ReLU(),
                               torch.nn.Linear(64, 5))
    ours_m, ref_m = copy.deepcopy(base), copy.deepcopy(base)
    ours = DistributedDataParallel(ours_m, bucket_cap_mb=0.01, first_bucket_mb=0.005, defer_tail_to_optimizer=True,
                                   tail_piece_mb=piece_mb, grad_comm_dtype=comm)
    ref = torch.nn.parallel.DistributedDataParallel(ref_m)
    assert len(ours.buckets) > 1
    if opt_kind == "adamw":
        opt_o = FusedAdamW(ours.parameters(), lr=1e-2, weight_decay=0.1)
        opt_r = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1)
    else:
        opt_o = FusedSGD(ours.parameters(), lr=0.1, momentum=0.9)
        opt_r = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(100 + rank)
    pending = []
    for _ in range(4):
        x = torch.randn(8, 20, generator=g)
        y = torch.randint(0, 5, (8,), generator=g)
        for m, opt in ((ours, opt_o), (ref, opt_r)):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            if m is ours:
                pending.append(len(ours.space.pending_tail) if ours.space.pending_tail else 0)
            opt.step()
        assert ours.space.pending_tail is None
    assert all(pending), pending
    err = max(float((a - b).abs().max()) for a, b in zip(ours_m.parameters(), ref_m.parameters()))
    return err, max(pending)


def test_ddp_deferred_tail_matches_torch():
    for kind in ("sgd", "adamw"):
        out = mp_util.run(_ddp_deferred_tail, 2, kind)
        assert max(e for e, _ in out) < 1e-5, (kind, out)
        assert all(n == 1 for _, n in out)  # the small tail: one collective


def test_ddp_tail_pieces_pipelined_into_optimizer_match_torch():
    """The deferred last bucket as several collectives (tail_piece_mb): the optimizer waits for
    and updates piece by piece (chunks cut at piece boundaries) - same parameters as torch DDP;
    with bf16 communication the same up to the bf16 rounding of the gradients."""
    for kind in ("sgd", "adamw"):
        out = mp_util.run(_ddp_deferred_tail, 2, kind, 0.002)
        assert max(e for e, _ in out) < 1e-5, (kind, out)
        assert all(n >= 3 for _, n in out), out
    out = mp_util.run(_ddp_deferred_tail, 2, "sgd", 0.002, "bf16")
    assert max(e for e, _ in out) < 5e-3 and all(n >= 2 for _, n in out), out


def _ddp_unused(rank, world):
    """A parameter without a gradient in a step contributes zeros (in-place gradient mode)."""
    from ray_torch_distributed_checkpoint_amd.optim import FusedSGD
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = torch.nn.ModuleDict({"a": torch.nn.Linear(8, 8), "b": torch.nn.Linear(8, 8)})

    class Net(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, x, use_b):
            y = self.m["a"](x)
            return self.m["b"](y) if use_b else y

    net = DistributedDataParallel(Net(m), bucket_cap_mb=0.0005, first_bucket_mb=0.0002)
    opt = FusedSGD(net.parameters(), lr=0.1)
    x = torch.randn(4, 8) * (rank + 1)
    net(x, True).sum().backward()
    opt.step()
    opt.zero_grad()
    w_before = m["b"].weight.detach().clone()
    net(x, False).sum().backward()
    gb = m["b"].weight.grad
    ok = gb is None or float(gb.abs().max()) == 0.0
    opt.step()
    return ok and torch.equal(w_before, m["b"].weight.detach())


def test_ddp_unused_parameter_zero_grad():
    out = mp_util.run(_ddp_unused, 2)
    assert all(out), out


def _sampler(rank, world):
    from torch.utils.data.distributed import DistributedSampler as TorchDS

    from ray_torch_distributed_checkpoint_amd.parallel.sampler import DistributedSampler

    ds = list(range(103))
    ours = DistributedSampler(ds, shuffle=True, seed=3)
    ref = TorchDS(ds, shuffle=True, seed=3)
    ok = True
    for ep in range(3):
        ours.set_epoch(ep)
        ref.set_epoch(ep)
        ok &= list(iter(ours)) == list(iter(ref))
    ours.start_index = 10
    ok &= list(iter(ours)) == list(iter(ref))[10:]
    return ok


def test_sampler_contract():
    assert all(mp_util.run(_sampler, 3))


def _dcp_save(rank, world, path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    torch.manual_seed(0)  # identical (replicated) state on every rank
    sd = {"model": {f"w{i}": torch.randn(50 + i, 7) for i in range(9)}, "step": 11, "hp": {"lr": 0.5}}
    h = dcp.async_save(sd, path)
    h.result()
    files = sorted(f for f in os.listdir(path) if f.endswith(".distcp"))
    return files, h.nbytes


def _dcp_load(rank, world, path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    torch.manual_seed(0)
    ref = {f"w{i}": torch.randn(50 + i, 7) for i in range(9)}
    sd = {"model": {f"w{i}": torch.zeros(50 + i, 7) for i in range(9)}, "step": 0, "hp": {"lr": 0.0}}
    dcp.load(sd, path)
    ok = all(torch.equal(sd["model"][k], ref[k]) for k in ref)
    return ok and sd["step"] == 11 and sd["hp"]["lr"] == 0.5


def test_dcp_sharded_save_dedup_and_reshard(tmp_path):
    path = str(tmp_path / "ck")
    out = mp_util.run(_dcp_save, 4, path)
    files = out[0][0]
    assert files == [f"__{r}_0.distcp" for r in range(4)]  # every rank wrote a shard
    total = sum(o[1] for o in out)
    expect = sum((50 + i) * 7 * 4 for i in range(9))
    assert expect <= total < expect + 4096  # each tensor written exactly once (dedup)
    assert all(mp_util.run(_dcp_load, 2, path))  # resharded restore at a different world size
    assert all(mp_util.run(_dcp_load, 3, path))
    # and a single process / stock torch can read it
    import torch.distributed.checkpoint as tdcp

    sd = {"model": {f"w{i}": torch.zeros(50 + i, 7) for i in range(9)}, "step": 0, "hp": {"lr": 0.0}}
    tdcp.load(sd, checkpoint_id=path)
    torch.manual_seed(0)
    assert torch.equal(sd["model"]["w0"], torch.randn(50, 7))


def _ddp_plan_mismatch(rank, world):
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    m = torch.nn.Linear(8, 8 if rank == 0 else 9)  # rank 1 built a different model
    try:
        DistributedDataParallel(m)
    except RuntimeError as e:
        return "differs across ranks" in str(e)
    return False


def test_ddp_detects_mismatched_models():
    assert all(mp_util.run(_ddp_plan_mismatch, 2))


def _ddp_seq_check(rank, world):
    os.environ["RTDC_COLLECTIVE_CHECK"] = "1"
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    net = DistributedDataParallel(torch.nn.Linear(8, 4))
    for _ in range(3):
        net(torch.randn(2, 8)).sum().backward()
    return net._steps == 3


def test_ddp_collective_sequence_check():
    assert all(mp_util.run(_ddp_seq_check, 2))


def _ddp_tail_split_mismatch(rank, world):
    """Ranks that disagree on the deferred tail's piece size would issue different numbers of
    collectives: the plan fingerprint must catch it before the first one."""
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 64))
    try:
        DistributedDataParallel(m, defer_tail_to_optimizer=True, tail_piece_mb=0.01 if rank == 0 else 0.02)
    except RuntimeError as e:
        return "differs across ranks" in str(e)
    return False


def test_ddp_detects_mismatched_tail_split():
    assert all(mp_util.run(_ddp_tail_split_mismatch, 2))


def _ddp_rewrap_clears_skip_ptr(rank, world):
    """A re-wrap of the same model (same flat space) without P2P must not keep the previous
    communicator's error word as the optimizer's skip flag."""
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = torch.nn.Linear(16, 16)
    a = DistributedDataParallel(m)
    a.space.skip_ptr = 0xDEAD000  # what a P2P wrap leaves behind
    a.detach()
    b = DistributedDataParallel(m, p2p_max_kb=0.0)
    return b.space is a.space and b.space.skip_ptr == 0


def test_ddp_rewrap_without_p2p_clears_skip_ptr():
    assert all(mp_util.run(_ddp_rewrap_clears_skip_ptr, 2))
