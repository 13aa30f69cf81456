"""Simulated ZeRO-1 shards (checkpoint/sharded.py simulated_zero_optimizer_state): W
single-process saves, one per simulated rank, each writing only that rank's owner chunks of
the optimizer state (and its dedup share of the parameters), together form a complete DCP
checkpoint that a replicated optimizer loads back exactly - the 1/W per-rank write an 8-GPU
ZeRO-1 job does, measured by one process (bench.py --simulate-world 8 --zero 1)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _model_opt(seed):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    torch.manual_seed(seed)
    model = GPT2(GPT2Config(vocab_size=256, n_positions=64, n_embd=64, n_layer=2, n_head=2))
    opt = FusedAdamW(model.parameters(), lr=1e-3)
    idx = torch.randint(0, 256, (2, 33))
    model(idx[:, :-1], idx[:, 1:]).backward()
    opt.step()
    return model, opt


def test_simulated_zero_shards_cover_the_state_and_restore(tmp_path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import simulated_zero_optimizer_state
    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict

    W = 4
    model, opt = _model_opt(0)
    path = str(tmp_path / "ck")
    sizes = []
    for r in range(W):
        osd = simulated_zero_optimizer_state(model, opt, W, r, bucket_cap_mb=0.01)
        h = dcp.save({"model": get_state_dict(model, None)[0], "optim": osd}, path, simulate=(W, r))
        sizes.append(h.nbytes)
    # every rank writes about 1/W of the bytes (owner shards), none writes everything
    total = sum(sizes)
    assert max(sizes) < 0.5 * total
    # a fresh replicated model/optimizer restores the full state
    model2, opt2 = _model_opt(1)
    msd, osd = get_state_dict(model2, opt2)
    sd = {"model": msd, "optim": osd}
    dcp.load(sd, path)
    set_state_dict(model2, opt2, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
    for (n, p), (_, q) in zip(model.named_parameters(), model2.named_parameters()):
        assert torch.equal(p, q), n
    a, b = get_state_dict(model, opt)[1], get_state_dict(model2, opt2)[1]
    for k, st in a["state"].items():
        for kk, v in st.items():
            assert torch.equal(v, b["state"][k][kk]), (k, kk)
    # a simulated rank's share read back in place by the simulated path
    osd3 = simulated_zero_optimizer_state(model2, opt2, W, 2, bucket_cap_mb=0.01)
    for st in osd3["state"].values():
        for v in st.values():
            if hasattr(v, "local"):
                for _, t in v.local:
                    t.zero_()
    dcp.load({"model": get_state_dict(model2, None)[0], "optim": osd3}, path, simulate=(W, 2))
    b2 = get_state_dict(model2, opt2)[1]
    for k, st in a["state"].items():
        for kk, v in st.items():
            assert torch.equal(v, b2["state"][k][kk]), (k, kk)


def test_simulated_checkpoint_is_refused_by_a_real_load(tmp_path):
    import pytest

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict

    model, opt = _model_opt(0)
    path = str(tmp_path / "ck")
    dcp.save({"model": get_state_dict(model, None)[0]}, path, simulate=(4, 1))
    with pytest.raises(ValueError, match="simulated"):
        dcp.load({"model": get_state_dict(model, None)[0]}, path)


def _real_zero_layout(rank, world, dtype):
    from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import simulated_zero_ranges
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    model = GPT2(GPT2Config(vocab_size=250, n_positions=64, n_embd=64, n_layer=3, n_head=2))
    net = DistributedDataParallel(model, bucket_cap_mb=0.02, first_bucket_mb=0.005, zero_stage=1,
                                  grad_comm_dtype=dtype)
    sp = net.space
    numels = [s.numel for s in sp.segments]
    offs, ranges = simulated_zero_ranges(numels, world, 0.02, 0.005, grad_comm_dtype=dtype)
    real = [(a, b) for a, b in sp.zero.owned if a < b]
    return offs == [s.offset for s in sp.segments] and ranges[rank] == real and len(net.buckets) > 2


def test_simulated_zero_ranges_are_the_real_ddp_layout():
    """the simulated per-rank ZeRO-1 shard must be the one a real W-rank
    DistributedDataParallel(zero_stage=1) owns - bucket-end padding to 64 x world, caps in
    communicated bytes - so the single-process per-rank save/restore figures are pinned to it."""
    from tests import mp_util

    for dtype in ("fp32", "bf16"):
        assert all(mp_util.run(_real_zero_layout, 4, dtype))
