"""Exact resume at production size (GPT-2-small, fused AdamW, 1.49 GB train state) through the
workload's own save / restore path (workloads._train_state -> dcp.async_save -> restore):

* every tensor of the restored train state (fp32 masters, AdamW moments, step, data position,
  RNG) is bitwise the live state at the save point, while training continued during the drain;
* the next optimizer steps after the restore produce bit-identical losses to the uninterrupted
  run (R/my_ray_module.py:177-205 save inside the loop, :253-264 restore; product path
  profiles/product_path_gpt2_r6.md).

The tiny-model resume tests (tests/test_ddp_gpu.py, tests/test_multigpu_gpu.py) keep every
tensor below the snapshot / engine chunk sizes; this one crosses them."""
import hashlib
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu


def _sha(t):
    return hashlib.sha1(t.detach().reshape(-1).contiguous().cpu().view(torch.uint8).numpy().tobytes()).hexdigest()


def _digests(model, opt):
    out = {"p." + n: _sha(p) for n, p in model.named_parameters()}
    for k, st in opt.state_dict()["state"].items():
        for n, v in st.items():
            out[f"o.{k}.{n}"] = _sha(v) if torch.is_tensor(v) else repr(v)
    return out


def _setup(W, dev, B):
    cfg = W.WorkloadConfig(model="gpt2-small", steps=8, batch_size_per_worker=B, seed=1234)
    torch.manual_seed(cfg.seed)
    wl = W.build(cfg, dev)
    stream = W.ShardedStream(wl.data, wl.batch, 1, 0, cfg.seed, dev)
    return wl, stream


def _step(wl, stream, probe=None):
    x, y = stream.next()
    loss = wl.loss_fn(wl.model, x, y)
    loss.backward()
    if probe is not None:  # the gradients this step's update reads
        from ray_torch_distributed_checkpoint_amd.ops.gemm import flush_wgrads

        flush_wgrads()
        torch.cuda.synchronize()
        probe["grad"] = {n: _sha(p.grad) for n, p in wl.model.named_parameters() if p.grad is not None}
    wl.optimizer.step()
    wl.optimizer.zero_grad(set_to_none=True)
    if probe is not None:
        torch.cuda.synchronize()
        probe["after"] = _digests(wl.model, wl.optimizer)
    return loss.detach()


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_gpt2_small_exact_resume_bitwise(tmp_path, mode):
    from ray_torch_distributed_checkpoint_amd import workloads as W
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.train.checkpoint import Checkpoint

    dev = torch.device("cuda", 0)
    B = 4
    wl, stream = _setup(W, dev, B)
    for _ in range(3):
        _step(wl, stream)
    torch.cuda.synchronize()
    saved = _digests(wl.model, wl.optimizer)
    saved_pos = (stream.epoch, stream.pos)
    state = W._train_state(wl.model, wl.optimizer, stream, 3, W._rng_blob(dev))
    path = str(tmp_path / "ck")
    live = {}
    if mode == "async":
        h = dcp.async_save(state, path)
        # training continues while the engine drains
        ref = [_step(wl, stream, live)] + [_step(wl, stream) for _ in range(2)]
        h.result()  # durable + .metadata committed
    else:
        dcp.save(state, path)
        ref = [_step(wl, stream, live)] + [_step(wl, stream) for _ in range(2)]
    ref = [float(v) for v in ref]

    wl2, stream2 = _setup(W, dev, B)
    start = W.restore(wl2.model, wl2.optimizer, stream2, Checkpoint.from_directory(path), "exact", dev, 0)
    torch.cuda.synchronize()
    assert start == 3 and (stream2.epoch, stream2.pos) == saved_pos
    got = _digests(wl2.model, wl2.optimizer)
    bad = sorted(k for k in saved if got.get(k) != saved[k])
    assert not bad, f"{len(bad)} of {len(saved)} restored entries differ, e.g. {bad[:6]}"
    res = {}
    out = [float(_step(wl2, stream2, res))] + [float(_step(wl2, stream2)) for _ in range(2)]
    gbad = sorted(k for k in live["grad"] if res["grad"].get(k) != live["grad"][k])
    assert not gbad, f"first step after the restore: {len(gbad)} gradients differ, e.g. {gbad[:6]}"
    abad = sorted(k for k in live["after"] if res["after"].get(k) != live["after"][k])
    assert not abad, f"first update after the restore: {len(abad)} of {len(live['after'])} entries differ, e.g. {abad[:8]}"
    assert out == ref, (out, ref)
