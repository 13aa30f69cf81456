"""BASELINE config 5 on the GPU: kill at step K, restore, bit-equal continuation.

* toy flow (my_ray_module, native fp32 MFMA kernels + Philox dropout + fused SGD): a worker
  is SIGKILLed at its 2nd report, the supervisor restarts it from the latest committed
  checkpoint and every later epoch's metrics equal the uninterrupted run bit for bit;
* GPT-2 (bf16 kernels, flash attention, deterministic embedding backward, fused AdamW):
  a DCP checkpoint of model + optimizer + Philox state taken at step K, restored into a
  fresh model, reproduces the next steps' losses bitwise.
"""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_toy_flow_kill_and_exact_resume_gpu(tmp_path, monkeypatch):
    import my_ray_module as m

    monkeypatch.setenv("RTDC_FMNIST_TRAIN", "4000")
    monkeypatch.setenv("RTDC_FMNIST_TEST", "1000")
    monkeypatch.delenv("RTDC_FORCE_CPU", raising=False)
    a = m.train_fashion_mnist(num_workers=1, use_gpu=True, epochs=3, checkpoint_storage_path=str(tmp_path / "a"),
                              seed=11, resume_mode="exact")
    monkeypatch.setenv("RTDC_FAIL_AT_REPORT", "2")
    b = m.train_fashion_mnist(num_workers=1, use_gpu=True, epochs=3, checkpoint_storage_path=str(tmp_path / "b"),
                              seed=11, resume_mode="exact", max_failures=1)
    rows_a = [json.loads(l) for l in open(os.path.join(a.path, "result.json"))]
    rows_b = [json.loads(l) for l in open(os.path.join(b.path, "result.json"))]
    assert len(rows_a) == len(rows_b) == 3
    for ra, rb in zip(rows_a, rows_b):
        assert ra["val_loss"] == rb["val_loss"] and ra["accuracy"] == rb["accuracy"], (ra, rb)


def test_gpt2_checkpoint_resume_bit_equal(tmp_path):
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    cfg = GPT2Config.named("gpt2-tiny")
    data = torch.randint(0, cfg.vocab_size, (8, 4, 129), device="cuda",
                         generator=torch.Generator(device="cuda").manual_seed(3))

    def make():
        torch.manual_seed(0)
        model = GPT2(cfg).cuda()
        return model, FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)

    def step(model, opt, i):
        loss = model(data[i, :, :-1], data[i, :, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss.detach().clone()

    K = 4
    model, opt = make()
    ops.manual_seed(1234)
    for i in range(K):
        step(model, opt, i)
    msd, osd = get_state_dict(model, opt)
    dcp.save({"model": msd, "optim": osd, "philox": ops.default_stream().state_dict()}, str(tmp_path / "ck"))
    ref = [step(model, opt, i) for i in range(K, 8)]

    model2, opt2 = make()
    ops.manual_seed(999)  # restored below
    msd2, osd2 = get_state_dict(model2, opt2)  # load targets, optimizer state materialised
    sd = {"model": msd2, "optim": osd2, "philox": ops.default_stream().state_dict()}
    dcp.load(sd, str(tmp_path / "ck"))
    set_state_dict(model2, opt2, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
    ops.default_stream().load_state_dict(sd["philox"])
    got = [step(model2, opt2, i) for i in range(K, 8)]
    for r, g in zip(ref, got):
        assert torch.equal(r, g), (ref, got)


def test_toy_hipgraph_step_equals_eager_gpu(tmp_path, monkeypatch):
    """The captured toy step (one hipGraph launch per batch) trains bit-identically to the
    eager native step: same kernels, same Philox dropout counters."""
    import my_ray_module as m

    monkeypatch.setenv("RTDC_FMNIST_TRAIN", "2048")
    monkeypatch.setenv("RTDC_FMNIST_TEST", "512")
    monkeypatch.delenv("RTDC_FORCE_CPU", raising=False)
    kw = dict(num_workers=1, use_gpu=True, epochs=2, seed=5, resume_mode="exact")
    g = m.train_fashion_mnist(checkpoint_storage_path=str(tmp_path / "g"), hipgraph=True, **kw)
    e = m.train_fashion_mnist(checkpoint_storage_path=str(tmp_path / "e"), hipgraph=False, **kw)
    rows_g = [json.loads(l) for l in open(os.path.join(g.path, "result.json"))]
    rows_e = [json.loads(l) for l in open(os.path.join(e.path, "result.json"))]
    for rg, re_ in zip(rows_g, rows_e):
        assert rg["val_loss"] == re_["val_loss"] and rg["accuracy"] == re_["accuracy"], (rg, re_)


def test_eval_device_pipeline_matches_numpy_path_gpu(tmp_path):
    """map_batches with the GPU predictor (pinned double buffer, one D2H) returns exactly the
    per-batch numpy predictor's outputs, in order, for the 10k-row eval set."""
    import time

    import numpy as np

    import my_ray_module as m
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave
    from ray_torch_distributed_checkpoint_amd.train import Checkpoint

    torch.manual_seed(3)
    net = m.NeuralNetwork()
    torchsave.save({"epoch": 0, "model_state_dict": net.state_dict()}, str(tmp_path / "best_model.pt"))
    ck = Checkpoint.from_directory(str(tmp_path))
    ds = m.get_dataloaders(batch_size=512, val_only=True, as_ray_ds=True)
    pred = m.TorchPredictor(checkpoint=ck)
    out = ds.map_batches(pred, batch_size=512, concurrency=1, num_gpus=1)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = ds.map_batches(pred, batch_size=512, concurrency=1, num_gpus=1).to_numpy()
    dt = time.perf_counter() - t0
    ref = [pred(b) for b in ds.iter_batches(512)]
    ref_logits = np.concatenate([r["logits"] for r in ref])
    assert out["logits"].shape == (ds.count(), 10)
    np.testing.assert_array_equal(out["logits"], ref_logits)
    np.testing.assert_array_equal(out["predicted_values"], np.concatenate([r["predicted_values"] for r in ref]))
    print(f"eval pass over {ds.count()} rows: {dt * 1e3:.1f} ms")
    assert dt < 0.05  # measured 10 ms on one MI355X (<= 50 ms for the 10k-row pass)
