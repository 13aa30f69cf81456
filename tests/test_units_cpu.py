"""CPU unit tests: reference op paths, models, flat parameter space, fused optimizers (CPU path),
columnar dataset, storage/retention helpers, config surface, build entry."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def test_gpt2_cpu_forward_backward_and_param_count():
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    assert GPT2(GPT2Config.named("gpt2-small")).num_params() == 124_439_808
    cfg = GPT2Config.named("gpt2-tiny")
    m = GPT2(cfg)
    idx = torch.randint(0, cfg.vocab_size, (2, 32))
    loss = m(idx, idx)
    loss.backward()
    assert torch.isfinite(loss) and m.wte.grad is not None and m.wte.grad[cfg.vocab_size:].abs().sum() == 0
    logits = m(idx)
    assert logits.shape == (2, 32, cfg.vocab_size)


def test_toy_mlp_matches_reference_structure():
    from ray_torch_distributed_checkpoint_amd.models import NeuralNetwork

    m = NeuralNetwork()
    ref = torch.nn.Sequential(torch.nn.Linear(784, 512), torch.nn.ReLU(), torch.nn.Dropout(0.25),
                              torch.nn.Linear(512, 512), torch.nn.ReLU(), torch.nn.Dropout(0.25),
                              torch.nn.Linear(512, 10), torch.nn.ReLU())
    keys = ["linear_relu_stack." + k for k in ref.state_dict()]
    assert list(m.state_dict()) == keys
    assert sum(p.numel() for p in m.parameters()) == 669_706
    m.eval()
    ref.load_state_dict({k.split(".", 1)[1]: v for k, v in m.state_dict().items()})
    ref.eval()
    x = torch.randn(4, 1, 28, 28)
    assert torch.allclose(m(x), ref(x.flatten(1)))


def test_attention_ref_gqa_equals_mha_when_repeated():
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    B, T, H, Dh = 2, 16, 4, 8
    q = torch.randn(B, T, H * Dh)
    kv = torch.randn(B, T, 2 * 2 * Dh)
    out_gqa = causal_attention_ref(torch.cat([q, kv], -1), B, T, H, 2, Dh)
    k, v = kv.split(2 * Dh, -1)
    k4 = k.view(B, T, 2, Dh).repeat_interleave(2, dim=2).reshape(B, T, H * Dh)
    v4 = v.view(B, T, 2, Dh).repeat_interleave(2, dim=2).reshape(B, T, H * Dh)
    out_mha = causal_attention_ref(torch.cat([q, k4, v4], -1), B, T, H, H, Dh)
    assert torch.allclose(out_gqa, out_mha, atol=1e-6)


def test_flat_param_space_and_cpu_optimizers_match_torch():
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD

    for kind in ("adamw", "sgd"):
        torch.manual_seed(0)
        ps = [torch.randn(7, 5, requires_grad=True), torch.randn(3, requires_grad=True)]
        qs = [p.detach().clone().requires_grad_(True) for p in ps]
        opt = FusedAdamW(ps, lr=0.01, weight_decay=0.1) if kind == "adamw" else FusedSGD(ps, lr=0.01, momentum=0.9)
        ref = (torch.optim.AdamW(qs, lr=0.01, weight_decay=0.1) if kind == "adamw"
               else torch.optim.SGD(qs, lr=0.01, momentum=0.9))
        for _ in range(3):
            for p, q in zip(ps, qs):
                g = torch.randn_like(p)
                p.grad, q.grad = g.clone(), g.clone()
            opt.step()
            ref.step()
        for p, q in zip(ps, qs):
            assert torch.allclose(p, q, atol=1e-6)
        # torch-compatible state_dict round trip
        sd = opt.state_dict()
        assert set(sd["state"][0]) >= ({"exp_avg", "exp_avg_sq", "step"} if kind == "adamw" else {"momentum_buffer"})


def test_flat_param_space_views():
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    ps = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(70))]
    vals = [p.detach().clone() for p in ps]
    sp = FlatParamSpace(ps)
    # a space built while a parameter holds a gradient keeps the accumulate views
    q = [torch.nn.Parameter(torch.randn(4)), torch.nn.Parameter(torch.randn(6))]
    q[0].grad = torch.ones(4)
    sq = FlatParamSpace(q)
    assert not sq.fresh and all(p.grad is not None and p.grad.data_ptr() == sq.grad.data_ptr() + 4 * s.offset
                                for p, s in zip(q, sq.segments))
    assert sp.numel == 128 + 64  # 64-element aligned segments
    for p, v, s in zip(ps, vals, sp.segments):
        assert torch.equal(p, v) and p.data_ptr() == sp.data.data_ptr() + 4 * s.offset
        # built before any backward: the per-step fresh-gradient mode (p.grad None; the first
        # contribution lands in the slice), as after zero_grad(set_to_none=True)
        assert p.grad is None and sp.fresh
        assert sp.grad_view(p).data_ptr() == sp.grad.data_ptr() + 4 * s.offset
    rows, n = sp.chunk_table(ps, [True, False])
    assert n == 2 and int(rows[0, 1]) >> 32 == 1 and int(rows[1, 1]) >> 32 == 0


def test_columnar_dataset_order_and_pandas():
    from ray_torch_distributed_checkpoint_amd.data import from_items

    ds = from_items([{"features": np.full((1, 2), i, np.float32), "labels": i} for i in range(10)])
    out = ds.map_batches(lambda b: {"twice": b["labels"] * 2}, batch_size=3)
    assert [r["twice"] for r in out.take_all()] == [2 * i for i in range(10)]
    df = ds.to_pandas()
    assert list(df.labels) == list(range(10)) and df.features[3].shape == (1, 2)


def test_synthetic_fashion_mnist_shape_and_range():
    from ray_torch_distributed_checkpoint_amd.data import SyntheticFashionMNIST, get_labels_map

    ds = SyntheticFashionMNIST(train=True, n=256)
    x, y = ds[0]
    assert x.shape == (1, 28, 28) and x.dtype == torch.float32 and -1.0 <= float(x.min()) and float(x.max()) <= 1.0
    assert 0 <= int(y) < 10 and len(get_labels_map()) == 10
    assert torch.equal(SyntheticFashionMNIST(train=True, n=256).data, ds.data)  # deterministic


def test_trial_logger_retention(tmp_path):
    from ray_torch_distributed_checkpoint_amd.train import storage

    log = storage.TrialLogger(str(tmp_path), num_to_keep=2)
    for i in range(4):
        d = storage.staging_dir(str(tmp_path), i)
        os.makedirs(d)
        p = storage.commit(str(tmp_path), i)
        log.log({"loss": float(i)}, i)
        log.register(i, p, {"loss": float(i)})
    assert [os.path.basename(p) for _, p in storage.list_committed(str(tmp_path))] == [
        "checkpoint_000002", "checkpoint_000003"]
    assert storage.latest_committed(str(tmp_path)).endswith("checkpoint_000003")


def test_config_surface():
    from ray_torch_distributed_checkpoint_amd import train

    rc = train.RunConfig(checkpoint_config=train.CheckpointConfig(num_to_keep=2), storage_path="/tmp/x", verbose=1)
    assert rc.resolved_storage_path() == "/tmp/x"
    with pytest.raises(ValueError):
        train.CheckpointConfig(num_to_keep=0)
    assert train.ScalingConfig(num_workers=2, use_gpu=True).num_gpus_per_worker == 1
    ck = train.Checkpoint.from_directory("/tmp")
    with ck.as_directory() as d:
        assert d == "/tmp"
    import pickle

    assert pickle.loads(pickle.dumps(ck)).path == "/tmp"


def test_result_json_roundtrip():
    from ray_torch_distributed_checkpoint_amd.train import Checkpoint, Result

    r = Result(metrics={"val_loss": 0.5}, checkpoint=Checkpoint("/tmp/c"), path="/tmp")
    r2 = Result.from_json(r.to_json())
    assert r2.checkpoint.path == "/tmp/c" and r2.metrics == {"val_loss": 0.5}


def test_philox_stream_state():
    from ray_torch_distributed_checkpoint_amd.ops import PhiloxStream

    s = PhiloxStream(seed=5)
    a = s.reserve(10)
    b = s.reserve(3)
    assert a == (5, 0) and b == (5, 3)
    st = s.state_dict()
    s2 = PhiloxStream()
    s2.load_state_dict(st)
    assert s2.reserve(1) == (5, 4)


def test_cards_render(tmp_path):
    from ray_torch_distributed_checkpoint_amd.flow.cards import Card, Markdown, Table

    c = Card("x")
    c.append(Markdown("### Misclassifications 3 out of 10"))
    c.append(Table([["a", 1]], headers=["Image", "True label"]))
    html = open(c.save(str(tmp_path), "t")).read()
    assert "<h3>Misclassifications 3 out of 10</h3>" in html and "<th>True label</th>" in html


def test_wgrad_round_split_rows():
    """Weight-gradient decomposition into full rounds of 256x256 tiles + a split-K tail
    (ops/gemm.py _round_split_rows) on a 256-CU device."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    G._ncu["fake"] = 256
    # GPT-2 LM head: 197 x 3 = 591 tiles = 2 full rounds + 79 -> rows of 170 row-tiles
    assert G._round_split_rows(50304, 768, 16384, "fake") == 170 * 256
    # whole rounds, or fewer tiles than CUs: no split
    assert G._round_split_rows(256 * 256, 256, 16384, "fake") == 0
    assert G._round_split_rows(3072, 768, 16384, "fake") == 0
    # a last round more than half full, or a short K: no split
    assert G._round_split_rows(256 * 200, 512, 16384, "fake") == 0
    assert G._round_split_rows(50304, 768, 2048, "fake") == 0
    # Llama-3 LM head over 16k tokens: 501 x 16 = 8016 tiles = 31 rounds + 80 -> 496 row-tiles
    assert G._round_split_rows(128256, 4096, 16384, "fake") == 496 * 256
    # the tail must stay a split-K candidate (< 200 tiles)
    assert G._round_split_rows(16 * 256, 257 * 256, 16384, "fake") == 0


def test_crc32_fast_matches_zlib():
    """The checkpoint writers' CRC-32 (carry-less-multiply folding + table tail,
    csrc/runtime/crc32_fast.h) equals zlib.crc32 for every length class (< 64 B table path,
    folds of 64 / 16 B with tails), unaligned starts and chained initial values."""
    import random
    import zlib

    from ray_torch_distributed_checkpoint_amd.ops import _ext

    ext = _ext.ext()
    rng = random.Random(7)
    buf = bytes(rng.getrandbits(8) for _ in range(300_000))
    lens = list(range(0, 200)) + [rng.randrange(200, 250_000) for _ in range(200)] + [250_000]
    for n in lens:
        off = rng.randrange(0, 64)
        init = 0 if n % 3 == 0 else rng.getrandbits(32)
        data = buf[off:off + n]
        assert ext.crc32(data, init) == zlib.crc32(data, init), (n, off, init)


def test_zip_data_records_native_matches_python(tmp_path):
    """The native batch locator of tensor data records (dcp._data_records ->
    ext.zip_data_records) returns what the Python parser returns for torch.save archives
    concatenated in one file (DCP's .distcp layout), written by torch itself."""
    import io
    import os

    import torch

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp

    path = os.path.join(tmp_path, "f.distcp")
    items = []
    with open(path, "wb") as f:
        for i, shape in enumerate([(3,), (17, 5), (0,), (1000,), (2, 3, 4)]):
            b = io.BytesIO()
            torch.save(torch.arange(int(torch.Size(shape).numel()), dtype=torch.float32).reshape(shape) + i, b)
            raw = b.getvalue()
            items.append((path, f.tell(), len(raw)))
            f.write(raw)
    py = [dcp._zip_data_record(p, base, ln) for p, base, ln in items]
    nat = dcp._data_records(items, threads=4)
    assert nat == [(int(o), int(n)) for o, n in py]
    with open(path, "rb") as f:
        for (o, n), (_p, base, ln) in zip(nat, items):
            f.seek(o)
            assert len(f.read(n)) == n and base <= o and o + n <= base + ln


def test_philox_graph_mode_is_reference_counted():
    """Two captured steps share the device counter base; closing the first must not drop it
    while the second still replays (utils/graphs.py CapturedStep)."""
    from ray_torch_distributed_checkpoint_amd.ops.random import PhiloxStream

    ph = PhiloxStream(seed=1, offset=100)
    ph.acquire_graph_mode("cpu")
    base = ph.device_base()
    ph.acquire_graph_mode("cpu")
    assert ph.device_base() is base
    ph.offset = 7
    ph.end_graph_step()  # a replayed step consumed 7
    ph.release_graph_mode()
    assert ph.device_base() is base and int(base.item()) == 107  # still live for the other capture
    ph.release_graph_mode()
    assert ph.device_base() is None and ph.offset == 107  # folded back once, by the last user
    ph.release_graph_mode()  # extra release is a no-op
    assert ph.offset == 107
