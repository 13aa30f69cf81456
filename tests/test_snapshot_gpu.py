"""Arena snapshot (checkpoint/snapshot.py take) against per-tensor clones, bitwise, over the
storage layouts a checkpoint can hand it: spans with gaps, overlapping and tied views
of one storage, mixed dtypes in one storage, host + device mixes, views whose byte offset is not
16-B aligned (the span's lo realignment), non-contiguous views, and arena reuse after the state
grows.  Also RTDC_CKPT_ARENA=0 (per-tensor clones)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu


def _layouts():
    dev = "cuda"
    flat = torch.randn(1 << 16, device=dev)
    raw = torch.randint(0, 255, (1 << 16,), dtype=torch.uint8, device=dev)
    f32 = raw[: 1 << 14].view(torch.float32)
    yield "gaps", [flat[0:1000], flat[5000:6000], flat[60000:65536]]
    yield "overlap_tied", [flat[0:4096], flat[1024:2048], flat[0:4096], flat[100:200]]
    yield "mixed_dtypes", [f32[0:64], raw[1024:1026].view(torch.bfloat16), raw[4096:8192].view(torch.float16),
                           raw[9000:9100]]
    yield "unaligned_lo", [flat[3:1003], flat[1003:2001], flat[2001:2013]]
    yield "host_device_mix", [flat[:300], torch.randn(77), flat[400:900], torch.arange(10)]
    m = torch.randn(64, 64, device=dev)
    yield "noncontig", [m.t(), m[:, 3], m[1:5], flat[10:20]]
    yield "many_storages", [torch.randn(n, device=dev) for n in (1, 5, 64, 1000, 4097)]


@pytest.mark.parametrize("arena", ["1", "0"])
def test_take_matches_clones_bitwise(monkeypatch, arena):
    from ray_torch_distributed_checkpoint_amd.checkpoint import snapshot

    monkeypatch.setenv("RTDC_CKPT_ARENA", arena)
    snapshot.clear()
    for name, ts in _layouts():
        ref = [t.clone() for t in ts]
        lease, out = snapshot.take(ts)
        # the sources change right after the snapshot (the next optimizer step)
        for t in ts:
            if t.is_floating_point():
                t.add_(1)
        torch.cuda.synchronize()
        for r, o in zip(ref, out):
            assert o.dtype == r.dtype and o.shape == r.shape and o.is_contiguous(), name
            assert o.device == r.device, name
            ob = o.contiguous().reshape(-1).view(torch.uint8)
            rb = r.contiguous().reshape(-1).view(torch.uint8)
            assert torch.equal(ob, rb), name
        if lease is not None:
            lease.release()


def test_arena_reused_and_regrown():
    from ray_torch_distributed_checkpoint_amd.checkpoint import snapshot

    if not snapshot.enabled():
        pytest.skip("arena disabled")
    snapshot.clear()
    flat = torch.randn(1 << 18, device="cuda")
    ts = [flat[:1000], flat[2000:9000]]
    lease, out = snapshot.take(ts)
    buf = lease.buf
    lease.release()
    lease2, out2 = snapshot.take(ts)
    assert lease2.buf.data_ptr() == buf.data_ptr()  # same arena, reused
    lease2.release()
    big = [flat, torch.randn(5000, device="cuda")]  # the state grew
    ref = [t.clone() for t in big]
    lease3, out3 = snapshot.take(big)
    torch.cuda.synchronize()
    assert lease3.buf.numel() > buf.numel()
    for r, o in zip(ref, out3):
        assert torch.equal(r, o)
    lease3.release()
    snapshot.clear()
