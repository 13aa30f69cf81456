"""GPU profiler (`@gpu_profile(interval=1)`, R/train_flow.py:51, R/eval_flow.py:57): the AMD SMI
sampler thread, its profile.jsonl output, summary and card; CPU path uses a fake amdsmi module."""
import json
import sys
import time
import types

import pytest


def _fake_amdsmi(n_gpus=2):
    m = types.ModuleType("amdsmi")
    m.calls = {"init": 0, "shutdown": 0}

    class AmdSmiClkType:
        GFX = "gfx"

    m.AmdSmiClkType = AmdSmiClkType
    m.amdsmi_init = lambda: m.calls.__setitem__("init", m.calls["init"] + 1)
    m.amdsmi_shut_down = lambda: m.calls.__setitem__("shutdown", m.calls["shutdown"] + 1)
    m.amdsmi_get_processor_handles = lambda: [f"h{i}" for i in range(n_gpus)]
    m.amdsmi_get_gpu_activity = lambda h: {"gfx_activity": 50 + int(h[1:]), "umc_activity": 10}
    m.amdsmi_get_gpu_vram_usage = lambda h: {"vram_used": 1000, "vram_total": 288 * 1024}
    m.amdsmi_get_power_info = lambda h: {"current_socket_power": 700}

    def clock(h, kind):
        assert kind == "gfx"
        return {"clk": 2400}

    m.amdsmi_get_clock_info = clock
    return m


def test_profiler_samples_writes_jsonl_and_card(tmp_path, monkeypatch):
    from ray_torch_distributed_checkpoint_amd.utils.profiling import GpuProfiler

    fake = _fake_amdsmi(2)
    monkeypatch.setitem(sys.modules, "amdsmi", fake)
    prof = GpuProfiler(interval=0.01, out_dir=str(tmp_path)).start()
    deadline = time.time() + 5
    while len(prof.samples) < 6 and time.time() < deadline:
        time.sleep(0.01)
    prof.stop()
    assert fake.calls == {"init": 1, "shutdown": 1}
    recs = [json.loads(l) for l in (tmp_path / "profile.jsonl").read_text().splitlines()]
    assert len(recs) == len(prof.samples) >= 6
    assert {r["gpu"] for r in recs} == {0, 1}
    r0 = next(r for r in recs if r["gpu"] == 1)
    assert r0["gfx_busy_pct"] == 51 and r0["vram_total_mb"] == 288 * 1024
    assert r0["power_w"] == 700 and r0["gfx_clock_mhz"] == 2400
    s = prof.summary()
    assert s["gpu0"]["mean_busy_pct"] == 50 and s["gpu1"]["max_vram_used_mb"] == 1000
    assert s["gpu0"]["mean_power_w"] == 700
    comps = prof.card_components()
    assert len(comps) == 2


def test_profiler_without_amdsmi_records_nothing(tmp_path, monkeypatch):
    from ray_torch_distributed_checkpoint_amd.utils.profiling import GpuProfiler, phase

    broken = types.ModuleType("amdsmi")

    def boom():
        raise RuntimeError("no driver")

    broken.amdsmi_init = boom
    monkeypatch.setitem(sys.modules, "amdsmi", broken)
    prof = GpuProfiler(interval=0.01, out_dir=str(tmp_path)).start().stop()
    assert prof.samples == [] and "no GPU samples" in prof.summary()["note"]
    assert (tmp_path / "profile.jsonl").read_text() == ""
    with phase("fwd"):  # roctx range is a no-op without a GPU
        pass


@pytest.mark.gpu
def test_profiler_real_amdsmi_on_gpu(tmp_path):
    import torch

    from ray_torch_distributed_checkpoint_amd.utils.profiling import GpuProfiler, phase

    prof = GpuProfiler(interval=0.05, out_dir=str(tmp_path)).start()
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    with phase("matmul"):
        for _ in range(20):
            a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
    time.sleep(0.3)
    prof.stop()
    assert prof.samples, f"no samples from amdsmi: {prof.error}"
    assert any(isinstance(s.get("vram_total_mb"), (int, float)) for s in prof.samples)
