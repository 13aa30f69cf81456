"""GPU utilisation/memory sampler (the reference's `@gpu_profile(interval=1)`,
R/train_flow.py:51, R/eval_flow.py:57) on AMD SMI, plus roctx-style phase ranges.

`GpuProfiler(interval)` samples every visible GPU each `interval` seconds in a background
thread (busy %, VRAM used/total, power, GFX clock) into `profile.jsonl` and renders a card.
On a machine without GPUs or without the amdsmi bindings it records nothing and says so.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time


class GpuProfiler:
    def __init__(self, interval: float = 1.0, out_dir: str | None = None):
        self.interval = interval
        self.out_dir = out_dir
        self.samples: list[dict] = []
        self._stop = threading.Event()
        self._thread = None
        self.error = None
        self._handles = []

    def _init(self):
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            self._handles = amdsmi.amdsmi_get_processor_handles()
        except Exception as e:  # no GPU / no driver
            self.error = repr(e)
            self._handles = []

    def _sample(self):
        smi = self._smi
        t = time.time()
        for i, h in enumerate(self._handles):
            rec = {"t": t, "gpu": i}
            try:
                act = smi.amdsmi_get_gpu_activity(h)
                rec["gfx_busy_pct"] = act.get("gfx_activity")
                rec["mem_busy_pct"] = act.get("umc_activity")
            except Exception:
                pass
            try:
                vram = smi.amdsmi_get_gpu_vram_usage(h)
                rec["vram_used_mb"] = vram.get("vram_used")
                rec["vram_total_mb"] = vram.get("vram_total")
            except Exception:
                pass
            try:
                pw = smi.amdsmi_get_power_info(h)
                rec["power_w"] = pw.get("current_socket_power") or pw.get("average_socket_power")
            except Exception:
                pass
            try:
                clk = smi.amdsmi_get_clock_info(h, smi.AmdSmiClkType.GFX)
                rec["gfx_clock_mhz"] = clk.get("clk")
            except Exception:
                pass
            self.samples.append(rec)

    def _loop(self):
        while not self._stop.is_set():
            try:
                self._sample()
            except Exception as e:
                self.error = repr(e)
                return
            self._stop.wait(self.interval)

    def start(self):
        self._init()
        if self._handles:
            self._thread = threading.Thread(target=self._loop, daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        try:
            if self._handles:
                self._smi.amdsmi_shut_down()
        except Exception:
            pass
        if self.out_dir:
            os.makedirs(self.out_dir, exist_ok=True)
            with open(os.path.join(self.out_dir, "profile.jsonl"), "w") as f:
                for s in self.samples:
                    f.write(json.dumps(s) + "\n")
        return self

    def summary(self) -> dict:
        out = {"samples": len(self.samples), "interval_s": self.interval}
        if self.error and not self.samples:
            out["note"] = f"no GPU samples ({self.error})"
        by = {}
        for s in self.samples:
            by.setdefault(s["gpu"], []).append(s)
        for g, ss in by.items():
            busy = [x.get("gfx_busy_pct") for x in ss if isinstance(x.get("gfx_busy_pct"), (int, float))]
            vram = [x.get("vram_used_mb") for x in ss if isinstance(x.get("vram_used_mb"), (int, float))]
            power = [x.get("power_w") for x in ss if isinstance(x.get("power_w"), (int, float))]
            out[f"gpu{g}"] = {"mean_busy_pct": sum(busy) / len(busy) if busy else None,
                              "max_vram_used_mb": max(vram) if vram else None,
                              "mean_power_w": sum(power) / len(power) if power else None}
        return out

    def card_components(self):
        from ..flow.cards import Markdown, Table

        s = self.summary()
        rows = [[k, json.dumps(v)] for k, v in s.items()]
        return [Markdown("## GPU profile"), Table(rows, headers=["key", "value"])]


@contextlib.contextmanager
def phase(name: str):
    """roctx range when rocTX is loadable (visible in rocprofv3 --marker-trace), else a no-op."""
    try:
        import torch

        torch.cuda.nvtx.range_push(name)  # maps to roctx on ROCm builds
        pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            try:
                torch.cuda.nvtx.range_pop()
            except Exception:
                pass
