"""Loader for the native `_C` extension (HIP kernels for gfx950 + C++ checkpoint runtime).

Policy: on a machine with a GPU the native extension is mandatory - a missing or stale build
raises instead of silently falling back to eager PyTorch (the GPU path must run the HIP
kernels).  On a CPU-only machine ops use their PyTorch reference implementations, and the C++
checkpoint runtime (which has no GPU dependency) is still used when the library is present.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

import torch

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _import():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    with _lock:
        if _mod is not None or _err is not None:
            return _mod
        try:
            alt = os.environ.get("RTDC_EXT_SO")  # A/B runs: another build of the same module
            if alt:
                spec = importlib.util.spec_from_file_location("ray_torch_distributed_checkpoint_amd._C", alt)
                _mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_mod)
            else:
                _mod = importlib.import_module("ray_torch_distributed_checkpoint_amd._C")
        except Exception as e:  # pragma: no cover - exercised on unbuilt trees
            if os.environ.get("RTDC_AUTOBUILD", "0") == "1":
                from .. import _build

                _build.build()
                _mod = importlib.import_module("ray_torch_distributed_checkpoint_amd._C")
            else:
                _err = e
    return _mod


def available() -> bool:
    return _import() is not None


def ext():
    """The native module; raises if it is not built."""
    m = _import()
    if m is None:
        raise RuntimeError(
            "ray_torch_distributed_checkpoint_amd native extension `_C` is not built: run "
            "`python -m ray_torch_distributed_checkpoint_amd._build` (hipcc, --offload-arch=gfx950). "
            f"Import error: {_err!r}"
        )
    return m


def gpu_ext():
    """Native module for a GPU op: always required (no eager fallback on a GPU)."""
    return ext()


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on the GPU: the op must run its HIP kernel."""
    return t.is_cuda


def require_dtype(t: torch.Tensor, op: str, allowed=(torch.bfloat16,)) -> None:
    """GPU tensors must be in a dtype the native kernel implements: raise instead of falling
    back to MIOpen / SDPA / ATen (the GPU path runs the HIP kernels or nothing)."""
    if t.dtype not in allowed:
        names = "/".join(str(d).replace("torch.", "") for d in allowed)
        raise TypeError(f"{op}: the native gfx950 kernel takes {names} GPU tensors, got {t.dtype} "
                        f"(cast explicitly; there is no silent eager fallback on the GPU)")
