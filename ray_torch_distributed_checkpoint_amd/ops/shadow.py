"""bf16 compute shadows of fp32 master parameters.

Models keep fp32 master `nn.Parameter`s (what autograd, DDP, the optimizer and the checkpoint
see).  The MFMA kernels read a bf16 copy.  The copy is cached on the parameter and refreshed
when the parameter's version counter moves (any in-place torch update: `load_state_dict`,
a torch optimizer, `copy_`).  The fused native optimizers update master AND shadow in the same
kernel pass without bumping the version, so a training step never re-converts.
"""
from __future__ import annotations

import os

import torch

from ._ext import gpu_ext


def shadow_of(p: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    if p.dtype == dtype:
        return p
    s = getattr(p, "_rtdc_shadow", None)
    ver = p._version
    if s is None or s.device != p.device or s.shape != p.shape or getattr(p, "_rtdc_shadow_ver", -1) != ver:
        if s is None or s.device != p.device or s.shape != p.shape:
            s = torch.empty(p.shape, dtype=dtype, device=p.device)
        with torch.no_grad():
            if (p.is_cuda and dtype == torch.bfloat16 and p.dtype == torch.float32 and s.stride() == p.stride()
                    and (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last))):
                gpu_ext().f32_to_bf16(p.detach(), s)  # same memory order (e.g. channels-last): raw conversion
            elif p.is_cuda and dtype == torch.bfloat16 and p.dtype == torch.float32 and s.is_contiguous():
                gpu_ext().f32_to_bf16(p.detach().contiguous(), s)
            else:
                s.copy_(p.detach())
        p._rtdc_shadow = s
        p._rtdc_shadow_ver = ver
    return s


def bind_shadow(p: torch.Tensor, s: torch.Tensor) -> None:
    """Attach an externally managed shadow (a view into a flat bf16 buffer)."""
    p._rtdc_shadow = s
    p._rtdc_shadow_ver = p._version


# ---- K-major images for the input-gradient GEMMs
# dx = dy @ W reads the [N, K] weight with the reduction index N as rows: the GEMM's B operand is
# then MN-major and its fragments come from transposing LDS reads (2x the LDS instructions of a
# K-major operand).  A bf16 [K, N] image of the fp32 master makes both operands K-major.  It is
# built once per optimizer step on a side stream while the forward runs (the forward never reads
# it) and waited for by the backward GEMM that consumes it.  Worth its transposition
# (6 B/element) only when the product is long in M: RTDC_DGRAD_KMAJOR = auto (token rows >=
# 8192: GPT-2's 16k-row steps, not Llama-3-8B's 2k) | 1 | 0 (default).  Isolated, the K-major
# dgrads run 3-11 % faster (at hipBLASLt's times); in the GPT-2 step the side-stream images cost
# more than that (18.19 / 18.10 vs 17.85 / 17.79 ms, profiles/r6/dgrad_kmajor_ab_r6.txt).
_KMAJOR = os.environ.get("RTDC_DGRAD_KMAJOR", "0")
_GEN = [0]


def bump_generation() -> None:
    """The fused optimizers call this after updating masters in place (no version bump)."""
    _GEN[0] += 1


def kmajor_wanted(w: torch.Tensor, rows: int) -> bool:
    if _KMAJOR == "0" or not (w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.is_contiguous()):
        return False
    if _KMAJOR != "1" and rows < 8192:
        return False
    return not torch.cuda.is_current_stream_capturing()


def kmajor_prefetch(w: torch.Tensor) -> None:
    """Start building this step's [in, out] bf16 image of the fp32 master `w` on a side stream
    (after everything the compute stream has queued, i.e. the last optimizer update)."""
    st = getattr(w, "_rtdc_kimg", None)
    if st is not None and st["gen"] == _GEN[0] and st["ver"] == w._version:
        return
    from .streams import side_stream

    if st is None:
        st = {"img": torch.empty((w.shape[1], w.shape[0]), dtype=torch.bfloat16, device=w.device),
              "ev": torch.cuda.Event()}
        w._rtdc_kimg = st
    side = side_stream(w.device, "wgrad")
    side.wait_stream(torch.cuda.current_stream(w.device))
    with torch.cuda.stream(side):
        gpu_ext().f32_to_bf16_t(w.detach(), st["img"])
        st["ev"].record(side)
    st["gen"], st["ver"] = _GEN[0], w._version


def kmajor_image(w: torch.Tensor) -> torch.Tensor:
    """This step's K-major image of `w`, ordered before the caller's next kernel."""
    st = getattr(w, "_rtdc_kimg", None)
    if st is None or st["gen"] != _GEN[0] or st["ver"] != w._version:
        kmajor_prefetch(w)
        st = w._rtdc_kimg
    torch.cuda.current_stream(w.device).wait_event(st["ev"])
    return st["img"]
