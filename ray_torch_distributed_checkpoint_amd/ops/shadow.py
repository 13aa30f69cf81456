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
# dgrads run 3-11 % faster (at hipBLASLt's times); in the GPT-2 step they save ~190 us against a
# 124 us batched transpose of the shadows - neutral within the run-to-run spread (17.02 vs
# 16.99 ms, profiles/r6/dgrad_kmajor_ab_r6.txt).
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


_registry: list = []   # weakrefs of the parameters that have a K-major image
_jobs: dict = {}       # device -> uint8 job-table buffer of the batched transpose


def _stale(p) -> bool:
    st = getattr(p, "_rtdc_kimg", None)
    return st is None or st["gen"] != _GEN[0] or st["ver"] != p._version


def kmajor_prefetch(w: torch.Tensor) -> None:
    """Start building this step's [in, out] bf16 image of `w` on a side stream, after
    everything the compute stream has queued (i.e. the last optimizer update).  Every other
    registered weight whose image is stale is transposed in the same launch (one batched
    transpose of the bf16 shadows per step, not one conversion per weight)."""
    import weakref

    from .streams import side_stream

    st = getattr(w, "_rtdc_kimg", None)
    if st is not None and not _stale(w):
        return
    if st is None:
        w._rtdc_kimg = {"img": torch.empty((w.shape[1], w.shape[0]), dtype=torch.bfloat16, device=w.device),
                        "gen": -1, "ver": -1, "ev": None}
        _registry.append(weakref.ref(w))
    live = [r() for r in _registry]
    _registry[:] = [r for r, p in zip(_registry, live) if p is not None]
    todo = [p for p in live if p is not None and p.device == w.device and _stale(p)]
    srcs = [shadow_of(p) for p in todo]  # (on the compute stream: refreshed there if stale)
    cur = torch.cuda.current_stream(w.device)
    side = side_stream(w.device, "wgrad")
    side.wait_stream(cur)
    jb = _jobs.get(w.device)
    if jb is None:
        jb = _jobs[w.device] = torch.empty(gpu_ext().bf16_transpose_jobs_bytes(), dtype=torch.uint8, device=w.device)
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        for i in range(0, len(todo), 96):
            gpu_ext().bf16_transpose_multi(srcs[i:i + 96], [p._rtdc_kimg["img"] for p in todo[i:i + 96]], jb)
        ev.record(side)
    for p, s_ in zip(todo, srcs):
        s_.record_stream(side)
        p._rtdc_kimg.update(gen=_GEN[0], ver=p._version, ev=ev)


def kmajor_image(w: torch.Tensor) -> torch.Tensor:
    """This step's K-major image of `w`, ordered before the caller's next kernel."""
    st = getattr(w, "_rtdc_kimg", None)
    if st is None or st["gen"] != _GEN[0] or st["ver"] != w._version:
        kmajor_prefetch(w)
        st = w._rtdc_kimg
    torch.cuda.current_stream(w.device).wait_event(st["ev"])
    return st["img"]
