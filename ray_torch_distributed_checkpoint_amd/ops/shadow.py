"""bf16 compute shadows of fp32 master parameters.

Models keep fp32 master `nn.Parameter`s (what autograd, DDP, the optimizer and the checkpoint
see).  The MFMA kernels read a bf16 copy.  The copy is cached on the parameter and refreshed
when the parameter's version counter moves (any in-place torch update: `load_state_dict`,
a torch optimizer, `copy_`).  The fused native optimizers update master AND shadow in the same
kernel pass without bumping the version, so a training step never re-converts.
"""
from __future__ import annotations

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
