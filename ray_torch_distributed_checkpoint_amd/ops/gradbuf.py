"""Where a native backward writes a parameter gradient.

With a FlatParamSpace in "fresh" mode (after `zero_grad(set_to_none=True)`) a parameter's
first gradient contribution of the step is written by the producing kernel straight into
the parameter's slice of the flat gradient buffer; torch's AccumulateGrad sees `p.grad is
None` and adopts that tensor as `p.grad` without a copy (the stealing path of
torch/csrc/autograd/functions/accumulate_grad.h), so there is neither an add kernel nor a
memset of the buffer per step, and the DDP buckets / fused optimizer find the gradient in
place.  A second contribution in the same step (tied weights) gets a fresh tensor and is
added by autograd as usual; anything that ends up outside the buffer is folded back by the
DDP hook / `FlatParamSpace.ensure_grad_views`.

A first contribution may be a DEFERRED weight gradient (ops/gemm.py `_WgradGroup`): its slice
is written only at the next flush, and the write overwrites.  Whenever a second contribution
of the same step is about to read or add to that slice (a weight shared by two linears, whose
second gradient autograd adds out of place; a linear head tied to an embedding, whose
backward adds in place through `claimed_target`), the pending products are flushed first.
"""
from __future__ import annotations

import torch


def grad_target(p: torch.Tensor | None) -> torch.Tensor | None:
    """The flat-buffer view to write p's gradient into, or None (allocate normally)."""
    if p is None:
        return None
    sp = getattr(p, "_rtdc_space", None)
    if sp is None or sp.grad is None or not sp.fresh or p.grad is not None:
        return None
    if getattr(p, "_rtdc_claim", -1) == sp.step_id:
        # already handed out this step (second use of a tied weight): autograd will add this
        # contribution to the slice - which must hold the first one by then
        _flush_if_pending(sp.grad_view(p))
        return None
    p._rtdc_claim = sp.step_id
    return sp.grad_view(p)


def _flush_if_pending(view: torch.Tensor) -> None:
    from .gemm import _WG, flush_wgrads

    # only a deferred PRODUCT overwrites its slice at the flush; a pending column-sum job into a
    # bias slot claimed twice is the LayerNorm offer protocol (ops/gemm.py colsum), which
    # retargets the job instead of reading the slot
    if _WG.pending_product(view):
        flush_wgrads()


def claimed_target(p: torch.Tensor | None) -> torch.Tensor | None:
    """For the second use of a tied weight in one step: the flat-buffer view that the first
    use's backward already wrote (handed out by grad_target, not yet adopted by AccumulateGrad),
    so a native backward can ADD its contribution in place and return no gradient - instead
    of a fresh zero-filled tensor that autograd adds out of place and the optimizer copies
    back into the buffer (3 full passes over a 154 MB GPT-2 table)."""
    if p is None:
        return None
    sp = getattr(p, "_rtdc_space", None)
    if sp is None or sp.grad is None or not sp.fresh or p.grad is not None:
        return None
    if getattr(p, "_rtdc_claim", -1) != sp.step_id:
        return None
    view = sp.grad_view(p)
    _flush_if_pending(view)  # the in-place add must land on the first use's written gradient
    return view
