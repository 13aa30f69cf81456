"""Fused cross-entropy (+ LM-head fusion) on the native row kernel.

`cross_entropy(logits, target)` = nn.CrossEntropyLoss() (mean over non-ignored rows) for fp32
or bf16 logits: one launch computes per-row loss, logsumexp and the gradient.
`lm_head_cross_entropy(x, w, target, vocab)` computes logits = x w^T on the MFMA GEMM into a
bf16 buffer that the xent kernel overwrites IN PLACE with d(loss)/d(logits), so the 1.6 GB
GPT-2 logits tensor is written once and read twice in the whole step; padded vocabulary
columns (vocab rounded up to a multiple of 128) carry exactly zero gradient.
`xent_metrics(logits, target)` = (summed loss, #correct) for evaluation (argmax fused).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext
from .gradbuf import grad_target
from .shadow import shadow_of

IGNORE_INDEX = -100


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, n_valid):
        M, V = logits.shape
        lg = logits.contiguous()
        loss = torch.empty(M, dtype=torch.float32, device=lg.device)
        grad = torch.empty_like(lg)
        gpu_ext().xent(lg, grad, target.contiguous(), loss, None, None, M, V, V, 1.0 / n_valid, IGNORE_INDEX)
        ctx.save_for_backward(grad)
        return loss.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g.to(grad.dtype), None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, n_valid: int | None = None) -> torch.Tensor:
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=IGNORE_INDEX)
    if n_valid is None:
        n_valid = target.numel()
    return _CrossEntropy.apply(logits, target, n_valid)


class _LMHeadXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, target, vocab, n_valid):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        ws = shadow_of(w)
        Vp = ws.shape[0]
        M = x2.shape[0]
        logits = G.linear_fwd(x2, ws)  # [M, Vp] bf16
        loss = torch.empty(M, dtype=torch.float32, device=x.device)
        gpu_ext().xent(logits, logits, target.reshape(-1).contiguous(), loss, None, None, M, vocab, Vp,
                       1.0 / n_valid, IGNORE_INDEX)
        ctx.save_for_backward(x2, ws, logits)
        ctx.in_shape = x.shape
        ctx.w = w
        return loss.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        x2, ws, dlogits = ctx.saved_tensors
        # the upstream loss gradient is applied as a device-side alpha inside both GEMMs
        gs = g.detach().to(torch.float32).reshape(1).contiguous()
        dx = G.linear_dgrad(dlogits, ws, alpha_dev=gs)
        dw = G.linear_wgrad(dlogits, x2, out=grad_target(ctx.w), alpha_dev=gs)
        return dx.view(ctx.in_shape), dw, None, None, None


def lm_head_cross_entropy(x, w, target, vocab: int, n_valid: int | None = None):
    if n_valid is None:
        n_valid = target.numel()
    if not x.is_cuda:
        logits = F.linear(x, w.to(x.dtype))[..., :vocab]
        return F.cross_entropy(logits.reshape(-1, vocab).float(), target.reshape(-1), ignore_index=IGNORE_INDEX)
    return _LMHeadXent.apply(x, w, target, vocab, n_valid)


@torch.no_grad()
def xent_metrics(logits: torch.Tensor, target: torch.Tensor, vocab: int | None = None):
    """(sum of per-row losses, number of correct argmax predictions) as 0-d tensors, no host sync."""
    M, ld = logits.shape
    V = vocab or ld
    if not logits.is_cuda:
        lg = logits[:, :V].float()
        loss = F.cross_entropy(lg, target, reduction="sum")
        correct = (lg.argmax(1) == target).sum()
        return loss, correct
    loss = torch.empty(M, dtype=torch.float32, device=logits.device)
    am = torch.empty(M, dtype=torch.int64, device=logits.device)
    gpu_ext().xent(logits.contiguous(), None, target.contiguous(), loss, None, am, M, V, ld, 0.0, IGNORE_INDEX)
    return loss.sum(), (am == target).sum()
