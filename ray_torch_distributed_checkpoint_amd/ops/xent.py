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

import os

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext
from .embedding import launch_pending_sorts
from .gradbuf import grad_target
from .shadow import kmajor_image, kmajor_prefetch, kmajor_wanted, shadow_of

IGNORE_INDEX = -100


def _check_target(target: torch.Tensor) -> None:
    if target.dtype != torch.int64:
        raise TypeError(f"cross_entropy: int64 class targets expected, got {target.dtype}")


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, n_valid):
        """n_valid: host int (fixed divisor) or None (count of non-ignored rows, on device)."""
        M, V = logits.shape
        lg = logits.contiguous()
        loss = torch.empty(M, dtype=torch.float32, device=lg.device)
        grad = torch.empty_like(lg)
        tgt = target.contiguous()
        # unscaled softmax gradient; the mean and the 1/divisor (device count of non-ignored
        # rows, or n_valid) come out of one native reduction - no ATen kernels in the step
        gpu_ext().xent(lg, grad, tgt, loss, None, None, M, V, V, 1.0, IGNORE_INDEX)
        out = torch.empty(2, dtype=torch.float32, device=lg.device)
        gpu_ext().xent_finalize(loss, tgt if n_valid is None else None, float(n_valid or 1), out)
        ctx.save_for_backward(grad, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        grad, out = ctx.saved_tensors
        dl = torch.empty_like(grad)
        gpu_ext().scale_dev(grad, dl, g.detach().to(torch.float32).reshape(1).contiguous(), out[1:2])
        return dl, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, n_valid: int | None = None) -> torch.Tensor:
    """nn.CrossEntropyLoss() (mean over rows whose target != -100).  On the GPU the divisor is
    counted on the device unless the caller passes `n_valid`."""
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=IGNORE_INDEX)
    _check_target(target)
    if logits.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"cross_entropy: fp32 or bf16 logits expected on the GPU, got {logits.dtype}")
    return _CrossEntropy.apply(logits, target, n_valid)


# Off by default: measured on GPT-2-small (B16 T1024, 1 MI355X, profiles/lmhead_chunk_ab.txt)
# the unchunked in-place form is fastest - 866.6 samples/s vs 864.2 (160 MB chunks), 854.2
# (96 MB), 810.1 (48 MB): the per-chunk GEMM tails cost more than the HBM round trip saves.
_LM_CHUNK_MB = float(os.environ.get("RTDC_LMHEAD_CHUNK_MB", "0"))
_chunk_bufs: dict = {}
# The logits product runs on the hand-written kernels like every other GEMM of the step (no
# vendor-library route: round 5's hipBLASLt default for this product was removed in round 6).


def _lm_chunk_rows(M: int, Vp: int) -> int:
    """Rows per LM-head chunk: about RTDC_LMHEAD_CHUNK_MB of bf16 logits, a multiple of 256
    (the GEMM row tile); 0 disables chunking."""
    if _LM_CHUNK_MB <= 0:
        return M
    r = int(_LM_CHUNK_MB * (1 << 20) / (2 * Vp)) // 256 * 256
    return M if r <= 0 or r >= M else r


def _chunk_buffer(device, numel: int) -> torch.Tensor:
    key = str(device)
    t = _chunk_bufs.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(numel, dtype=torch.bfloat16, device=device)
        _chunk_bufs[key] = t
    return t


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
        loss = torch.empty(M, dtype=torch.float32, device=x.device)
        scale = 1.0 / n_valid if n_valid is not None else 1.0
        tgt = target.reshape(-1).contiguous()
        # the logits' input gradient on a K-major image of the (tied) vocabulary matrix, built
        # on a side stream under the logits GEMM and the loss kernel (ops/shadow.py)
        ctx.kimg = ctx.needs_input_grad[0] and kmajor_wanted(w, M)
        if ctx.kimg:
            kmajor_prefetch(w)
        R = _lm_chunk_rows(M, Vp)
        if R >= M:
            # [M, Vp] bf16, softmax gradient written in place (the logits product on the
            # persistent native GEMM: ops/gemm.py linear_fwd)
            logits = G.linear_fwd(x2, ws)
            launch_pending_sorts()  # the embedding backward's token sort, under the xent kernel
            gpu_ext().xent(logits, logits, tgt, loss, None, None, M, vocab, Vp, scale, IGNORE_INDEX)
        else:
            # row chunks: each chunk's logits land in one reused buffer small enough to stay in
            # the 256 MB Infinity Cache next to the weight, the cross-entropy reads them from
            # there and writes the chunk's softmax gradient into the full-size gradient buffer -
            # the full [M, V] logits never make an HBM round trip
            logits = torch.empty((M, Vp), dtype=torch.bfloat16, device=x.device)  # -> dlogits
            buf = _chunk_buffer(x.device, R * Vp)
            for r0 in range(0, M, R):
                n = min(R, M - r0)
                chunk = buf[: n * Vp].view(n, Vp)
                G.gemm_bf16(x2[r0:r0 + n], ws, chunk, n, Vp, C, C, C, Vp, True, True)
                gpu_ext().xent(chunk, logits[r0:r0 + n], tgt[r0:r0 + n], loss[r0:r0 + n], None, None, n, vocab,
                               Vp, scale, IGNORE_INDEX)
        launch_pending_sorts()
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        # out[0] = mean loss; out[1] = divisor (device count of non-ignored rows, or n_valid -
        # whose 1/n_valid the kernel already folded into the gradient)
        gpu_ext().xent_finalize(loss, tgt if n_valid is None else None, float(n_valid or 1), out)
        ctx.save_for_backward(x2, ws, logits, out[1:2] if n_valid is None else None)
        ctx.in_shape = x.shape
        ctx.w = w
        return out[0]

    @staticmethod
    def backward(ctx, g):
        x2, ws, dlogits, cnt = ctx.saved_tensors
        # the upstream loss gradient (and the 1/#valid divisor) is a device-side alpha inside both GEMMs
        gs = g.detach().to(torch.float32).reshape(1).contiguous()
        if cnt is not None:
            a = torch.empty(1, dtype=torch.float32, device=gs.device)
            gpu_ext().xent_alpha(gs, cnt, a)
            gs = a
        dx = G.linear_dgrad(dlogits, ws, alpha_dev=gs, w_kmajor=kmajor_image(ctx.w) if ctx.kimg else None)
        dw = G.linear_wgrad(dlogits, x2, out=grad_target(ctx.w), alpha_dev=gs)
        return dx.view(ctx.in_shape), dw, None, None, None


def lm_head_cross_entropy(x, w, target, vocab: int, n_valid: int | None = None):
    """Tied/untied LM head + mean cross-entropy over non-ignored targets (see cross_entropy)."""
    if not x.is_cuda:
        logits = F.linear(x, w.to(x.dtype))[..., :vocab]
        return F.cross_entropy(logits.reshape(-1, vocab).float(), target.reshape(-1), ignore_index=IGNORE_INDEX)
    _check_target(target)
    if x.dtype != torch.bfloat16:
        raise TypeError(f"lm_head_cross_entropy: bf16 activations expected on the GPU, got {x.dtype}")
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
