"""Causal multi-head self-attention composed from the native batched MFMA GEMM + row softmax.

Inputs are the packed QKV activations [B, T, 3C] written by the c_attn GEMM, read in place
through batch strides (no split/transpose copies): per (b, h)

    S  = (Q K^T) / sqrt(Dh)        GEMM, tiles above the diagonal skipped       (causal=1)
    P  = softmax_causal(S)         wave64 row kernel, writes exact zeros above the diagonal
    O  = P V                       GEMM, k-range limited to the causal prefix    (causal=2)

backward:  dP = dO V^T (causal=1) -> dS = P*(dP - rowsum(P*dP)) -> dQ = dS K / sqrt(Dh)
(causal=2), dK = dS^T Q / sqrt(Dh) and dV = P^T dO (causal=3: k >= the key tile).

The probability matrix is materialised (B*H*T*T bf16 per layer) - affordable in 288 GB of
HBM and it keeps every product on the well-tested GEMM; a flash-style fused kernel replaces
this path when T grows.  GQA (Llama) reuses it with per-head K/V strides.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import gemm as G
from ._ext import gpu_ext, require_dtype
from .streams import side_stream


def _qkv_layout(B, T, H, Hkv, Dh):
    C = H * Dh
    row = C + 2 * Hkv * Dh  # qkv row width
    return C, row


class _CausalAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, T, H, Hkv, Dh):
        C, row = _qkv_layout(B, T, H, Hkv, Dh)
        qkv = qkv.contiguous()
        dev = qkv.device
        alpha = 1.0 / math.sqrt(Dh)
        grp = H // Hkv
        P = torch.empty((B, H, T, T), dtype=torch.bfloat16, device=dev)
        q = qkv
        k = qkv[..., C:]
        v = qkv[..., C + Hkv * Dh:]
        # GQA: head h reads kv head h // grp -> inner stride over heads is Dh/grp per q-head...
        # expressed with batch_inner = H and explicit strides: kv offset = (h // grp) * Dh.
        if grp == 1:
            kstride = Dh
        else:
            kstride = None
        out = torch.empty((B, T, C), dtype=torch.bfloat16, device=dev)
        if kstride is not None:
            G.gemm_bf16(q, k, P, T, T, Dh, row, row, T, True, True, alpha=alpha, causal=G.CAUSAL_SKIP_UPPER,
                        batch=B * H, batch_inner=H, strides=(T * row, Dh, T * row, Dh, H * T * T, T * T))
            gpu_ext().softmax_fwd(P, P, None, B * H * T, T, True)
            G.gemm_bf16(P, v, out, T, Dh, T, T, row, C, True, False, causal=G.CAUSAL_K_UPTO_M,
                        batch=B * H, batch_inner=H, strides=(H * T * T, T * T, T * row, Dh, T * C, Dh))
        else:
            for g in range(grp):  # q heads h = j*grp + g share kv head j
                G.gemm_bf16(q[..., g * Dh:], k, P[:, g::grp], T, T, Dh, row, row, T, True, True, alpha=alpha,
                            causal=G.CAUSAL_SKIP_UPPER, batch=B * Hkv, batch_inner=Hkv,
                            strides=(T * row, grp * Dh, T * row, Dh, H * T * T, grp * T * T))
            gpu_ext().softmax_fwd(P, P, None, B * H * T, T, True)
            for g in range(grp):
                G.gemm_bf16(P[:, g::grp], v, out[..., g * Dh:], T, Dh, T, T, row, C, True, False,
                            causal=G.CAUSAL_K_UPTO_M, batch=B * Hkv, batch_inner=Hkv,
                            strides=(H * T * T, grp * T * T, T * row, Dh, T * C, grp * Dh))
        ctx.save_for_backward(qkv, P)
        ctx.dims = (B, T, H, Hkv, Dh)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, P = ctx.saved_tensors
        B, T, H, Hkv, Dh = ctx.dims
        C, row = _qkv_layout(B, T, H, Hkv, Dh)
        grp = H // Hkv
        alpha = 1.0 / math.sqrt(Dh)
        dout = dout.contiguous()
        dev = qkv.device
        q, k, v = qkv, qkv[..., C:], qkv[..., C + Hkv * Dh:]
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv, dqkv[..., C:], dqkv[..., C + Hkv * Dh:]
        dP = torch.empty((B, H, T, T), dtype=torch.bfloat16, device=dev)
        for g in range(grp):
            # dP = dO V^T
            G.gemm_bf16(dout[..., g * Dh:], v, dP[:, g::grp], T, T, Dh, C, row, T, True, True,
                        causal=G.CAUSAL_SKIP_UPPER, batch=B * Hkv, batch_inner=Hkv,
                        strides=(T * C, grp * Dh, T * row, Dh, H * T * T, grp * T * T))
        gpu_ext().softmax_bwd(P, dP, dP, B * H * T, T, True)
        for g in range(grp):
            # dQ = alpha * dS K
            G.gemm_bf16(dP[:, g::grp], k, dq[..., g * Dh:], T, Dh, T, T, row, row, True, False, alpha=alpha,
                        causal=G.CAUSAL_K_UPTO_M, batch=B * Hkv, batch_inner=Hkv,
                        strides=(H * T * T, grp * T * T, T * row, Dh, T * row, grp * Dh))
        # dK, dV sum over the q-heads of a group: first group writes, the rest accumulate
        for g in range(grp):
            acc = g > 0
            G.gemm_bf16(dP[:, g::grp], q[..., g * Dh:], dk, T, Dh, T, T, row, row, False, False, alpha=alpha,
                        Cin=dk if acc else None, beta=1.0 if acc else 0.0, causal=G.CAUSAL_K_FROM_M,
                        batch=B * Hkv, batch_inner=Hkv,
                        strides=(H * T * T, grp * T * T, T * row, grp * Dh, T * row, Dh))
            G.gemm_bf16(P[:, g::grp], dout[..., g * Dh:], dv, T, Dh, T, T, C, row, False, False,
                        Cin=dv if acc else None, beta=1.0 if acc else 0.0, causal=G.CAUSAL_K_FROM_M,
                        batch=B * Hkv, batch_inner=Hkv,
                        strides=(H * T * T, grp * T * T, T * C, grp * Dh, T * row, Dh))
        return dqkv, None, None, None, None, None


# RTDC_FA_CONCURRENT=1: the flash backward's dQ and dK/dV passes on two streams (delta computed
# by its own kernel first); 0: both on the compute stream, dQ first (it stores delta)
_FA_CONCURRENT = os.environ.get("RTDC_FA_CONCURRENT", "0") == "1"


class _FlashAttention(torch.autograd.Function):
    """Fused causal flash attention (csrc/kernels/attn_flash.hip): no T x T matrix in HBM."""

    @staticmethod
    def forward(ctx, qkv, B, T, H, Hkv, Dh):
        qkv = qkv.contiguous()
        out = torch.empty((B, T, H * Dh), dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty((B * H, T), dtype=torch.float32, device=qkv.device)
        scale = 1.0 / math.sqrt(Dh)
        gpu_ext().flash_fwd(qkv, out, lse, B, T, H, Hkv, Dh, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.dims = (B, T, H, Hkv, Dh, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, T, H, Hkv, Dh, scale = ctx.dims
        dqkv = torch.empty_like(qkv)
        delta = torch.empty((B * H, T), dtype=torch.float32, device=qkv.device)
        # the column sums of dqkv (the qkv projection's bias gradient) as per-16-row partials
        # written by the kernels on the way out, offered to that projection's colsum()
        Wd = qkv.shape[-1]
        cs = torch.empty((B * T // 16, Wd), dtype=torch.float32, device=qkv.device) if G.partials_wanted() else None
        qs = _dkdv_head_split(B, T, H, Hkv, qkv.device)
        part = torch.empty(qs * B * T * Hkv * 2 * Dh, dtype=torch.float32, device=qkv.device) if qs > 1 else None
        dout = dout.contiguous()
        if _FA_CONCURRENT:
            # delta alone first, then the dQ pass here and the dK/dV pass on a side stream: the two
            # latency-bound kernels share the CUs and fill each other's causal tails
            gpu_ext().flash_delta(out, dout, delta, B, T, H, Dh)
            cur = torch.cuda.current_stream(qkv.device)
            side = side_stream(qkv.device, "sort")  # (idle in the backward: the token sort runs under the LM head)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                gpu_ext().flash_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, cs, part, qs,
                                    which=2, delta_ready=True)
            gpu_ext().flash_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, cs, part, qs,
                                which=1, delta_ready=True)
            cur.wait_stream(side)
            for t in (qkv, out, dout, lse, delta, dqkv, cs, part):
                if t is not None:
                    t.record_stream(side)
        else:
            gpu_ext().flash_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, Hkv, Dh, scale, cs, part, qs)
        if cs is not None:
            G.offer_colsum_partials(dqkv, cs)
        return dqkv, None, None, None, None, None


def _dkdv_head_split(B: int, T: int, H: int, Hkv: int, device) -> int:
    """q-head subsets per GQA group for the dK/dV pass.  One dK/dV block owns 64 keys of one
    kv-head and loops over every q-head of its group, so a short batch (Llama-3-8B at B=1,
    T=2048: 8 kv-heads x 32 key blocks = 256 blocks, the heaviest with 4x32 steps) fills one
    block per CU with a 2:1 load imbalance.  Splitting the group over `qs` blocks multiplies the
    block count (partials summed in a fixed order by dkdv_reduce_kernel: deterministic) and lets
    the heavy-first order balance them.  RTDC_FA_QS forces a value (1 = no split)."""
    grp = H // Hkv
    forced = int(os.environ.get("RTDC_FA_QS", "0"))
    if forced:
        return forced if grp % forced == 0 else 1
    from .gemm import _num_cus

    blocks, cus = B * Hkv * (T // 64), _num_cus(device)
    qs = 1
    while grp % (qs * 2) == 0 and blocks * qs < 4 * cus:
        qs *= 2
    return qs


def flash_supported(T: int, Dh: int) -> bool:
    return T % 64 == 0 and Dh in (64, 128)


def causal_attention_ref(qkv, B, T, H, Hkv, Dh):
    C = H * Dh
    q = qkv[..., :C].reshape(B, T, H, Dh).transpose(1, 2)
    k = qkv[..., C:C + Hkv * Dh].reshape(B, T, Hkv, Dh).transpose(1, 2)
    v = qkv[..., C + Hkv * Dh:].reshape(B, T, Hkv, Dh).transpose(1, 2)
    if Hkv != H:
        k = k.repeat_interleave(H // Hkv, dim=1)
        v = v.repeat_interleave(H // Hkv, dim=1)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    return o.transpose(1, 2).reshape(B, T, C)


def causal_attention(qkv: torch.Tensor, n_head: int, n_kv_head: int | None = None) -> torch.Tensor:
    """qkv: [B, T, (H + 2*Hkv) * Dh] -> [B, T, H*Dh]."""
    B, T, W = qkv.shape
    Hkv = n_kv_head or n_head
    Dh = W // (n_head + 2 * Hkv)
    if qkv.is_cuda:
        require_dtype(qkv, "causal_attention")
    else:
        return causal_attention_ref(qkv, B, T, n_head, Hkv, Dh)
    impl = os.environ.get("RTDC_ATTN", "flash")
    if impl == "flash" and flash_supported(T, Dh):
        return _FlashAttention.apply(qkv, B, T, n_head, Hkv, Dh)
    return _CausalAttention.apply(qkv, B, T, n_head, Hkv, Dh)
