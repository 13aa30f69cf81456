"""GPT-2 (BASELINE config 3: GPT-2-small DDP on 8xMI355X) on the native gfx950 kernels.

Per block: LayerNorm (wave64 row kernel) -> c_attn GEMM (+bias epilogue) -> causal attention
on packed QKV (batched MFMA GEMMs + row softmax, no split/transpose copies) -> c_proj GEMM
with the residual add fused in its epilogue -> LayerNorm -> fused MLP (c_fc GEMM writes
GELU(h) and h in one epilogue; backward applies GELU' inside the c_proj dgrad GEMM) with
the residual fused.  The tied LM head + cross-entropy writes d(logits) in place over the
logits buffer.  Vocabulary is padded 50257 -> 50304 (multiple of 128 = the GEMM tile) with
padded columns masked out of the softmax, so every GEMM is tile-aligned.

Parameters are fp32 masters (what DDP all-reduces and the optimizer/checkpoint see); compute
is bf16 through cached shadows.  Random init follows GPT-2 (N(0, 0.02), residual projections
scaled by 1/sqrt(2 n_layer)).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    pad_vocab_multiple: int = 128
    layer_norm_eps: float = 1e-5

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return (self.vocab_size + m - 1) // m * m

    @classmethod
    def named(cls, name: str) -> "GPT2Config":
        table = {
            "gpt2-small": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
            "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
            "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
            "gpt2-tiny": dict(n_embd=128, n_layer=2, n_head=2, vocab_size=1000, n_positions=256),
        }
        return cls(**table[name])


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        self.c_attn = Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = Linear(cfg.n_embd, cfg.n_embd)

    def forward(self, x, residual):
        qkv = self.c_attn(x)
        y = ops.causal_attention(qkv, self.n_head)
        return self.c_proj(y, residual=residual)


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = Linear(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x, residual):
        return ops.fused_mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias, residual)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd, cfg.layer_norm_eps)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd, cfg.layer_norm_eps)
        self.mlp = MLP(cfg)

    def forward(self, x, prev_bias=None):
        # the residual stream passes through each LayerNorm so its gradient is summed inside
        # the norm's backward kernel (no separate add of the two branches' gradients); that
        # kernel also reduces the bias gradient of the projection that wrote the stream
        # (prev_bias: the previous block's MLP c_proj, then this block's attention c_proj)
        h, x = self.ln_1(x, passthrough=True, grad_sum_into=prev_bias)
        x = self.attn(h, residual=x)
        h, x = self.ln_2(x, passthrough=True, grad_sum_into=self.attn.c_proj.bias)
        return self.mlp(h, residual=x)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd))
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_eps)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = 0.02
        nn.init.normal_(self.wte, std=std)
        self.wte[self.cfg.vocab_size:].zero_()
        nn.init.normal_(self.wpe, std=0.01)
        for blk in self.h:
            for lin in (blk.attn.c_attn, blk.attn.c_proj, blk.mlp.c_fc, blk.mlp.c_proj):
                nn.init.normal_(lin.weight, std=std)
                nn.init.zeros_(lin.bias)
            blk.attn.c_proj.weight.mul_(1 / math.sqrt(2 * self.cfg.n_layer))
            blk.mlp.c_proj.weight.mul_(1 / math.sqrt(2 * self.cfg.n_layer))

    def num_params(self, exclude_padding=True) -> int:
        n = sum(p.numel() for p in self.parameters())
        if exclude_padding:
            n -= (self.cfg.padded_vocab - self.cfg.vocab_size) * self.cfg.n_embd
        return n

    def forward(self, idx: torch.Tensor, targets: torch.Tensor | None = None):
        x = ops.embedding(idx, self.wte, self.wpe)
        prev_bias = None
        for blk in self.h:
            x = blk(x, prev_bias)
            prev_bias = blk.mlp.c_proj.bias
        x = self.ln_f(x, grad_sum_into=prev_bias)
        if targets is not None:
            return ops.lm_head_cross_entropy(x, self.wte, targets, self.cfg.vocab_size)
        logits = ops.linear(x, self.wte)
        return logits[..., : self.cfg.vocab_size]

    def flops_per_token(self, T: int, causal: bool = True) -> float:
        """Training FLOPs per token (6N + attention), N without the embedding table."""
        c = self.cfg
        n = self.num_params() - c.n_positions * c.n_embd
        # attention scores + weighted sum: 12·L·d·T per token over the full T×T square; a causal
        # mask computes only the lower triangle, so the causal count is half of that
        return 6 * n + (6 if causal else 12) * c.n_layer * c.n_embd * T
