"""Llama-3 (BASELINE config 4: Llama-3 8B sharded state_dict on 8xMI355X) on the native kernels.

RMSNorm (wave64 row kernel) -> fused QKV GEMM (q, k, v heads packed: 32 + 8 + 8 heads x 128
for 8B) -> RoPE on the packed buffer (host cos/sin tables, theta 500000) -> GQA flash
attention reading the packed buffer in place -> o_proj GEMM with the residual fused ->
RMSNorm -> SwiGLU MLP with gate|up as ONE [2F, C] GEMM (w13) -> down GEMM + residual ->
final RMSNorm -> untied LM head fused with cross-entropy.

Sizing for 288 GB of HBM: 8.03 B params; DDP with fp32 master + AdamW m, v +
fp32 grads + bf16 shadows = 18 B/param = 144.5 GB per GPU (fits one MI355X, so plain DDP,
no ZeRO), and the per-rank DCP shard of the full train state is ~14 GB.

State-dict keys follow the Meta/HF naming (`layers.N.attention.wqkv`, `feed_forward.w13`...)
with Q/K/V and gate/up stored fused; `split_qkv_w13()` returns the unfused HF-style tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from ..ops.llama_ops import apply_rope, swiglu_mlp
from .layers import RMSNorm


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192
    pad_vocab_multiple: int = 128

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return (self.vocab_size + m - 1) // m * m

    @classmethod
    def named(cls, name: str) -> "LlamaConfig":
        table = {
            "llama3-8b": dict(),
            "llama3-1b": dict(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192),
            "llama3-tiny": dict(vocab_size=1024, dim=256, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=512,
                                max_seq_len=512),
        }
        return cls(**table[name])


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.wqkv = nn.Parameter(torch.empty((cfg.n_heads + 2 * cfg.n_kv_heads) * hd, cfg.dim))
        self.wo = nn.Parameter(torch.empty(cfg.dim, cfg.n_heads * hd))

    def forward(self, x, residual):
        c = self.cfg
        qkv = ops.linear(x, self.wqkv)
        qkv = apply_rope(qkv, c.n_heads, c.n_kv_heads, c.rope_theta)
        y = ops.causal_attention(qkv, c.n_heads, c.n_kv_heads)
        return ops.linear(y, self.wo, residual=residual)


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w13 = nn.Parameter(torch.empty(2 * cfg.ffn_dim, cfg.dim))
        self.w2 = nn.Parameter(torch.empty(cfg.dim, cfg.ffn_dim))

    def forward(self, x, residual):
        return swiglu_mlp(x, self.w13, self.w2, residual)


class TransformerBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x):
        h, x = self.attention_norm(x, passthrough=True)
        x = self.attention(h, residual=x)
        h, x = self.ffn_norm(x, passthrough=True)
        return self.feed_forward(h, residual=x)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None):
        super().__init__()
        self.cfg = cfg
        factory = {"device": device} if device is not None else {}
        with torch.device(device) if device is not None else _nullctx():
            self.tok_embeddings = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.dim))
            self.layers = nn.ModuleList([TransformerBlock(cfg) for _ in range(cfg.n_layers)])
            self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
            self.output = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.dim))
        del factory
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = 0.02
        nn.init.normal_(self.tok_embeddings, std=std)
        nn.init.normal_(self.output, std=std)
        self.output[self.cfg.vocab_size:].zero_()
        for blk in self.layers:
            nn.init.normal_(blk.attention.wqkv, std=std)
            nn.init.normal_(blk.attention.wo, std=std / math.sqrt(2 * self.cfg.n_layers))
            nn.init.normal_(blk.feed_forward.w13, std=std)
            nn.init.normal_(blk.feed_forward.w2, std=std / math.sqrt(2 * self.cfg.n_layers))

    def num_params(self) -> int:
        pad = (self.cfg.padded_vocab - self.cfg.vocab_size) * self.cfg.dim * 2
        return sum(p.numel() for p in self.parameters()) - pad

    def forward(self, idx, targets=None):
        x = ops.embedding(idx, self.tok_embeddings)
        for blk in self.layers:
            x = blk(x)
        x = self.norm(x)
        if targets is not None:
            return ops.lm_head_cross_entropy(x, self.output, targets, self.cfg.vocab_size)
        return ops.linear(x, self.output)[..., : self.cfg.vocab_size]

    def split_qkv_w13(self) -> dict:
        """HF-style unfused view of the weights (q/k/v_proj, gate/up_proj)."""
        c = self.cfg
        hd = c.head_dim
        out = {}
        for i, blk in enumerate(self.layers):
            q, k, v = blk.attention.wqkv.split([c.n_heads * hd, c.n_kv_heads * hd, c.n_kv_heads * hd])
            g, u = blk.feed_forward.w13.split([c.ffn_dim, c.ffn_dim])
            out.update({f"layers.{i}.q_proj": q, f"layers.{i}.k_proj": k, f"layers.{i}.v_proj": v,
                        f"layers.{i}.gate_proj": g, f"layers.{i}.up_proj": u})
        return out

    def flops_per_token(self, T: int, causal: bool = True) -> float:
        c = self.cfg
        n = self.num_params() - c.vocab_size * c.dim  # input embedding is a gather
        # attention scores + weighted sum: 12·L·d·T per token over the full T×T square; a causal
        # mask computes only the lower triangle, so the causal count is half of that
        return 6 * n + (6 if causal else 12) * c.n_layers * c.dim * T


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
