"""Persistent stream-K 4-wave GEMM (csrc/kernels/gemm4s.hip, tile_cfg 14) against an fp32 PyTorch
reference of the same product: all operand layouts, the fused epilogues the models use, products
whose tiles are split over 2..16 blocks (stream-K fix-up in contributor order), ragged edges, and
run-to-run bitwise determinism.  Whole-tile (data-parallel) products accumulate each element in
the same K order as the per-tile one-barrier kernel (tile_cfg 12): bitwise equal to it."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N): what the plan does with them on 256 CUs
    (16384, 768, 2304),   # GPT-2 qkv: 576 tiles = 1 whole round + 320 stream-K tiles
    (2048, 4096, 4096),   # Llama o: 128 tiles, every tile split over 2 blocks
    (2048, 4096, 6144),   # Llama qkv: 192 tiles, 2-3 blocks per tile
    (512, 4096, 512),     # 4 tiles over 64 blocks: 16 contributors per tile
    (1000, 320, 776),     # ragged rows / columns, 5 K-tiles, data-parallel
    (4096, 768, 50304),   # LM-head-like: 3152 tiles (11 whole rounds + stream-K)
]


def _ref(a, b, a_kmajor, b_kmajor):
    A = a.float() if a_kmajor else a.float().t()
    B = b.float() if b_kmajor else b.float().t()
    return A @ B.t()


def _run(M, K, N, a_kmajor, b_kmajor, cfg, **kw):
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    a = torch.randn((M, K) if a_kmajor else (K, M), device="cuda", generator=g).bfloat16()
    b = torch.randn((N, K) if b_kmajor else (K, N), device="cuda", generator=g).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    lda = K if a_kmajor else M
    ldb = K if b_kmajor else N
    G.gemm_bf16(a, b, c, M, N, K, lda, ldb, N, a_kmajor, b_kmajor, tile_cfg=cfg, **kw)
    torch.cuda.synchronize()
    return a, b, c


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("layout", [(True, True), (True, False)], ids=["fwd", "dgrad"])
def test_gemm4s_matches_fp32_reference_and_is_deterministic(M, K, N, layout):
    ak, bk = layout
    a, b, c = _run(M, K, N, ak, bk, 14)
    ref = _ref(a, b, ak, bk)
    err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    _, _, c2 = _run(M, K, N, ak, bk, 14)
    assert torch.equal(c, c2), "stream-K result differs run to run"


@pytest.mark.parametrize("layout", [(False, False), (False, True)], ids=["mn_mn", "mn_k"])
def test_gemm4s_mn_major_a(layout):
    ak, bk = layout
    a, b, c = _run(2048, 1024, 2304, ak, bk, 14)
    ref = _ref(a, b, ak, bk)
    assert (c.float() - ref).abs().max().item() / ref.abs().max().item() < 1e-2


def test_gemm4s_whole_tiles_bitwise_equal_per_tile_kernel():
    """256 x 8 tiles on 256 blocks: every tile whole (no split), same K order as cfg 12."""
    _, _, c14 = _run(8192, 1024, 2048, True, True, 14)
    _, _, c12 = _run(8192, 1024, 2048, True, True, 12)
    assert torch.equal(c14, c12)


@pytest.mark.parametrize("M,K,N", [(16384, 768, 3072), (2048, 4096, 4096)])
def test_gemm4s_fused_epilogues(M, K, N):
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    pre_ref = x.float() @ w.float().t() + bias
    # bias + GELU with the pre-activation side output (fp32 bias, as the models pass it)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre = torch.empty_like(y)
    G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=14)
    torch.cuda.synchronize()
    gelu_ref = torch.nn.functional.gelu(pre_ref, approximate="tanh")
    assert (pre.float() - pre_ref).abs().max() / pre_ref.abs().max() < 1e-2
    assert (y.float() - gelu_ref).abs().max() / gelu_ref.abs().max() < 1e-2
    # bias + residual
    y2 = torch.empty_like(y)
    G.gemm_bf16(x, w, y2, M, N, K, K, K, N, True, True, Cin=res, bias=bias, beta=1.0, tile_cfg=14)
    torch.cuda.synchronize()
    r_ref = pre_ref + res.float()
    assert (y2.float() - r_ref).abs().max() / r_ref.abs().max() < 1e-2
    # dgrad with GELU' (aux_in) + column sums (the MLP backward's c_fc bias gradient)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    cs = torch.empty(K, device="cuda", dtype=torch.float32)
    xa = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    G.gemm_bf16(dy, w, dx, M, K, N, N, K, K, True, False, aux_in=xa, act=G.ACT_GELU_BWD, colsum_out=cs,
                tile_cfg=14)
    G.flush_wgrads()
    torch.cuda.synchronize()
    xf = xa.float()
    t = torch.tanh(0.7978845608028654 * (xf + 0.044715 * xf ** 3))
    dgelu = 0.5 * (1 + t) + 0.5 * xf * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * xf * xf)
    d_ref = (dy.float() @ w.float()) * dgelu
    assert (dx.float() - d_ref).abs().max() / d_ref.abs().max() < 1e-2
    # (the epilogue sums the fp32 values before their bf16 rounding: compare with the fp32 product)
    cs_ref = d_ref.sum(0)
    assert (cs - cs_ref).abs().max() / cs_ref.abs().max() < 5e-3
