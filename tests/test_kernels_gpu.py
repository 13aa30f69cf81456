"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference (GPU only).

Operands are random (never zero/identity, cdna_hip_programming.md §5.4 rule 25-26); the
asymmetric layouts catch transposed C writes.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ext():
    from ray_torch_distributed_checkpoint_amd.ops import _ext

    return _ext.ext()


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def _close(out, ref, rel):
    err = (out.float() - ref.float()).abs().max().item()
    mag = ref.float().abs().max().item() + 1e-6
    assert err <= rel * mag, f"max err {err} vs {rel}*{mag}"


def test_native_loaded():
    m = _ext()
    assert hasattr(m, "gemm_bf16")


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 72, 192), (384, 640, 512)])
def test_gemm_bf16_layouts(a_k, b_k, M, N, K):
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(M + N + K)
    A = _bf(M, K) if a_k else _bf(K, M)
    B = _bf(N, K) if b_k else _bf(K, N)
    Af = A.float() if a_k else A.float().t()
    Bf = B.float().t() if b_k else B.float()
    ref = Af @ Bf
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k)
    _close(C, ref, 1e-5)
    Cb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, Cb, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k)
    _close(Cb, ref, 1e-2)


def test_gemm_bf16_epilogues():
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(1)
    M, N, K = 256, 384, 256
    A, B = _bf(M, K), _bf(N, K)
    bias = torch.randn(N, device=DEV)
    base = A.float() @ B.float().t()
    # bias + relu
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, K, K, N, bias=bias, act=G.ACT_RELU)
    _close(C, torch.relu(base + bias), 1e-5)
    # alpha + residual accumulate (fp32)
    R = torch.randn(M, N, device=DEV)
    C2 = R.clone()
    G.gemm_bf16(A, B, C2, M, N, K, K, K, N, Cin=C2, beta=1.0, alpha=0.5)
    _close(C2, 0.5 * base + R, 1e-5)
    # gelu with pre-activation output (bf16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    Cg = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, Cg, M, N, K, K, K, N, bias=bias, act=G.ACT_GELU, aux_out=pre)
    _close(pre, base + bias, 1e-2)
    _close(Cg, F.gelu(base + bias, approximate="tanh"), 1e-2)
    # gelu backward epilogue
    h = _bf(M, N)
    Cb = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, Cb, M, N, K, K, K, N, act=G.ACT_GELU_BWD, aux_in=h)
    hf = h.float().requires_grad_(True)
    y = F.gelu(hf, approximate="tanh")
    (gd,) = torch.autograd.grad(y.sum(), hf)
    _close(Cb, base * gd, 1e-4)


@pytest.mark.parametrize("cfg", [-1, 6, 7, 10])
def test_gemm_gelu_bwd_colsum(cfg):
    """dpre = (dy @ W) * gelu'(pre) with the column sums of dpre (the c_fc bias gradient)
    reduced by the 8-wave epilogue (cfg 6 / 7: 256x256 / 256x192 tiles; rows past M and a
    partial last row tile excluded) or by the fallback reduction (cfg -1 picks the 4-wave
    kernel at this size)."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(11)
    M, N, K = 1000, 256, 768  # dx[M, K] = dy[M, N] @ w[N, K]
    dy, w, pre = _bf(M, N), _bf(N, K, scale=0.1), _bf(M, K)
    out = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    cs = torch.full((K,), float("nan"), device=DEV)
    G.gemm_bf16(dy, w, out, M, K, N, N, K, K, True, False, aux_in=pre, act=G.ACT_GELU_BWD, tile_cfg=cfg,
                colsum_out=cs)
    hf = pre.float().requires_grad_(True)
    (gd,) = torch.autograd.grad(F.gelu(hf, approximate="tanh").sum(), hf)
    ref = (dy.float() @ w.float()) * gd
    _close(out, ref, 1e-2)
    _close(cs, ref.sum(0), 5e-3)


@pytest.mark.parametrize("cfg", [-1, 0, 6, 7, 9, 10])
def test_gemm_gelu_saved_derivative_roundtrip(cfg):
    """act 5: y = gelu(x W^T + b) with aux_out = gelu'(pre) (bf16), act 6: dx = (dy W) * aux_in
    with the fused column sums - together the GELU forward/backward pair of the MLP, against
    fp32 torch autograd, on the 4-wave, 8-wave (256x256 / 256x192) and persistent kernels."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(13)
    M, K, N = 1024, 256, 768
    x, w, b = _bf(M, K), _bf(N, K, scale=0.1), _bf(N, scale=0.5)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    gp = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True, bias=b, aux_out=gp, act=G.ACT_GELU_SAVE_GRAD, tile_cfg=cfg)
    pre = (x.float() @ w.float().t() + b.float()).requires_grad_(True)
    yr = F.gelu(pre, approximate="tanh")
    (gd,) = torch.autograd.grad(yr.sum(), pre)
    _close(y, yr, 1e-2)
    _close(gp, gd, 1e-2)
    # dgrad through the saved derivative: dpre[M, N] = (dz[M, K2] @ w2[K2, N]) * gp
    K2 = 256
    dz, w2 = _bf(M, K2), _bf(K2, N, scale=0.1)
    dpre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    cs = torch.full((N,), float("nan"), device=DEV)
    G.gemm_bf16(dz, w2, dpre, M, N, K2, K2, N, N, True, False, aux_in=gp, act=G.ACT_MUL,
                tile_cfg=cfg if cfg in (-1, 0, 6, 7, 10) else -1, colsum_out=cs)
    ref = (dz.float() @ w2.float()) * gp.float()
    _close(dpre, ref, 1e-2)
    _close(cs, ref.sum(0), 5e-3)


@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_round_split(monkeypatch, accumulate):
    """LM-head-shaped weight gradient (591 tiles on 256 CUs): the full-rounds GEMM + split-K
    tail decomposition equals the fp32 reference, with and without accumulation."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    M, N, K = 16384, 50304, 768
    assert G._round_split_rows(N, K, M, torch.device(DEV)) > 0
    dy, x = _bf(M, N, scale=0.05), _bf(M, K)
    base = torch.randn(N, K, device=DEV) if accumulate else None
    ref = dy.float().t() @ x.float() * 0.5 + (base if accumulate else 0.0)
    out = base.clone() if accumulate else torch.empty(N, K, device=DEV)
    monkeypatch.setattr(G, "_ROUND_SPLIT", True)
    G.linear_wgrad(dy, x, out=out, accumulate=accumulate, alpha=0.5)
    torch.cuda.synchronize()
    _close(out, ref, 2e-3)
    out1 = base.clone() if accumulate else torch.empty(N, K, device=DEV)
    monkeypatch.setattr(G, "_ROUND_SPLIT", False)
    G.linear_wgrad(dy, x, out=out1, accumulate=accumulate, alpha=0.5)
    torch.cuda.synchronize()
    _close(out, out1, 1e-3)


def test_gemm_bf16_batched_strided():
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(2)
    Bn, H, T, Dh = 2, 3, 256, 64
    x = _bf(Bn, T, H * Dh)
    y = _bf(Bn, T, H * Dh)
    out = torch.empty(Bn, H, T, T, device=DEV, dtype=torch.float32)
    C = H * Dh
    G.gemm_bf16(x, y, out, T, T, Dh, C, C, T, True, True, batch=Bn * H, batch_inner=H,
                strides=(T * C, Dh, T * C, Dh, H * T * T, T * T))
    xr = x.float().view(Bn, T, H, Dh).transpose(1, 2)
    yr = y.float().view(Bn, T, H, Dh).transpose(1, 2)
    _close(out, xr @ yr.transpose(-1, -2), 1e-5)


def test_linear_bf16_autograd():
    from ray_torch_distributed_checkpoint_amd.ops import linear

    torch.manual_seed(3)
    M, K, N = 512, 384, 256
    x = _bf(M, K).requires_grad_(True)
    w = (torch.randn(N, K, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(N, device=DEV).requires_grad_(True)
    res = _bf(M, N).requires_grad_(True)
    y = linear(x, w, b, relu=False, residual=res)
    g = _bf(M, N)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True)
    yr = F.linear(xr, wr, br) + rr
    yr.backward(g.float())
    _close(y, yr, 1e-2)
    _close(x.grad, xr.grad, 1e-2)
    _close(w.grad, wr.grad, 1e-4)
    _close(b.grad, br.grad, 1e-4)
    _close(res.grad, rr.grad, 1e-6)
    # relu variant
    x.grad = None
    w.grad = None
    y2 = linear(x, w, b, relu=True)
    y2.backward(g)
    xr.grad = None
    wr.grad = None
    yr2 = torch.relu(F.linear(xr, wr, br.detach()))
    yr2.backward(g.float())
    _close(x.grad, xr.grad, 2e-2)
    _close(w.grad, wr.grad, 1e-3)


def test_fused_mlp():
    from ray_torch_distributed_checkpoint_amd.ops import fused_mlp

    torch.manual_seed(4)
    M, C = 256, 128
    x = _bf(M, C).requires_grad_(True)
    wf = (torch.randn(4 * C, C, device=DEV) * 0.05).requires_grad_(True)
    bfc = (torch.randn(4 * C, device=DEV) * 0.1).requires_grad_(True)
    wp = (torch.randn(C, 4 * C, device=DEV) * 0.05).requires_grad_(True)
    bp = (torch.randn(C, device=DEV) * 0.1).requires_grad_(True)
    y = fused_mlp(x, wf, bfc, wp, bp, residual=x)
    g = _bf(M, C)
    y.backward(g)
    ps = [x.detach().float(), wf.detach().bfloat16().float(), bfc.detach(), wp.detach().bfloat16().float(), bp.detach()]
    ps = [p.clone().requires_grad_(True) for p in ps]
    h = F.gelu(F.linear(ps[0], ps[1], ps[2]), approximate="tanh")
    yr = F.linear(h, ps[3], ps[4]) + ps[0]
    yr.backward(g.float())
    _close(y, yr, 2e-2)
    _close(x.grad, ps[0].grad, 3e-2)
    _close(wf.grad, ps[1].grad, 2e-2)
    _close(wp.grad, ps[3].grad, 2e-2)
    _close(bfc.grad, ps[2].grad, 2e-2)
    _close(bp.grad, ps[4].grad, 1e-4)


@pytest.mark.parametrize("R,C", [(768, 3072), (100, 72), (65, 130)])
def test_f32_to_bf16_transposed(R, C):
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    w = torch.randn(R, C, device=DEV)
    t = torch.empty(C, R, dtype=torch.bfloat16, device=DEV)
    gpu_ext().f32_to_bf16_t(w, t)
    assert torch.equal(t, w.t().contiguous().to(torch.bfloat16))


def test_fused_mlp_kmajor_dgrad_matches(monkeypatch):
    """GPT-2 shape (3 tile rounds): c_proj's dgrad on the K-major weight image (persistent
    kernel) against the N-major kernel - same products, same K order."""
    import importlib

    from ray_torch_distributed_checkpoint_amd.ops import fused_mlp

    S = importlib.import_module("ray_torch_distributed_checkpoint_amd.ops.shadow")
    torch.manual_seed(5)
    M, C = 16384, 768
    x0 = _bf(M, C)
    wf = (torch.randn(4 * C, C, device=DEV) * 0.02).requires_grad_(True)
    bfc = (torch.randn(4 * C, device=DEV) * 0.1).requires_grad_(True)
    wp = (torch.randn(C, 4 * C, device=DEV) * 0.02).requires_grad_(True)
    bp = (torch.randn(C, device=DEV) * 0.1).requires_grad_(True)
    g = _bf(M, C)
    grads = []
    for on in (True, False):
        monkeypatch.setattr(S, "_KMAJOR", "1" if on else "0")
        x = x0.clone().requires_grad_(True)
        for p in (wf, bfc, wp, bp):
            p.grad = None
        fused_mlp(x, wf, bfc, wp, bp).backward(g)
        torch.cuda.synchronize()
        grads.append([t.grad.float().clone() for t in (x, wf, bfc)])
    for a, b in zip(*grads):
        _close(a, b, 1e-2)


@pytest.mark.parametrize("H,Hkv", [(4, 4), (4, 2)])
def test_causal_attention(H, Hkv):
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    torch.manual_seed(5)
    Bn, T, Dh = 2, 256, 64
    W = (H + 2 * Hkv) * Dh
    qkv = _bf(Bn, T, W).requires_grad_(True)
    out = causal_attention(qkv, H, Hkv)
    g = _bf(Bn, T, H * Dh)
    out.backward(g)
    qr = qkv.detach().float().requires_grad_(True)
    ref = causal_attention_ref(qr, Bn, T, H, Hkv, Dh)
    ref.backward(g.float())
    _close(out, ref, 2e-2)
    _close(qkv.grad, qr.grad, 3e-2)


@pytest.mark.parametrize("H,Hkv,Dh", [(4, 4, 64), (4, 2, 128)])
def test_flash_bwd_colsum_partials(H, Hkv, Dh):
    """The flash backward's per-16-row column sums of dqkv (the qkv bias gradient, offered to
    the projection's colsum) equal the column sums of the dqkv it stored."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(6)
    Bn, T = 2, 256
    W = (H + 2 * Hkv) * Dh
    qkv = _bf(Bn, T, W).requires_grad_(True)
    out = causal_attention(qkv, H, Hkv)
    out.backward(_bf(Bn, T, H * Dh))
    d2 = qkv.grad.view(-1, W)
    ref = d2.float().sum(0)
    cs = G.colsum(d2)  # takes the offered partials
    torch.cuda.synchronize()
    _close(cs, ref, 1e-5)
    assert G._take_partials(d2) is None  # consumed


def test_layernorm_rmsnorm():
    from ray_torch_distributed_checkpoint_amd.ops import layer_norm, rms_norm

    torch.manual_seed(6)
    for D in (768, 256, 4096, 200):  # 768 / 256: the 8-B-chunk backward (3 / 1 chunks per lane)
        M = 64
        x = _bf(M, D, scale=2.0).requires_grad_(True)
        w = (1 + 0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
        b = (0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
        g = _bf(M, D)
        y = layer_norm(x, w, b)
        y.backward(g)
        xr = x.detach().float().requires_grad_(True)
        wr = w.detach().bfloat16().float().requires_grad_(True)
        br = b.detach().bfloat16().float().requires_grad_(True)
        yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
        yr.backward(g.float())
        _close(y, yr, 2e-2)
        _close(x.grad, xr.grad, 2e-2)
        _close(w.grad, wr.grad, 1e-3)
        _close(b.grad, br.grad, 1e-3)
        x.grad = None
        w.grad = None
        y2 = rms_norm(x, w)
        y2.backward(g)
        xr2 = x.detach().float().requires_grad_(True)
        wr2 = w.detach().bfloat16().float().requires_grad_(True)
        yr2 = xr2 * torch.rsqrt(xr2.pow(2).mean(-1, keepdim=True) + 1e-5) * wr2
        yr2.backward(g.float())
        _close(y2, yr2, 2e-2)
        _close(x.grad, xr2.grad, 2e-2)
        _close(w.grad, wr2.grad, 1e-3)


@pytest.mark.parametrize("M,N", [(100, 72), (4096, 768), (16384, 2304), (65536, 64)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_colsum_two_level_reduce(M, N, accumulate):
    """Bias-gradient column sums (partial rows + the one-launch wide reduce or the single-stage
    form for few partial rows) equal the fp32 reference, and repeat bitwise."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    x = _bf(M, N)
    base = torch.randn(N, device=DEV)
    out = base.clone() if accumulate else torch.empty(N, device=DEV)
    G.colsum(x, out=out, accumulate=accumulate)
    ref = x.float().sum(0) + (base if accumulate else 0.0)
    torch.cuda.synchronize()
    _close(out, ref, 1e-4 * math.sqrt(M))
    out2 = base.clone() if accumulate else torch.empty(N, device=DEV)
    G.colsum(x, out=out2, accumulate=accumulate)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


def test_layernorm_bwd_offers_dx_colsum():
    """LayerNorm backward also reduces the column sums of the residual-stream gradient it
    writes (passthrough form, dres added); colsum() of that gradient takes them (no second
    reduction) and they match a plain fp32 sum, also when accumulating into a bias grad."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.ops import layer_norm

    torch.manual_seed(8)
    M, D = 4096, 768
    x = _bf(M, D, scale=2.0).requires_grad_(True)
    w = (1 + 0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    producer_bias = torch.zeros(D, device=DEV, requires_grad=True)  # the projection that wrote x
    y, xp = layer_norm(x, w, b, passthrough=True, grad_sum_into=producer_bias)
    dres = _bf(M, D)
    torch.autograd.backward([y, xp], [_bf(M, D), dres])
    dx = x.grad
    assert len(G._offered) > 0
    ref = dx.float().sum(0)
    got = G.colsum(dx.view(M, D))
    _close(got, ref, 5e-3)  # fp32 sums of the unrounded dx vs the bf16 dx
    assert G._take_colsum(dx.view(M, D)) is None  # taken once
    acc = torch.ones(D, device=DEV)
    G.offer_colsum(dx, got.clone())
    G.colsum(dx.view(M, D), out=acc, accumulate=True)
    _close(acc, ref + 1, 5e-3)
    # a tensor modified in place after the offer is reduced again, not served stale sums
    G.offer_colsum(dx, got.clone())
    dx.mul_(2)
    _close(G.colsum(dx.view(M, D)), 2 * ref, 1e-3)


@pytest.mark.parametrize("dtype,V,ld",[(torch.float32, 10, 10), (torch.bfloat16, 1000, 1024), (torch.float32, 333, 333),
                                        (torch.bfloat16, 1000, 1000), (torch.bfloat16, 50257, 50257),
                                        (torch.bfloat16, 128256, 128256)])
def test_cross_entropy(dtype, V, ld):
    from ray_torch_distributed_checkpoint_amd.ops import cross_entropy, xent_metrics

    torch.manual_seed(7)
    M = 64
    logits = (torch.randn(M, V, device=DEV) * 3).to(dtype).requires_grad_(True)
    tgt = torch.randint(0, V, (M,), device=DEV)
    loss = cross_entropy(logits, tgt)
    loss.backward()
    lr_ = logits.detach().float().requires_grad_(True)
    ref = F.cross_entropy(lr_, tgt)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    _close(logits.grad, lr_.grad, 2e-2 if dtype == torch.bfloat16 else 1e-4)
    ls, nc = xent_metrics(logits.detach(), tgt)
    assert abs(ls.item() - ref.item() * M) < 1e-2 * M
    assert nc.item() == (lr_.detach().argmax(1) == tgt).sum().item()


def test_lm_head_cross_entropy_padded_vocab():
    from ray_torch_distributed_checkpoint_amd.ops import lm_head_cross_entropy

    torch.manual_seed(8)
    M, C, V, Vp = 128, 128, 1000, 1024
    x = _bf(M, C).requires_grad_(True)
    w = (torch.randn(Vp, C, device=DEV) * 0.1).requires_grad_(True)
    tgt = torch.randint(0, V, (M,), device=DEV)
    loss = lm_head_cross_entropy(x, w, tgt, V)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    ref = F.cross_entropy(F.linear(xr, wr)[:, :V], tgt)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-2
    _close(x.grad, xr.grad, 3e-2)
    _close(w.grad, wr.grad, 3e-2)
    assert w.grad[V:].abs().max().item() == 0.0


def test_embedding():
    from ray_torch_distributed_checkpoint_amd.ops import embedding

    torch.manual_seed(9)
    Bn, T, D, V = 4, 64, 128, 500
    idx = torch.randint(0, V, (Bn, T), device=DEV)
    wte = torch.randn(V, D, device=DEV).requires_grad_(True)
    wpe = torch.randn(128, D, device=DEV).requires_grad_(True)
    y = embedding(idx, wte, wpe)
    g = _bf(Bn, T, D)
    y.backward(g)
    wr = wte.detach().bfloat16().float().requires_grad_(True)
    pr = wpe.detach().bfloat16().float().requires_grad_(True)
    yr = F.embedding(idx, wr) + pr[:T]
    yr.backward(g.float())
    _close(y, yr, 1e-2)
    _close(wte.grad, wr.grad, 1e-4)
    _close(wpe.grad, pr.grad, 1e-4)

    # heavy id repetition: the sorted-run reduction must be bitwise reproducible
    idx = torch.randint(0, 7, (8, 256), device=DEV)
    g = _bf(8, 256, D)
    grads = []
    for _ in range(3):
        w = torch.randn(V, D, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)).requires_grad_(True)
        embedding(idx, w, None).backward(g)
        grads.append(w.grad)
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])
    ref = torch.zeros(V, D, device=DEV).index_add_(0, idx.reshape(-1), g.reshape(-1, D).float())
    _close(grads[0], ref, 1e-5)


def test_dropout_mask_consistency():
    from ray_torch_distributed_checkpoint_amd.ops import dropout

    torch.manual_seed(10)
    x = torch.randn(100_003, device=DEV).requires_grad_(True)
    y = dropout(x, 0.25, True)
    keep = y.detach() != 0
    frac = keep.float().mean().item()
    assert 0.73 < frac < 0.77
    _close(y[keep], x.detach()[keep] / 0.75, 1e-6)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, keep)


def test_linear_f32():
    from ray_torch_distributed_checkpoint_amd.ops import linear

    torch.manual_seed(11)
    for (M, K, N) in [(16, 784, 512), (16, 512, 10), (37, 100, 70)]:
        x = torch.randn(M, K, device=DEV).requires_grad_(True)
        w = (torch.randn(N, K, device=DEV) * 0.05).requires_grad_(True)
        b = torch.randn(N, device=DEV).requires_grad_(True)
        y = linear(x, w, b, relu=True)
        g = torch.randn(M, N, device=DEV)
        y.backward(g)
        xr, wr, br = [t.detach().clone().double().requires_grad_(True) for t in (x, w, b)]
        yr = torch.relu(F.linear(xr, wr, br))
        yr.backward(g.double())
        _close(y, yr, 1e-5)
        _close(x.grad, xr.grad, 1e-5)
        _close(w.grad, wr.grad, 1e-5)
        _close(b.grad, br.grad, 1e-5)


def test_fused_optimizers_match_torch():
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD

    torch.manual_seed(12)
    shapes = [(64, 33), (7,), (128, 128), (3, 5, 9)]
    for kind in ("adamw", "sgd"):
        ps = [torch.randn(*s, device=DEV, requires_grad=True) for s in shapes]
        qs = [p.detach().clone().requires_grad_(True) for p in ps]
        if kind == "adamw":
            opt = FusedAdamW(ps, lr=1e-2, weight_decay=0.1)
            ref = torch.optim.AdamW(qs, lr=1e-2, weight_decay=0.1, foreach=False)
        else:
            opt = FusedSGD(ps, lr=1e-2, momentum=0.9)
            ref = torch.optim.SGD(qs, lr=1e-2, momentum=0.9, foreach=False)
        for step in range(4):
            grads = [torch.randn_like(p) for p in ps]
            opt.zero_grad()
            ref.zero_grad()
            for p, q, g in zip(ps, qs, grads):
                p.grad = g.clone() if p.grad is None else p.grad.copy_(g)
                q.grad = g.clone()
            opt.step()
            ref.step()
        for p, q in zip(ps, qs):
            _close(p, q, 1e-5)


def test_ckpt_engine_writes_torch_loadable(tmp_path):
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave

    torch.manual_seed(13)
    sd = {"w": torch.randn(300, 77, device=DEV), "b": torch.arange(10, device=DEV),
          "h": torch.randn(5, device=DEV).bfloat16(), "meta": {"epoch": 3, "losses": [1.5, 2.0]}}
    p = str(tmp_path / "x.pt")
    torchsave.save(sd, p)
    got = torch.load(p, weights_only=True)
    assert got["meta"] == sd["meta"]
    for k in ("w", "b", "h"):
        assert torch.equal(got[k], sd[k].cpu())


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 10])
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_tile_configs(cfg, a_k, b_k):
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(cfg * 7 + a_k * 2 + b_k)
    M, N, K = 520, 392, 320  # partial tiles in every configuration
    A = _bf(M, K) if a_k else _bf(K, M)
    B = _bf(N, K) if b_k else _bf(K, N)
    Af = A.float() if a_k else A.float().t()
    Bf = B.float().t() if b_k else B.float()
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k, tile_cfg=cfg)
    _close(C, Af @ Bf, 1e-5)


@pytest.mark.parametrize("b_k", [True, False])
def test_gemm_256x128_tiles(b_k):
    """cfg 11: the 8-wave kernel on 256x128 tiles (one B half = 64 rows = one glds per wave,
    so the counted vmcnt waits count per event kind): plain bf16 output with partial tiles, a
    long-K product that takes split-K, and the fused epilogues (bias + GELU with the saved
    pre-activation, residual, GELU-backward with the column sums) against fp32 torch."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(31 + b_k)
    for M, N, K in ((520, 392, 320), (512, 384, 4096), (2048, 1024, 1024)):
        A = _bf(M, K, scale=0.2)
        B = _bf(N, K, scale=0.2) if b_k else _bf(K, N, scale=0.2)
        Bf = B.float().t() if b_k else B.float()
        ref = A.float() @ Bf
        C = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        G.gemm_bf16(A, B, C, M, N, K, K, B.shape[1], N, True, b_k, tile_cfg=11)
        _close(C, ref, 1e-2)
    M, N, K = 1000, 640, 768
    x = _bf(M, K)
    w = _bf(N, K, scale=0.05) if b_k else _bf(K, N, scale=0.05)
    wf = w.float().t() if b_k else w.float()
    bias = torch.randn(N, device=DEV)
    res = _bf(M, N)
    pre_ref = x.float() @ wf + bias
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, y, M, N, K, K, w.shape[1], N, True, b_k, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=11)
    _close(pre, pre_ref, 1e-2)
    _close(y, F.gelu(pre_ref, approximate="tanh"), 1e-2)
    y2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, y2, M, N, K, K, w.shape[1], N, True, b_k, Cin=res, beta=1.0, bias=bias, tile_cfg=11)
    _close(y2, pre_ref + res.float(), 1e-2)
    if not b_k:  # dgrad layout: dpre = (dy @ W) * gelu'(pre) + its column sums
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        cs = torch.full((N,), float("nan"), device=DEV)
        G.gemm_bf16(x, w, out, M, N, K, K, N, N, True, False, aux_in=pre, act=G.ACT_GELU_BWD, tile_cfg=11,
                    colsum_out=cs)
        hf = pre.float().requires_grad_(True)
        (gd,) = torch.autograd.grad(F.gelu(hf, approximate="tanh").sum(), hf)
        r = (x.float() @ wf) * gd
        _close(out, r, 1e-2)
        _close(cs, r.sum(0), 5e-3)


@pytest.mark.parametrize("cfg", [8, 9, 10])
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("K", [128, 320])
def test_gemm_persistent_multi_tile(cfg, a_k, b_k, K):
    """Persistent 8-wave kernel (cfg 8: 256x256, 9: 256x192): > 256 tiles so blocks walk
    several tiles (cross-tile DMA stream, deferred epilogue), partial edge tiles, K = 2 and 5
    K-tiles per tile."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(cfg * 100 + K + a_k * 2 + b_k)
    M, N = 4352 + 40, 4160  # 18 x 17 (256) / 18 x 22 (192) tiles, last row/column partial
    A = _bf(M, K) if a_k else _bf(K, M)
    B = _bf(N, K) if b_k else _bf(K, N)
    Af = A.float() if a_k else A.float().t()
    Bf = B.float().t() if b_k else B.float()
    ref = Af @ Bf
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k, tile_cfg=cfg)
    _close(C, ref, 1e-5)
    Cb = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, Cb, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k, tile_cfg=cfg)
    _close(Cb, ref, 1e-2)


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("K", [64, 128, 192, 320, 768])
def test_gemm_4wave_one_barrier(a_k, b_k, K):
    """tile_cfg 12 (gemm4b.hip: 4 waves, 128x128 per wave, one barrier per K-tile), every operand
    layout: 1, 2, 3, 5 and 12 K-tiles (the last two K-tiles are peeled out of the steady-state
    loop), partial edge tiles, fp32 and bf16 outputs, and (forward layout) the fused bias + GELU /
    residual epilogues."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(1200 + K + 2 * a_k + b_k)
    M, N = 1024 + 40, 768 + 8
    A = _bf(M, K) if a_k else _bf(K, M)
    B = _bf(N, K) if b_k else _bf(K, N)
    Af = A.float() if a_k else A.float().t()
    Bf = B.float().t() if b_k else B.float()
    ref = Af @ Bf
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k, tile_cfg=12)
    _close(C, ref, 1e-5)
    Cb = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, Cb, M, N, K, A.shape[1], B.shape[1], N, a_k, b_k, tile_cfg=12)
    _close(Cb, ref, 1e-2)
    if not (a_k and b_k):
        return
    bias = torch.randn(N, device=DEV)
    pre_ref = ref + bias
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, y, M, N, K, K, K, N, True, True, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=12)
    _close(pre, pre_ref, 1e-2)
    _close(y, F.gelu(pre_ref, approximate="tanh"), 1e-2)
    res = _bf(M, N)
    y2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, y2, M, N, K, K, K, N, True, True, Cin=res, beta=1.0, bias=bias, tile_cfg=12)
    _close(y2, pre_ref + res.float(), 1e-2)


@pytest.mark.parametrize("M,N,K", [(2048, 28672, 4096), (2048, 4096, 14336), (4096, 4096, 4096)])
def test_gemm_auto_long_k_forward_routes_to_one_barrier(M, N, K):
    """Long-K forward products (Llama-3-8B gate/up and down projections, 4096^3) take the
    one-barrier 4-wave kernel automatically (RTDC_GEMM4B_AUTO=2, the default: bitwise the forced
    cfg 12 result, split-K included) and match the fp32 reference."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(M + N + K)
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=DEV)
    G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True)  # the native dispatcher's own choice
    y12 = torch.empty_like(y)
    G.gemm_bf16(x, w, y12, M, N, K, K, K, N, True, True, tile_cfg=12)
    assert torch.equal(y, y12)
    _close(y, x.float() @ w.float().t(), 1e-2)


@pytest.mark.parametrize("M,N,K,res", [(2048, 4096, 4096, True), (2048, 6144, 4096, False), (16384, 768, 768, True)])
def test_linear_plain_products_native(M, N, K, res):
    """Plain products (Llama's qkv / o / gate|up / down at 2048 tokens, GPT-2's 16k-row ones) run
    on the hand-written kernels - no vendor-library route (round 6) - with the residual fused as
    beta * Cin, forward and input gradient against the fp32 reference."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(M + N)
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    r = _bf(M, N) if res else None
    assert not hasattr(G, "_blaslt_plain")
    y = G.linear_fwd(x, w, residual=r)
    ref = x.float() @ w.float().t() + (r.float() if res else 0.0)
    _close(y, ref, 1e-2)
    dy = _bf(M, N)
    dx = G.linear_dgrad(dy, w)
    _close(dx, dy.float() @ w.float(), 1e-2)


def test_gemm_4wave_one_barrier_dgrad_gelu():
    """cfg 12 with the dgrad layout and the GELU-backward epilogue (aux_in, column sums)."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(1277)
    M, N, K = 2048, 1024, 768  # dx[M, N] = dy[M, K] . W[K, N]
    dy, w, pre = _bf(M, K), _bf(K, N, scale=0.05), _bf(M, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    cs = torch.empty(N, device=DEV)
    G.gemm_bf16(dy, w, out, M, N, K, K, N, N, True, False, aux_in=pre, act=G.ACT_GELU_BWD, tile_cfg=12,
                colsum_out=cs)
    x = pre.float().requires_grad_(True)
    F.gelu(x, approximate="tanh").backward(torch.ones_like(x))
    ref = (dy.float() @ w.float()) * x.grad
    _close(out, ref, 1e-2)
    _close(cs, ref.sum(0), 2e-2)


@pytest.mark.parametrize("K", [64, 128, 192, 768])
def test_gemm_8wave_one_barrier(K):
    """tile_cfg 13 (gemm8b.hip: 8 waves, 128x64 per wave, one barrier per K-tile; K-major A and B):
    1-3 and 12 K-tiles, partial edge tiles, fp32 / bf16 outputs, split-K, bias + GELU epilogue."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(1300 + K)
    M, N = 1024 + 40, 768 + 8
    A, B = _bf(M, K), _bf(N, K)
    ref = A.float() @ B.float().t()
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, K, K, N, True, True, tile_cfg=13)
    _close(C, ref, 1e-5)
    Cb = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, Cb, M, N, K, K, K, N, True, True, tile_cfg=13)
    _close(Cb, ref, 1e-2)
    bias = torch.randn(N, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(A, B, y, M, N, K, K, K, N, True, True, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=13)
    _close(pre, ref + bias, 1e-2)
    _close(y, F.gelu(ref + bias, approximate="tanh"), 1e-2)
    Ms, Ns, Ks = 512, 512, 8192  # few tiles, long K: split-K slabs
    A2, B2 = _bf(Ms, Ks), _bf(Ns, Ks)
    C2 = torch.empty(Ms, Ns, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A2, B2, C2, Ms, Ns, Ks, Ks, Ks, Ns, True, True, tile_cfg=13)
    _close(C2, A2.float() @ B2.float().t(), 1e-5)


def test_gemm_4wave_one_barrier_splitk_and_large():
    """cfg 12 through split-K (a long-K product with few tiles: fp32 slabs + reduce) and on a
    GPT-2 c_fc-sized forward (768 tiles, 12 K-tiles)."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(1299)
    M, N, K = 512, 512, 8192
    A, B = _bf(M, K), _bf(N, K)
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, B, C, M, N, K, K, K, N, True, True, tile_cfg=12)
    _close(C, A.float() @ B.float().t(), 1e-5)
    # GPT-2 c_fc-sized forward (768 tiles, 3 per CU): plain, bias + GELU with the pre-activation
    # side output, and residual epilogues
    M, N, K = 16384 + 128, 3072, 768
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    bias, res = torch.randn(N, device=DEV), _bf(M, N)
    ref = x.float() @ w.float().t()
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True, tile_cfg=12)
    _close(y, ref, 1e-2)
    yg = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, yg, M, N, K, K, K, N, True, True, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=12)
    _close(pre, ref + bias, 1e-2)
    _close(yg, F.gelu(ref + bias, approximate="tanh"), 1e-2)
    yr = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm_bf16(x, w, yr, M, N, K, K, K, N, True, True, Cin=res, beta=1.0, bias=bias, tile_cfg=12)
    _close(yr, ref + bias + res.float(), 1e-2)


def test_gemm_persistent_epilogues():
    """bias + GELU (pre-activation side output) and residual epilogues through the persistent
    kernel, against the 2-launch reference."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(77)
    M, N, K = 4608, 3072, 768
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    bias = torch.randn(N, device=DEV)
    res = _bf(M, N)
    pre_ref = x.float() @ w.float().t() + bias
    for cfg in (8, 9, 10):
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True, bias=bias, aux_out=pre, act=G.ACT_GELU, tile_cfg=cfg)
        _close(pre, pre_ref, 1e-2)
        _close(y, F.gelu(pre_ref, approximate="tanh"), 1e-2)
        y2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        G.gemm_bf16(x, w, y2, M, N, K, K, K, N, True, True, Cin=res, beta=1.0, bias=bias, tile_cfg=cfg)
        _close(y2, pre_ref + res.float(), 1e-2)


@pytest.mark.parametrize("cfg", [6, 7, 8, 9, 12])
def test_gemm_epilogue_input_combinations(cfg):
    """The 8-wave / 4-wave / persistent epilogues' optional inputs: bias (fp32 or bf16) and
    residual, each alone and combined, and an input-gradient activation WITH a residual, on
    partial tiles against fp32 torch."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(41 + cfg)
    M, N, K = 1800, 1152, 768
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    base = x.float() @ w.float().t()
    res = _bf(M, N)
    for bias in (None, torch.randn(N, device=DEV), torch.randn(N, device=DEV).bfloat16()):
        bf = 0.0 if bias is None else bias.float()
        for r in (None, res):
            y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
            G.gemm_bf16(x, w, y, M, N, K, K, K, N, True, True, bias=bias, Cin=r, beta=0.0 if r is None else 0.5,
                        tile_cfg=cfg)
            _close(y, base + bf + (0.0 if r is None else 0.5 * res.float()), 1e-2)
    if cfg in (6, 7):  # dgrad layout with GELU' and a residual
        dy, w2, pre = _bf(M, K), _bf(K, N, scale=0.05), _bf(M, N)
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        G.gemm_bf16(dy, w2, out, M, N, K, K, N, N, True, False, aux_in=pre, act=G.ACT_GELU_BWD, Cin=res, beta=1.0,
                    tile_cfg=cfg)
        hf = pre.float().requires_grad_(True)
        (gd,) = torch.autograd.grad(F.gelu(hf, approximate="tanh").sum(), hf)
        _close(out, (dy.float() @ w2.float() + res.float()) * gd, 1e-2)


def test_gemm_persistent_auto_matches_plain(monkeypatch):
    """The automatic persistent dispatch (RTDC_GEMM_PERSIST, default on) is bitwise identical
    to the per-tile launch: same tiles, same MFMA order, only the schedule differs."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(5)
    x, w = _bf(16384, 768), _bf(3072, 768)
    y_auto = G.linear_fwd(x, w)
    y6 = torch.empty_like(y_auto)
    G.gemm_bf16(x, w, y6, 16384, 3072, 768, 768, 768, 3072, True, True, tile_cfg=6)
    y8 = torch.empty_like(y_auto)
    G.gemm_bf16(x, w, y8, 16384, 3072, 768, 768, 768, 3072, True, True, tile_cfg=8)
    assert torch.equal(y6, y8)
    _close(y_auto, x.float() @ w.float().t(), 1e-2)


def test_gemm_splitk_wgrad():
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(21)
    M, N, K = 16384, 768, 256  # wgrad: dW[N,K] = dY^T X with 16384-long reduction
    dy, x = _bf(M, N), _bf(M, K)
    out = G.linear_wgrad(dy, x)
    _close(out, dy.float().t() @ x.float(), 1e-5)
    acc = torch.randn(N, K, device=DEV)
    ref = acc + dy.float().t() @ x.float()
    G.linear_wgrad(dy, x, out=acc, accumulate=True)
    _close(acc, ref, 1e-5)


@pytest.mark.parametrize("impl", ["flash", "gemm"])
@pytest.mark.parametrize("H,Hkv,Dh,T", [(4, 4, 64, 256), (4, 2, 64, 192), (2, 1, 128, 128), (3, 3, 128, 320),
                                         (2, 2, 64, 1024), (2, 1, 128, 640)])
def test_attention_impls(monkeypatch, impl, H, Hkv, Dh, T):
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    monkeypatch.setenv("RTDC_ATTN", impl)
    torch.manual_seed(H * 100 + Dh + T)
    Bn = 2
    W = (H + 2 * Hkv) * Dh
    qkv = _bf(Bn, T, W).requires_grad_(True)
    out = causal_attention(qkv, H, Hkv)
    g = _bf(Bn, T, H * Dh)
    out.backward(g)
    qr = qkv.detach().float().requires_grad_(True)
    ref = causal_attention_ref(qr, Bn, T, H, Hkv, Dh)
    ref.backward(g.float())
    _close(out, ref, 2e-2)
    C = H * Dh
    _close(qkv.grad[..., :C], qr.grad[..., :C], 3e-2)            # dQ
    _close(qkv.grad[..., C:C + Hkv * Dh], qr.grad[..., C:C + Hkv * Dh], 3e-2)  # dK
    _close(qkv.grad[..., C + Hkv * Dh:], qr.grad[..., C + Hkv * Dh:], 3e-2)    # dV


@pytest.mark.parametrize("Dh,H,Hkv", [(64, 2, 2), (128, 2, 1)])
def test_flash_forward_lazy_rescale_branch(Dh, H, Hkv):
    """The forward kernels rescale O and l only when a row's running max grows by more than 2^8
    (a rare, data-dependent, wave-uniform branch): spike Q.K scores at LATER key blocks so the
    branch fires mid-row (twice, at key blocks 3 and 4 for query 300, once at block 6 for query
    450), and compare the whole output and the gradients against the fp32 reference
    (cdna_hip_programming.md §5.4 rule 26).  Dh 64 runs fwd_kernel, Dh 128 fwd2_kernel."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    torch.manual_seed(7)
    Bn, T = 1, 512
    C = H * Dh
    qkv = _bf(Bn, T, (H + 2 * Hkv) * Dh, scale=0.5)
    for q, k, v in [(300, 200, 1.5), (300, 290, 2.0), (450, 420, 2.0)]:
        for h in range(H):
            qkv[0, q, h * Dh:(h + 1) * Dh] = v
        for kh in range(Hkv):
            qkv[0, k, C + kh * Dh:C + (kh + 1) * Dh] = v
    qkv.requires_grad_(True)
    out = causal_attention(qkv, H, Hkv)
    g = _bf(Bn, T, C)
    out.backward(g)
    qr = qkv.detach().float().requires_grad_(True)
    ref = causal_attention_ref(qr, Bn, T, H, Hkv, Dh)
    ref.backward(g.float())
    _close(out, ref, 2e-2)
    _close(out[0, 300], ref[0, 300], 2e-2)  # the spiked rows themselves
    _close(out[0, 450], ref[0, 450], 2e-2)
    _close(qkv.grad, qr.grad, 3e-2)


def test_flash_attention_deterministic():
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention

    torch.manual_seed(31)
    qkv = _bf(2, 256, 3 * 4 * 64).requires_grad_(True)
    g = _bf(2, 256, 4 * 64)
    grads = []
    for _ in range(2):
        qkv.grad = None
        causal_attention(qkv, 4).backward(g)
        grads.append(qkv.grad.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("H,Hkv,Dh", [(12, 12, 64), (8, 2, 128)])
def test_flash_bwd_concurrent_passes_match(monkeypatch, H, Hkv, Dh):
    """RTDC_FA_CONCURRENT: delta by its own kernel, then the dQ and dK/dV passes on two streams -
    bitwise deterministic, and equal to the sequential pass up to delta's summation order."""
    from ray_torch_distributed_checkpoint_amd.ops import attention as A

    torch.manual_seed(23)
    B, T = 2, 512
    qkv = _bf(B, T, (H + 2 * Hkv) * Dh)
    g = _bf(B, T, H * Dh)
    grads = {}
    for mode in (False, True, True):
        monkeypatch.setattr(A, "_FA_CONCURRENT", mode)
        x = qkv.clone().requires_grad_(True)
        A.causal_attention(x, H, Hkv).backward(g)
        torch.cuda.synchronize()
        grads.setdefault(mode, []).append(x.grad.float())
    seq, (c1, c2) = grads[False][0], grads[True]
    assert torch.equal(c1, c2)
    assert (c1 - seq).abs().max() / seq.abs().max() < 1e-2


@pytest.mark.parametrize("M,K,N,p", [(16, 784, 512, 0.25), (16, 512, 512, 0.25), (37, 100, 130, 0.5)])
def test_fp32_linear_fused_dropout_equals_separate_kernel(M, K, N, p):
    """Linear + ReLU + Dropout as one fp32 GEMM (Philox mask in the epilogue) == the GEMM with
    the ReLU epilogue followed by the standalone dropout kernel on the same Philox stream -
    bitwise, forward and all three gradients (the fused backward reads the mask off the output)."""
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.ops.random import PhiloxStream

    torch.manual_seed(M + K)
    x0 = torch.randn(M, K, device="cuda")
    w0 = torch.randn(N, K, device="cuda") * 0.05
    b0 = torch.randn(N, device="cuda") * 0.1
    dy = torch.randn(M, N, device="cuda")

    def run(fused):
        x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        st = PhiloxStream(seed=1234, offset=77)
        if fused:
            y = ops.linear(x, w, b, relu=True, dropout=p, stream=st)
        else:
            y = ops.dropout(ops.linear(x, w, b, relu=True), p, True, st)
        y.backward(dy)
        return y.detach(), x.grad, w.grad, b.grad

    a, r = run(True), run(False)
    for u, v in zip(a, r):
        assert torch.equal(u, v)
    assert (a[0] == 0).float().mean().item() > p * 0.5  # really dropped


@pytest.mark.parametrize("n,V", [(1, 10), (63, 50257), (1000, 7), (16384, 50257), (2048, 128256), (5000, 1 << 24),
                                 (16385, 50257), (32768, 128256)])
def test_sort_ids_matches_stable_sort(n, V):
    """Native one-workgroup radix sort == torch's stable sort (ids and original positions); up to
    16384 ids the register-resident kernel, above it the chunk-loop kernel."""
    from ray_torch_distributed_checkpoint_amd.ops.embedding import sort_ids

    g = torch.Generator(device=DEV).manual_seed(n)
    ids = torch.randint(0, V, (n,), device=DEV, generator=g)
    if n >= 1000:
        ids[: n // 3] = ids[0]  # long runs of one id: the stability order matters
    s, p = sort_ids(ids, V)
    rs, rp = torch.sort(ids, stable=True)
    assert torch.equal(s, rs)
    assert torch.equal(p, rp)


def test_synth_tokens_matches_cpu_hash():
    """The native synthetic-token kernel reproduces workloads.SyntheticTokens' CPU hash."""
    from ray_torch_distributed_checkpoint_amd.workloads import SyntheticTokens

    ds = SyntheticTokens(1 << 20, 1024, 50257, seed=1234)
    ids = torch.tensor([0, 5, 1 << 19, (1 << 20) - 1, 77], dtype=torch.int64)
    ci, ct = ds.batch(ids)
    gi, gt = ds.batch(ids.to(DEV))
    assert gi.is_contiguous() and gt.is_contiguous()
    assert torch.equal(gi.cpu(), ci) and torch.equal(gt.cpu(), ct)
    assert torch.equal(gi[:, 1:], gt[:, :-1])


@pytest.mark.parametrize("a_k,b_k", [(False, False), (True, False)])
def test_gemm4w_splitk_weight_gradient(a_k, b_k):
    """4-wave kernel (cfg 10) on a long-K weight-gradient product: split-K slabs + reduce."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(31)
    Mt, N, K = 16384, 768, 512  # dW[N, K] = dY^T X over Mt tokens
    dy, x = _bf(Mt, N), _bf(Mt, K)
    A = dy if not a_k else dy.t().contiguous()
    dw = torch.empty(N, K, device=DEV, dtype=torch.float32)
    G.gemm_bf16(A, x, dw, N, K, Mt, A.shape[1], K, K, a_k, b_k, tile_cfg=10)
    _close(dw, dy.float().t() @ x.float(), 1e-5)


@pytest.mark.parametrize("Dh,qs", [(128, 2), (128, 4), (64, 4)])
def test_flash_dkdv_head_split_matches_unsplit_and_reference(monkeypatch, Dh, qs):
    """GQA dK/dV with the group's q-heads split over `qs` blocks (fp32 partials summed in a
    fixed order by dkdv_reduce_kernel): same gradients as the unsplit kernel (to fp32 rounding)
    and the fp32 reference, bitwise run to run, and the offered colsum partials match dqkv."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    torch.manual_seed(Dh + qs)
    Bn, T, H, Hkv = 1, 512, 8, 2
    W = (H + 2 * Hkv) * Dh
    qkv0 = _bf(Bn, T, W)
    g = _bf(Bn, T, H * Dh)

    def grads(split):
        monkeypatch.setenv("RTDC_FA_QS", str(split))
        qkv = qkv0.clone().requires_grad_(True)
        causal_attention(qkv, H, Hkv).backward(g)
        d2 = qkv.grad.view(-1, W)
        cs = G.colsum(d2)  # the kernels' offered 16-row partials
        torch.cuda.synchronize()
        return qkv.grad.clone(), cs.clone()

    a, cs_a = grads(qs)
    a2, _ = grads(qs)
    b, _ = grads(1)
    assert torch.equal(a, a2), "head-split backward is not deterministic"
    C = H * Dh
    _close(a[..., C:], b[..., C:], 1e-2)      # dK | dV: split vs unsplit (bf16 rounding of each)
    assert torch.equal(a[..., :C], b[..., :C])  # dQ untouched by the split
    qr = qkv0.float().requires_grad_(True)
    causal_attention_ref(qr, Bn, T, H, Hkv, Dh).backward(g.float())
    _close(a[..., C:C + Hkv * Dh], qr.grad[..., C:C + Hkv * Dh], 3e-2)
    _close(a[..., C + Hkv * Dh:], qr.grad[..., C + Hkv * Dh:], 3e-2)
    _close(cs_a, a.view(-1, W).float().sum(0), 1e-5)


@pytest.mark.parametrize("H,Hkv,T", [(4, 4, 256), (4, 2, 512), (2, 2, 1024)])
def test_flash_dkdv_32_keys_per_wave_equals_16(monkeypatch, H, Hkv, T):
    """The Dh = 64 dK/dV kernel with two 16-key groups per wave (bwd_dkdv2_kernel) computes
    every key's dK / dV with the same MFMA sequence as the 16-keys-per-wave kernel (the extra
    fully-masked q block adds exact zeros): bitwise equal gradients, colsum partials included."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(T + H)
    Dh, Bn = 64, 2
    W = (H + 2 * Hkv) * Dh
    qkv0 = _bf(Bn, T, W)
    g = _bf(Bn, T, H * Dh)
    out = {}
    for v in ("1", "2"):
        monkeypatch.setenv("RTDC_FA_DKDV", v)
        qkv = qkv0.clone().requires_grad_(True)
        causal_attention(qkv, H, Hkv).backward(g)
        cs = G.colsum(qkv.grad.view(-1, W))
        torch.cuda.synchronize()
        out[v] = (qkv.grad.clone(), cs.clone())
    assert torch.equal(out["1"][0], out["2"][0])
    _close(out["1"][1], out["2"][1], 1e-6)


@pytest.mark.parametrize("Dh,H,Hkv,T", [(64, 4, 4, 256), (64, 4, 2, 512), (64, 2, 2, 1024), (128, 4, 1, 384)])
def test_flash_dq_32_rows_per_wave_equals_16(monkeypatch, Dh, H, Hkv, T):
    """dQ with two 16-row query groups per wave (bwd_dq2_kernel, RTDC_FA_DQ=2) runs every row
    over the same key tiles in the same MFMA order as the 16-rows-per-wave kernel (a tile the
    wave's upper group reaches but its lower one does not adds exact zeros): bitwise equal
    gradients and row terms; colsum partials equal to fp32 rounding."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    torch.manual_seed(T + H + Dh)
    Bn = 2
    W = (H + 2 * Hkv) * Dh
    qkv0 = _bf(Bn, T, W)
    g = _bf(Bn, T, H * Dh)
    out = {}
    for v in ("1", "2"):
        monkeypatch.setenv("RTDC_FA_DQ", v)
        qkv = qkv0.clone().requires_grad_(True)
        causal_attention(qkv, H, Hkv).backward(g)
        cs = G.colsum(qkv.grad.view(-1, W))
        torch.cuda.synchronize()
        out[v] = (qkv.grad.clone(), cs.clone())
    assert torch.equal(out["1"][0], out["2"][0])
    _close(out["1"][1], out["2"][1], 1e-6)
    qr = qkv0.float().requires_grad_(True)
    causal_attention_ref(qr, Bn, T, H, Hkv, Dh).backward(g.float())
    _close(out["2"][0][..., :H * Dh], qr.grad[..., :H * Dh], 3e-2)


@pytest.mark.parametrize("H,Hkv,T", [(4, 1, 384), (8, 2, 512)])
def test_flash_dkdv_32_keys_per_wave_dh128(monkeypatch, H, Hkv, T):
    """Opt-in Dh = 128 dK/dV with two 16-key groups per wave (RTDC_FA_DKDV=2, occupancy 1):
    bitwise equal to the 16-keys-per-wave kernel, as at Dh = 64."""
    from ray_torch_distributed_checkpoint_amd.ops import causal_attention

    torch.manual_seed(T + H)
    Dh, Bn = 128, 2
    W = (H + 2 * Hkv) * Dh
    qkv0 = _bf(Bn, T, W)
    g = _bf(Bn, T, H * Dh)
    out = {}
    for v in ("1", "2"):
        monkeypatch.setenv("RTDC_FA_DKDV", v)
        qkv = qkv0.clone().requires_grad_(True)
        causal_attention(qkv, H, Hkv).backward(g)
        torch.cuda.synchronize()
        out[v] = qkv.grad.clone()
    assert torch.equal(out["1"], out["2"])


@pytest.mark.parametrize("M,N,K,bias", [(2048, 28672, 4096, False), (2048, 9216, 2048, True), (1024, 17408, 2048, False),
                                         (512, 33024, 8192, False)])
def test_gemm_tail_split_forward(monkeypatch, M, N, K, bias):
    """A 256x256-tile forward whose last round of tiles fills at most half the chip runs as
    whole rounds + the remaining columns on 256x128 tiles (RTDC_GEMM_TAIL, default on): equal
    to the single-launch product (same per-element K order) and to the fp32 reference."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    torch.manual_seed(M + N + K)
    x, w = _bf(M, K), _bf(N, K, scale=0.05)
    b = _bf(N) if bias else None
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("RTDC_GEMM_TAIL", v)
        out[v] = G.linear_fwd(x, w, bias=b)
        torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    _close(out["1"], ref, 1e-2)
    _close(out["1"], out["0"], 1e-2)
    print("bitwise equal:", torch.equal(out["1"], out["0"]))
    if M == 512:
        # a 4-tile tail over K = 8192 is a split-K candidate on its own: the tail launch must
        # still accumulate in one pass, i.e. bitwise the single launch
        assert torch.equal(out["1"], out["0"])


@pytest.mark.parametrize("H,Hkv,T", [(4, 4, 64), (4, 4, 256), (4, 2, 512), (2, 2, 1024)])
def test_flash_forward_pipelined_equals_plain(monkeypatch, H, Hkv, T):
    """Forward with the next key tile's scores issued before this tile's softmax (fwd3_kernel,
    RTDC_FA_FWD=3: 3-slot K ring, 2-slot V ring) performs the same operations in the same
    order as the 16-rows-per-wave kernel: bitwise equal output and row log-sum-exp, including
    one-tile (T = 64) and two-tile heads."""
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention_ref

    torch.manual_seed(T + H)
    Dh, Bn = 64, 2
    W = (H + 2 * Hkv) * Dh
    qkv = _bf(Bn, T, W)
    ext = gpu_ext()
    res = {}
    for v in ("1", "3"):
        monkeypatch.setenv("RTDC_FA_FWD", v)
        o = torch.empty((Bn, T, H * Dh), dtype=torch.bfloat16, device="cuda")
        lse = torch.empty((Bn * H, T), dtype=torch.float32, device="cuda")
        ext.flash_fwd(qkv, o, lse, Bn, T, H, Hkv, Dh, Dh ** -0.5)
        torch.cuda.synchronize()
        res[v] = (o, lse)
    assert torch.equal(res["1"][0], res["3"][0])
    assert torch.equal(res["1"][1], res["3"][1])
    ref = causal_attention_ref(qkv.float(), Bn, T, H, Hkv, Dh)
    _close(res["3"][0].float(), ref.view_as(res["3"][0]).float(), 3e-2)
