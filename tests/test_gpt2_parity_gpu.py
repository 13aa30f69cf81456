"""GPT-2-small at its production shape (T=1024, B=2) on the native bf16 kernels vs a plain
PyTorch fp32 implementation with IDENTICAL initial weights, data and AdamW hyper-parameters,
for 5 optimizer steps.  The full-size shapes select the kernel variants the tiny models never
reach (persistent 256x256 / 256x192 GEMMs, split-K wgrad, fused column sums, the flash kernel
at T=1024, the 50304-wide fused LM head); the per-step loss must stay within 1e-2 relative
of the fp32 reference."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_loss(P, idx, tgt, cfg):
    """fp32 GPT-2 forward from a name -> tensor dict with our state-dict names."""
    B, T = idx.shape
    C, H = cfg.n_embd, cfg.n_head
    x = F.embedding(idx, P["wte"]) + P["wpe"][:T]
    for i in range(cfg.n_layer):
        p = lambda n: P[f"h.{i}.{n}"]  # noqa: E731
        h = F.layer_norm(x, (C,), p("ln_1.weight"), p("ln_1.bias"), cfg.layer_norm_eps)
        qkv = F.linear(h, p("attn.c_attn.weight"), p("attn.c_attn.bias"))
        q, k, v = (t.reshape(B, T, H, C // H).transpose(1, 2) for t in qkv.split(C, dim=-1))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, C)
        x = x + F.linear(y, p("attn.c_proj.weight"), p("attn.c_proj.bias"))
        h = F.layer_norm(x, (C,), p("ln_2.weight"), p("ln_2.bias"), cfg.layer_norm_eps)
        h = F.gelu(F.linear(h, p("mlp.c_fc.weight"), p("mlp.c_fc.bias")), approximate="tanh")
        x = x + F.linear(h, p("mlp.c_proj.weight"), p("mlp.c_proj.bias"))
    x = F.layer_norm(x, (C,), P["ln_f.weight"], P["ln_f.bias"], cfg.layer_norm_eps)
    logits = F.linear(x, P["wte"][: cfg.vocab_size])
    return F.cross_entropy(logits.reshape(-1, cfg.vocab_size), tgt.reshape(-1))


def test_gpt2_small_full_shape_matches_fp32_reference():
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW

    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    cfg = GPT2Config.named("gpt2-small")
    torch.manual_seed(0)
    model = GPT2(cfg)
    P = {k: v.detach().clone().to(dev).requires_grad_(True) for k, v in model.state_dict().items()}
    model = model.to(dev)
    hp = dict(lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    opt = FusedAdamW(model.parameters(), **hp)
    ref_opt = torch.optim.AdamW(list(P.values()), foreach=False, **hp)
    g = torch.Generator().manual_seed(1)
    data = [torch.randint(0, cfg.vocab_size, (2, 1025), generator=g).to(dev) for _ in range(5)]
    rel = []
    for d in data:
        loss = model(d[:, :-1], d[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        ref = _ref_loss(P, d[:, :-1], d[:, 1:], cfg)
        ref.backward()
        ref_opt.step()
        ref_opt.zero_grad()
        a, b = float(loss.detach()), float(ref.detach())
        assert math.isfinite(a)
        rel.append(abs(a - b) / abs(b))
    print("per-step relative loss error:", [f"{r:.2e}" for r in rel])
    assert max(rel) < 1e-2, rel
    # the weights moved the same way too (AdamW normalises each element's update, so bf16
    # rounding of near-zero gradients shows up as ~1% on the small-init residual projections)
    for name in ("wte", "h.0.attn.c_attn.weight", "h.11.mlp.c_proj.weight", "ln_f.weight"):
        ours = dict(model.named_parameters())[name].detach()
        err = (ours - P[name].detach()).norm() / P[name].detach().norm()
        assert err < 3e-2, (name, float(err))


def test_gpt2_small_full_shape_per_parameter_gradients_match_fp32():
    """Every parameter's gradient after one backward at the production shape (B=2, T=1024,
    768 wide, 12 layers, 50304-wide tied head) within 1.5e-2 relative norm (LayerNorm scales
    2e-2; measured maxima 1.09e-2 / 1.19e-2, see below) of an fp32 twin that
    starts from the same bf16-representable weights - so a wrong gradient on any single
    parameter family (a transposed wgrad, a dropped bias colsum, a mis-scaled tied head) fails
    here even when the loss trajectory still looks right."""
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    cfg = GPT2Config.named("gpt2-small")
    torch.manual_seed(0)
    model = GPT2(cfg)
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.bfloat16().float())  # masters == their bf16 compute shadows
    P = {k: v.detach().clone().to(dev).requires_grad_(True) for k, v in model.state_dict().items()}
    model = model.to(dev)
    g = torch.Generator().manual_seed(2)
    d = torch.randint(0, cfg.vocab_size, (2, 1025), generator=g).to(dev)
    model(d[:, :-1], d[:, 1:]).backward()
    _ref_loss(P, d[:, :-1], d[:, 1:], cfg).backward()
    torch.cuda.synchronize()
    worst = []
    for n, p in model.named_parameters():
        r = P[n].grad
        if n == "wte":
            r = r[: p.shape[0]]
        err = float((p.grad.float() - r).norm() / (r.norm() + 1e-30))
        worst.append((err, n))
    worst.sort(reverse=True)
    print("worst per-parameter relative gradient errors:", [(n, f"{e:.2e}") for e, n in worst[:6]])
    # What bf16 activation storage costs against the fp32 twin (which keeps the residual stream,
    # LayerNorm outputs and the GELU pre-activation in fp32), measured on MI355X: <= 1.1e-2 on
    # the weight matrices (c_fc: 1.07-1.09e-2 on every layer) and up to 1.2e-2 on the LayerNorm
    # scales (dgamma = sum_rows dy * xhat, a cancelling sum) - uniform across layers, as expected
    # of random-init statistics.  A wrong gradient (transposed / dropped / mis-scaled term) is
    # off by O(1); the bounds below leave ~35 % headroom over the measured storage error.
    bad = [(e, n) for e, n in worst if e >= (2e-2 if n.endswith(("ln_1.weight", "ln_2.weight", "ln_f.weight"))
                                             else 1.5e-2)]
    assert not bad, bad[:6]


def test_llama3_8b_decoder_layer_full_width_gradients_match_fp32():
    """One Llama-3-8B decoder layer at full width (dim 4096, GQA 32/8 heads x 128, SwiGLU 14336,
    RoPE theta 5e5) on the native kernels vs the same layer's fp32 PyTorch path (CPU) from the
    same bf16-representable weights: output, input gradient and every weight gradient within
    1.5e-2 relative norm (measured <= 1.03e-2)."""
    from ray_torch_distributed_checkpoint_amd.models.llama import LlamaConfig, TransformerBlock

    cfg = LlamaConfig.named("llama3-8b")
    torch.manual_seed(0)
    ref = TransformerBlock(cfg)
    with torch.no_grad():
        for p in ref.parameters():
            if p.dim() > 1:
                torch.nn.init.normal_(p, std=0.02)
            p.copy_(p.bfloat16().float())
    import copy

    gpu = copy.deepcopy(ref).cuda()
    B, T = 1, 512
    x = (torch.randn(B, T, cfg.dim) * 0.5).bfloat16()
    gy = torch.randn(B, T, cfg.dim).bfloat16()
    xr = x.float().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy.float())
    xg = x.cuda().requires_grad_(True)
    yg = gpu(xg)
    yg.backward(gy.cuda())
    torch.cuda.synchronize()

    def rel(a, b):
        return float((a.float().cpu() - b).norm() / (b.norm() + 1e-30))

    errs = {"y": rel(yg, yr.detach()), "dx": rel(xg.grad, xr.grad)}
    for (n, p), (_, q) in zip(ref.named_parameters(), gpu.named_parameters()):
        errs[n] = rel(q.grad, p.grad)
    print({k: f"{v:.2e}" for k, v in errs.items()})
    # measured on MI355X: y 7.4e-3, dx 9.4e-3, weights 7.4e-3 .. 1.03e-2 (wqkv, attention_norm) -
    # the bf16 activation storage against the fp32 twin; same bounds as the GPT-2 test
    bad = {k: v for k, v in errs.items() if not v < 1.5e-2}
    assert not bad, bad
