"""Conv / BatchNorm / pooling kernels (ResNet-18 path) vs plain PyTorch fp32 references (GPU)."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(out, ref, rel, what=""):
    err = (out.float() - ref.float()).abs().max().item()
    mag = ref.float().abs().max().item() + 1e-6
    assert err <= rel * mag, f"{what} max err {err} vs {rel}*{mag}"


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize(
    "B,H,C,Cout,k,s,p",
    [
        (2, 16, 64, 64, 3, 1, 1),  # stage conv
        (2, 16, 64, 128, 3, 2, 1),  # strided stage entry
        (2, 16, 64, 128, 1, 2, 0),  # projection shortcut
        (2, 32, 3, 64, 7, 2, 3),  # stem (C=3: scalar im2col, K padded 147 -> 192)
        (2, 224, 3, 64, 7, 2, 3),  # ImageNet stem: LDS-staged im2col (224 wide)
        (4, 8, 128, 64, 1, 1, 0),  # 1x1/s1: direct (no im2col)
        (1, 7, 64, 64, 3, 1, 1),  # M = 49: rows padded to 64
        (2, 14, 128, 256, 3, 1, 1),  # implicit GEMM, 128x128 tiles
        (4, 28, 128, 64, 3, 1, 1),  # Cout = 64: 256x64 fwd tile, 64x256 wgrad tile
        (2, 9, 64, 64, 3, 2, 1),  # odd spatial size, strided
        (3, 56, 64, 64, 3, 1, 1),  # 3x3/s1 weight gradient with input reuse: one row per chunk, split
        (2, 9, 64, 64, 3, 1, 1),  # ... 7 rows per chunk, the second chunk of each image partial
        (2, 7, 512, 256, 3, 1, 1),  # (many output tiles: the implicit GEMM)
        (2, 28, 128, 128, 3, 1, 1),  # ... four output tiles, two rows per chunk
        (1, 5, 64, 128, 3, 1, 1),  # ... one chunk per image (5 of 12 rows), two tiles
        (1, 64, 64, 64, 3, 1, 1),  # ... halo too large (W = 64): the implicit GEMM takes it
    ],
)
def test_conv2d(B, H, C, Cout, k, s, p):
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(B * H + C + k)
    x = torch.randn(B, C, H, H, device=DEV)
    w = torch.randn(Cout, C, k, k, device=DEV) * 0.1
    xb = x.to(torch.bfloat16)
    ref_x = xb.float().requires_grad_(C != 3)
    ref_w = w.to(torch.bfloat16).float().requires_grad_(True)
    ref = F.conv2d(ref_x, ref_w, stride=s, padding=p)
    gy = torch.randn_like(ref)
    ref.backward(gy)

    xin = _nhwc(xb).requires_grad_(C != 3)
    wp = w.clone().requires_grad_(True)
    y = cnn.conv2d(xin, wp, s, p)
    assert y.shape == (B, ref.shape[2], ref.shape[3], Cout)
    _close(y, _nhwc(ref), 0.02, "y")
    y.backward(_nhwc(gy).to(torch.bfloat16))
    _close(wp.grad, ref_w.grad, 0.02, "dw")
    if C != 3:
        _close(xin.grad, _nhwc(ref_x.grad), 0.03, "dx")


@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("B,H,C", [(4, 14, 64), (2, 7, 512), (8, 56, 64)])
def test_batch_norm_train(relu, res, B, H, C):
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(C + H)
    x = (torch.randn(B, H, H, C, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    r = torch.randn(B, H, H, C, device=DEV).to(torch.bfloat16) if res else None
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.1
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()

    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    ref = F.batch_norm(xr.permute(0, 3, 1, 2), rm2, rv2, gr, br, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    if res:
        ref = ref + rr
    if relu:
        ref = torch.relu(ref)
    gy = torch.randn_like(ref)
    ref.backward(gy)

    xi = x.clone().requires_grad_(True)
    gi, bi = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ri = r.clone().requires_grad_(True) if res else None
    y = cnn.batch_norm(xi, gi, bi, rm, rv, True, 0.1, 1e-5, residual=ri, relu=relu)
    _close(y, ref, 0.02, "y")
    _close(rm, rm2, 1e-4, "running_mean")
    _close(rv, rv2, 1e-4, "running_var")
    y.backward(gy.to(torch.bfloat16))
    _close(xi.grad, xr.grad, 0.03, "dx")
    _close(gi.grad, gr.grad, 0.01, "dgamma")
    _close(bi.grad, br.grad, 0.01, "dbeta")
    if res:
        _close(ri.grad, rr.grad, 0.01, "dres")


def test_batch_norm_eval_and_determinism():
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(3)
    C = 128
    x = (torch.randn(16, 28, 28, C, device=DEV) + 3).to(torch.bfloat16)
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    outs = []
    for _ in range(2):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        outs.append((cnn.batch_norm(x, g, b, rm, rv, True), rm, rv))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    rm, rv = outs[0][1], outs[0][2]
    y = cnn.batch_norm(x, g, b, rm, rv, False, relu=True)
    ref = torch.relu(F.batch_norm(x.float().permute(0, 3, 1, 2), rm, rv, g, b, False).permute(0, 2, 3, 1))
    _close(y, ref, 0.02, "eval")


@pytest.mark.parametrize("hw,stats", [(56, True), (28, False), (27, True)])
@pytest.mark.parametrize("gather_bwd", [False, True])
def test_stem_bn_relu_maxpool_equals_unfused(hw, stats, gather_bwd, monkeypatch):
    """The stem's one-pass BN + ReLU + 3x3/2 max-pool == batch_norm(relu) then max_pool2d,
    bitwise: output, running statistics and every gradient (x, gamma, beta) - including with
    the BatchNorm statistics handed over by a convolution epilogue.  gather_bwd: the backward
    that never stores the pool gradient (pool_bn_bwd) - its (sum g, sum g xhat) reduction runs
    in another order, so dgamma / dbeta / dx are compared to rounding, and it is checked to be
    run-to-run bitwise."""
    import importlib

    cnn = importlib.import_module("ray_torch_distributed_checkpoint_amd.ops.cnn")
    monkeypatch.setattr(cnn, "_POOL_BN_FUSED", gather_bwd)

    torch.manual_seed(hw)
    C = 64
    if stats:
        x0 = (torch.randn(4, hw, hw, C, device=DEV) + 0.3).bfloat16()
        w = (torch.randn(C, C, 3, 3, device=DEV) * 0.05).requires_grad_(True)
        y0 = cnn.conv2d(x0, w, 1, 1, bn_stats=True)
        x = y0.detach()
        x._rtdc_bn_stats = y0._rtdc_bn_stats
    else:
        x = (torch.randn(4, hw, hw, C, device=DEV) * 2 - 0.5).bfloat16()
    g0 = torch.randn(C, device=DEV)  # negative gammas too: the window max is not a monotone map
    b0 = torch.randn(C, device=DEV) * 0.5
    outs = []
    for fused in (False, True):
        g, b = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        xi = x.detach().clone().requires_grad_(True)
        if stats:
            xi._rtdc_bn_stats = x._rtdc_bn_stats
        if fused:
            y = cnn.batch_norm_relu_max_pool(xi, g, b, rm, rv, True, 0.1, 1e-5)
        else:
            y = cnn.max_pool2d(cnn.batch_norm(xi, g, b, rm, rv, True, 0.1, 1e-5, relu=True), 3, 2, 1)
        gy = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)).bfloat16()
        y.backward(gy)
        outs.append((y, rm, rv, xi.grad, g.grad, b.grad))
    names = ("y", "running_mean", "running_var", "dx", "dgamma", "dbeta")
    for n, a, b in zip(names, outs[0], outs[1]):
        if gather_bwd and n in ("dx", "dgamma", "dbeta"):
            _close(b, a, 2e-2 if n == "dx" else 1e-4, n)
        else:
            assert torch.equal(a, b), f"{n} differs between the fused and the unfused stem"
    if gather_bwd:  # deterministic: a second fused backward is bitwise the first
        g, b = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        xi = x.detach().clone().requires_grad_(True)
        if stats:
            xi._rtdc_bn_stats = x._rtdc_bn_stats
        y = cnn.batch_norm_relu_max_pool(xi, g, b, torch.zeros(C, device=DEV), torch.ones(C, device=DEV), True, 0.1,
                                         1e-5)
        y.backward(torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)).bfloat16())
        for n, a, b2 in zip(("dx", "dgamma", "dbeta"), outs[1][3:], (xi.grad, g.grad, b.grad)):
            assert torch.equal(a, b2), f"{n}: fused stem backward not run-to-run bitwise"
    # and against fp32 torch
    xr = x.float().requires_grad_(True)
    ref = F.max_pool2d(torch.relu(F.batch_norm(xr.permute(0, 3, 1, 2), None, None, g0, b0, True)), 3, 2, 1)
    _close(outs[1][0], _nhwc(ref), 0.02, "y vs torch")


@pytest.mark.parametrize("B,H", [(2, 224), (3, 64), (2, 36)])
def test_stem_space_to_depth_conv_matches_torch(B, H):
    """The 7x7/2 stem as a 4x4/1 implicit GEMM over the space-to-depth image == F.conv2d (fp32
    reference on the same bf16-rounded operands): output, fused BN statistics, weight gradient
    (written through the channels-last gradient slot); and == the im2col path."""
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(B * H)
    x = torch.randn(B, 3, H, H, device=DEV)
    w = (torch.randn(64, 3, 7, 7, device=DEV) * 0.1).to(memory_format=torch.channels_last).requires_grad_(True)
    assert cnn.stem_supported(x, w, 2, 3)
    y = cnn.stem_conv(x, w, bn_stats=True)
    xr = x.bfloat16().float()
    wr = w.detach().bfloat16().float().requires_grad_(True)
    ref = F.conv2d(xr, wr, stride=2, padding=3).permute(0, 2, 3, 1)
    _close(y, ref, 0.01, "stem y")
    st = y._rtdc_bn_stats
    mean_tiles, rows = st[0], st[2]
    yf = y.float().reshape(-1, 64)
    n_full = yf.shape[0] // rows
    if n_full:
        torch.testing.assert_close(mean_tiles[:n_full], yf[: n_full * rows].view(n_full, rows, 64).mean(1),
                                   rtol=1e-3, atol=1e-3)
    gy = torch.randn(y.shape, device=DEV).bfloat16()
    y.backward(gy)
    ref.backward(gy.float())
    _close(w.grad, wr.grad, 0.01, "stem dW")
    # the generic im2col path on the NHWC bf16 image gives the same output
    y2 = cnn.conv2d(cnn.to_nhwc_bf16(x), w.detach(), 2, 3)
    _close(y, y2, 0.01, "stem vs im2col")


def test_pools_and_classifier():
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(5)
    for hw in (28, 27):  # even / odd size (the odd one has a partial last window)
        x = torch.randn(4, 64, hw, hw, device=DEV).to(torch.bfloat16)
        xr = x.float().requires_grad_(True)
        ref = F.max_pool2d(xr, 3, 2, 1)
        gy = torch.randn_like(ref)
        ref.backward(gy)
        xi = _nhwc(x).requires_grad_(True)
        y = cnn.max_pool2d(xi, 3, 2, 1)
        _close(y, _nhwc(ref), 1e-6, "maxpool")
        y.backward(_nhwc(gy).to(torch.bfloat16))
        _close(xi.grad, _nhwc(xr.grad), 0.01, "maxpool dx")

    xa = torch.randn(6, 7, 7, 512, device=DEV).to(torch.bfloat16)
    xar = xa.float().requires_grad_(True)
    ref = xar.mean((1, 2))
    g2 = torch.randn_like(ref)
    ref.backward(g2)
    xai = xa.clone().requires_grad_(True)
    y = cnn.global_avg_pool(xai)
    _close(y, ref, 0.01, "avgpool")
    y.backward(g2.to(torch.bfloat16))
    _close(xai.grad, xar.grad, 0.01, "avgpool dx")

    h = torch.randn(6, 512, device=DEV).to(torch.bfloat16)
    w, b = torch.randn(10, 512, device=DEV) * 0.05, torch.randn(10, device=DEV)
    hr, wr, br = h.float().requires_grad_(True), w.to(torch.bfloat16).float().requires_grad_(True), b.clone().requires_grad_(True)
    ref = F.linear(hr, wr, br)
    g3 = torch.randn_like(ref)
    ref.backward(g3)
    hi, wi, bi = h.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = cnn.classifier(hi, wi, bi)
    _close(y, ref, 0.02, "fc")
    y.backward(g3.to(torch.bfloat16))
    _close(hi.grad, hr.grad, 0.02, "fc dx")
    _close(wi.grad, wr.grad, 0.02, "fc dw")
    _close(bi.grad, br.grad, 0.01, "fc db")

    # ImageNet head shape class (N % 8 == 0, batch % 64 == 0): unpadded forward / weight
    # gradient, padded reduction axis only in the input gradient
    for N in (1000, 1024):
        h = torch.randn(64, 512, device=DEV).to(torch.bfloat16)
        w, b = torch.randn(N, 512, device=DEV) * 0.05, torch.randn(N, device=DEV)
        hr = h.float().requires_grad_(True)
        wr, br = w.to(torch.bfloat16).float().requires_grad_(True), b.clone().requires_grad_(True)
        ref = F.linear(hr, wr, br)
        g3 = torch.randn_like(ref)
        ref.backward(g3)
        hi, wi, bi = h.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        y = cnn.classifier(hi, wi, bi)
        _close(y, ref, 0.02, f"fc{N}")
        y.backward(g3.to(torch.bfloat16))
        _close(hi.grad, hr.grad, 0.02, f"fc{N} dx")
        _close(wi.grad, wr.grad, 0.02, f"fc{N} dw")
        _close(bi.grad, br.grad, 0.01, f"fc{N} db")


def _bf16_emulated_grads(model, x, t):
    """CPU fp32 reference with every conv/BN output (and its gradient) rounded to bf16: the
    precision floor a bf16 network can reach, used to calibrate the GPU comparison."""
    from ray_torch_distributed_checkpoint_amd.models import resnet as R
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    oc, ob = cnn.conv2d, cnn.batch_norm
    R.cnn.conv2d = lambda x_, w, s=1, p=0, bn_stats=False, grad_accum=None: oc(x_, w.bfloat16().float(), s, p).bfloat16().float()
    R.cnn.batch_norm = lambda *a, **k: ob(*a, **k).bfloat16().float()
    try:
        F.cross_entropy(model(x), t).backward()
    finally:
        R.cnn.conv2d, R.cnn.batch_norm = oc, ob
    return {n: p.grad for n, p in model.named_parameters()}


def test_resnet18_matches_reference_and_trains():
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.models import ResNet18
    from ray_torch_distributed_checkpoint_amd.optim import FusedSGD

    torch.manual_seed(0)
    ref = ResNet18(10)
    emu = copy.deepcopy(ref)
    gpu = copy.deepcopy(ref).cuda()
    x = torch.randn(8, 3, 64, 64)
    t = torch.randint(0, 10, (8,))
    lr = F.cross_entropy(ref(x), t)
    lr.backward()
    emu_grads = _bf16_emulated_grads(emu, x, t)
    lg = ops.cross_entropy(gpu(x.cuda()), t.cuda())
    lg.backward()
    assert abs(lg.item() - lr.item()) < 0.05 * lr.item() + 0.02
    for (n, p), (_, q) in zip(ref.named_parameters(), gpu.named_parameters()):
        cos_gpu = F.cosine_similarity(p.grad.flatten(), q.grad.cpu().flatten(), dim=0).item()
        cos_emu = F.cosine_similarity(p.grad.flatten(), emu_grads[n].flatten(), dim=0).item()
        assert cos_gpu > min(0.97, cos_emu - 0.05), f"{n}: cos(gpu, fp32)={cos_gpu:.4f} vs bf16 floor {cos_emu:.4f}"
    for (n, b1), (_, b2) in zip(ref.named_buffers(), gpu.named_buffers()):
        _close(b2.cpu(), b1, 0.02, n)
    opt = FusedSGD(gpu.parameters(), lr=0.05, momentum=0.9)
    xs = torch.randn(16, 3, 64, 64, device=DEV)
    ts = torch.randint(0, 10, (16,), device=DEV)
    losses = []
    for _ in range(15):
        opt.zero_grad()
        l = ops.cross_entropy(gpu(xs), ts)
        l.backward()
        opt.step()
        losses.append(l.item())
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.parametrize("B,H,C,Cout,s", [(4, 28, 64, 64, 1), (2, 14, 128, 256, 2), (2, 13, 64, 128, 1),
                                             (16, 56, 64, 64, 1), (3, 30, 64, 128, 1)])
def test_conv_fused_bn_statistics(B, H, C, Cout, s):
    """BatchNorm statistics computed in the implicit-GEMM epilogue == the separate pass (the
    larger shapes merge hundreds of tile partials through the split merge, with a partial last
    split)."""
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(B + H + Cout)
    x = (torch.randn(B, H, H, C, device=DEV) + 0.7).to(torch.bfloat16)
    w = torch.randn(Cout, C, 3, 3, device=DEV) * 0.1
    y = cnn.conv2d(x, w.requires_grad_(True), s, 1, bn_stats=True)
    assert getattr(y, "_rtdc_bn_stats", None) is not None
    g, b = torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV)
    rm1, rv1 = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    out_fused = cnn.batch_norm(y, g, b, rm1, rv1, True, relu=True)
    out_ref = cnn.batch_norm(y.detach().clone(), g, b, rm2, rv2, True, relu=True)
    _close(out_fused, out_ref, 0.01, "y")
    _close(rm1, rm2, 1e-4, "running_mean")
    _close(rv1, rv2, 1e-4, "running_var")


@pytest.mark.parametrize("shortcut", ["identity", "downsample"])
def test_grad_join_matches_autograd_add(shortcut):
    """GradStash: the block input's two gradients summed inside the dgrad kernels (implicit GEMM
    epilogue / col2im addend / BN residual) == autograd's own add, in either backward order."""
    from ray_torch_distributed_checkpoint_amd.ops import cnn

    torch.manual_seed(0)
    B, H, C = 4, 16, 64
    Cout = C if shortcut == "identity" else 128
    s = 1 if shortcut == "identity" else 2
    x0 = torch.randn(B, H, H, C, device=DEV).bfloat16()
    w1 = (torch.randn(Cout, C, 3, 3, device=DEV) * 0.05)
    wd = (torch.randn(Cout, C, 1, 1, device=DEV) * 0.1)
    g = torch.ones(Cout, device=DEV)
    b = torch.zeros(Cout, device=DEV)
    dy = torch.randn(B, H // s, H // s, Cout, device=DEV).bfloat16()

    def run(join):
        x = x0.clone().requires_grad_(True)
        st = cnn.GradStash(2) if join else None
        h = cnn.conv2d(x, w1, s, 1, grad_accum=st)
        rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
        if shortcut == "identity":
            y = cnn.batch_norm(h, g, b, rm, rv, True, residual=x, relu=True, residual_grad_to=st)
        else:
            sc = cnn.conv2d(x, wd, s, 0, grad_accum=st)
            y = cnn.batch_norm(h, g, b, rm, rv, True, residual=sc, relu=True)
        y.backward(dy)
        return x.grad.float()

    ref, got = run(False), run(True)
    err = (got - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("residual", [False, True])
def test_bn_backward_statistics_in_dgrad_epilogue(C, residual, monkeypatch):
    """conv1 -> BN + ReLU -> conv2 (stride 1): with RTDC_BNB_FUSED the BatchNorm backward's
    statistics come from conv2's dgrad epilogue (conv_gemm_bnb) instead of a pass over the
    gradient - same gradients to rounding, against the unfused path and fp32 torch, including a
    partial last row tile; run-to-run bitwise."""
    import importlib

    cnn = importlib.import_module("ray_torch_distributed_checkpoint_amd.ops.cnn")
    torch.manual_seed(C)
    B, H = 3, 13  # 507 pixels: partial last tile for 128- and 256-row tiles
    x0 = torch.randn(B, H, H, C, device=DEV).bfloat16()
    w1 = torch.randn(C, C, 3, 3, device=DEV) * 0.05
    w2 = torch.randn(C, C, 3, 3, device=DEV) * 0.05
    g0 = torch.randn(C, device=DEV)
    b0 = torch.randn(C, device=DEV) * 0.5
    dy = torch.randn(B, H, H, C, device=DEV).bfloat16()
    taken = []
    orig = cnn._take_bnb

    def spy(g):
        r = orig(g)
        taken.append(r is not None)
        return r

    monkeypatch.setattr(cnn, "_take_bnb", spy)

    def run(fused):
        monkeypatch.setattr(cnn, "_BNB_FUSED", fused)
        x = x0.clone().requires_grad_(True)
        g, b = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        h = cnn.conv2d(x, w1, 1, 1)
        # residual: relu(BN(h) + x) - the backward's mask comes from the output (bnb_y)
        z = cnn.batch_norm(h, g, b, rm, rv, True, relu=True, residual=x if residual else None)
        y = cnn.conv2d(z, w2, 1, 1)
        y.backward(dy)
        run.h = h.detach()
        return [t.grad.float().clone() for t in (x, g, b)]

    ref = run(False)
    assert taken == [False]
    got = run(True)
    assert taken == [False, True]
    again = run(True)
    for n, a, r, a2 in zip(("dx", "dgamma", "dbeta"), got, ref, again):
        _close(a, r, 1e-2 if n == "dx" else 1e-4, n)
        assert torch.equal(a, a2), f"{n}: not run-to-run bitwise"
    # fp32 torch from the same bf16 BatchNorm input (a conv output recomputed in fp32 would move
    # elements across the ReLU boundary and change dbeta by whole gradient values)
    gr, br = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    hr = run.h.float().permute(0, 3, 1, 2)
    zr = F.batch_norm(hr, None, None, gr, br, True)
    if residual:
        zr = zr + x0.float().permute(0, 3, 1, 2)
    zr = torch.relu(zr)
    yr = F.conv2d(zr, w2.bfloat16().float(), padding=1)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    _close(got[1], gr.grad, 3e-2, "dgamma vs torch")
    _close(got[2], br.grad, 3e-2, "dbeta vs torch")
