"""Grouped weight gradients (ops/gemm.py `_WgradGroup`, gemm_8ph.hip `gemm8g_kernel`).

* the grouped launch of GPT-2's four linear weight-gradient shapes equals an fp32 reference;
* a model's backward with deferral on gives the gradients of the immediate (split-K) path;
* two DDP ranks (gloo, sharing cuda:0) whose buckets hold deferred gradients all-reduce the
  final values - a bucket collective launched before the grouped kernel wrote its slice would
  average garbage.
"""
import os
import socket
import sys
import traceback

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]  # (N out, K in) of qkv / proj / fc / mlp_proj


def test_grouped_wgrad_matches_fp32_reference():
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    torch.manual_seed(0)
    M = 4096
    dev = torch.device("cuda", 0)
    dys, xs, outs, dims = [], [], [], []
    for N, K in SHAPES * 2:  # two layers: 8 products, 216 tiles
        dys.append(torch.randn(M, N, device=dev).bfloat16())
        xs.append(torch.randn(M, K, device=dev).bfloat16())
        outs.append(torch.full((N, K), float("nan"), device=dev))
        dims += [N, K, M, N, K, K]
    gpu_ext().gemm_bf16_grouped(dys, xs, outs, dims, False, False)
    torch.cuda.synchronize()
    for dy, x, out in zip(dys, xs, outs):
        ref = dy.float().t() @ x.float()
        err = (out - ref).norm() / ref.norm()
        assert torch.isfinite(out).all() and err < 1e-5, f"{tuple(out.shape)}: {err:.3e}"


def test_grouped_wgrad_persistent_multi_round_ragged():
    """The persistent grouped kernel (gemm8gp_kernel: one block per CU walking several tiles,
    products switching mid-run, edge tiles of N = 1000 / K-in = 2736) against fp32: K = 2048
    tokens like a Llama-3-8B layer, 332 tiles > one round of the chip."""
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    torch.manual_seed(1)
    M = 2048
    dev = torch.device("cuda", 0)
    dys, xs, outs, dims = [], [], [], []
    for N, K in [(4096, 4096), (1000, 2736), (2048, 1024)]:
        dys.append(torch.randn(M, N, device=dev).bfloat16())
        xs.append(torch.randn(M, K, device=dev).bfloat16())
        outs.append(torch.full((N, K), float("nan"), device=dev))
        dims += [N, K, M, N, K, K]
    gpu_ext().gemm_bf16_grouped(dys, xs, outs, dims, False, False)
    torch.cuda.synchronize()
    for dy, x, out in zip(dys, xs, outs):
        ref = dy.float().t() @ x.float()
        err = (out - ref).norm() / ref.norm()
        assert torch.isfinite(out).all() and err < 1e-5, f"{tuple(out.shape)}: {err:.3e}"
    # run-to-run bitwise (fixed per-tile K order)
    again = [torch.empty_like(o) for o in outs]
    gpu_ext().gemm_bf16_grouped(dys, xs, again, dims, False, False)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(outs, again))


def _mlp_model(dev, n_layer=2):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=1024, n_positions=1024, n_embd=768, n_layer=n_layer, n_head=12)
    return GPT2(cfg).to(dev)


def _grads(group_on: bool, data, n_layer=2):
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    old = G._GROUP_ON
    G._GROUP_ON = group_on
    try:
        dev = data.device
        model = _mlp_model(dev, n_layer)
        sp = FlatParamSpace(list(reversed(list(model.parameters()))))
        sp.zero_grad(set_to_none=True)  # fresh mode: gradients written into the flat buffer
        loss = model(data[:, :-1], data[:, 1:])
        loss.backward()
        torch.cuda.synchronize()
        assert not G._WG.items and not G._WG.waiters
        return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}
    finally:
        G._GROUP_ON = old


def test_model_backward_grouped_equals_immediate():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    data = torch.randint(0, 1024, (4, 1025), generator=g).to(dev)  # 4096 tokens: groupable
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    launched = []
    orig = G._WgradGroup.flush

    def spy(self, *a, **k):
        launched.append(len(self.items))
        return orig(self, *a, **k)

    G._WgradGroup.flush = spy
    try:
        a = _grads(True, data)
    finally:
        G._WgradGroup.flush = orig
    assert sum(launched) == 8, launched  # 2 layers x 4 linear weight gradients went through the group
    b = _grads(False, data)
    for n in a:
        err = (a[n] - b[n]).norm() / b[n].norm().clamp_min(1e-12)
        assert err < 1e-4, f"{n}: {err:.3e}"


def test_small_remainder_goes_split_k_and_equals_immediate():
    """One layer's four products are 108 tiles, under half a round: the end-of-backward flush
    launches them one by one with split-K - bitwise the immediate path."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    data = torch.randint(0, 1024, (4, 1025), generator=g).to(dev)
    a = _grads(True, data, n_layer=1)
    b = _grads(False, data, n_layer=1)
    for n in a:
        assert torch.equal(a[n], b[n]), n


def test_deferred_colsums_bitwise_equal_immediate():
    """Bias / LayerNorm-parameter gradients reduced in the deferred window (one colsum_multi
    launch per flush) are bitwise the immediate reductions."""
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    data = torch.randint(0, 1024, (4, 1025), generator=g).to(dev)
    njobs = []
    orig = G._WgradGroup._launch_jobs

    def spy(jobs):
        njobs.append(len(jobs))
        return orig(jobs)

    G._WgradGroup._launch_jobs = staticmethod(spy)
    try:
        a = _grads(True, data, n_layer=3)
    finally:
        G._WgradGroup._launch_jobs = staticmethod(orig)
    # per layer: ln_1 / ln_2 (dgamma, dbeta, dx colsum = the residual projections' biases),
    # c_attn bias, c_fc bias; + ln_f
    assert sum(njobs) >= 3 * 8, njobs
    assert not G._WG.jobs
    old = G._DEFER_ON
    G._DEFER_ON = False
    try:
        b = _grads(True, data, n_layer=3)
    finally:
        G._DEFER_ON = old
    for n in a:
        if n.endswith("c_attn.bias"):
            # from the flash backward's 16-row partials (RTDC_COLSUM_DEFER=0: a pass over dqkv):
            # another summation order
            err = (a[n] - b[n]).abs().max() / b[n].abs().max()
            assert err < 1e-5, f"{n}: {err:.3e}"
        else:
            assert torch.equal(a[n], b[n]), n


def test_deferred_small_reductions_bitwise_equal_unflattened():
    """A handful of partial rows (128 tokens: LayerNorm backward with few blocks): the deferred
    reduction into a flat-buffer slot and the immediate one into a plain tensor sum in the same
    order - a gradient's bits must not depend on where it is written (the 1-rank RCCL DDP test
    compares exactly that)."""
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    data = torch.randint(0, 1024, (2, 65), generator=g).to(dev)

    def run(flat):
        model = _mlp_model(dev, 2)
        if flat:
            FlatParamSpace(list(reversed(list(model.parameters())))).zero_grad(set_to_none=True)
        model(data[:, :-1], data[:, 1:]).backward()
        torch.cuda.synchronize()
        return {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.dim() == 1}

    a, b = run(True), run(False)
    assert a.keys() == b.keys() and len(a) >= 8
    for n in a:
        assert torch.equal(a[n], b[n]), n


def test_colsum_multi_matches_sum():
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext

    torch.manual_seed(8)
    dev = torch.device("cuda", 0)
    shapes = [(768, 768), (64, 2304), (3, 100), (4096, 72)]
    ws = [torch.randn(W, D, device=dev) for W, D in shapes]
    outs = [torch.randn(D, device=dev) for _, D in shapes]
    base = [o.clone() for o in outs]
    acc = [0, 1, 0, 1]
    gpu_ext().colsum_multi([w.reshape(-1) for w in ws], outs, [W for W, _ in shapes], [D for _, D in shapes], acc)
    torch.cuda.synchronize()
    for w, o, b, a in zip(ws, outs, base, acc):
        ref = w.double().sum(0) + (b.double() if a else 0.0)
        assert torch.allclose(o.double(), ref, rtol=1e-5, atol=1e-4)


def test_greedy_packing_fills_rounds():
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(6)
    data = torch.randint(0, 1024, (4, 1025), generator=g).to(dev)
    sizes = []
    orig = G._WgradGroup._launch

    def spy(self, items):
        sizes.append(sum(it[3] for it in items))
        return orig(self, items)

    G._WgradGroup._launch = spy
    try:
        _grads(True, data, n_layer=5)  # 5 x 108 tiles: 252 + 252 + 36 (split-K remainder)
    finally:
        G._WgradGroup._launch = orig
    assert sizes == [252, 252], sizes


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ray_torch_distributed_checkpoint_amd.ops import gemm as G
        from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

        model = _mlp_model(dev)
        net = DistributedDataParallel(model, bucket_cap_mb=8.0, first_bucket_mb=1.0)
        g = torch.Generator().manual_seed(11)
        data = torch.randint(0, 1024, (world * 4, 1025), generator=g).to(dev)[rank * 4:(rank + 1) * 4]
        flushed = []
        orig = G._WgradGroup.flush

        def spy(self, *a, **k):
            flushed.append(len(self.items))
            return orig(self, *a, **k)

        G._WgradGroup.flush = spy
        net.space.zero_grad(set_to_none=True)
        loss = net(data[:, :-1], data[:, 1:])
        loss.backward()
        torch.cuda.synchronize()
        G._WgradGroup.flush = orig
        grads = {n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()}
        q.put((rank, "ok", (grads, sum(flushed))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def test_ddp_buckets_wait_for_grouped_wgrads():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, st, v = q.get(timeout=240)
            assert st == "ok", v
            out[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert out[0][1] == 8 and out[1][1] == 8  # every transformer weight gradient was deferred
    # reference: one process, the concatenated batch, deferral on as well
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    data = torch.randint(0, 1024, (world * 4, 1025), generator=g).to(dev)
    ref = _grads(True, data)
    for n, v in ref.items():
        g0 = torch.from_numpy(out[0][0][n])
        assert torch.equal(g0, torch.from_numpy(out[1][0][n])), f"ranks differ on {n}"
        err = (g0 - v.cpu()).norm() / v.cpu().norm().clamp_min(1e-12)
        assert err < 5e-3, f"{n}: relative error {err:.3e}"


def _shared_grads(group_on: bool, x, tied_head: bool):
    """Gradients of a weight used twice in one step - by two native linears (shared), or by an
    embedding and a linear head (tied) - with weight-gradient deferral on or off."""
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    old = G._GROUP_ON
    G._GROUP_ON = group_on
    try:
        dev = x.device
        torch.manual_seed(1)
        w = torch.nn.Parameter(torch.randn(1024, 1024, device=dev) * 0.03)
        w2 = torch.nn.Parameter(torch.randn(1024, 1024, device=dev) * 0.03)
        sp = FlatParamSpace([w2, w])
        sp.zero_grad(set_to_none=True)
        if tied_head:
            ids = ((x[:, 0].float().abs() * 1000).long() % 1024).view(4, 1024)  # [B, T] token ids
            h = ops.embedding(ids, w)
            h = ops.linear(h.bfloat16(), w2)
            y = ops.linear(h, w)  # head tied to the embedding table
        else:
            h = ops.linear(x, w, relu=True)
            h = ops.linear(h, w2)
            y = ops.linear(h, w)  # second use of w
        (y.float() ** 2).mean().backward()
        torch.cuda.synchronize()
        assert not G._WG.items and not G._WG.jobs
        return w.grad.detach().clone(), w2.grad.detach().clone()
    finally:
        G._GROUP_ON = old


@pytest.mark.parametrize("tied_head", [False, True])
def test_shared_weight_gradients_with_deferral_equal_immediate(tied_head):
    """A deferred (grouped) weight gradient is written only at the flush, overwriting its slice:
    a second contribution to the same weight in the same step must see the first one written
    (ops/gradbuf.py flushes before it), so deferral on == deferral off."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(4096, 1024, device=dev).bfloat16()  # 4096 rows: groupable products
    on = _shared_grads(True, x, tied_head)
    off = _shared_grads(False, x, tied_head)
    for a, b in zip(on, off):
        assert torch.isfinite(a).all()
        err = (a - b).norm() / b.norm()
        assert err < 1e-5, f"deferred vs immediate: {err:.3e}"


def test_short_k_multi_round_products_pack_whole_rounds():
    """Llama-3-8B at 2048 tokens/GPU: weight gradients of >= 256 tiles over a short K are packed
    until the group is a whole number of rounds (ops/gemm.py `_groupable` whole_rounds).  A chain
    of 6144x4096, 4096x6144 and 4096x4096 weights gives 384 + 384 + 256 tiles: the last layer's
    256 tiles flush alone, the other two as one 768-tile (3-round) launch - bitwise the
    one-by-one 256x256 launches (same tiles, same MFMA order)."""
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G
    from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

    dev = torch.device("cuda", 0)
    torch.manual_seed(21)
    x0 = (torch.randn(2048, 4096, device=dev) * 0.5).bfloat16()
    ws0 = [torch.randn(6144, 4096, device=dev) * 0.02, torch.randn(4096, 6144, device=dev) * 0.02,
           torch.randn(4096, 4096, device=dev) * 0.02]

    def run(big):
        old = G._GROUP_BIG
        G._GROUP_BIG = big
        sizes = []
        orig = G._WgradGroup.flush

        def spy(self, *a, **k):
            if self.items:
                sizes.append(sum(it[3] for it in self.items))
            return orig(self, *a, **k)

        G._WgradGroup.flush = spy
        try:
            ws = [torch.nn.Parameter(w.clone()) for w in ws0]
            sp = FlatParamSpace(list(reversed(ws)))
            sp.zero_grad(set_to_none=True)
            h = x0
            for w in ws:
                h = ops.linear(h, w)
            h.float().square().mean().backward()
            torch.cuda.synchronize()
            assert not G._WG.items and not G._WG.waiters
            return [w.grad.detach().clone() for w in ws], sizes
        finally:
            G._WgradGroup.flush = orig
            G._GROUP_BIG = old

    (ga, sa), (gb, sb) = run(True), run(False)
    assert sa == [256, 768], sa
    assert sb == [], sb
    for a, b in zip(ga, gb):
        assert torch.isfinite(a).all() and torch.equal(a, b)
