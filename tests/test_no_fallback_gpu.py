"""No silent eager fallback on the GPU: a native op handed a dtype its gfx950 kernel does not
implement raises instead of quietly running MIOpen / SDPA / ATen."""
import pytest
import torch

from ray_torch_distributed_checkpoint_amd import ops
from ray_torch_distributed_checkpoint_amd.ops import cnn, llama_ops

pytestmark = pytest.mark.gpu


def _cases():
    d = "cuda"
    x4 = torch.randn(2, 8, 8, 64, device=d)           # NHWC fp32
    w = torch.randn(64, 64, 3, 3, device=d)
    g = torch.ones(64, device=d)
    z = torch.zeros(64, device=d)
    qkv = torch.randn(1, 64, 3 * 128, device=d)
    return [
        ("conv2d", lambda: cnn.conv2d(x4, w, 1, 1)),
        ("batch_norm", lambda: cnn.batch_norm(x4, g, z, z.clone(), g.clone(), True)),
        ("max_pool2d", lambda: cnn.max_pool2d(x4)),
        ("global_avg_pool", lambda: cnn.global_avg_pool(x4)),
        ("classifier", lambda: cnn.classifier(torch.randn(4, 64, device=d), torch.randn(10, 64, device=d),
                                              torch.zeros(10, device=d))),
        ("layer_norm", lambda: ops.layer_norm(torch.randn(4, 64, device=d), g, z)),
        ("rms_norm", lambda: ops.rms_norm(torch.randn(4, 64, device=d), g)),
        ("causal_attention", lambda: ops.causal_attention(qkv, 2)),
        ("apply_rope", lambda: llama_ops.apply_rope(qkv, 2, 2)),
        ("swiglu_mlp", lambda: llama_ops.swiglu_mlp(torch.randn(4, 64, device=d), torch.randn(256, 64, device=d),
                                                    torch.randn(64, 128, device=d))),
        ("cross_entropy", lambda: ops.cross_entropy(torch.randn(4, 10, device=d).half(),
                                                    torch.zeros(4, dtype=torch.int64, device=d))),
        ("cross_entropy", lambda: ops.cross_entropy(torch.randn(4, 10, device=d),
                                                    torch.zeros(4, dtype=torch.int32, device=d))),
    ]


@pytest.mark.parametrize("i", range(12))
def test_gpu_op_rejects_unsupported_dtype(i):
    name, fn = _cases()[i]
    with pytest.raises(TypeError):
        fn()


def test_cross_entropy_ignore_index_counts_valid_rows_gpu():
    """rows with target -100 are excluded from the mean (torch semantics), also for
    the fused LM-head path, without a host sync."""
    torch.manual_seed(0)
    logits = torch.randn(64, 50, device="cuda", requires_grad=True)
    tgt = torch.randint(0, 50, (64,), device="cuda")
    tgt[::3] = -100
    ref_l = logits.detach().clone().requires_grad_(True)
    loss = ops.cross_entropy(logits, tgt)
    ref = torch.nn.functional.cross_entropy(ref_l, tgt, ignore_index=-100)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(logits.grad, ref_l.grad, rtol=1e-4, atol=1e-6)
    # LM-head fusion (bf16) against the same math in fp32
    x = torch.randn(2, 64, 128, device="cuda").bfloat16().requires_grad_(True)
    wt = torch.nn.Parameter(torch.randn(256, 128, device="cuda") * 0.05)
    t2 = torch.randint(0, 250, (2, 64), device="cuda")
    t2[:, ::4] = -100
    l2 = ops.lm_head_cross_entropy(x, wt, t2, 250)
    xr = x.detach().float().requires_grad_(True)
    wr = wt.detach().clone().requires_grad_(True)
    r2 = torch.nn.functional.cross_entropy((xr @ wr.t())[..., :250].reshape(-1, 250), t2.reshape(-1),
                                           ignore_index=-100)
    l2.backward()
    r2.backward()
    torch.testing.assert_close(l2.float(), r2, rtol=2e-2, atol=2e-2)
    gerr = (wt.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert gerr < 3e-2
