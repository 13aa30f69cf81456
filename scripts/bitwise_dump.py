"""Dump a kernel family's outputs (fixed seeds) to a .pt file, so two builds of the extension
(RTDC_EXT_SO=<path>) can be compared bitwise - the check behind every "bitwise equal" A/B record
in profiles/.

    python scripts/bitwise_dump.py attn|norm|resnet|gemm OUT.pt
    python -c "import torch; a, b = torch.load('A.pt'), torch.load('B.pt'); ..."   (compare)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def attn():
    from ray_torch_distributed_checkpoint_amd.ops.attention import causal_attention

    out = {}
    for name, B, T, H, Hkv, Dh in [("gpt2", 4, 1024, 12, 12, 64), ("gqa64", 2, 512, 8, 2, 64),
                                   ("llama", 1, 1024, 32, 8, 128)]:
        torch.manual_seed(7)
        qkv = (torch.randn(B, T, (H + 2 * Hkv) * Dh, device="cuda") * 0.5).bfloat16().requires_grad_(True)
        y = causal_attention(qkv, H, Hkv)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        out[name] = (y.detach().cpu(), qkv.grad.detach().cpu())
    return out


def norm():
    from ray_torch_distributed_checkpoint_amd.ops.norm import layer_norm, rms_norm

    out = {}
    for kind, M, D in [("rms", 2048, 4096), ("ln", 512, 4096), ("rms", 1024, 1024), ("ln", 4096, 768),
                       ("ln", 256, 2048)]:
        torch.manual_seed(M + D)
        x = torch.randn(M, D, device="cuda").bfloat16().requires_grad_(True)
        w = torch.nn.Parameter(1 + 0.1 * torch.randn(D, device="cuda"))
        b = torch.nn.Parameter(0.1 * torch.randn(D, device="cuda"))
        y = rms_norm(x, w) if kind == "rms" else layer_norm(x, w, b)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        out[f"{kind}_{M}x{D}"] = (y.detach().cpu(), x.grad.cpu(), w.grad.cpu(),
                                  b.grad.cpu() if b.grad is not None else torch.zeros(1))
    return out


def resnet():
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.models import ResNet18

    torch.manual_seed(3)
    model = ResNet18(num_classes=10).cuda()
    x = torch.randn(32, 3, 128, 128, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")
    loss = ops.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    out = {"loss": loss.detach().cpu()}
    for n, p in model.named_parameters():
        out["grad." + n] = p.grad.detach().cpu()
    for n, b in model.named_buffers():
        out["buf." + n] = b.detach().cpu()
    return out


def gemm():
    from ray_torch_distributed_checkpoint_amd.ops import gemm as G

    out = {}
    for name, M, K, N in [("qkv", 16384, 768, 2304), ("lm", 4096, 768, 50304), ("l_o", 2048, 4096, 4096),
                          ("l_qkv", 2048, 4096, 6144)]:
        torch.manual_seed(M + N)
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        out[name] = (G.linear_fwd(x, w).cpu(), G.linear_dgrad(dy, w).cpu())
    return out


if __name__ == "__main__":
    torch.save({"attn": attn, "norm": norm, "resnet": resnet, "gemm": gemm}[sys.argv[1]](), sys.argv[2])
