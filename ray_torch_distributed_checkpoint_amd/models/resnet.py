"""ResNet-18 (BASELINE config 2: "ResNet-18 DDP bf16 on 2xMI355X, sharded DCP save every N
steps") on the native channels-last kernels (ops/cnn.py).

No torchvision in this image, so the network is defined here with the standard ResNet-18
topology (7x7/2 stem + 3x3/2 max-pool, four stages of two BasicBlocks with 64/128/256/512
channels, 1x1/2 projection shortcuts, global average pool, FC) and the usual state-dict keys
(`conv1.weight`, `bn1.running_mean`, `layer2.0.downsample.1.weight`, `fc.bias`, ...), so a
checkpoint lines up with any other ResNet-18 of the same class count.  10 classes -> 11.18 M
parameters.

On the GPU activations are NHWC bf16 end to end: the input NCHW fp32 batch is converted once,
every BatchNorm is fused with its ReLU (and with the residual add + ReLU at the end of a
block).  On CPU the same module runs the fp32 PyTorch reference ops (gloo/CPU tests).
BatchNorm running statistics are buffers: DDP broadcasts them from rank 0 before every
forward and they are part of the DCP checkpoint.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from ..ops import cnn


class BatchNorm2d(nn.Module):
    """BatchNorm over the channel axis of NHWC activations, optionally fused with a residual
    add and ReLU: y = relu?(BN(x) + residual?)."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def forward(self, x, residual=None, relu: bool = False, residual_grad_to=None):
        return cnn.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                              self.momentum, self.eps, residual=residual, relu=relu,
                              num_batches_tracked=self.num_batches_tracked, residual_grad_to=residual_grad_to)

    def relu_max_pool(self, x, k: int = 3, s: int = 2, p: int = 1):
        """max_pool2d(relu(self(x))) in one pass (the stem; the BN output is never stored)."""
        return cnn.batch_norm_relu_max_pool(x, self.weight, self.bias, self.running_mean, self.running_var,
                                            self.training, self.momentum, self.eps,
                                            num_batches_tracked=self.num_batches_tracked, k=k, s=s, p=p)

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, layout=NHWC"


class Conv2d(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int = 1, pad: int = 0):
        super().__init__()
        self.stride, self.pad = stride, pad
        # channels-last weight ([O][KH][KW][I] in memory, [O, I, KH, KW] logically, like any
        # Conv2d state dict): its bf16 shadow is the implicit-GEMM operand as it stands
        w = torch.empty(cout, cin, k, k)
        nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")  # same values in either layout
        if os.environ.get("RTDC_CONV_WEIGHT_CL", "1") == "1":
            w = w.to(memory_format=torch.channels_last)
        self.weight = nn.Parameter(w)

    def forward(self, x, grad_accum=None):
        # every convolution of the network feeds a BatchNorm: its statistics come out of the
        # GEMM epilogue (training mode), the BN then skips its own pass over the activation
        return cnn.conv2d(x, self.weight, self.stride, self.pad, bn_stats=self.training, grad_accum=grad_accum)

    def extra_repr(self):
        o, i, k, _ = self.weight.shape
        return f"{i}, {o}, kernel_size={k}, stride={self.stride}, padding={self.pad}, bias=False, layout=NHWC"


class Downsample(nn.Sequential):
    """1x1/stride projection + BN, keys `downsample.0.weight`, `downsample.1.*`."""

    def __init__(self, cin, cout, stride):
        super().__init__(Conv2d(cin, cout, 1, stride, 0), BatchNorm2d(cout))


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = Conv2d(cin, cout, 3, stride, 1)
        self.bn1 = BatchNorm2d(cout)
        self.conv2 = Conv2d(cout, cout, 3, 1, 1)
        self.bn2 = BatchNorm2d(cout)
        self.downsample = Downsample(cin, cout, stride) if (stride != 1 or cin != cout) else None

    def forward(self, x):
        if x.is_cuda and torch.is_grad_enabled():
            # the block input's two gradients (conv1's and the shortcut's) are summed inside the
            # dgrad kernel of whichever backward runs last, not by an autograd add over x
            stash = cnn.GradStash(2)
            h = self.bn1(self.conv1(x, grad_accum=stash), relu=True)
            if self.downsample is None:
                return self.bn2(self.conv2(h), residual=x, relu=True, residual_grad_to=stash)
            sc = self.downsample[1](self.downsample[0](x, grad_accum=stash))
            return self.bn2(self.conv2(h), residual=sc, relu=True)
        h = self.bn1(self.conv1(x), relu=True)
        sc = x if self.downsample is None else self.downsample[1](self.downsample[0](x))
        return self.bn2(self.conv2(h), residual=sc, relu=True)


class ResNet18(nn.Module):
    def __init__(self, num_classes: int = 10, in_channels: int = 3, widths=(64, 128, 256, 512)):
        super().__init__()
        self.num_classes = num_classes
        self.conv1 = Conv2d(in_channels, widths[0], 7, 2, 3)
        self.bn1 = BatchNorm2d(widths[0])
        cin = widths[0]
        for i, w in enumerate(widths):
            stride = 1 if i == 0 else 2
            setattr(self, f"layer{i + 1}", nn.Sequential(BasicBlock(cin, w, stride), BasicBlock(w, w, 1)))
            cin = w
        self.fc_in = cin
        self.fc = _FC(cin, num_classes)

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def forward(self, x):
        """x: NCHW images (any float dtype).  Returns [B, num_classes] logits."""
        c1 = self.conv1
        if cnn.stem_supported(x, c1.weight, c1.stride, c1.pad):
            # space-to-depth implicit GEMM straight from the NCHW fp32 images (no im2col matrix)
            h = cnn.stem_conv(x, c1.weight, bn_stats=self.training)
        else:
            h = cnn.to_nhwc_bf16(x) if x.is_cuda else x.permute(0, 2, 3, 1).float().contiguous()
            h = c1(h)
        h = self.bn1.relu_max_pool(h, 3, 2, 1)
        h = self.layer4(self.layer3(self.layer2(self.layer1(h))))
        return self.fc(cnn.global_avg_pool(h))

    def flops_per_sample(self, hw: int = 224) -> float:
        """Training FLOPs (3x forward MACs x 2) at a square input of side `hw`."""
        macs = 0
        for m, (ho, wo) in _spatial_sizes(self, hw).items():
            o, i, k, _ = m.weight.shape
            macs += o * i * k * k * ho * wo
        macs += self.fc_in * self.num_classes
        return 6.0 * macs


class _FC(nn.Module):
    def __init__(self, cin, n):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n, cin))
        self.bias = nn.Parameter(torch.empty(n))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1 / math.sqrt(cin)
        nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return cnn.classifier(x, self.weight, self.bias)


def _spatial_sizes(model: ResNet18, hw: int) -> dict:
    out = {}

    def conv_out(m, h):
        k = m.weight.shape[-1]
        return (h + 2 * m.pad - k) // m.stride + 1

    h = conv_out(model.conv1, hw)
    out[model.conv1] = (h, h)
    h = (h + 2 - 3) // 2 + 1  # max-pool
    for li in range(1, 5):
        for blk in getattr(model, f"layer{li}"):
            h1 = conv_out(blk.conv1, h)
            out[blk.conv1] = (h1, h1)
            out[blk.conv2] = (h1, h1)
            if blk.downsample is not None:
                out[blk.downsample[0]] = (h1, h1)
            h = h1
    return out
