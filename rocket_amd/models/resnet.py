"""ResNet-18 (CIFAR-10 variant) and ResNet-50 (ImageNet shape) for the BASELINE DDP configs.

MI355X layout: activations are channels-last (NHWC) end to end — the native implicit-GEMM
convolutions (:class:`~rocket_amd.ops.iconv.IConv2d`, ``native/kernels/conv.hip``) gather NHWC
pixels straight into LDS and the fused BatchNorm kernels (:mod:`rocket_amd.ops.norm`) reduce over
contiguous channels.  Every ``conv → BN (→ +identity) → ReLU`` tail is
one BN-statistics launch plus one fused apply launch (``BatchNormAct2d``), so the
residual add and the ReLU never make their own pass over HBM; a block's first conv and its
shortcut form one autograd node (:func:`~rocket_amd.ops.iconv.conv_entry`), so the two gradients
of the block input meet in a conv epilogue instead of an add kernel.

The forward follows the reference batch contract: ``(img, label) -> (img, label, logits)``.
Architecture per He et al. (basic/bottleneck blocks, stride on the 3×3 conv as in
"ResNet v1.5"); the CIFAR variant uses a 3×3 stride-1 stem without max-pool.
"""

from __future__ import annotations

import os

from typing import List, Type

import torch
import torch.nn.functional as F
from torch import nn

from rocket_amd.ops.iconv import IConv2d, bn_relu_conv, conv_entry, stem_ok
from rocket_amd.ops.linear import native_route
from rocket_amd.ops.mlinear import MLinear, pooled_head, pooled_head_ok
from rocket_amd.ops.norm import BatchNormAct2d
from rocket_amd.ops.pool import global_avg_pool

# global average pool fused into the classifier head's launches when the head runs on head.hip
POOLED_HEAD = os.environ.get("ROCKET_POOLED_HEAD", "1") != "0"


def _conv(cin, cout, k, stride=1):
    # native implicit-GEMM MFMA conv (ops/iconv.py; the 3-channel stem falls back to nn.Conv2d).
    # Every conv here feeds a BatchNormAct2d: its epilogue emits the BatchNorm's tile statistics.
    conv = IConv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False)
    conv.emit_bn_stats = True
    return conv


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, width: int, stride: int = 1):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = _conv(cin, width, 3, stride)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.conv2 = _conv(width, cout, 3)
        self.bn2 = BatchNormAct2d(cout, relu=True)  # relu(bn2(.) + identity), fused
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(_conv(cin, cout, 1, stride), BatchNormAct2d(cout))

    def forward(self, x):
        # conv1 and the shortcut as one node: x's two input gradients meet in conv1's dgrad epilogue
        y1, short = conv_entry(x, self.conv1, self.down[0] if self.down is not None else None)
        identity = short if self.down is None else self.down[1](short)
        # conv2(relu(bn1(y1))): bn1 applied inside conv2's operand staging (ops/iconv.py bn_relu_conv)
        return self.bn2(bn_relu_conv(self.bn1, self.conv2, y1), residual=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = _conv(cin, width, 1)
        self.bn1 = BatchNormAct2d(width, relu=True)
        self.conv2 = _conv(width, width, 3, stride)
        self.bn2 = BatchNormAct2d(width, relu=True)
        self.conv3 = _conv(width, cout, 1)
        self.bn3 = BatchNormAct2d(cout, relu=True)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(_conv(cin, cout, 1, stride), BatchNormAct2d(cout))

    def forward(self, x):
        y1, short = conv_entry(x, self.conv1, self.down[0] if self.down is not None else None)
        identity = short if self.down is None else self.down[1](short)
        # bn1 / bn2 (+ ReLU) folded into conv2 / conv3 where the fold applies (stride-1 consumer)
        out = bn_relu_conv(self.bn1, self.conv2, y1)
        out = bn_relu_conv(self.bn2, self.conv3, out)
        return self.bn3(out, residual=identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[nn.Module], layers: List[int], num_classes: int = 1000, cifar_stem: bool = False,
                 zero_init_residual: bool = True):
        super().__init__()
        self.cifar_stem = cifar_stem
        if cifar_stem:
            self.stem = nn.Sequential(_conv(3, 64, 3), BatchNormAct2d(64, relu=True))
        else:
            # BN + ReLU + the 3x3/s2 max-pool in one pass (norm.hip bn_relu_maxpool)
            self.stem = nn.Sequential(_conv(3, 64, 7, 2), BatchNormAct2d(64, relu=True, maxpool=True))
        cin = 64
        stages = []
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            blocks = []
            for j in range(n):
                stride = 2 if (i > 0 and j == 0) else 1
                blocks.append(block(cin, width, stride))
                cin = width * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        # nn.Linear on the native MFMA GEMM (ops/mlinear.py MLinear: the small-product route of the
        # default GEMM routing; plain nn.Linear when the class count is not a multiple of 8 or the
        # fused kernels are off)
        self.fc = MLinear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                last = getattr(m, "bn3", None) if isinstance(m, Bottleneck) else getattr(m, "bn2", None)
                if isinstance(m, (Bottleneck, BasicBlock)) and last is not None:
                    nn.init.zeros_(last.weight)

    def logits(self, x: torch.Tensor) -> torch.Tensor:
        if not torch.is_autocast_enabled(x.device.type):
            x = x.to(self.fc.weight.dtype if hasattr(self, "fc") else self.head.weight.dtype)  # bf16-stored images
        if not stem_ok(self.stem[0], x):  # the native stem reads the image in any layout
            x = x.contiguous(memory_format=torch.channels_last)
        x = self.stem(x)  # ImageNet stem: the max-pool is inside its BatchNormAct2d
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if native_route() and POOLED_HEAD and pooled_head_ok(self.fc, x):
            return pooled_head(self.fc, x)  # the pool inside the head's two launches (head.hip)
        if native_route():
            x = global_avg_pool(x)  # one pooling launch, one broadcast launch in the backward
        else:
            x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)

    def forward(self, batch):
        if isinstance(batch, torch.Tensor):
            return self.logits(batch)
        img, label = batch[0], batch[1]
        return (img, label, self.logits(img))


def resnet18(num_classes: int = 10, cifar: bool = True) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, cifar_stem=cifar)


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes)
